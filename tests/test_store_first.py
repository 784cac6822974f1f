"""Store-first gradient slots (train/variables.py claim_store / note_accumulate / unclaimed_skips and
parallel/flat.py zero_grad(skip_stored)): CPU bookkeeping checks; the kernel side is in test_kernels_gpu.py
(test_grad_store_first_matches_zero_and_accumulate, test_fill_ranges_zero)."""
import torch

from mdtf.parallel.flat import FlatGroup
from mdtf.train import variables as V


def _group():
    vs = [V.Variable("a", torch.ones(5, 3)), V.Variable("b", torch.ones(7)), V.Variable("c", torch.ones(130))]
    return FlatGroup(vs, "cpu", None, False), vs


def test_zero_grad_skips_only_store_written_slots():
    g, (a, b, c) = _group()
    g.grad.fill_(1.0)
    b.store_first = True
    g.zero_grad(skip_stored=True)
    assert a.grad.abs().sum() == 0 and c.grad.abs().sum() == 0
    assert torch.equal(b.grad, torch.ones(7)) and b.skip_zero
    assert g.grad.sum() == 7                      # alignment gaps zeroed too
    g.grad.fill_(1.0)
    g.zero_grad()                                 # the full fill (backup replicas, async PS) ignores the flags
    assert g.grad.abs().sum() == 0 and not b.skip_zero


def test_claim_store_first_write_only(monkeypatch):
    monkeypatch.setattr(V, "STORE_FIRST", True)
    g, (a, b, c) = _group()
    V.begin_grad_epoch()
    assert V.claim_store(a)                       # the step's first (full-slot) write: overwrite
    assert not V.claim_store(a)                   # a second write the same step accumulates
    V.note_accumulate(b)                          # b's first write accumulates ...
    assert not V.claim_store(b)                   # ... so a later full-slot writer must too
    assert a.store_first and not b.store_first
    # next step: a's slot is skipped by the fill; an accumulating first write zeroes it before adding
    g.grad.fill_(3.0)
    g.zero_grad(skip_stored=True)
    V.begin_grad_epoch()
    assert a.skip_zero and a.grad.sum() == 45
    V.note_accumulate(a)
    assert a.grad.abs().sum() == 0 and not a.store_first
    # a skipped slot nobody writes in a step is zeroed at the end of backward
    a.store_first = True
    g.grad.fill_(2.0)
    g.zero_grad(skip_stored=True)
    V.begin_grad_epoch()
    V.unclaimed_skips([a, b, c])
    assert a.grad.abs().sum() == 0


def test_claim_store_disabled(monkeypatch):
    monkeypatch.setattr(V, "STORE_FIRST", False)
    _, (a, _, _) = _group()
    V.begin_grad_epoch()
    a.uses = 1
    assert not V.claim_store(a)
