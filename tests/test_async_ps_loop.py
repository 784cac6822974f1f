"""The async parameter server's request loop (``mdtf.parallel.async_ps.service_loop``) driven by fake works.

The multi-process tests run it on gloo, whose receives complete only inside ``wait()`` (helper-thread flags).
Here the RCCL branch is covered too: works whose ``is_completed()`` flips after a number of polls, the way an
RCCL work answers from its HIP event (reference: PS placement ``distribute_train.py:95-96,109-110``;
``replicas_to_aggregate`` ``distribute_flags.py:26-29``)."""
import threading

import pytest

from mdtf.parallel import async_ps as A


class FakeWork(object):
    """Completes after ``polls`` calls of is_completed() (RCCL-like) or when its wait() returns (gloo-like)."""

    def __init__(self, polls=0, fail=None, delay_s=0.0):
        self.polls = polls
        self.fail = fail
        self.delay_s = delay_s
        self.waited = False

    def is_completed(self):
        if self.polls > 0:
            self.polls -= 1
            return False
        return True

    def wait(self):
        if self.delay_s:
            threading.Event().wait(self.delay_s)
        if self.fail is not None:
            raise self.fail
        self.waited = True
        return True


def _script(requests, polls=3):
    """workers -> list of headers (kind, version) they send in order; payload of a push = 2 works."""
    log = {"applied": [], "served": [], "posted_hdr": {}, "payload_posts": 0}
    cursor = {w: 0 for w in requests}

    def post_header(w):
        log["posted_hdr"][w] = log["posted_hdr"].get(w, 0) + 1
        return FakeWork(polls=polls + w)

    def read_header(w):
        h = requests[w][cursor[w]]
        cursor[w] += 1
        return h

    def post_payload(w):
        log["payload_posts"] += 1
        return [FakeWork(polls=polls), FakeWork(polls=2 * polls)]

    def serve(w, kind, ver):
        log["served"].append((w, kind))
        return kind != A.K_DONE

    def apply_batch(batch):
        log["applied"].append(list(batch))
    return log, post_header, read_header, post_payload, serve, apply_batch


@pytest.mark.parametrize("threaded", [False, True], ids=["rccl-is_completed", "threaded"])
def test_service_loop_serves_every_worker(threaded):
    reqs = {1: [(A.K_PULL, 0), (A.K_PUSH, 0), (A.K_PUSH, 1), (A.K_DONE, 2)],
            2: [(A.K_PULL, 0), (A.K_PUSH, 0), (A.K_MASTER, 1), (A.K_DONE, 1)]}
    log, ph, rh, pp, serve, apply_batch = _script(reqs)
    st = {"idle": 0.0}
    A.service_loop([1, 2], ph, rh, pp, serve, apply_batch, threaded, st)
    pushes = sorted((w, v) for b in log["applied"] for w, v in b)
    assert pushes == [(1, 0), (1, 1), (2, 0)]
    assert log["payload_posts"] == 3
    assert sorted(log["served"]) == sorted([(1, A.K_PULL), (1, A.K_DONE), (2, A.K_PULL), (2, A.K_MASTER), (2, A.K_DONE)])
    # a header receive is re-posted after every served request and applied push, never after done
    assert log["posted_hdr"] == {1: 4, 2: 4}
    assert st["idle"] >= 0.0


def test_service_loop_batches_concurrent_pushes():
    """Pushes of several workers whose payloads complete in the same poll round are applied as ONE batch."""
    reqs = {w: [(A.K_PUSH, 0), (A.K_DONE, 1)] for w in (1, 2, 3)}
    log, ph, rh, pp, serve, apply_batch = _script(reqs, polls=0)
    A.service_loop([1, 2, 3], lambda w: FakeWork(0), rh, lambda w: [FakeWork(0)], serve, apply_batch, False,
                   {"idle": 0.0})
    assert [sorted(b) for b in log["applied"]] == [[(1, 0), (2, 0), (3, 0)]]


def test_posted_receive_failure_reaches_the_loop():
    """A helper thread whose wait() raises (peer died, gloo timeout) hands the error to the service loop, which
    re-raises it (no silent spin)."""
    boom = RuntimeError("peer closed the connection")
    reqs = {1: [(A.K_PUSH, 0), (A.K_DONE, 1)]}
    log, ph, rh, pp, serve, apply_batch = _script(reqs)
    with pytest.raises(RuntimeError, match="peer closed"):
        A.service_loop([1], lambda w: FakeWork(delay_s=0.01), rh, lambda w: [FakeWork(fail=boom)], serve,
                       apply_batch, True, {"idle": 0.0})
    p = A._Posted(FakeWork(fail=boom), True)
    p.ev.wait(5)
    with pytest.raises(RuntimeError):
        p.done()
    with pytest.raises(RuntimeError):
        p.wait()


def test_idle_wait_is_woken_by_completion():
    """The threaded loop sleeps on an event the helper threads set, not a GIL-holding spin: a long-delayed
    receive costs idle time, but the loop still finishes promptly after it completes."""
    import time
    reqs = {1: [(A.K_DONE, 0)]}
    log, ph, rh, pp, serve, apply_batch = _script(reqs)
    st = {"idle": 0.0}
    t0 = time.time()
    A.service_loop([1], lambda w: FakeWork(delay_s=0.2), rh, pp, serve, apply_batch, True, st, idle_wait_s=0.05)
    dt = time.time() - t0
    assert 0.18 <= dt < 2.0
    assert st["idle"] > 0.1
