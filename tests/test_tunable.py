"""The shipped hipBLASLt/rocBLAS solution table (mdtf/ops/tunable.py)."""
import csv
import os

import pytest
import torch

from mdtf.ops import tunable


def test_table_is_well_formed():
    rows = list(csv.reader(open(tunable.TABLE)))
    validators = {r[1]: r[2] for r in rows if r and r[0] == "Validator"}
    assert validators["GCN_ARCH_NAME"].startswith("gfx950")
    assert {"PT_VERSION", "HIP_VERSION", "HIPBLASLT_VERSION", "ROCBLAS_VERSION"} <= set(validators)
    gemms = [r for r in rows if r and r[0] != "Validator"]
    assert len(gemms) >= 8 and all(len(r) == 4 for r in gemms)
    # the BERT-base projections (tokens 8192 = batch 64 x seq 128) are in it
    assert any("8192_768" in r[1] for r in gemms)


def test_cpu_is_a_no_op():
    assert tunable.ensure(torch.device("cpu")) is False


@pytest.mark.gpu
def test_tuned_gemm_numerics():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    dev = torch.device("cuda")
    if "PYTORCH_TUNABLEOP_ENABLED" in os.environ or os.environ.get("MDTF_TUNABLEOP") == "0":
        pytest.skip("tuning table disabled in this environment")
    assert tunable.ensure(dev)
    torch.manual_seed(0)
    x = torch.randn(8192, 768, device=dev).bfloat16()
    w = (torch.randn(768, 3072, device=dev) * 0.05).bfloat16()
    b = torch.randn(3072, device=dev).bfloat16()
    y = torch.addmm(b, x, w)                       # a shape the table covers
    ref = x.float() @ w.float() + b.float()
    assert ((y.float() - ref).norm() / ref.norm()).item() < 1e-2


def test_user_tunableop_settings_take_precedence(monkeypatch):
    """A user's own PYTORCH_TUNABLEOP_* environment (or MDTF_TUNABLEOP=0) leaves TunableOp alone."""
    class _Dev(object):
        type = "cuda"
    for env in ({"PYTORCH_TUNABLEOP_ENABLED": "1"}, {"MDTF_TUNABLEOP": "0"}):
        monkeypatch.setattr(tunable, "_done", set())
        for k, v in env.items():
            monkeypatch.setenv(k, v)
        assert tunable.ensure(_Dev()) is False
        assert "skip" in tunable._done
        for k in env:
            monkeypatch.delenv(k)
