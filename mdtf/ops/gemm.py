"""Dense / matmul on the GPU: GEMM + fused bias/activation epilogue kernel.

The plain GEMM goes to hipBLASLt (``torch.matmul``) — the library path the
design allows for plain GEMMs — and bias + activation (+ their gradients, the
bias column sums) run on the mdtf kernels.  The hand-written MFMA GEMM of
``csrc/gemm.hip`` takes over per shape once it wins (see ``ops/autotune.py``).
"""
import torch

from . import kernels


def matmul(a, b):
    return torch.matmul(a, b)


def dense(x, w, b=None, act=None):
    y = torch.matmul(x, w.to(x.dtype))
    if x.dtype != torch.bfloat16:
        if b is not None:
            y = y + b.to(y.dtype)
        if act == "relu":
            y = torch.relu(y)
        elif act == "gelu":
            y = torch.nn.functional.gelu(y, approximate="tanh")
        return y
    if b is None and act is None:
        return y
    return kernels.bias_act(y, b, act)
