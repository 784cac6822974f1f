"""Ops: NHWC neural-network ops on hand-written HIP/CDNA4 kernels (torch reference on CPU)."""
from . import nn  # noqa: F401
from ._native import set_deterministic, deterministic, set_sync_check  # noqa: F401
