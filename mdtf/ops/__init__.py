"""Ops: NHWC neural-network ops on hand-written HIP/CDNA4 kernels (torch reference on CPU)."""
from . import nn  # noqa: F401
