"""Loader for the hand-written HIP/CDNA4 kernel library.

The kernels live in ``mdtf/csrc/*.hip`` and are compiled by
``mdtf/csrc/build.py`` (``hipcc --offload-arch=gfx950``) into
``mdtf/csrc/build/libmdtf_kernels.so`` — in-tree, so the shared object travels
with the repository snapshot to the GPU box.  The library exposes a plain C ABI
(pointers, sizes, ``hipStream_t``) and is loaded with ``ctypes`` *after*
``torch``: both link ``libamdhip64.so.7``, so the already-loaded HIP runtime of
torch is shared and kernels run on torch's current stream (hipGraph capture of
a training step therefore records them too).

Kernel selection: ``MDTF_KERNELS=native`` (default) runs the HIP kernels for
every tensor on a GPU and raises if the library is missing — there is no
silent fallback.  ``MDTF_KERNELS=torch`` selects the stock PyTorch-ROCm ops
(MIOpen/hipBLASLt) and is used only as the comparator baseline.  CPU tensors
always use the PyTorch reference implementations (unit tests).
"""
import ctypes
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_DIR = os.path.join(os.path.dirname(_HERE), "csrc", "build")
# MDTF_KERNELS_LIB: load another build of the kernel library (A/B of two builds on one box)
LIB_PATH = os.environ.get("MDTF_KERNELS_LIB") or os.path.join(LIB_DIR, "libmdtf_kernels.so")

_lib = None
_load_error = None


def mode():
    return os.environ.get("MDTF_KERNELS", "native")


def lib():
    """The ctypes handle (raises if the library is not built)."""
    global _lib, _load_error
    if _lib is not None:
        return _lib
    if _load_error is not None:
        raise _load_error
    if not os.path.exists(LIB_PATH):
        _load_error = RuntimeError(
            "mdtf HIP kernel library not found at %s — build it with "
            "`python -m mdtf.csrc.build` (or __graft_entry__.build())" % LIB_PATH)
        raise _load_error
    try:
        _lib = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
    except OSError as e:  # pragma: no cover - depends on the box
        _load_error = RuntimeError("failed to load %s: %s" % (LIB_PATH, e))
        raise _load_error
    _declare(_lib)
    if _DETERMINISTIC:
        _lib.mdtf_set_deterministic(ctypes.c_int(1))
    return _lib


def available():
    try:
        lib()
        return True
    except RuntimeError:
        return False


def use_native(*tensors):
    """True if these (GPU) tensors must run on the HIP kernels."""
    t = tensors[0]
    if not t.is_cuda:
        return False
    if mode() == "torch":
        return False
    lib()  # raise loudly if missing
    return True


def stream_ptr(device=None):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)


_SYNC_CHECK = os.environ.get("MDTF_SYNC_CHECK", "0") not in ("0", "", "false")
_DETERMINISTIC = os.environ.get("MDTF_DETERMINISTIC", "0") not in ("0", "", "false")


def check(rc, what):
    if rc != 0:
        raise RuntimeError("mdtf kernel %s failed: %s (code %d)" % (what, _error_string(rc), rc))
    if _SYNC_CHECK and not torch.cuda.is_current_stream_capturing():
        # debug mode (MDTF_SYNC_CHECK=1): serialize after every native launch so a faulting
        # kernel is named here instead of surfacing at some later synchronization
        import torch
        try:
            torch.cuda.synchronize()
        except RuntimeError as e:
            raise RuntimeError("mdtf kernel %s faulted: %s" % (what, e))


def set_deterministic(flag=True):
    """Fixed-order reductions everywhere the native kernels would use cross-block float
    atomics (BN statistics rows, split-K weight gradients, column-sum / LayerNorm
    partial reductions, embedding scatter-add).  Slower; for debugging and
    bitwise-reproducible runs.  Also settable with ``MDTF_DETERMINISTIC=1``."""
    global _DETERMINISTIC
    _DETERMINISTIC = bool(flag)
    if _lib is not None:
        _lib.mdtf_set_deterministic(ctypes.c_int(int(_DETERMINISTIC)))


def deterministic():
    return _DETERMINISTIC


def set_sync_check(flag=True):
    global _SYNC_CHECK
    _SYNC_CHECK = bool(flag)


def _error_string(rc):
    try:
        s = _lib.mdtf_error_string(ctypes.c_int(rc))
        return s.decode() if s else "?"
    except Exception:  # pragma: no cover
        return "?"


# ---------------------------------------------------------------------------
# C ABI declarations (kept next to the loader so signatures are checked once)
# ---------------------------------------------------------------------------
_P = ctypes.c_void_p
_I = ctypes.c_int
_L = ctypes.c_longlong
_F = ctypes.c_float

SIGNATURES = {
    "mdtf_error_string": ([_I], ctypes.c_char_p),
    "mdtf_version": ([], _I),
}


def register(name, argtypes, restype=_I):
    SIGNATURES[name] = (argtypes, restype)


def _declare(handle):
    for name, (args, res) in SIGNATURES.items():
        fn = getattr(handle, name, None)
        if fn is None:
            continue
        fn.argtypes = args
        fn.restype = res


def fn(name):
    f = getattr(lib(), name)
    if name in SIGNATURES and f.argtypes is None:
        args, res = SIGNATURES[name]
        f.argtypes, f.restype = args, res
    return f


P, I, L, F = _P, _I, _L, _F
U = ctypes.c_uint
