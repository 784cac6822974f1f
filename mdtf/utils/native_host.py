"""ctypes bindings of the host C++ library (``mdtf/csrc/host/io.cpp``).

CRC32C runs on the SSE4.2 ``crc32`` instruction in C++; a pure-Python
table-driven fallback exists only so that tiny unit-test inputs work before
the library has been built.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(os.path.dirname(_HERE), "csrc", "build", "libmdtf_host.so")
_lib = None


def lib(required=False):
    global _lib
    if _lib is None and os.path.exists(LIB_PATH):
        h = ctypes.CDLL(LIB_PATH)
        h.mdtf_crc32c.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint32]
        h.mdtf_crc32c.restype = ctypes.c_uint32
        h.mdtf_masked_crc32c.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
        h.mdtf_masked_crc32c.restype = ctypes.c_uint32
        h.mdtf_tfr_open.argtypes = [ctypes.c_char_p, ctypes.c_int]
        h.mdtf_tfr_open.restype = ctypes.c_void_p
        h.mdtf_tfr_next.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_char_p)]
        h.mdtf_tfr_next.restype = ctypes.c_longlong
        h.mdtf_tfr_close.argtypes = [ctypes.c_void_p]
        h.mdtf_tfw_open.argtypes = [ctypes.c_char_p]
        h.mdtf_tfw_open.restype = ctypes.c_void_p
        h.mdtf_tfw_write.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_ulonglong]
        h.mdtf_tfw_write.restype = ctypes.c_int
        h.mdtf_tfw_close.argtypes = [ctypes.c_void_p]
        h.mdtf_tfw_close.restype = ctypes.c_int
        h.mdtf_loader_create.argtypes = [ctypes.POINTER(ctypes.c_char_p), ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                         ctypes.c_ulonglong, ctypes.c_ulonglong, ctypes.c_ulonglong, ctypes.c_int]
        h.mdtf_loader_create.restype = ctypes.c_void_p
        h.mdtf_loader_next.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_ulonglong]
        h.mdtf_loader_next.restype = ctypes.c_longlong
        h.mdtf_loader_errors.argtypes = [ctypes.c_void_p]
        h.mdtf_loader_errors.restype = ctypes.c_longlong
        h.mdtf_loader_destroy.argtypes = [ctypes.c_void_p]
        _lib = h
    if _lib is None and required:
        raise RuntimeError("host library %s not built (python -m mdtf.csrc.build)" % LIB_PATH)
    return _lib


_TABLE = None


def _table():
    global _TABLE
    if _TABLE is None:
        t = []
        for i in range(256):
            c = i
            for _ in range(8):
                c = (c >> 1) ^ (0x82F63B78 if c & 1 else 0)
            t.append(c)
        _TABLE = t
    return _TABLE


def _as_buffer(data):
    if isinstance(data, (bytes, bytearray)):
        return bytes(data)
    return memoryview(data).tobytes()


def crc32c(data, init=0):
    h = lib()
    if h is not None:
        if isinstance(data, bytes):
            return h.mdtf_crc32c(data, len(data), init)
        mv = memoryview(data).cast("B")
        buf = (ctypes.c_char * len(mv)).from_buffer(mv) if not mv.readonly else ctypes.create_string_buffer(mv.tobytes(), len(mv))
        return h.mdtf_crc32c(ctypes.addressof(buf), len(mv), init)
    t = _table()
    c = init ^ 0xFFFFFFFF
    for b in _as_buffer(data):
        c = t[(c ^ b) & 0xFF] ^ (c >> 8)
    return c ^ 0xFFFFFFFF


def crc32c_ptr(ptr, n, init=0):
    """CRC32C of raw memory (e.g. a pinned tensor's data_ptr())."""
    return lib(required=True).mdtf_crc32c(ctypes.c_void_p(ptr), n, init)


MASK_DELTA = 0xa282ead8


def mask(crc):
    return (((crc >> 15) | (crc << 17)) + MASK_DELTA) & 0xFFFFFFFF


def unmask(masked):
    rot = (masked - MASK_DELTA) & 0xFFFFFFFF
    return ((rot >> 17) | (rot << 15)) & 0xFFFFFFFF


def masked_crc32c(data):
    return mask(crc32c(data))
