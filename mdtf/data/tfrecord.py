"""TFRecord files: framing = ``u64 length | masked crc32c(length) | data |
masked crc32c(data)``.  Reading, writing and the multi-threaded shuffling
record loader are native C++ (``csrc/host/io.cpp``); this module wraps them.

Reference: ``tf.TFRecordReader`` + ``string_input_producer`` + ``shuffle_batch``
queue runners (``distribute_input.py:54-106``, ``distribute_train.py:120-122``).
"""
import ctypes
import glob
import os
import struct

from ..utils import native_host


class TFRecordWriter(object):
    def __init__(self, path):
        self.path = path
        h = native_host.lib()
        if h is not None:
            self._h = h.mdtf_tfw_open(path.encode())
            if not self._h:
                raise IOError("cannot open %s" % path)
            self._py = None
        else:
            self._h = None
            self._py = open(path, "wb")

    def write(self, record):
        if isinstance(record, str):
            record = record.encode()
        if self._h is not None:
            if native_host.lib().mdtf_tfw_write(self._h, record, len(record)) != 0:
                raise IOError("write failed: %s" % self.path)
            return
        hdr = struct.pack("<Q", len(record))
        self._py.write(hdr + struct.pack("<I", native_host.masked_crc32c(hdr)) + record +
                       struct.pack("<I", native_host.masked_crc32c(record)))

    def close(self):
        if self._h is not None:
            native_host.lib().mdtf_tfw_close(self._h)
            self._h = None
        if self._py is not None:
            self._py.close()
            self._py = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()


def tf_record_iterator(path, verify=True):
    h = native_host.lib()
    if h is not None:
        r = h.mdtf_tfr_open(path.encode(), int(verify))
        if not r:
            raise IOError("cannot open %s" % path)
        try:
            p = ctypes.c_char_p()
            while True:
                n = h.mdtf_tfr_next(r, ctypes.byref(p))
                if n == -1:
                    return
                if n < 0:
                    raise IOError("corrupt record in %s (code %d)" % (path, n))
                yield ctypes.string_at(p, n)
        finally:
            h.mdtf_tfr_close(r)
        return
    with open(path, "rb") as f:
        while True:
            hdr = f.read(12)
            if not hdr:
                return
            n = struct.unpack("<Q", hdr[:8])[0]
            if verify and native_host.masked_crc32c(hdr[:8]) != struct.unpack("<I", hdr[8:])[0]:
                raise IOError("corrupt record header in %s" % path)
            data = f.read(n)
            crc = struct.unpack("<I", f.read(4))[0]
            if verify and native_host.masked_crc32c(data) != crc:
                raise IOError("corrupt record in %s" % path)
            yield data


def expand_paths(paths):
    out = []
    for p in ([paths] if isinstance(paths, str) else paths):
        if os.path.isdir(p):
            out.extend(sorted(os.path.join(p, f) for f in os.listdir(p) if not f.startswith(".")))
        elif any(c in p for c in "*?["):
            out.extend(sorted(glob.glob(p)))
        else:
            out.append(p)
    return out


class NameQueue(object):
    """``string_input_producer`` result: the list of files to read."""

    def __init__(self, files, num_epochs=None, shuffle=True, seed=None):
        self.files = expand_paths(files)
        self.num_epochs = num_epochs
        self.shuffle = shuffle
        self.seed = seed
        self._pos = 0

    def __iter__(self):
        return iter(self.files)

    def dequeue(self):
        f = self.files[self._pos % len(self.files)]
        self._pos += 1
        return f


def string_input_producer(string_tensor, num_epochs=None, shuffle=True, seed=None, capacity=32, name=None):
    return NameQueue(string_tensor, num_epochs, shuffle, seed)


class ShuffledRecordLoader(object):
    """Native threaded shuffle buffer over TFRecord files."""

    def __init__(self, files, epochs=None, shuffle=True, capacity=10000, min_after_dequeue=0, seed=0,
                 num_threads=4, max_record_bytes=64 << 20):
        self.files = expand_paths(files)
        if not self.files:
            raise ValueError("no input files")
        h = native_host.lib(required=True)
        arr = (ctypes.c_char_p * len(self.files))(*[f.encode() for f in self.files])
        self._h = h.mdtf_loader_create(arr, len(self.files), int(epochs or 0), int(bool(shuffle)), int(capacity),
                                       int(min_after_dequeue), int(seed), int(num_threads))
        self._buf = ctypes.create_string_buffer(1 << 20)
        self._max = max_record_bytes

    def next(self):
        h = native_host.lib()
        while True:
            n = h.mdtf_loader_next(self._h, self._buf, len(self._buf))
            if n >= 0:
                return self._buf.raw[:n]
            if n == -1:
                raise StopIteration
            need = -n - 16
            if need > self._max:
                raise IOError("record of %d bytes exceeds max_record_bytes" % need)
            self._buf = ctypes.create_string_buffer(need)

    __next__ = next

    def __iter__(self):
        return self

    def errors(self):
        return native_host.lib().mdtf_loader_errors(self._h)

    def close(self):
        if self._h:
            native_host.lib().mdtf_loader_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
