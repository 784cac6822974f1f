"""TF tensor-bundle V2 checkpoints (``tf.train.Saver`` layout) without TF.

Files for prefix ``P`` (SURVEY §5 "Checkpoint / resume"):

* ``P.index`` — SSTable: key ``""`` → ``BundleHeaderProto{num_shards,
  endianness=LITTLE, version{producer=1}}``; key ``<tensor name>`` →
  ``BundleEntryProto{dtype, shape, shard_id, offset, size, crc32c}`` where
  ``crc32c`` is the masked CRC32C of the tensor bytes;
* ``P.data-0000k-of-0000N`` — raw little-endian tensor bytes, one file per
  shard (the reference's sharded Saver writes one per PS device).

The reference delegates this to TF's C++ ``BundleWriter`` (Saver created by
``Scaffold``, ``distribute_train.py:171-175``).  Tensor bytes are hashed with
the SSE4.2 CRC32C of ``libmdtf_host.so``.
"""
import os

import numpy as np
import torch

from . import proto as P
from .sstable import TableReader, TableWriter
from ..utils import native_host

_DT_FROM_TORCH = {
    torch.float32: P.DT_FLOAT, torch.float64: P.DT_DOUBLE, torch.int32: P.DT_INT32, torch.uint8: P.DT_UINT8,
    torch.int16: P.DT_INT16, torch.int8: P.DT_INT8, torch.int64: P.DT_INT64, torch.bool: P.DT_BOOL,
    torch.bfloat16: P.DT_BFLOAT16, torch.float16: P.DT_HALF,
}
_TORCH_FROM_DT = {v: k for k, v in _DT_FROM_TORCH.items()}


def data_filename(prefix, shard, num_shards):
    return "%s.data-%05d-of-%05d" % (prefix, shard, num_shards)


def _header(num_shards):
    version = P.f_varint(1, 1)  # VersionDef.producer = kTensorBundleVersion
    return P.f_varint(1, num_shards) + P.f_varint(2, 0) + P.f_bytes(3, version)


def _shape_proto(shape):
    return b"".join(P.f_bytes(2, P.f_varint(1, d)) for d in shape)


def _entry(dtype, shape, shard_id, offset, size, crc):
    msg = P.f_varint(1, dtype) + P.f_bytes(2, _shape_proto(shape))
    if shard_id:
        msg += P.f_varint(3, shard_id)
    if offset:
        msg += P.f_varint(4, offset)
    msg += P.f_varint(5, size) + P.f_fixed32(6, crc)
    return msg


def _tensor_bytes(t):
    t = t.detach()
    if t.device.type != "cpu":
        t = t.cpu()
    t = t.contiguous()
    if t.dtype == torch.bfloat16:
        return t.view(torch.int16).numpy().tobytes()
    return t.numpy().tobytes()


class BundleWriter(object):
    """Write named tensors into ``num_shards`` data files + one index."""

    def __init__(self, prefix, num_shards=1):
        self.prefix = prefix
        self.num_shards = num_shards
        d = os.path.dirname(prefix)
        if d:
            os.makedirs(d, exist_ok=True)
        self._files = [open(data_filename(prefix, s, num_shards) + ".tempstate", "wb") for s in range(num_shards)]
        self._offsets = [0] * num_shards
        self._entries = {}

    def add(self, name, tensor, shard_id=0):
        if name in self._entries:
            raise ValueError("duplicate tensor name %r" % name)
        if not isinstance(tensor, torch.Tensor):
            tensor = torch.as_tensor(np.asarray(tensor))
        dt = _DT_FROM_TORCH.get(tensor.dtype)
        if dt is None:
            raise TypeError("unsupported dtype %s for %s" % (tensor.dtype, name))
        data = _tensor_bytes(tensor)
        crc = native_host.mask(native_host.crc32c(data))
        f = self._files[shard_id]
        f.write(data)
        self._entries[name] = _entry(dt, tuple(tensor.shape), shard_id, self._offsets[shard_id], len(data), crc)
        self._offsets[shard_id] += len(data)

    def finish(self):
        for s, f in enumerate(self._files):
            f.close()
            os.replace(f.name, data_filename(self.prefix, s, self.num_shards))
        tw = TableWriter(self.prefix + ".index.tempstate")
        tw.add(b"", _header(self.num_shards))
        for name in sorted(self._entries, key=lambda n: n.encode()):
            tw.add(name.encode(), self._entries[name])
        tw.finish()
        os.replace(self.prefix + ".index.tempstate", self.prefix + ".index")


class BundleEntry(object):
    __slots__ = ("dtype", "shape", "shard_id", "offset", "size", "crc32c")


def _parse_entry(buf):
    f = P.parse(buf)
    e = BundleEntry()
    e.dtype = f.get(1, [P.DT_FLOAT])[0]
    shape = []
    if 2 in f:
        sp = P.parse(f[2][0])
        for dim in sp.get(2, []):
            shape.append(P.signed64(P.parse(dim).get(1, [0])[0]))
    e.shape = tuple(shape)
    e.shard_id = f.get(3, [0])[0]
    e.offset = f.get(4, [0])[0]
    e.size = f.get(5, [0])[0]
    e.crc32c = f.get(6, [None])[0]
    return e


class BundleReader(object):
    def __init__(self, prefix, verify=True):
        self.prefix = prefix
        self.verify = verify
        table = TableReader(prefix + ".index", verify_checksums=verify)
        self.entries = {}
        self.num_shards = 1
        for k, v in table.items():
            if k == b"":
                h = P.parse(v)
                self.num_shards = h.get(1, [1])[0]
                if h.get(2, [0])[0] != 0:
                    raise ValueError("big-endian bundles are not supported")
            else:
                self.entries[k.decode()] = _parse_entry(v)
        self._data = {}

    def _shard(self, s):
        if s not in self._data:
            path = data_filename(self.prefix, s, self.num_shards)
            self._data[s] = np.memmap(path, dtype=np.uint8, mode="r") if os.path.getsize(path) else np.zeros(0, np.uint8)
        return self._data[s]

    def keys(self):
        return sorted(self.entries)

    def __contains__(self, name):
        return name in self.entries

    def shape(self, name):
        return self.entries[name].shape

    def get_tensor(self, name):
        e = self.entries[name]
        raw = self._shard(e.shard_id)[e.offset:e.offset + e.size]
        buf = raw.tobytes()
        if self.verify and e.crc32c is not None:
            if native_host.mask(native_host.crc32c(buf)) != e.crc32c:
                raise ValueError("checksum mismatch for tensor %s" % name)
        dt = _TORCH_FROM_DT.get(e.dtype)
        if dt is None:
            raise TypeError("unsupported dtype %d for %s" % (e.dtype, name))
        if dt == torch.bfloat16:
            return torch.from_numpy(np.frombuffer(buf, dtype=np.int16).copy()).view(torch.bfloat16).reshape(e.shape)
        np_dt = torch.empty(0, dtype=dt).numpy().dtype
        return torch.from_numpy(np.frombuffer(buf, dtype=np_dt).copy()).reshape(e.shape)


def list_variables(prefix):
    r = BundleReader(prefix, verify=False)
    return [(k, list(r.shape(k))) for k in r.keys()]


def load_variable(prefix, name):
    return BundleReader(prefix).get_tensor(name)
