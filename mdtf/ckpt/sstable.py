"""LevelDB-format SSTable writer/reader (the format of a TF bundle ``.index``).

Layout written (uncompressed, TF's ``table::TableBuilder`` conventions):

  [data block]* [metaindex block] [index block] [footer 48 B]

* block: prefix-compressed entries ``varint shared | varint non_shared |
  varint value_len | key_delta | value``, restart point every 16 entries,
  then ``uint32 restarts[]`` and ``uint32 num_restarts``; each block is followed
  by a 5-byte trailer: compression type (0) + masked CRC32C(block + type);
* index block: one entry per data block, key ≥ last key of the block,
  value = BlockHandle (varint64 offset, varint64 size);
* footer: metaindex handle + index handle, zero padded to 40 bytes, then the
  magic ``0xdb4775248b80fb57`` (little-endian fixed64).
"""
import struct

from ..utils import native_host
from .proto import read_varint, varint

MAGIC = 0xdb4775248b80fb57
FOOTER_LEN = 48
RESTART_INTERVAL = 16
BLOCK_SIZE = 256 << 10


class _BlockBuilder(object):
    def __init__(self, restart_interval=RESTART_INTERVAL):
        self.buf = bytearray()
        self.restarts = [0]
        self.counter = 0
        self.last_key = b""
        self.interval = restart_interval

    def add(self, key, value):
        shared = 0
        if self.counter < self.interval:
            m = min(len(self.last_key), len(key))
            while shared < m and self.last_key[shared] == key[shared]:
                shared += 1
        else:
            self.restarts.append(len(self.buf))
            self.counter = 0
        self.buf += varint(shared) + varint(len(key) - shared) + varint(len(value))
        self.buf += key[shared:] + value
        self.last_key = key
        self.counter += 1

    def finish(self):
        out = bytes(self.buf) + b"".join(struct.pack("<I", r) for r in self.restarts)
        return out + struct.pack("<I", len(self.restarts))

    def size_estimate(self):
        return len(self.buf) + 4 * len(self.restarts) + 4

    def empty(self):
        return not self.buf


class TableWriter(object):
    def __init__(self, path):
        self.f = open(path, "wb")
        self.offset = 0
        self.block = _BlockBuilder()
        self.index = _BlockBuilder(restart_interval=1)
        self.last_key = None
        self.pending_handle = None

    def _write_block(self, contents):
        trailer_type = b"\x00"
        crc = native_host.mask(native_host.crc32c(contents + trailer_type))
        handle = (self.offset, len(contents))
        self.f.write(contents + trailer_type + struct.pack("<I", crc))
        self.offset += len(contents) + 5
        return handle

    def add(self, key, value):
        if isinstance(key, str):
            key = key.encode()
        if self.last_key is not None and key <= self.last_key:
            raise ValueError("keys must be added in strictly increasing order: %r after %r" % (key, self.last_key))
        if self.pending_handle is not None:
            self.index.add(self.last_key, varint(self.pending_handle[0]) + varint(self.pending_handle[1]))
            self.pending_handle = None
        self.block.add(key, value)
        self.last_key = key
        if self.block.size_estimate() >= BLOCK_SIZE:
            self._flush()

    def _flush(self):
        if self.block.empty():
            return
        self.pending_handle = self._write_block(self.block.finish())
        self.block = _BlockBuilder()

    def finish(self):
        self._flush()
        if self.pending_handle is not None:
            self.index.add(self.last_key, varint(self.pending_handle[0]) + varint(self.pending_handle[1]))
            self.pending_handle = None
        meta = self._write_block(_BlockBuilder().finish())
        idx = self._write_block(self.index.finish())
        footer = varint(meta[0]) + varint(meta[1]) + varint(idx[0]) + varint(idx[1])
        footer += b"\x00" * (40 - len(footer))
        footer += struct.pack("<II", MAGIC & 0xFFFFFFFF, MAGIC >> 32)
        self.f.write(footer)
        self.f.close()


def _read_block_entries(data):
    num_restarts = struct.unpack_from("<I", data, len(data) - 4)[0]
    limit = len(data) - 4 - 4 * num_restarts
    pos = 0
    key = b""
    out = []
    while pos < limit:
        shared, pos = read_varint(data, pos)
        non_shared, pos = read_varint(data, pos)
        vlen, pos = read_varint(data, pos)
        key = key[:shared] + bytes(data[pos:pos + non_shared])
        pos += non_shared
        out.append((key, bytes(data[pos:pos + vlen])))
        pos += vlen
    return out


class TableReader(object):
    def __init__(self, path, verify_checksums=True):
        with open(path, "rb") as f:
            self.data = f.read()
        self.verify = verify_checksums
        if len(self.data) < FOOTER_LEN:
            raise ValueError("%s: file too short to be an sstable" % path)
        footer = self.data[-FOOTER_LEN:]
        lo, hi = struct.unpack_from("<II", footer, 40)
        if (hi << 32 | lo) != MAGIC:
            raise ValueError("%s: bad sstable magic" % path)
        pos = 0
        _, pos = read_varint(footer, pos)
        _, pos = read_varint(footer, pos)
        io, pos = read_varint(footer, pos)
        isz, pos = read_varint(footer, pos)
        self.index = _read_block_entries(self._block(io, isz))

    def _block(self, off, size):
        contents = self.data[off:off + size]
        if self.verify:
            trailer = self.data[off + size:off + size + 5]
            if trailer[0] != 0:
                raise ValueError("compressed sstable blocks are not supported")
            crc = struct.unpack_from("<I", trailer, 1)[0]
            if native_host.mask(native_host.crc32c(contents + trailer[:1])) != crc:
                raise ValueError("sstable block checksum mismatch at offset %d" % off)
        return contents

    def items(self):
        for _, handle in self.index:
            off, pos = read_varint(handle, 0)
            size, _ = read_varint(handle, pos)
            for kv in _read_block_entries(self._block(off, size)):
                yield kv
