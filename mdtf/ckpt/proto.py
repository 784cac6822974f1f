"""Minimal protobuf wire-format codec (no generated code, no TF).

Enough to read/write the messages the framework needs to stay
TF-checkpoint/TFRecord compatible: ``BundleHeaderProto``,
``BundleEntryProto``/``TensorShapeProto`` (tensor bundles) and
``tf.train.Example`` / ``Features`` / ``Feature`` (TFRecord inputs).
"""
import struct


def varint(v):
    if v < 0:
        v += 1 << 64
    out = bytearray()
    while True:
        b = v & 0x7F
        v >>= 7
        if v:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def read_varint(buf, pos):
    shift = 0
    result = 0
    while True:
        b = buf[pos]
        pos += 1
        result |= (b & 0x7F) << shift
        if not b & 0x80:
            return result, pos
        shift += 7
        if shift > 63:
            raise ValueError("varint too long")


def key(field, wire):
    return varint((field << 3) | wire)


def f_varint(field, v):
    return key(field, 0) + varint(int(v))


def f_bytes(field, b):
    if isinstance(b, str):
        b = b.encode()
    return key(field, 2) + varint(len(b)) + b


def f_fixed32(field, v):
    return key(field, 5) + struct.pack("<I", v & 0xFFFFFFFF)


def f_fixed64(field, v):
    return key(field, 1) + struct.pack("<Q", v)


def parse(buf):
    """Decode a message into {field: [values]} (raw: ints or bytes)."""
    out = {}
    pos = 0
    n = len(buf)
    while pos < n:
        k, pos = read_varint(buf, pos)
        field, wire = k >> 3, k & 7
        if wire == 0:
            v, pos = read_varint(buf, pos)
        elif wire == 1:
            v = struct.unpack_from("<Q", buf, pos)[0]
            pos += 8
        elif wire == 2:
            ln, pos = read_varint(buf, pos)
            v = bytes(buf[pos:pos + ln])
            pos += ln
        elif wire == 5:
            v = struct.unpack_from("<I", buf, pos)[0]
            pos += 4
        else:
            raise ValueError("unsupported wire type %d" % wire)
        out.setdefault(field, []).append(v)
    return out


def signed64(v):
    return v - (1 << 64) if v >= (1 << 63) else v


def packed_varints(b):
    vals, pos = [], 0
    while pos < len(b):
        v, pos = read_varint(b, pos)
        vals.append(signed64(v))
    return vals


# ---------------------------------------------------------------------------
# tensorflow/core/framework/types.proto DataType
DT_FLOAT, DT_DOUBLE, DT_INT32, DT_UINT8, DT_INT16, DT_INT8, DT_STRING = 1, 2, 3, 4, 5, 6, 7
DT_INT64, DT_BOOL, DT_BFLOAT16, DT_HALF = 9, 10, 14, 19
