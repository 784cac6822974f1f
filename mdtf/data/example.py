"""``tf.train.Example`` encode/parse without TF (hand-written protobuf codec).

Reference: ``tf.parse_single_example(serialized, self.features)`` with
``tf.FixedLenFeature([], tf.string / tf.int64)`` (``distribute.py:30-35``,
``distribute_input.py:97-99``).

Message structure: Example{features: Features{feature: map<string, Feature>}},
Feature{oneof bytes_list=1 / float_list=2 / int64_list=3}, lists hold a
repeated ``value`` (floats/ints packed).
"""
import struct

import numpy as np
import torch

from ..ckpt import proto as P

string = "string"
int64 = "int64"
float32 = "float32"


def _norm_dtype(dtype):
    if dtype in (string, "bytes", bytes, str):
        return string
    if dtype in (int64, "int32", torch.int64, torch.int32, np.int64, np.int32, int):
        return int64
    if dtype in (float32, "float", "float64", torch.float32, torch.float64, np.float32, np.float64, float):
        return float32
    raise ValueError("unsupported feature dtype %r" % (dtype,))


class FixedLenFeature(object):
    def __init__(self, shape, dtype, default_value=None):
        self.shape = list(shape)
        self.dtype = _norm_dtype(dtype)
        self.default_value = default_value


class VarLenFeature(object):
    def __init__(self, dtype):
        self.dtype = _norm_dtype(dtype)


# -- encoding -----------------------------------------------------------------
def _feature_bytes(values):
    return P.f_bytes(1, b"".join(P.f_bytes(1, v if isinstance(v, bytes) else str(v).encode()) for v in values))


def _feature_floats(values):
    packed = struct.pack("<%df" % len(values), *values)
    return P.f_bytes(2, P.f_bytes(1, packed))


def _feature_ints(values):
    packed = b"".join(P.varint(int(v)) for v in values)
    return P.f_bytes(3, P.f_bytes(1, packed))


def bytes_feature(v):
    return ("bytes", [v] if isinstance(v, (bytes, str)) else list(v))


def int64_feature(v):
    return ("int64", [int(x) for x in np.asarray(v).reshape(-1)])


def float_feature(v):
    return ("float", [float(x) for x in np.asarray(v, dtype=np.float64).reshape(-1)])


def serialize_example(features):
    """``{name: bytes|int|float|ndarray|(kind, values)}`` -> serialized Example."""
    entries = []
    for name in sorted(features):
        v = features[name]
        if isinstance(v, tuple) and len(v) == 2 and v[0] in ("bytes", "int64", "float"):
            kind, vals = v
        elif isinstance(v, (bytes, str)):
            kind, vals = "bytes", [v]
        else:
            arr = np.asarray(v)
            if arr.dtype.kind in "iub":
                kind, vals = "int64", [int(x) for x in arr.reshape(-1)]
            else:
                kind, vals = "float", [float(x) for x in arr.reshape(-1)]
        feat = {"bytes": _feature_bytes, "int64": _feature_ints, "float": _feature_floats}[kind](vals)
        entry = P.f_bytes(1, name) + P.f_bytes(2, feat)      # map entry {key=1, value=2}
        entries.append(P.f_bytes(1, entry))                    # Features.feature (field 1)
    return P.f_bytes(1, b"".join(entries))                     # Example.features (field 1)


# -- parsing ------------------------------------------------------------------
def _decode_feature(buf):
    f = P.parse(buf)
    if 1 in f:
        return string, list(P.parse(f[1][0]).get(1, [])) if f[1][0] else []
    if 2 in f:
        vals = []
        for item in P.parse(f[2][0]).get(1, []) if f[2][0] else []:
            if isinstance(item, bytes):
                vals.extend(struct.unpack("<%df" % (len(item) // 4), item))
            else:
                vals.append(struct.unpack("<f", struct.pack("<I", item))[0])
        return float32, vals
    if 3 in f:
        vals = []
        for item in P.parse(f[3][0]).get(1, []) if f[3][0] else []:
            if isinstance(item, bytes):
                vals.extend(P.packed_varints(item))
            else:
                vals.append(P.signed64(item))
        return int64, vals
    return None, []


def parse_example_raw(serialized):
    out = {}
    ex = P.parse(serialized)
    for feats in ex.get(1, []):
        for entry in P.parse(feats).get(1, []):
            e = P.parse(entry)
            name = e.get(1, [b""])[0].decode()
            out[name] = _decode_feature(e.get(2, [b""])[0])
    return out


def parse_single_example(serialized, features):
    """Parse with a feature spec -> dict of numpy arrays / bytes."""
    raw = parse_example_raw(serialized)
    out = {}
    for name, spec in features.items():
        if name not in raw:
            if isinstance(spec, FixedLenFeature) and spec.default_value is not None:
                out[name] = np.asarray(spec.default_value)
                continue
            if isinstance(spec, VarLenFeature):
                out[name] = np.zeros((0,), np.int64 if spec.dtype == int64 else np.float32)
                continue
            raise KeyError("feature %r missing from example" % name)
        kind, vals = raw[name]
        if kind is not None and kind != spec.dtype:
            raise TypeError("feature %r: expected %s, got %s" % (name, spec.dtype, kind))
        if spec.dtype == string:
            if isinstance(spec, FixedLenFeature) and not spec.shape:
                out[name] = vals[0]
            else:
                out[name] = list(vals)
            continue
        arr = np.asarray(vals, dtype=np.int64 if spec.dtype == int64 else np.float32)
        if isinstance(spec, FixedLenFeature):
            arr = arr.reshape(spec.shape) if spec.shape else arr.reshape(())
        out[name] = arr
    return out


def decode_raw(b, dtype=np.uint8):
    """``tf.decode_raw``: bytes -> 1-D array."""
    return np.frombuffer(b, dtype=dtype)
