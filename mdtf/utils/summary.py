"""Scalar summaries (``tf.summary.scalar``) and a TensorBoard event writer.

The reference records per-tower loss scalars with the ``tower_N/`` prefix
stripped (``distribute_tower.py:139-143``) and lets the chief's
SummarySaverHook write them.  ``scalar()`` records a (detached) value for the
current step; :class:`FileWriter` appends them to ``events.out.tfevents.*``
files (TFRecord-framed ``Event`` protos — readable by TensorBoard) and to a
``summaries.jsonl`` side file.
"""
import json
import os
import re
import socket
import struct
import time

import torch

from ..ckpt import proto as P
from ..config import constants
from . import native_host

_STEP_SCALARS = {}


def _strip_tower(name):
    return re.sub('%s_[0-9]*/' % constants.TOWER_NAME, '', name)


def scalar(name, tensor, collections=None):
    """Record a scalar for this step (device tensors are synced only when written)."""
    if isinstance(tensor, torch.Tensor):
        tensor = tensor.detach()
    _STEP_SCALARS[_strip_tower(name)] = tensor
    return tensor


def collect_step_scalars():
    out = {}
    for k, v in _STEP_SCALARS.items():
        out[k] = float(v) if not isinstance(v, torch.Tensor) else float(v.float().item())
    return out


def _frame(data):
    hdr = struct.pack("<Q", len(data))
    return (hdr + struct.pack("<I", native_host.masked_crc32c(hdr)) + data +
            struct.pack("<I", native_host.masked_crc32c(data)))


def _event(wall_time, step, summary=None, file_version=None):
    msg = P.key(1, 1) + struct.pack("<d", wall_time) + P.f_varint(2, step)
    if file_version is not None:
        msg += P.f_bytes(3, file_version)
    if summary is not None:
        msg += P.f_bytes(5, summary)
    return msg


def _scalar_summary(tag, value):
    val = P.f_bytes(1, tag) + P.key(2, 5) + struct.pack("<f", float(value))   # Summary.Value{tag, simple_value}
    return P.f_bytes(1, val)                                                  # Summary{value}


class FileWriter(object):
    def __init__(self, logdir):
        os.makedirs(logdir, exist_ok=True)
        self.logdir = logdir
        fname = "events.out.tfevents.%d.%s" % (int(time.time()), socket.gethostname())
        self._f = open(os.path.join(logdir, fname), "ab")
        self._json = open(os.path.join(logdir, "summaries.jsonl"), "a")
        self._f.write(_frame(_event(time.time(), 0, file_version=b"brain.Event:2")))

    def add_scalar(self, tag, value, step):
        self._f.write(_frame(_event(time.time(), int(step), summary=_scalar_summary(tag, value))))
        self._json.write(json.dumps({"step": int(step), "tag": tag, "value": float(value)}) + "\n")

    def flush(self):
        self._f.flush()
        self._json.flush()

    def close(self):
        if not self._f.closed:
            self._f.close()
            self._json.close()


def read_events(path):
    """Yield (step, tag, value) from an event file (tests / tooling)."""
    with open(path, "rb") as f:
        data = f.read()
    pos = 0
    while pos + 12 <= len(data):
        n = struct.unpack_from("<Q", data, pos)[0]
        rec = data[pos + 12:pos + 12 + n]
        pos += 12 + n + 4
        ev = P.parse(rec)
        step = ev.get(2, [0])[0]
        for summ in ev.get(5, []):
            for val in P.parse(summ).get(1, []):
                vf = P.parse(val)
                tag = vf.get(1, [b""])[0].decode()
                v = struct.unpack("<f", struct.pack("<I", vf.get(2, [0])[0]))[0]
                yield step, tag, v
