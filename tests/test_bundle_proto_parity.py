"""Pin mdtf's tensor-bundle V2 checkpoint encoding against TensorFlow's wire format
without TensorFlow (reference distribute_train.py:171,175 — Scaffold/Saver
into checkpoint_dir).

Everything mdtf wrote is decoded by code independent of mdtf.ckpt:
* the ``.index`` SSTable by a LevelDB-table parser written here from the format spec
  (footer = metaindex/index BlockHandles + 0xdb4775248b80fb57 magic; prefix-compressed block
  entries; masked CRC32C block trailers, CRC32C implemented here bit by bit);
* every index value by ``google.protobuf`` dynamic messages built from TensorFlow's field
  numbers (tensor_bundle.proto BundleHeaderProto / BundleEntryProto, tensor_shape.proto,
  versions.proto VersionDef, checkpoint_state.proto CheckpointState via text_format).
TF's own byte output is not available here, so parity is to the published schemas.
"""
import os
import struct

import numpy as np
import pytest
import torch

pb = pytest.importorskip("google.protobuf")
from google.protobuf import descriptor_pb2, descriptor_pool, message_factory, text_format  # noqa: E402

# ---------------------------------------------------------------- independent CRC32C
_POLY = 0x82F63B78
_TABLE = []
for _i in range(256):
    _c = _i
    for _ in range(8):
        _c = (_c >> 1) ^ _POLY if _c & 1 else _c >> 1
    _TABLE.append(_c)


def crc32c(data):
    c = 0xFFFFFFFF
    for b in data:
        c = _TABLE[(c ^ b) & 0xFF] ^ (c >> 8)
    return c ^ 0xFFFFFFFF


def masked(crc):
    return (((crc >> 15) | (crc << 17)) + 0xA282EAD8) & 0xFFFFFFFF


# ---------------------------------------------------------------- independent SSTable parser
def _varint(buf, pos):
    shift = val = 0
    while True:
        b = buf[pos]
        pos += 1
        val |= (b & 0x7F) << shift
        if not b & 0x80:
            return val, pos
        shift += 7


def _block(data, handle):
    off, p = _varint(handle, 0)
    size, _ = _varint(handle, p)
    contents = data[off:off + size]
    ctype = data[off + size]
    assert ctype == 0, "uncompressed blocks expected"
    (stored,) = struct.unpack_from("<I", data, off + size + 1)
    assert stored == masked(crc32c(contents + bytes([ctype]))), "block CRC"
    nrest = struct.unpack_from("<I", contents, len(contents) - 4)[0]
    end = len(contents) - 4 - 4 * nrest
    out, pos, key = [], 0, b""
    while pos < end:
        shared, pos = _varint(contents, pos)
        nons, pos = _varint(contents, pos)
        vlen, pos = _varint(contents, pos)
        key = key[:shared] + contents[pos:pos + nons]
        pos += nons
        out.append((key, contents[pos:pos + vlen]))
        pos += vlen
    return out


def read_table(path):
    data = open(path, "rb").read()
    footer = data[-48:]
    assert struct.unpack_from("<Q", footer, 40)[0] == 0xDB4775248B80FB57
    _, p = _varint(footer, 0)           # metaindex offset
    _, p = _varint(footer, p)           # metaindex size
    io, p = _varint(footer, p)
    isz, _ = _varint(footer, p)
    def enc(v):
        out = bytearray()
        while True:
            b = v & 0x7F
            v >>= 7
            out.append(b | (0x80 if v else 0))
            if not v:
                return bytes(out)
    entries = []
    for _, h in _block(data, enc(io) + enc(isz)):
        entries.extend(_block(data, h))
    keys = [k for k, _ in entries]
    assert keys == sorted(keys), "sstable keys must be sorted bytewise"
    return entries


# ---------------------------------------------------------------- TF schemas as dynamic messages
def _messages():
    fdp = descriptor_pb2.FileDescriptorProto(name="mdtf_tf_schema_pin.proto", package="tfpin", syntax="proto3")
    F = descriptor_pb2.FieldDescriptorProto

    def msg(name, fields, nested=()):
        m = fdp.message_type.add(name=name)
        for n in nested:
            m.nested_type.add().CopyFrom(n)
        for fname, num, ftype, label, tname in fields:
            f = m.field.add(name=fname, number=num, type=ftype, label=label)
            if tname:
                f.type_name = tname
        return m

    opt, rep = F.LABEL_OPTIONAL, F.LABEL_REPEATED
    dim = descriptor_pb2.DescriptorProto(name="Dim")
    dim.field.add(name="size", number=1, type=F.TYPE_INT64, label=opt)
    dim.field.add(name="name", number=2, type=F.TYPE_STRING, label=opt)
    msg("TensorShapeProto", [("dim", 2, F.TYPE_MESSAGE, rep, ".tfpin.TensorShapeProto.Dim"),
                             ("unknown_rank", 3, F.TYPE_BOOL, opt, None)], nested=[dim])
    msg("VersionDef", [("producer", 1, F.TYPE_INT32, opt, None), ("min_consumer", 2, F.TYPE_INT32, opt, None),
                       ("bad_consumers", 3, F.TYPE_INT32, rep, None)])
    msg("BundleHeaderProto", [("num_shards", 1, F.TYPE_INT32, opt, None), ("endianness", 2, F.TYPE_INT32, opt, None),
                              ("version", 3, F.TYPE_MESSAGE, opt, ".tfpin.VersionDef")])
    msg("BundleEntryProto", [("dtype", 1, F.TYPE_INT32, opt, None),
                             ("shape", 2, F.TYPE_MESSAGE, opt, ".tfpin.TensorShapeProto"),
                             ("shard_id", 3, F.TYPE_INT32, opt, None), ("offset", 4, F.TYPE_INT64, opt, None),
                             ("size", 5, F.TYPE_INT64, opt, None), ("crc32c", 6, F.TYPE_FIXED32, opt, None)])
    msg("CheckpointState", [("model_checkpoint_path", 1, F.TYPE_STRING, opt, None),
                            ("all_model_checkpoint_paths", 2, F.TYPE_STRING, rep, None),
                            ("all_model_checkpoint_timestamps", 3, F.TYPE_DOUBLE, rep, None),
                            ("last_preserved_timestamp", 4, F.TYPE_DOUBLE, opt, None)])
    pool = descriptor_pool.DescriptorPool()
    pool.Add(fdp)
    get = lambda n: message_factory.GetMessageClass(pool.FindMessageTypeByName("tfpin." + n))  # noqa: E731
    return {n: get(n) for n in ("BundleHeaderProto", "BundleEntryProto", "CheckpointState")}


DT_FLOAT, DT_INT32, DT_INT64, DT_BFLOAT16, DT_HALF = 1, 3, 9, 14, 19   # tensorflow/core/framework/types.proto


def test_bundle_index_and_data_decode_with_tf_schema(tmp_path):
    from mdtf.ckpt.tensor_bundle import BundleWriter
    M = _messages()
    g = torch.Generator().manual_seed(0)
    tensors = {
        "conv1/weights": (torch.randn(3, 3, 8, 16, generator=g), 0, DT_FLOAT),
        "conv1/weights/Momentum": (torch.randn(3, 3, 8, 16, generator=g), 1, DT_FLOAT),
        "global_step": (torch.tensor(1234, dtype=torch.int64), 0, DT_INT64),
        "bn/moving_mean": (torch.randn(16, generator=g).to(torch.bfloat16), 1, DT_BFLOAT16),
        "ids": (torch.arange(7, dtype=torch.int32), 0, DT_INT32),
        "half": (torch.randn(2, 5, generator=g).half(), 1, DT_HALF),
        "scalar": (torch.tensor(0.5), 0, DT_FLOAT),
    }
    prefix = str(tmp_path / "model.ckpt-1234")
    w = BundleWriter(prefix, num_shards=2)
    for name, (t, shard, _) in tensors.items():
        w.add(name, t, shard)
    w.finish()

    entries = read_table(prefix + ".index")
    assert entries[0][0] == b""                           # the header sorts first
    hdr = M["BundleHeaderProto"].FromString(entries[0][1])
    assert hdr.num_shards == 2 and hdr.endianness == 0 and hdr.version.producer == 1
    by_name = {k.decode(): M["BundleEntryProto"].FromString(v) for k, v in entries[1:]}
    assert set(by_name) == set(tensors)
    shards = [open("%s.data-%05d-of-%05d" % (prefix, s, 2), "rb").read() for s in range(2)]
    for name, (t, shard, dt) in tensors.items():
        e = by_name[name]
        assert e.dtype == dt, name
        assert [d.size for d in e.shape.dim] == list(t.shape), name
        assert e.shard_id == shard
        raw = shards[shard][e.offset:e.offset + e.size]
        assert e.crc32c == masked(crc32c(raw)), name     # TF stores the MASKED crc32c of the bytes
        ref = (t.view(torch.int16) if t.dtype == torch.bfloat16 else t).numpy()
        assert np.frombuffer(raw, dtype=ref.dtype.newbyteorder("<")).tobytes() == ref.astype(
            ref.dtype.newbyteorder("<")).tobytes(), name
        assert e.size == ref.nbytes
    # each shard file is exactly the concatenation of its tensors (no headers / padding)
    for s in range(2):
        assert len(shards[s]) == sum(by_name[n].size for n, (_, sh, _) in tensors.items() if sh == s)


def test_checkpoint_state_parses_as_tf_text_proto(tmp_path):
    from mdtf.ckpt.checkpoint_state import write_state
    M = _messages()
    d = str(tmp_path)
    write_state(d, os.path.join(d, "model.ckpt-20"), [os.path.join(d, "model.ckpt-10"), os.path.join(d, "model.ckpt-20")])
    st = text_format.Parse(open(os.path.join(d, "checkpoint")).read(), M["CheckpointState"]())
    assert st.model_checkpoint_path == "model.ckpt-20"            # relative to the directory, as TF writes
    assert list(st.all_model_checkpoint_paths) == ["model.ckpt-10", "model.ckpt-20"]


def test_saver_checkpoint_decodes_with_tf_schema(tmp_path):
    """A real Saver.save of a trained model: every entry decodes, TF slot names and dtypes."""
    import sys
    sys.path.insert(0, os.path.dirname(__file__))
    import dist_helpers
    import mdtf
    from mdtf.train import step as S
    from mdtf.train import variables as V
    V.reset_default_graph()
    S.reset()
    Lin, MSE, xs, ys, x_ph, y_ph, Tower, Net = dist_helpers._linear_setup(0, 1, 4)
    opt = mdtf.train.AdamOptimizer(0.01)
    tg = []
    Tower(Net(Lin()), "tower_0/", tg, x_ph, y_ph, MSE(), opt, batch_size=4).process()
    gs = mdtf.train.get_or_create_global_step()
    op = opt.apply_gradients(Tower.average_gradients(tg), global_step=gs)
    sess = mdtf.train.MonitoredTrainingSession(log_step_count_steps=0)
    for _ in range(2):
        sess.run(op, feed_dict={x_ph: xs, y_ph: ys})
    prefix = mdtf.train.Saver().save(sess, str(tmp_path / "model.ckpt"), global_step=gs)
    M = _messages()
    names = {k.decode(): M["BundleEntryProto"].FromString(v) for k, v in read_table(prefix + ".index")[1:]}
    assert names["dense/w"].dtype == DT_FLOAT and [d.size for d in names["dense/w"].shape.dim] == [8, 3]
    for slot in ("dense/w/Adam", "dense/w/Adam_1", "dense/b/Adam", "dense2/w/Adam_1"):
        assert names[slot].dtype == DT_FLOAT, slot
    assert names["beta1_power"].dtype == DT_FLOAT and list(names["beta1_power"].shape.dim) == []
    assert names["global_step"].dtype == DT_INT64 and list(names["global_step"].shape.dim) == []
    data = open(prefix + ".data-00000-of-00001", "rb").read()
    e = names["global_step"]
    assert struct.unpack("<q", data[e.offset:e.offset + 8])[0] == 2
