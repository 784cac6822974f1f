"""Native host I/O: CRC32C, TFRecord framing, tf.Example codec, tensor bundles, loaders."""
import os

import numpy as np
import pytest
import torch

from mdtf.ckpt import checkpoint_state as CS
from mdtf.ckpt.sstable import TableReader, TableWriter
from mdtf.ckpt.tensor_bundle import BundleReader, BundleWriter, list_variables
from mdtf.data import example as E
from mdtf.data import tfrecord as TFR
from mdtf.utils import native_host


def test_crc32c_known_vectors():
    # RFC 3720 test vectors
    assert native_host.crc32c(b"") == 0
    assert native_host.crc32c(b"123456789") == 0xE3069283
    assert native_host.crc32c(bytes(32)) == 0x8A9136AA
    assert native_host.crc32c(bytes([0xFF] * 32)) == 0x62A8AB43
    assert native_host.crc32c(bytes(range(32))) == 0x46DD794E
    big = os.urandom(100003)
    assert native_host.crc32c(big) == native_host.crc32c(big[:50000] + big[50000:])
    m = native_host.mask(0x12345678)
    assert native_host.unmask(m) == 0x12345678


def test_crc_native_vs_python_fallback():
    data = os.urandom(1000)
    native = native_host.crc32c(data)
    saved = native_host._lib
    native_host._lib = None
    try:
        path = native_host.LIB_PATH
        native_host.LIB_PATH = "/nonexistent"
        assert native_host.crc32c(data) == native
    finally:
        native_host.LIB_PATH = path
        native_host._lib = saved


def test_tfrecord_roundtrip_and_corruption(tmp_path):
    p = str(tmp_path / "a.tfrecord")
    recs = [os.urandom(n) for n in (0, 1, 100, 4096)]
    with TFR.TFRecordWriter(p) as w:
        for r in recs:
            w.write(r)
    assert list(TFR.tf_record_iterator(p)) == recs
    data = bytearray(open(p, "rb").read())
    data[20] ^= 0xFF
    open(p, "wb").write(bytes(data))
    with pytest.raises(IOError):
        list(TFR.tf_record_iterator(p))


def test_example_codec():
    img = np.arange(12, dtype=np.uint8).tobytes()
    ser = E.serialize_example({"image_raw": img, "height": 3, "width": np.int64(4), "vals": np.array([1.5, -2.0]),
                               "neg": -7})
    feats = {"image_raw": E.FixedLenFeature([], E.string), "height": E.FixedLenFeature([], E.int64),
             "width": E.FixedLenFeature([], E.int64), "vals": E.FixedLenFeature([2], E.float32),
             "neg": E.FixedLenFeature([], E.int64), "missing": E.FixedLenFeature([], E.int64, default_value=9)}
    out = E.parse_single_example(ser, feats)
    assert out["image_raw"] == img and int(out["height"]) == 3 and int(out["width"]) == 4
    assert np.allclose(out["vals"], [1.5, -2.0]) and int(out["neg"]) == -7 and int(out["missing"]) == 9
    assert np.array_equal(E.decode_raw(out["image_raw"]), np.arange(12, dtype=np.uint8))


def test_sstable_roundtrip(tmp_path):
    p = str(tmp_path / "t.sst")
    w = TableWriter(p)
    keys = sorted("key%05d" % i for i in range(3000))
    for k in keys:
        w.add(k, (k * 3).encode())
    w.finish()
    got = list(TableReader(p).items())
    assert [k.decode() for k, _ in got] == keys
    assert got[123][1] == (keys[123] * 3).encode()
    with pytest.raises(ValueError):
        TableWriter(str(tmp_path / "u.sst")).add("b", b"") or None
        w2 = TableWriter(str(tmp_path / "v.sst"))
        w2.add("b", b"")
        w2.add("a", b"")


def test_tensor_bundle_roundtrip(tmp_path):
    prefix = str(tmp_path / "model.ckpt-7")
    tensors = {"conv1/weights": torch.randn(3, 3, 2, 4), "global_step": torch.tensor(7, dtype=torch.int64),
               "fc/biases": torch.randn(10), "bf": torch.randn(5).bfloat16(), "i32": torch.arange(6, dtype=torch.int32)}
    w = BundleWriter(prefix, num_shards=2)
    for i, (k, v) in enumerate(sorted(tensors.items())):
        w.add(k, v, shard_id=i % 2)
    w.finish()
    assert os.path.exists(prefix + ".index") and os.path.exists(prefix + ".data-00001-of-00002")
    r = BundleReader(prefix)
    assert r.num_shards == 2
    for k, v in tensors.items():
        assert torch.equal(r.get_tensor(k), v)
    assert dict(list_variables(prefix))["conv1/weights"] == [3, 3, 2, 4]
    # corrupt a data byte -> checksum error
    d = prefix + ".data-00000-of-00002"
    b = bytearray(open(d, "rb").read())
    b[0] ^= 1
    open(d, "wb").write(bytes(b))
    with pytest.raises(ValueError):
        for k in tensors:
            BundleReader(prefix).get_tensor(k)


def test_checkpoint_state_file(tmp_path):
    d = str(tmp_path)
    CS.write_state(d, os.path.join(d, "model.ckpt-20"), [os.path.join(d, "model.ckpt-10"),
                                                          os.path.join(d, "model.ckpt-20")])
    txt = open(os.path.join(d, "checkpoint")).read()
    assert 'model_checkpoint_path: "model.ckpt-20"' in txt
    st = CS.read_state(d)
    assert st["all_model_checkpoint_paths"][0].endswith("model.ckpt-10")
    assert CS.latest_checkpoint(d) is None      # no .index yet
    open(os.path.join(d, "model.ckpt-20.index"), "w").close()
    assert CS.latest_checkpoint(d).endswith("model.ckpt-20")


def test_native_shuffled_loader(tmp_path):
    files = []
    for f in range(3):
        p = str(tmp_path / ("f%d.tfrecord" % f))
        with TFR.TFRecordWriter(p) as w:
            for i in range(50):
                w.write(("%d-%d" % (f, i)).encode() * (1 + i % 7))
        files.append(p)
    ld = TFR.ShuffledRecordLoader(files, epochs=1, shuffle=True, capacity=32, num_threads=3, seed=1)
    got = list(ld)
    ld.close()
    assert len(got) == 150 and len(set(got)) == 150
    ld = TFR.ShuffledRecordLoader(files, epochs=2, shuffle=False, capacity=8, num_threads=1)
    assert len(list(ld)) == 300
