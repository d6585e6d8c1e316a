"""T0: TF on-disk formats written by the native runtime (no TF available: spec-level golden checks)."""
import gzip
import os
import struct

import numpy as np
import torch

from dtfe import ckpt
from dtfe.utils import native


def rt():
    return native.rt()


def test_crc32c_known_vectors():
    # RFC 3720 / iSCSI test vectors
    assert rt().crc32c(b"123456789") == 0xE3069283
    assert rt().crc32c(b"\x00" * 32) == 0x8A9136AA
    assert rt().crc32c(b"\xff" * 32) == 0x62A8AB43
    c = rt().crc32c(b"hello")
    masked = rt().masked_crc32c(b"hello")
    assert masked == ((((c >> 15) | (c << 17)) & 0xFFFFFFFF) + 0xA282EAD8) & 0xFFFFFFFF


def test_sstable_roundtrip_multi_block():
    kv = sorted((("key%05d" % i).encode(), os.urandom(i % 50)) for i in range(1000))
    blob = rt().sstable_build(kv, 512)  # tiny blocks -> many data blocks + restarts
    assert struct.unpack("<Q", blob[-8:])[0] == 0xDB4775248B80FB57
    back = rt().sstable_parse(blob)
    assert [(bytes(k), bytes(v)) for k, v in back] == kv


def test_bundle_roundtrip_and_layout(tmp_path):
    prefix = str(tmp_path / "model.ckpt-7")
    tensors = {
        "Variable": torch.randn(3, 4),
        "Variable_1": torch.arange(5, dtype=torch.int32),
        "global_step": torch.tensor(7, dtype=torch.int64),
        "rnn/basic_lstm_cell/kernel": torch.randn(6, 8),
        "bf": torch.randn(4).to(torch.bfloat16),
    }
    ckpt.save_bundle(prefix, tensors)
    for suf in (".index", ".data-00000-of-00001", ".meta"):
        assert os.path.exists(prefix + suf)
    back = ckpt.load_bundle(prefix)
    assert set(back) == set(tensors)
    for k, v in tensors.items():
        assert back[k].dtype == v.dtype and torch.equal(back[k], v), k
    # the data file is the tensors concatenated in sorted-key order
    data = open(prefix + ".data-00000-of-00001", "rb").read()
    exp = b"".join(ckpt._tensor_bytes(tensors[k]) for k in sorted(tensors))
    assert data == exp
    # index: first entry is the empty-key BundleHeaderProto {num_shards: 1, version {producer: 1}}
    entries = rt().sstable_parse(open(prefix + ".index", "rb").read())
    assert bytes(entries[0][0]) == b""
    hdr = rt().pb_parse(entries[0][1])
    assert (1, 0, 1, b"") in [(f, w, v, bytes(s)) for f, w, v, s in hdr]
    ver = [bytes(s) for f, w, v, s in hdr if f == 3][0]
    assert rt().pb_parse(ver)[0][:3] == (1, 0, 1)
    # entry: dtype DT_FLOAT=1, shape dims, offset/size, masked crc32c of the bytes
    idx = rt().read_bundle_index(prefix)
    dt, shape, off, size, crc, slices = idx["Variable"]
    assert dt == 1 and list(shape) == [3, 4] and size == 48 and slices == []
    assert crc == rt().crc32c(ckpt._tensor_bytes(tensors["Variable"]))
    # corrupting the data file is detected by the crc
    with open(prefix + ".data-00000-of-00001", "r+b") as f:
        f.seek(0)
        f.write(b"\x00\x00\x00\x01")
    try:
        ckpt.load_bundle(prefix)
        raise AssertionError("crc mismatch not detected")
    except RuntimeError as e:
        assert "crc" in str(e)


def test_saver_max_to_keep_and_state_file(tmp_path):
    d = str(tmp_path)
    s = ckpt.Saver(d, max_to_keep=5)
    for gs in range(0, 70, 10):
        s.save({"Variable": torch.full((2,), float(gs))}, gs)
    latest, allp = ckpt.read_checkpoint_state(d)
    assert latest.endswith("model.ckpt-60")
    assert [os.path.basename(p) for p in allp] == ["model.ckpt-%d" % g for g in (20, 30, 40, 50, 60)]
    assert not os.path.exists(os.path.join(d, "model.ckpt-0.index"))
    assert not os.path.exists(os.path.join(d, "model.ckpt-10.index"))
    text = open(os.path.join(d, "checkpoint")).read().splitlines()
    assert text[0].startswith("model_checkpoint_path: ") and len(text) == 6
    assert ckpt.latest_checkpoint(d).endswith("model.ckpt-60")
    assert float(s.restore()["Variable"][0]) == 60.0
    # a new Saver on the same dir continues the retention list
    s2 = ckpt.Saver(d, max_to_keep=5)
    s2.save({"Variable": torch.zeros(2)}, 70)
    _, allp = ckpt.read_checkpoint_state(d)
    assert len(allp) == 5 and allp[-1].endswith("model.ckpt-70")


def test_events_file(tmp_path):
    w = ckpt.EventWriter(str(tmp_path))
    w.add_scalars(10, {"global_step/sec": 12.5, "loss": 0.25})
    w.add_graph_of_variables([("Variable", ckpt.DT_FLOAT, [3, 4])])
    w.close()
    assert os.path.basename(w.path).startswith("events.out.tfevents.")
    recs = rt().read_tfrecords(w.path)
    assert len(recs) == 3
    first = {f: (v, bytes(s)) for f, _w, v, s in rt().pb_parse(recs[0])}
    assert first[3][1] == b"brain.Event:2"
    ev = {f: (v, bytes(s)) for f, _w, v, s in rt().pb_parse(recs[1])}
    assert ev[2][0] == 10
    vals = [bytes(s) for f, _w, v, s in rt().pb_parse(ev[5][1])]
    tags = []
    for v in vals:
        fields = {f: (vv, bytes(s)) for f, _w, vv, s in rt().pb_parse(v)}
        tags.append((fields[1][1].decode(), struct.unpack("<f", struct.pack("<I", fields[2][0]))[0]))
    assert tags == [("global_step/sec", 12.5), ("loss", 0.25)]


def test_graph_pbtxt(tmp_path):
    ckpt.write_graph_pbtxt(str(tmp_path), [("Variable", ckpt.DT_FLOAT, [784, 256])])
    t = open(tmp_path / "graph.pbtxt").read()
    assert 'name: "Variable"' in t and "size: 784" in t and "DT_FLOAT" in t


def _write_idx(path, arr):
    hdr = bytes([0, 0, 8, arr.ndim]) + b"".join(struct.pack(">I", d) for d in arr.shape)
    with gzip.open(path, "wb") as f:
        f.write(hdr + arr.astype(np.uint8).tobytes())


def test_idx_reader(tmp_path):
    a = np.random.randint(0, 256, size=(7, 28, 28), dtype=np.uint8)
    p = str(tmp_path / "train-images-idx3-ubyte.gz")
    _write_idx(p, a)
    b = rt().idx_read(p)
    assert b.shape == (7, 28, 28) and (b == a).all()


def test_epoch_batcher_semantics():
    b = rt().EpochBatcher(10, 123)
    first = np.concatenate([b.next(3), b.next(3), b.next(3)])
    assert len(set(first.tolist())) == 9          # no repeats inside an epoch
    stitched = b.next(3)                           # 1 from epoch 0 + 2 from epoch 1
    assert b.epochs_completed == 1
    assert stitched[0] not in first
    assert len(stitched) == 3
