"""Partitioned variables of the ps mode (--ps_partition_mb; parallel/partition.py): names, sizes,
round-robin placement of the parts, optimizer var lists, the TF tensor-slice checkpoint layout
(BundleEntryProto.slices + EncodeTensorNameSlice keys) and a partitioned 2-ps cluster whose
checkpoint restores with and without partitioning.  Parity with TF is unpinned (no TF in this
image, no checkpoint fixtures in the reference): the slice keys are checked against the
OrderedCode rules written out by hand below."""
import os

import pytest
import torch

from dtfe import ckpt
from dtfe.models.mnist_cnn import MnistCnnModel
from dtfe.optim import FlatParams
from dtfe.parallel.partition import PartitionedModel, split_rows
from dtfe.parallel.placement import round_robin
from dtfe.utils import native


def test_split_rows_matches_tf_iter_slices():
    assert split_rows(10, 3) == [(0, 4), (4, 3), (7, 3)]
    assert split_rows(1024, 4) == [(0, 256), (256, 256), (512, 256), (768, 256)]


def test_cnn_fc1_partitions_and_placement():
    m = MnistCnnModel()
    pm = PartitionedModel(m, 4 << 20)  # fc1 weight: 12.8 MB fp32 -> 4 parts of 256 rows (3.2 MB)
    names = [s.name for s in pm.specs]
    assert [n for n in names if "part" in n] == ["Variable_2/part_%d" % i for i in range(4)]
    parts = {s.name: s for s in pm.specs if "part" in s.name}
    assert all(s.shape == (256, 3136) and s.tf_shape == (3136, 256) for s in parts.values())
    assert pm.axis == {"Variable_2": 1}  # TF [in, out]: our rows are TF columns
    # created consecutively in place of Variable_2: round-robin deals them to alternating ps tasks
    pl = round_robin(pm.var_order, 2)
    assert [pl["Variable_2/part_%d" % i] for i in range(4)] == [0, 1, 0, 1]
    # optimizer var lists follow the parts
    (_cfg, vl, _bp), = pm.opt_groups
    assert "Variable_2" not in vl and all(n in vl for n in parts)
    # whole-variable placement (the reference) is unchanged without the flag
    assert [s.name for s in PartitionedModel(m, 0).specs] == [s.name for s in m.specs]
    # part TF layout: the variable's conversion applied to the rows of the part
    t = torch.randn(256, 3136)
    assert torch.equal(pm.to_tf("Variable_2/part_1", t), t.t())


def test_worker_aliases_address_the_full_buffer():
    m = MnistCnnModel()
    pm = PartitionedModel(m, 4 << 20)
    P = FlatParams(m.specs, "cpu", seed=3)
    pm.add_aliases(P)
    full = P.view("Variable_2")
    for i in range(4):
        assert torch.equal(P.view("Variable_2/part_%d" % i), full[256 * i:256 * (i + 1)])
        assert P.view("Variable_2/part_%d" % i).data_ptr() == full[256 * i].data_ptr()
    P.gview("Variable_2/part_3").fill_(7.0)
    assert (P.gview("Variable_2")[768:] == 7.0).all() and (P.gview("Variable_2")[:768] == 0).all()


def _oc_signed(v):
    """OrderedCode::WriteSignedNumIncreasing for the small values used here (|v| < 64, or < 8192)."""
    if -64 <= v < 64:
        return bytes([(0x80 ^ v) & 0xff])
    assert 0 <= v < 8192
    return bytes([0xc0 ^ (v >> 8), v & 0xff])


def test_tensor_name_slice_key_encoding():
    rt = native.rt()
    key = rt.encode_tensor_name_slice("Variable_2", [(0, -1), (512, 256)])
    want = (b"\x00" + b"Variable_2" + b"\x00\x01" + b"\x01\x02" + _oc_signed(0) + _oc_signed(-1)
            + _oc_signed(512) + _oc_signed(256))
    assert key == want
    # an embedded 0x00 / 0xff in the name is escaped
    assert rt.encode_tensor_name_slice("a\x00", [(0, -1)]).startswith(b"\x00a\x00\xff\x00\x01")


def test_sliced_bundle_round_trip(tmp_path):
    prefix = str(tmp_path / "model.ckpt-5")
    full = torch.randn(3136, 1024)
    slot = torch.randn(3136, 1024)
    bounds = split_rows(1024, 4)
    ckpt.save_bundle(prefix, {"Variable_2": ckpt.Sliced(full, 1, bounds),
                              "Variable_2/Adam": ckpt.Sliced(slot, 1, bounds),
                              "Variable_8": torch.tensor(5, dtype=torch.int32)})
    idx = native.rt().read_bundle_index(prefix)
    assert set(idx) == {"Variable_2", "Variable_2/Adam", "Variable_8"}  # slice data keys are not names
    dt, shape, _off, size, _crc, slices = idx["Variable_2"]
    assert shape == [3136, 1024] and size == 0 and len(slices) == 4
    assert slices[1] == [(0, -1), (256, 256)]
    back = ckpt.load_bundle(prefix)
    assert torch.equal(back["Variable_2"], full) and torch.equal(back["Variable_2/Adam"], slot)
    assert int(back["Variable_8"]) == 5


def test_merge_and_split_tf_round_trip():
    m = MnistCnnModel()
    pm = PartitionedModel(m, 4 << 20)
    full = torch.randn(3136, 1024)
    shards = pm.split_tf({"Variable_2": full, "Variable_2/Adam": full * 2, "Variable": torch.ones(5, 5, 1, 32)})
    assert set(shards) == {"Variable_2/part_%d" % i for i in range(4)} | \
        {"Variable_2/part_%d/Adam" % i for i in range(4)} | {"Variable"}
    assert torch.equal(shards["Variable_2/part_2"], full[:, 512:768])
    merged = pm.merge_tf(shards)
    assert isinstance(merged["Variable_2"], ckpt.Sliced) and torch.equal(merged["Variable_2"].full, full)
    assert torch.equal(merged["Variable_2/Adam"].full, full * 2) and torch.equal(merged["Variable"], shards["Variable"])


@pytest.mark.slow
def test_partitioned_two_ps_cluster_checkpoint_restores(tmp_path):
    """softmax, 2 ps + 1 worker, the 784x10 kernel in 3 partitions over both ps tasks: the chief's
    checkpoint holds it as TF slices; a restart with partitioning resumes from it, and so does a
    restart without (the checkpoint stores the full variable whatever the partitioning)."""
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "launch"))
    import local_cluster
    md = str(tmp_path / "ck")
    common = ["--data_dir=/nonexistent", "--device=cpu", "--seed=1", "--workers=1", "--model_dir=" + md,
              "--save_model_secs=0.05"]
    part = ["--ps_partition_mb=0.012"]  # 784 x 10 x 4 B = 31 KB -> 3 partitions of <= 12.6 KB
    codes, out, _ = local_cluster.launch("softmax", 2, 1, common + part + ["--num_steps=30"], timeout=240,
                                         stream=False)
    assert all(c == 0 for c in codes.values()), out
    latest = ckpt.latest_checkpoint(md)
    idx = native.rt().read_bundle_index(latest)
    kernel = next(n for n, e in idx.items() if e[1] == [784, 10])
    assert len(idx[kernel][5]) == 3, idx[kernel]
    saved = ckpt.load_bundle(latest)
    gs0 = int(saved["Variable_2"])
    assert gs0 > 0 and saved[kernel].shape == (784, 10) and float(saved[kernel].abs().sum()) > 0
    for extra in (part, []):
        codes, out, _ = local_cluster.launch("softmax", 2, 1, common + extra + ["--num_steps=%d" % (gs0 + 5)],
                                             timeout=240, stream=False)
        assert all(c == 0 for c in codes.values()), out
        import re
        gs = [int(mm.group(1)) for l in out[("worker", 0)] for mm in [re.match(r"Global step (\d+) ", l)] if mm]
        assert gs[0] == gs0 + 1, (extra, gs0, gs[:3])
        gs0 = int(ckpt.load_bundle(ckpt.latest_checkpoint(md))["Variable_2"])
