"""Checkpoint tests: native save/restore + pruning + CRC, TF tensor_bundle
structure and round trip, reshard-on-load of mod-sharded tables."""
import json
import os
import struct

import numpy as np
import pytest
import torch

import hipfm
from hipfm.ckpt import tf_bundle as tb
from hipfm.ckpt.native import CheckpointManager, reshard_rows
from hipfm.models.reference import GoldenDeepFM


def test_native_save_restore_prune(tmp_path):
    m = CheckpointManager(str(tmp_path), keep_max=2)
    st = {"a": torch.randn(10, 3), "b": torch.arange(7), "c": torch.randn(4).to(torch.bfloat16)}
    for step in (1, 2, 3):
        m.save(step, {k: v + step if v.dtype != torch.int64 else v for k, v in st.items()}, {"x": step})
    idx = json.load(open(tmp_path / "hipfm_checkpoint.json"))
    assert idx["all"] == ["ckpt-2", "ckpt-3"] and not (tmp_path / "ckpt-1").exists()
    assert m.latest().endswith("ckpt-3")
    got = m.load_rank(m.latest(), 0)
    assert torch.equal(got["a"], st["a"] + 3) and torch.equal(got["b"], st["b"])
    assert torch.equal(got["c"], st["c"] + 3)
    assert m.load_manifest(m.latest())["meta"] == {"x": 3}
    # corrupt a byte -> CRC error
    p = tmp_path / "ckpt-3" / "rank0.bin"
    raw = bytearray(open(p, "rb").read())
    raw[3] ^= 1
    open(p, "wb").write(raw)
    with pytest.raises(IOError):
        m.load_rank(m.latest(), 0)


def test_reshard_rows(tmp_path):
    V, K, N_old = 23, 4, 3
    full = torch.randn(V, K)
    m = CheckpointManager(str(tmp_path / "ck"), world=N_old)
    path = str(tmp_path / "ck" / "ckpt-5")
    os.makedirs(path)
    R_old = (V + N_old - 1) // N_old
    for r in range(N_old):
        loc = torch.zeros(R_old, K)
        rows = full[r::N_old]
        loc[: rows.shape[0]] = rows
        from hipfm.ckpt.native import write_tensors
        idx = write_tensors(os.path.join(path, f"rank{r}.bin"), {"fm_v": loc})
        json.dump({"tensors": idx, "meta": {}}, open(os.path.join(path, f"rank{r}.json"), "w"))
    for N_new in (1, 2, 4):
        R_new = (V + N_new - 1) // N_new
        for r in range(N_new):
            got = reshard_rows(path, "fm_v", N_old, N_new, r, R_new, (K,))
            want = full[r::N_new]
            assert torch.equal(got[: want.shape[0]], want)


def test_sstable_structure_and_roundtrip(tmp_path):
    items = [(f"key{i:04d}".encode(), bytes([i % 256]) * (i % 50)) for i in range(300)]
    p = str(tmp_path / "t.sst")
    tb.write_sstable(p, items)
    raw = open(p, "rb").read()
    assert struct.unpack("<Q", raw[-8:])[0] == tb.TABLE_MAGIC
    assert tb.read_sstable(p) == sorted(items)


def test_tf_bundle_roundtrip_reference_names(tmp_path):
    g = GoldenDeepFM(1000, 39, 8, [32, 16], [1.0, 1.0])
    ids = torch.randint(0, 1000, (64, 39))
    g.train_step(ids, torch.rand(64, 39), (torch.rand(64) < 0.3).float())
    v = g.tf_variables()
    names = set(v)
    for n in ("fm_bias", "fm_w", "fm_v", "Deep-part/mlp0/weights", "Deep-part/mlp1/biases",
              "Deep-part/deep_out/weights", "fm_v/Adam", "fm_v/Adam_1", "beta1_power", "global_step"):
        assert n in names, n
    assert tuple(v["Deep-part/mlp0/weights"].shape) == (39 * 8, 32)   # TF [in, out] layout
    prefix = str(tmp_path / "model.ckpt-1")
    tb.write_bundle(prefix, v)
    back = tb.read_bundle(prefix)
    assert set(back) == names
    for k in names:
        assert np.array_equal(back[k], v[k].numpy()), k
    # header entry + sorted keys + entry fields
    items = tb.read_sstable(prefix + ".index")
    assert items[0][0] == b"" and [k for k, _ in items] == sorted(k for k, _ in items)
    e = tb.parse_entry(dict(items)[b"fm_v"])
    assert e["dtype"] == tb.DT_FLOAT and e["shape"] == [1000, 8] and e["size"] == 1000 * 8 * 4
    tb.write_checkpoint_state(str(tmp_path), "model.ckpt-1", ["model.ckpt-1"])
    assert tb.read_checkpoint_state(str(tmp_path)) == "model.ckpt-1"


def test_tf_bundle_streams_large_tensor(tmp_path):
    t = torch.randn(5000, 8)
    prefix = str(tmp_path / "big")
    tb.write_bundle(prefix, {"fm_v": t}, chunk_bytes=4096)     # forces the chunked CRC path
    assert np.array_equal(tb.read_bundle(prefix)["fm_v"], t.numpy())
