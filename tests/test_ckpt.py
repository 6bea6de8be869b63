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


def test_multi_shard_bundle_roundtrip(tmp_path):
    """Every variable whole in one of N data shards (the PS-job layout), one merged index."""
    prefix = str(tmp_path / "model.ckpt-7")
    rng = np.random.default_rng(0)
    tensors = {"fm_v": rng.standard_normal((1000, 4)).astype(np.float32),
               "fm_w": rng.standard_normal(1000).astype(np.float32),
               "Deep-part/mlp0/weights": rng.standard_normal((156, 8)).astype(np.float32),
               "global_step": np.array(7, dtype=np.int64)}
    writers = [tb.ShardWriter(prefix, r, 3) for r in range(3)]
    for i, (k, v) in enumerate(sorted(tensors.items())):
        w = writers[i % 3]
        if k == "fm_v":                                   # streamed in row chunks
            w.add(k, v.shape, (v[a:a + 300] for a in range(0, 1000, 300)))
        else:
            w.add(k, v.shape, [v])
    entries = []
    for w in writers:
        w.close()
        entries += w.entries
    tb.write_index(prefix, entries, 3)
    for r in range(3):
        assert os.path.exists(tb.data_path(prefix, r, 3))
    got = tb.read_bundle(prefix)
    assert set(got) == set(tensors)
    for k in tensors:
        np.testing.assert_array_equal(got[k], tensors[k])
    hdr = [v for k, v in tb.read_sstable(prefix + ".index") if not k][0]
    assert tb.parse_header(hdr)["num_shards"] == 3


def _decode(b):
    from hipfm.data.tfrecord import _fields
    return list(_fields(b))


def _map(entries, field):
    out = {}
    for f, _, v in entries:
        if f == field:
            kv = dict((ff, vv) for ff, _, vv in _decode(v))
            out[kv[1].decode()] = kv.get(2, b"")
    return out


@pytest.mark.parametrize("bn", [False, True])
def test_saved_model_pb_structure(tmp_path, bn):
    """saved_model.pb decodes to one MetaGraphDef (tag serve) whose serving_default signature is
    the reference's (feat_ids int64[-1,F], feat_vals float[-1,F] -> prob float[-1]), whose graph
    holds the placeholders, a VariableV2 per variable of the exported bundle and the
    Gather/MatMul/Sigmoid inference path, and whose V2 saver restores exactly the bundle's names."""
    from hipfm.ckpt.export import export_servable
    from hipfm.ckpt.saved_model import DT_FLOAT, DT_INT64
    from hipfm.models.reference import init_params
    V, F, K, layers = 500, 6, 4, [16, 8]
    params = init_params(V, F, K, layers, bn, seed=1)
    params["global_step"] = torch.tensor(3, dtype=torch.int64)
    cfg = {"feature_size": V, "field_size": F, "embedding_size": K, "deep_layers": layers,
           "dropout_keep": [1.0, 1.0], "batch_norm": bn, "loss_type": "log_loss"}
    d = export_servable(params, cfg, str(tmp_path), timestamp=123)
    sm = _decode(open(os.path.join(d, "saved_model.pb"), "rb").read())
    assert [v for f, _, v in sm if f == 1] == [1]
    metas = [v for f, _, v in sm if f == 2]
    assert len(metas) == 1
    meta = _decode(metas[0])
    info = _decode([v for f, _, v in meta if f == 1][0])
    assert b"serve" in [v for f, _, v in info if f == 4]
    sig = _decode(_map(meta, 5)["serving_default"])
    ins, outs = _map(sig, 1), _map(sig, 2)
    assert set(ins) == {"feat_ids", "feat_vals"} and set(outs) == {"prob"}

    def ti(b):
        t = dict((f, v) for f, _, v in _decode(b))
        dims = [dict((ff, vv) for ff, _, vv in _decode(d)).get(1, 0) for f2, _, d in _decode(t[3]) if f2 == 2]
        dims = [x - (1 << 64) if x >= (1 << 63) else x for x in dims]
        return t[1].decode(), t[2], dims
    assert ti(ins["feat_ids"]) == ("feat_ids:0", DT_INT64, [-1, F])
    assert ti(ins["feat_vals"]) == ("feat_vals:0", DT_FLOAT, [-1, F])
    assert ti(outs["prob"]) == ("prob:0", DT_FLOAT, [-1])
    assert [v for f, _, v in sig if f == 3] == [b"tensorflow/serving/predict"]
    graph = _decode([v for f, _, v in meta if f == 2][0])
    nodes = {}
    for f, _, n in graph:
        if f == 1:
            nd = _decode(n)
            nodes[[v for ff, _, v in nd if ff == 1][0].decode()] = (
                [v for ff, _, v in nd if ff == 2][0].decode(), [v.decode() for ff, _, v in nd if ff == 3])
    assert nodes["feat_ids"][0] == "Placeholder" and nodes["feat_vals"][0] == "Placeholder"
    assert nodes["prob"][0] == "Sigmoid"
    assert nodes["First-order/embedding_lookup"] == ("GatherV2", ["fm_w/read", "feat_ids", "Const/axis0"])
    bundle = set(tb.read_bundle(os.path.join(d, "variables", "variables")))
    var_nodes = {k for k, (op, _) in nodes.items() if op == "VariableV2"}
    assert var_nodes == bundle, (var_nodes ^ bundle)
    saver = dict((f, v) for f, _, v in _decode([v for f, _, v in meta if f == 3][0]))
    assert saver[3] == b"save/restore_all" and saver[7] == 2
    assert nodes["save/RestoreV2"][0] == "RestoreV2"
    restore_inputs = [i for i in nodes["save/restore_all"][1]]
    assert len(restore_inputs) == len(bundle)
