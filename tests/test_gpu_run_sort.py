"""Run-level slot sort (csrc/kernels/fsort_run.h): the field sorts of every batch of a multi-step
graph run as two launches at the graph's start (4K-row chunk sorts reading the ids in place, then
the chunk merge).  Its output is the stable global sort of each batch, and training through it
is bitwise the per-step side-stream sort (HIPFM_RUN_SORT=0) and the unprefetched step.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # collected on CPU, skipped there
    pytest.skip("needs a GPU", allow_module_level=True)

import hipfm  # noqa: E402,F401
import hipfm.models.deepfm as D  # noqa: E402
from hipfm.data.synthetic import make_synth  # noqa: E402
from hipfm.models.deepfm import NativeDeepFM, graph_capture  # noqa: E402
from hipfm.models.reference import init_params  # noqa: E402
from hipfm.ops import kernels as KN  # noqa: E402

DEV = torch.device("cuda", 0)


@pytest.mark.parametrize("preset,B,G", [("criteo_1tb", 16384, 3), ("criteo_kaggle", 1024, 4),
                                        ("criteo_1tb", 6000, 2), ("criteo_kaggle", 12288, 5),
                                        ("reference", 4096, 2), ("criteo_1tb", 32768, 2), ("criteo_kaggle", 40000, 2)])
def test_run_sort_is_the_stable_sort(preset, B, G):
    """Every batch of the run gets exactly the stable global sort of its B*F slot ids (keys and
    slot positions), row-major and field-major ids, eager and as a replayed graph."""
    synth = make_synth(preset, seed=31)
    F = synth.F
    fs = KN.FieldSort(synth.field_ranges(), B, DEV, max_pb=0)
    for fm in (False, True):
        bats = [synth.batch(B, step=s + 7 * fm, device=DEV, id_dtype=torch.int32)[0] for s in range(G)]
        ids = [b.t().contiguous() if fm else b.contiguous() for b in bats]     # [F, B] or [B, F]
        outs = [(torch.full((B * F,), -7, dtype=torch.int32, device=DEV),
                 torch.full((B * F,), -7, dtype=torch.int32, device=DEV)) for _ in range(G)]
        plan = fs.run_plan([(i.reshape(-1), B, fm, k, p) for i, (k, p) in zip(ids, outs)])
        fs.run_sort(plan)
        g = torch.cuda.CUDAGraph()
        with graph_capture(g):
            fs.run_sort(plan)
        for it in range(2):
            if it:
                for s, i in enumerate(ids):
                    nb = synth.batch(B, step=100 + s, device=DEV, id_dtype=torch.int32)[0]
                    i.copy_(nb.t() if fm else nb)
                    bats[s] = nb
                g.replay()
            torch.cuda.synchronize()
            assert int(fs.err.item()) == 0
            for b, (k, p) in zip(bats, outs):
                rk, rp = torch.sort(b.reshape(-1).long(), stable=True)
                assert torch.equal(k.long(), rk) and torch.equal(p.long(), rp), (preset, B, fm, it)


def test_run_sort_flags_out_of_range_ids():
    synth = make_synth("criteo_kaggle", seed=34)
    B, F = 2048, synth.F
    fs = KN.FieldSort(synth.field_ranges(), B, DEV, max_pb=0)
    ids = synth.batch(B, 0, device=DEV, id_dtype=torch.int32)[0].contiguous()
    ids[5, 20] = synth.field_ranges()[21][0]          # an id of field 21 in field 20
    k, p = torch.empty(B * F, dtype=torch.int32, device=DEV), torch.empty(B * F, dtype=torch.int32, device=DEV)
    fs.run_sort(fs.run_plan([(ids.reshape(-1), B, False, k, p)]))
    assert int(fs.err.item()) != 0


@pytest.mark.parametrize("B,mlp_dtype,emb_dtype,update", [(16384, "bf16", "fp32", "lazy"), (1024, "bf16", "fp32", "lazy"),
                                                          (6000, "fp8", "bf16", "lazy"),
                                                          (16384, "bf16", "fp32", "tf1_dense"),
                                                          (8192, "bf16", "fp32", "tf1_dense")])
def test_run_sort_training_bitwise_equals_side_stream(monkeypatch, B, mlp_dtype, emb_dtype, update):
    """Multi-step graphs with the run-level sort give bitwise the parameters, slots and step
    counter of multi-step graphs with the per-step side-stream sort and of single steps."""
    synth = make_synth("criteo_kaggle", seed=32)
    K, layers = 8, [128, 64, 32]
    params = init_params(synth.feature_size, synth.F, K, layers, False, seed=5)
    pool = [synth.batch(B, step=s, device=DEV, id_dtype=torch.int32) for s in range(4)]
    out = []
    for run, multi in ((True, True), (False, True), (False, False)):
        monkeypatch.setattr(D, "_RUN_SORT", run)
        m = NativeDeepFM(synth.feature_size, synth.F, K, layers, [0.5] * 3, batch_size=B, device=DEV,
                         init=False, sparse_update=update, mlp_dtype=mlp_dtype, emb_dtype=emb_dtype,
                         field_ranges=synth.field_ranges())
        m.load_tf_params(params)
        if multi:
            for r in range(3):            # graphs captured once, replayed
                m.train_steps(pool[:2], next_ids=(pool[2][0], pool[3][0]))
                m.train_steps(pool[2:], next_ids=(pool[0][0], pool[1][0]))
        else:
            for s in range(12):
                ids, vals, lab = pool[s % 4]
                m.train_step(ids, vals, lab, use_graph=True, next_ids=pool[(s + 1) % 4][0])
        torch.cuda.synchronize()
        m.check_errors()
        assert m.global_step() == 12
        if run and multi:
            assert m._run_sort_ok(pool[:2])            # the run path ran (tf1_dense: merged sweep)
        out.append([m.tv.clone(), m.tw.clone(), m.p.clone(), m.step.clone()] +
                   [s.clone() for s in m.sv if s.numel()])
        del m
    for k, ref in enumerate(out[1:]):
        for i, (x, y) in enumerate(zip(out[0], ref)):
            assert torch.equal(x, y), (k, i, (x.float() - y.float()).abs().max().item())


def test_growing_runs_keep_earlier_graphs_valid(monkeypatch):
    """A run longer than every earlier one grows the run-sort scratch; the graphs captured from
    the shorter runs still read their own plans (FsJob arrays, scratch), so replaying them after
    the growth is bitwise the per-step sorted training (a freed plan under a captured graph made
    the bench's warm-up replay fault)."""
    synth = make_synth("criteo_kaggle", seed=36)
    B, K, layers = 1024, 8, [128, 64, 32]
    params = init_params(synth.feature_size, synth.F, K, layers, False, seed=6)
    pool = [synth.batch(B, step=s, device=DEV, id_dtype=torch.int32) for s in range(6)]
    order = [(0, 2), (2, 4), (0, 6), (2, 4), (4, 6), (0, 6), (2, 4)]
    out = []
    for run in (True, False):
        monkeypatch.setattr(D, "_RUN_SORT", run)
        m = NativeDeepFM(synth.feature_size, synth.F, K, layers, [0.5] * 3, batch_size=B, device=DEV,
                         init=False, field_ranges=synth.field_ranges())
        m.load_tf_params(params)
        for lo, hi in order:
            m.train_steps(pool[lo:hi], next_ids=(pool[hi % 6][0], pool[(hi + 1) % 6][0]))
        torch.cuda.synchronize()
        m.check_errors()
        assert m.global_step() == sum(hi - lo for lo, hi in order)
        out.append([m.tv.clone(), m.tw.clone(), m.p.clone(), m.step.clone()] + [s.clone() for s in m.sv if s.numel()])
        del m
    for i, (x, y) in enumerate(zip(*out)):
        assert torch.equal(x, y), (i, (x.float() - y.float()).abs().max().item())


@pytest.mark.parametrize("run,update", [(True, "lazy"), (False, "lazy"), (False, "tf1_dense")])
def test_reset_plan_state_replays_without_recapture(monkeypatch, run, update):
    """bench's capture pass and its warm-up / timed windows start from ``reset_plan_state``: the
    second pass over the same runs replays every graph (no capture) and trains bitwise like
    eager single steps over the same batches."""
    monkeypatch.setattr(D, "_RUN_SORT", run)
    synth = make_synth("criteo_kaggle", seed=37)
    B, K, layers = 1024, 8, [128, 64, 32]
    params = init_params(synth.feature_size, synth.F, K, layers, False, seed=7)
    pool = [synth.batch(B, step=s, device=DEV, id_dtype=torch.int32) for s in range(6)]
    seq = [pool[0]] + pool + pool
    out = []
    for graphs in (True, False):
        m = NativeDeepFM(synth.feature_size, synth.F, K, layers, [0.5] * 3, batch_size=B, device=DEV,
                         init=False, field_ranges=synth.field_ranges(), sparse_update=update)
        m.load_tf_params(params)
        if graphs:
            m.warm_step(*pool[0])
            if run:
                assert m._run_sort_ok(pool[:3])
            for p in range(2):
                m.reset_plan_state()
                n0 = len(m._graphs)
                m.train_steps(pool[:3], next_ids=(pool[3][0], pool[4][0]))
                m.train_steps(pool[3:], next_ids=(pool[0][0], pool[1][0]))
                if p:
                    assert len(m._graphs) == n0           # replays only
        else:
            for b in seq:
                m.train_step(*b, use_graph=False)
        torch.cuda.synchronize()
        m.check_errors()
        assert m.global_step() == len(seq)
        out.append([m.tv.clone(), m.tw.clone(), m.p.clone(), m.step.clone()] + [s.clone() for s in m.sv if s.numel()])
        del m
    for i, (x, y) in enumerate(zip(*out)):
        assert torch.equal(x, y), (i, (x.float() - y.float()).abs().max().item())
