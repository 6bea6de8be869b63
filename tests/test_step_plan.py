"""Step planner (models/step_plan.py): the step shape of every execution mode, and invariants over
the whole mode x knob matrix (CPU only: the planner is a pure function; the GPU tests check that
the executor following each plan is bitwise equal to its oracle)."""
import itertools

import pytest

import hipfm  # noqa: F401
from hipfm.models.step_plan import IDLE, ModeSpec, StepKnobs, plan_step

RUN = ("run", False, None, 0)                  # sorted at the start of the run
PREFETCHED = (0, False, (1234, 16384))         # sorted during the previous step, next batch forked
INLINE = (0, True, None)                       # sorted in this step


def mode(**kw):
    base = dict(K=8, fused=True, gather_fused=True, sharded=False, exchange=False, native_exchange=False,
                row_sharded=False, lazy_rows=True, lazy=True, tf1_split=False, fp8=False, wgfin_fits=True,
                fin_covers_all=True)
    base.update(kw)
    return ModeSpec(**base)


ONE_GPU = mode()
ONE_GPU_TF1 = mode(lazy=False, tf1_split=True)
ROW_SHARDED = mode(sharded=True, exchange=True, native_exchange=True, row_sharded=True)
REPLICATED = mode(exchange=True, native_exchange=True)
PER_LAYER = mode(fused=False, gather_fused=False, fin_covers_all=False)     # batch norm


def dense_opt_sites(p):
    return [p.fuse_opt, p.dense_early and not p.fuse_opt, p.sh_apply_dense, p.dense_opt_after]


def test_one_gpu_run_sorted_is_tower_plus_sfwg():
    p = plan_step(ONE_GPU, StepKnobs(), 16384, RUN, tf1=False)
    assert p.run_sorted and p.presorted and not p.fork_sort and not p.prefetch_next
    assert p.sfwg and p.fuse_opt and p.dense_early and p.defer_wgrad
    assert not (p.dense_branch or p.dense_opt_after or p.xfuse)


def test_one_gpu_prefetched_and_inline_sorts():
    p = plan_step(ONE_GPU, StepKnobs(), 16384, PREFETCHED, tf1=False)
    assert p.prefetch_next and p.presorted and not p.fork_sort and p.sfwg
    p = plan_step(ONE_GPU, StepKnobs(), 16384, INLINE, tf1=False)
    assert p.fork_sort and p.join_sort and p.presorted and p.sfwg
    p = plan_step(ONE_GPU, StepKnobs(sort_side_stream=False), 16384, INLINE, tf1=False)
    assert not p.presorted and not p.fork_sort and not p.dense_early and p.dense_opt_after


def test_tf1_sweep_merges_at_large_batches_and_k32():
    big = plan_step(ONE_GPU_TF1, StepKnobs(), 16384, PREFETCHED, tf1=True)
    assert big.tf1_merged and big.sfwg and not big.tf1_branch
    small = plan_step(ONE_GPU_TF1, StepKnobs(), 1024, PREFETCHED, tf1=True)
    assert small.tf1_branch and not small.tf1_merged
    k32 = plan_step(mode(K=32, lazy=False, tf1_split=True), StepKnobs(), 1024, PREFETCHED, tf1=True)
    assert k32.tf1_merged
    run = plan_step(ONE_GPU_TF1, StepKnobs(), 16384, RUN, tf1=True)
    assert run.tower_stamp and run.tf1_merged
    with pytest.raises(RuntimeError, match="merged sweep"):
        plan_step(ONE_GPU_TF1, StepKnobs(), 1024, RUN, tf1=True)


def test_native_exchange_steps():
    for m in (ROW_SHARDED, REPLICATED):
        p = plan_step(m, StepKnobs(), 16384, None, tf1=False)
        # dense gradient from the sparse launch, all-gathered with the rows; dense optimizer in the
        # owner launch; no process-group all-reduce and no dense branch
        assert p.xfuse and p.sh_apply_dense and p.defer_wgrad
        assert not (p.exchange_allreduce or p.dense_branch or p.dense_early or p.sfwg)
        tf1 = plan_step(mode(**{**m.__dict__, "lazy": False, "lazy_rows": False}), StepKnobs(), 16384, None,
                        tf1=False)
        assert tf1.exchange_allreduce and tf1.dense_branch and tf1.dense_opt_after and not tf1.xfuse
    assert not plan_step(ROW_SHARDED, StepKnobs(), 16384, INLINE, tf1=False).fork_sort


def test_overlapped_exchange_step():
    """HIPFM_SH_OVERLAP: the dense gradient leaves the sparse launch (deferred past the tower, then
    its own wgfin launch) and is all-reduced while the sparse backward runs on a branch; the
    owner launch keeps the dense optimizer.  tf1_dense exchange steps keep their plan."""
    for m in (ROW_SHARDED, REPLICATED):
        p = plan_step(m, StepKnobs(sh_overlap=True), 16384, None, tf1=False)
        assert p.overlap_dense and p.exchange_allreduce and p.sh_apply_dense and p.defer_wgrad
        assert not (p.xfuse or p.dense_branch or p.dense_early or p.sfwg or p.grow_rows)
        tf1 = plan_step(mode(**{**m.__dict__, "lazy": False, "lazy_rows": False}), StepKnobs(sh_overlap=True),
                        16384, None, tf1=False)
        assert not tf1.overlap_dense
    assert not plan_step(ONE_GPU, StepKnobs(sh_overlap=True), 16384, RUN, tf1=False).overlap_dense


def test_per_layer_tower_and_fp8_quantize_sites():
    p = plan_step(PER_LAYER, StepKnobs(), 4096, INLINE, tf1=False)
    assert p.dense_early and not p.fuse_opt and not p.sfwg and not p.defer_wgrad
    p = plan_step(mode(fp8=True), StepKnobs(wgfin=False), 16384, INLINE, tf1=False)
    assert p.fuse_opt and p.w8_after_fin and not p.sfwg
    p = plan_step(mode(**{**ROW_SHARDED.__dict__, "fp8": True}), StepKnobs(), 16384, None, tf1=False)
    assert p.w8_after_owner and not p.w8_after_fin


def _modes():
    for (fused, gather, fp8, K) in ((True, True, False, 8), (True, True, True, 32), (True, False, False, 8),
                                    (False, False, False, 16)):
        for ex in ("local", "row_sharded", "replicated", "legacy_sharded", "legacy_replicated"):
            for upd in ("lazy", "tf1_split", "tf1_scatter", "tf1_xsplit"):
                if upd == "tf1_split" and ex != "local":
                    continue
                if upd == "tf1_xsplit" and ex not in ("row_sharded", "replicated"):
                    continue
                for fits, covers in ((True, True), (False, True), (True, False)):
                    yield ModeSpec(K=K, fused=fused, gather_fused=gather, fp8=fp8,
                                   sharded=ex in ("row_sharded", "legacy_sharded"), exchange=ex != "local",
                                   native_exchange=ex in ("row_sharded", "replicated"),
                                   row_sharded=ex == "row_sharded", lazy_rows=upd in ("lazy", "tf1_split"),
                                   lazy=upd == "lazy", tf1_split=upd == "tf1_split", wgfin_fits=fits,
                                   fin_covers_all=covers and fused, tf1x=upd == "tf1_xsplit")


def _knob_sets():
    bools = [True, False]
    for (sss, wg, sf, shd, impl, sw, rs, pipe) in itertools.product(
            bools, bools, bools, bools, ("fused", "seg"), ("auto", "merged", "branch"), bools, bools):
        for ovl in ((False, True) if pipe else (False,)):
            yield StepKnobs(sort_side_stream=sss, wgfin=wg, sfwg=sf, sh_apply_dense=shd, sparse_impl=impl,
                            sweep_mode=sw, run_sort=rs, shard_pipeline=pipe, sh_overlap=ovl)


def test_plan_invariants_over_the_mode_matrix():
    """Every plan the planner returns for any mode x knob x binding: exactly one dense-optimizer
    site, the dense gradient produced wherever the tower deferred it, exchange collectives only
    where an exchange exists, and the merged sweep only inside sfwg."""
    n = 0
    knobs = list(_knob_sets())
    for m in _modes():
        for kn in knobs:
            for B in (1024, 16384):
                for sp in (None, RUN, PREFETCHED, INLINE):
                    if sp is not None and (m.sharded or m.exchange):
                        continue          # per-step slot-sort plans are bound on one GPU only
                    for tf1 in ((False, True) if m.tf1_split else (False,)):
                        try:
                            p = plan_step(m, kn, B, sp, tf1)
                        except RuntimeError:
                            assert tf1     # only a tf1 step whose sweep cannot merge refuses
                            continue
                        n += 1
                        assert sum(dense_opt_sites(p)) == 1, (m, kn, B, sp, p)
                        assert p.defer_wgrad == (p.dense_branch or p.sfwg or p.xfuse or p.overlap_dense)
                        assert not p.overlap_dense or (m.native_exchange and (m.lazy or m.tf1x)
                                                       and p.exchange_allreduce and p.sh_apply_dense
                                                       and not p.xfuse)
                        assert not p.sfwg or (p.fuse_opt and p.dense_early and not m.exchange)
                        assert not p.fuse_opt or (m.fused and p.dense_early)
                        assert not p.tf1_merged or p.sfwg
                        assert not (p.tf1_merged and p.tf1_branch)
                        assert not p.xfuse or (m.native_exchange and p.sh_apply_dense and (m.lazy or m.tf1x))
                        if m.tf1x and m.fused and m.wgfin_fits and kn.wgfin and kn.sh_apply_dense:
                            assert (p.xfuse or p.overlap_dense) and p.sh_apply_dense   # the sweep's owner launch
                        assert not p.exchange_allreduce or (m.native_exchange and not p.xfuse)
                        assert not p.sh_apply_dense or m.native_exchange
                        assert not (p.run_sorted and (p.fork_sort or p.prefetch_next))
                        assert not p.fork_sort or (not m.sharded and p.presorted and p.join_sort)
                        assert not p.dense_early or not m.exchange
                        assert not m.fused or not p.dense_early or p.presorted
                        assert not (p.w8_after_fin and p.w8_after_owner)
                        assert not (p.w8_after_fin or p.w8_after_owner) or m.fp8
                        if not m.fused:
                            assert not (p.fuse_opt or p.sfwg or p.xfuse or p.dense_branch)
    assert n > 10000
    assert IDLE == type(IDLE)()
