"""Step planner: which kernels, launches and graph branches ONE training step enqueues.

``NativeDeepFM.train_step_enqueue`` used to decide this inline from a dozen execution-mode knobs
while it enqueued; here the decision is a pure function of

  * the model's mode (``ModeSpec``: tower fusion, table sharding / exchange, sparse update rule,
    dtypes, whether the sparse + wgfin launch fits),
  * the execution-mode knobs (``StepKnobs``: every one a supported, tested mode or a test oracle;
    ``utils/knobs.py`` documents each one's measurement),
  * the step's host-side bindings (batch size, slot-sort plan, tf1_dense flag-set plan),

so every combination can be enumerated and checked on the CPU (``tests/test_step_plan.py``) and
the executor only follows the plan.  The step shapes it chooses between (reference semantics:
model_fn HVD:141-287, DistributedOptimizer HVD:262, the PS update path PS:439-442):

  one GPU, lazy rows        tower (gather-fused) -> sfwg (sparse backward + wgfin + dense opt)
  one GPU, tf1_dense split  the same, the l2-only sweep of every other row merged into sfwg or on
                            its own branch (small batches)
  row-sharded / replicated  tower -> sparse backward producing gradient rows (+ wgfin) ->
  exchange (native engine)  ONE grouped collective -> owner update (+ dense optimizer)
  per-layer tower (BN)      layer kernels -> finalize -> sparse kernels -> dense optimizer
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional, Tuple


@dataclass(frozen=True)
class StepKnobs:
    """Snapshot of the execution-mode knobs a step plan depends on (read at plan time, so
    tests that switch a knob between steps see the switch).
    (Round 4 fixed the experiments that had settled: the dense optimizer runs early and inside the
    finalize / wgfin launch, fm_fwd writes field-major ids for the per-layer path's sort, the
    dense-gradient branch forks only under an exchange, the next routing forks at the step start,
    and the fused exchange carries the dense gradient whenever the owner launch applies it.)"""
    sort_side_stream: bool = True    # HIPFM_SORT_SIDE_STREAM: the inline slot sort on a graph branch
    sparse_impl: str = "fused"       # HIPFM_SPARSE: fused | seg (two-kernel test oracle)
    wgfin: bool = True               # HIPFM_WGFIN: one weight-gradient + optimizer launch
    sfwg: bool = True                # HIPFM_SFWG: wgfin inside the sparse backward's launch
    sh_apply_dense: bool = True      # HIPFM_SH_APPLY_DENSE: dense optimizer (+ fused dense exchange) in the owner launch
    sweep_mode: str = "auto"         # HIPFM_SWEEP_MODE: auto | merged | branch
    # multi-step execution (models/runner.py)
    run_sort: bool = True            # HIPFM_RUN_SORT: a run's batches sorted / routed up front
    shard_pipeline: bool = True      # HIPFM_SHARD_PIPELINE: next batches' routing prefetched
    sh_overlap: bool = False         # HIPFM_SH_OVERLAP: the dense all-reduce beside the sparse backward


@dataclass(frozen=True)
class ModeSpec:
    """The model's execution mode (fixed after construction)."""
    K: int
    fused: bool                # one-launch deep tower
    gather_fused: bool         # ... with the FM gather as its prologue
    sharded: bool              # row-sharded table (owner = id % N)
    exchange: bool             # multi-rank (or forced) exchange of sparse gradients
    native_exchange: bool      # the exchange runs on the native fixed-capacity engine (shx / rpx)
    row_sharded: bool          # ... and it is the row-sharded one (shx; rpx: replicated table)
    lazy_rows: bool            # sparse rows take the lazy (touched-rows-only) update
    lazy: bool                 # sparse_update == "lazy" (tf1_dense split form: lazy_rows, not lazy)
    tf1_split: bool            # tf1_dense split form (flags + sweep)
    fp8: bool
    wgfin_fits: bool           # the wgfin work fits the sparse + wgfin launch (splits <= SFWG_MAX_NS)
    fin_covers_all: bool       # the finalize launch covers every dense parameter
    grow_ok: bool = False      # the tower (K <= 16) or its dX0 launch (K = 32) can write sorted gradient rows
    tf1x: bool = False         # tf1_dense split form under the native exchange (lazy owner update +
                               # flagged l2-only sweep in the owner launch)


@dataclass(frozen=True)
class StepPlan:
    # slot sort
    run_sorted: bool = False       # sorted at the start of the captured run (fsort_run.h)
    presorted: bool = False        # the sparse backward finds the batch sorted (no inline sort)
    fork_sort: bool = False        # this batch's sort on a graph branch forked after the tower
    sort_idst: bool = False        # ... reading the ids fm_fwd wrote field-major
    prefetch_next: bool = False    # the next batch's sort on a root branch joined at the step end
    join_sort: bool = False        # main waits for the forked sort before the sparse backward
    # tf1_dense split form
    tf1_merged: bool = False       # the l2-only sweep rides in the sfwg launch
    tf1_branch: bool = False       # ... else on its own branch, joined at the step end
    tower_stamp: bool = False      # run-sorted: the batch's row flags stamped by tower workgroups
    # dense part
    defer_wgrad: bool = False      # the tower launch stops before the weight gradients
    dense_branch: bool = False     # weight gradients (+ all-reduce) on a branch beside the sparse part
    dense_early: bool = False      # dense optimizer before the sparse backward (advances the step)
    fuse_opt: bool = False         # ... inside the finalize / wgfin launch
    sfwg: bool = False             # ... and that launch merged into the sparse backward
    dense_opt_after: bool = False  # dense optimizer launched at the end of the step
    # native exchange
    xfuse: bool = False            # dense gradient from the sparse launch, all-gathered with the rows
    exchange_allreduce: bool = False  # dense gradient all-reduced inside the exchange group
    sh_apply_dense: bool = False   # dense optimizer inside the owner update launch
    w8_after_fin: bool = False     # fp8: quantize the weights after the fused finalize optimizer
    w8_after_owner: bool = False   # fp8: ... after the owner launch's dense optimizer
    grow_rows: bool = False        # run-sorted sfwg step: the tower writes each slot's gradient row
                                   # to its sorted position; the sparse launch streams them
    overlap_dense: bool = False    # multi-rank lazy / tf1 split step: the dense gradient (its own wgfin launch
                                   # after the tower) is all-reduced on the main stream WHILE the
                                   # sparse backward runs on a graph branch


IDLE = StepPlan()


def sweep_merges(mode: ModeSpec, kn: StepKnobs, B: int) -> bool:
    """tf1_dense split sweep inside the merged sparse launch.  Small batches take the branch:
    their tower / sparse launches leave most CUs idle (B = 1024, K = 8: branch 0.069 vs merged
    0.077 ms/step; B = 16384: merged 0.156 vs branch 0.160-0.163).  K = 32 always merges: a
    concurrent K = 32 sweep slowed its latency-bound tower 41 -> 76 us."""
    return kn.sweep_mode == "merged" or (kn.sweep_mode == "auto" and (B >= 8192 or mode.K > 16))


def sfwg_possible(mode: ModeSpec, kn: StepKnobs) -> bool:
    """The sparse backward + wgfin merged launch applies (given the fused dense optimizer)."""
    return (kn.wgfin and kn.sfwg and mode.wgfin_fits and not mode.native_exchange and not mode.sharded and
            mode.fused and mode.fin_covers_all and not mode.exchange and
            mode.lazy_rows and kn.sparse_impl == "fused")


def plan_step(mode: ModeSpec, kn: StepKnobs, B: int, sort_plan: Optional[Tuple], tf1: bool,
              field_sort: bool = False, idst_capable: bool = False, routed_run: bool = False) -> StepPlan:
    """The plan of one training step.  ``sort_plan``: the host-side slot-sort binding (None:
    sort inline; ("run", ...): sorted at the run start; (set, inline, next_key): per-step sets,
    prefetched by the previous step unless ``inline``, the next batch's sort forked when
    ``next_key``); ``tf1``: a tf1_dense split flag-set plan is bound; ``field_sort`` /
    ``idst_capable``: the batch takes the per-field sort / fm_fwd can write its ids field-major;
    ``routed_run``: a row-sharded step of a run routed at its start (parallel/sharded.py)."""
    run = sort_plan is not None and sort_plan[0] == "run"
    prefetch = sort_plan is not None and not run and sort_plan[2] is not None
    inline = sort_plan is None or (not run and bool(sort_plan[1]))
    fork = inline and not mode.sharded and kn.sort_side_stream
    presorted = (not inline) or fork
    merged = tf1 and sweep_merges(mode, kn, B) and sfwg_possible(mode, kn)
    if run and tf1 and not merged:
        raise RuntimeError("run-level sort with tf1_dense needs the merged sweep")
    # row-sharded / replicated lazy step with wgfin: the dense gradient is computed in the sparse
    # backward's launch and travels with the gradient rows (all-gather, summed in rank order by
    # the owner launch): no comm stream, no all-reduce, no cross-stream joins
    owner_lazy = mode.lazy or mode.tf1x          # the owner launch applies the rows lazily
    # overlap: the dense gradient leaves the sparse launch (its own wgfin launch, gradient only,
    # right after the tower) so its all-reduce (G2a) runs on the main stream while the sparse
    # backward runs on a branch; the gradient rows follow in G2b after the join
    # (the tf1_dense split form too: its flagged rows take the lazy owner update and the owner
    # launch sweeps every other row, whichever way the dense gradient travelled)
    ovl = (kn.sh_overlap and mode.native_exchange and owner_lazy and mode.fused and kn.wgfin and
           kn.sh_apply_dense)
    xfuse = (mode.native_exchange and owner_lazy and kn.wgfin and mode.fused and
             kn.sh_apply_dense and mode.wgfin_fits and not ovl)
    # fused tower, multi-rank: the weight gradients only feed the dense optimizer, so they run on
    # their own branch beside the sparse exchange (0.210 -> 0.199 ms); on one GPU a concurrent
    # wgrad slows the sparse backward more than it saves (0.156 -> 0.161 ms)
    split = mode.fused and not xfuse and mode.exchange and not ovl
    # one GPU, lazy rows: the dense optimizer needs only the finished dense gradient, so it runs
    # before the sparse backward (inside the gap a join costs anyway); with the fused tower it
    # rides on the finalize launch, and with wgfin inside the sparse backward's launch (sfwg)
    early = (presorted and not mode.exchange and not split and mode.lazy_rows and
             kn.sparse_impl == "fused")
    fuse_opt = early and mode.fused and mode.fin_covers_all
    sfwg = fuse_opt and sfwg_possible(mode, kn)
    if merged and not sfwg:
        raise RuntimeError("tf1_dense merged sweep planned but the step took another path")
    ex_ar = mode.native_exchange and not xfuse
    sh_dense = mode.native_exchange and owner_lazy and kn.sh_apply_dense and not early
    return StepPlan(
        run_sorted=run, presorted=presorted, fork_sort=fork,
        sort_idst=fork and not mode.gather_fused and field_sort and idst_capable,
        prefetch_next=prefetch, join_sort=fork,
        tf1_merged=merged, tf1_branch=tf1 and not merged,
        tower_stamp=run and tf1 and mode.fused and mode.gather_fused,
        defer_wgrad=split or sfwg or xfuse or ovl, dense_branch=split, dense_early=early, fuse_opt=fuse_opt,
        sfwg=sfwg, dense_opt_after=not sh_dense and not early,
        xfuse=xfuse, exchange_allreduce=ex_ar, sh_apply_dense=sh_dense,
        w8_after_fin=mode.fp8 and fuse_opt and not kn.wgfin, w8_after_owner=mode.fp8 and sh_dense,
        grow_rows=mode.grow_ok and ((run and sfwg) or (routed_run and xfuse and mode.row_sharded)),
        overlap_dense=ovl)
