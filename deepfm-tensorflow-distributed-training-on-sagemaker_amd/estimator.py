"""Estimator-style training API (reference L4: tf.estimator.Estimator + train_and_evaluate).

Reference call sites:
  Estimator(model_fn, model_dir, params, config)                     PS:435, HVD:365-368
  train_and_evaluate(TrainSpec, EvalSpec(throttle_secs, start_delay))   PS:439-442
  for epoch: train(input_fn(num_epochs=1), hooks=[bcast]); rank0 evaluate   HVD:390-394
  evaluate -> {auc, loss, global_step};  predict(predict_keys="prob")       PS:443-449
  export_savedmodel(servable_model_dir, raw receiver)                        PS:451-467
Differences by design (MI355X):
  * one persistent training loop; the epoch boundary is a counter (Q11) and the model state
    never leaves the GPU between epochs (no per-epoch re-broadcast);
  * every rank evaluates its shard and the AUC histograms / loss sums are all-reduced (Q10) —
    no idle ranks while rank 0 evaluates;
  * checkpoints: every rank saves its own state, atomic publish, auto-resume (§5.4);
  * equal steps per rank are enforced up front (Horovod "uneven data" shutdown, DOC p.22-23).
Backends: ``cuda`` -> NativeDeepFM (HIP kernels; fails loudly without its library),
``cpu`` -> GoldenDeepFM (reference-semantics PyTorch; data parallel over gloo).
"""
from __future__ import annotations

import math
import os
import shutil
import time
from dataclasses import dataclass
from typing import Callable, Dict, Iterable, Iterator, List, Optional

import torch
import torch.distributed as dist

from .ckpt.export import export_servable
from .ckpt.native import CheckpointManager, reshard_rows
from .config import RunConfig
from .ops.metrics import auc_from_hist, hist_torch
from .utils.fault import Watchdog, maybe_inject_fault
from .utils.logging import MetricsLogger, StepTimer
from .utils.profiling import StepWindow
from .utils.profiling import range as prof_range


def _dist_on() -> bool:
    return dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1


def resolve_device(cfg: RunConfig):
    if cfg.device == "cpu":
        return torch.device("cpu")
    if cfg.device in ("cuda", "gpu") or (cfg.device == "auto" and torch.cuda.is_available()):
        if not torch.cuda.is_available():
            raise RuntimeError("--device cuda requested but no GPU is visible")
        from .parallel.dist import local_device_index
        return torch.device("cuda", local_device_index())
    return torch.device("cpu")


class PositionedBatch(tuple):
    """(ids, vals, labels) plus ``pos`` = the data position (epoch, batches of that epoch done)
    once this batch is trained: set on the Estimator after the batch's step, so a checkpoint
    records what was trained even when the source is read ahead."""

    def __new__(cls, batch, pos):
        t = super().__new__(cls, tuple(batch))
        t.pos = (int(pos[0]), int(pos[1]))
        t.ring, t.slot = getattr(batch, "ring", None), getattr(batch, "slot", None)   # (RingBatch)
        return t


@dataclass
class TrainSpec:
    input_fn: Callable[[], Iterable]
    max_steps: Optional[int] = None
    hooks: tuple = ()


@dataclass
class EvalSpec:
    input_fn: Callable[[], Iterable]
    steps: Optional[int] = None
    start_delay_secs: float = 0.0     # reference: 1000 (PS:441)
    throttle_secs: float = 0.0        # reference: 1200 (PS:441)


class Estimator:
    def __init__(self, cfg: RunConfig, device=None):
        cfg.validate()
        self.cfg = cfg
        self.device = torch.device(device) if device is not None else resolve_device(cfg)
        self.native = self.device.type == "cuda"
        self.rank = dist.get_rank() if _dist_on() else 0
        self.world = dist.get_world_size() if _dist_on() else 1
        torch.manual_seed(cfg.seed)
        # host-side control messages (per-step "still have data" votes of stream inputs) travel
        # over a gloo group, so they never wait on the GPU stream the way an RCCL op would
        self._ctl = None
        if self.world > 1 and dist.get_backend() != "gloo":
            self._ctl = dist.new_group(backend="gloo")
        self.comm = None
        if self.native:
            from .models.deepfm import NativeDeepFM, field_ranges_from_sizes
            ranges = None
            if cfg.field_sizes:
                ranges = field_ranges_from_sizes([int(x) for x in cfg.field_sizes.split(",") if x.strip()])
            if self.world > 1:
                from .parallel.dist import Comm
                mode = cfg.embedding_mode
                if mode == "auto":
                    mode = "sharded" if cfg.feature_size * cfg.embedding_size > (1 << 27) else "replicated"
                self.comm = Comm(sharded=(mode == "sharded"))
            self.model = NativeDeepFM(cfg.feature_size, cfg.field_size, cfg.embedding_size, cfg.layers,
                                      cfg.keep_probs, l2_reg=cfg.l2_reg, learning_rate=cfg.learning_rate,
                                      optimizer=cfg.optimizer, loss_type=cfg.loss_type,
                                      sparse_update=cfg.sparse_update, seed=cfg.seed,
                                      batch_size=cfg.batch_size, device=self.device, comm=self.comm,
                                      batch_norm=cfg.batch_norm, batch_norm_decay=cfg.batch_norm_decay,
                                      mlp_dtype=cfg.mlp_dtype, emb_dtype=cfg.emb_dtype, field_ranges=ranges)
        else:
            from .models.reference import GoldenDeepFM
            self.model = GoldenDeepFM(cfg.feature_size, cfg.field_size, cfg.embedding_size, cfg.layers,
                                      cfg.keep_probs, batch_norm=cfg.batch_norm,
                                      batch_norm_decay=cfg.batch_norm_decay, l2_reg=cfg.l2_reg,
                                      learning_rate=cfg.learning_rate, optimizer=cfg.optimizer,
                                      loss_type=cfg.loss_type, sparse_update=cfg.sparse_update,
                                      seed=cfg.seed, world_size=self.world)
        barrier = (lambda: dist.barrier()) if _dist_on() else None
        self.ckpt = CheckpointManager(cfg.ckpt_dir, cfg.keep_checkpoint_max, self.rank, self.world,
                                      barrier) if cfg.ckpt_dir else None
        mpath = cfg.metrics_file or (os.path.join(cfg.ckpt_dir, "metrics.jsonl") if cfg.ckpt_dir else None)
        self.log = MetricsLogger(mpath, self.rank)
        # TensorBoard scalars like the reference Estimator's default summary hooks (rank 0):
        # <model_dir>/events.out.tfevents.* (loss, global_step/sec) and <model_dir>/eval/ (auc, loss)
        self._tb = self._tb_eval = None
        self._tb_on = bool(cfg.ckpt_dir) and self.rank == 0 and getattr(cfg, "tensorboard", True)
        self.timer = StepTimer()
        # data-iterator position: epoch index and batches of that epoch already
        # trained on.  Saved with every checkpoint and restored with it, so a resumed job skips
        # what it already trained on instead of replaying the epoch.
        self.epoch = 0
        self.epoch_batch = 0
        self._last_save_t = time.time()
        self._last_eval_t = 0.0
        self.restored_from = self.restore_latest()
        if self.world > 1:
            self.broadcast_state()

    # ------------------------------------------------------------------ state
    @property
    def global_step(self) -> int:
        return self.model.global_step() if self.native else int(self.model.global_step)

    def _state(self):
        return self.model.state_dict_local()

    def _meta(self):
        if self.native:
            meta = dict(self.model.ckpt_meta())
        else:
            meta = {"format": "hipfm-golden", "V": self.cfg.feature_size, "F": self.cfg.field_size,
                    "K": self.cfg.embedding_size, "layers": self.cfg.layers,
                    "optimizer": self.cfg.optimizer, "world": self.world, "sharding": "replicated"}
        meta["data_pos"] = {"epoch": self.epoch, "batch": self.epoch_batch}
        return meta

    def save(self) -> Optional[str]:
        if self.ckpt is None:
            return None
        t0 = time.perf_counter()
        if self.native:
            torch.cuda.synchronize(self.device)
            self.model.check_errors()        # never publish a checkpoint of a flagged step
        with prof_range("checkpoint"):
            path = self.ckpt.save(self.global_step, self._state(), self._meta())
        self.timer.add("ckpt", time.perf_counter() - t0)
        self._last_save_t = time.time()
        self.log.info(f"Saving checkpoints for {self.global_step} into {path}.")
        return path

    def restore_latest(self) -> Optional[str]:
        if self.ckpt is None:
            return None
        path = self.ckpt.latest()
        if path is None:
            return None
        man = self.ckpt.load_manifest(path)
        meta = man["meta"]
        fmt_ok = meta.get("format") == self._meta().get("format")
        if not fmt_ok:
            raise RuntimeError(f"checkpoint {path} was written by {meta.get('format')}; this job "
                               f"runs {self._meta().get('format')} (convert via TF bundle export)")
        if man["world"] == self.world and meta.get("sharding") == self._meta().get("sharding"):
            st = self.ckpt.load_rank(path, self.rank)
        else:
            st = self._reshard_load(path, man)
        self.model.load_state_dict_local(st)
        pos = meta.get("data_pos") or {}
        if man["world"] == self.world:
            # the data position is per rank-shard: it carries over only to the same world size
            self.epoch, self.epoch_batch = int(pos.get("epoch", 0)), int(pos.get("batch", 0))
        self.log.info(f"Restoring parameters from {path} (global_step {self.global_step}, "
                      f"epoch {self.epoch} batch {self.epoch_batch})")
        return path

    def broadcast_state(self):
        """Rank 0's replicated state to every rank (reference C23: BroadcastGlobalVariablesHook(0)
        on every train() call, HVD:371-372,392).  Done once per job here: the state never leaves
        device memory between epochs, so there is nothing to re-synchronize per epoch.  The
        golden (CPU) path broadcasts a golden model's global_step separately."""
        if not _dist_on():
            return
        for t in self.model.replicated_state():
            if t.dtype == torch.float32 or t.dtype == torch.int64:
                dist.broadcast(t, src=0)
        if self.native:
            self.model._host_step = None      # step counter came from rank 0
            self.model._reset_sync()          # hand-off flags are tagged with the step index
            self.model.refresh_shadows()      # bf16 / fp8 weight copies of the broadcast params
        if not self.native:
            gs = torch.tensor([int(self.model.global_step)], dtype=torch.int64)
            dist.broadcast(gs, src=0)
            self.model.global_step = int(gs.item())

    def _reshard_load(self, path: str, man: dict) -> Dict[str, torch.Tensor]:
        """Resume on a different world size / sharding: replicated rows are sliced, mod-sharded
        rows are regrouped (owner = id % N)."""
        old_world = man["world"]
        old_sh = man["meta"].get("sharding", "replicated")
        base = self.ckpt.load_rank(path, 0)
        if not self.native:
            return base
        out = dict(base)
        m = self.model
        table_keys = [k for k in base if k.startswith("fm_")]
        for k in table_keys:
            row_shape = tuple(base[k].shape[1:])
            if old_sh == "replicated":
                full = base[k]
            else:
                full = None
            if m.sharded:
                if full is not None:
                    loc = full[m.rank::m.world]
                    t = torch.zeros((m.R,) + row_shape)
                    t[: loc.shape[0]] = loc
                    out[k] = t
                else:
                    out[k] = reshard_rows(path, k, old_world, m.world, m.rank, m.R, row_shape)
            else:
                if full is not None:
                    out[k] = full
                else:
                    out[k] = reshard_rows(path, k, old_world, 1, 0, m.R, row_shape)
        return out

    # ------------------------------------------------------------------ DP helpers (golden)
    def _golden_grad_sync(self, grads, touched):
        if self.world == 1:
            return grads, touched
        out = {}
        for k, g in grads.items():
            t = g.contiguous().clone()
            dist.all_reduce(t)
            out[k] = t / self.world
        mask = torch.zeros(self.cfg.feature_size, dtype=torch.int32)
        mask[touched] = 1
        dist.all_reduce(mask, op=dist.ReduceOp.MAX)
        return out, torch.nonzero(mask).reshape(-1)

    def _enforce_equal_steps(self, pipeline):
        """Every rank runs the same number of steps per epoch (min over ranks).  Files are
        counted up front; streams (Pipe mode) cannot be, see ``_agreed_batches``."""
        if self.world == 1 or not hasattr(pipeline, "local_records"):
            return
        if not getattr(pipeline, "countable", True):
            return
        n = pipeline.local_records() // pipeline.B
        t = torch.tensor([n], dtype=torch.int64, device=self.device if self.native else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
        pipeline.max_batches = int(t.item())

    def _agreed_batches(self, batches: Iterable) -> Iterator:
        """Equal steps on uncountable (stream) inputs: before each step every rank votes whether
        it still has a batch, and all ranks stop at the first rank's end of stream (the
        reference's equal-data rule against Horovod's uneven-data shutdown, DOC p.22-23, applied
        without reading any stream twice).  Costs one tiny gloo all-reduce per step."""
        it = iter(batches)
        while True:
            b = next(it, None)
            flag = torch.tensor([0 if b is None else 1], dtype=torch.int32)
            dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=self._ctl)
            if int(flag.item()) == 0:
                close = getattr(it, "close", None)
                if close is not None:
                    close()
                return
            yield b

    # ------------------------------------------------------------------ train
    def _agreed_due(self, due: bool) -> bool:
        """A time-based decision (checkpoint every N secs, throttled eval) taken identically on
        every rank: rank 0's clock decides and the bit travels over the host control group, so
        no rank enters a collective save / evaluation alone."""
        if self.world == 1:
            return due
        t = torch.tensor([1 if due else 0], dtype=torch.int32)
        dist.broadcast(t, src=0, group=self._ctl)
        return bool(t.item())

    def _next(self, it):
        t0 = time.perf_counter()
        with prof_range("data_wait"):
            b = next(it, None)
        self.timer.add("data_wait", time.perf_counter() - t0)
        return b

    def train(self, batches: Iterable, max_steps: Optional[int] = None,
              eval_fn: Optional[Callable[[], dict]] = None,
              eval_due: Optional[Callable[[], bool]] = None) -> int:
        """Train over ``batches`` (device or host tensors).  The native path keeps one batch of
        look-ahead: a resident next batch has its slot sort / routing computed during the current
        step; batches replayed from the HBM cache run as captured graphs, ``graph_steps`` of them
        per graph; one-off streamed batches are staged into the static input buffers and replay
        one graph.  Host timers (data wait, H2D, step enqueue, checkpoint, eval) go to the metrics
        log; roctx ranges mark the same phases.  ``eval_due`` (PS schedule): polled at the agreed
        decision steps, evaluates when it returns True."""
        cfg = self.cfg
        if hasattr(batches, "local_records"):
            self._enforce_equal_steps(batches)
        src = batches
        if self.world > 1 and not getattr(batches, "countable", True):
            batches = self._agreed_batches(batches)
        start_step = self.global_step
        use_graph = cfg.graph and self.native
        gsteps = max(1, int(getattr(cfg, "graph_steps", 1)))
        check_every = max(1, int(getattr(cfg, "time_check_steps", 20)))
        wd = Watchdog(cfg.watchdog_secs, self.rank).start()
        window = StepWindow()
        # streamed epochs of an InputPipeline land in its device ring when this loop releases the
        # slots (every run enqueued -> RingBatch.ring.release): no per-batch copy on this thread
        rpipe = getattr(src, "pipe", None)
        if rpipe is None and hasattr(src, "ring_steps"):
            rpipe = src
        if rpipe is not None and hasattr(rpipe, "ring_steps") and self.native and use_graph and gsteps > 1:
            rpipe.ring_steps = gsteps
        else:
            rpipe = None
        try:
            self._train_loop(batches, src, it=iter(batches), max_steps=max_steps, eval_fn=eval_fn,
                             eval_due=eval_due, wd=wd, window=window, use_graph=use_graph, gsteps=gsteps,
                             check_every=check_every)
        finally:
            if rpipe is not None:
                rpipe.ring_steps = 0
                if getattr(rpipe, "_ring", None) is not None:     # (slots an early exit still held)
                    rpipe._ring.release_all(torch.cuda.current_stream(self.device))
        if self.native:
            torch.cuda.synchronize(self.device)
            self.model.check_errors()
        wd.stop()
        return self.global_step - start_step

    def _train_loop(self, batches, src, it, max_steps, eval_fn, eval_due, wd, window, use_graph, gsteps,
                    check_every):
        cfg = self.cfg
        t_log = time.time()
        n_log = 0
        cur = self._next(it)
        while cur is not None:
            if max_steps is not None and self.global_step >= max_steps:
                break
            from_cache = bool(getattr(src, "from_cache", False)) or bool(
                getattr(getattr(src, "pipe", None), "from_cache", False))
            run = [cur]
            nxt = self._next(it)
            # streamed batches: a run of them is copied into a ring of static device buffers and
            # trained as ONE captured multi-step graph keyed by the ring (run-level sort), replayed
            # for every later run -- the cached epoch's fast path, without a cache
            ring = self.native and use_graph and gsteps > 1 and not from_cache and self._ring_ok(cur)
            if self.native and use_graph and gsteps > 1 and (from_cache or ring):
                lim = gsteps if max_steps is None else min(gsteps, max_steps - self.global_step)
                while len(run) < lim and nxt is not None and (from_cache or self._ring_ok(nxt)):
                    run.append(nxt)
                    nxt = self._next(it)
            t0 = time.perf_counter()
            B = int(run[0][0].shape[0])
            pos = getattr(run[-1], "pos", None)      # data position after this run (if tagged)
            if self.native:
                if not run[0][0].is_cuda:
                    t1 = time.perf_counter()
                    with prof_range("h2d"):
                        run = [tuple(x.to(self.device, non_blocking=True) for x in b) for b in run]
                    self.timer.add("h2d", time.perf_counter() - t1)
                released = [b for b in run if getattr(b, "ring", None) is not None]
                if ring and len(run) > 1:
                    run = self._ring_run(run)
                nxt_ids = nxt[0] if (nxt is not None and nxt[0].is_cuda) else None
                with prof_range("step"):
                    if len(run) > 1:
                        self.model.train_steps(run, next_ids=None if ring else nxt_ids)
                    else:
                        ids, vals, labels = run[0]
                        # replayed cache batches: bound in place (one graph per batch); one-off
                        # streamed batches: staged into the static buffers (one shared graph)
                        self.model.train_step(ids, vals, labels, use_graph=use_graph,
                                              next_ids=nxt_ids if from_cache else None,
                                              stage=not from_cache)
                if released:               # every kernel reading these ring slots is enqueued
                    released[0].ring.release([b.slot for b in released],
                                             torch.cuda.current_stream(self.device))
                # device error words (bad ids, capacity overflow, hand-off failures): copied
                # asynchronously after every call, raised on at the next one
                self.model.poll_errors()
                if cfg.debug_sync:
                    torch.cuda.synchronize(self.device)
                    self.model.check_errors()
                    self._nan_check()
            else:
                for ids, vals, labels in run:
                    self.model.train_step(ids, vals, labels, grad_sync=self._golden_grad_sync)
            self.timer.add("step_enqueue", time.perf_counter() - t0)
            prev = self.global_step - len(run)
            if pos is not None:
                self.epoch, self.epoch_batch = pos
            else:
                self.epoch_batch += len(run)
            n_log += B * len(run)
            step = self.global_step
            wd.beat(step)
            window.step(step)
            maybe_inject_fault(step, self.rank, prev)
            crossed = lambda every: bool(every) and step // every > prev // every  # noqa: E731
            if crossed(cfg.log_steps):
                if self.native:
                    torch.cuda.synchronize(self.device)
                dt = max(1e-9, time.time() - t_log)
                loss = self.model.loss_value(B) if self.native else self.model.last_loss
                sps = n_log / dt
                self.log.info(f"loss = {loss:.6f}, step = {step} ({dt:.3f} sec)")
                self.log.info(f"global_step/sec: {n_log / B / dt:.4g}")
                self.log.log("train", step=step, loss=loss, samples_per_sec_rank=sps,
                             samples_per_sec_job=sps * self.world, **self.timer.summary(),
                             comm_bytes=getattr(self.comm, "bytes_sent", 0))
                self._summary("train", step, {"loss": loss, "global_step/sec": n_log / B / dt,
                                              "examples/sec": sps * self.world})
                t_log, n_log = time.time(), 0
            if self.ckpt is not None:
                due = crossed(cfg.save_checkpoints_steps)
                if not cfg.save_checkpoints_steps and cfg.save_checkpoints_secs and crossed(check_every):
                    due = self._agreed_due(time.time() - self._last_save_t >= cfg.save_checkpoints_secs)
                if due:
                    self.save()
            if eval_fn is not None and crossed(cfg.eval_every_steps):
                eval_fn()
            elif eval_due is not None and crossed(check_every) and self._agreed_due(eval_due()):
                eval_fn_ps = getattr(eval_due, "run", None)
                if eval_fn_ps is not None:
                    eval_fn_ps()
            cur = nxt

    def agree_cache(self, pipeline) -> bool:
        """See ``agree_cache`` (module level): keep the cached epoch only if every rank has one."""
        return agree_cache(pipeline, self.world, self._ctl, self.log.info)

    def _ring_ok(self, b) -> bool:
        """A streamed batch can go through the staging ring: full batch of the model's size."""
        return (b is not None and int(b[0].shape[0]) == self.model.M and b[0].dim() == 2 and
                int(b[0].shape[1]) == self.cfg.field_size)

    def _ring_run(self, run):
        """A run of streamed batches as the executor trains it: consecutive slots of the pipeline's
        device ring -> that ring's persistent slot list (same list and buffers every time: one
        captured graph, replayed through the host fast path); anything else is copied into the
        estimator's own staging ring."""
        r0 = getattr(run[0], "ring", None)
        if r0 is not None:
            first = run[0].slot
            if all(getattr(b, "ring", None) is r0 and b.slot == first + i for i, b in enumerate(run)):
                return r0.run_list(first, len(run))
        return self._to_ring(run)

    def _to_ring(self, run):
        """Copy a run of streamed device batches into the staging ring (static buffers, so the
        run's captured graph is found again by the next run).  Stream-ordered: a slot is
        overwritten only after the previous run's graph, which read it, was enqueued."""
        m = self.model
        ring = getattr(self, "_ring", None)
        G = max(1, int(getattr(self.cfg, "graph_steps", 1)))
        if ring is None:
            dev, M, F = self.device, m.M, self.cfg.field_size
            ring = [(torch.empty(M, F, dtype=torch.int32, device=dev), torch.empty(M, F, dtype=torch.float32, device=dev),
                     torch.empty(M, dtype=torch.float32, device=dev)) for _ in range(G)]
            self._ring = ring
        out = []
        for slot, b in zip(ring, run):
            for dst, src in zip(slot, b):
                dst.copy_(src.reshape(dst.shape), non_blocking=True)
            out.append(PositionedBatch(slot, b.pos) if hasattr(b, "pos") else slot)
        return out

    def adopt_field_ranges(self, pipeline) -> bool:
        """After the first epoch was cached: per-field id ranges derived from it switch the slot
        sort to the per-field LDS sort (when the fields' ids are disjoint and increasing; with
        --field_sizes they are known from the start).  Returns True if the model took them.
        Every rank trains on its own shard, so the per-field min / max ids are combined over ALL
        ranks (MIN / MAX all-reduce) before the ranges are derived: ranges from one rank's shard
        could miss ids another rank sees.  The decision is then identical on every rank."""
        if not self.native or self.model.field_ranges is not None:
            return False
        from .data.pipeline import agreed_field_ranges
        r = agreed_field_ranges(pipeline, self.cfg.feature_size, self.world, self._ctl)
        if r is None:
            return False
        # earlier graph replays may still read the sort buffers this replaces
        torch.cuda.synchronize(self.device)
        self.model.set_field_ranges(r)
        self.log.info("per-field id ranges derived from the cached epoch: per-field slot sort on")
        return True

    def calibrate_exchange(self, pipeline, slack: float = 1.3, pad: int = 1024) -> bool:
        """After the first epoch was cached: measure the fixed-size exchange's capacity on the
        cached batches (unique ids per owner / per batch), agree on the MAX over ranks, and
        re-plan the exchange with it when it is smaller than the current (uncalibrated) one.  The
        margin covers evaluation batches, which route through the same exchange (an overflow
        raises, rows are never dropped).  Returns True if the exchange was re-planned."""
        m = self.model if self.native else None
        cached = getattr(pipeline, "_cached", None)
        if m is None or not m.exchange or m.exchange_capacity() is None:
            return False
        from .parallel.dist import agree_max, exchange_capacity
        have = agree_max(0 if not cached else 1, self._ctl)   # MAX: does any rank have a cache?
        have_all = -agree_max(-(1 if cached else 0), self._ctl)
        if not have or not have_all:
            return False
        cap = exchange_capacity((b[0] for b in cached), self.world, m.sharded, slack=slack, pad=pad,
                                group=self._ctl)
        if cap >= m.exchange_capacity():
            return False
        torch.cuda.synchronize(self.device)
        m.set_exchange_capacity(cap)
        self.log.info(f"exchange capacity calibrated on the cached epoch: {cap} "
                      f"({'per owner' if m.sharded else 'per rank'})")
        return True

    def _nan_check(self):
        for name, t in (("fm_v", self.model.tv), ("dense", self.model.p)):
            if not torch.isfinite(t).all():
                raise FloatingPointError(f"non-finite values in {name} at step {self.global_step}")

    # ------------------------------------------------------------------ evaluate / predict
    def evaluate(self, batches: Iterable, steps: Optional[int] = None) -> dict:
        t0 = time.perf_counter()
        with prof_range("eval"):
            res = self._evaluate(batches, steps)
        self.timer.add("eval", time.perf_counter() - t0)
        return res

    def _evaluate(self, batches: Iterable, steps: Optional[int] = None) -> dict:
        dev = self.device if self.native else torch.device("cpu")
        if self.native:
            self.model.check_errors()
        hist = torch.zeros(2, 201, dtype=torch.int64, device=dev)
        loss_sum = torch.zeros(1, dtype=torch.float64, device=dev)
        n = torch.zeros(1, dtype=torch.float64, device=dev)
        for b in self._lockstep(batches, steps):
            if b is None:                 # this rank's shard is done; the others' is not
                self.model.join_forward()
                continue
            ids, vals, labels = b
            B = ids.shape[0]
            if self.native:
                self.model.eval_batch(ids.to(dev), vals.to(dev), labels.to(dev), hist)
                loss_sum += self.model.eval_loss_sum.double()
            else:
                with torch.no_grad():
                    y = self.model.forward(ids, vals, train=False)
                    p = torch.sigmoid(y)
                    hist += hist_torch(p, labels)
                    _, data = self.model.loss(y, labels)
                    loss_sum += float(data) * B
            n += B
        if _dist_on():
            dist.all_reduce(hist)
            dist.all_reduce(loss_sum)
            dist.all_reduce(n)
        nn = max(1.0, float(n.item()))
        data_loss = float(loss_sum.item()) / nn
        l2 = self.model.l2_value() if self.native else float(
            self.cfg.l2_reg * 0.5 * ((self.model.params["fm_w"] ** 2).sum() + (self.model.params["fm_v"] ** 2).sum()))
        res = {"auc": auc_from_hist(hist.cpu()), "loss": data_loss + l2, "logloss": data_loss,
               "global_step": self.global_step, "examples": int(nn)}
        self._last_eval_t = time.time()
        self.log.info("Saving dict for global step %d: auc = %.6f, global_step = %d, loss = %.6f"
                      % (res["global_step"], res["auc"], res["global_step"], res["loss"]))
        self.log.log("eval", **res)
        self._summary("eval", res["global_step"], {"auc": res["auc"], "loss": res["loss"]})
        return res

    def _summary(self, kind: str, step: int, values: dict):
        """Scalar summaries for TensorBoard (reference: Estimator default hooks)."""
        if not self._tb_on:
            return
        from .utils.tfevents import EventFileWriter
        if kind == "train":
            if self._tb is None:
                self._tb = EventFileWriter(self.cfg.ckpt_dir)
            self._tb.scalars(step, values)
        else:
            if self._tb_eval is None:
                self._tb_eval = EventFileWriter(os.path.join(self.cfg.ckpt_dir, "eval"))
            self._tb_eval.scalars(step, values)

    @property
    def forward_collective(self) -> bool:
        """Every rank must run each forward pass together (row-sharded table at N > 1)."""
        return self.native and self.world > 1 and bool(getattr(self.model, "forward_collective", False))

    def _lockstep(self, batches: Iterable, steps: Optional[int] = None) -> Iterator:
        return lockstep_batches(batches, steps, self.forward_collective, self._ctl)

    def predict(self, batches: Iterable) -> Iterator[torch.Tensor]:
        """Probabilities per batch.  Collective forward passes (row-sharded table at N > 1): call
        it on EVERY rank -- ranks without batches (``[]``) join the others' passes and yield
        nothing."""
        for b in self._lockstep(batches):
            if b is None:
                self.model.join_forward()
                continue
            ids, vals, _ = b
            if self.native:
                yield self.model.predict(ids.to(self.device), vals.to(self.device)).cpu()
            else:
                yield self.model.predict(ids, vals)

    # ------------------------------------------------------------------ export
    def tf_variables(self):
        if self.native and self.model.sharded:
            raise NotImplementedError("TF-layout export of a row-sharded table: gather first "
                                      "(Estimator.export gathers when the table fits)")
        return self.model.tf_variables()

    def model_config(self) -> dict:
        c = self.cfg
        return {"feature_size": c.feature_size, "field_size": c.field_size,
                "embedding_size": c.embedding_size, "deep_layers": c.layers,
                "dropout_keep": c.keep_probs, "batch_norm": c.batch_norm, "loss_type": c.loss_type}

    def _write_tf_bundle(self, prefix: str, serve_only: bool = False) -> None:
        """Distributed TF1 ``tensor_bundle`` writer: one data shard per rank
        (``prefix.data-0000r-of-0000N``, the reference PS job's layout of one shard per PS task),
        every variable whole in one shard, the merged ``prefix.index`` by rank 0.  The big
        embedding variables are spread over the ranks; a row-sharded one is gathered onto its
        writer rank's GPU (never onto every rank or host) and streamed to disk in global row order
        in 256 MB chunks.  Optimizer slots are left out with ``serve_only`` (servable export)."""
        from .ckpt.export import is_training_only
        from .ckpt.tf_bundle import ShardWriter, write_index
        if self.native:
            srcs = self.model.tf_variable_sources()
        else:
            srcs = {k: (v, False, tuple(v.shape)) for k, v in self.model.tf_variables().items()}
        names = sorted(n for n in srcs if not (serve_only and is_training_only(n)))
        world, rank = self.world, self.rank
        big = sorted((n for n in names if srcs[n][0].numel() >= (1 << 20)),
                     key=lambda n: -srcs[n][0].numel())
        owner = {n: 0 for n in names}
        for i, n in enumerate(big):
            owner[n] = i % world
        sw = ShardWriter(prefix, rank, world)
        for n in names:
            t, sharded, shape = srcs[n]
            if sharded and world > 1:
                loc = t.contiguous()
                if dist.get_backend() == "gloo" and loc.is_cuda:
                    loc = loc.cpu()          # (gloo gathers host tensors: the same-device rehearsal)
                parts = [torch.empty_like(loc) for _ in range(world)] if rank == owner[n] else None
                dist.gather(loc, parts, dst=owner[n])
                if rank == owner[n]:
                    sw.add(n, shape, _interleaved_chunks(parts, shape[0]))
                del parts, loc
            elif rank == owner[n]:
                sw.add(n, shape, _row_chunks(t))
        sw.close()
        entries = sw.entries
        if world > 1:
            allv = [None] * world
            dist.all_gather_object(allv, entries, group=self._ctl)
            entries = [e for part in allv for e in part]
        if rank == 0:
            write_index(prefix, entries, world)
        if _dist_on():
            dist.barrier(group=self._ctl)

    def export(self, servable_dir: str) -> Optional[str]:
        """SavedModel directory (reference C33, PS:451-467): ``<dir>/<unix ts>/saved_model.pb``
        (MetaGraphDef with the serving_default signature) + ``variables/`` (multi-shard bundle
        written by every rank)."""
        if not servable_dir:
            return None
        from .ckpt.export import finish_servable
        ts = torch.tensor([int(time.time())], dtype=torch.int64)
        if _dist_on():
            dist.broadcast(ts, src=0, group=self._ctl)
        d = os.path.join(servable_dir, str(int(ts.item())))
        tmp = d + ".tmp"
        self._write_tf_bundle(os.path.join(tmp, "variables", "variables"), serve_only=True)
        path = None
        if self.rank == 0:
            path = finish_servable(tmp, d, self.model_config())
            self.log.info(f"SavedModel written to: {path}")
        if _dist_on():
            dist.barrier(group=self._ctl)
        return path

    def export_tf_checkpoint(self, model_dir: str) -> Optional[str]:
        """TF1 tensor_bundle ``model.ckpt-<step>`` + ``checkpoint`` state file (§2.7.4), one data
        shard per rank."""
        from .ckpt.tf_bundle import write_checkpoint_state
        name = f"model.ckpt-{self.global_step}"
        self._write_tf_bundle(os.path.join(model_dir, name))
        if self.rank != 0:
            return None
        write_checkpoint_state(model_dir, name, [name])
        return os.path.join(model_dir, name)


def lockstep_batches(batches: Iterable, steps: Optional[int], collective: bool, group=None) -> Iterator:
    """Batches of an evaluation / predict pass.  With ``collective`` forward passes (row-sharded
    table at N > 1) the ranks vote before every batch (MAX over the host control ``group``: does
    ANY rank still have one?) and a rank whose shard is exhausted gets ``None`` -- it joins that
    batch's collectives with a dummy batch -- until every rank is done.  Shards of unequal length
    (file-level sharding of va files, Pipe-mode evaluation read by rank 0 alone, predict on rank
    0's test files) then never leave a rank waiting inside an all-to-all its peers never issue."""
    it = iter(batches)
    k = 0
    while True:
        b = next(it, None) if (steps is None or k < steps) else None
        if collective:
            t = torch.tensor([0 if b is None else 1], dtype=torch.int32)
            dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
            if int(t.item()) == 0:
                return
        elif b is None:
            return
        k += 1
        yield b


def agree_cache(pipeline, world: int, group=None, log=None) -> bool:
    """After an epoch that may have filled the HBM cache: every rank keeps its cache only if EVERY
    rank has one (MIN over the host control ``group``).  Each rank checks its own shard against a
    budget from its own device, so one rank can overflow while another caches; the step path
    depends on the cache (captured multi-step runs with run-level routing vs staged single steps),
    so mixed decisions would issue different collective sequences on the shared communicator.
    Returns True if this rank's cache stays."""
    have = getattr(pipeline, "_cached", None) is not None
    if world == 1:
        return have
    t = torch.tensor([1 if have else 0], dtype=torch.int64)
    dist.all_reduce(t, op=dist.ReduceOp.MIN, group=group)
    if int(t.item()) == 1:
        return True
    if have and log is not None:
        log("another rank's epoch outgrew its cache budget: every rank streams")
    if hasattr(pipeline, "drop_cache"):
        pipeline.drop_cache()
    return False


def _row_chunks(t: torch.Tensor, chunk_bytes: int = 1 << 28):
    """Row blocks of a tensor for the bundle writer; bf16 embedding rows (mixed precision) are
    upcast to the fp32 TF variables block by block."""
    up = (lambda x: x.float()) if t.dtype == torch.bfloat16 else (lambda x: x)
    if t.dim() == 0 or t.numel() * 4 <= chunk_bytes:
        yield up(t)
        return
    rows = max(1, chunk_bytes // max(1, t[0].numel() * 4))
    for a in range(0, t.shape[0], rows):
        yield up(t[a:a + rows])


def _interleaved_chunks(parts, V: int, chunk_bytes: int = 1 << 28):
    """Global row order of a row-sharded table from its per-rank parts (global row = local row *
    N + rank), chunk by chunk on the device."""
    N = len(parts)
    R = parts[0].shape[0]
    row_bytes = max(1, parts[0][0].numel() * 4)        # blocks are upcast to fp32 below
    rows = max(1, chunk_bytes // (row_bytes * N))
    for a in range(0, R, rows):
        blk = torch.stack([p[a:a + rows].float() for p in parts], dim=1)
        blk = blk.reshape((-1,) + tuple(parts[0].shape[1:]))
        lo = a * N
        yield blk[: max(0, min(blk.shape[0], V - lo))]


def train_and_evaluate(est: Estimator, train_spec: TrainSpec, eval_spec: EvalSpec) -> dict:
    """tf.estimator.train_and_evaluate (PS:439-442): train; once ``start_delay_secs`` have passed,
    evaluate at most every ``throttle_secs`` -- each time on a freshly saved checkpoint, like
    TF's evaluator that evaluates the latest checkpoint -- and a final evaluation at the end.
    Time decisions are rank 0's and broadcast, so all ranks evaluate together."""
    t0 = time.time()
    last = {"t": None}

    def due() -> bool:
        now = time.time()
        return (now - t0 >= eval_spec.start_delay_secs and
                (last["t"] is None or now - last["t"] >= eval_spec.throttle_secs))

    def run():
        last["t"] = time.time()
        est.save()
        est.evaluate(eval_spec.input_fn(), eval_spec.steps)
    due.run = run
    est.train(train_spec.input_fn(), train_spec.max_steps, eval_due=due)
    est.save()
    return est.evaluate(eval_spec.input_fn(), eval_spec.steps)
