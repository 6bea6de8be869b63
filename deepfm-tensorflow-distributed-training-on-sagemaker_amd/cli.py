"""Entrypoint with the reference's flags and task dispatch (reference L5, PS:341-467, HVD:289-431).

  python -m hipfm --task_type train --training_data_dir D --val_data_dir V --model_dir M \
      --feature_size 117581 --field_size 39 --batch_size 1024 --deep_layers 128,64,32 ...
  python -m hipfm.launch --nproc_per_node 8 -m hipfm --task_type train ...     (data parallel)

task_type (PS:61):
  train   per epoch: train one epoch, then evaluate (HVD:390-394 file mode) — all ranks evaluate
          their shard (Q10); pipe mode: one pass over num_epochs FIFO epochs (HVD:396-405);
          then export the servable (train|export, PS:450-467)
  eval    evaluate va* files (PS:443-444)
  infer   predict te* files from val_data_dir -> "<val_data_dir>/pred.txt" ("%f\\n" per row,
          PS:445-449); ``--pred_path`` overrides (Q9)
  export  export the servable only
"""
from __future__ import annotations

import json
import os
import shutil
import sys
from typing import List, Optional, Sequence

import torch
import torch.distributed as dist

from .config import RunConfig, parse_flags
from .data.pipeline import InputPipeline, discover_files, shard_spec
from .estimator import Estimator, PositionedBatch


def _channels() -> List[str]:
    raw = os.environ.get("SM_CHANNELS")
    if not raw:
        return []
    try:
        return list(json.loads(raw))
    except ValueError:
        return [c for c in raw.split(",") if c]


def _init_dist(cfg: RunConfig):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world > 1 and not dist.is_initialized():
        from .parallel.dist import init_distributed, local_device_index
        dev = cfg.device
        backend = "gloo" if dev == "cpu" or (dev == "auto" and not torch.cuda.is_available()) else "nccl"
        if backend == "nccl":
            torch.cuda.set_device(local_device_index())
        init_distributed(backend)


def cache_budget_bytes(device, fraction: float = 0.8, reserve: int = 4 << 30) -> int:
    """Bytes the cached epoch may take: a fraction of the device memory still free once the
    model is allocated (minus a reserve for step buffers / graphs), or of available host RAM for
    the CPU path.  An epoch that outgrows it streams every epoch instead (data/pipeline.py)."""
    if device is not None and torch.device(device).type == "cuda":
        free, _ = torch.cuda.mem_get_info(device)
    else:
        import psutil
        free = psutil.virtual_memory().available
    return max(0, int(free * fraction) - reserve)


def build_pipelines(cfg: RunConfig, est: Estimator):
    rank, world = est.rank, est.world
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    fmt = cfg.data_format
    shard = shard_spec(world, rank, local_rank, cfg.worker_per_host, len(cfg.hosts),
                       cfg.enable_s3_shard, bool(cfg.pipe_mode), cfg.enable_data_multi_path)
    # native path: batches go to the GPU through pinned buffers + a copy stream, ids as int32 (the
    # device id type: no staging cast per step), and the first epoch stays HBM-resident (cache())
    dev = est.device if est.native else None
    id_dtype = torch.int32 if est.native else torch.int64
    common = dict(fmt=fmt, seed=cfg.seed, threads=max(1, min(os.cpu_count() or 1, cfg.num_threads)),
                  device=dev, id_dtype=id_dtype, id_limit=cfg.feature_size)
    if cfg.pipe_mode:
        ch = _channels()
        tr_ch = cfg.training_channel_name or (ch[1 + local_rank] if len(ch) > 1 + local_rank else "training")
        ev_ch = cfg.evaluation_channel_name or (ch[0] if ch else "evaluation")
        tr = lambda epochs: InputPipeline([], cfg.field_size, cfg.batch_size, epochs, shard=shard,
                                          pipe_channel=tr_ch, **common)

        # one FIFO has one reader: rank 0 evaluates the whole evaluation channel (HVD:403-405);
        # the other ranks contribute empty histograms to the all-reduced AUC
        def va():
            if rank != 0:
                return []
            return InputPipeline([], cfg.field_size, cfg.batch_size, 1, shard=(1, 0),
                                 pipe_channel=ev_ch, **{**common, "device": None})
        te = va
        return tr, va, te
    ext = "tfrecord" if fmt == "tfrecord" else "libsvm"
    tr_files = discover_files(cfg.training_data_dir, "tr", ext)
    va_files = discover_files(cfg.val_data_dir, "va", ext)
    te_files = discover_files(cfg.val_data_dir, "te", ext)
    est.log.info(f"tr_files: {tr_files}")
    est.log.info(f"va_files: {va_files}")
    est.log.info(f"te_files: {te_files}")
    cache_tr = InputPipeline(tr_files, cfg.field_size, cfg.batch_size, 1, shard=shard,
                             cache=cfg.cache_data, cache_budget=(cfg.cache_budget_mb << 20 if cfg.cache_budget_mb >= 0
                                           else cache_budget_bytes(est.device)), **common)

    def tr(epochs):
        return cache_tr
    va = lambda: InputPipeline(va_files, cfg.field_size, cfg.batch_size, 1, shard=(world, rank),
                               shuffle_files=False, **common)
    te = lambda: InputPipeline(te_files, cfg.field_size, cfg.batch_size, 1, shard=(1, 0),
                               shuffle_files=False, drop_remainder=False, **common)
    return tr, va, te


def run(cfg: RunConfig) -> dict:
    _init_dist(cfg)
    # CPU threading (reference C25: intra/inter-op threads = num_cpus, PS:405-432): torch's CPU
    # pool for the golden path and host-side tensor work; loader threads use the same budget
    torch.set_num_threads(max(1, cfg.num_threads))
    rank = dist.get_rank() if dist.is_initialized() else 0
    if rank == 0:
        print(sys.argv, flush=True)
        print(cfg.dump(), flush=True)
    if cfg.clear_existing_model and cfg.ckpt_dir and rank == 0:     # HVD:334-340
        try:
            shutil.rmtree(cfg.ckpt_dir)
            print(f"existing model cleaned at {cfg.ckpt_dir}")
        except Exception as e:  # noqa: BLE001
            print(e, "at clear_existing_model")
    if dist.is_initialized():
        dist.barrier()
    est = Estimator(cfg)
    tr, va, te = build_pipelines(cfg, est)
    result = {}
    if cfg.task_type == "train":
        max_steps = cfg.max_steps or None
        if cfg.schedule == "ps" and not cfg.pipe_mode:
            # PS recipe: train_and_evaluate(TrainSpec(all epochs), EvalSpec(start delay, throttle))
            from .estimator import EvalSpec, TrainSpec, train_and_evaluate
            pipe = tr(1)
            first, skip = est.epoch, est.epoch_batch
            if first >= cfg.num_epochs:
                first, skip = 0, 0

            def all_epochs():
                # every batch carries the data position AFTER it (PositionedBatch): the Estimator
                # reads more than one batch ahead (graph runs), so the generator's own progress
                # is not the trained position
                for epoch in range(first, cfg.num_epochs):
                    k = skip if epoch == first else 0
                    view = _EpochView(pipe, epoch, k)
                    est._enforce_equal_steps(view)
                    it = iter(view)
                    b = next(it, None)
                    while b is not None:
                        nb = next(it, None)
                        yield PositionedBatch(b, (epoch, k + 1) if nb is not None else (epoch + 1, 0))
                        k += 1
                        b = nb
                    est.agree_cache(pipe)
                    est.adopt_field_ranges(pipe)
                    est.calibrate_exchange(pipe)

            class _Run:                  # the whole run as one batch source (cache flag visible)
                countable = True

                def __iter__(self):
                    return all_epochs()
            _Run.pipe = pipe
            result = train_and_evaluate(est, TrainSpec(_Run, max_steps),
                                        EvalSpec(va, None, cfg.eval_start_delay_secs, cfg.eval_throttle_secs))
        elif cfg.pipe_mode:
            pipe = tr(cfg.num_epochs)
            est.train(pipe, max_steps, eval_fn=lambda: est.evaluate(va()))
            est.save()
            result = est.evaluate(va())
        else:
            pipe = tr(1)
            # resume from the checkpoint's data position: its epoch, minus the batches of that
            # epoch already trained on
            first, skip = est.epoch, est.epoch_batch
            if first >= cfg.num_epochs:
                # the checkpoint's run completed its epochs: this job trains num_epochs more on
                # top of it (the reference re-runs its epoch loop on restored weights, HVD:390-392)
                first, skip = 0, 0
            for epoch in range(first, cfg.num_epochs):
                pipe.num_epochs = 1
                est.epoch, est.epoch_batch = epoch, (skip if epoch == first else 0)
                est.train(_EpochView(pipe, epoch, est.epoch_batch), max_steps,
                          eval_fn=lambda: est.evaluate(va()))
                est.epoch, est.epoch_batch = epoch + 1, 0
                est.agree_cache(pipe)
                est.adopt_field_ranges(pipe)
                est.calibrate_exchange(pipe)
                result = est.evaluate(va())
                if max_steps is not None and est.global_step >= max_steps:
                    break
            est.save()
    elif cfg.task_type == "eval":
        result = est.evaluate(va())
    elif cfg.task_type == "infer":
        path = cfg.pred_path or os.path.join(cfg.val_data_dir, "pred.txt")
        if est.rank == 0:
            n = 0
            with open(path, "w") as fo:
                for prob in est.predict(te()):
                    for p in prob.tolist():
                        fo.write("%f\n" % p)
                        n += 1
            result = {"pred_path": path, "rows": n}
            est.log.info(f"wrote {n} predictions to {path}")
        elif est.forward_collective:
            # row-sharded table: rank 0's test batches need every rank's rows (each forward is a
            # collective); the other ranks serve them, batch for batch, and write nothing
            for _ in est.predict([]):
                pass
    if cfg.task_type in ("export", "train") and cfg.servable_model_dir:
        path = est.export(cfg.servable_model_dir)
        result["export_dir"] = path
    if cfg.task_type in ("export", "train") and cfg.export_tf_bundle and cfg.ckpt_dir:
        # the Estimator-style TF1 checkpoint model.ckpt-<step> next to the native one (§2.7.4)
        result["tf_checkpoint"] = est.export_tf_checkpoint(cfg.ckpt_dir)
    est.log.close()
    return result


class _EpochView:
    """One epoch of an InputPipeline (from batch ``skip`` on) that still exposes local_records
    (equal-steps logic)."""

    def __init__(self, pipe: InputPipeline, epoch: int, skip: int = 0):
        self.pipe, self.epoch, self.skip = pipe, epoch, int(skip)
        self.B = pipe.B

    @property
    def countable(self):
        return self.pipe.countable

    def local_records(self):
        return self.pipe.local_records(self.epoch)     # the whole epoch: max_batches counts skips

    @property
    def max_batches(self):
        return self.pipe.max_batches

    @max_batches.setter
    def max_batches(self, v):
        self.pipe.max_batches = v

    def __iter__(self):
        return self.pipe.iter_epoch(self.epoch, skip=self.skip)


def main(argv: Optional[Sequence[str]] = None) -> dict:
    cfg = parse_flags(argv)
    res = run(cfg)
    if dist.is_initialized():
        dist.barrier()
        dist.destroy_process_group()
    return res


if __name__ == "__main__":
    main()
