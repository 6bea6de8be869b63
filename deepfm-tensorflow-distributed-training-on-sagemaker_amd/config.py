"""Flag system (reference C01/C02/C09).

Same flag names, defaults and semantics as the reference scripts
(``1-ps-cpu/DeepFM-dist-ps-for-multipleCPU-multiInstance.py:35-71`` and
``2-hvd-gpu/DeepFM-hvd-tfrecord-vectorized-map.py:40-68``), parsed with argparse:

* unknown flags are tolerated with a warning (TF1 absl did the same for e.g.
  ``--perform_shuffle`` passed by the notebooks, ``NBPS:92``);
* ``SM_*`` SageMaker environment variables are optional inputs with local defaults
  (fixes quirk Q7: the reference crashes with ``json.loads(None)`` outside SageMaker);
* ``dropout`` values are *keep probabilities* (quirk Q3, ``PS:218``);
* ``optimizer=GD`` is implemented (quirk Q4; the reference advertises but crashes);
* ``log_steps`` is wired to training logging and ``loss_type=square_loss`` is implemented (Q5).

New MI355X-specific flags are grouped at the end of ``_DEFS``.
"""
from __future__ import annotations

import argparse
import dataclasses
import json
import os
import sys
import warnings
from typing import List, Optional, Sequence


def _str2bool(v) -> bool:
    if isinstance(v, bool):
        return v
    s = str(v).strip().lower()
    if s in ("1", "true", "t", "yes", "y"):
        return True
    if s in ("0", "false", "f", "no", "n", ""):
        return False
    raise argparse.ArgumentTypeError(f"not a boolean: {v!r}")


def _env_hosts() -> List[str]:
    raw = os.environ.get("SM_HOSTS")
    if not raw:
        return ["algo-1"]
    try:
        return list(json.loads(raw))
    except ValueError:
        return [h for h in raw.split(",") if h]


# (name, type, default, help)
_DEFS = [
    # ---- reference flags (PS:35-71, HVD:40-68) ----
    ("dist_mode", int, 0, "PS-only legacy flag (dead set_dist_env, Q6); accepted and ignored"),
    ("ps_hosts", str, "", "PS-only legacy flag; ignored"),
    ("worker_hosts", str, "", "PS-only legacy flag; ignored"),
    ("job_name", str, "", "PS-only legacy flag; ignored"),
    ("task_index", int, 0, "PS-only legacy flag; ignored"),
    ("num_threads", int, 16, "CPU threads for host-side work (reference: unused, Q5)"),
    ("feature_size", int, 0, "Number of features V (embedding table rows)"),
    ("field_size", int, 0, "Number of fields F"),
    ("embedding_size", int, 32, "Embedding size K"),
    ("num_epochs", int, 10, "Number of epochs"),
    ("batch_size", int, 64, "Per-worker batch size"),
    ("log_steps", int, 1000, "Log loss / throughput every N steps"),
    ("learning_rate", float, 0.0005, "Learning rate (x world size under data parallelism, HVD:149)"),
    ("l2_reg", float, 0.0001, "L2 regularization on fm_w and fm_v (whole tables, PS:244-246)"),
    ("loss_type", str, "log_loss", "loss type {log_loss, square_loss}"),
    ("optimizer", str, "Adam", "optimizer {Adam, Adagrad, GD, Momentum, ftrl}"),
    ("deep_layers", str, "256,128,64", "deep layers (csv)"),
    ("dropout", str, "0.5,0.5,0.5", "dropout KEEP probabilities per deep layer (csv)"),
    ("batch_norm", _str2bool, False, "batch normalization after ReLU in the deep part"),
    ("batch_norm_decay", float, 0.9, "moving-average decay for batch norm"),
    ("training_data_dir", str, "", "training data dir (tr*.tfrecords, recursive)"),
    ("val_data_dir", str, "", "validation data dir (va*/te*.tfrecords; pred.txt is written here)"),
    ("model_dir", str, "", "checkpoint dir (PS flag name)"),
    ("checkpoint_dir", str, "", "checkpoint dir (HVD flag name; alias of model_dir)"),
    ("servable_model_dir", str, "", "export servable model dir"),
    ("task_type", str, "train", "task type {train, eval, infer, export}"),
    ("clear_existing_model", _str2bool, False, "remove checkpoint_dir before training"),
    ("current_host", str, os.environ.get("SM_CURRENT_HOST", "algo-1"), "this host's name"),
    ("pipe_mode", int, 0, "read records from a stream/FIFO channel instead of files"),
    ("worker_per_host", int, 1, "worker processes per host (shard math)"),
    ("training_channel_name", str, "", "training channel name (pipe mode)"),
    ("evaluation_channel_name", str, "", "evaluation channel name (pipe mode)"),
    ("enable_s3_shard", _str2bool, False, "data is pre-sharded per host (ShardedByS3Key)"),
    ("enable_data_multi_path", _str2bool, False, "each channel holds a different pre-split path (pipe mode)"),
    # ---- hipfm (MI355X) flags ----
    ("device", str, "auto", "auto | cuda | cpu  (cuda = native HIP kernels; cpu = golden PyTorch path)"),
    ("seed", int, 1234, "global seed (params init, dropout RNG, data order)"),
    ("data_format", str, "tfrecord", "tfrecord | libsvm"),
    ("embedding_mode", str, "auto", "auto | replicated | sharded (row-sharded table + all-to-all)"),
    ("sparse_update", str, "tf1_dense", "tf1_dense (reference non-lazy semantics: every row moves "
     "every step, full-table L2) | lazy (touched rows only)"),
    ("mlp_dtype", str, "bf16", "bf16 | fp8 (deep-part GEMM input precision; accumulation is fp32)"),
    ("emb_dtype", str, "fp32", "fp32 | bf16: fm_v rows + their optimizer slots (bf16: stochastic "
     "rounding, lazy updates, gather-fused tower; config #5 mixed-precision embeddings)"),
    ("save_checkpoints_steps", int, 0, "checkpoint every N steps (0: use save_checkpoints_secs)"),
    ("save_checkpoints_secs", int, 600, "checkpoint every N seconds (TF Estimator default 600)"),
    ("keep_checkpoint_max", int, 5, "checkpoints to keep (TF default 5)"),
    ("eval_every_steps", int, 0, "evaluate every N steps during train (0: per epoch, rank-parallel)"),
    ("schedule", str, "hvd", "hvd: per-epoch train + evaluate (HVD:390-394) | ps: train_and_evaluate with "
     "throttled evaluation (PS:439-442)"),
    ("eval_start_delay_secs", float, 1000.0, "ps schedule: no evaluation before this (EvalSpec default "
     "of the reference, PS:441)"),
    ("eval_throttle_secs", float, 1200.0, "ps schedule: at most one evaluation per this many seconds "
     "(PS:441)"),
    ("time_check_steps", int, 20, "steps between the (rank-agreed) checks of time-based triggers"),
    ("graph_steps", int, 32, "consecutive steps over the HBM-cached epoch captured per HIP graph "
     "(Kaggle-shape CLI run: 32 -> 6,121 vs 8 -> 5,992 steps/s)"),
    ("field_sizes", str, "", "csv per-field vocabulary sizes (fields own consecutive id ranges): "
     "enables the per-field slot sort; empty: derived from the first cached epoch when possible"),
    ("pred_path", str, "", "predictions output file (default <val_data_dir>/pred.txt, Q9)"),
    ("export_tf_bundle", _str2bool, True, "also write a TF1 tensor_bundle checkpoint on export"),
    ("metrics_file", str, "", "JSONL metrics output (default <model_dir>/metrics.jsonl)"),
    ("cache_data", _str2bool, True, "keep the decoded dataset resident in device memory (cache())"),
    ("cache_budget_mb", int, -1, "most MB the cached epoch may take (-1: 80 % of the device memory "
     "free after the model is allocated, minus 4 GB); a larger epoch streams every epoch"),
    ("graph", _str2bool, True, "capture the train step in a HIP graph when possible"),
    ("max_steps", int, 0, "stop after this many steps (0 = run num_epochs)"),
    ("debug_sync", _str2bool, False, "synchronize + NaN/Inf check after each step (debug mode)"),
    ("watchdog_secs", float, 1800.0, "abort a rank whose training step stalls this long (0 = off)"),
]


@dataclasses.dataclass
class RunConfig:
    """Parsed flags.  Field names equal the reference flag names."""

    dist_mode: int = 0
    ps_hosts: str = ""
    worker_hosts: str = ""
    job_name: str = ""
    task_index: int = 0
    num_threads: int = 16
    feature_size: int = 0
    field_size: int = 0
    embedding_size: int = 32
    num_epochs: int = 10
    batch_size: int = 64
    log_steps: int = 1000
    learning_rate: float = 0.0005
    l2_reg: float = 0.0001
    loss_type: str = "log_loss"
    optimizer: str = "Adam"
    deep_layers: str = "256,128,64"
    dropout: str = "0.5,0.5,0.5"
    batch_norm: bool = False
    batch_norm_decay: float = 0.9
    training_data_dir: str = ""
    val_data_dir: str = ""
    model_dir: str = ""
    checkpoint_dir: str = ""
    servable_model_dir: str = ""
    task_type: str = "train"
    clear_existing_model: bool = False
    current_host: str = "algo-1"
    pipe_mode: int = 0
    worker_per_host: int = 1
    training_channel_name: str = ""
    evaluation_channel_name: str = ""
    enable_s3_shard: bool = False
    enable_data_multi_path: bool = False
    device: str = "auto"
    seed: int = 1234
    data_format: str = "tfrecord"
    embedding_mode: str = "auto"
    sparse_update: str = "tf1_dense"
    mlp_dtype: str = "bf16"
    emb_dtype: str = "fp32"
    save_checkpoints_steps: int = 0
    save_checkpoints_secs: int = 600
    keep_checkpoint_max: int = 5
    eval_every_steps: int = 0
    schedule: str = "hvd"
    eval_start_delay_secs: float = 1000.0
    eval_throttle_secs: float = 1200.0
    time_check_steps: int = 20
    graph_steps: int = 32
    field_sizes: str = ""
    pred_path: str = ""
    export_tf_bundle: bool = True
    metrics_file: str = ""
    cache_data: bool = True
    cache_budget_mb: int = -1
    graph: bool = True
    max_steps: int = 0
    debug_sync: bool = False
    watchdog_secs: float = 1800.0
    hosts: List[str] = dataclasses.field(default_factory=_env_hosts)

    # ---- derived views (reference C09: CSV parsing with list(map(...)), PS:153-163) ----
    @property
    def layers(self) -> List[int]:
        return [int(x) for x in str(self.deep_layers).split(",") if x.strip()]

    @property
    def keep_probs(self) -> List[float]:
        return [float(x) for x in str(self.dropout).split(",") if x.strip()]

    @property
    def ckpt_dir(self) -> str:
        return self.checkpoint_dir or self.model_dir

    def model_params(self) -> dict:
        """The reference's ``model_params`` dict (PS:391-400)."""
        return {
            "field_size": self.field_size,
            "feature_size": self.feature_size,
            "embedding_size": self.embedding_size,
            "learning_rate": self.learning_rate,
            "batch_norm_decay": self.batch_norm_decay,
            "l2_reg": self.l2_reg,
            "deep_layers": self.deep_layers,
            "dropout": self.dropout,
        }

    def validate(self) -> None:
        if self.optimizer not in ("Adam", "Adagrad", "GD", "Momentum", "ftrl"):
            raise ValueError(f"unknown optimizer {self.optimizer!r}")
        if self.task_type not in ("train", "eval", "infer", "export"):
            raise ValueError(f"unknown task_type {self.task_type!r}")
        if self.loss_type not in ("log_loss", "square_loss"):
            raise ValueError(f"unknown loss_type {self.loss_type!r}")
        if self.sparse_update not in ("tf1_dense", "lazy"):
            raise ValueError(f"unknown sparse_update {self.sparse_update!r}")
        if self.mlp_dtype not in ("bf16", "fp8"):
            raise ValueError(f"unknown mlp_dtype {self.mlp_dtype!r} (bf16 | fp8)")
        if self.emb_dtype not in ("fp32", "bf16"):
            raise ValueError(f"unknown emb_dtype {self.emb_dtype!r} (fp32 | bf16)")
        if self.schedule not in ("hvd", "ps"):
            raise ValueError(f"unknown schedule {self.schedule!r} (hvd | ps)")
        if self.field_sizes:
            fs = [int(x) for x in self.field_sizes.split(",") if x.strip()]
            if len(fs) != self.field_size or sum(fs) > self.feature_size or min(fs) < 1:
                raise ValueError("field_sizes: one positive size per field, summing to <= feature_size")
        if self.embedding_mode not in ("auto", "replicated", "sharded"):
            raise ValueError(f"unknown embedding_mode {self.embedding_mode!r}")
        kp = self.keep_probs
        if len(kp) != len(self.layers):
            raise ValueError("dropout must have one keep-prob per deep layer")
        if any(not (0.0 < p <= 1.0) for p in kp):
            raise ValueError("dropout values are keep probabilities in (0, 1]")

    def dump(self) -> str:
        """Startup flag dump (reference C35 prints every flag, HVD:298-314)."""
        d = dataclasses.asdict(self)
        return "\n".join(f"{k} {d[k]}" for k in sorted(d))


def build_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(prog="hipfm", allow_abbrev=False,
                                description="MI355X-native DeepFM (flag-compatible with the reference)")
    for name, typ, default, helptext in _DEFS:
        p.add_argument(f"--{name}", type=typ, default=default, help=helptext)
    p.add_argument("--hosts", type=lambda s: [h for h in s.split(",") if h], default=None,
                   help="comma-separated host list (default: $SM_HOSTS or ['algo-1'])")
    return p


def parse_flags(argv: Optional[Sequence[str]] = None) -> RunConfig:
    """Parse ``argv`` into a RunConfig.  Unknown flags warn instead of failing."""
    parser = build_parser()
    ns, unknown = parser.parse_known_args(list(sys.argv[1:] if argv is None else argv))
    if unknown:
        warnings.warn(f"ignoring unknown flags: {unknown}")
    d = vars(ns)
    hosts = d.pop("hosts")
    cfg = RunConfig(**d)
    if hosts:
        cfg.hosts = hosts
    return cfg
