"""Native checkpoints: per-rank tensor files + JSON manifest, atomic publish, auto-resume.

Reference behaviour: Estimator saves ``model.ckpt-<step>`` every 600 s
keeping the last 5, restores the latest checkpoint of ``model_dir`` on every ``train()``; under
Horovod only rank 0 writes (HVD:359,365-368).  Here:

* every rank writes its OWN state (a row-sharded table is saved shard by shard: no gather),
  streamed in chunks from HBM (an 882M-row table never needs a host-side full copy);
* a checkpoint is written to ``ckpt-<step>.partial/`` and published by an atomic rename after
  all ranks finished (write-then-rename), then ``hipfm_checkpoint.json`` is updated;
* ``keep_checkpoint_max`` old checkpoints are pruned;
* the manifest records the world size and the sharding function (owner = id % N, row = id // N)
  so a job can resume with a different number of GPUs (``restore`` reshards row tables);
* tensors carry CRC32C checksums (verified on load).
Interop with TensorFlow's layout (variable names, ``[in, out]`` weights, tensor_bundle files) is
in ``tf_bundle.py`` / ``export.py``.
"""
from __future__ import annotations

import json
import os
import shutil
import time
from typing import Callable, Dict, List, Optional

import numpy as np
import torch

from ..data import native_io as nio

INDEX = "hipfm_checkpoint.json"
ALIGN = 64
_DT = {torch.float32: "f32", torch.int64: "i64", torch.int32: "i32", torch.bfloat16: "bf16",
       torch.float64: "f64", torch.uint8: "u8"}
_DT_INV = {v: k for k, v in _DT.items()}


def _tensor_bytes_iter(t: torch.Tensor, chunk: int = 1 << 28):
    t = t.detach()
    if not t.is_contiguous() and t.dim() >= 1 and t.shape[0] > 0:
        # strided views (row-record table layout): stream row blocks, never a full-table copy
        row_bytes = max(1, t[0].numel() * t.element_size())
        rows = max(1, chunk // row_bytes)
        for i in range(0, t.shape[0], rows):
            yield from _tensor_bytes_iter(t[i: i + rows].contiguous(), chunk)
        return
    t = t.contiguous().view(-1)
    es = t.element_size()
    step = max(1, chunk // es)
    for i in range(0, t.numel(), step):
        part = t[i: i + step]
        if part.dtype == torch.bfloat16:
            part = part.view(torch.int16)
        yield part.cpu().numpy().tobytes()


def write_tensors(path: str, tensors: Dict[str, torch.Tensor]) -> Dict[str, dict]:
    index = {}
    off = 0
    with open(path, "wb") as f:
        for name, t in tensors.items():
            pad = (-off) % ALIGN
            if pad:
                f.write(b"\0" * pad)
                off += pad
            crc, n = 0, 0
            for b in _tensor_bytes_iter(t):
                f.write(b)
                crc = nio.crc32c_extend(crc, b)
                n += len(b)
            index[name] = {"dtype": _DT[t.dtype], "shape": list(t.shape), "offset": off,
                           "nbytes": n, "crc32c": crc}
            off += n
    return index


def read_tensor(path: str, meta: dict, verify: bool = True, device=None) -> torch.Tensor:
    dt = _DT_INV[meta["dtype"]]
    np_dt = {torch.float32: np.float32, torch.int64: np.int64, torch.int32: np.int32,
             torch.bfloat16: np.int16, torch.float64: np.float64, torch.uint8: np.uint8}[dt]
    mm = np.memmap(path, dtype=np.uint8, mode="r", offset=meta["offset"], shape=(meta["nbytes"],)) \
        if meta["nbytes"] else np.zeros(0, np.uint8)
    if verify and meta["nbytes"]:
        crc = 0
        step = 1 << 28
        for i in range(0, meta["nbytes"], step):
            crc = nio.crc32c_extend(crc, bytes(mm[i: i + step]))
        if crc != meta["crc32c"]:
            raise IOError(f"checkpoint tensor CRC mismatch in {path}")
    arr = np.frombuffer(bytes(mm), dtype=np_dt).reshape(meta["shape"]) if meta["nbytes"] else \
        np.zeros(meta["shape"], np_dt)
    t = torch.from_numpy(arr.copy())
    if dt == torch.bfloat16:
        t = t.view(torch.bfloat16)
    return t.to(device) if device is not None else t


class CheckpointManager:
    def __init__(self, model_dir: str, keep_max: int = 5, rank: int = 0, world: int = 1,
                 barrier: Optional[Callable[[], None]] = None):
        self.dir = model_dir
        self.keep = max(1, int(keep_max))
        self.rank, self.world = rank, world
        self.barrier = barrier or (lambda: None)
        if model_dir:
            os.makedirs(model_dir, exist_ok=True)

    # -------------------------------------------------------------- index
    def _index_path(self):
        return os.path.join(self.dir, INDEX)

    def index(self) -> dict:
        p = self._index_path()
        if not os.path.exists(p):
            return {"latest": None, "all": []}
        return json.load(open(p))

    def latest(self) -> Optional[str]:
        if not self.dir:
            return None
        idx = self.index()
        if idx.get("latest") and os.path.isdir(os.path.join(self.dir, idx["latest"])):
            return os.path.join(self.dir, idx["latest"])
        return None

    # -------------------------------------------------------------- save
    def save(self, step: int, state: Dict[str, torch.Tensor], meta: dict) -> str:
        name = f"ckpt-{step}"
        final = os.path.join(self.dir, name)
        part = final + ".partial"
        if self.rank == 0:
            if os.path.exists(part):
                shutil.rmtree(part)
            os.makedirs(part, exist_ok=True)
        self.barrier()
        os.makedirs(part, exist_ok=True)
        idx = write_tensors(os.path.join(part, f"rank{self.rank}.bin"), state)
        with open(os.path.join(part, f"rank{self.rank}.json"), "w") as f:
            json.dump({"tensors": idx, "meta": meta}, f)
        self.barrier()
        if self.rank == 0:
            with open(os.path.join(part, "manifest.json"), "w") as f:
                json.dump({"step": step, "world": self.world, "time": time.time(), "meta": meta,
                           "sharding": meta.get("sharding", "replicated")}, f, indent=1)
            if os.path.exists(final):
                shutil.rmtree(final)
            os.replace(part, final)                       # atomic publish
            idx_all = [c for c in self.index().get("all", []) if c != name] + [name]
            while len(idx_all) > self.keep:
                old = idx_all.pop(0)
                shutil.rmtree(os.path.join(self.dir, old), ignore_errors=True)
            tmp = self._index_path() + ".tmp"
            with open(tmp, "w") as f:
                json.dump({"latest": name, "all": idx_all}, f, indent=1)
            os.replace(tmp, self._index_path())
        self.barrier()
        return final

    # -------------------------------------------------------------- restore
    def load_manifest(self, path: str) -> dict:
        return json.load(open(os.path.join(path, "manifest.json")))

    def load_rank(self, path: str, rank: int, device=None, verify: bool = True,
                  names: Optional[List[str]] = None) -> Dict[str, torch.Tensor]:
        info = json.load(open(os.path.join(path, f"rank{rank}.json")))
        out = {}
        for k, m in info["tensors"].items():
            if names is not None and k not in names:
                continue
            out[k] = read_tensor(os.path.join(path, f"rank{rank}.bin"), m, verify, device)
        return out


def reshard_rows(path: str, name: str, old_world: int, new_world: int, new_rank: int,
                 local_rows: int, row_shape: tuple, device=None) -> torch.Tensor:
    """Assemble this rank's rows of a mod-sharded table from an N_old-rank checkpoint.

    Global id g lives at (rank g % N, row g // N); the new rank r' owns ids g % N' == r'."""
    out = torch.zeros((local_rows,) + tuple(row_shape), dtype=torch.float32)
    mgr = CheckpointManager(os.path.dirname(path))
    for r in range(old_world):
        t = mgr.load_rank(path, r, names=[name])[name]
        n = t.shape[0]
        g = torch.arange(n, dtype=torch.int64) * old_world + r
        keep = (g % new_world) == new_rank
        rows = (g[keep] // new_world)
        ok = rows < local_rows
        out[rows[ok]] = t[keep][ok].float()
    return out.to(device) if device is not None else out
