"""Parameter and state I/O of the native executor (``NativeDeepFM``): TF-named parameter
loading (reference variable names and layouts), the host step mirror, the native
checkpoint state (local shard + replicated dense state), and the TF1 ``tensor_bundle`` variable
views (fm_w / fm_v and the Adam / Adagrad / Momentum / FTRL slots, upcast from bf16 tables).

A mixin of ``models.deepfm.NativeDeepFM``: it reads the executor's buffers (flat dense parameters
``p`` and their segments, the embedding record ``rec`` / views ``tv``, ``tw``, slots ``sv``) but
launches no step kernels.
"""
from __future__ import annotations

from collections import OrderedDict
from typing import Dict, List, Optional

import torch


class NativeStateMixin:
    # ------------------------------------------------------------------ parameters
    def load_tf_params(self, params: Dict[str, torch.Tensor]):
        """Load TF-named / TF-layout parameters (reference §2.7.4) into the native buffers."""
        with torch.no_grad():
            fw, fv = params.get("fm_w"), params.get("fm_v")
            if fw is None:
                pass
            elif self.sharded:
                r, N = self.rank, self.world
                self.tw.zero_()
                self.tv.zero_()
                loc_w = fw[r::N].to(self.device, torch.float32)
                loc_v = fv[r::N].to(self.device, torch.float32)
                self.tw[: loc_w.shape[0]].copy_(loc_w)
                self.tv[: loc_v.shape[0]].copy_(loc_v)
            else:
                self.tw.copy_(fw.to(self.device, torch.float32))
                self.tv.copy_(fv.to(self.device, torch.float32))
            self.p.zero_()
            for name, s in self.dense_segs.items():
                if name not in params:
                    continue
                self._dense_view(self.p, s).copy_(self._tf_to_native(name, params[name]).to(self.device))
            for i in range(len(self.bn_mm)):
                for key, dst in ((f"Deep-part/bn_{i}/moving_mean", self.bn_mm[i]),
                                 (f"Deep-part/bn_{i}/moving_variance", self.bn_mv[i])):
                    if key in params:
                        t = params[key].detach().reshape(-1).to(self.device, torch.float32)
                        dst[: t.numel()].copy_(t)
        self.refresh_shadows()

    def _dense_view(self, flat: torch.Tensor, s: DenseSeg) -> torch.Tensor:
        n = int(torch.Size(s.shape).numel())
        return flat[s.off: s.off + n].view(s.shape)

    def _tf_to_native(self, name: str, t: torch.Tensor) -> torch.Tensor:
        s = self.dense_segs[name]
        t = t.detach().float().cpu()
        out = torch.zeros(s.shape, dtype=torch.float32)
        if name.endswith("/weights") and "deep_out" not in name:
            din, L = t.shape
            out[:L, :din] = t.t()
        elif "deep_out/weights" in name:
            out[: t.shape[0]] = t.reshape(-1)
        else:
            out[: t.numel()] = t.reshape(-1)
        return out

    def _native_to_tf(self, name: str, flat: torch.Tensor) -> torch.Tensor:
        s = self.dense_segs[name]
        v = self._dense_view(flat, s).detach().float().cpu()
        if name.endswith("/weights") and "deep_out" not in name:
            din, L = s.tf_shape
            return v[:L, :din].t().contiguous()
        n = int(torch.Size(s.tf_shape).numel())
        return v.reshape(-1)[:n].reshape(s.tf_shape).clone()

    def dense_tf_params(self, flat: Optional[torch.Tensor] = None) -> "OrderedDict[str, torch.Tensor]":
        flat = self.p if flat is None else flat
        return OrderedDict((n, self._native_to_tf(n, flat)) for n in self.dense_segs)

    # ------------------------------------------------------------------ state export
    def global_step(self) -> int:
        """Host mirror of the device step counter: read once (sync), then advanced by
        train_step, so the training loop never blocks on the GPU just to know the step."""
        if self._host_step is None:
            self._host_step = int(self.step.item())
        return self._host_step

    def sparse_tables_tf(self):
        """fm_w / fm_v of THIS rank (full tables when replicated; local rows when sharded)."""
        return self.tw, self.tv

    # ------------------------------------------------------------------ checkpoint protocol
    SLOT_NAMES = {"Adam": ("Adam", "Adam_1"), "Adagrad": ("Adagrad", None),
                  "Momentum": ("Momentum", None), "ftrl": ("Ftrl", "Ftrl_1"), "GD": (None, None)}

    def state_dict_local(self) -> "OrderedDict[str, torch.Tensor]":
        """This rank's state in native layout (row-sharded tables: local rows only)."""
        d = OrderedDict(fm_v=self.tv, fm_w=self.tw, dense=self.p, global_step=self.step)
        for i, t in enumerate(self.sv):
            if t.numel():
                d[f"fm_slot{i}"] = t
        for i, t in enumerate(self.sd):
            if t.numel():
                d[f"dense_slot{i}"] = t
        if self.batch_norm:
            d["bn_moving"] = self.bn_moving
        return d

    def replicated_state(self) -> List[torch.Tensor]:
        """Tensors every rank must hold identically (broadcast from rank 0 at start, like the
        reference's BroadcastGlobalVariablesHook(0), HVD:372): dense params + slots + step, and
        the tables/slots when the table is replicated rather than row-sharded."""
        out = [self.p, self.step] + [t for t in self.sd if t.numel()]
        if self.batch_norm:
            out.append(self.bn_moving)
        if not self.sharded:
            if self.record:
                out.append(self.rec)          # collectives need contiguous tensors
            else:
                out += [self.tv, self.tw] + [t for t in self.sv if t.numel()]
        return out

    def ckpt_meta(self) -> dict:
        return {"format": "hipfm-native", "V": self.V, "F": self.F, "K": self.K,
                "layers": self.layers, "keep": self.keep, "optimizer": self.optimizer,
                "world": self.world, "rank": self.rank, "R": self.R, "batch_norm": self.batch_norm,
                "emb_dtype": "bf16" if self.emb_bf16 else "fp32",
                "sharding": "mod" if self.sharded else "replicated", "P": self.P,
                "dense_segs": [[s.name, s.off, list(s.shape), list(s.tf_shape)]
                               for s in self.dense_segs.values()]}

    def load_state_dict_local(self, d: Dict[str, torch.Tensor]):
        self._host_step = None
        cur = self.state_dict_local()
        with torch.no_grad():
            for k, v in d.items():
                if k in cur:
                    if cur[k].shape != v.shape:
                        raise ValueError(f"checkpoint tensor {k}: shape {tuple(v.shape)} != "
                                         f"model {tuple(cur[k].shape)}")
                    cur[k].copy_(v.to(cur[k].device, cur[k].dtype))
        self.refresh_shadows()
        self._reset_sync()
        self._drop_graphs()

    def tf_variables(self, tables=None, upcast: bool = True) -> "OrderedDict[str, torch.Tensor]":
        """TF1 checkpoint view: reference variable names, [in,out] weights,
        optimizer slots ``<var>/Adam`` ..., ``beta{1,2}_power``, ``global_step``.
        ``tables=(fm_w, fm_v, slots...)`` overrides the local tables (gathered full tables).
        bf16 embedding rows are returned as fp32 (TF's variables are fp32) unless ``upcast`` is
        off (the chunked bundle writer upcasts chunk by chunk)."""
        out = OrderedDict()
        dense = self.dense_tf_params()
        tw, tv = (self.tw, self.tv) if tables is None else tables[:2]
        sv = self.sv if tables is None else tables[2]
        if upcast and tv.dtype != torch.float32:
            tv = tv.float()
            sv = [t.float() if t.dtype != torch.float32 else t for t in sv]
        out["fm_bias"] = dense["fm_bias"]
        out["fm_w"], out["fm_v"] = tw, tv
        for k, v in dense.items():
            if k != "fm_bias":
                out[k] = v
        for i, L in enumerate(self.layers[: len(self.bn_mm)]):
            out[f"Deep-part/bn_{i}/moving_mean"] = self.bn_mm[i][:L].detach().cpu().clone()
            out[f"Deep-part/bn_{i}/moving_variance"] = self.bn_mv[i][:L].detach().cpu().clone()
        s0n, s1n = self.SLOT_NAMES[self.optimizer]
        for slot_i, sname in ((0, s0n), (1, s1n)):
            if sname is None:
                continue
            if self.sd[slot_i].numel():
                for k, v in self.dense_tf_params(self.sd[slot_i]).items():
                    out[f"{k}/{sname}"] = v
            vt, wt = sv[slot_i], sv[2 + slot_i]
            if vt.numel():
                out[f"fm_v/{sname}"] = vt
                out[f"fm_w/{sname}"] = wt
        t = self.global_step()
        out["global_step"] = torch.tensor(t, dtype=torch.int64)
        if self.optimizer == "Adam":
            out["beta1_power"] = torch.tensor(0.9 ** (t + 1), dtype=torch.float32)
            out["beta2_power"] = torch.tensor(0.999 ** (t + 1), dtype=torch.float32)
        return out

    def tf_variable_sources(self) -> "OrderedDict[str, tuple]":
        """name -> (tensor, row_sharded, TF shape) for a distributed TF checkpoint writer: the
        embedding tables and their slots are THIS rank's local rows when row-sharded (global row =
        local row * N + rank), everything else is the full tensor."""
        out = OrderedDict()
        full = self.tf_variables(upcast=False)
        tables = {"fm_w": (self.tw, (self.V,)), "fm_v": (self.tv, (self.V, self.K))}
        s0n, s1n = self.SLOT_NAMES[self.optimizer]
        for slot_i, sname in ((0, s0n), (1, s1n)):
            if sname is not None and self.sv[slot_i].numel():
                tables[f"fm_v/{sname}"] = (self.sv[slot_i], (self.V, self.K))
                tables[f"fm_w/{sname}"] = (self.sv[2 + slot_i], (self.V,))
        for k, v in full.items():
            if k in tables:
                t, shape = tables[k]
                out[k] = (t, self.sharded, shape)
            else:
                out[k] = (v, False, tuple(v.shape))
        return out

    def load_tf_variables(self, tv: Dict[str, torch.Tensor]):
        """Inverse of ``tf_variables`` for replicated tables (params + slots + step)."""
        self.load_tf_params({k: torch.as_tensor(v) for k, v in tv.items()
                             if k in ("fm_w", "fm_v") or k in self.dense_segs or "moving_" in k})
        s0n, s1n = self.SLOT_NAMES[self.optimizer]
        with torch.no_grad():
            for slot_i, sname in ((0, s0n), (1, s1n)):
                if sname is None:
                    continue
                if self.sd[slot_i].numel():
                    for name, s in self.dense_segs.items():
                        key = f"{name}/{sname}"
                        if key in tv:
                            self._dense_view(self.sd[slot_i], s).copy_(
                                self._tf_to_native(name, torch.as_tensor(tv[key])).to(self.device))
                for tname, dst in (("fm_v", self.sv[slot_i]), ("fm_w", self.sv[2 + slot_i])):
                    key = f"{tname}/{sname}"
                    if key in tv and dst.numel() and not self.sharded:
                        dst.copy_(torch.as_tensor(tv[key]).to(dst))
            if "global_step" in tv:
                self.step.fill_(int(torch.as_tensor(tv["global_step"])))
                self._host_step = None
                self._reset_sync()
        self._drop_graphs()
