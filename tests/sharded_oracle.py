"""Test oracle: host-synchronous row-sharded embedding routing over torch.distributed (the
algorithm of the native fixed-capacity exchange, parallel/sharded.py, in plain torch code with
variable all-to-all splits).  Only the multi-process CPU tests use it (gloo); the package runs the
native engine.  SURVEY P4 / §2.6 "row-sharded mode", BASELINE config #4.

The reference spreads variables over Parameter-Server tasks and documents
``fixed_size_partitioner`` for big embeddings (DOC p.32); every step the workers pull rows over
gRPC and push gradients for asynchronous updates (PS:414-442).  The MI355X replacement keeps
the table in HBM, row-sharded over the ranks of one process group, synchronously:

  owner(id) = id % N          (mod sharding spreads Zipf-hot ids over all ranks)
  row(id)   = id // N         (local row on the owner)

  forward : unique ids of the local batch -> grouped by owner -> all-to-all (counts, then ids)
            -> owners gather their rows -> all-to-all back -> rows in unique-id order
  backward: per-unique-id gradient rows -> all-to-all to the owners -> owner sums duplicates
            (ids requested by several ranks) -> row update on the owner only

``Router`` is device-agnostic torch code; ``make_sharded_golden`` wraps the golden model with it.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Callable, List, Optional, Tuple

import torch
import torch.distributed as dist


def owner_of(ids: torch.Tensor, world: int) -> torch.Tensor:
    return ids % world


def local_row(ids: torch.Tensor, world: int) -> torch.Tensor:
    return ids // world


def local_rows_count(V: int, world: int) -> int:
    return (V + world - 1) // world


@dataclass
class RoutePlan:
    order: torch.Tensor        # permutation: unique index -> position in the send buffer
    send_counts: List[int]     # ids sent to each owner
    recv_counts: List[int]     # ids received from each requester
    recv_ids: torch.Tensor     # global ids this rank owns and must serve, grouped by requester


class Router:
    def __init__(self, world: int, rank: int, group=None):
        self.world, self.rank, self.group = world, rank, group
        self.bytes_sent = 0

    def _a2a(self, out: torch.Tensor, inp: torch.Tensor, out_splits, in_splits):
        self.bytes_sent += inp.numel() * inp.element_size()
        dist.all_to_all_single(out, inp, output_split_sizes=out_splits,
                               input_split_sizes=in_splits, group=self.group)

    def route(self, uniq: torch.Tensor) -> RoutePlan:
        """``uniq``: this rank's unique ids (any order)."""
        N = self.world
        u = uniq.long()
        owner = owner_of(u, N)
        order = torch.argsort(owner, stable=True)
        send_ids = u[order].to(torch.int32)
        sc_t = torch.bincount(owner, minlength=N).to(torch.int64)
        rc_t = torch.empty_like(sc_t)
        dist.all_to_all_single(rc_t, sc_t, group=self.group)
        sc, rc = sc_t.tolist(), rc_t.tolist()
        recv_ids = torch.empty(sum(rc), dtype=torch.int32, device=uniq.device)
        self._a2a(recv_ids, send_ids, rc, sc)
        return RoutePlan(order, sc, rc, recv_ids)

    def fetch_rows(self, plan: RoutePlan, serve: Callable[[torch.Tensor], torch.Tensor]) -> torch.Tensor:
        """Owners serve ``serve(local_rows) -> [n, C]``; returns rows in the caller's unique
        order ([U, C])."""
        rows = serve(local_row(plan.recv_ids.long(), self.world))
        U = plan.order.numel()
        got = torch.empty((U,) + tuple(rows.shape[1:]), dtype=rows.dtype, device=rows.device)
        self._a2a(got, rows.contiguous(), plan.send_counts, plan.recv_counts)
        out = torch.empty_like(got)
        out[plan.order] = got
        return out

    def push_grads(self, plan: RoutePlan, grads_u: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
        """Send per-unique-id gradient rows to their owners; returns (global ids, rows) received
        by this rank (ids may repeat: one row per requesting rank)."""
        send = grads_u[plan.order].contiguous()
        recv = torch.empty((plan.recv_ids.numel(),) + tuple(grads_u.shape[1:]), dtype=grads_u.dtype,
                           device=grads_u.device)
        self._a2a(recv, send, plan.recv_counts, plan.send_counts)
        return plan.recv_ids, recv


def reduce_rows_torch(ids: torch.Tensor, rows: torch.Tensor, world: int, R: int
                      ) -> Tuple[torch.Tensor, torch.Tensor]:
    """Owner-side dedup (CPU reference of the HIP sort + reduce): unique local rows and their
    summed gradients, in ascending id order (deterministic)."""
    u, inv = torch.unique(ids.long(), return_inverse=True)
    acc = torch.zeros((u.numel(),) + tuple(rows.shape[1:]), dtype=rows.dtype, device=rows.device)
    acc.index_add_(0, inv, rows)
    return local_row(u, world), acc


# ---------------------------------------------------------------------------------------------
# CPU / gloo reference of the row-sharded data-parallel step (tests + config #1 multi-process).
def make_sharded_golden(*args, world: int, rank: int, group=None, **kw):
    """A GoldenDeepFM whose fm_w / fm_v (and their optimizer slots) hold only this rank's rows
    (ids r, r+N, ...), trained with the Router exchange — the algorithm of the MI355X sharded
    path in plain PyTorch (distributed logic tested without a cluster)."""
    from hipfm.models.reference import GoldenDeepFM

    class ShardedGoldenDeepFM(GoldenDeepFM):
        def __init__(self):
            super().__init__(*args, world_size=world, **kw)
            self.N, self.rank = world, rank
            self.router = Router(world, rank, group)
            R = local_rows_count(self.V, world)
            self.R = R

            def local(t):
                out = torch.zeros((R,) + tuple(t.shape[1:]), dtype=t.dtype)
                rows = t[rank::world]
                out[: rows.shape[0]] = rows
                return out
            for k in ("fm_w", "fm_v"):
                self.params[k] = local(self.params[k])
            for k in list(self.slots):
                if k.startswith("fm_w/") or k.startswith("fm_v/"):
                    self.slots[k] = local(self.slots[k])

        def train_step(self, ids, vals, labels, grad_sync=None) -> float:
            K, B = self.K, ids.shape[0]
            uniq, inv = torch.unique(ids.reshape(-1).long(), return_inverse=True)
            plan = self.router.route(uniq)
            P = self.params
            rows = self.router.fetch_rows(
                plan, lambda loc: torch.cat([P["fm_v"][loc], P["fm_w"][loc].unsqueeze(1)], 1))
            v_u = rows[:, :K].clone().requires_grad_(True)
            w_u = rows[:, K].clone().requires_grad_(True)
            dense = [k for k in self.trainable() if k not in ("fm_w", "fm_v")]
            Pc = {k: (v.detach().requires_grad_(True) if k in dense else v) for k, v in P.items()}
            Pc["fm_v"], Pc["fm_w"] = v_u, w_u
            y = self.forward(inv.reshape(B, -1), vals, train=True, params=Pc)
            import torch.nn.functional as Fn
            lab = labels.reshape(-1).float()
            data = (((torch.sigmoid(y) - lab) ** 2).mean() if self.loss_type == "square_loss"
                    else Fn.binary_cross_entropy_with_logits(y, lab))
            gs = torch.autograd.grad(data, [Pc[k] for k in dense] + [v_u, w_u])
            grads = dict(zip(dense, gs[: len(dense)]))
            for k in dense:                       # Horovod average of the dense gradients
                t = grads[k].contiguous().clone()
                dist.all_reduce(t, group=group)
                grads[k] = t / self.N
            g_u = torch.cat([gs[-2], gs[-1].unsqueeze(1)], 1) / self.N
            rid, rrows = self.router.push_grads(plan, g_u)
            loc, summed = reduce_rows_torch(rid, rrows, self.N, self.R)
            gv = self.l2 * P["fm_v"]              # whole-table l2 term, applied by the owner
            gw = self.l2 * P["fm_w"]
            gv = gv.index_add(0, loc, summed[:, :K])
            gw = gw.index_add(0, loc, summed[:, K])
            grads["fm_v"], grads["fm_w"] = gv, gw
            with torch.no_grad():
                self._apply(grads, loc)
            self.global_step += 1
            self.last_loss = float(data)
            return float(data)

        def full_table(self, name: str) -> torch.Tensor:
            """Gather the full [V, ...] table (tests / export)."""
            t = self.params[name].contiguous()
            parts = [torch.empty_like(t) for _ in range(self.N)]
            dist.all_gather(parts, t, group=group)
            full = torch.zeros((self.R * self.N,) + tuple(t.shape[1:]), dtype=t.dtype)
            for r in range(self.N):
                full[r::self.N] = parts[r]
            return full[: self.V]

    return ShardedGoldenDeepFM()
