"""Golden DeepFM: a pure-PyTorch transcription of the reference's TF1 semantics.

This is (a) the numerical oracle for every native HIP kernel and (b) the CPU execution path
(config #1: plumbing on a 1k-row dataset without a GPU).  It follows the reference model_fn
(``2-hvd-gpu/DeepFM-hvd-tfrecord-vectorized-map.py:141-287``, identical in
``1-ps-cpu/...:149-292``):

* FM first order  ``y_w = sum_f w[id]*x``                       (HVD:169-171)
* FM second order ``y_v = 1/2 sum_k ((sum_f E)^2 - sum_f E^2)``  (HVD:173-179)
* deep tower      ``fully_connected`` (ReLU) -> [BN] -> dropout(keep_prob), TRAIN only (HVD:195-218)
* output          ``y = b + y_w + y_v + y_d``, ``p = sigmoid(y)``  (HVD:220-224)
* loss            ``mean(sigmoid_CE) + l2*(l2_loss(fm_w) + l2_loss(fm_v))``; l2_loss = sum(x^2)/2
                  over the WHOLE tables; the MLP l2_regularizer is never added (quirk Q2) (HVD:236-238)
* optimizers      TF1 Adam / Adagrad / Momentum / FTRL (+ GD, quirk Q4) (HVD:252-263); the
                  embedding gradient (IndexedSlices of the gather + dense l2 term) makes TF1's
                  sparse apply touch every row every step ("tf1_dense"); "lazy" updates only
                  the rows present in the batch (for 800M-row tables, quirk Q8).
* initializers    fm_bias 0, fm_w/fm_v glorot_normal (truncated normal, fan_avg), MLP weights
                  xavier uniform, biases 0 (HVD:158-160 + tf.contrib.layers defaults).

Parameter names and layouts are the TF1 checkpoint names: MLP weights are
``[in, out]`` (``x @ W``).
"""
from __future__ import annotations

import math
from collections import OrderedDict
from typing import Dict, List, Optional

import torch
import torch.nn.functional as Fn

from ..utils.rng import dropout_keep_mask

TRUNC_NORMAL_STDDEV_CORRECTION = 0.87962566103423978  # TF VarianceScaling truncated_normal


def pad32(n: int) -> int:
    return (n + 31) // 32 * 32


def glorot_normal_(t: torch.Tensor, gen: Optional[torch.Generator] = None) -> torch.Tensor:
    """TF ``glorot_normal_initializer``: truncated normal (+-2 std), std = sqrt(1/fan_avg)/0.8796."""
    shape = t.shape
    if len(shape) == 0:
        fan_in = fan_out = 1
    elif len(shape) == 1:
        fan_in = fan_out = shape[0]
    else:
        fan_in, fan_out = shape[0], shape[1]
    n = max(1.0, (fan_in + fan_out) / 2.0)
    std = math.sqrt(1.0 / n) / TRUNC_NORMAL_STDDEV_CORRECTION
    with torch.no_grad():
        torch.nn.init.trunc_normal_(t, mean=0.0, std=std, a=-2 * std, b=2 * std, generator=gen)
    return t


def xavier_uniform_(t: torch.Tensor, gen: Optional[torch.Generator] = None) -> torch.Tensor:
    """``tf.contrib.layers.xavier_initializer()`` (uniform, fan_avg) for a [in, out] weight."""
    fan_in, fan_out = t.shape[0], t.shape[1]
    limit = math.sqrt(6.0 / (fan_in + fan_out))
    with torch.no_grad():
        t.uniform_(-limit, limit, generator=gen)
    return t


def _bf16_round(t: torch.Tensor) -> torch.Tensor:
    """Round to bf16 and back (autograd: the gradient is rounded to bf16 on the way back)."""
    return t.to(torch.bfloat16).to(torch.float32)


def param_shapes(V: int, F: int, K: int, layers: List[int], batch_norm: bool) -> "OrderedDict[str, tuple]":
    shapes = OrderedDict()
    shapes["fm_bias"] = (1,)
    shapes["fm_w"] = (V,)
    shapes["fm_v"] = (V, K)
    d_in = F * K
    for i, L in enumerate(layers):
        shapes[f"Deep-part/mlp{i}/weights"] = (d_in, L)
        shapes[f"Deep-part/mlp{i}/biases"] = (L,)
        if batch_norm:
            for n in ("beta", "gamma", "moving_mean", "moving_variance"):
                shapes[f"Deep-part/bn_{i}/{n}"] = (L,)
        d_in = L
    shapes["Deep-part/deep_out/weights"] = (d_in, 1)
    shapes["Deep-part/deep_out/biases"] = (1,)
    return shapes


def glorot_std(shape) -> float:
    if len(shape) == 1:
        fan_in = fan_out = shape[0]
    else:
        fan_in, fan_out = shape[0], shape[1]
    return math.sqrt(1.0 / max(1.0, (fan_in + fan_out) / 2.0)) / TRUNC_NORMAL_STDDEV_CORRECTION


def init_params(V: int, F: int, K: int, layers: List[int], batch_norm: bool, seed: int,
                device="cpu", tables: bool = True) -> "OrderedDict[str, torch.Tensor]":
    """Deterministic TF-equivalent initialization (distributions, not TF's exact bit stream).

    ``tables=False`` skips fm_w/fm_v (callers initialize huge tables in place, sharded)."""
    gen = torch.Generator(device=device)
    gen.manual_seed(seed)
    out = OrderedDict()
    for name, shape in param_shapes(V, F, K, layers, batch_norm).items():
        if not tables and name in ("fm_w", "fm_v"):
            continue
        t = torch.zeros(shape, dtype=torch.float32, device=device)
        if name in ("fm_w", "fm_v"):
            glorot_normal_(t, gen)
        elif name.endswith("/weights"):
            xavier_uniform_(t, gen)
        elif name.endswith("/gamma") or name.endswith("/moving_variance"):
            t.fill_(1.0)
        out[name] = t
    return out


SPARSE_VARS = ("fm_w", "fm_v")


class GoldenDeepFM:
    """Reference-semantics DeepFM with explicit TF1 optimizer state.

    ``world_size`` reproduces Horovod's LR scaling (``lr * hvd.size()``, HVD:149): training the
    golden model on the concatenated global batch with ``world_size=N`` is mathematically the
    same as N synchronous ranks with gradient averaging.
    """

    def __init__(self, feature_size: int, field_size: int, embedding_size: int = 32,
                 deep_layers=(256, 128, 64), keep_probs=(0.5, 0.5, 0.5), batch_norm: bool = False,
                 batch_norm_decay: float = 0.9, l2_reg: float = 1e-4, learning_rate: float = 5e-4,
                 optimizer: str = "Adam", loss_type: str = "log_loss",
                 sparse_update: str = "tf1_dense", seed: int = 1234, world_size: int = 1,
                 device="cpu", params: Optional[Dict[str, torch.Tensor]] = None,
                 adam_epsilon: float = 1e-8, adagrad_init: float = 1e-8, mlp_bf16: bool = False):
        # mlp_bf16: round the deep-tower GEMM operands to bf16 like the native MFMA path does
        # (tests use it to separate kernel bugs from bf16 rounding amplified by batch norm)
        self.mlp_bf16 = bool(mlp_bf16)
        self.adam_eps = float(adam_epsilon)      # TF AdamOptimizer epsilon (HVD:253)
        self.adagrad_init = float(adagrad_init)  # initial_accumulator_value (HVD:255)
        self.V, self.F, self.K = int(feature_size), int(field_size), int(embedding_size)
        self.layers = [int(x) for x in deep_layers]
        self.keep = [float(x) for x in keep_probs]
        self.batch_norm = bool(batch_norm)
        self.bn_decay = float(batch_norm_decay)
        self.l2 = float(l2_reg)
        self.lr = float(learning_rate) * world_size
        self.optimizer = optimizer
        self.loss_type = loss_type
        self.sparse_update = sparse_update
        self.seed = int(seed)
        self.device = torch.device(device)
        self.global_step = 0
        if params is None:
            params = init_params(self.V, self.F, self.K, self.layers, self.batch_norm, self.seed,
                                 device=self.device)
        self.params: "OrderedDict[str, torch.Tensor]" = OrderedDict(
            (k, v.detach().clone().to(self.device, torch.float32)) for k, v in params.items())
        self.slots: Dict[str, torch.Tensor] = {}
        self._init_slots()

    # ------------------------------------------------------------------ optimizer state
    def trainable(self) -> List[str]:
        return [k for k in self.params if "moving_" not in k]

    def _init_slots(self):
        for name in self.trainable():
            p = self.params[name]
            if self.optimizer == "Adam":
                self.slots[f"{name}/Adam"] = torch.zeros_like(p)
                self.slots[f"{name}/Adam_1"] = torch.zeros_like(p)
            elif self.optimizer == "Adagrad":
                self.slots[f"{name}/Adagrad"] = torch.full_like(p, self.adagrad_init)  # HVD:255
            elif self.optimizer == "Momentum":
                self.slots[f"{name}/Momentum"] = torch.zeros_like(p)
            elif self.optimizer == "ftrl":
                self.slots[f"{name}/Ftrl"] = torch.full_like(p, 0.1)   # initial_accumulator_value
                self.slots[f"{name}/Ftrl_1"] = torch.zeros_like(p)     # linear
        if self.optimizer == "Adam":
            self.slots["beta1_power"] = torch.tensor(0.9, dtype=torch.float32, device=self.device)
            self.slots["beta2_power"] = torch.tensor(0.999, dtype=torch.float32, device=self.device)

    # ------------------------------------------------------------------ forward
    def forward(self, ids: torch.Tensor, vals: torch.Tensor, train: bool,
                params: Optional[Dict[str, torch.Tensor]] = None, step: Optional[int] = None):
        P = self.params if params is None else params
        step = self.global_step if step is None else step
        ids = ids.reshape(-1, self.F).long()
        x = vals.reshape(-1, self.F).float()
        B = ids.shape[0]
        w = P["fm_w"][ids]                                   # [B,F]
        y_w = (w * x).sum(1)
        E = P["fm_v"][ids] * x.unsqueeze(-1)                 # [B,F,K]
        S = E.sum(1)
        y_v = 0.5 * (S * S - (E * E).sum(1)).sum(1)
        h = E.reshape(B, self.F * self.K)
        for i, L in enumerate(self.layers):
            w = P[f"Deep-part/mlp{i}/weights"]
            if self.mlp_bf16:
                h, w = _bf16_round(h), _bf16_round(w)
            h = torch.relu(h @ w + P[f"Deep-part/mlp{i}/biases"])
            if self.batch_norm:
                h = self._bn(h, i, P, train)
            if train and self.keep[i] < 1.0:
                m = dropout_keep_mask(self.seed, step, i, B, L, pad32(L), self.keep[i], device=h.device)
                h = h * m.to(h.dtype) / self.keep[i]
        y_d = (h @ P["Deep-part/deep_out/weights"] + P["Deep-part/deep_out/biases"]).reshape(-1)
        y = P["fm_bias"] + y_w + y_v + y_d
        return y

    def _bn(self, h, i, P, train):
        eps = 1e-3  # tf.contrib.layers.batch_norm default epsilon
        beta, gamma = P[f"Deep-part/bn_{i}/beta"], P[f"Deep-part/bn_{i}/gamma"]
        mm, mv = f"Deep-part/bn_{i}/moving_mean", f"Deep-part/bn_{i}/moving_variance"
        if train:
            mean = h.mean(0)
            var = h.var(0, unbiased=False)
            n = h.shape[0]
            with torch.no_grad():  # updates_collections=None: in-place moving-average update
                d = self.bn_decay
                self.params[mm].mul_(d).add_(mean.detach() * (1 - d))
                unb = var.detach() * (n / max(n - 1, 1))  # fused batch norm reports Bessel-corrected var
                self.params[mv].mul_(d).add_(unb * (1 - d))
        else:
            mean, var = P[mm], P[mv]
        return gamma * (h - mean) / torch.sqrt(var + eps) + beta

    def predict(self, ids, vals) -> torch.Tensor:
        with torch.no_grad():
            return torch.sigmoid(self.forward(ids, vals, train=False))

    def loss(self, y, labels, P=None):
        P = self.params if P is None else P
        labels = labels.reshape(-1).float()
        if self.loss_type == "square_loss":
            data = ((torch.sigmoid(y) - labels) ** 2).mean()
        else:
            data = Fn.binary_cross_entropy_with_logits(y, labels)
        reg = self.l2 * (0.5 * (P["fm_w"] ** 2).sum() + 0.5 * (P["fm_v"] ** 2).sum())
        return data + reg, data

    # ------------------------------------------------------------------ train
    def compute_grads(self, ids, vals, labels):
        """(total loss, data loss, {name: dense gradient}) of one training forward."""
        P = OrderedDict((k, (v.detach().requires_grad_(True) if "moving_" not in k else v))
                        for k, v in self.params.items())
        y = self.forward(ids, vals, train=True, params=P)
        total, data = self.loss(y, labels, P)
        names = self.trainable()
        grads = torch.autograd.grad(total, [P[n] for n in names])
        return total.detach(), data.detach(), dict(zip(names, grads))

    def train_step(self, ids, vals, labels, grad_sync=None) -> float:
        """One step.  ``grad_sync(grads, touched) -> (grads, touched)`` lets a data-parallel
        caller average gradients across ranks (Horovod DistributedOptimizer semantics) and
        union the touched rows before the identical update on every rank."""
        total, data, grads = self.compute_grads(ids, vals, labels)
        touched = torch.unique(ids.reshape(-1).long())
        if grad_sync is not None:
            grads, touched = grad_sync(grads, touched)
        with torch.no_grad():
            self._apply(grads, touched)
        self.global_step += 1
        self.last_loss = float(data)
        return float(total)

    # ------------------------------------------------------------------ state
    def state_dict_local(self) -> "OrderedDict[str, torch.Tensor]":
        """TF-named variables + optimizer slots + global_step (SURVEY §2.7.4 names)."""
        d = OrderedDict((k, v) for k, v in self.params.items())
        d.update((k, v) for k, v in self.slots.items())
        d["global_step"] = torch.tensor(self.global_step, dtype=torch.int64)
        return d

    def load_state_dict_local(self, d: Dict[str, torch.Tensor]):
        with torch.no_grad():
            for k, v in d.items():
                if k == "global_step":
                    self.global_step = int(v)
                elif k in self.params:
                    self.params[k].copy_(v.to(self.params[k]))
                elif k in self.slots:
                    self.slots[k].copy_(v.to(self.slots[k]))

    def tf_variables(self) -> "OrderedDict[str, torch.Tensor]":
        return self.state_dict_local()

    def replicated_state(self) -> List[torch.Tensor]:
        """Tensors broadcast from rank 0 at start (BroadcastGlobalVariablesHook(0), HVD:372)."""
        return list(self.params.values()) + list(self.slots.values())

    def _apply(self, grads: Dict[str, torch.Tensor], touched: torch.Tensor):
        lr = self.lr
        opt = self.optimizer
        if opt == "Adam":
            b1, b2, eps = 0.9, 0.999, self.adam_eps
            b1p, b2p = self.slots["beta1_power"], self.slots["beta2_power"]
            lr_t = lr * torch.sqrt(1 - b2p) / (1 - b1p)
        for name, g in grads.items():
            p = self.params[name]
            rows = None
            if self.sparse_update == "lazy" and name in SPARSE_VARS:
                rows = touched
            sel = (lambda t: t[rows]) if rows is not None else (lambda t: t)

            def put(t, val):
                if rows is not None:
                    t[rows] = val
                else:
                    t.copy_(val)
            gs = sel(g)
            if opt == "Adam":
                m, v = self.slots[f"{name}/Adam"], self.slots[f"{name}/Adam_1"]
                mn = sel(m) * b1 + (1 - b1) * gs
                vn = sel(v) * b2 + (1 - b2) * gs * gs
                put(m, mn)
                put(v, vn)
                put(p, sel(p) - lr_t * mn / (torch.sqrt(vn) + eps))
            elif opt == "Adagrad":
                a = self.slots[f"{name}/Adagrad"]
                an = sel(a) + gs * gs
                put(a, an)
                put(p, sel(p) - lr * gs / torch.sqrt(an))
            elif opt == "Momentum":
                a = self.slots[f"{name}/Momentum"]
                an = sel(a) * 0.95 + gs
                put(a, an)
                put(p, sel(p) - lr * an)
            elif opt == "ftrl":
                acc, lin = self.slots[f"{name}/Ftrl"], self.slots[f"{name}/Ftrl_1"]
                a0 = sel(acc)
                an = a0 + gs * gs
                sigma = (torch.sqrt(an) - torch.sqrt(a0)) / lr
                ln = sel(lin) + gs - sigma * sel(p)
                quad = torch.sqrt(an) / lr
                put(acc, an)
                put(lin, ln)
                put(p, -ln / quad)   # l1 = l2 = 0 (TF FtrlOptimizer defaults)
            elif opt == "GD":
                put(p, sel(p) - lr * gs)
            else:
                raise ValueError(opt)
        if opt == "Adam":
            self.slots["beta1_power"] *= 0.9
            self.slots["beta2_power"] *= 0.999
