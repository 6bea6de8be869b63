"""Synthetic Criteo-shaped data with learnable signal (SURVEY §7.1 tools row, BASELINE configs).

No dataset can be downloaded here, so every benchmark/test runs on synthetic records with the
reference's schema (``label``, ``ids[F]``, ``values[F]``; ``CONV:25-32``):

* F = 39 = 13 integer ("dense") fields + 26 categorical fields, as in Criteo.
* Dense field j uses the fixed feature id ``j`` with a value in [0, 1) (the libsvm convention of
  the reference data, ``PS:74``); categorical field c uses ids in its own vocabulary range with
  value 1.0.
* Categorical ids are Zipf(s~1)-distributed (P(r) ~ 1/(r+1)) and then scrambled by a bijective
  affine map so hot ids are spread across the table, like hashed production features.
* Labels come from a hidden teacher (first-order hashed weights + a pairwise term), so a
  correctly trained model reaches AUC well above 0.5 — this is what the AUC checks measure.

Vocabulary presets:
* ``criteo_1tb``    — per-field cardinalities of the Criteo Terabyte click logs (~882M ids),
                      the BASELINE "Criteo-1TB-shape" config (#4).
* ``criteo_kaggle`` — Kaggle-display-advertising shape scaled to ~1M ids (config #2).
* ``reference``     — the notebooks' feature_size=117581 (``NBPS:85``).
"""
from __future__ import annotations

import math
from typing import List, Optional, Tuple

import torch

from ..utils.rng import M32

N_DENSE = 13

CRITEO_1TB_CAT = [227605432, 39060, 17295, 7424, 20265, 3, 7122, 1543, 63, 130229467, 3067956,
                  405282, 10, 2209, 11938, 155, 4, 976, 14, 292775614, 40790948, 187188510,
                  590152, 12973, 108, 36]
CRITEO_KAGGLE_CAT = [1460, 583, 305000, 220000, 305, 24, 12517, 633, 3, 93145, 5683, 250000,
                     3194, 27, 14992, 180000, 10, 5652, 2173, 4, 200000, 18, 15, 28618, 105, 14257]


def _scale_to(vocab: List[int], total: int) -> List[int]:
    s = sum(vocab)
    out = [max(2, int(round(v * total / s))) for v in vocab]
    out[int(max(range(len(out)), key=lambda i: out[i]))] += total - sum(out)
    return out


def vocab_preset(name: str) -> List[int]:
    """Categorical vocab sizes (26 fields) for a preset."""
    if name == "criteo_1tb":
        return list(CRITEO_1TB_CAT)
    if name == "criteo_kaggle":
        return list(CRITEO_KAGGLE_CAT)
    if name == "reference":
        return _scale_to(CRITEO_KAGGLE_CAT, 117581 - N_DENSE)
    if name.startswith("total:"):
        return _scale_to(CRITEO_KAGGLE_CAT, int(name.split(":")[1]) - N_DENSE)
    raise ValueError(f"unknown vocab preset {name!r}")


class CriteoSynth:
    """Generator of (ids int64/int32 [B,F], vals f32 [B,F], labels f32 [B]) batches."""

    def __init__(self, cat_vocab: List[int], seed: int = 2024, n_dense: int = N_DENSE,
                 teacher_scale: float = 1.2, ctr_bias: float = -1.1):
        self.n_dense = n_dense
        self.cat_vocab = [int(v) for v in cat_vocab]
        self.F = n_dense + len(self.cat_vocab)
        offs = [n_dense]
        for v in self.cat_vocab[:-1]:
            offs.append(offs[-1] + v)
        self.offsets = offs
        self.V = n_dense + sum(self.cat_vocab)
        self.seed = seed
        self.teacher_scale = teacher_scale
        self.ctr_bias = ctr_bias
        # bijective scramble r -> (a*r + c) mod n per field
        self.aff = []
        for j, n in enumerate(self.cat_vocab):
            a = (2654435761 + 7919 * j) % n if n > 2 else 1
            while a == 0 or math.gcd(a, n) != 1:
                a = (a + 1) % n
            c = (40503 * (j + 1)) % n
            self.aff.append((a, c))

    @property
    def feature_size(self) -> int:
        return self.V

    def field_ranges(self) -> List[Tuple[int, int]]:
        """Per-field id ranges [lo, hi): dense field j -> {j}, categorical c -> its vocabulary."""
        dense = [(j, j + 1) for j in range(self.n_dense)]
        return dense + [(o, o + v) for o, v in zip(self.offsets, self.cat_vocab)]

    def _teacher_w(self, ids: torch.Tensor) -> torch.Tensor:
        h = (ids.long() * 0x9E3779B1 + self.seed) & M32
        h = h ^ (h >> 16)
        h = (h * 0x85EBCA6B) & M32
        h = h ^ (h >> 13)
        u = h.double() / 4294967296.0 - 0.5
        return u.float()

    def batch(self, B: int, step: int, device="cpu", id_dtype=torch.int64) -> Tuple[torch.Tensor, ...]:
        g = torch.Generator(device=device)
        g.manual_seed((self.seed * 1000003 + step) & 0x7FFFFFFFFFFFFFFF)
        F, nd = self.F, self.n_dense
        ids = torch.empty(B, F, dtype=torch.int64, device=device)
        vals = torch.empty(B, F, dtype=torch.float32, device=device)
        ids[:, :nd] = torch.arange(nd, device=device)
        vals[:, :nd] = torch.rand(B, nd, generator=g, device=device) ** 2
        u = torch.rand(B, F - nd, generator=g, device=device, dtype=torch.float64)
        n = torch.tensor(self.cat_vocab, dtype=torch.float64, device=device)
        r = torch.floor(torch.exp(u * torch.log1p(n))) - 1.0
        r = torch.minimum(torch.clamp(r, min=0), n - 1).long()
        a = torch.tensor([x[0] for x in self.aff], dtype=torch.int64, device=device)
        c = torch.tensor([x[1] for x in self.aff], dtype=torch.int64, device=device)
        nl = torch.tensor(self.cat_vocab, dtype=torch.int64, device=device)
        # (a*r + c) mod n without int64 overflow: r < 2^28, a < 2^32 -> product < 2^60
        loc = (r * a + c) % nl
        ids[:, nd:] = loc + torch.tensor(self.offsets, dtype=torch.int64, device=device)
        vals[:, nd:] = 1.0
        # teacher: first-order hashed weights + one pairwise interaction
        tw = self._teacher_w(ids) * vals
        logit = self.teacher_scale * 2.0 * tw.sum(1) + 1.5 * tw[:, nd] * tw[:, nd + 1] * 4 + self.ctr_bias
        p = torch.sigmoid(logit)
        labels = (torch.rand(B, generator=g, device=device) < p).float()
        return ids.to(id_dtype), vals, labels


def make_synth(preset: str = "criteo_kaggle", seed: int = 2024) -> CriteoSynth:
    return CriteoSynth(vocab_preset(preset), seed=seed)
