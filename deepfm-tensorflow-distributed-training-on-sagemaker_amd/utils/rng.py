"""Counter-based RNG shared by the HIP kernels and the PyTorch golden model.

Dropout masks are *stateless*: keep(seed, step, layer, flat_index) is a pure hash, so the
backward pass never stores a mask and the golden model can reproduce the native kernels'
masks bit-for-bit (csrc/kernels/common.h implements the identical ``fmix32`` chain).
The reference uses ``tf.nn.dropout`` (``PS:218``), a stateful Philox stream; exact mask
parity with TF is impossible without TF and is not a goal — keep-probability semantics are.
"""
from __future__ import annotations

import torch

M32 = 0xFFFFFFFF


def fmix32_int(h: int) -> int:
    h &= M32
    h ^= h >> 16
    h = (h * 0x85EBCA6B) & M32
    h ^= h >> 13
    h = (h * 0xC2B2AE35) & M32
    h ^= h >> 16
    return h


def fmix32_t(h: torch.Tensor) -> torch.Tensor:
    """fmix32 on an int64 tensor holding uint32 values."""
    h = h & M32
    h = h ^ (h >> 16)
    h = (h * 0x85EBCA6B) & M32
    h = h ^ (h >> 13)
    h = (h * 0xC2B2AE35) & M32
    h = h ^ (h >> 16)
    return h


def dropout_salt(seed: int, step: int, layer: int) -> int:
    return fmix32_int((seed & M32) ^ fmix32_int((step + layer * 0x632BE5AB) & M32))


def keep_threshold(keep: float) -> int:
    """uint32 threshold: element kept iff hash < threshold (keep >= 1 -> always)."""
    if keep >= 1.0:
        return 1 << 32
    return min(int(keep * 4294967296.0), M32)


def dropout_keep_mask(seed: int, step: int, layer: int, rows: int, cols: int, ld: int,
                      keep: float, device=None) -> torch.Tensor:
    """Bool mask [rows, cols]; flat index = row * ld + col (ld = padded row stride)."""
    thr = keep_threshold(keep)
    if thr > M32:
        return torch.ones(rows, cols, dtype=torch.bool, device=device)
    salt = dropout_salt(seed, step, layer)
    r = torch.arange(rows, dtype=torch.int64, device=device).view(-1, 1)
    c = torch.arange(cols, dtype=torch.int64, device=device).view(1, -1)
    x = (r * ld + c) & M32
    h = fmix32_t(((x * 0x9E3779B1) & M32) ^ salt)
    return h < thr
