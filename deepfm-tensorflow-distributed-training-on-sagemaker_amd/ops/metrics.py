"""Evaluation metrics (reference C18: ``tf.metrics.auc(labels, pred)``, HVD:241-249).

* ``auc_from_hist``  — TF1 ``tf.metrics.auc`` (num_thresholds=200, curve=ROC,
  summation_method=trapezoidal) computed from the per-bucket histogram the HIP kernel
  ``hfm_auc_hist`` (csrc/kernels/metrics.hip) accumulates.  Bucket b of a prediction p is the
  number of thresholds t_i < p, with TF's float32 thresholds.
* ``hist_torch``     — the same histogram in PyTorch (CPU path and kernel oracle).
* ``exact_auc``      — rank-based (Mann-Whitney) AUC for reporting next to TF's estimate.
"""
from __future__ import annotations

import numpy as np
import torch

NUM_THRESHOLDS = 200
_KEPS = 1e-7


def tf_thresholds() -> torch.Tensor:
    t = [(i + 1) * 1.0 / (NUM_THRESHOLDS - 1) for i in range(NUM_THRESHOLDS - 2)]
    t = [0.0 - _KEPS] + t + [1.0 + _KEPS]
    return torch.tensor(t, dtype=torch.float32)


def hist_torch(pred: torch.Tensor, labels: torch.Tensor) -> torch.Tensor:
    """[2, 201] int64 histogram: row 0 negatives, row 1 positives."""
    thr = tf_thresholds().to(pred.device)
    p = pred.reshape(-1).float()
    b = torch.searchsorted(thr, p, right=False)  # count of thresholds strictly < p
    pos = (labels.reshape(-1) > 0.5).long()
    h = torch.zeros(2, NUM_THRESHOLDS + 1, dtype=torch.int64, device=pred.device)
    h.index_put_((pos, b), torch.ones_like(b), accumulate=True)
    return h


def confusion_from_hist(hist: torch.Tensor):
    h = hist.to(torch.float64).cpu().numpy()
    neg, pos = h[0], h[1]
    # TP[i] = #pos with bucket > i  (pred > t_i)
    tp = np.array([pos[i + 1:].sum() for i in range(NUM_THRESHOLDS)])
    fp = np.array([neg[i + 1:].sum() for i in range(NUM_THRESHOLDS)])
    fn = pos.sum() - tp
    tn = neg.sum() - fp
    return tp, fn, tn, fp


def auc_from_hist(hist: torch.Tensor) -> float:
    tp, fn, tn, fp = confusion_from_hist(hist)
    eps = 1.0e-6
    tp, fn, tn, fp = (x.astype(np.float32) for x in (tp, fn, tn, fp))
    rec = (tp + eps) / (tp + fn + eps)
    fpr = fp / (fp + tn + eps)
    x, y = fpr, rec
    return float(np.sum((x[:-1] - x[1:]) * (y[:-1] + y[1:]) / 2.0))


def exact_auc(pred: torch.Tensor, labels: torch.Tensor) -> float:
    p = pred.reshape(-1).double().cpu().numpy()
    y = (labels.reshape(-1).cpu().numpy() > 0.5)
    npos, nneg = int(y.sum()), int((~y).sum())
    if npos == 0 or nneg == 0:
        return float("nan")
    order = np.argsort(p, kind="mergesort")
    ranks = np.empty(len(p), dtype=np.float64)
    sp = p[order]
    i = 0
    while i < len(sp):          # average ranks over ties
        j = i
        while j + 1 < len(sp) and sp[j + 1] == sp[i]:
            j += 1
        ranks[order[i: j + 1]] = (i + j) / 2.0 + 1.0
        i = j + 1
    return float((ranks[y].sum() - npos * (npos + 1) / 2.0) / (npos * nneg))


def logloss(pred: torch.Tensor, labels: torch.Tensor) -> float:
    p = pred.reshape(-1).double().clamp(1e-7, 1 - 1e-7)
    y = labels.reshape(-1).double()
    return float(-(y * torch.log(p) + (1 - y) * torch.log(1 - p)).mean())
