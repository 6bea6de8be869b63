"""Golden-model semantics checked against hand-written formulas, plus flags/AUC."""
import math
import os

import numpy as np
import pytest
import torch

import hipfm
from hipfm.config import parse_flags
from hipfm.models.reference import GoldenDeepFM, glorot_std, init_params
from hipfm.ops.metrics import auc_from_hist, exact_auc, hist_torch
from hipfm.utils.rng import dropout_keep_mask


def test_flags_defaults_and_unknown_tolerated(monkeypatch):
    monkeypatch.setenv("SM_HOSTS", '["algo-1","algo-2"]')
    with pytest.warns(UserWarning):
        c = parse_flags(["--feature_size", "117581", "--field_size", "39", "--perform_shuffle", "0",
                         "--deep_layers", "128,64,32", "--batch_norm", "True"])
    assert c.embedding_size == 32 and c.batch_size == 64 and c.learning_rate == 0.0005
    assert c.layers == [128, 64, 32] and c.keep_probs == [0.5, 0.5, 0.5] and c.batch_norm
    assert c.hosts == ["algo-1", "algo-2"] and c.optimizer == "Adam" and c.task_type == "train"
    monkeypatch.delenv("SM_HOSTS")
    assert parse_flags([]).hosts == ["algo-1"]          # Q7: no SageMaker env needed


def test_forward_matches_formula():
    V, F, K = 50, 4, 3
    g = GoldenDeepFM(V, F, K, [8], [1.0])
    ids = torch.randint(0, V, (5, F))
    x = torch.rand(5, F)
    P = g.params
    w, v = P["fm_w"], P["fm_v"]
    y_w = (w[ids] * x).sum(1)
    y_v = torch.zeros(5)
    for b in range(5):
        for i in range(F):
            for j in range(i + 1, F):       # FM pairwise form == 0.5((sum)^2 - sum of squares)
                y_v[b] += (v[ids[b, i]] * v[ids[b, j]]).sum() * x[b, i] * x[b, j]
    h = torch.relu((v[ids] * x[..., None]).reshape(5, -1) @ P["Deep-part/mlp0/weights"]
                   + P["Deep-part/mlp0/biases"])
    y_d = (h @ P["Deep-part/deep_out/weights"]).reshape(-1) + P["Deep-part/deep_out/biases"]
    y = P["fm_bias"] + y_w + y_v + y_d
    assert torch.allclose(g.forward(ids, x, train=False), y, atol=1e-5)


def test_loss_includes_whole_table_l2_not_mlp():
    g = GoldenDeepFM(100, 3, 4, [8], [1.0], l2_reg=0.1)
    y = torch.zeros(2)
    tot, data = g.loss(y, torch.tensor([0.0, 1.0]))
    reg = 0.1 * 0.5 * ((g.params["fm_w"] ** 2).sum() + (g.params["fm_v"] ** 2).sum())
    assert abs(float(tot - data - reg)) < 1e-6 and abs(float(data) - math.log(2)) < 1e-6


def test_tf1_adam_dense_semantics_touch_every_row():
    g = GoldenDeepFM(100, 3, 4, [8], [1.0], learning_rate=0.01, sparse_update="tf1_dense")
    before = g.params["fm_v"].clone()
    ids = torch.tensor([[1, 2, 3]])
    g.train_step(ids, torch.ones(1, 3), torch.ones(1))
    moved = (g.params["fm_v"] != before).any(1)
    assert moved.all()            # l2 gradient moves untouched rows too (TF1 non-lazy Adam)
    # first Adam step: lr_t = lr*sqrt(1-b2)/(1-b1); |update| ~= lr_t for |g| >> eps
    # (m/sqrt(v) = (1-b1)/sqrt(1-b2) so the step is ~lr, minus eps=1e-8 against the tiny
    # l2-only gradient of an untouched row)
    d = (g.params["fm_v"][50] - before[50]).abs()
    assert torch.all(d <= 0.01 * 1.0001) and torch.all(d >= 0.01 * 0.5)


def test_lazy_touches_only_batch_rows():
    g = GoldenDeepFM(100, 3, 4, [8], [1.0], sparse_update="lazy")
    before = g.params["fm_v"].clone()
    g.train_step(torch.tensor([[1, 2, 3]]), torch.ones(1, 3), torch.ones(1))
    moved = torch.nonzero((g.params["fm_v"] != before).any(1)).reshape(-1).tolist()
    assert moved == [1, 2, 3]


def test_glorot_init_statistics():
    p = init_params(20000, 39, 8, [64], False, seed=1)
    std = glorot_std((20000, 8))
    assert abs(p["fm_v"].std().item() / (std * 0.8796) - 1) < 0.05   # truncation shrinks std
    assert p["fm_v"].abs().max().item() <= 2 * std + 1e-6
    assert p["fm_bias"].item() == 0


def test_dropout_mask_keep_rate_and_determinism():
    m1 = dropout_keep_mask(7, 3, 1, 512, 128, 128, 0.7)
    m2 = dropout_keep_mask(7, 3, 1, 512, 128, 128, 0.7)
    m3 = dropout_keep_mask(7, 4, 1, 512, 128, 128, 0.7)
    assert torch.equal(m1, m2) and not torch.equal(m1, m3)
    assert abs(m1.float().mean().item() - 0.7) < 0.01


def test_tf_auc_estimate_close_to_exact():
    torch.manual_seed(0)
    p = torch.rand(50000)
    y = (torch.rand(50000) < p).float()
    a = auc_from_hist(hist_torch(p, y))
    e = exact_auc(p, y)
    assert abs(a - e) < 2e-3 and abs(e - 5 / 6) < 0.01
