"""The wide-layer GEMM (csrc/kernels/mlp.hip gemm_lds_kernel, tile 8: 128 x 128 workgroup tile,
LDS-DMA double-buffered 64-deep panels) against a PyTorch fp32 reference of the same op, for every
epilogue the per-layer tower uses, and bitwise against the register-fed tiles it replaces where
their reduction order is the same (one MFMA chain per output over k in order)."""
import pytest
import torch

pytestmark = pytest.mark.gpu
if not torch.cuda.is_available():
    pytest.skip("needs a GPU", allow_module_level=True)

import hipfm  # noqa: E402
from hipfm.ops import kernels as KN  # noqa: E402
from hipfm.ops._lib import EpiArgs  # noqa: E402
from hipfm.utils.rng import keep_threshold  # noqa: E402

DEV = torch.device("cuda", 0)


def _ops(M, N, K, seed=0):
    g = torch.Generator(device=DEV).manual_seed(seed)
    A = (torch.rand(M, K, generator=g, device=DEV) * 2 - 1).bfloat16()
    B = (torch.rand(N, K, generator=g, device=DEV) * 2 - 1).bfloat16()
    return A, B


def _ref(A, B):
    return A.float() @ B.float().t()


@pytest.mark.parametrize("tile,M,N,K,split", [(8, 256, 128, 64, 1), (8, 384, 256, 320, 1), (8, 256, 512, 4096, 1),
                                              (8, 512, 256, 2048, 4), (8, 1024, 1024, 1024, 2),
                                              (9, 256, 256, 64, 1), (9, 512, 768, 320, 1), (9, 512, 512, 4096, 1),
                                              (9, 768, 256, 2048, 4), (9, 1024, 1024, 1024, 2),
                                              (10, 512, 768, 320, 1), (10, 768, 256, 2048, 4), (10, 1024, 1024, 1024, 2),
                                              (11, 256, 256, 64, 1), (11, 512, 768, 320, 1), (11, 512, 512, 4096, 1),
                                              (11, 768, 256, 2048, 4), (11, 1024, 1024, 1024, 2),
                                              (12, 256, 256, 128, 1), (12, 512, 768, 320, 1), (12, 512, 512, 4096, 1),
                                              (12, 768, 256, 2048, 4), (12, 1024, 1024, 1024, 2),
                                              (12, 2048, 1024, 8192, 1),
                                              (13, 256, 256, 128, 1), (13, 512, 768, 320, 1), (13, 512, 512, 4096, 1),
                                              (13, 768, 256, 2048, 4), (13, 1024, 1024, 1024, 2),
                                              (13, 2048, 1024, 8192, 1)])
def test_lds_gemm_f32_matches_reference(tile, M, N, K, split):
    A, B = _ops(M, N, K, seed=M + N + K)
    out = torch.full((split, M, N), float("nan"), device=DEV)
    ep = EpiArgs()
    ep.out = out.data_ptr()
    KN.gemm_nt(KN.EPI_F32, tile, A, K, B, K, M, N, K, split, ep)
    torch.cuda.synchronize()
    ref = _ref(A, B)
    got = out.sum(0)
    assert torch.isfinite(got).all()
    assert (got - ref).abs().max().item() <= 1e-4 * max(1.0, ref.abs().max().item()) + 1e-3
    # the register-fed 64x64 tile sums k in the same MFMA order: bitwise equal
    o2 = torch.zeros(split, M, N, device=DEV)
    ep.out = o2.data_ptr()
    KN.gemm_nt(KN.EPI_F32, 0, A, K, B, K, M, N, K, split, ep)
    torch.cuda.synchronize()
    assert torch.equal(out, o2)


@pytest.mark.parametrize("tile", [8, 9, 10, 11, 12, 13])
@pytest.mark.parametrize("epi", ["fwd", "fwd_eval", "dgrad", "relu_f32"])
def test_lds_gemm_epilogues_match_register_tile(tile, epi):
    M, N, K = 512, 256, 640
    A, B = _ops(M, N, K, seed=3)
    big = tile
    bias = torch.randn(N, device=DEV)
    step = torch.tensor([7], dtype=torch.int64, device=DEV)
    hprev = torch.randn(M, N, device=DEV).bfloat16()
    outs = []
    for tile in (big, 0):
        f32 = epi == "relu_f32"
        o = torch.zeros(M, N, device=DEV, dtype=torch.float32 if f32 else torch.bfloat16)
        ot = torch.zeros(N, M, device=DEV, dtype=torch.bfloat16)
        ep = EpiArgs()
        ep.bias, ep.step, ep.out = bias.data_ptr(), step.data_ptr(), o.data_ptr()
        ep.out_t = 0 if f32 else ot.data_ptr()
        ep.seed, ep.layer, ep.keep_thr, ep.drop, ep.scale = 1234, 1, keep_threshold(0.5), 1, 2.0
        kind = {"fwd": KN.EPI_FWD, "fwd_eval": KN.EPI_FWD_EVAL, "dgrad": KN.EPI_DGRAD,
                "relu_f32": KN.EPI_RELU_F32}[epi]
        if epi == "dgrad":
            ep.hprev = hprev.data_ptr()
        KN.gemm_nt(kind, tile, A, K, B, K, M, N, K, 1, ep)
        torch.cuda.synchronize()
        outs.append((o, ot))
    (o8, ot8), (o0, ot0) = outs
    assert torch.equal(o8, o0) and torch.equal(ot8, ot0)
    ref = _ref(A, B)
    if epi in ("fwd_eval", "relu_f32"):
        r = torch.relu(ref + bias)
        assert (o8.float() - r).abs().max().item() <= 2e-2 * r.abs().max().item()
    if not epi == "relu_f32":
        assert torch.equal(ot8.t(), o8)                  # the transposed copy


@pytest.mark.parametrize("epi", ["fwd", "fwd_eval", "dgrad", "dgrad_nomask"])
def test_epi_pass_matches_fused_epilogue(epi):
    """mlp.hip epi_pass_kernel over the fp32 product equals the fused epilogue of the same GEMM
    (register tile: the F32 output is exactly its accumulator), bit for bit, out and out_t."""
    M, N, K = 512, 256, 640
    A, B = _ops(M, N, K, seed=11)
    bias = torch.randn(N, device=DEV)
    step = torch.tensor([5], dtype=torch.int64, device=DEV)
    hprev = torch.randn(M, N, device=DEV).bfloat16()
    kind = {"fwd": KN.EPI_FWD, "fwd_eval": KN.EPI_FWD_EVAL, "dgrad": KN.EPI_DGRAD,
            "dgrad_nomask": KN.EPI_DGRAD}[epi]
    cf = torch.zeros(M, N, device=DEV)
    e0 = EpiArgs()
    e0.out = cf.data_ptr()
    KN.gemm_nt(KN.EPI_F32, 0, A, K, B, K, M, N, K, 1, e0)
    outs = []
    for fused in (True, False):
        o = torch.zeros(M, N, device=DEV, dtype=torch.bfloat16)
        ot = torch.zeros(N, M, device=DEV, dtype=torch.bfloat16)
        ep = EpiArgs()
        ep.bias, ep.step, ep.out, ep.out_t = bias.data_ptr(), step.data_ptr(), o.data_ptr(), ot.data_ptr()
        ep.seed, ep.layer, ep.keep_thr, ep.drop, ep.scale = 99, 2, keep_threshold(0.5), 1, 2.0
        if epi == "dgrad":
            ep.hprev = hprev.data_ptr()
        if fused:
            KN.gemm_nt(kind, 0, A, K, B, K, M, N, K, 1, ep)
        else:
            KN.epi_pass(kind, cf, M, N, ep)
        torch.cuda.synchronize()
        outs.append((o, ot))
    (o1, t1), (o2, t2) = outs
    assert torch.equal(o1, o2) and torch.equal(t1, t2)
    assert torch.equal(t2.t(), o2)
    if epi == "dgrad":
        assert (o2[hprev <= 0] == 0).all() and (o2 != 0).any()


@pytest.mark.parametrize("bn", [False, True])
def test_wide_tower_library_gemm_matches_fused_tiles(monkeypatch, bn):
    """The 4096-wide tower with its forward / dgrad GEMMs as library GEMM + epilogue pass (batch
    norm: the plain fp32 dgrad GEMM) trains like the hand-written ping-pong tiles (fp32
    accumulation order may differ)."""
    import hipfm.models.layers as D
    from hipfm.data.synthetic import make_synth
    from hipfm.models.deepfm import NativeDeepFM
    from hipfm.models.reference import init_params
    synth = make_synth("total:20000", seed=9)
    F, K, layers, keep, B = synth.F, 8, [4096, 4096, 4096], [0.5, 0.5, 0.5], 2048
    params = init_params(synth.feature_size, F, K, layers, bn, seed=4)
    data = [synth.batch(B, step=s, device=DEV, id_dtype=torch.int32) for s in range(2)]
    outs = []
    for lib in (True, False):
        monkeypatch.setattr(D, "_EPI_BLAS", lib)
        monkeypatch.setattr(D, "_DX0_BLAS", lib)
        m = NativeDeepFM(synth.feature_size, F, K, layers, keep, batch_size=B, device=DEV, init=False,
                         batch_norm=bn, learning_rate=1e-3, fused=False)
        m.load_tf_params(params)
        assert (m.cbuf.numel() > 0) == (lib and not bn)
        for ids, vals, lab in data:
            m.train_step(ids, vals, lab)
        torch.cuda.synchronize()
        m.check_errors()
        outs.append((m.p.clone(), m.tv[:synth.feature_size].clone(), m.H[2].clone()))
    (p1, v1, h1), (p0, v0, h0) = outs
    assert (p1 - p0).abs().max().item() <= 1e-4 * p0.abs().max().item()
    assert (v1 - v0).abs().max().item() <= 1e-4 * v0.abs().max().item()


def test_lds_gemm_rejects_bad_shapes():
    A, B = _ops(256, 256, 96)
    ep = EpiArgs()
    out = torch.zeros(256, 256, device=DEV)
    ep.out = out.data_ptr()
    with pytest.raises(RuntimeError):
        KN.gemm_nt(KN.EPI_F32, KN.TILE_LDS, A, 96, B, 96, 256, 256, 96, 1, ep)   # K % 64 != 0


@pytest.mark.parametrize("bn", [False, True])
def test_wide_tower_step_matches_register_tiles(monkeypatch, bn):
    """A per-layer (wide) tower trained with the LDS / ping-pong tiles equals the same model on the
    register-fed tiles to fp32 reassociation (split-K counts differ), batch norm included."""
    import hipfm.models.layers as D      # (the per-layer path's tile choices live there)
    from hipfm.data.synthetic import make_synth
    from hipfm.models.deepfm import NativeDeepFM
    from hipfm.models.reference import init_params
    synth = make_synth("total:20000", seed=5)
    F, K, layers, keep, B = synth.F, 8, [512, 512], [0.5, 0.5], 8192
    params = init_params(synth.feature_size, F, K, layers, bn, seed=2)
    data = [synth.batch(B, step=s, device=DEV, id_dtype=torch.int32) for s in range(2)]
    outs = []
    for lds in (True, False):
        monkeypatch.setattr(D, "_LDS_GEMM", lds)
        m = NativeDeepFM(synth.feature_size, F, K, layers, keep, batch_size=B, device=DEV, init=False,
                         batch_norm=bn, learning_rate=1e-3, fused=False)
        m.load_tf_params(params)
        assert not m.fused                                # the per-layer path
        for ids, vals, lab in data:
            m.train_step(ids, vals, lab)
        torch.cuda.synchronize()
        m.check_errors()
        # the 512 x 512 weight segments take the tiled transposed-shadow pass (optim.hip)
        assert m._shadow_t is not None
        for w16, wt16 in zip(m.W16, m.WT16):
            assert torch.equal(wt16, w16.t())
        outs.append((m.p.clone(), m.tv[:synth.feature_size].clone()))
    (p8, v8), (p0, v0) = outs
    assert (p8 - p0).abs().max().item() <= 1e-4 * p0.abs().max().item()
    assert (v8 - v0).abs().max().item() <= 1e-4 * v0.abs().max().item()


@pytest.mark.parametrize("blas", [False, True])
def test_wide_wgrad_direct_matches_split_slabs(monkeypatch, blas):
    """A 4096 x 4096 layer's weight gradient (256 ping-pong tiles) computed unsplit straight into
    the flat gradient -- by the ping-pong tile or (blas) the library GEMM -- equals the split-K
    slabs summed by finalize, to fp32 reassociation."""
    import hipfm.models.layers as D
    from hipfm.data.synthetic import make_synth
    from hipfm.models.deepfm import NativeDeepFM
    from hipfm.models.reference import init_params
    synth = make_synth("total:20000", seed=7)
    F, K, layers, keep, B = synth.F, 8, [4096, 4096], [1.0, 1.0], 2048
    params = init_params(synth.feature_size, F, K, layers, False, seed=3)
    ids, vals, lab = synth.batch(B, step=0, device=DEV, id_dtype=torch.int32)
    grads = []
    monkeypatch.setattr(D, "_WG_BLAS", blas)
    for direct in (True, False):
        monkeypatch.setattr(D, "_WG_DIRECT", direct)
        m = NativeDeepFM(synth.feature_size, F, K, layers, keep, batch_size=B, device=DEV, init=False,
                         batch_norm=False, learning_rate=1e-3, fused=False)
        m.load_tf_params(params)
        assert m.wg_direct == [False, direct]
        m.train_step(ids, vals, lab)
        torch.cuda.synchronize()
        m.check_errors()
        grads.append((m.g.clone(), m.p.clone()))
    (gd, pd), (gs, ps) = grads
    assert (gd - gs).abs().max().item() <= 1e-5 * gs.abs().max().item()
    assert (pd - ps).abs().max().item() <= 1e-5 * ps.abs().max().item()


@pytest.mark.parametrize("L,M,nvalid,train,dh", [(4096, 1024, 1000, True, False), (512, 200, 200, True, False),
                                                 (768, 256, 256, True, True), (1024, 128, 128, False, False),
                                                 (320, 192, 190, True, False)])
def test_wide_head_matches_fp32_reference(L, M, nvalid, train, dh):
    """hfm_head for a last layer > 256 units (head_wide_dot / head_wide_bwd at L % 256 == 0, the
    one-launch head_wide_kernel otherwise) against a plain fp32 PyTorch head: probabilities, loss,
    dlogit, dZ = [h > 0] dlogit w / keep (bf16) and its transpose, or the batch-norm dh, and the
    per-64-row partial sums (deep_out weight gradient, dlogit and loss sums)."""
    from hipfm.ops._lib import HeadArgs
    g = torch.Generator(device=DEV).manual_seed(L + M)
    h = torch.relu(torch.randn(M, L, generator=g, device=DEV) - 0.3).bfloat16()
    w = torch.randn(L, generator=g, device=DEV) * 0.05
    b = torch.tensor([0.1], device=DEV)
    yfm = torch.randn(M, generator=g, device=DEV) * 0.3
    lab = (torch.rand(M, generator=g, device=DEV) < 0.4).float()
    nb = (M + 63) // 64
    prob, logit, dlog = (torch.full((M,), -9.0, device=DEV) for _ in range(3))
    dz = torch.zeros(M, L, device=DEV).bfloat16()
    dzt = torch.zeros(L, M, device=DEV).bfloat16()
    dhb = torch.zeros(M, L, device=DEV) if dh else None
    part = torch.full((nb, L + 2), -9.0, device=DEV)
    a = HeadArgs()
    a.h, a.w_out, a.b_out, a.y_fm, a.labels = h.data_ptr(), w.data_ptr(), b.data_ptr(), yfm.data_ptr(), lab.data_ptr()
    a.M, a.L, a.nvalid, a.square_loss, a.train = M, L, nvalid, 0, int(train)
    a.gscale, a.scale_l = 1.0 / nvalid, 2.0
    a.prob, a.logit, a.dlogit, a.dz, a.dz_t, a.partial = (prob.data_ptr(), logit.data_ptr(), dlog.data_ptr(),
                                                          dz.data_ptr(), dzt.data_ptr(), part.data_ptr())
    a.dh = dhb.data_ptr() if dh else 0
    KN.head(a)
    torch.cuda.synchronize()
    hf = h.float()
    y = yfm + hf @ w + b
    p = torch.sigmoid(y)
    valid = torch.arange(M, device=DEV) < nvalid
    dl = torch.where(valid, (p - lab) / nvalid, torch.zeros_like(p))
    loss = torch.where(valid, torch.relu(y) - y * lab + torch.log1p(torch.exp(-y.abs())), torch.zeros_like(p))
    assert torch.allclose(prob, p, atol=1e-5) and torch.allclose(logit, y, atol=1e-4)
    pad = nb * 64 - M
    blk = lambda t: torch.nn.functional.pad(t, (0, pad)).view(nb, 64)   # noqa: E731
    assert torch.allclose(part[:, L + 1], blk(loss).sum(1), rtol=1e-4, atol=1e-5)
    if not train:
        assert (part[:, :L] == 0).all()
        return
    assert torch.allclose(dlog, dl, atol=1e-7)
    assert torch.allclose(part[:, L], blk(dl).sum(1), rtol=1e-4, atol=1e-7)
    ref_part = torch.nn.functional.pad(dl[:, None] * hf, (0, 0, 0, pad)).view(nb, 64, L).sum(1)
    assert torch.allclose(part[:, :L], ref_part, rtol=1e-3, atol=1e-6)
    if dh:
        assert torch.allclose(dhb, dlog[:, None] * w[None, :], rtol=1e-6, atol=1e-9)
    else:
        # dZ from the kernel's own dlogit: bf16 rounding of the same fp32 product
        ref = torch.where(hf > 0, dlog[:, None] * w[None, :] * 2.0, torch.zeros_like(hf)).bfloat16()
        assert torch.equal(dz, ref) and torch.equal(dzt, ref.t().contiguous())


def test_wide_first_layer_padded_input_matches_golden():
    """A per-layer tower with a wide first layer pads its input to 128 columns (K0p 320 -> 384
    at F = 39, K = 8: the layer-0 weight-gradient / dX0 GEMMs take the LDS tile); the trained
    dense parameters, exported in TF shapes, still match the fp32 golden model and the padding
    columns of W0 stay exactly zero."""
    from hipfm.data.synthetic import make_synth
    from hipfm.models.deepfm import NativeDeepFM
    from hipfm.models.reference import GoldenDeepFM, init_params
    synth = make_synth("total:4000", seed=21)
    F, K, layers, keep = synth.F, 8, [1024, 64], [1.0, 1.0]
    V = synth.feature_size
    params = init_params(V, F, K, layers, False, seed=3)
    kw = dict(adam_epsilon=1e-2)
    nat = NativeDeepFM(V, F, K, layers, keep, batch_size=512, device=DEV, init=False, learning_rate=1e-3,
                       fused=False, **kw)
    assert not nat.fused and nat.K0p == 384 and nat.d0 == F * K
    nat.load_tf_params(params)
    gold = GoldenDeepFM(V, F, K, layers, keep, params=params, learning_rate=1e-3, **kw)
    for s in range(2):
        ids, vals, labels = synth.batch(512, step=s)
        gold.train_step(ids, vals, labels)
        nat.train_step(ids.to(DEV, torch.int32), vals.to(DEV), labels.to(DEV))
    torch.cuda.synchronize()
    nat.check_errors()
    seg = nat.dense_segs["Deep-part/mlp0/weights"]
    w0 = nat.p[seg.off:seg.off + nat.Np[0] * nat.K0p].view(nat.Np[0], nat.K0p)
    assert not w0[:, nat.d0:].any()
    dense = nat.dense_tf_params()
    for k, v in dense.items():
        g = gold.params[k]
        assert (v - g).abs().max().item() <= 2e-3 * max(1.0, g.abs().max().item()), k
