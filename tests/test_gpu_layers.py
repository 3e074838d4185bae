"""GPU parity of norm / attention / element-wise kernels (fwd + bwd) against plain torch fp32 references."""
import math

import pytest
import torch

import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


@pytest.mark.parametrize("B,HW,C,silu", [(2, 256, 320, True), (2, 64, 640, False), (1, 1024, 1280, True),
                                          (2, 4096, 128, True), (1, 100, 2560, False)])
def test_group_norm_fwd_bwd(cuda, B, HW, C, silu):
    from pairwise_sample_optimization_amd import kernels as K
    x = (torch.randn(B, HW, C, device=cuda) * 2 + 0.5).bfloat16()
    gm = (1 + 0.1 * torch.randn(C, device=cuda)).bfloat16()
    bt = (0.1 * torch.randn(C, device=cuda)).bfloat16()
    xr = x.float().permute(0, 2, 1).requires_grad_(True)  # [B,C,HW]
    gmr, btr = gm.float().requires_grad_(True), bt.float().requires_grad_(True)
    ref = F.group_norm(xr, 32, gmr, btr, eps=1e-5)
    if silu:
        ref = F.silu(ref)
    y, st = K.group_norm_fwd(x, gm, bt, 32, 1e-5, silu)
    assert _rel(y.permute(0, 2, 1), ref) < 8e-3
    dy = torch.randn_like(y)
    gx, ggm, gbt = torch.autograd.grad(ref, (xr, gmr, btr), dy.float().permute(0, 2, 1))
    dadd = torch.randn_like(x)
    dg = torch.zeros(C, device=cuda)
    db = torch.zeros(C, device=cuda)
    dx = K.group_norm_bwd(x, dy, st, gm, bt, silu, dadd=dadd, dgamma=dg, dbeta=db)
    assert _rel(dx.permute(0, 2, 1), gx + dadd.float().permute(0, 2, 1)) < 1e-2
    # dgamma / dbeta (the full-UNet weight gradients; split reduction when B * HW / 64 >= 4)
    assert _rel(dg, ggm) < 1e-2 and _rel(db, gbt) < 1e-2
    dg2, db2 = dg.clone(), db.clone()
    K.group_norm_bwd(x, dy, st, gm, bt, silu, dadd=dadd, dgamma=dg2, dbeta=db2, accumulate=True)
    assert _rel(dg2, 2 * ggm) < 1e-2 and _rel(db2, 2 * gbt) < 1e-2


@pytest.mark.parametrize("M,C", [(300, 640), (77, 1280), (1024, 320), (64, 2048)])
def test_layer_norm_fwd_bwd(cuda, M, C):
    from pairwise_sample_optimization_amd import kernels as K
    x = (torch.randn(M, C, device=cuda) + 0.3).bfloat16()
    gm = (1 + 0.1 * torch.randn(C, device=cuda)).bfloat16()
    bt = (0.1 * torch.randn(C, device=cuda)).bfloat16()
    xr = x.float().requires_grad_(True)
    ref = F.layer_norm(xr, (C,), gm.float(), bt.float(), 1e-5)
    y, st = K.layer_norm_fwd(x, gm, bt, 1e-5)
    assert _rel(y, ref) < 8e-3
    dy = torch.randn_like(y)
    (gx,) = torch.autograd.grad(ref, xr, dy.float())
    dx = K.layer_norm_bwd(x, dy, st, gm)
    assert _rel(dx, gx) < 1e-2


def _attn_ref(q, k, v, H):
    B, Sq, C = q.shape
    f = lambda t: t.float().reshape(B, t.shape[1], H, 64).transpose(1, 2)
    o = F.scaled_dot_product_attention(f(q), f(k), f(v))
    return o.transpose(1, 2).reshape(B, Sq, C)


@pytest.mark.parametrize("B,H,Sq,Sk", [(2, 2, 256, 256), (1, 10, 4096, 4096), (2, 5, 300, 77), (1, 4, 128, 1000),
                                        (2, 20, 1024, 1024), (1, 2, 100, 100)])
def test_attention_fwd_bwd(cuda, B, H, Sq, Sk):
    from pairwise_sample_optimization_amd import kernels as K
    C = H * 64
    g = torch.Generator(device="cuda").manual_seed(Sq + Sk)
    # q/k/v as column slices of a fused projection output, like the UNet does
    qkv = torch.randn(B, Sq, 3 * C, device=cuda, generator=g).bfloat16()
    q = qkv[..., :C]
    if Sk == Sq:
        k, v = qkv[..., C:2 * C], qkv[..., 2 * C:]
    else:
        kv = torch.randn(B, Sk, 2 * C, device=cuda, generator=g).bfloat16()
        k, v = kv[..., :C], kv[..., C:]
    o, lse = K.attention_fwd(q, k, v, H)
    qr, kr, vr = (t.float().requires_grad_(True) for t in (q, k, v))
    ref = _attn_ref(qr, kr, vr, H)
    assert _rel(o, ref) < 1e-2
    do = torch.randn(B, Sq, C, device=cuda, generator=g).bfloat16()
    gq, gk, gv = torch.autograd.grad(ref, (qr, kr, vr), do.float())
    dq, dk, dv = K.attention_bwd(q, k, v, o, lse, do, H)
    assert _rel(dq, gq) < 2e-2
    assert _rel(dk, gk) < 2e-2
    assert _rel(dv, gv) < 2e-2


@pytest.mark.parametrize("B,H,Sq,Sk", [(2, 5, 300, 77), (4, 10, 4096, 77), (2, 20, 1024, 77), (1, 3, 64, 96),
                                        (3, 2, 190, 33), (1, 1, 1, 5), (16, 20, 1024, 77)])
def test_attention_bwd_short_kv_fused(cuda, B, H, Sq, Sk):
    """The short-key backward (Sk <= 96: the cross-attention over the 77 text tokens) makes dQ, dK and dV in one pass
    over the query tiles (attn_bwd_x_kernel; -delta formed in the kernel, dQ through an LDS dS^T tile), with and
    without query splits, ragged query tiles, Sk not a multiple of 16 or 32: against fp32 autograd, and bit-reproducible
    run to run."""
    from pairwise_sample_optimization_amd import kernels as K
    C = H * 64
    g = torch.Generator(device="cuda").manual_seed(11 * Sq + Sk)
    q = torch.randn(B, Sq, C, device=cuda, generator=g).bfloat16()
    k = torch.randn(B, Sk, C, device=cuda, generator=g).bfloat16()
    v = torch.randn(B, Sk, C, device=cuda, generator=g).bfloat16()
    do = torch.randn(B, Sq, C, device=cuda, generator=g).bfloat16()
    o, lse = K.attention_fwd(q, k, v, H)
    a = [x.clone() for x in K.attention_bwd(q, k, v, o, lse, do, H)]
    b = K.attention_bwd(q, k, v, o, lse, do, H)
    for x, y in zip(a, b):
        assert torch.equal(x, y)
    hs = min(H, 4)  # fp32 reference on the first heads
    f = lambda t: t.float().view(B, -1, H, 64)[:, :, :hs].transpose(1, 2).detach().requires_grad_(True)
    qf, kf, vf = f(q), f(k), f(v)
    ref = torch.softmax(qf @ kf.transpose(-1, -2) / 8.0, -1) @ vf
    ref.backward(do.float().view(B, -1, H, 64)[:, :, :hs].transpose(1, 2))
    for name, mine, r in zip(("dq", "dk", "dv"), a, (qf.grad, kf.grad, vf.grad)):
        m = mine.float().view(B, -1, H, 64)[:, :, :hs].transpose(1, 2)
        assert ((m - r).norm() / r.norm()).item() < 2e-2, name
        assert torch.isfinite(mine).all(), name


@pytest.mark.parametrize("B,H,Sq,Sk", [(2, 5, 300, 77), (1, 2, 100, 100), (1, 4, 130, 1000)])
def test_attention_partial_tiles_poisoned_tail(cuda, B, H, Sq, Sk):
    """Partial last key / query tiles with NaN in the memory right past the last row of Q, K, V and dO: the staging
    loads of the forward, dQ and dK/dV kernels must never let a row past the end reach the arithmetic (0 * NaN)."""
    from pairwise_sample_optimization_amd import kernels as K
    C = H * 64
    g = torch.Generator(device="cuda").manual_seed(7 * Sq + Sk)

    def poisoned(S):
        buf = torch.full((B * S + 192, C), float("nan"), device=cuda, dtype=torch.bfloat16)
        t = buf[:B * S]
        t.copy_(torch.randn(B * S, C, device=cuda, generator=g).bfloat16())
        return t.view(B, S, C)

    q, k, v, do = poisoned(Sq), poisoned(Sk), poisoned(Sk), poisoned(Sq)
    o, lse = K.attention_fwd(q, k, v, H)
    qr, kr, vr = (t.float().requires_grad_(True) for t in (q, k, v))
    ref = _attn_ref(qr, kr, vr, H)
    assert torch.isfinite(o).all() and _rel(o, ref) < 1e-2
    gq, gk, gv = torch.autograd.grad(ref, (qr, kr, vr), do.float())
    dq, dk, dv = K.attention_bwd(q, k, v, o, lse, do, H)
    for got, want in ((dq, gq), (dk, gk), (dv, gv)):
        assert torch.isfinite(got).all() and _rel(got, want) < 2e-2


@pytest.mark.knobs
@pytest.mark.parametrize("variant", [2, 4])
@pytest.mark.parametrize("B,H,Sq,Sk", [(2, 2, 256, 256), (2, 5, 300, 77), (1, 4, 130, 1000), (3, 20, 1024, 1024)])
def test_attention_fwd_tiles(cuda, variant, B, H, Sq, Sk):
    """Both tile shapes of the forward (128 / 256 queries per workgroup) and of the dK/dV kernel (128 / 256 keys per
    workgroup) on partial query and key tiles."""
    from pairwise_sample_optimization_amd import kernels as K
    C = H * 64
    g = torch.Generator(device="cuda").manual_seed(Sq * 7 + Sk)
    q = torch.randn(B, Sq, C, device=cuda, generator=g).bfloat16()
    k = torch.randn(B, Sk, C, device=cuda, generator=g).bfloat16()
    v = torch.randn(B, Sk, C, device=cuda, generator=g).bfloat16()
    do = torch.randn(B, Sq, C, device=cuda, generator=g).bfloat16()
    K.lib().pso_attention_set_variant(variant * 11)  # same tile choice for the forward and the dK/dV kernel
    try:
        o, lse = K.attention_fwd(q, k, v, H)
        dq, dk, dv = K.attention_bwd(q, k, v, o, lse, do, H)
    finally:
        K.lib().pso_attention_set_variant(0)
    qr, kr, vr = (t.float().requires_grad_(True) for t in (q, k, v))
    ref = _attn_ref(qr, kr, vr, H)
    assert _rel(o, ref) < 1e-2
    f = lambda t: t.float().reshape(B, t.shape[1], H, 64).transpose(1, 2)
    ref_lse = torch.logsumexp(f(q) @ f(k).transpose(-1, -2) * 0.125, dim=-1)
    assert (lse - ref_lse).abs().max().item() < 2e-3
    gq, gk, gv = torch.autograd.grad(ref, (qr, kr, vr), do.float())
    assert _rel(dq, gq) < 2e-2
    assert _rel(dk, gk) < 2e-2
    assert _rel(dv, gv) < 2e-2


@pytest.mark.knobs
@pytest.mark.parametrize("variant", [2, 4, 7, 9])  # 2 / 4: deferred-rescale forward, 32 / 64 rows per wave; 7 / 9: first-round loop
@pytest.mark.parametrize("case", ["ramp", "spike"])
def test_attention_fwd_rescale_paths(cuda, variant, case):
    """The forward's deferred rescale: keys scaled up along the sequence make every row's max creep up tile after
    tile (growth below the threshold: P exceeds 1 and the rescale is skipped), a late spike key makes some rows' max
    jump by far more than the threshold after 60 tiles (the rescale fires with O, l and the max all moving)."""
    from pairwise_sample_optimization_amd import kernels as K
    B, H, Sq, Sk = 1, 2, 512, 4096
    C = H * 64
    g = torch.Generator(device="cuda").manual_seed(11)
    q = torch.randn(B, Sq, C, device=cuda, generator=g)
    k = torch.randn(B, Sk, C, device=cuda, generator=g)
    v = torch.randn(B, Sk, C, device=cuda, generator=g)
    if case == "ramp":
        k = k * torch.linspace(0.5, 3.0, Sk, device=cuda)[None, :, None]
    else:
        k[:, Sk - 70] = 2.0 * q[:, 5]      # query 5 (and its neighbours by chance) meets a key ~20 log2 units up
        k[:, Sk - 3] = -1.5 * q[:, 300]
    q, k, v = q.bfloat16(), k.bfloat16(), v.bfloat16()
    K.lib().pso_attention_set_variant(variant)
    try:
        o, lse = K.attention_fwd(q, k, v, H)
    finally:
        K.lib().pso_attention_set_variant(0)
    ref = _attn_ref(q, k, v, H)
    f = lambda t: t.float().reshape(B, t.shape[1], H, 64).transpose(1, 2)
    ref_lse = torch.logsumexp(f(q) @ f(k).transpose(-1, -2) * 0.125, dim=-1)
    assert _rel(o, ref) < 1e-2
    assert (lse - ref_lse).abs().max().item() < 2e-3 * max(1.0, ref_lse.abs().max().item() / 8)
    # row-wise: the spiked rows are dominated by one key, so their output is that key's value row
    assert (o.float() - ref).abs().max().item() < 0.06


@pytest.mark.knobs
@pytest.mark.parametrize("variant", [0, 32])  # 0: 2-phase 256x256 kernel; 32: the 8-phase kernel where K % 128 == 0
@pytest.mark.parametrize("M,dim", [(8192, 1280), (300, 64), (1000, 640)])
def test_gemm_geglu_fused(cuda, M, dim, variant):
    """GEGLU in the GEMM epilogue (interleaved weight rows) and its backward fused into the dout GEMM, vs torch fp32."""
    from pairwise_sample_optimization_amd import kernels as K
    K.gemm_set_variant(variant)
    try:
        _geglu_case(cuda, M, dim)
    finally:
        K.gemm_set_variant(0)


def _geglu_case(cuda, M, dim):
    from pairwise_sample_optimization_amd import kernels as K
    Fd = 4 * dim
    g = torch.Generator(device="cuda").manual_seed(M + dim)
    x = torch.randn(M, dim, device=cuda, generator=g).bfloat16()
    w = (torch.randn(2 * Fd, dim, device=cuda, generator=g) / dim ** 0.5).bfloat16()
    b = (0.1 * torch.randn(2 * Fd, device=cuda, generator=g)).bfloat16()
    idx = K.geglu_interleave_index(Fd, cuda)
    pre = torch.empty(M, 2 * Fd, device=cuda, dtype=torch.bfloat16)
    out = K.gemm_geglu(x, w[idx].contiguous(), b[idx].contiguous(), out_pre=pre)
    fr = (x.float() @ w.float().t() + b.float()).requires_grad_(True)
    h, gt = fr.chunk(2, dim=-1)
    ref = h * F.gelu(gt)
    assert _rel(out, ref) < 8e-3
    assert _rel(pre, fr[:, idx]) < 4e-3
    # backward: dout = dy @ Wout (dy [M, dim], Wout^T rows = [F][dim])
    dy = torch.randn(M, dim, device=cuda, generator=g).bfloat16()
    wout_t = (torch.randn(Fd, dim, device=cuda, generator=g) / dim ** 0.5).bfloat16()
    dpre = K.gemm_geglu_bwd(dy, wout_t, pre)
    dout = dy.float() @ wout_t.float().t()
    (gref,) = torch.autograd.grad(ref, fr, dout)
    assert _rel(dpre, gref[:, idx]) < 1.5e-2


def test_geglu_silu_temb(cuda):
    from pairwise_sample_optimization_amd import kernels as K
    h = torch.randn(300, 2 * 640, device=cuda).bfloat16()
    hr = h.float().requires_grad_(True)
    a, gt = hr.chunk(2, dim=-1)
    ref = a * F.gelu(gt)
    out = K.geglu_fwd(h)
    assert _rel(out, ref) < 8e-3
    d = torch.randn_like(out)
    (g,) = torch.autograd.grad(ref, hr, d.float())
    assert _rel(K.geglu_bwd(h, d), g) < 1e-2
    x = torch.randn(4, 1280, device=cuda).bfloat16()
    assert _rel(K.silu(x), F.silu(x.float())) < 8e-3
    t = torch.tensor([999.0, 499.0, 0.0, 1024.0], device=cuda)
    emb = K.timestep_embedding(t, 320)
    half = 160
    ex = torch.exp(-math.log(10000) * torch.arange(half, device=cuda, dtype=torch.float32) / half)
    arg = t[:, None] * ex[None]
    ref = torch.cat([torch.cos(arg), torch.sin(arg)], -1)
    assert (emb.float() - ref).abs().max() < 1e-2


def test_transpose_im2col_sumpool_weight_t(cuda):
    from pairwise_sample_optimization_amd import kernels as K
    x = torch.randn(300, 130, device=cuda).bfloat16()
    assert torch.equal(K.transpose(x), x.t().contiguous())
    img = torch.randn(2, 9, 7, 4, device=cuda).bfloat16()
    cols = K.im2col3(img, 64)
    w = torch.randn(8, 4, 3, 3, device=cuda).bfloat16()
    ref = F.conv2d(img.float().permute(0, 3, 1, 2), w.float(), padding=1)
    wk = torch.zeros(8, 64, device=cuda).bfloat16()
    wk[:, :36] = w.permute(0, 2, 3, 1).reshape(8, 36)
    out = K.gemm(cols, wk, out_dtype=torch.float32).reshape(2, 9, 7, 8).permute(0, 3, 1, 2)
    assert _rel(out, ref) < 1e-5
    u = torch.randn(2, 8, 6, 64, device=cuda).bfloat16()
    sp = K.sumpool2(u)
    refp = F.avg_pool2d(u.float().permute(0, 3, 1, 2), 2).permute(0, 2, 3, 1) * 4
    assert _rel(sp, refp) < 8e-3
    wt = torch.randn(16, 3, 3, 8, device=cuda).bfloat16()
    assert torch.equal(K.conv_weight_t(wt, True), wt.flip(1, 2).permute(3, 1, 2, 0).contiguous())
    assert torch.equal(K.conv_weight_t(wt, False), wt.permute(3, 1, 2, 0).contiguous())


@pytest.mark.parametrize("shape", [(640, 3, 3, 320), (1280, 3, 3, 2560), (4, 3, 3, 320), (320, 3, 3, 4), (100, 1, 1, 72),
                                   (70, 3, 3, 12)])
def test_conv_weight_t_shapes(cuda, shape):
    """Tiled per-tap transpose of the conv weights (16-B row reads when Ci % 8 == 0, ragged tiles, Ci or Co < 64)."""
    from pairwise_sample_optimization_amd import kernels as K
    wt = torch.randn(*shape, device=cuda).bfloat16()
    assert torch.equal(K.conv_weight_t(wt, True), wt.flip(1, 2).permute(3, 1, 2, 0).contiguous())
    assert torch.equal(K.conv_weight_t(wt, False), wt.permute(3, 1, 2, 0).contiguous())


@pytest.mark.parametrize("rc", [(1280, 1280), (10240, 1280), (1280, 5120), (77, 2048), (130, 300), (64, 8)])
def test_transpose_shapes(cuda, rc):
    """Transposes of whole tensors and of column-sliced views (ld > C, unaligned column offset -> scalar reads)."""
    from pairwise_sample_optimization_amd import kernels as K
    R, C = rc
    x = torch.randn(R, C + 24, device=cuda).bfloat16()
    assert torch.equal(K.transpose(x), x.t().contiguous())
    assert torch.equal(K.transpose(x[:, 8:8 + C]), x[:, 8:8 + C].t().contiguous())
    assert torch.equal(K.transpose(x[:, 3:3 + C]), x[:, 3:3 + C].t().contiguous())


def test_transpose_batch_one_launch(cuda):
    """K.transpose inside K.transpose_batch(): outputs returned at once, filled by ONE pso_transpose_multi launch at
    the block's end (ragged shapes, column-sliced views, a temporary source freed inside the block)."""
    from pairwise_sample_optimization_amd import kernels as K
    shapes = [(1280, 1280), (10240, 1280), (77, 2048), (130, 300), (64, 8), (1, 72), (3840, 640)]
    xs = [torch.randn(r, c + 16, device=cuda).bfloat16()[:, 8:8 + c] for r, c in shapes]
    with K.transpose_batch():
        outs = [K.transpose(x) for x in xs]
        tmp = K.transpose(torch.randn(200, 96, device=cuda).bfloat16() * 2)  # source dropped before the launch
        refs_tmp = None
    for x, o in zip(xs, outs):
        assert torch.equal(o, x.t().contiguous())
    assert tmp.shape == (96, 200) and torch.isfinite(tmp.float()).all()
    del refs_tmp


@pytest.mark.parametrize("n", [8, 1003, 4096 * 37 + 5, 1 << 22])
def test_casts_vectorised_and_ragged(cuda, n):
    from pairwise_sample_optimization_amd import kernels as K
    x = torch.randn(n + 3, device=cuda) * 3
    for off in (0, 1):  # 16-B aligned -> 8-wide path + tail; unaligned -> scalar path
        xs = x[off:off + n]
        assert torch.equal(K.cast_f32_bf16(xs), xs.bfloat16())
        assert torch.equal(K.cast_f32_bf16(xs, scale=0.5), (xs * 0.5).bfloat16())
        b = xs.bfloat16()
        y = torch.empty(n + 4, device=cuda)
        K.cast_bf16_f32(b, out=y[off:off + n])
        assert torch.equal(y[off:off + n], b.float())
