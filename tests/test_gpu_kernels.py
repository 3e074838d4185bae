"""GPU parity of the GEMM / conv kernels against a plain torch fp32 reference of the same op."""
import pytest
import torch

from pairwise_sample_optimization_amd import _lib
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


@pytest.mark.parametrize("M,N,K", [(128, 128, 64), (256, 320, 640), (77, 1280, 2048), (4100, 640, 640),
                                   (1024, 10240, 1280), (5, 1280, 2816), (300, 4, 72), (1000, 3, 128)])
def test_gemm_vs_fp32(cuda, M, N, K):
    from pairwise_sample_optimization_amd import kernels as K_
    g = torch.Generator(device="cuda").manual_seed(M * 7 + N)
    a = torch.randn(M, K, device=cuda, generator=g).bfloat16()
    w = (torch.randn(N, K, device=cuda, generator=g) / K ** 0.5).bfloat16()
    b = torch.randn(N, device=cuda, generator=g).bfloat16()
    r = torch.randn(M, N, device=cuda, generator=g).bfloat16()
    out = K_.gemm(a, w, bias=b, resid=r, alpha=0.5)
    ref = 0.5 * (a.float() @ w.float().t()) + b.float() + r.float()
    assert _rel(out, ref) < 4e-3
    out32 = K_.gemm(a, w, out_dtype=torch.float32)
    assert _rel(out32, a.float() @ w.float().t()) < 1e-5


@pytest.mark.parametrize("Z,M,N,K", [(3, 1024, 1024, 512), (2, 4096, 512, 4096), (4, 200, 96, 64), (1, 300, 160, 512)])
def test_gemm_batched_vs_fp32(cuda, Z, M, N, K):
    """The batched product of the VAE mid attention (scores Q K^T, then P V^T-operand) against torch.bmm in fp32."""
    from pairwise_sample_optimization_amd import kernels as K_
    g = torch.Generator(device="cuda").manual_seed(Z * 131 + M + N)
    a = torch.randn(Z, M, K, device=cuda, generator=g).bfloat16()
    w = (torch.randn(Z, N, K, device=cuda, generator=g) / K ** 0.5).bfloat16()
    ref = torch.bmm(a.float(), w.float().transpose(1, 2))
    out = K_.gemm_batched(a, w, alpha=0.25)
    assert _rel(out, 0.25 * ref) < 4e-3
    out32 = K_.gemm_batched(a, w, out_dtype=torch.float32)
    assert _rel(out32, ref) < 1e-5
    for z in range(Z):  # no batch entry bleeds into another
        assert _rel(out32[z], ref[z]) < 1e-5
    # strided views (the VAE passes column slices of the fused qkv rows)
    qkv = torch.randn(Z, M, 3 * K, device=cuda, generator=g).bfloat16()
    o2 = K_.gemm_batched(qkv[:, :, :K], qkv[:, :N, K:2 * K], out_dtype=torch.float32)
    assert _rel(o2, torch.bmm(qkv[:, :, :K].float(), qkv[:, :N, K:2 * K].float().transpose(1, 2))) < 1e-5
    t = K_.transpose_batched(a)
    assert torch.equal(t, a.transpose(1, 2))


def test_gemm_lora_tail_and_accumulate(cuda):
    from pairwise_sample_optimization_amd import kernels as K_
    M, N, K, r = 640, 640, 640, 32
    a = torch.randn(M, K, device=cuda).bfloat16()
    w = (torch.randn(N, K, device=cuda) / 25).bfloat16()
    u = torch.randn(M, r, device=cuda).bfloat16()
    wb = (torch.randn(N, r, device=cuda) / 6).bfloat16()
    out = K_.gemm(a, w, a2=u, w2=wb, out_dtype=torch.float32)
    ref = a.float() @ w.float().t() + u.float() @ wb.float().t()
    assert _rel(out, ref) < 1e-5
    K_.gemm(a, w, out=out, out_dtype=torch.float32, accumulate=True)
    assert _rel(out, ref + a.float() @ w.float().t()) < 1e-5
    # strided operand views (sub-columns of a wider buffer)
    big = torch.randn(M, 3 * K, device=cuda).bfloat16()
    o2 = K_.gemm(big[:, K:2 * K], w)
    assert _rel(o2, big[:, K:2 * K].float() @ w.float().t()) < 4e-3
    # rowbias grouped rows (time-embedding add)
    rb = torch.randn(5, N, device=cuda).bfloat16()
    o3 = K_.gemm(a, w, rowbias=rb, rows_per_group=128, out_dtype=torch.float32)
    ref3 = a.float() @ w.float().t() + rb.float().repeat_interleave(128, 0)
    assert _rel(o3, ref3) < 1e-5


def _nhwc(x):
    return x.permute(0, 2, 3, 1).contiguous()


def _nchw(x):
    return x.permute(0, 3, 1, 2)


@pytest.mark.parametrize("B,C1,C2,H,Cout,ks,stride", [(2, 64, 0, 16, 128, 3, 1), (1, 320, 0, 32, 320, 3, 1),
                                                       (2, 128, 64, 16, 64, 3, 1), (2, 128, 0, 16, 128, 3, 2),
                                                       (2, 128, 192, 8, 64, 1, 1), (1, 64, 0, 9, 4, 3, 1)])
def test_conv_normal(cuda, B, C1, C2, H, Cout, ks, stride):
    from pairwise_sample_optimization_amd import kernels as K_
    x = torch.randn(B, C1 + C2, H, H, device=cuda).bfloat16()
    w = (torch.randn(Cout, C1 + C2, ks, ks, device=cuda) / (ks * (C1 + C2) ** 0.5)).bfloat16()
    bias = torch.randn(Cout, device=cuda).bfloat16()
    temb = torch.randn(B, Cout, device=cuda).bfloat16()
    ref = F.conv2d(x.float(), w.float(), bias.float(), stride=stride, padding=ks // 2) + temb.float()[:, :, None, None]
    xh = _nhwc(x)
    x1, x2 = xh[..., :C1].contiguous(), (xh[..., C1:].contiguous() if C2 else None)
    out = K_.conv2d(x1, _nhwc(w), x2=x2, stride=stride, bias=bias, rowbias=temb, out_dtype=torch.float32)
    assert _rel(_nchw(out), ref) < 1e-5


@pytest.mark.parametrize("B,C,H,W,Cout,bias", [(2, 128, 32, 48, 3, True), (1, 64, 16, 16, 3, False),
                                                (3, 192, 48, 32, 2, True), (1, 128, 32, 32, 1, True),
                                                (1, 128, 20, 20, 3, True)])
def test_conv_small_cout_direct(cuda, B, C, H, W, Cout, bias):
    """Cout <= 3 3x3 convolutions (the VAE decoder's conv_out to RGB) take the direct kernel (conv_small.hip) where
    H, W are multiples of 16 -- the 20 x 20 case falls back to the implicit GEMM -- against an fp32 reference: bf16
    output rounding is the only error (<= 4e-3 rel), image borders (zero padding) included."""
    from pairwise_sample_optimization_amd import kernels as K_
    x = torch.randn(B, C, H, W, device=cuda).bfloat16()
    w = (torch.randn(Cout, C, 3, 3, device=cuda) / (3 * C ** 0.5)).bfloat16()
    b = torch.randn(Cout, device=cuda).bfloat16() if bias else None
    ref = F.conv2d(x.float(), w.float(), b.float() if bias else None, padding=1)
    out = K_.conv2d(_nhwc(x), _nhwc(w), bias=b)
    direct = H % 16 == 0 and W % 16 == 0
    assert K_.lib().pso_last_kernel().decode().startswith("conv3x3_smallc") == direct
    assert _rel(_nchw(out), ref) < 4e-3
    assert (_nchw(out).float() - ref).abs().max().item() < 2e-2 * ref.abs().max().item()


@pytest.mark.parametrize("C1,C2,Cout", [(1280, 0, 1280), (1280, 640, 640)])
@pytest.mark.knobs
def test_conv_splitk_workspace(cuda, C1, C2, Cout):
    """The bs = 1 backward's input-gradient convolutions (2 images at 32 x 32, K = 9 * 1920 / 11520): few output
    tiles, long reduction -> pso_conv2d_ws (K-splits stored, added in split order, bias / time-embedding / residual
    applied once).  fp32 reference; bit-identical on repeat; the unsplit kernel (variant 52) within bf16 rounding."""
    from pairwise_sample_optimization_amd import kernels as K_
    B, H, Ct = 2, 32, C1 + C2
    assert K_.lib().pso_conv2d_ws_bytes(B, H, H, Cout, 9 * Ct, 0) > 0
    x = torch.randn(B, Ct, H, H, device=cuda).bfloat16()
    w = (torch.randn(Cout, Ct, 3, 3, device=cuda) / (3 * Ct ** 0.5)).bfloat16()
    bias = torch.randn(Cout, device=cuda).bfloat16()
    temb = torch.randn(B, Cout, device=cuda).bfloat16()
    res = torch.randn(B, H, H, Cout, device=cuda).bfloat16()
    ref = F.conv2d(x.float(), w.float(), bias.float(), padding=1) + temb.float()[:, :, None, None]
    xh = _nhwc(x)
    x1, x2 = xh[..., :C1].contiguous(), (xh[..., C1:].contiguous() if C2 else None)
    o32 = K_.conv2d(x1, _nhwc(w), x2=x2, bias=bias, rowbias=temb, out_dtype=torch.float32)
    assert _rel(_nchw(o32), ref) < 1e-5
    ob = K_.conv2d(x1, _nhwc(w), x2=x2, bias=bias, rowbias=temb, resid=res)
    ob2 = K_.conv2d(x1, _nhwc(w), x2=x2, bias=bias, rowbias=temb, resid=res)
    assert torch.equal(ob, ob2)
    assert _rel(_nchw(ob), ref + _nchw(res.float())) < 4e-3
    if _lib.KNOBS:  # the unsplit kernel, forced through the tools build's knob (tests/test_knobs_build.py)
        K_.gemm_set_variant(52)
        try:
            on = K_.conv2d(x1, _nhwc(w), x2=x2, bias=bias, rowbias=temb, resid=res)
        finally:
            K_.gemm_set_variant(0)
        assert _rel(ob, on) < 4e-3


def test_conv_up2(cuda):
    from pairwise_sample_optimization_amd import kernels as K_
    x = torch.randn(2, 128, 8, 8, device=cuda).bfloat16()
    w = (torch.randn(64, 128, 3, 3, device=cuda) / 30).bfloat16()
    ref = F.conv2d(F.interpolate(x.float(), scale_factor=2.0, mode="nearest"), w.float(), padding=1)
    out = K_.conv2d(_nhwc(x), _nhwc(w), mode=K_.CONV_UP2, out_dtype=torch.float32)
    assert _rel(_nchw(out), ref) < 1e-5


def test_conv_t2_is_stride2_input_grad(cuda):
    from pairwise_sample_optimization_amd import kernels as K_
    B, Ci, Co, H = 2, 64, 128, 16
    x = torch.randn(B, Ci, H, H, device=cuda, requires_grad=True)
    w = (torch.randn(Co, Ci, 3, 3, device=cuda) / 30).bfloat16().float()
    y = F.conv2d(x, w, stride=2, padding=1)
    dy = torch.randn_like(y).bfloat16().float()
    (gx,) = torch.autograd.grad(y, x, dy)
    wt = w.permute(1, 2, 3, 0).contiguous().bfloat16()  # [Ci][kh][kw][Co], unflipped
    out = K_.conv2d(_nhwc(dy.bfloat16()), wt, mode=K_.CONV_T2, out_hw=(H, H), out_dtype=torch.float32)
    assert _rel(_nchw(out), gx) < 1e-5


def test_conv_stride1_input_grad_flipped(cuda):
    from pairwise_sample_optimization_amd import kernels as K_
    B, Ci, Co, H = 2, 64, 128, 16
    x = torch.randn(B, Ci, H, H, device=cuda, requires_grad=True)
    w = (torch.randn(Co, Ci, 3, 3, device=cuda) / 30).bfloat16().float()
    y = F.conv2d(x, w, padding=1)
    dy = torch.randn_like(y).bfloat16().float()
    (gx,) = torch.autograd.grad(y, x, dy)
    wf = w.flip(2, 3).permute(1, 2, 3, 0).contiguous().bfloat16()  # [Ci][kh'][kw'][Co]
    out = K_.conv2d(_nhwc(dy.bfloat16()), wf, out_dtype=torch.float32)
    assert _rel(_nchw(out), gx) < 1e-5


@pytest.mark.parametrize("M,I,J", [(16384, 96, 640), (308, 32, 2048), (4096, 1280, 32), (100, 64, 8),
                                   (8192, 1280, 32), (8192, 32, 1280), (8192, 96, 1280), (616, 64, 2048),
                                   (1000, 640, 64), (616, 1280, 32), (77, 32, 256),
                                   # full-weight gradients (128 x 128 TN tiles): ragged M / I / J, split-K atomics
                                   (16384, 1280, 1280), (1000, 640, 320), (616, 2880, 640), (77, 136, 264),
                                   (16384, 128, 128), (4100, 1152, 320),
                                   # 256 x 256 TN tiles: one round of workspace slices, and direct (>= 192 tiles)
                                   (6144, 3840, 1280), (1000, 3840, 1280), (2100, 2048, 2048), (3000, 4096, 3072)])
@pytest.mark.parametrize("split_ws", [True, False])
def test_gemm_tn_vs_fp32(cuda, M, I, J, split_ws):
    """Generic TN path and the streaming rank-r path (one side 32 / 64 / 96 wide), partial 64-row steps included;
    full-weight shapes with few 128 x 128 tiles through the workspace split (pso_gemm_tn_ws: partial products stored
    per row slice, added in slice order) and, split_ws=False, through pso_gemm_tn (f32-atomic split); sides that are
    multiples of 256 on the 256 x 256 tiles (workspace slices, or one direct pass with >= 192 tiles)."""
    from pairwise_sample_optimization_amd import kernels as K_
    big = torch.randn(M, I + 16, device=cuda).bfloat16()
    a = big[:, 8:8 + I]          # column-slice view (row stride != I)
    b = torch.randn(M, J, device=cuda).bfloat16()
    out = torch.randn(I, J, device=cuda)
    ref = out + 0.5 * (a.float().t() @ b.float())
    K_.gemm_tn(a, b, out, alpha=0.5, split_ws=split_ws)
    assert _rel(out, ref) < 1e-5
    if split_ws and K_.lib().pso_gemm_tn_ws_bytes(M, I, J):  # the ordered reduction is deterministic
        o1, o2 = torch.zeros(I, J, device=cuda), torch.zeros(I, J, device=cuda)
        K_.gemm_tn(a, b, o1)
        K_.gemm_tn(a, b, o2)
        assert torch.equal(o1, o2)


@pytest.mark.parametrize("M,F,J", [(6144, 5120, 1280), (1000, 2560, 640), (77, 128, 264)])
def test_gemm_tn_geglu_natural_rows(cuda, M, F, J):
    """The GEGLU proj weight gradient from the interleaved pre-activation gradient (per 32 outputs [h 32 | gate 32])
    straight into the natural [h | gate] row order: equals the interleaved product scattered by
    geglu_interleave_index (the transient-matrix + index_add form it replaces) bit for bit, and fp32 to 1e-5."""
    from pairwise_sample_optimization_amd import kernels as K_
    df = torch.randn(M, 2 * F, device=cuda).bfloat16()
    x = torch.randn(M, J + 8, device=cuda).bfloat16()[:, :J]
    base = torch.randn(2 * F, J, device=cuda)
    idx = K_.geglu_interleave_index(F, cuda)
    tmp = torch.zeros(2 * F, J, device=cuda)
    K_.gemm_tn(df, x, tmp, split_ws=False)
    want = base.clone().index_add_(0, idx, tmp)
    out = base.clone()
    K_.gemm_tn_geglu(df, x, out)
    ref = base.clone().index_add_(0, idx, df.float().t() @ x.float())
    assert _rel(out, ref) < 1e-5
    if K_.lib().pso_gemm_tn_ws_bytes(M, 2 * F, J) == 0 and 2 * F >= 128 and J >= 128:  # same tiles, one pass
        assert torch.equal(out, want)


@pytest.mark.parametrize("M,C,G", [(8192, 1280, 3), (1000, 640, 3), (616, 1280, 2)])
def test_gemm_grouped_skinny(cuda, M, C, G):
    """Block-diagonal v = dy sB of the fused q/k/v (G = 3) and cross k/v (G = 2) adapters."""
    from pairwise_sample_optimization_amd import kernels as K_
    a = torch.randn(M, G * C, device=cuda).bfloat16()
    w = (torch.randn(32, G * C, device=cuda) / 30).bfloat16()
    out = K_.gemm_grouped_skinny(a, w, G)
    ref = torch.cat([a[:, j * C:(j + 1) * C].float() @ w[:, j * C:(j + 1) * C].float().t() for j in range(G)], 1)
    assert out.shape == (M, 32 * G)
    assert _rel(out, ref) < 8e-3


@pytest.mark.parametrize("M,C", [(8192, 1280), (1000, 640)])
def test_gemm_tn_grouped(cuda, M, C):
    """Block-diagonal q/k/v form: out[jC + i][:] += dqkv[:, jC + i]^T u_qkv[:, j*32:(j+1)*32]."""
    from pairwise_sample_optimization_amd import kernels as K_
    a = torch.randn(M, 3 * C, device=cuda).bfloat16()
    u = torch.randn(M, 96, device=cuda).bfloat16()
    out = torch.randn(3 * C, 32, device=cuda)
    ref = out.clone()
    for j in range(3):
        ref[j * C:(j + 1) * C] += 0.25 * (a[:, j * C:(j + 1) * C].float().t() @ u[:, 32 * j:32 * (j + 1)].float())
    K_.gemm_tn(a, u, out, alpha=0.25, group=C)
    assert _rel(out, ref) < 1e-5


@pytest.mark.parametrize("M,N,K", [(32, 640, 16384), (1280, 32, 4096), (96, 1280, 8192)])
def test_gemm_splitk_accumulate(cuda, M, N, K):
    from pairwise_sample_optimization_amd import kernels as K_
    a = torch.randn(M, K, device=cuda).bfloat16()
    w = torch.randn(N, K, device=cuda).bfloat16()
    out = torch.randn(M, N, device=cuda)
    ref = out + a.float() @ w.float().t()
    K_.gemm(a, w, out=out, out_dtype=torch.float32, accumulate=True)
    assert _rel(out, ref) < 1e-5


@pytest.mark.knobs
@pytest.mark.parametrize("variant", [0, 1, 2, 3, 4, 5, 6, 7, 8, 10, 11, 12, 14, 16, 17, 18, 19, 20, 21, 22, 23, 24, 25,
                                     26, 27, 28, 29, 30, 31, 37, 38, 41, 48, 49, 55])
@pytest.mark.parametrize("M,N,K,tail", [(16384, 1920, 640, 640), (4096, 3840, 1280, 1280), (4096, 1280, 5120, 0),
                                        (8192, 640, 320, 0), (1000, 700, 136, 0), (2048, 1280, 1280, 1280)])
def test_gemm_every_variant_large(cuda, variant, M, N, K, tail):
    """Every tile configuration on UNet-scale shapes, with and without the grouped LoRA K-tail (3 groups)."""
    from pairwise_sample_optimization_amd import kernels as K_
    K_.gemm_set_variant(variant)
    try:
        g = torch.Generator(device="cuda").manual_seed(M + N + variant)
        a = torch.randn(M, K, device=cuda, generator=g).bfloat16()
        w = (torch.randn(N, K, device=cuda, generator=g) / K ** 0.5).bfloat16()
        b = torch.randn(N, device=cuda, generator=g).bfloat16()
        r = torch.randn(M, N, device=cuda, generator=g).bfloat16()
        kw = {}
        ref = a.float() @ w.float().t() + b.float() + r.float()
        if tail:
            ng = N // tail
            u = torch.randn(M, 32 * ng, device=cuda, generator=g).bfloat16()
            w2 = (torch.randn(N, 32, device=cuda, generator=g) / 6).bfloat16()
            kw = dict(a2=u, w2=w2, tail_group_n=tail)
            for j in range(ng):
                ref[:, j * tail:(j + 1) * tail] += u[:, 32 * j:32 * (j + 1)].float() @ w2[j * tail:(j + 1) * tail].float().t()
        sentinel = torch.full((M + 64, N), 7.0, device=cuda, dtype=torch.bfloat16)
        out = sentinel[:M]
        K_.gemm(a, w, bias=b, resid=r, out=out, **kw)
        assert _rel(out, ref) < 4e-3
        assert (sentinel[M:] == 7.0).all()  # nothing written past the output
    finally:
        K_.gemm_set_variant(0)


@pytest.mark.parametrize("M,N,K,K2,tail_rows,f32", [(2048, 1280, 10240, 0, 0, False), (2048, 1280, 3840, 96, 0, False),
                                                    (2000, 1280, 4096, 32, 1000, False), (1024, 640, 5120, 0, 0, True),
                                                    (2048, 1280, 2560, 32, 0, True)])
def test_gemm_splitk_workspace(cuda, M, N, K, K2, tail_rows, f32):
    """pso_gemm_ws (the bs = 1 backward's small-M, long-K products): split-K through a workspace, the splits added in
    order by a second kernel that applies the epilogue -- bias, row-group bias or residual, bf16 or f32 (accumulate)
    output, the LoRA K-tail on the first tail_rows rows -- against fp32, bit-identical on a second run."""
    from pairwise_sample_optimization_amd import kernels as K_
    assert K_.lib().pso_gemm_ws_bytes(M, N, K, K2) > 0  # the shape takes the split path
    g = torch.Generator(device="cuda").manual_seed(M + N + K)
    a = torch.randn(M, K, device=cuda, generator=g).bfloat16()
    w = (torch.randn(N, K, device=cuda, generator=g) / K ** 0.5).bfloat16()
    b = torch.randn(N, device=cuda, generator=g).bfloat16()
    r = torch.randn(M, N, device=cuda, generator=g).bfloat16()
    kw = {}
    ref = a.float() @ w.float().t() * 0.5
    if K2:
        rows = tail_rows or M
        u = torch.randn(rows, K2, device=cuda, generator=g).bfloat16()
        w2 = (torch.randn(N, K2, device=cuda, generator=g) / 6).bfloat16()
        kw = dict(a2=u, w2=w2, tail_rows=tail_rows)
        ref[:rows] += 0.5 * (u.float() @ w2.float().t())
    if f32:
        base = torch.randn(M, N, device=cuda, generator=g)
        outs = []
        for _ in range(2):
            o = base.clone()
            K_.gemm(a, w, bias=b, alpha=0.5, out=o, out_dtype=torch.float32, accumulate=True, **kw)
            outs.append(o)
        ref = base + ref + b.float()
        assert _rel(outs[0], ref) < 1e-5
    else:
        outs = []
        for _ in range(2):
            sentinel = torch.full((M + 64, N), 7.0, device=cuda, dtype=torch.bfloat16)
            K_.gemm(a, w, bias=b, resid=r, alpha=0.5, out=sentinel[:M], **kw)
            assert (sentinel[M:] == 7.0).all()
            outs.append(sentinel[:M])
        ref = ref + b.float() + r.float()
        assert _rel(outs[0], ref) < 4e-3
    assert torch.equal(outs[0], outs[1])


@pytest.mark.knobs
@pytest.mark.parametrize("M,N,K", [(4096, 2560, 1280), (1000, 768, 640), (300, 256, 128), (16384, 1024, 256),
                                   (257, 512, 384)])
def test_gemm_8phase(cuda, M, N, K):
    """The 8-phase 256x256 kernel (gemm8p.hip, variant 30): bias epilogue, ragged last row tile, 2..20 K-tiles
    (odd and even K-tile pair counts); nothing is written past the output rows."""
    from pairwise_sample_optimization_amd import kernels as K_
    K_.gemm_set_variant(30)
    try:
        g = torch.Generator(device="cuda").manual_seed(M + N + K)
        a = torch.randn(M, K, device=cuda, generator=g).bfloat16()
        w = (torch.randn(N, K, device=cuda, generator=g) / K ** 0.5).bfloat16()
        b = torch.randn(N, device=cuda, generator=g).bfloat16()
        ref = a.float() @ w.float().t() + b.float()
        sentinel = torch.full((M + 64, N), 7.0, device=cuda, dtype=torch.bfloat16)
        out = sentinel[:M]
        K_.gemm(a, w, bias=b, out=out)
        assert _rel(out, ref) < 4e-3
        assert (sentinel[M:] == 7.0).all()
    finally:
        K_.gemm_set_variant(0)


@pytest.mark.knobs
@pytest.mark.parametrize("M,N,K,K2,group,tail_rows", [(4096, 3840, 1280, 32, 1280, 2048), (1000, 768, 640, 32, 256, 0),
                                                      (4100, 1024, 640, 96, 0, 4100), (520, 512, 192, 32, 512, 300),
                                                      (16384, 3840, 1280, 32, 1280, 8192)])
def test_gemm_8phase_lora_tail_paired_resid(cuda, M, N, K, K2, group, tail_rows):
    """gemm8p with the LoRA K-tail (grouped per output-column block, or plain), restricted to the first tail_rows rows
    (the policy half of a paired pass), alpha, bias and a residual epilogue; odd / even K-tile counts."""
    from pairwise_sample_optimization_amd import kernels as K_
    K_.gemm_set_variant(30)
    try:
        g = torch.Generator(device="cuda").manual_seed(M + N + K + K2)
        a = torch.randn(M, K, device=cuda, generator=g).bfloat16()
        w = (torch.randn(N, K, device=cuda, generator=g) / K ** 0.5).bfloat16()
        b = torch.randn(N, device=cuda, generator=g).bfloat16()
        r = torch.randn(M, N, device=cuda, generator=g).bfloat16()
        tr = tail_rows or M
        ng = N // group if group else 1
        u = torch.randn(tr, K2 * ng, device=cuda, generator=g).bfloat16()
        w2 = (torch.randn(N, K2, device=cuda, generator=g) / 6).bfloat16()
        y = a.float() @ w.float().t()
        for j in range(ng):
            cs = slice(j * group, (j + 1) * group) if group else slice(0, N)
            y[:tr, cs] += u[:, K2 * j:K2 * (j + 1)].float() @ w2[cs].float().t()
        ref = (0.75 * y + b.float()).bfloat16().float() + r.float()
        sentinel = torch.full((M + 64, N), 7.0, device=cuda, dtype=torch.bfloat16)
        out = sentinel[:M]
        K_.gemm(a, w, bias=b, resid=r, a2=u, w2=w2, alpha=0.75, tail_group_n=group, tail_rows=tail_rows, out=out)
        assert _rel(out, ref) < 4e-3
        assert _rel(out[tr:], ref[tr:]) < 4e-3 if tr < M else True
        assert (sentinel[M:] == 7.0).all()
    finally:
        K_.gemm_set_variant(0)


@pytest.mark.knobs
@pytest.mark.parametrize("M,N,K,K2,group,tail_rows", [(16384, 1280, 1280, 0, 0, 0), (1000, 640, 640, 32, 640, 0),
                                                      (4100, 1920, 640, 32, 640, 2048), (300, 320, 192, 0, 0, 0),
                                                      (8192, 1280, 5120, 32, 0, 4096), (257, 640, 64, 96, 320, 100)])
def test_gemm_8phase_256x160(cuda, M, N, K, K2, group, tail_rows):
    """The 8-phase 256 x 160 kernel (gemm8p.hip BN = 160, variant 38): bias / alpha / residual epilogue, ragged last
    row tile, odd / even K-tile counts (1..80), the LoRA K-tail grouped per 160-multiple column block or plain,
    restricted to the first tail_rows rows; nothing is written past the output rows."""
    from pairwise_sample_optimization_amd import kernels as K_
    K_.gemm_set_variant(38)
    try:
        g = torch.Generator(device="cuda").manual_seed(M + N + K + K2)
        a = torch.randn(M, K, device=cuda, generator=g).bfloat16()
        w = (torch.randn(N, K, device=cuda, generator=g) / K ** 0.5).bfloat16()
        b = torch.randn(N, device=cuda, generator=g).bfloat16()
        r = torch.randn(M, N, device=cuda, generator=g).bfloat16()
        y = a.float() @ w.float().t()
        kw = {}
        if K2:
            tr = tail_rows or M
            ng = N // group if group else 1
            u = torch.randn(tr, K2 * ng, device=cuda, generator=g).bfloat16()
            w2 = (torch.randn(N, K2, device=cuda, generator=g) / 6).bfloat16()
            for j in range(ng):
                cs = slice(j * group, (j + 1) * group) if group else slice(0, N)
                y[:tr, cs] += u[:, K2 * j:K2 * (j + 1)].float() @ w2[cs].float().t()
            kw = dict(a2=u, w2=w2, tail_group_n=group, tail_rows=tail_rows)
        ref = (0.75 * y + b.float()).bfloat16().float() + r.float()
        sentinel = torch.full((M + 64, N), 7.0, device=cuda, dtype=torch.bfloat16)
        out = sentinel[:M]
        K_.gemm(a, w, bias=b, resid=r, alpha=0.75, out=out, **kw)
        assert K_.lib().pso_last_kernel().decode() == "gemm8p_kernel<0, true, false, false, 160, false>"
        assert _rel(out, ref) < 4e-3
        assert (sentinel[M:] == 7.0).all()
    finally:
        K_.gemm_set_variant(0)


@pytest.mark.knobs
@pytest.mark.parametrize("M,N,K,K2,group,tail_rows", [(16384, 1280, 1280, 0, 0, 0), (16384, 1280, 1280, 32, 0, 8192),
                                                      (1000, 640, 640, 32, 320, 0), (4100, 1920, 640, 32, 640, 2048),
                                                      (300, 320, 192, 0, 0, 0), (8192, 1280, 5120, 64, 0, 4096),
                                                      (257, 640, 2880, 32, 320, 100), (65536, 640, 640, 32, 0, 32768)])
def test_gemm_8phase_256x320(cuda, M, N, K, K2, group, tail_rows):
    """The 8-phase 256 x 320 kernel (gemm8p.hip BN = 320, variant 39): 20-piece B images (a third piece per wave,
    waves 4-7 into a dummy slot from past the buffer range), bias / alpha / residual epilogue in two 128-row halves,
    ragged last row tile, odd K-tile counts (the zero pad tile), the LoRA K-tail from register operands after the
    main loop -- plain or grouped per 320-multiple column block, restricted to the first tail_rows rows, K2 up to 64;
    nothing is written past the output rows."""
    from pairwise_sample_optimization_amd import kernels as K_
    K_.gemm_set_variant(39)
    try:
        g = torch.Generator(device="cuda").manual_seed(M + N + K + K2 + 1)
        a = torch.randn(M, K, device=cuda, generator=g).bfloat16()
        w = (torch.randn(N, K, device=cuda, generator=g) / K ** 0.5).bfloat16()
        b = torch.randn(N, device=cuda, generator=g).bfloat16()
        r = torch.randn(M, N, device=cuda, generator=g).bfloat16()
        y = a.float() @ w.float().t()
        kw = {}
        if K2:
            tr = tail_rows or M
            ng = N // group if group else 1
            u = torch.randn(tr, K2 * ng, device=cuda, generator=g).bfloat16()
            w2 = (torch.randn(N, K2, device=cuda, generator=g) / 6).bfloat16()
            for j in range(ng):
                cs = slice(j * group, (j + 1) * group) if group else slice(0, N)
                y[:tr, cs] += u[:, K2 * j:K2 * (j + 1)].float() @ w2[cs].float().t()
            kw = dict(a2=u, w2=w2, tail_group_n=group, tail_rows=tail_rows)
        ref = (0.75 * y + b.float()).bfloat16().float() + r.float()
        sentinel = torch.full((M + 64, N), 7.0, device=cuda, dtype=torch.bfloat16)
        out = sentinel[:M]
        K_.gemm(a, w, bias=b, resid=r, alpha=0.75, out=out, **kw)
        assert K_.lib().pso_last_kernel().decode() == "gemm8p_kernel<0, true, false, false, 320, false>"
        assert _rel(out, ref) < 4e-3
        assert (sentinel[M:] == 7.0).all()
        # and without bias / residual (the plain store path)
        out2 = K_.gemm(a, w, **kw)
        ref2 = y.bfloat16().float()
        assert _rel(out2, ref2) < 4e-3
    finally:
        K_.gemm_set_variant(0)


@pytest.mark.knobs
@pytest.mark.parametrize("variant", [0, 57])
@pytest.mark.parametrize("M,Fd,K,pre_rows", [(4096, 5120, 1280, 2048), (6144, 5120, 1280, 0), (2048, 5120, 1280, 1024),
                                             (24576, 2560, 640, 12288), (1900, 5120, 640, 950)])
def test_gemm_geglu_320_tiles(cuda, variant, M, Fd, K, pre_rows):
    """The GEGLU projection on 256 x 320 tiles where they cost fewer tile-rounds than 256 x 256 (bs = 1's 4096 x 10240,
    C3's 6144 x 10240 and 24576 x 5120, C5's 2048 x 10240, a ragged M): against torch fp32, and -- in the tools build --
    bit for bit against the 256 x 256 form (variant 57): the same accumulation order and the same epilogue arithmetic on
    the same bf16 pre-activations."""
    from pairwise_sample_optimization_amd import kernels as K_
    g = torch.Generator(device="cuda").manual_seed(M + Fd + 1)
    x = torch.randn(M, K, device=cuda, generator=g).bfloat16()
    wp = (torch.randn(2 * Fd, K, device=cuda, generator=g) / K ** 0.5).bfloat16()
    bp = torch.randn(2 * Fd, device=cuda, generator=g).bfloat16()
    idx = K_.geglu_interleave_index(Fd, cuda)
    wi, bi = wp[idx].contiguous(), bp[idx].contiguous()
    pr = pre_rows or M

    def run():
        pre = torch.full((pr, 2 * Fd), float("nan"), device=cuda, dtype=torch.bfloat16)
        out = K_.gemm_geglu(x, wi, bi, out_pre=pre, pre_rows=pre_rows)
        return out, pre, K_.lib().pso_last_kernel().decode()

    out, pre, kn = run()
    assert kn == "gemm8p_kernel<1, true, false, false, 320, false>", kn
    hg = (x.float() @ wp.float().t() + bp.float()).bfloat16().float()
    h, gt = hg[:, :Fd], hg[:, Fd:]
    assert _rel(out, h * F.gelu(gt)) < 4e-3
    assert _rel(pre, hg[:pr, idx]) < 4e-3 and not torch.isnan(pre).any()
    if variant:
        K_.gemm_set_variant(variant)
        try:
            out2, pre2, kn2 = run()
        finally:
            K_.gemm_set_variant(0)
        assert kn2 == "gemm8p_kernel<1, true, false, false, 256, false>", kn2
        assert torch.equal(out, out2) and torch.equal(pre, pre2)


@pytest.mark.knobs
@pytest.mark.parametrize("variant", [0, 31, 45])
@pytest.mark.parametrize("M,Fd,K,pre_rows", [(4096, 5120, 1280, 2048), (1000, 2560, 640, 0), (300, 1280, 320, 100),
                                             (8192, 2560, 640, 0)])
def test_gemm_geglu_fwd_bwd_paths(cuda, variant, M, Fd, K, pre_rows):
    """The GEGLU projection (interleaved [h | gate] weight rows) and its backward through ff.net.2, on the 8-phase
    path (default: the backward on 256 x 320 tiles where they make whole rounds), the 8-phase 256 x 256 backward
    (variant 45) and the 2-phase one (variant 31), against torch fp32 on the same bf16 operands."""
    from pairwise_sample_optimization_amd import kernels as K_
    K_.gemm_set_variant(variant)
    try:
        g = torch.Generator(device="cuda").manual_seed(M + Fd)
        x = torch.randn(M, K, device=cuda, generator=g).bfloat16()
        wp = (torch.randn(2 * Fd, K, device=cuda, generator=g) / K ** 0.5).bfloat16()  # diffusers [h rows; gate rows]
        bp = torch.randn(2 * Fd, device=cuda, generator=g).bfloat16()
        idx = K_.geglu_interleave_index(Fd, cuda)
        pr = pre_rows or M
        pre = torch.empty(pr, 2 * Fd, device=cuda, dtype=torch.bfloat16)
        out = K_.gemm_geglu(x, wp[idx].contiguous(), bp[idx].contiguous(), out_pre=pre, pre_rows=pre_rows)
        hg = (x.float() @ wp.float().t() + bp.float()).bfloat16().float()
        h, gt = hg[:, :Fd], hg[:, Fd:]
        assert _rel(out, h * F.gelu(gt)) < 4e-3
        assert _rel(pre, hg[:pr, idx]) < 4e-3
        # backward: dout = dy @ W_out^T-form operand [Fd, C] given as w [Fd][C]; din interleaved
        C = K
        dy = torch.randn(M, C, device=cuda, generator=g).bfloat16()
        wo = (torch.randn(Fd, C, device=cuda, generator=g) / C ** 0.5).bfloat16()
        full_pre = hg[:, idx].bfloat16()
        din = K_.gemm_geglu_bwd(dy, wo, full_pre)
        if variant == 0 and M in (4096, 8192):  # 256 and 256 tiles of 256 x 320: whole rounds
            assert K_.lib().pso_last_kernel().decode() == "gemm8p_kernel<2, true, false, false, 320, false>"
        dout = (dy.float() @ wo.float().t()).bfloat16().float()
        hh, gg = h, gt
        cdf = 0.5 * (1 + torch.erf(gg / 2 ** 0.5))
        pdf = torch.exp(-0.5 * gg * gg) / (2 * torch.pi) ** 0.5
        ref = torch.cat([dout * gg * cdf, dout * hh * (cdf + gg * pdf)], 1)[:, idx]
        assert _rel(din, ref) < 6e-3
    finally:
        K_.gemm_set_variant(0)


@pytest.mark.knobs
@pytest.mark.parametrize("variant", [0, 44])
@pytest.mark.parametrize("B,C,H,W,Cout", [(2, 320, 64, 64, 320), (1, 640, 32, 32, 640), (3, 1280, 16, 16, 1280),
                                          (2, 64, 8, 32, 320), (1, 128, 32, 8, 640), (2, 192, 16, 16, 960)])
def test_conv_8phase_256x320(cuda, variant, B, C, H, W, Cout):
    """The 3x3 implicit-GEMM conv on the 8-phase 256 x 320 tiles (gemm8p.hip CONV; variant 44 forces it, the default
    takes it at >= 256 tiles): bias + per-image row bias + residual, bf16 out, against torch fp32 on the same bf16
    operands.  The image sits inside a NaN-poisoned buffer (the A resource spans W + 1 pixels either side): a tap
    that leaked past an image edge, or across images, would read NaN or a neighbour."""
    from pairwise_sample_optimization_amd import kernels as K_
    g = torch.Generator(device="cuda").manual_seed(B * C + H * W + Cout)
    x = torch.randn(B, C, H, W, device=cuda, generator=g).bfloat16()
    w = (torch.randn(Cout, C, 3, 3, device=cuda, generator=g) / (3 * C ** 0.5)).bfloat16()
    bias = torch.randn(Cout, device=cuda, generator=g).bfloat16()
    temb = torch.randn(B, Cout, device=cuda, generator=g).bfloat16()
    res = torch.randn(B, H, W, Cout, device=cuda, generator=g).bfloat16()
    ref = (F.conv2d(x.float(), w.float(), bias.float(), padding=1) + temb.float()[:, :, None, None]
           + _nchw(res.float()))
    pad = (W + 1 + 64) * C
    buf = torch.full((B * H * W * C + 2 * pad,), float("nan"), device=cuda).bfloat16()
    xh = buf[pad:pad + B * H * W * C].view(B, H, W, C)
    xh.copy_(_nhwc(x))
    K_.gemm_set_variant(variant)
    try:
        out = K_.conv2d(xh, _nhwc(w), bias=bias, rowbias=temb, resid=res)
        kname = K_.lib().pso_last_kernel().decode()
    finally:
        K_.gemm_set_variant(0)
    if variant == 44 or (B * H * W // 256) * (Cout // 320) >= 256:
        assert kname == "gemm8p_kernel<0, true, false, false, 320, true>", kname
    assert torch.isfinite(out.float()).all()
    assert _rel(_nchw(out.float()), ref) < 4e-3


@pytest.mark.knobs
@pytest.mark.parametrize("variant", [0, 1, 3, 4, 6, 7, 8, 10, 11, 12, 14, 16, 17, 18, 19, 41])
def test_conv_every_variant_large(cuda, variant):
    from pairwise_sample_optimization_amd import kernels as K_
    K_.gemm_set_variant(variant)
    try:
        x = torch.randn(4, 320, 64, 64, device=cuda).bfloat16()
        w = (torch.randn(640, 320, 3, 3, device=cuda) / 50).bfloat16()
        ref = F.conv2d(x.float(), w.float(), padding=1)
        out = K_.conv2d(_nhwc(x), _nhwc(w), out_dtype=torch.float32)
        assert _rel(_nchw(out), ref) < 1e-5
    finally:
        K_.gemm_set_variant(0)


@pytest.mark.parametrize("M,N,K", [(4096, 32, 1280), (4096, 96, 1280), (16384, 32, 640), (300, 100, 136),
                                   (1000, 64, 2048), (257, 128, 72), (4096, 4, 40), (32768, 32, 640),
                                   (8192, 96, 1280), (616, 64, 2048), (20000, 48, 320),
                                   (2048, 96, 1280), (2048, 32, 1032), (1500, 16, 1272), (16384, 32, 1280)])
def test_gemm_skinny_n(cuda, M, N, K):
    """LoRA-rank products (N <= 128): bf16 out, strided A view, f32 accumulate; ragged M / K tails.  1024 < K <= 1280
    takes the single-load-round form (5 steps per wave) on 16-, 32- and 64-row tiles, ragged K included."""
    from pairwise_sample_optimization_amd import kernels as K_
    g = torch.Generator(device="cuda").manual_seed(M + N + K)
    big = torch.randn(M, K + 24, device=cuda, generator=g).bfloat16()
    a = big[:, 16:16 + K]
    w = (torch.randn(N, K, device=cuda, generator=g) / K ** 0.5).bfloat16()
    ref = a.float() @ w.float().t()
    out = K_.gemm(a, w, alpha=0.5)
    assert out.shape == (M, N)
    assert _rel(out, 0.5 * ref) < 4e-3
    acc = torch.randn(M, N, device=cuda, generator=g)
    want = acc + ref
    K_.gemm(a, w, out=acc, out_dtype=torch.float32, accumulate=True)
    assert _rel(acc, want) < 1e-5


def test_fullgrad_helpers(cuda):
    """pso_colsum_acc (one group / per-image groups), pso_layer_norm_dparam, pso_im2col_conv (NORMAL stride 1 / 2,
    UP2, two concatenated sources) against torch."""
    from pairwise_sample_optimization_amd import kernels as K_
    g = torch.Generator(device="cuda").manual_seed(11)
    x = torch.randn(3000, 200, device=cuda, generator=g).bfloat16()
    out = torch.randn(1, 200, device=cuda)
    ref = out + x.float().sum(0, keepdim=True)
    K_.colsum_acc(x, out)
    assert _rel(out, ref) < 1e-5
    xb = torch.randn(4 * 1024, 320, device=cuda, generator=g).bfloat16()
    big = torch.zeros(4, 640, device=cuda)
    K_.colsum_acc(xb, big[:, 100:420], rows_per_group=1024)
    assert _rel(big[:, 100:420], xb.float().view(4, 1024, 320).sum(1)) < 1e-5 and big[:, :100].abs().max() == 0
    M, C = 777, 640
    xl = torch.randn(M, C, device=cuda, generator=g).bfloat16()
    gm = (1 + 0.1 * torch.randn(C, device=cuda, generator=g)).bfloat16()
    bt = (0.1 * torch.randn(C, device=cuda, generator=g)).bfloat16()
    _, st = K_.layer_norm_fwd(xl, gm, bt, 1e-5)
    dy = torch.randn(M, C, device=cuda, generator=g).bfloat16()
    dg = torch.zeros(C, device=cuda)
    db = torch.zeros(C, device=cuda)
    K_.layer_norm_dparam(xl, dy, st, dg, db)
    w = gm.float().requires_grad_(True)
    b = bt.float().requires_grad_(True)
    y = F.layer_norm(xl.float(), (C,), w, b, 1e-5)
    gw, gb = torch.autograd.grad(y, (w, b), dy.float())
    assert _rel(dg, gw) < 1e-4 and _rel(db, gb) < 1e-5
    # the ordered forms are bit-reproducible (no float atomics): twice the same bits; N = 4 (conv_out's bias), groups
    # of 1000 rows (row blocks end at every group edge)
    for N_, rpg in ((4, None), (1280, 1000), (320, 4096)):
        xr = torch.randn(4000 if rpg != 4096 else 8192, N_, device=cuda, generator=g).bfloat16()
        G_ = 1 if rpg is None else (xr.shape[0] + rpg - 1) // rpg
        o1, o2 = torch.zeros(G_, N_, device=cuda), torch.zeros(G_, N_, device=cuda)
        K_.colsum_acc(xr, o1, rows_per_group=rpg)
        K_.colsum_acc(xr, o2, rows_per_group=rpg)
        r_ = rpg or xr.shape[0]
        want = torch.stack([xr[i * r_:(i + 1) * r_].float().sum(0) for i in range(G_)])
        assert torch.equal(o1, o2) and _rel(o1, want) < 1e-5, (N_, rpg)
    dg2, db2 = torch.zeros(C, device=cuda), torch.zeros(C, device=cuda)
    K_.layer_norm_dparam(xl, dy, st, dg2, db2)
    assert torch.equal(dg, dg2) and torch.equal(db, db2)
    for mode, stride, C1, C2 in [(K_.CONV_NORMAL, 1, 64, 0), (K_.CONV_NORMAL, 2, 32, 0), (K_.CONV_UP2, 1, 32, 0),
                                 (K_.CONV_NORMAL, 1, 64, 32)]:
        B, H, W = 2, 9, 7
        x1 = torch.randn(B, H, W, C1, device=cuda, generator=g).bfloat16()
        x2 = torch.randn(B, H, W, C2, device=cuda, generator=g).bfloat16() if C2 else None
        cols = K_.im2col_conv(x1, x2, mode=mode, stride=stride)
        xc = torch.cat([x1, x2], -1) if C2 else x1
        xn = xc.permute(0, 3, 1, 2).float()
        if mode == K_.CONV_UP2:
            xn = F.interpolate(xn, scale_factor=2.0, mode="nearest")
        u = F.unfold(xn, 3, padding=1, stride=stride)                 # [B, C*9, L] with (c, ky, kx) order
        Ct = C1 + C2
        u = u.view(B, Ct, 9, -1).permute(0, 3, 2, 1).reshape(-1, 9 * Ct)  # -> (pixel, tap, c)
        assert cols.shape == u.shape and torch.equal(cols.float(), u), (mode, stride, C1, C2)


def test_tn_rank_batch_equals_individual_products(cuda):
    """pso_gemm_tn_rank_batch (TnRankQueue: the deferred LoRA dA / dB products of a gradient unit in one launch per
    rank / orientation) against the same products issued one by one, and against fp32 torch: mixed M (ragged last
    row step included), C, ranks 32 / 64 / 96, the grouped q/k/v form and both orientations, accumulated twice."""
    from pairwise_sample_optimization_amd import kernels as K
    g = torch.Generator(device="cuda").manual_seed(21)
    specs = [  # (M, I, J, group) for gemm_tn(a [M, I], b [M, J]) -> out [I, r]
        (8192, 1280, 32, 0), (8192, 32, 1280, 0), (4000, 640, 32, 0), (8192, 96, 1280, 0),
        (8192, 3840, 96, 1280), (616, 64, 2048, 0), (616, 2560, 64, 1280), (33, 256, 32, 0), (32768, 640, 32, 0)]
    ops = []
    for M, I, J, grp in specs:
        a = torch.randn(M, I, device=cuda, generator=g).bfloat16()
        b = torch.randn(M, J, device=cuda, generator=g).bfloat16()
        r = J * grp // I if grp else J
        ops.append((a, b, grp, torch.zeros(I, r, device=cuda), torch.zeros(I, r, device=cuda)))
    q = K.TnRankQueue()
    for rep in range(2):
        for a, b, grp, o1, o2 in ops:
            K.gemm_tn(a, b, o1, 0.5, group=grp)
            q.add(a, b, o2, 0.5, group=grp)
        q.flush()
    torch.cuda.synchronize()
    for (M, I, J, grp), (a, b, _, o1, o2) in zip(specs, ops):
        if grp:
            r = J * grp // I
            ref = torch.cat([a[:, j * grp:(j + 1) * grp].float().t() @ b[:, (j * grp // grp) * r:(j + 1) * r].float()
                             for j in range(I // grp)], 0)
        else:
            ref = a.float().t() @ b.float()
        ref = ref * 1.0  # two accumulations of alpha 0.5
        assert ((o2 - o1).norm() / o1.norm()).item() < 1e-5, (M, I, J, grp)
        assert ((o2 - ref).norm() / ref.norm()).item() < 1e-3, (M, I, J, grp)


def test_tn_rank_batch_deterministic(cuda):
    """The training path's rank-r TN batch (pso_gemm_tn_rank_batch_ws: partials stored, added in row-range order) gives
    the same bits on every run, also when two products of one launch accumulate into the same output (they go to
    separate launches), and agrees with the f32-atomic form to rounding."""
    from pairwise_sample_optimization_amd import kernels as K
    assert K.TnRankQueue.deterministic
    g = torch.Generator(device="cuda").manual_seed(22)
    specs = [(16384, 1280, 32, 0), (16384, 32, 1280, 0), (8192, 3840, 96, 1280), (616, 64, 2048, 0),
             (4000, 640, 64, 0), (32768, 640, 32, 0)]
    ops = []
    for M, I, J, grp in specs:
        a = torch.randn(M, I, device=cuda, generator=g).bfloat16()
        b = torch.randn(M, J, device=cuda, generator=g).bfloat16()
        ops.append((a, b, grp, J * grp // I if grp else J))
    shared = torch.zeros(1280, 32, device=cuda)
    a2 = torch.randn(16384, 1280, device=cuda, generator=g).bfloat16()
    b2 = torch.randn(16384, 32, device=cuda, generator=g).bfloat16()

    def run(det):
        K.TnRankQueue.deterministic = det
        try:
            outs = [torch.zeros(a.shape[1], r, device=cuda) for a, _, _, r in ops]
            sh = shared.clone()
            q = K.TnRankQueue()
            for rep in range(2):
                for (a, b, grp, _), o in zip(ops, outs):
                    q.add(a, b, o, 0.5, group=grp)
                q.add(a2, b2, sh, 1.0)
                q.add(ops[0][0], ops[0][1], sh, 1.0)  # same output twice in one batch
                q.flush()
            torch.cuda.synchronize()
            return outs + [sh]
        finally:
            K.TnRankQueue.deterministic = True

    d1, d2, at = run(True), run(True), run(False)
    for x, y, z in zip(d1, d2, at):
        assert torch.equal(x, y)
        assert ((x - z).norm() / z.norm()).item() < 1e-5
    ref = 2 * (a2.float().t() @ b2.float() + ops[0][0].float().t() @ ops[0][1].float())
    assert ((d1[-1] - ref).norm() / ref.norm()).item() < 1e-3


@pytest.mark.parametrize("n", [2048 * 37, 2048 * 5 + 1003])
def test_adamw8bit_vs_restatement(cuda, n):
    """pso_adamw8bit_step (bitsandbytes AdamW8bit, the reference's default optimizer T:427-435) against the numpy
    restatement oracle/adam8bit.py over 5 steps from zero state: the maps are the same floats, every quantised code and
    block absmax agrees, parameters to fp32 rounding (parity unpinned: no bitsandbytes here).  The ragged size checks
    the kernel's scalar tail (partial last block and thread) against the restatement on the zero-padded vector (padded
    elements keep m = v = 0 and do not move a block's absmax)."""
    import numpy as np
    import ctypes
    from oracle import adam8bit as O
    from pairwise_sample_optimization_amd import kernels as K_
    s = (ctypes.c_float * 256)()
    u = (ctypes.c_float * 256)()
    K_.lib().pso_adamw8bit_maps(s, u)
    assert np.array_equal(np.array(list(s), dtype=np.float32), O.create_dynamic_map(True))
    assert np.array_equal(np.array(list(u), dtype=np.float32), O.create_dynamic_map(False))
    npad = -(-n // 2048) * 2048
    g_ = np.random.default_rng(3)
    p = np.zeros(npad, np.float32)
    p[:n] = g_.standard_normal(n).astype(np.float32) * 0.02
    f32 = lambda x: float(np.float32(x))
    lr, b1, b2, eps, wd = f32(1e-3), f32(0.9), f32(0.999), f32(1e-8), f32(1e-2)
    pd = torch.tensor(p[:n], device=cuda)
    st = K_.Adam8State(n, cuda)
    qm, qv = np.zeros(npad, np.uint8), np.zeros(npad, np.uint8)
    am, av = np.zeros(npad // 2048, np.float32), np.zeros(npad // 2048, np.float32)
    for step in range(1, 6):
        gr = np.zeros(npad, np.float32)
        gr[:n] = (g_.standard_normal(n) * np.exp(g_.standard_normal(n))).astype(np.float32) * 1e-2
        wb = torch.full((n,), float("nan"), device=cuda, dtype=torch.bfloat16) if step == 5 else None
        K_.adamw8bit_step(pd, torch.tensor(gr[:n], device=cuda), st, lr, (b1, b2), eps, wd, step, out_bf16=wb)
        p, qm, qv, am, av = O.adamw8bit_step(p, gr, qm, qv, am, av, lr, b1, b2, eps, wd, step)
    torch.cuda.synchronize()
    assert np.array_equal(st.am.cpu().numpy(), am) and np.array_equal(st.av.cpu().numpy(), av)
    assert (st.qm.cpu().numpy() == qm[:n]).mean() > 0.9999 and (st.qv.cpu().numpy() == qv[:n]).mean() > 0.9999
    assert np.abs(pd.cpu().numpy() - p[:n]).max() <= 1e-6 * np.abs(p).max()
    assert torch.equal(wb, pd.bfloat16())  # the fused bf16 working copy = RNE cast of the updated parameters
    # it is an Adam step: against fp32 AdamW the parameters move the same way (codes cost a few % of the update)
    m, v = st.dequant()
    assert torch.isfinite(m).all() and (v >= 0).all()


def test_adamw8bit_per_tensor_vs_restatement(cuda):
    """pso_adamw8bit_step_blocks: bitsandbytes' per-tensor semantics on a flat buffer of mixed-size tensors (T:428-448,
    ADVICE r3): blocks restart at every tensor, tensors under 4096 elements keep 32-bit state, alignment pads between
    tensors are never touched, and non-finite gradient elements (injected at step 3) leave the parameter and its state
    unchanged -- against oracle/adam8bit.adamw8bit_step_tensors over 5 steps (parity unpinned: no bitsandbytes)."""
    import numpy as np
    from oracle import adam8bit as O
    from pairwise_sample_optimization_amd import kernels as K_
    sizes = [5000, 1000, 4096, 4095, 20480, 64, 2049, 320]
    segs, off = [], 0
    for k in sizes:
        segs.append((off, k))
        off += -(-k // 64) * 64  # 64-element slots, as FullGradState lays the UNet parameters out
    n = off
    g_ = np.random.default_rng(4)
    p = (g_.standard_normal(n) * 0.02).astype(np.float32)
    pads = np.ones(n, bool)
    for o, k in segs:
        pads[o:o + k] = False
    f32 = lambda x: float(np.float32(x))
    lr, b1, b2, eps, wd = f32(1e-3), f32(0.9), f32(0.999), f32(1e-8), f32(1e-2)
    pd = torch.tensor(p, device=cuda)
    wb = torch.zeros(n, device=cuda, dtype=torch.bfloat16)
    st = K_.Adam8State(n, cuda, segments=segs)
    assert st.nblk == sum(-(-k // 2048) for k in sizes)
    ost = {}
    p0 = p.copy()
    for step in range(1, 6):
        # per-tensor gradient scales 1e-4 .. 1: a shared absmax would round the small tensors' state to code 0
        gr = np.zeros(n, np.float32)
        for i, (o, k) in enumerate(segs):
            gr[o:o + k] = g_.standard_normal(k).astype(np.float32) * np.float32(10.0 ** (-(i % 5)))
        if step == 3:
            gr[[3, 5001, 7000, 12000]] = [np.nan, np.inf, -np.inf, np.nan]
        gr[pads] = 7.0  # never read: the pads are no block's
        gd = torch.tensor(gr, device=cuda)
        # odd steps also zero the gradient they read (pso_adamw8bit_step_blocks_zero_grad, optimizer.zero_grad T:861)
        zg = K_.adamw8bit_step(pd, gd, st, lr, (b1, b2), eps, wd, step, out_bf16=wb, zero_grad=step % 2 == 1)
        gk = gd.cpu().numpy()
        assert zg == (step % 2 == 1) and np.array_equal(gk[pads], gr[pads])
        assert (not (gk[~pads] != 0).any()) if zg else np.array_equal(gk, gr, equal_nan=True)
        p = O.adamw8bit_step_tensors(p, gr, segs, ost, lr, b1, b2, eps, wd, step)
    torch.cuda.synchronize()
    pk = pd.cpu().numpy()
    assert np.isfinite(pk).all()
    assert np.array_equal(pk[pads], p0[pads])                       # pads untouched
    assert np.abs(pk - p).max() <= 1e-6 * np.abs(p).max()
    qm, qv = st.qm.cpu().numpy(), st.qv.cpu().numpy()
    am, av = st.am.cpu().numpy(), st.av.cpu().numpy()
    m32, v32 = st.m32.cpu().numpy(), st.v32.cpu().numpy()
    for b, (o, k, so, _) in enumerate(st.rows):
        seg_off = max(so_ for so_, _ in segs if so_ <= o)
        ref = ost[seg_off]
        if so >= 0:  # 32-bit tensor (one block: k < 4096 < 2 * 2048 only when k <= 2048; else two)
            r0 = o - seg_off
            assert np.allclose(m32[so:so + k], ref["m32"][r0:r0 + k], rtol=1e-6, atol=1e-12)
            assert np.allclose(v32[so:so + k], ref["v32"][r0:r0 + k], rtol=1e-6, atol=1e-14)
        else:
            bi = (o - seg_off) // 2048
            assert am[b] == ref["am"][bi] and av[b] == ref["av"][bi], (b, o)
            r0 = o - seg_off
            assert (qm[o:o + k] == ref["qm"][r0:r0 + k]).mean() > 0.999
            assert (qv[o:o + k] == ref["qv"][r0:r0 + k]).mean() > 0.999
    keep = torch.tensor(~pads, device=cuda)
    assert torch.equal(wb[keep], pd.bfloat16()[keep])  # the fused bf16 working copy (pads: never written)
