"""Thin Python wrappers over the libpso_amd C-ABI (one function per entry point of include/pso_amd.h).

Tensors are plain torch device tensors used as memory; every computation happens in the HIP library.  Activations
are channels-last bf16: linear inputs are [tokens, C] (any 2-D row-strided view), images are NHWC [B, H, W, C].
There is no CPU / eager fallback: a missing library or a host tensor raises PsoLibError.
"""
import ctypes
import os

import torch

from . import _lib
from ._lib import check, lib, ptr, require_cuda, stream_ptr, dtype_code, PSO_BF16, PSO_F32

CONV_NORMAL, CONV_UP2, CONV_T2 = 1, 2, 3
BF16 = torch.bfloat16

# Optional per-launch accounting of the MFMA GEMM/conv kernel (bench.py roofline): list of (flops, ev0, ev1)
PROFILE = None


def _prof_begin():
    if PROFILE is None:
        return None
    e0 = torch.cuda.Event(enable_timing=True)
    e0.record()
    return e0


def _prof_end(e0, flops, nbytes=0.0, tag=None):
    """nbytes: algorithmic HBM bytes of the launch (every operand read once, the output written once).  Each record
    carries the launched kernel's rocprofv3 name (pso_last_kernel) so timings can be grouped per kernel."""
    if e0 is not None:
        e1 = torch.cuda.Event(enable_timing=True)
        e1.record()
        PROFILE.append((flops, nbytes, e0, e1, tag, lib().pso_last_kernel().decode()))


class SideStream:
    """Second HIP stream for launches off the critical path (the LoRA weight gradients of the backward): they only
    accumulate into the flat fp32 grad buffer, so they can run beside the next input-gradient GEMMs and fill the CU
    slots those leave (the dW kernels are latency-bound HBM streams).  `launch` orders the side stream after
    everything the main stream has issued so far, and ties every tensor the launches read to the side stream
    (caching-allocator record_stream), so no buffer is reused before they finish; `join` makes the main stream wait
    for all of them (before the optimizer reads the grads).  Opt-in: PSO_SIDE_STREAM=1."""

    enabled = os.environ.get("PSO_SIDE_STREAM", "0") == "1"  # measured neutral on the C2 step (31.35 vs 31.44 imgs/s)

    def __init__(self, enabled=None):
        """enabled: None = the class default (PSO_SIDE_STREAM); the full-UNet backward turns it on for its weight
        gradients (PSO_FULL_SIDE_STREAM=0 keeps them in line)."""
        self.on = SideStream.enabled if enabled is None else enabled
        self.s = None
        self.pending = False

    def launch(self, fn, *tensors):
        if not (self.on and SideStream.enabled_any):
            fn()
            return
        main = torch.cuda.current_stream()
        if self.s is None:
            # ONE side stream per device for the process: the caching allocator keeps freed blocks per stream, so a
            # fresh pool stream per step (torch hands them out round-robin) could never reuse the previous step's
            # side-stream buffers -- every step allocated anew until the cache was released (a device sync: a 9 ms
            # idle gap per C3 step)
            self.s = SideStream._streams.get(main.device)
            if self.s is None:
                self.s = SideStream._streams[main.device] = torch.cuda.Stream(device=main.device)
        self.s.wait_stream(main)
        with torch.cuda.stream(self.s):
            fn()
        for t in tensors:
            t.record_stream(self.s)
        self.pending = True

    def join(self):
        if self.pending:
            torch.cuda.current_stream().wait_stream(self.s)
            self.pending = False


SideStream._streams = {}
SideStream.enabled_any = True  # False: every launch in line (profiling with serial event timing, bench.roofline)


def _row_stride(t):
    assert t.dim() == 2 and t.stride(1) == 1, "operand must be a 2-D view with contiguous rows"
    return t.stride(0)


_GEMM_WS = {}  # (M, N, K1, K2) -> pso_gemm_ws_bytes of the current dispatch variant


def gemm_set_variant(v):
    """pso_gemm_set_variant (A/B knob of the GEMM dispatch, TOOLS build only: PSO_LIB=knobs) + a flush of the
    workspace-size cache: the split-K plan, and so the workspace a product needs, depends on the variant.
    Variant 0 is the automatic dispatch, which the product library always runs: a no-op there."""
    if not _lib.KNOBS and int(v) == 0:
        return
    _lib.require_knobs("pso_gemm_set_variant")
    lib().pso_gemm_set_variant(int(v))
    _GEMM_WS.clear()


def gemm(a, w, *, bias=None, resid=None, a2=None, w2=None, alpha=1.0, rowbias=None, rows_per_group=1, out=None,
         out_dtype=BF16, accumulate=False, tail_group_n=0, tail_rows=0):
    """out[M,N] = alpha*(a @ w^T + a2 @ w2^T) + bias + rowbias[m // rows_per_group] + resid.
    tail_group_n > 0: output column group j uses a2[:, j*K2:(j+1)*K2] with w2 [N, K2].
    tail_rows > 0: only the first tail_rows rows take the a2 term (a2 has tail_rows rows)."""
    require_cuda(a, w)
    M, K1 = a.shape
    N = w.shape[0]
    assert w.shape[1] == K1 and a.dtype == BF16 and w.dtype == BF16
    K2 = 0
    if a2 is not None:
        K2 = w2.shape[1]
        assert w2.shape[0] == N and a2.shape[0] == (tail_rows if tail_rows else M)
        assert a2.shape[1] == (K2 * (N // tail_group_n) if tail_group_n else K2)
    if out is None:
        out = torch.empty((M, N), device=a.device, dtype=out_dtype)
    key = (M, N, K1, K2)
    wsb = _GEMM_WS.get(key)
    if wsb is None:
        wsb = _GEMM_WS[key] = int(lib().pso_gemm_ws_bytes(M, N, K1, K2))
    args = (M, N, ptr(a), _row_stride(a), K1, ptr(w), _row_stride(w),
            ptr(a2), _row_stride(a2) if a2 is not None else 0, K2,
            ptr(w2), _row_stride(w2) if w2 is not None else 0,
            float(alpha), ptr(bias), ptr(rowbias), rowbias.stride(0) if rowbias is not None else 0,
            int(rows_per_group), ptr(resid), _row_stride(resid) if resid is not None else 0,
            ptr(out), _row_stride(out), dtype_code(out), int(accumulate), int(tail_group_n), int(tail_rows))
    e0 = _prof_begin()
    if wsb:  # small M x N, long K: deterministic split-K through a workspace (pso_gemm_ws)
        ws = torch.empty(wsb, device=a.device, dtype=torch.uint8)
        check(lib().pso_gemm_ws(*args, ptr(ws), wsb, stream_ptr()), "pso_gemm_ws")
    else:
        check(lib().pso_gemm(*args, stream_ptr()), "pso_gemm")
    _prof_end(e0, 2.0 * M * N * K1 + 2.0 * (tail_rows if 0 < tail_rows < M else M) * N * K2,
              2.0 * (M * (K1 + (a2.shape[1] if a2 is not None else 0)) + N * (K1 + K2)) + out.element_size() * M * N,
              ("gemm", M, N, K1, K2, tail_group_n, out.dtype == torch.float32))
    return out


def gemm_batched(a, w, alpha=1.0, out=None, out_dtype=BF16):
    """out[z] = alpha * a[z] @ w[z]^T for a [Z, M, K], w [Z, N, K] (bf16, rows contiguous) -> [Z, M, N]."""
    require_cuda(a, w)
    Z, M, Kd = a.shape
    N = w.shape[1]
    assert w.shape[0] == Z and w.shape[2] == Kd and a.dtype == BF16 and w.dtype == BF16
    assert a.stride(2) == 1 and w.stride(2) == 1
    if out is None:
        out = torch.empty((Z, M, N), device=a.device, dtype=out_dtype)
    assert out.stride(2) == 1 and tuple(out.shape) == (Z, M, N)
    e0 = _prof_begin()
    check(lib().pso_gemm_batched(Z, M, N, Kd, ptr(a), a.stride(1), a.stride(0), ptr(w), w.stride(1), w.stride(0),
                                 float(alpha), ptr(out), out.stride(1), out.stride(0), dtype_code(out), stream_ptr()),
          "pso_gemm_batched")
    _prof_end(e0, 2.0 * Z * M * N * Kd, 2.0 * Z * (M * Kd + N * Kd) + out.element_size() * Z * M * N,
              ("gemm_batched", Z, M, N, Kd))
    return out


def gemm_grouped_skinny(a, w, groups, out=None, alpha=1.0):
    """Block-diagonal skinny product: out[:, g*N:(g+1)*N] = alpha * a[:, g*K:(g+1)*K] @ w[:, g*K:(g+1)*K]^T, bf16."""
    M, KG = a.shape
    N = w.shape[0]
    Kg = KG // groups
    assert w.shape[1] == KG and KG == Kg * groups
    if out is None:
        out = torch.empty((M, groups * N), device=a.device, dtype=BF16)
    e0 = _prof_begin()
    check(lib().pso_gemm_skinny_grouped(M, N, Kg, ptr(a), _row_stride(a), ptr(w), _row_stride(w), float(alpha),
                                        ptr(out), _row_stride(out), int(groups), stream_ptr()), "pso_gemm_skinny_grouped")
    _prof_end(e0, 2.0 * M * N * KG, 2.0 * (M * KG + N * KG + M * N * groups), ("gemm_grouped", M, N, KG, groups))
    return out


_GEGLU_IDX = {}


def geglu_interleave_index(F, device=None):
    """Row order of the GEGLU proj weight for the fused epilogue: per 32 outputs, [h rows 32 | gate rows 32].
    Cached per (F, device): the full-UNet backward and every re-prepare ask for it again."""
    key = (F, str(device))
    if key not in _GEGLU_IDX:
        g = torch.arange(F // 32, device=device).view(-1, 1)
        j = torch.arange(32, device=device).view(1, -1)
        _GEGLU_IDX[key] = torch.cat([g * 32 + j, F + g * 32 + j], 1).reshape(-1)
    return _GEGLU_IDX[key]


def gemm_geglu(a, w_int, b_int, out_pre=None, out=None, pre_rows=0):
    """diffusers GEGLU with the activation in the GEMM epilogue: out [M, F] = h * gelu(gate) where
    [h | gate] = a @ W^T + b, given the interleaved weight / bias (geglu_interleave_index).  out_pre (optional)
    [pre_rows or M, 2F] receives the interleaved pre-activation of the first pre_rows rows for the backward."""
    M, Kd = a.shape
    N = w_int.shape[0]
    if out is None:
        out = torch.empty((M, N // 2), device=a.device, dtype=BF16)
    e0 = _prof_begin()
    check(lib().pso_gemm_geglu(M, N, ptr(a), _row_stride(a), Kd, ptr(w_int), _row_stride(w_int), ptr(b_int),
                               ptr(out), _row_stride(out), ptr(out_pre),
                               _row_stride(out_pre) if out_pre is not None else 0, int(pre_rows), stream_ptr()),
          "pso_gemm_geglu")
    _prof_end(e0, 2.0 * M * N * Kd, 2.0 * (M * Kd + N * Kd + M * N // 2 + (M * N if out_pre is not None else 0)),
              ("gemm_geglu", M, N, Kd, out_pre is not None))
    return out


def gemm_geglu_bwd(a, w, pre, out=None):
    """Input gradient of the fused GEGLU: dout = a @ w^T ([M, F], F = w rows), pre = interleaved pre-activation
    [M, 2F]; returns the interleaved [dout*gelu(g) | dout*h*gelu'(g)] [M, 2F]."""
    M, Kd = a.shape
    N = w.shape[0]
    if out is None:
        out = torch.empty((M, 2 * N), device=a.device, dtype=BF16)
    e0 = _prof_begin()
    check(lib().pso_gemm_geglu_bwd(M, N, ptr(a), _row_stride(a), Kd, ptr(w), _row_stride(w), ptr(pre),
                                   _row_stride(pre), ptr(out), _row_stride(out), stream_ptr()), "pso_gemm_geglu_bwd")
    _prof_end(e0, 2.0 * M * N * Kd, 2.0 * (M * Kd + N * Kd + 4 * M * N), ("gemm_geglu_bwd", M, N, Kd))
    return out


def quant_rows_fp8(x, q=None, e=None):
    """Row-wise OCP e4m3 quantisation with a power-of-two scale per row: returns (q uint8 [M, K], e uint8 [M]) with
    x[m] ~= e4m3(q[m]) * 2^(e[m] - 127) (pso_quant_rows_fp8; activations per token, weights per output channel)."""
    require_cuda(x)
    assert x.dtype == BF16 and x.dim() == 2
    M, Kd = x.shape
    if q is None:
        q = torch.empty((M, Kd), device=x.device, dtype=torch.uint8)
    if e is None:
        e = torch.empty((M,), device=x.device, dtype=torch.uint8)
    check(lib().pso_quant_rows_fp8(M, Kd, ptr(x), _row_stride(x), ptr(q), _row_stride(q), ptr(e), stream_ptr()),
          "pso_quant_rows_fp8")
    return q, e


def dequant_rows_fp8(q, e):
    """Host-side view of quant_rows_fp8's output as fp32 (tests / references only)."""
    return q.view(torch.float8_e4m3fn).float() * torch.exp2(e.float() - 127.0)[:, None]


FP8_LAUNCHES = [0]  # pso_gemm_fp8 calls issued by this process (tests assert that an fp8 path really ran)


def gemm_fp8(a, w, *, a2=None, w2=None, tail_rows=0, tail_group_n=0, alpha=1.0, bias=None, resid=None, out=None,
             geglu=False, out_pre=None, pre_rows=0):
    """fp8 forward GEMM (pso_gemm_fp8): a = (q [M, K], e [M]) and w = (q [N, K], e [N]) from quant_rows_fp8, likewise
    the LoRA tail a2 [tail_rows or M, K2*groups] / w2 [N, K2].  Plain: out [M, N] = bf16(alpha*acc + bias) (+ resid);
    geglu: the GEGLU epilogue of gemm_geglu on interleaved weight rows (out [M, N/2], out_pre rows < pre_rows)."""
    (aq, ae), (wq, we) = a, w
    require_cuda(aq, wq)
    FP8_LAUNCHES[0] += 1
    M, Kd = aq.shape
    N = wq.shape[0]
    assert wq.shape[1] == Kd and aq.dtype == torch.uint8 and wq.dtype == torch.uint8
    K2, tr = 0, (tail_rows if 0 < tail_rows < M else M)
    if a2 is not None:
        K2 = w2[0].shape[1]
        assert a2[0].shape[0] == tr and w2[0].shape[0] == N
    if out is None:
        out = torch.empty((M, N // 2 if geglu else N), device=aq.device, dtype=BF16)
    e0 = _prof_begin()
    check(lib().pso_gemm_fp8(1 if geglu else 0, M, N, Kd, ptr(aq), _row_stride(aq), ptr(ae), ptr(wq), _row_stride(wq),
                             ptr(we), ptr(a2[0]) if a2 is not None else None,
                             _row_stride(a2[0]) if a2 is not None else 0, K2,
                             ptr(a2[1]) if a2 is not None else None, ptr(w2[0]) if a2 is not None else None,
                             _row_stride(w2[0]) if a2 is not None else 0, ptr(w2[1]) if a2 is not None else None,
                             tr, int(tail_group_n), float(alpha), ptr(bias), ptr(resid),
                             _row_stride(resid) if resid is not None else 0, ptr(out), _row_stride(out),
                             ptr(out_pre), _row_stride(out_pre) if out_pre is not None else 0, int(pre_rows),
                             stream_ptr()), "pso_gemm_fp8")
    _prof_end(e0, 2.0 * M * N * Kd + 2.0 * tr * N * K2, 1.0 * (M * Kd + N * Kd) + 2.0 * M * N,
              ("gemm_fp8", M, N, Kd, K2, tail_group_n, geglu))
    return out


TN_RANKS = (16, 32, 64, 96)  # rank widths of the streaming TN kernel (grouped form needs one of them)


def gemm_tn(a, b, out, alpha=1.0, group=0, split_ws=True):
    """out[I,J] (f32, accumulated) += alpha * a^T @ b  with a [M,I], b [M,J] (row-strided views).
    group > 0 (block-diagonal, fused q/k/v adapters): out [I, r] with r = J * group / I; column block
    a[:, g*group:(g+1)*group] pairs with b[:, g*r:(g+1)*r]."""
    M, I = a.shape
    J = b.shape[1]
    r = J * group // I if group else J
    assert b.shape[0] == M and out.shape == (I, r) and out.dtype == torch.float32
    if split_ws and TnRankQueue.deterministic and _tn_rank_form(a, b, group) is not None:
        q = TnRankQueue()  # a rank-r product (grouped or not): the ordered workspace form, issued at once
        q.add(a, b, out, alpha, group)
        q.flush()
        return out
    e0 = _prof_begin()
    wsb = lib().pso_gemm_tn_ws_bytes(M, I, J) if group == 0 and split_ws else 0
    if wsb:  # full-weight gradient with few 128 x 128 tiles: split rows, ordered reduction through a workspace
        ws = torch.empty(wsb, device=a.device, dtype=torch.uint8)
        check(lib().pso_gemm_tn_ws(M, I, J, ptr(a), _row_stride(a), ptr(b), _row_stride(b), float(alpha), ptr(out),
                                   _row_stride(out), ptr(ws), wsb, stream_ptr()), "pso_gemm_tn_ws")
    else:
        check(lib().pso_gemm_tn_grouped(M, I, J, ptr(a), _row_stride(a), ptr(b), _row_stride(b), float(alpha),
                                        ptr(out), _row_stride(out), int(group), stream_ptr()), "pso_gemm_tn")
    _prof_end(e0, 2.0 * M * I * r, 2.0 * M * (I + J) + 8.0 * I * r, ("gemm_tn", M, I, J, group))
    return out


def gemm_tn_geglu(df, x, out, alpha=1.0):
    """out[F2, J] (f32, accumulated) += alpha * df^T @ x with df [M, F2] in the GEGLU interleave (geglu_interleave_index)
    and out in the natural [h | gate] row order: the full-UNet ff.net.0.proj weight gradient without a transient
    interleaved matrix (pso_gemm_tn_geglu)."""
    M, F2 = df.shape
    J = x.shape[1]
    assert x.shape[0] == M and out.shape == (F2, J) and out.dtype == torch.float32
    e0 = _prof_begin()
    check(lib().pso_gemm_tn_geglu(M, F2, J, ptr(df), _row_stride(df), ptr(x), _row_stride(x), float(alpha), ptr(out),
                                  _row_stride(out), stream_ptr()), "pso_gemm_tn_geglu")
    _prof_end(e0, 2.0 * M * F2 * J, 2.0 * M * (F2 + J) + 8.0 * F2 * J, ("gemm_tn", M, F2, J, 0))
    return out


def _tn_rank_form(a, b, group):
    """(key, x, u, R, group_c) of a TN product gemm_tn(a, b, ...) that the rank-r streaming kernel takes, else None:
    x the >= 128-wide side, u the rank-R side, key = (R, out_jc)."""
    I, J = a.shape[1], b.shape[1]
    r = J * group // I if group else J
    rk = lambda v: v in TN_RANKS
    if I % 128 == 0 and (rk(J) if group == 0 else (group % 128 == 0 and I % group == 0 and rk(r))):
        return (r, 0), a, b, r, group
    if J % 128 == 0 and group == 0 and rk(I):
        return (I, 1), b, a, I, 0
    return None


class TnRankQueue:
    """Deferred LoRA weight-gradient products (gemm_tn calls whose one side is a rank-16/32/64/96 projection).  The
    backward records them as it goes (add) and issues them per gradient unit (flush) as ONE pso_gemm_tn_rank_batch
    launch per (rank, orientation): the ~700 rank-r products of a C2 step become a few dozen launches, each with
    enough workgroups to fill the chip, and fewer f32 atomics per byte streamed.  The queue holds a reference to
    every operand until its launch, so the caching allocator cannot recycle them early.  Products the rank kernel
    does not take run at once through gemm_tn (same arithmetic either way)."""

    # PSO_TN_DETERMINISTIC=0 selects the f32-atomic epilogue (A/B knob); the default is the ordered workspace form
    deterministic = os.environ.get("PSO_TN_DETERMINISTIC", "1") != "0"

    def __init__(self):
        self.pending = {}  # (R, out_jc) -> [(problem, operands, flop, bytes)]

    def add(self, a, b, out, alpha=1.0, group=0):
        M, I = a.shape
        J = b.shape[1]
        r = J * group // I if group else J
        assert b.shape[0] == M and out.shape == (I, r) and out.dtype == torch.float32
        form = _tn_rank_form(a, b, group)
        if form is None:
            return gemm_tn(a, b, out, alpha, group)
        key, x, u, R, gc = form
        require_cuda(x, u, out)
        prob = _lib.PsoTnRankProblem(ptr(x), _row_stride(x), ptr(u), _row_stride(u), ptr(out), _row_stride(out),
                                     M, x.shape[1], gc, float(alpha))
        self.pending.setdefault(key, []).append((prob, (x, u, out), 2.0 * M * I * r, 2.0 * M * (I + J) + 8.0 * I * r))
        return out

    def flush(self):
        for (R, ojc), items in self.pending.items():
            arr = (_lib.PsoTnRankProblem * len(items))(*[it[0] for it in items])
            e0 = _prof_begin()
            if TnRankQueue.deterministic:
                # ordered reduction through a workspace (no f32 atomics): bit-identical runs and hipGraph replays
                wsb = lib().pso_gemm_tn_rank_batch_ws_bytes(R, ojc, len(items), arr)
                ws = torch.empty(max(int(wsb), 16), device=items[0][1][2].device, dtype=torch.uint8)
                check(lib().pso_gemm_tn_rank_batch_ws(R, ojc, len(items), arr, ptr(ws), ws.numel(), stream_ptr()),
                      "pso_gemm_tn_rank_batch_ws")
            else:
                check(lib().pso_gemm_tn_rank_batch(R, ojc, len(items), arr, stream_ptr()), "pso_gemm_tn_rank_batch")
            _prof_end(e0, sum(it[2] for it in items), sum(it[3] for it in items), ("gemm_tn_batch", R, ojc, len(items)))
        self.pending = {}


def conv2d(x, weight, *, x2=None, mode=CONV_NORMAL, stride=1, pad=None, out_hw=None, bias=None, rowbias=None,
           resid=None, a2=None, w2=None, alpha=1.0, out=None, out_dtype=BF16, accumulate=False):
    """NHWC implicit-GEMM conv.  x [B,H,W,C1] (+ x2 [B,H,W,C2] concatenated on channels); weight [Cout,ks,ks,C1+C2].
    Returns [B,Ho,Wo,Cout]."""
    require_cuda(x, weight)
    B, H, W, C1 = x.shape
    C2 = x2.shape[3] if x2 is not None else 0
    Cout, ks, ks2, Ct = weight.shape
    assert ks == ks2 and Ct == C1 + C2 and x.is_contiguous() and weight.is_contiguous()
    if pad is None:
        pad = ks // 2
    if out_hw is None:
        if mode == CONV_UP2:
            out_hw = (2 * H, 2 * W)
        elif mode == CONV_T2:
            out_hw = (2 * H, 2 * W)
        else:
            out_hw = ((H + 2 * pad - ks) // stride + 1, (W + 2 * pad - ks) // stride + 1)
    Ho, Wo = out_hw
    if out is None:
        out = torch.empty((B, Ho, Wo, Cout), device=x.device, dtype=out_dtype)
    K2 = a2.shape[1] if a2 is not None else 0
    o2 = out.view(B * Ho * Wo, -1) if out.is_contiguous() else None
    ldo = Cout if o2 is None else o2.stride(0)
    key = ("conv", B, Ho, Wo, Cout, ks * ks * Ct, K2)
    wsb = _GEMM_WS.get(key)
    if wsb is None:
        wsb = _GEMM_WS[key] = int(lib().pso_conv2d_ws_bytes(B, Ho, Wo, Cout, ks * ks * Ct, K2))
    args = (mode, B, ptr(x), C1, ptr(x2), C2, H, W, Ho, Wo, ks, stride, pad, ptr(weight), Cout,
            ptr(a2), _row_stride(a2) if a2 is not None else 0, K2,
            ptr(w2), _row_stride(w2) if w2 is not None else 0, float(alpha), ptr(bias),
            ptr(rowbias), rowbias.stride(0) if rowbias is not None else 0,
            ptr(resid), Cout if resid is not None else 0, ptr(out), ldo, dtype_code(out), int(accumulate))
    e0 = _prof_begin()
    if wsb:  # small output, long reduction (bs = 1 backward): deterministic split-K through a workspace
        ws = torch.empty(wsb, device=x.device, dtype=torch.uint8)
        check(lib().pso_conv2d_ws(*args, ptr(ws), wsb, stream_ptr()), "pso_conv2d_ws")
    else:
        check(lib().pso_conv2d(*args, stream_ptr()), "pso_conv2d")
    _prof_end(e0, 2.0 * B * Ho * Wo * Cout * (ks * ks * (C1 + C2) + K2),
              2.0 * (B * H * W * (C1 + C2) + Cout * ks * ks * (C1 + C2) + B * Ho * Wo * K2 + Cout * K2)
              + out.element_size() * B * Ho * Wo * Cout, ("conv", mode, B, H, W, C1, C2, Cout, ks, stride, K2))
    return out


# ------------------------------------------------------------------------------------------------------------------
# PSO step / loss
# ------------------------------------------------------------------------------------------------------------------
def step_logprob(mode, sample, eps, coef, prev=None, noise=None, noise_shared=False):
    """One scheduler step + Gaussian log-prob.  sample/prev/noise fp32 [B, ...]; eps fp32|bf16; coef [B, 8]."""
    require_cuda(sample, eps, coef, prev, noise)
    B = sample.shape[0]
    n = sample[0].numel()
    sample = sample.contiguous()
    eps = eps.contiguous()
    lp = torch.empty(B, device=sample.device, dtype=torch.float32)
    prev_out = None if prev is not None else torch.empty_like(sample, dtype=torch.float32)
    ws_bytes = lib().pso_step_logprob_ws_bytes(B, n)
    ws = torch.empty(ws_bytes, device=sample.device, dtype=torch.uint8)
    check(lib().pso_step_logprob(mode, B, n, ptr(sample), ptr(eps), dtype_code(eps),
                                 ptr(prev.contiguous()) if prev is not None else None,
                                 ptr(noise.contiguous()) if noise is not None else None, int(noise_shared),
                                 ptr(coef.contiguous()), ptr(prev_out), ptr(lp), ptr(ws), ws_bytes, stream_ptr()),
          "pso_step_logprob")
    return (prev if prev is not None else prev_out), lp


def pair_loss_ws(P, n, device):
    return torch.empty(lib().pso_pair_loss_ws_bytes(P, n), device=device, dtype=torch.uint8)


def _check_pair_operands(x, x_prev, eps_pol, coef, pref, eps_ref=None):
    """Shape / dtype / layout contract of pso_pair_loss_fwd/bwd (the C-ABI reads raw pointers): x, x_prev fp32
    contiguous [2P, ...]; eps in one dtype (fp32 or bf16), contiguous, same shape; coef fp32 [2P, 8]; pref fp32 [P, 2]."""
    require_cuda(x, x_prev, eps_pol, eps_ref, coef, pref)
    if x.dtype != torch.float32 or x_prev.dtype != torch.float32:
        raise _lib.PsoLibError("pair loss: x / x_prev must be float32")
    if x.shape != x_prev.shape or x.shape != eps_pol.shape or (eps_ref is not None and eps_ref.shape != x.shape):
        raise _lib.PsoLibError(f"pair loss: shape mismatch x {tuple(x.shape)} x_prev {tuple(x_prev.shape)} "
                               f"eps_pol {tuple(eps_pol.shape)}" +
                               (f" eps_ref {tuple(eps_ref.shape)}" if eps_ref is not None else ""))
    if eps_ref is not None and eps_ref.dtype != eps_pol.dtype:
        raise _lib.PsoLibError(f"pair loss: eps_pol {eps_pol.dtype} and eps_ref {eps_ref.dtype} differ")
    dtype_code(eps_pol)
    if x.shape[0] % 2:
        raise _lib.PsoLibError("pair loss: batch must be 2P images (pair p, member k at row 2p + k)")
    P = x.shape[0] // 2
    if coef.dtype != torch.float32 or tuple(coef.shape) != (2 * P, _lib.COEF_STRIDE):
        raise _lib.PsoLibError(f"pair loss: coef must be float32 [{2 * P}, {_lib.COEF_STRIDE}]")
    if pref.dtype != torch.float32 or tuple(pref.shape) != (P, 2):
        raise _lib.PsoLibError(f"pair loss: pref must be float32 [{P}, 2]")
    for t in (x, x_prev, eps_pol, eps_ref, coef, pref):
        if t is not None and not t.is_contiguous():
            raise _lib.PsoLibError("pair loss: operands must be contiguous")


def pair_loss_fwd(mode, x, x_prev, eps_pol, eps_ref, coef, pref, beta, clip_eps, ws):
    _check_pair_operands(x, x_prev, eps_pol, coef, pref, eps_ref)
    P = x.shape[0] // 2
    n = x[0].numel()
    lp = torch.empty((2 * P, 2), device=x.device, dtype=torch.float32)
    loss = torch.empty((), device=x.device, dtype=torch.float32)
    check(lib().pso_pair_loss_fwd(mode, P, n, ptr(x), ptr(x_prev), ptr(eps_pol), ptr(eps_ref), dtype_code(eps_pol),
                                  ptr(coef), ptr(pref), float(beta), float(clip_eps), ptr(lp), ptr(loss), ptr(ws),
                                  ws.numel(), stream_ptr()), "pso_pair_loss_fwd")
    return loss, lp


def pair_loss_bwd(mode, x, x_prev, eps_pol, coef, pref, beta, clip_eps, ws, grad_out=None, grad_scale=1.0,
                  out_dtype=BF16):
    _check_pair_operands(x, x_prev, eps_pol, coef, pref)
    P = x.shape[0] // 2
    n = x[0].numel()
    deps = torch.empty(eps_pol.shape, device=x.device, dtype=out_dtype)
    check(lib().pso_pair_loss_bwd(mode, P, n, ptr(x), ptr(x_prev), ptr(eps_pol), dtype_code(eps_pol), ptr(coef),
                                  ptr(pref), float(beta), float(clip_eps), ptr(grad_out), float(grad_scale),
                                  ptr(deps), dtype_code(deps), ptr(ws), ws.numel(), stream_ptr()),
          "pso_pair_loss_bwd")
    return deps


def pair_loss_from_lp(mode, lp_pol, lp_ref, pref, beta, clip_eps):
    """T:844-850 on given log-probs lp_pol / lp_ref / pref [P, 2] fp32 -> (loss, dL/d lp_pol [P, 2])."""
    require_cuda(lp_pol, lp_ref, pref)
    P = lp_pol.shape[0]
    for t in (lp_pol, lp_ref, pref):
        assert t.dtype == torch.float32 and tuple(t.shape) == (P, 2)
    loss = torch.empty((), device=lp_pol.device, dtype=torch.float32)
    dlp = torch.empty((P, 2), device=lp_pol.device, dtype=torch.float32)
    check(lib().pso_pair_loss_from_lp(mode, P, ptr(lp_pol.contiguous()), ptr(lp_ref.contiguous()),
                                      ptr(pref.contiguous()), float(beta), float(clip_eps), ptr(loss), ptr(dlp),
                                      stream_ptr()), "pso_pair_loss_from_lp")
    return loss, dlp


DB_SIGMOID, DB_HINGE = 0, 1  # PSO_DB_* ("pso", "pso_db")


def db_loss_ws(B, n, device):
    return torch.empty(lib().pso_db_loss_ws_bytes(B, n), device=device, dtype=torch.uint8)


def db_loss_fwd(loss_type, eps, noisy, x0, sigma, beta, neg_defactor, prior_w, ws, eps_ref=None):
    """DreamBooth PSO loss (DB:1847-1935).  eps [2B,...] (instance rows first, negatives second), noisy / x0 fp32 of
    the same shape, sigma fp32 [2B].  Returns (loss, per-image losses [2B or 4B], logits [B])."""
    B2 = eps.shape[0]
    n = eps[0].numel()
    B = B2 // 2
    losses = torch.empty((2 * B2 if eps_ref is not None else B2,), device=eps.device, dtype=torch.float32)
    logits = torch.empty((B,), device=eps.device, dtype=torch.float32)
    loss = torch.empty((), device=eps.device, dtype=torch.float32)
    check(lib().pso_db_loss_fwd(loss_type, B, n, ptr(eps), ptr(eps_ref), dtype_code(eps), ptr(noisy), ptr(x0),
                                ptr(sigma), float(beta), float(neg_defactor), float(prior_w), ptr(losses), ptr(logits),
                                ptr(loss), ptr(ws), ws.numel(), stream_ptr()), "pso_db_loss_fwd")
    return loss, losses, logits


def db_loss_bwd(loss_type, eps, noisy, x0, sigma, beta, neg_defactor, prior_w, ws, grad_out=None, grad_scale=1.0,
                out_dtype=BF16):
    B = eps.shape[0] // 2
    n = eps[0].numel()
    deps = torch.empty(eps.shape, device=eps.device, dtype=out_dtype)
    check(lib().pso_db_loss_bwd(loss_type, B, n, ptr(eps), dtype_code(eps), ptr(noisy), ptr(x0), ptr(sigma),
                                float(beta), float(neg_defactor), float(prior_w), ptr(grad_out), float(grad_scale),
                                ptr(deps), dtype_code(deps), ptr(ws), ws.numel(), stream_ptr()), "pso_db_loss_bwd")
    return deps


# ------------------------------------------------------------------------------------------------------------------
# Norms
# ------------------------------------------------------------------------------------------------------------------
def group_norm_fwd(x, gamma, beta, groups, eps, silu):
    """x NHWC [B,H,W,C] (or [B,HW,C]) bf16 -> (y, stats[B,G,2])."""
    B, C = x.shape[0], x.shape[-1]
    HW = x.numel() // (B * C)
    y = torch.empty_like(x)
    stats = torch.empty((B, groups, 2), device=x.device, dtype=torch.float32)
    wsb = lib().pso_group_norm_ws_bytes(B, HW, C)
    ws = torch.empty(wsb, device=x.device, dtype=torch.uint8)
    check(lib().pso_group_norm_fwd(B, HW, C, groups, float(eps), ptr(x), ptr(gamma), ptr(beta), int(silu), ptr(y),
                                   ptr(stats), ptr(ws), wsb, stream_ptr()), "pso_group_norm_fwd")
    return y, stats


def group_norm_bwd(x, dy, stats, gamma, beta, silu, dadd=None, dgamma=None, dbeta=None, accumulate=False):
    B, C = x.shape[0], x.shape[-1]
    G = stats.shape[1]
    HW = x.numel() // (B * C)
    dx = torch.empty_like(x)
    wsb = lib().pso_group_norm_ws_bytes(B, HW, C)
    ws = torch.empty(wsb, device=x.device, dtype=torch.uint8)
    check(lib().pso_group_norm_bwd(B, HW, C, G, ptr(x), ptr(dy.contiguous()), ptr(stats), ptr(gamma), ptr(beta),
                                   int(silu), ptr(dadd), ptr(dx), ptr(dgamma), ptr(dbeta), int(accumulate), ptr(ws),
                                   wsb, stream_ptr()), "pso_group_norm_bwd")
    return dx


def layer_norm_fwd(x, gamma, beta, eps):
    """x [M, C] (row-strided view ok) -> (y [M,C], stats [M,2])."""
    M, C = x.shape
    y = torch.empty((M, C), device=x.device, dtype=x.dtype)
    stats = torch.empty((M, 2), device=x.device, dtype=torch.float32)
    check(lib().pso_layer_norm_fwd(M, C, float(eps), ptr(x), _row_stride(x), ptr(gamma), ptr(beta), ptr(y), C,
                                   ptr(stats), stream_ptr()), "pso_layer_norm_fwd")
    return y, stats


def layer_norm_bwd(x, dy, stats, gamma, dadd=None):
    M, C = x.shape
    dx = torch.empty((M, C), device=x.device, dtype=x.dtype)
    check(lib().pso_layer_norm_bwd(M, C, ptr(x), _row_stride(x), ptr(dy), _row_stride(dy), ptr(stats), ptr(gamma),
                                   ptr(dadd), _row_stride(dadd) if dadd is not None else 0, ptr(dx), C,
                                   stream_ptr()), "pso_layer_norm_bwd")
    return dx


# ------------------------------------------------------------------------------------------------------------------
# Attention: q/k/v/o are [B, S, H*64] tensors (views with unit last stride)
# ------------------------------------------------------------------------------------------------------------------
def _bsd(t):
    assert t.dim() == 3 and t.stride(2) == 1
    return t.stride(1), t.stride(0)


def attention_fwd(q, k, v, heads, scale=None, out=None):
    B, Sq, C = q.shape
    Sk = k.shape[1]
    assert C == heads * 64
    if scale is None:
        scale = 64 ** -0.5
    if out is None:
        out = torch.empty((B, Sq, C), device=q.device, dtype=q.dtype)
    lse = torch.empty((B, heads, Sq), device=q.device, dtype=torch.float32)
    (ldq, sqb), (ldk, skb), (ldv, svb), (ldo, sob) = _bsd(q), _bsd(k), _bsd(v), _bsd(out)
    check(lib().pso_attention_fwd(B, heads, Sq, Sk, ptr(q), ldq, sqb, ptr(k), ldk, skb, ptr(v), ldv, svb,
                                  float(scale), ptr(out), ldo, sob, ptr(lse), stream_ptr()), "pso_attention_fwd")
    return out, lse


def attention_bwd(q, k, v, o, lse, do, heads, scale=None, dq=None, dk=None, dv=None):
    B, Sq, C = q.shape
    Sk = k.shape[1]
    if scale is None:
        scale = 64 ** -0.5
    dq = torch.empty_like(q, memory_format=torch.contiguous_format) if dq is None else dq
    dk = torch.empty((B, Sk, C), device=q.device, dtype=q.dtype) if dk is None else dk
    dv = torch.empty((B, Sk, C), device=q.device, dtype=q.dtype) if dv is None else dv
    if Sk <= 256:
        assert dk.stride(0) == Sk * dk.stride(1) and dv.stride(0) == Sk * dv.stride(1)
    wsb = lib().pso_attention_bwd_ws_bytes(B, heads, Sq, Sk)
    ws = torch.empty(wsb, device=q.device, dtype=torch.uint8)
    do = do.contiguous()
    a = [_bsd(t) for t in (q, k, v, o, do, dq, dk, dv)]
    check(lib().pso_attention_bwd(B, heads, Sq, Sk, ptr(q), *a[0], ptr(k), *a[1], ptr(v), *a[2], ptr(o), *a[3],
                                  ptr(lse), ptr(do), *a[4], float(scale), ptr(dq), *a[5], ptr(dk), *a[6], ptr(dv),
                                  *a[7], ptr(ws), wsb, stream_ptr()), "pso_attention_bwd")
    return dq, dk, dv


# ------------------------------------------------------------------------------------------------------------------
# Element-wise
# ------------------------------------------------------------------------------------------------------------------
def geglu_fwd(h):
    M, F2 = h.shape
    F = F2 // 2
    out = torch.empty((M, F), device=h.device, dtype=h.dtype)
    check(lib().pso_geglu_fwd(M, F, ptr(h), _row_stride(h), ptr(out), F, stream_ptr()), "pso_geglu_fwd")
    return out


def geglu_bwd(h, dout):
    M, F2 = h.shape
    F = F2 // 2
    din = torch.empty((M, F2), device=h.device, dtype=h.dtype)
    check(lib().pso_geglu_bwd(M, F, ptr(h), _row_stride(h), ptr(dout), _row_stride(dout), ptr(din), F2,
                              stream_ptr()), "pso_geglu_bwd")
    return din


def silu(x):
    y = torch.empty_like(x)
    check(lib().pso_silu(x.numel(), ptr(x.contiguous()), ptr(y), stream_ptr()), "pso_silu")
    return y


def timestep_embedding(t, dim, out=None, out_col=0):
    t = t.reshape(-1).float().contiguous()
    if out is None:
        out = torch.empty((t.shape[0], dim), device=t.device, dtype=BF16)
    check(lib().pso_timestep_embedding(t.shape[0], dim, ptr(t), ptr(out), out.stride(0), out_col, stream_ptr()),
          "pso_timestep_embedding")
    return out


_TRANSPOSE_BATCH = None  # list of pending (src, dst) while a transpose_batch() block is open


class transpose_batch:
    """Context: every K.transpose inside returns its (allocated) output at once but runs at the block's end, all of
    them as ONE pso_transpose_multi launch (the full-UNet prepare() after each optimizer step: ~460 transposes whose
    per-call host cost exceeded their GPU time).  The sources are kept alive until the launch is enqueued; nothing
    inside the block may read a transposed output."""

    def __enter__(self):
        global _TRANSPOSE_BATCH
        self.prev, _TRANSPOSE_BATCH = _TRANSPOSE_BATCH, []
        return self

    def __exit__(self, *exc):
        global _TRANSPOSE_BATCH
        items, _TRANSPOSE_BATCH = _TRANSPOSE_BATCH, self.prev
        if items and exc[0] is None:
            _transpose_multi(items)
        return False


def _transpose_multi(items):
    import numpy as np
    dt = np.dtype([("src", "<u8"), ("dst", "<u8"), ("ldi", "<i8"), ("ldo", "<i8"), ("R", "<i4"), ("C", "<i4"),
                   ("tiles_c", "<i4"), ("tile0", "<i4")])
    assert dt.itemsize == 48
    rec = np.zeros(len(items), dt)
    tile = 0
    for i, (x, out) in enumerate(items):
        R, C = x.shape
        tc = -(-C // 64)
        rec[i] = (x.data_ptr(), out.data_ptr(), _row_stride(x), _row_stride(out), R, C, tc, tile)
        tile += -(-R // 64) * tc
    assert tile < 2 ** 31
    dev = items[0][1].device
    # pinned + non_blocking: a pageable copy would synchronise the stream (the host would stop getting ahead of the
    # GPU); torch's caching host allocator keeps the pinned block until the copy has run
    d = torch.from_numpy(rec.view(np.uint8)).pin_memory().to(dev, non_blocking=True)
    check(lib().pso_transpose_multi(len(items), ptr(d), tile, stream_ptr()), "pso_transpose_multi")


def transpose(x, out=None, pad_rows_to=1):
    """[R, C] -> [C, Rp], Rp = R rounded up to pad_rows_to (pad columns are zero)."""
    R, C = x.shape
    Rp = -(-R // pad_rows_to) * pad_rows_to
    if out is None:
        out = torch.empty((C, Rp), device=x.device, dtype=x.dtype)
    if _TRANSPOSE_BATCH is not None and Rp == R and x.dtype == torch.bfloat16 and R > 0 and C > 0:
        _row_stride(x)
        _row_stride(out)
        _TRANSPOSE_BATCH.append((x, out))
        return out
    check(lib().pso_transpose(R, Rp, C, ptr(x), _row_stride(x), ptr(out), _row_stride(out), stream_ptr()),
          "pso_transpose")
    return out


def im2col3(x, kp):
    B, H, W, C = x.shape
    out = torch.empty((B * H * W, kp), device=x.device, dtype=x.dtype)
    check(lib().pso_im2col3(B, H, W, C, ptr(x.contiguous()), ptr(out), kp, stream_ptr()), "pso_im2col3")
    return out


def sumpool2(x, dadd=None):
    B, H2, W2, C = x.shape
    out = torch.empty((B, H2 // 2, W2 // 2, C), device=x.device, dtype=x.dtype)
    check(lib().pso_sumpool2(B, H2 // 2, W2 // 2, C, ptr(x.contiguous()), ptr(dadd), ptr(out), stream_ptr()),
          "pso_sumpool2")
    return out


def axpby(a, x, b=0.0, z=None, out=None):
    out = torch.empty_like(x) if out is None else out
    check(lib().pso_axpby(x.numel(), float(a), ptr(x.contiguous()), float(b),
                          ptr(z.contiguous()) if z is not None else None, ptr(out), stream_ptr()), "pso_axpby")
    return out


_FULLGRAD_ATOMIC = os.environ.get("PSO_FULLGRAD_ATOMIC", "0") == "1"
_STREAM_WS = {}  # (device index, stream handle) -> uint8 scratch of the ordered parameter-sum reductions


def _stream_ws(nbytes, device):
    """Scratch for a reduction issued on the current stream: one buffer per (device, stream), grown on demand.  Its
    users are ordered by their stream, so reusing it needs no synchronisation (and no allocation per call)."""
    key = (device.index, torch.cuda.current_stream(device).cuda_stream)
    ws = _STREAM_WS.get(key)
    if ws is None or ws.numel() < nbytes:
        ws = _STREAM_WS[key] = torch.empty(max(int(nbytes * 1.25), 1 << 16), device=device, dtype=torch.uint8)
    return ws


def colsum_acc(x, out, rows_per_group=None):
    """out [G, N] f32 += per-group column sums of x [M, N] bf16 (G = M / rows_per_group; bias / row-bias grads), in a
    fixed summation order (pso_colsum_acc_ws: per-row-block partials through a workspace, no float atomics)."""
    M, N = x.shape
    rpg = M if rows_per_group is None else rows_per_group
    if _FULLGRAD_ATOMIC:  # A/B of the ordered form's cost (PSO_FULLGRAD_ATOMIC=1): f32 atomics, not reproducible
        check(lib().pso_colsum_acc(M, N, ptr(x), _row_stride(x), rpg, ptr(out),
                                   out.stride(0) if out.dim() > 1 else N, stream_ptr()), "pso_colsum_acc")
        return out
    wsb = int(lib().pso_colsum_acc_ws_bytes(M, N, rpg))
    ws = _stream_ws(wsb, x.device)
    check(lib().pso_colsum_acc_ws(M, N, ptr(x), _row_stride(x), rpg, ptr(out), out.stride(0) if out.dim() > 1 else N,
                                  ptr(ws), ws.numel(), stream_ptr()), "pso_colsum_acc_ws")
    return out


def layer_norm_dparam(x, dy, stats, dgamma, dbeta):
    """dgamma / dbeta [C] f32 += LayerNorm weight / bias grads (stats from layer_norm_fwd), in a fixed summation order
    (pso_layer_norm_dparam_ws)."""
    M, C = x.shape
    if _FULLGRAD_ATOMIC:
        check(lib().pso_layer_norm_dparam(M, C, ptr(x), _row_stride(x), ptr(dy), _row_stride(dy), ptr(stats),
                                          ptr(dgamma), ptr(dbeta), stream_ptr()), "pso_layer_norm_dparam")
        return
    wsb = int(lib().pso_layer_norm_dparam_ws_bytes(M, C))
    ws = _stream_ws(wsb, x.device)
    check(lib().pso_layer_norm_dparam_ws(M, C, ptr(x), _row_stride(x), ptr(dy), _row_stride(dy), ptr(stats),
                                         ptr(dgamma), ptr(dbeta), ptr(ws), ws.numel(), stream_ptr()),
          "pso_layer_norm_dparam_ws")


def im2col_conv(x, x2=None, mode=CONV_NORMAL, stride=1, pad=1, out_hw=None):
    """3x3 patch matrix [B*Ho*Wo, 9*(C1+C2)] (tap-major, channel-minor) of an NHWC conv input (+ concat source)."""
    B, H, W, C1 = x.shape
    C2 = x2.shape[3] if x2 is not None else 0
    if out_hw is None:
        out_hw = (2 * H, 2 * W) if mode == CONV_UP2 else ((H + 2 * pad - 3) // stride + 1, (W + 2 * pad - 3) // stride + 1)
    Ho, Wo = out_hw
    out = torch.empty((B * Ho * Wo, 9 * (C1 + C2)), device=x.device, dtype=BF16)
    check(lib().pso_im2col_conv(mode, B, ptr(x.contiguous()), C1, ptr(x2.contiguous()) if x2 is not None else None, C2,
                                H, W, Ho, Wo, stride, pad, ptr(out), out.stride(0), stream_ptr()), "pso_im2col_conv")
    return out


def add(x, z):
    return axpby(1.0, x, 1.0, z)


def cast_f32_bf16(x, scale=1.0, out=None):
    out = torch.empty(x.shape, device=x.device, dtype=BF16) if out is None else out
    check(lib().pso_cast_f32_bf16(x.numel(), ptr(x.contiguous()), float(scale), ptr(out), stream_ptr()),
          "pso_cast_f32_bf16")
    return out


def cast_bf16_f32(x, out=None):
    out = torch.empty(x.shape, device=x.device, dtype=torch.float32) if out is None else out
    check(lib().pso_cast_bf16_f32(x.numel(), ptr(x.contiguous()), ptr(out), stream_ptr()), "pso_cast_bf16_f32")
    return out


def conv_weight_t(w, flip):
    """[Co,k,k,Ci] -> [Ci,k,k,Co] (flip rotates the taps)."""
    Co, ks, _, Ci = w.shape
    out = torch.empty((Ci, ks, ks, Co), device=w.device, dtype=w.dtype)
    check(lib().pso_conv_weight_t(Co, ks, Ci, int(flip), ptr(w.contiguous()), ptr(out), stream_ptr()),
          "pso_conv_weight_t")
    return out


def concat_channels(x1, x2):
    """[..., C1] ++ [..., C2] -> [..., C1+C2] (contiguous channels-last)."""
    C1, C2 = x1.shape[-1], x2.shape[-1]
    out = torch.empty(x1.shape[:-1] + (C1 + C2,), device=x1.device, dtype=x1.dtype)
    npix = x1.numel() // C1
    check(lib().pso_concat_channels(npix, C1, ptr(x1.contiguous()), C2, ptr(x2.contiguous()), ptr(out),
                                    stream_ptr()), "pso_concat_channels")
    return out


def split_channels(x, C1, add2=None):
    """inverse of concat_channels; the second part gets `add2` added when given."""
    C = x.shape[-1]
    C2 = C - C1
    y1 = torch.empty(x.shape[:-1] + (C1,), device=x.device, dtype=x.dtype)
    y2 = torch.empty(x.shape[:-1] + (C2,), device=x.device, dtype=x.dtype)
    npix = x.numel() // C
    check(lib().pso_split_channels(npix, C1, C2, ptr(x.contiguous()), ptr(y1), ptr(y2),
                                   ptr(add2.contiguous()) if add2 is not None else None, stream_ptr()),
          "pso_split_channels")
    return y1, y2


def nchw_to_nhwc(x, pad_to=None, scale=1.0):
    """[B,C,H,W] fp32|bf16 -> [B,H,W,Cp] bf16 (channels zero-padded to Cp, values times scale)."""
    B, C, H, W = x.shape
    Cp = pad_to or C
    out = torch.empty((B, H, W, Cp), device=x.device, dtype=BF16)
    check(lib().pso_nchw_to_nhwc(B, C, Cp, H * W, ptr(x.contiguous()), dtype_code(x), float(scale), ptr(out),
                                 stream_ptr()), "pso_nchw_to_nhwc")
    return out


def softmax_rows(x):
    """in-place row softmax of a bf16 [M, N] matrix (row-strided view)."""
    M, N = x.shape
    check(lib().pso_softmax_rows(M, N, ptr(x), _row_stride(x), stream_ptr()), "pso_softmax_rows")
    return x


def nhwc_to_nchw(x, dtype=torch.float32):
    B, H, W, C = x.shape
    out = torch.empty((B, C, H, W), device=x.device, dtype=dtype)
    check(lib().pso_nhwc_to_nchw(B, C, H * W, ptr(x.contiguous()), ptr(out), dtype_code(out), stream_ptr()),
          "pso_nhwc_to_nchw")
    return out


# ------------------------------------------------------------------------------------------------------------------
# optimizer / clipping / preference
# ------------------------------------------------------------------------------------------------------------------
def grad_clip_coef(grad, max_norm, grad_scale=1.0, out=None):
    """-> float32[2] device tensor (norm, clip coefficient)."""
    n = grad.numel()
    out = torch.empty(2, device=grad.device, dtype=torch.float32) if out is None else out
    wsb = lib().pso_grad_clip_ws_bytes(n)
    ws = torch.empty(wsb, device=grad.device, dtype=torch.uint8)
    check(lib().pso_grad_clip_coef(n, ptr(grad), float(grad_scale), float(max_norm), ptr(out), ptr(ws), wsb,
                                   stream_ptr()), "pso_grad_clip_coef")
    return out


def adamw_step(param, grad, exp_avg, exp_avg_sq, lr, betas, eps, weight_decay, step, grad_scale=1.0, clip=None):
    check(lib().pso_adamw_step(param.numel(), ptr(param), ptr(grad), ptr(exp_avg), ptr(exp_avg_sq), float(lr),
                               float(betas[0]), float(betas[1]), float(eps), float(weight_decay), int(step),
                               float(grad_scale), ptr(clip), stream_ptr()), "pso_adamw_step")


class Adam8State:
    """State of the blockwise 8-bit AdamW (bitsandbytes AdamW8bit) for a flat fp32 parameter buffer of n elements:
    uint8 codes of m and v, one fp32 absmax per block of each; zero-initialised like bitsandbytes.

    segments = [(offset, numel)] of the parameter TENSORS inside the flat buffer (what bitsandbytes is handed at
    T:428-448): blocks of 2048 restart at every tensor, and a tensor under MIN_8BIT_SIZE = 4096 elements (bitsandbytes'
    min_8bit_size) keeps 32-bit m / v.  None: the whole buffer is one tensor (uniform blocks)."""

    BLOCK = 2048
    MIN_8BIT_SIZE = 4096

    def __init__(self, n, device, segments=None):
        self.n = n
        self.qm = torch.zeros(n, dtype=torch.uint8, device=device)
        self.qv = torch.zeros(n, dtype=torch.uint8, device=device)
        self.desc = None
        self.m32 = self.v32 = None
        if segments is None:
            nb = lib().pso_adamw8bit_blocks(n)
            self.block_start = None
        else:
            rows, n32 = [], 0
            for off, k in sorted(segments):
                assert 0 <= off and off + k <= n, (off, k, n)
                if k < self.MIN_8BIT_SIZE:  # 32-bit state, 8-aligned slot in the fp32 arrays
                    for b0 in range(0, k, self.BLOCK):
                        rows.append((off + b0, min(self.BLOCK, k - b0), n32 + b0, 0))
                    n32 += -(-k // 8) * 8
                else:
                    for b0 in range(0, k, self.BLOCK):
                        rows.append((off + b0, min(self.BLOCK, k - b0), -1, 0))
            for (o1, l1, _, _), (o2, _, _, _) in zip(rows, rows[1:]):
                assert o1 + l1 <= o2, "parameter segments overlap"
            nb = len(rows)
            self.desc = torch.tensor(rows, dtype=torch.int64).to(device)
            self.block_start = torch.tensor([r[0] for r in rows], dtype=torch.int64)
            self.rows = rows
            self.m32 = torch.zeros(max(n32, 8), dtype=torch.float32, device=device)
            self.v32 = torch.zeros(max(n32, 8), dtype=torch.float32, device=device)
        self.nblk = int(nb)
        self.am = torch.zeros(max(self.nblk, 1), dtype=torch.float32, device=device)
        self.av = torch.zeros(max(self.nblk, 1), dtype=torch.float32, device=device)

    @staticmethod
    def maps(device):
        """bitsandbytes' signed (m) / unsigned (v) dynamic code maps, 256 fp32 values each."""
        s = (ctypes.c_float * 256)()
        u = (ctypes.c_float * 256)()
        lib().pso_adamw8bit_maps(s, u)
        return torch.tensor(list(s), device=device), torch.tensor(list(u), device=device)

    _CHUNK_ROWS = 16384  # block-table rows per vectorised slice (bounds the per-element index tensors to ~32M)

    def _row_chunks(self):
        """(row ids, element positions, element -> row-in-chunk) per chunk of the block table, on the device."""
        dev = self.qm.device
        d = self.desc
        for r0 in range(0, self.nblk, self._CHUNK_ROWS):
            rows = torch.arange(r0, min(r0 + self._CHUNK_ROWS, self.nblk), device=dev)
            off, ln = d[rows, 0], d[rows, 1]
            blk = torch.repeat_interleave(torch.arange(rows.numel(), device=dev), ln)
            first = torch.cumsum(ln, 0) - ln
            pos = off[blk] + (torch.arange(blk.numel(), device=dev) - first[blk])
            yield rows, pos, blk

    def dequant(self):
        """(m, v) as fp32 over the flat buffer (tests / checkpoints; elements outside every tensor read 0).
        Vectorised over slices of the block table (full-UNet mode has ~1.25M rows)."""
        dev = self.qm.device
        cs, cu = self.maps(dev)
        n = self.qm.numel()
        if self.desc is None:
            blk = torch.arange(n, device=dev) // self.BLOCK
            return cs[self.qm.long()] * self.am[blk], cu[self.qv.long()] * self.av[blk]
        m = torch.zeros(n, device=dev)
        v = torch.zeros(n, device=dev)
        for rows, pos, blk in self._row_chunks():
            so = self.desc[rows, 2][blk]
            r32 = so >= 0
            p8, b8 = pos[~r32], rows[blk[~r32]]
            m[p8] = cs[self.qm[p8].long()] * self.am[b8]
            v[p8] = cu[self.qv[p8].long()] * self.av[b8]
            p32 = pos[r32]
            if p32.numel():
                i32 = so[r32] + (p32 - self.desc[rows, 0][blk[r32]])
                m[p32] = self.m32[i32]
                v[p32] = self.v32[i32]
        return m, v

    def load_dense(self, m, v):
        """Quantise fp32 moments m, v over the flat buffer into this state: per block absmax, nearest code of the
        normalised value (resume from a checkpoint written with another block layout)."""
        dev = self.qm.device
        m, v = m.to(dev, torch.float32), v.to(dev, torch.float32)
        cs, cu = self.maps(dev)

        def nearest(x, cmap):
            vals, order = torch.sort(cmap)
            i = torch.clamp(torch.searchsorted(vals, x), 1, vals.numel() - 1)
            lo, hi = vals[i - 1], vals[i]
            i = torch.where((x - lo) <= (hi - x), i - 1, i)
            return order[i].to(torch.uint8)

        if self.desc is None:
            nb = self.am.numel()
            pad = nb * self.BLOCK - m.numel()
            for x, q, a, cmap in ((m, self.qm, self.am, cs), (v, self.qv, self.av, cu)):
                xb = torch.nn.functional.pad(x, (0, pad)).view(nb, self.BLOCK)
                a.copy_(xb.abs().amax(1))
                q.copy_(nearest((xb / a.clamp_min(1e-30)[:, None]).reshape(-1)[:x.numel()], cmap))
            return
        for rows, pos, blk in self._row_chunks():
            so = self.desc[rows, 2][blk]
            r32 = so >= 0
            p32 = pos[r32]
            if p32.numel():
                i32 = so[r32] + (p32 - self.desc[rows, 0][blk[r32]])
                self.m32[i32] = m[p32]
                self.v32[i32] = v[p32]
            p8, b8 = pos[~r32], rows[blk[~r32]]
            for x, q, a, cmap in ((m, self.qm, self.am, cs), (v, self.qv, self.av, cu)):
                xa = x[p8]
                amax = torch.zeros(self.nblk, device=dev).index_reduce_(0, b8, xa.abs(), "amax", include_self=False)
                a[rows] = torch.where(self.desc[rows, 2] >= 0, a[rows], amax[rows])
                q[p8] = nearest(xa / a[b8].clamp_min(1e-30), cmap)

    def tensors(self):
        """The state tensors a checkpoint holds (name -> tensor)."""
        out = {"exp_avg_q": self.qm, "exp_avg_sq_q": self.qv, "absmax_m": self.am, "absmax_v": self.av}
        if self.desc is not None:
            out.update(exp_avg_32=self.m32, exp_avg_sq_32=self.v32, block_table=self.desc)
        return out


def adamw8bit_step(param, grad, state, lr, betas, eps, weight_decay, step, grad_scale=1.0, clip=None, out_bf16=None,
                   zero_grad=False):
    """One 8-bit AdamW step on the flat fp32 param; out_bf16 (same numel, bf16) also receives the updated parameters
    rounded to bf16 (the working copy), in the same pass.  zero_grad (per-tensor block tables only): the step also
    zeroes the gradient elements its blocks cover after reading them; returns whether it did."""
    require_cuda(param, grad)
    if out_bf16 is not None:
        assert out_bf16.dtype == torch.bfloat16 and out_bf16.numel() == param.numel() and out_bf16.is_contiguous()
    if state.desc is not None:
        fn = "pso_adamw8bit_step_blocks_zero_grad" if zero_grad else "pso_adamw8bit_step_blocks"
        check(getattr(lib(), fn)(param.numel(), state.nblk, ptr(state.desc), ptr(param), ptr(out_bf16),
                                              ptr(grad), ptr(state.qm), ptr(state.qv), ptr(state.am), ptr(state.av),
                                              ptr(state.m32), ptr(state.v32), float(lr), float(betas[0]),
                                              float(betas[1]), float(eps), float(weight_decay), int(step),
                                              float(grad_scale), ptr(clip), stream_ptr()), fn)
        return zero_grad
    check(lib().pso_adamw8bit_step_bf16(param.numel(), ptr(param), ptr(out_bf16), ptr(grad), ptr(state.qm),
                                        ptr(state.qv), ptr(state.am), ptr(state.av), float(lr), float(betas[0]),
                                        float(betas[1]), float(eps), float(weight_decay), int(step), float(grad_scale),
                                        ptr(clip), stream_ptr()),
          "pso_adamw8bit_step_bf16")
    return False


def zero_(x):
    check(lib().pso_zero_f32(x.numel(), ptr(x), stream_ptr()), "pso_zero_f32")
    return x


def preference(rewards, mode, reward_idx=None, out=None):
    """rewards [P, 2, m] fp32 -> pref [P, 2]."""
    P, _, m = rewards.shape
    out = torch.empty((P, 2), device=rewards.device, dtype=torch.float32) if out is None else out
    if reward_idx is not None:
        reward_idx = reward_idx.to(torch.int64).contiguous()
    check(lib().pso_preference(P, m, ptr(rewards.float().contiguous()), ptr(reward_idx), int(mode), ptr(out),
                               stream_ptr()), "pso_preference")
    return out


class BatchedTranspose:
    """A fixed list of (src [R,C], dst [C,R]) bf16 pairs transposed by ONE kernel launch (descriptor table on
    device, built once: the buffers are persistent)."""

    def __init__(self, pairs, device):
        import numpy as np
        dt = np.dtype([("src", "<u8"), ("dst", "<u8"), ("R", "<i4"), ("C", "<i4"), ("ldi", "<i8"), ("ldo", "<i8")])
        arr = np.zeros(len(pairs), dtype=dt)
        self.max_r = self.max_c = 1
        for i, (s, d) in enumerate(pairs):
            R, C = s.shape
            assert d.shape[0] == C and d.shape[1] >= R and s.stride(1) == 1 and d.stride(1) == 1
            arr[i] = (s.data_ptr(), d.data_ptr(), R, C, s.stride(0), d.stride(0))
            self.max_r, self.max_c = max(self.max_r, R), max(self.max_c, C)
        self.n = len(pairs)
        self.keep = pairs
        self.desc = torch.from_numpy(arr.view(np.uint8)).to(device)

    def __call__(self):
        if self.n:
            check(lib().pso_transpose_batched(self.n, ptr(self.desc), self.max_r, self.max_c, stream_ptr()),
                  "pso_transpose_batched")


def transpose_batched(x, out=None):
    """[Z, R, C] (rows contiguous) -> [Z, C, R] bf16 in one launch (a descriptor per matrix)."""
    Z, R, C = x.shape
    if out is None:
        out = torch.empty((Z, C, R), device=x.device, dtype=x.dtype)
    BatchedTranspose([(x[z], out[z]) for z in range(Z)], x.device)()
    return out


def gather_rows(src, idx, out=None):
    """out[i] = src[idx[i]] along dim 0 (rows of src[0].nbytes bytes)."""
    n = idx.numel()
    row_bytes = src[0].numel() * src.element_size()
    out = torch.empty((n,) + tuple(src.shape[1:]), device=src.device, dtype=src.dtype) if out is None else out
    check(lib().pso_gather_rows(n, row_bytes, ptr(src.contiguous()), ptr(idx.to(torch.int64).contiguous()),
                                ptr(out), stream_ptr()), "pso_gather_rows")
    return out


# ---------------------------------------------------------------------------------------------------------------------
# CLIP towers / reward image path (clip.hip)
# ---------------------------------------------------------------------------------------------------------------------
ACT_GELU, ACT_QUICK_GELU = 0, 1  # PSO_ACT_*


def attention_small(q, k, v, B, S, H, causal, scale, out=None):
    """q / k / v token-row views [B*S, H*D] (row-strided, e.g. column slices of a fused qkv) -> o [B*S, H*D] bf16."""
    require_cuda(q, k, v)
    HD = q.shape[1]
    D = HD // H
    if out is None:
        out = torch.empty((B * S, HD), device=q.device, dtype=BF16)
    sq, sk, sv, so = _row_stride(q), _row_stride(k), _row_stride(v), _row_stride(out)
    check(lib().pso_attention_small(B, H, S, D, ptr(q), sq, S * sq, ptr(k), sk, S * sk, ptr(v), sv, S * sv,
                                    int(bool(causal)), float(scale), ptr(out), so, S * so, stream_ptr()),
          "pso_attention_small")
    return out


def activation_(x, mode):
    assert x.is_contiguous() and x.dtype == BF16
    check(lib().pso_activation(x.numel(), ptr(x), int(mode), stream_ptr()), "pso_activation")
    return x


def embed_tokens(ids, tok, pos):
    """ids [B, S] int64 (device) -> [B*S, C] = tok[ids] + pos[:S]."""
    require_cuda(ids, tok, pos)
    B, S = ids.shape
    C = tok.shape[1]
    out = torch.empty((B * S, C), device=tok.device, dtype=BF16)
    check(lib().pso_embed_tokens(B, S, C, ptr(ids.contiguous()), ptr(tok), ptr(pos), ptr(out), stream_ptr()),
          "pso_embed_tokens")
    return out


def embed_vision(patch, cls, pos, B, P):
    C = patch.shape[1]
    out = torch.empty((B * (P + 1), C), device=patch.device, dtype=BF16)
    check(lib().pso_embed_vision(B, P, C, ptr(patch), ptr(cls), ptr(pos), ptr(out), stream_ptr()), "pso_embed_vision")
    return out


def cosine_rows(a, b):
    """[n, C] fp32 x [n, C] fp32 -> cos(a_i, b_i) [n] fp32."""
    require_cuda(a, b)
    n, C = a.shape
    assert a.dtype == torch.float32 and b.dtype == torch.float32 and b.shape == a.shape
    out = torch.empty(n, device=a.device, dtype=torch.float32)
    check(lib().pso_cosine_rows(n, C, ptr(a), _row_stride(a), ptr(b), _row_stride(b), ptr(out), stream_ptr()),
          "pso_cosine_rows")
    return out


def row_mean(x):
    """[B, ...] bf16 (contiguous) -> per-row mean [B] fp32."""
    require_cuda(x)
    B = x.shape[0]
    out = torch.empty(B, device=x.device, dtype=torch.float32)
    check(lib().pso_row_mean(B, x[0].numel(), ptr(x.contiguous()), ptr(out), stream_ptr()), "pso_row_mean")
    return out


def patchify(x, P, kpad):
    """processed pixel values NCHW [B, C, S, S] -> patch rows [B * (S/P)^2, kpad] bf16."""
    require_cuda(x)
    B, C, S, _ = x.shape
    out = torch.empty((B * (S // P) ** 2, kpad), device=x.device, dtype=BF16)
    check(lib().pso_patchify(B, C, S, P, kpad, ptr(x.float().contiguous()), ptr(out), stream_ptr()), "pso_patchify")
    return out


def clip_preprocess(img, size, P, kpad, mean, std):
    """decoded images NHWC [B, H, W, 3] (bf16 / f32 in [-1, 1], or uint8) -> patch rows [B * (size/P)^2, kpad] bf16
    (uint8 quantisation, PIL bicubic resize, centre crop, rescale, normalise)."""
    require_cuda(img)
    B, H, W, C = img.shape
    assert C == 3 and img.dtype in (BF16, torch.float32, torch.uint8) and img.is_contiguous()
    ws = torch.empty(lib().pso_clip_preprocess_ws_bytes(B, H, W, size), device=img.device, dtype=torch.uint8)
    out = torch.empty((B * (size // P) ** 2, kpad), device=img.device, dtype=BF16)
    m = (ctypes.c_float * 3)(*mean)
    sd = (ctypes.c_float * 3)(*std)
    code = 2 if img.dtype == torch.uint8 else dtype_code(img)  # PSO_U8
    check(lib().pso_clip_preprocess(B, H, W, ptr(img), code, size, P, kpad, m, sd, ptr(out), ptr(ws),
                                    ws.numel(), stream_ptr()), "pso_clip_preprocess")
    return out
