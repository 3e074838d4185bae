"""SDXL UNet2DConditionModel (+ peft-style LoRA) on the libpso_amd HIP kernels, forward AND hand-written backward.

Drop-in surface: `unet(sample, timestep, encoder_hidden_states, added_cond_kwargs={"time_ids",
"text_embeds"}, return_dict=True)` -> object with `.sample` (or a tuple); `.config.in_channels`; `add_adapter(cfg)`;
`disable_adapters()` / `enable_adapters()`; `enable_gradient_checkpointing()` (accepted, not needed: 288 GB HBM);
`parameters()`; `load_state_dict()` / `state_dict()` in diffusers key layout; `from_config(...)`.
Architecture restated from diffusers 0.27.0 (environment.yml:15; called at T:775-805, D:777-806,
DP/sdxl_turbo_with_logprob.py:126-132): conv_in -> 3 down blocks (320/640/1280; transformer depth 0/2/10) -> mid
(depth 10) -> 3 up blocks -> GroupNorm+SiLU -> conv_out; Timesteps(320)->MLP time embedding + the SDXL "text_time"
added embedding; BasicTransformerBlock = LN/self-attn/LN/cross-attn(77x2048)/LN/GEGLU FF; LoRA (rank r, alpha r) on
to_q/to_k/to_v/to_out.0 of all attentions (T:338-345).

MI355X-first design:
  * activations channels-last bf16 ([tokens, C] / NHWC), fp32 statistics and accumulation;
  * each diffusers Linear/Conv is one MFMA GEMM launch with bias / time-embedding / residual fused in the epilogue;
    self-attention q/k/v is ONE fused projection whose three LoRA up-projections are fused as a grouped K-tail;
  * the whole UNet is ONE autograd node: forward keeps exactly the tensors its hand-written backward needs (no
    gradient checkpoint recompute -- the reference's T:358 trades 6.8 TFLOP/img for memory that 288 GB HBM has);
  * LoRA masters are one flat fp32 buffer and their gradients one flat fp32 buffer that the backward GEMMs
    accumulate into directly (f32-accumulate epilogue) -- the all-reduce bucket and the optimizer operand.
"""
import math
import os
from dataclasses import dataclass, field, replace
from types import SimpleNamespace

import torch
import torch.nn as nn

from . import kernels as K

BF16 = torch.bfloat16
# batched (per gradient unit) LoRA weight-gradient launches; PSO_TN_BATCH=0 issues every product at once (A/B knob)
TN_BATCH = os.environ.get("PSO_TN_BATCH", "1") != "0"


# ======================================================================================================================
# config
# ======================================================================================================================
@dataclass
class UNetConfig:
    in_channels: int = 4
    out_channels: int = 4
    block_out_channels: tuple = (320, 640, 1280)
    layers_per_block: int = 2
    transformer_layers_per_block: tuple = (1, 2, 10)
    down_has_attn: tuple = (False, True, True)
    head_dim: int = 64
    cross_attention_dim: int = 2048
    addition_time_embed_dim: int = 256
    text_embed_dim: int = 1280
    norm_num_groups: int = 32
    norm_eps: float = 1e-5
    time_proj_dim: int = 320
    sample_size: int = 128

    @property
    def time_embed_dim(self):
        return 4 * self.block_out_channels[0]

    @property
    def projection_class_embeddings_input_dim(self):
        return self.text_embed_dim + 6 * self.addition_time_embed_dim

    @staticmethod
    def sdxl(sample_size=128):
        return UNetConfig(sample_size=sample_size)

    @staticmethod
    def tiny(sample_size=16):
        """Same topology, small widths (parity tests)."""
        return UNetConfig(block_out_channels=(64, 128, 128), transformer_layers_per_block=(1, 1, 2),
                          cross_attention_dim=128, addition_time_embed_dim=32, text_embed_dim=64, time_proj_dim=64,
                          sample_size=sample_size)


# ======================================================================================================================
# parameter holders (diffusers names / layouts) + kernel-layout caches
# ======================================================================================================================
def _param(*shape):
    return nn.Parameter(torch.empty(*shape, dtype=BF16), requires_grad=False)


def _uniform_(p, bound, g):
    """U(-bound, bound) on the parameter's own device (PyTorch-default-style fan-in init, synthetic weights)."""
    with torch.no_grad():
        p.copy_((torch.rand(p.shape, generator=g, device=p.device, dtype=torch.float32) * 2 - 1) * bound)


class Linear(nn.Module):
    def __init__(self, fin, fout, bias=True):
        super().__init__()
        self.in_features, self.out_features = fin, fout
        self.weight = _param(fout, fin)
        self.bias = _param(fout) if bias else None

    def reset(self, g):
        bound = 1.0 / math.sqrt(self.in_features)
        _uniform_(self.weight, bound, g)
        if self.bias is not None:
            _uniform_(self.bias, bound, g)

    def prepare(self):
        self.wt = K.transpose(self.weight.data)  # [in][out] for the input gradient


class Conv2d(nn.Module):
    def __init__(self, cin, cout, k, stride=1, bias=True):
        super().__init__()
        self.cin, self.cout, self.k, self.stride = cin, cout, k, stride
        self.weight = _param(cout, cin, k, k)
        self.bias = _param(cout) if bias else None

    def reset(self, g):
        bound = 1.0 / math.sqrt(self.cin * self.k * self.k)
        _uniform_(self.weight, bound, g)
        if self.bias is not None:
            _uniform_(self.bias, bound, g)

    def prepare(self):
        w = self.weight.data
        self.w_nhwc = w.permute(0, 2, 3, 1).contiguous()  # [Co][kh][kw][Ci]  (one-time layout change at load)
        if self.k == 1:
            self.w_mat = self.w_nhwc.view(self.cout, self.cin)
            self.wt = K.transpose(self.w_mat)
        elif self.cin % 64 != 0:  # conv_in: im2col GEMM, K = 9*Ci padded to 64
            kp = 64 * ((9 * self.cin + 63) // 64)
            self.kp = kp
            self.w_col = torch.zeros(self.cout, kp, device=w.device, dtype=BF16)
            self.w_col[:, :9 * self.cin] = self.w_nhwc.reshape(self.cout, -1)
        else:
            # input-gradient weights: stride 1 -> rotated taps; stride 2 -> unrotated taps (T2 gather)
            self.w_dx = K.conv_weight_t(self.w_nhwc, flip=(self.stride == 1))
            if self.cout % 64 != 0:  # conv_out (Co=4): the input-gradient conv has C=4 -> im2col GEMM
                kp = 64 * ((9 * self.cout + 63) // 64)
                self.kp_dx = kp
                self.w_dx_col = torch.zeros(self.cin, kp, device=w.device, dtype=BF16)
                self.w_dx_col[:, :9 * self.cout] = self.w_dx.reshape(self.cin, -1)


class Norm(nn.Module):
    def __init__(self, c):
        super().__init__()
        self.weight = _param(c)
        self.bias = _param(c)

    def reset(self, g):
        with torch.no_grad():
            self.weight.fill_(1.0)
            self.bias.zero_()


def _stacked(ws):
    """torch.cat(ws, 0) of same-width row-major weights -- as a zero-copy view when they already lie back to back in
    memory (the full-UNet flat working copy keeps a block's q/k/v, and k/v, adjacent), else a new tensor."""
    w0 = ws[0]
    base = w0.untyped_storage().data_ptr()
    adjacent = all(w.is_contiguous() and w.dtype == w0.dtype and w.shape[1:] == w0.shape[1:] and
                   w.untyped_storage().data_ptr() == base for w in ws)  # one storage (not merely adjacent blocks)
    if adjacent:
        off = w0.data_ptr()
        for w in ws:
            adjacent = adjacent and w.data_ptr() == off
            off += w.numel() * w.element_size()
    if adjacent:
        rows = sum(w.shape[0] for w in ws)
        return torch.as_strided(w0, (rows,) + tuple(w0.shape[1:]), w0.stride(), w0.storage_offset())
    return torch.cat(ws, 0)


# ======================================================================================================================
# Full-UNet training state (BASELINE C3 / C4, SURVEY §8a a6 "full dW in C3 (build-only)")
# ======================================================================================================================
class FullGradState:
    """Every UNet parameter trainable (the reference always trains LoRA -- App. A #4 -- so this is the build-only C3 /
    C4 mode).  ONE flat fp32 master (initialised from the bf16 module weights) and ONE flat fp32 grad (the all-reduce
    bucket / optimizer operand) in named_parameters order, with a per-parameter view of each; the module parameters
    stay the bf16 working copies the kernels read, rewritten from the master by refresh() (then the kernel-layout
    caches are rebuilt by UNet2DConditionModel.prepare())."""

    def __init__(self, unet):
        # flat layout in the order the backward COMPLETES the parameters (UNet2DConditionModel.grad_units), so each
        # all-reduce bucket of the overlapped gradient sync is one contiguous range that is final when issued
        named = dict(unet.named_parameters())
        order, seen = [], set()
        for _, names in unet.grad_units():
            for nm in names:
                if nm in named and nm not in seen:
                    order.append(nm)
                    seen.add(nm)
        order += [nm for nm in named if nm not in seen]
        self.names = order
        params = [named[nm] for nm in order]
        # every tensor starts on a 64-element boundary of the flat buffers (its bf16 working view then has the 16-B
        # aligned rows the kernels need); the pads are zero in master and grad and stay zero under the optimizer
        slot = lambda k: -(-k // self.ALIGN) * self.ALIGN
        n = sum(slot(p.numel()) for p in params)
        dev = params[0].device
        self.params = params
        self.master = torch.zeros(n, device=dev, dtype=torch.float32)
        self.grad = torch.zeros(n, device=dev, dtype=torch.float32)
        # the bf16 module weights become views of ONE flat working copy in the master's layout, so refresh() is one
        # cast kernel (it was one copy per tensor: ~1,700 launches per optimizer step)
        assert all(p.dtype == params[0].dtype for p in params), "full-UNet training needs one parameter dtype"
        self.work = torch.zeros(n, device=dev, dtype=params[0].dtype)
        self._g, self._m = {}, {}
        self.offsets = {}
        off = 0
        for nm, p in zip(order, params):
            k = p.numel()
            self.offsets[nm] = (off, slot(k))  # the slot (with its pad): units of them tile the flat buffers
            self._m[id(p)] = self.master[off:off + k].view(p.shape)
            self._g[id(p)] = self.grad[off:off + k].view(p.shape)
            self._m[id(p)].copy_(p.data.float())
            w = self.work[off:off + k].view(p.shape)
            w.copy_(p.data)
            p.data = w
            off += slot(k)
        self.numel = n
        self.trigger = torch.zeros(1, device=dev, requires_grad=True)  # autograd hook for UNet.forward (_UNetFn)

    ALIGN = 64  # elements per flat-buffer slot boundary

    def g(self, p):
        """fp32 gradient view of module parameter p (same shape)."""
        return self._g[id(p)]

    def master_from_params(self):
        """bf16 module weights -> fp32 master (after the weights were changed in place)."""
        with torch.no_grad():
            K.cast_bf16_f32(self.work, out=self.master)

    def refresh(self, cast=True):
        """master -> bf16 module weights (the caller re-runs prepare()): one cast over the flat buffers (cast=False:
        the optimizer already wrote them)."""
        if cast:
            with torch.no_grad():
                K.cast_f32_bf16(self.master, out=self.work)


_FULL_SIDE = os.environ.get("PSO_FULL_SIDE_STREAM", "1") == "1"
# fp8 forward (config 5): which LayerNorm-fed projections take the e4m3 kernel (diagnostics: tools/diag_fp8_grads.py)
# "tail": the LoRA up-projection as an e4m3 K-tail; "qkv" (the self-attention q/k/v) is off by default, see
# enable_fp8_forward
FP8_KINDS = {"q2", "ff", "tail"}
FP8_MIN_TILES = int(os.environ.get("PSO_FP8_MIN_TILES", "192"))  # see BasicTransformerBlock.fwd (0: no occupancy rule)
# The e4m3 GEGLU form has 256 x 256 tiles only, while the bf16 one takes 256 x 320 tiles where they need fewer
# tile-rounds (gemm.hip pso_gemm_geglu: rounds x tile width).  A round of e4m3 tiles costs ~1/1.3 of a bf16 one on
# these shapes (the 2x MFMA rate less the row quantisation and the longer prologue: C5's GEGLU 5.7 -> 4.2 ms at equal
# tiles), so the ff kind stays on e4m3 only while its rounds x 256 undercut 1.3 x the bf16 form's rounds x width.
FP8_ROUND_GAIN = 1.3


def fp8_geglu_pays(M, n_out):
    """True when the e4m3 GEGLU projection (256 x 256 tiles) is expected to beat the bf16 one's tile choice."""
    mt = (M + 255) // 256
    w8 = (mt * (n_out // 256) + 255) // 256 * 256
    w16 = w8 if n_out % 320 else min(w8, (mt * (n_out // 320) + 255) // 256 * 320)
    return w8 < FP8_ROUND_GAIN * w16
_GEGLU_TN = os.environ.get("PSO_GEGLU_TN", "1") == "1"
# diagnostics (tools/c2_window_diag.py): the forward's LoRA-augmented projections rounded as torch/peft round them --
# bf16(base + bias), bf16(LoRA term), bf16 add, then bf16 residual add -- instead of one rounding of the fused sum
_TORCH_ROUND = os.environ.get("PSO_TORCH_ROUND", "0") == "1"


def _gemm_fwd(a, w, *, a2=None, w2=None, tail_group_n=0, tail_rows=0, bias=None, resid=None, **kw):
    """K.gemm for the forward's LoRA-augmented projections (PSO_TORCH_ROUND=1: the torch/peft rounding sequence)."""
    if not _TORCH_ROUND or a2 is None:
        return K.gemm(a, w, a2=a2, w2=w2, tail_group_n=tail_group_n, tail_rows=tail_rows, bias=bias, resid=resid,
                      **kw)
    base = K.gemm(a, w, bias=bias)
    rows = tail_rows if tail_rows else a.shape[0]
    N = w.shape[0]
    if tail_group_n:
        r = w2.shape[1]
        lo = torch.cat([K.gemm(a2[:, j * r:(j + 1) * r].contiguous(), w2[j * tail_group_n:(j + 1) * tail_group_n])
                        for j in range(N // tail_group_n)], 1)
    else:
        lo = K.gemm(a2, w2)
    base[:rows] = (base[:rows].float() + lo.float()).to(BF16)
    if resid is not None:
        base = (base.float() + resid.float()).to(BF16)
    return base  # ff.proj dW straight into the natural rows (pso_gemm_tn_geglu)


def _lin_dw(fg, lin, dy, x, rt=None):
    """nn.Linear weight / bias grads: dW += dy^T x (TN GEMM), db += column sums of dy (on rt's side stream)."""
    def run():
        K.gemm_tn(dy, x, fg.g(lin.weight))
        if lin.bias is not None:
            K.colsum_acc(dy, fg.g(lin.bias).view(1, -1))
    if rt is None:
        run()
    else:
        rt.side.launch(run, dy, x)


def _conv_dw(fg, conv, dy2d, src, rt=None, cols_fn=None):
    """3x3 conv weight / bias grads from the patch matrix cols [M, 9*Cin] (tap-major) = cols_fn(src): dW_nhwc =
    dy^T cols, then into the diffusers [Cout][Cin][kh][kw] grad view (the patch matrix is built on rt's side stream
    too).  cols_fn None: src is the patch matrix."""
    def run():
        cols = cols_fn(src) if cols_fn is not None else src
        tmp = torch.zeros((dy2d.shape[1], cols.shape[1]), device=cols.device, dtype=torch.float32)
        K.gemm_tn(dy2d, cols, tmp)
        co = conv.cout
        fg.g(conv.weight).add_(tmp[:co, :9 * conv.cin].view(co, 3, 3, conv.cin).permute(0, 3, 1, 2))
        if conv.bias is not None:
            K.colsum_acc(dy2d[:, :co] if dy2d.shape[1] != co else dy2d, fg.g(conv.bias).view(1, -1))
    if rt is None:
        run()
    else:
        rt.side.launch(run, dy2d, src)


def _tn_stacked(fg, lins, dy, x):
    """dW of nn.Linears whose weights are stacked rows of one flat-gradient range (q / k / v; cross k / v) fed by the
    column blocks of one dy: ONE TN GEMM over the stacked rows when their grads are adjacent, else one per weight."""
    gs = [fg.g(l.weight) for l in lins]
    n = gs[0].numel()
    if all(g.data_ptr() == gs[0].data_ptr() + i * n * 4 for i, g in enumerate(gs)):
        K.gemm_tn(dy, x, gs[0].view(-1).as_strided((len(gs) * gs[0].shape[0], gs[0].shape[1]), (gs[0].shape[1], 1)))
    else:
        C = gs[0].shape[0]
        for j, g in enumerate(gs):
            K.gemm_tn(dy[:, j * C:(j + 1) * C], x, g)


# ======================================================================================================================
# LoRA state: flat fp32 masters + flat fp32 grads (the all-reduce bucket), bf16 working copies
# ======================================================================================================================
LORA_TARGETS = ("to_k", "to_q", "to_v", "to_out.0")  # T:342, D:365, DB:1324


class LoraConfig:
    """The fields of peft 0.11's `LoraConfig` that shape a UNet adapter, with peft's defaults (peft is not a
    dependency here; `add_adapter` also takes peft's own object or any namespace with these attribute names)."""

    def __init__(self, r=8, lora_alpha=8, target_modules=None, init_lora_weights=True, lora_dropout=0.0,
                 bias="none", use_rslora=False, use_dora=False, fan_in_fan_out=False, modules_to_save=None,
                 layers_to_transform=None, layers_pattern=None, rank_pattern=None, alpha_pattern=None, **kw):
        self.r, self.lora_alpha, self.target_modules = r, lora_alpha, target_modules
        self.init_lora_weights, self.lora_dropout, self.bias = init_lora_weights, lora_dropout, bias
        self.use_rslora, self.use_dora, self.fan_in_fan_out = use_rslora, use_dora, fan_in_fan_out
        self.modules_to_save, self.layers_to_transform, self.layers_pattern = modules_to_save, layers_to_transform, \
            layers_pattern
        self.rank_pattern, self.alpha_pattern = rank_pattern or {}, alpha_pattern or {}
        for k, v in kw.items():  # task_type, inference_mode, revision, ...: no effect on the adapter arithmetic
            setattr(self, k, v)


def check_lora_config(cfg):
    """(r, lora_alpha) of a peft-style LoraConfig, after checking that it asks for the adapters the reference trains:
    LoRA (not DoRA / rsLoRA) on exactly to_q / to_k / to_v / to_out.0 of every attention, gaussian init, no dropout, no
    bias, no per-module rank / alpha patterns, no extra trained modules.  A field the object does not carry counts as
    the reference's value (namespace configs: SimpleNamespace(r=..., lora_alpha=...)); a field that differs raises
    ValueError naming it -- the kernels would otherwise train other adapters than the config asks for."""
    def get(name, ref):
        return getattr(cfg, name, ref)

    r = get("r", 32)
    if isinstance(r, bool) or not isinstance(r, int) or r <= 0 or r % 8:
        raise ValueError(f"LoraConfig.r must be a positive multiple of 8 (the rank kernels' granule), got {r!r}")
    alpha = get("lora_alpha", r)
    if isinstance(alpha, bool) or not isinstance(alpha, (int, float)) or not alpha > 0:
        raise ValueError(f"LoraConfig.lora_alpha must be a positive number, got {alpha!r}")
    tm = get("target_modules", LORA_TARGETS)
    if isinstance(tm, str) or tm is None or sorted(tm) != sorted(LORA_TARGETS) or len(set(tm)) != len(tm):
        raise ValueError(f"LoraConfig.target_modules must be {list(LORA_TARGETS)} (T:342), got {tm!r}")
    init = get("init_lora_weights", "gaussian")
    if init != "gaussian" or isinstance(init, bool):
        raise ValueError(f"LoraConfig.init_lora_weights must be 'gaussian' (T:341), got {init!r}")
    checks = (("lora_dropout", 0.0, lambda v: v == 0), ("bias", "none", lambda v: v == "none"),
              ("use_rslora", False, lambda v: v is False), ("use_dora", False, lambda v: v is False),
              ("fan_in_fan_out", False, lambda v: v is False), ("modules_to_save", None, lambda v: not v),
              ("layers_to_transform", None, lambda v: v is None), ("layers_pattern", None, lambda v: v is None),
              ("rank_pattern", {}, lambda v: not v), ("alpha_pattern", {}, lambda v: not v),
              ("megatron_config", None, lambda v: v is None), ("loftq_config", {}, lambda v: not v))
    for name, ref, ok in checks:
        v = get(name, ref)
        if not ok(v):
            raise ValueError(f"LoraConfig.{name}={v!r} is not implemented (the reference uses {ref!r})")
    return r, alpha

class LoraState:
    """peft LoraConfig(r, lora_alpha=r, init_lora_weights="gaussian", target_modules=[to_k,to_q,to_v,to_out.0])
    (T:338-345): A ~ N(0, 1/r) [r, in], B = 0 [out, r], scaling alpha/r.

    Storage: ONE flat fp32 master, ONE flat fp32 grad (the all-reduce bucket / optimizer operand), ONE flat bf16
    working copy.  Transformer blocks are laid out in reverse forward order (the order the backward finishes their
    gradients); inside a block the adapters that are used together are adjacent so their stacks are plain views:
      attn1: [A_q A_k A_v] (3r x C) [B_q B_k B_v] (3C x r) A_o B_o | attn2: A_q B_q [A_k A_v] [B_k B_v] A_o B_o
    After each optimizer step `refresh()` = one cast kernel + one batched-transpose kernel for the transposed forms the
    backward GEMMs need (A^T, (sB)^T)."""

    def __init__(self, blocks, r, alpha, device):
        self.r, self.alpha, self.scale = r, alpha, alpha / r
        self.blocks = blocks  # [(path, C, Dc)] forward order
        self.layout = {}
        off = 0
        for path, C, Dc in reversed(blocks):
            segs = {}
            for key, rows, cols in (("attn1.A_qkv", 3 * r, C), ("attn1.B_qkv", 3 * C, r), ("attn1.A_o", r, C),
                                    ("attn1.B_o", C, r), ("attn2.A_q", r, C), ("attn2.B_q", C, r),
                                    ("attn2.A_kv", 2 * r, Dc), ("attn2.B_kv", 2 * C, r), ("attn2.A_o", r, C),
                                    ("attn2.B_o", C, r)):
                segs[key] = (off, rows, cols)
                off += rows * cols
            self.layout[path] = segs
        self.numel = off
        self.master = torch.zeros(off, device=device, dtype=torch.float32)
        self.grad = torch.zeros(off, device=device, dtype=torch.float32)
        self.work = torch.zeros(off, device=device, dtype=BF16)
        self.param = nn.Parameter(self.master, requires_grad=True)  # autograd trigger for the UNet node
        self.blk = {}
        pairs = []
        for path, C, Dc in blocks:
            w = lambda k: self.seg(self.work, path, k)
            ns = SimpleNamespace()
            ns.A_qkv, ns.sB_qkv, ns.A_o1, ns.sB_o1 = w("attn1.A_qkv"), w("attn1.B_qkv"), w("attn1.A_o"), w("attn1.B_o")
            ns.A_q2, ns.sB_q2, ns.A_kv2, ns.sB_kv2 = w("attn2.A_q"), w("attn2.B_q"), w("attn2.A_kv"), w("attn2.B_kv")
            ns.A_o2, ns.sB_o2 = w("attn2.A_o"), w("attn2.B_o")
            ns.At_qkv = torch.empty(C, 3 * r, device=device, dtype=BF16)
            ns.sBt_qkv = torch.empty(r, 3 * C, device=device, dtype=BF16)
            ns.At_o1 = torch.empty(C, r, device=device, dtype=BF16)
            ns.sBt_o1 = torch.empty(r, C, device=device, dtype=BF16)
            ns.At_q2 = torch.empty(C, r, device=device, dtype=BF16)
            ns.sBt_q2 = torch.empty(r, C, device=device, dtype=BF16)
            ns.sBt_kv2 = torch.empty(r, 2 * C, device=device, dtype=BF16)
            ns.At_o2 = torch.empty(C, r, device=device, dtype=BF16)
            ns.sBt_o2 = torch.empty(r, C, device=device, dtype=BF16)
            pairs += [(ns.A_qkv, ns.At_qkv), (ns.sB_qkv, ns.sBt_qkv), (ns.A_o1, ns.At_o1), (ns.sB_o1, ns.sBt_o1),
                      (ns.A_q2, ns.At_q2), (ns.sB_q2, ns.sBt_q2), (ns.sB_kv2, ns.sBt_kv2), (ns.A_o2, ns.At_o2),
                      (ns.sB_o2, ns.sBt_o2)]
            self.blk[path] = ns
        self._transposes = K.BatchedTranspose(pairs, device) if device.type == "cuda" else None
        # per width C: the k/v adapters of its blocks stacked in block order, A [n*2r, Dc] and sB [n*2C, r], for the
        # width-batched text K/V projection (UNet2DConditionModel.kv_text); rebuilt by refresh()
        by_c = {}
        for path, C, Dc in blocks:
            by_c.setdefault(C, []).append(self.blk[path])
        self.kv_stacks = {C: (torch.empty(len(bl) * 2 * r, bl[0].A_kv2.shape[1], device=device, dtype=BF16),
                              torch.empty(len(bl) * 2 * C, r, device=device, dtype=BF16), bl)
                          for C, bl in by_c.items()}
        self._b_views = [self.seg(self.work, p, k) for p, _, _ in blocks for k in self.layout[p] if ".B_" in k]

    def seg(self, t, path, key):
        off, rows, cols = self.layout[path][key]
        return t[off:off + rows * cols].view(rows, cols)

    # peft per-adapter views (A [r][in], B [out][r]) of a flat tensor
    def adapter_views(self, t, name):
        path, attn, mod = name.rsplit(".", 2)[0], name.rsplit(".", 2)[1], name.rsplit(".", 2)[2]
        if mod == "0":  # to_out.0
            path, attn = name.rsplit(".", 3)[0], name.rsplit(".", 3)[1]
            mod = "to_out.0"
        r = self.r
        if attn == "attn1":
            if mod in ("to_q", "to_k", "to_v"):
                j = ("to_q", "to_k", "to_v").index(mod)
                A = self.seg(t, path, "attn1.A_qkv")[j * r:(j + 1) * r]
                Bm = self.seg(t, path, "attn1.B_qkv")
                C = Bm.shape[0] // 3
                return A, Bm[j * C:(j + 1) * C]
            return self.seg(t, path, "attn1.A_o"), self.seg(t, path, "attn1.B_o")
        if mod == "to_q":
            return self.seg(t, path, "attn2.A_q"), self.seg(t, path, "attn2.B_q")
        if mod in ("to_k", "to_v"):
            j = ("to_k", "to_v").index(mod)
            Bm = self.seg(t, path, "attn2.B_kv")
            C = Bm.shape[0] // 2
            return self.seg(t, path, "attn2.A_kv")[j * r:(j + 1) * r], Bm[j * C:(j + 1) * C]
        return self.seg(t, path, "attn2.A_o"), self.seg(t, path, "attn2.B_o")

    def adapter_names(self):
        for path, _, _ in self.blocks:
            for a in ("attn1", "attn2"):
                for m in ("to_q", "to_k", "to_v", "to_out.0"):
                    yield f"{path}.{a}.{m}"

    def init_gaussian(self, seed=0, b_std=0.0):
        g = torch.Generator(device="cpu").manual_seed(seed)
        for name in self.adapter_names():
            A, B = self.adapter_views(self.master, name)
            A.copy_(torch.randn(A.shape, generator=g) / self.r)  # peft gaussian: std 1/r
            if b_std:
                B.copy_(torch.randn(B.shape, generator=g) * b_std)
            else:
                B.zero_()
        self.refresh()

    def refresh(self, cast=True):
        """bf16 working copies (B pre-scaled by alpha/r) and their transposed forms after a master update (cast=False:
        the optimizer already wrote work = bf16(master))."""
        self.version = getattr(self, "version", 0) + 1  # keys the fp8 copies of the sB stacks (fp8 forward)
        if cast:
            K.cast_f32_bf16(self.master, out=self.work)
        if self.scale != 1.0:
            for Bw in self._b_views:
                K.axpby(self.scale, Bw, out=Bw)
        self._transposes()
        for A, sB, bl in self.kv_stacks.values():
            torch.cat([L.A_kv2 for L in bl], 0, out=A)
            torch.cat([L.sB_kv2 for L in bl], 0, out=sB)

    def grad_seg(self, path, key):
        return self.seg(self.grad, path, key)

    def state_dict_peft(self):
        """{module_path.lora_A.weight, module_path.lora_B.weight} (get_peft_model_state_dict naming)."""
        out = {}
        for name in self.adapter_names():
            A, B = self.adapter_views(self.master, name)
            out[f"{name}.lora_A.weight"] = A.detach().clone()
            out[f"{name}.lora_B.weight"] = B.detach().clone()
        return out

    def grad_dict_peft(self):
        out = {}
        for name in self.adapter_names():
            A, B = self.adapter_views(self.grad, name)
            out[f"{name}.lora_A.weight"] = A
            out[f"{name}.lora_B.weight"] = B
        return out

    def load_peft(self, sd):
        for name in self.adapter_names():
            A, B = self.adapter_views(self.master, name)
            A.copy_(sd[f"{name}.lora_A.weight"])
            B.copy_(sd[f"{name}.lora_B.weight"])
        self.refresh()


# ======================================================================================================================
# blocks: fwd(x, rt) -> y (saving what bwd needs in a dict when rt.save) ; bwd(dy, saved, rt) -> dx
# ======================================================================================================================
class Attention(nn.Module):
    """diffusers Attention (heads = dim/64, to_q/to_k/to_v without bias, to_out.0 with bias)."""

    def __init__(self, dim, kv_dim):
        super().__init__()
        self.dim, self.kv_dim, self.heads = dim, kv_dim, dim // 64
        self.to_q = Linear(dim, dim, bias=False)
        self.to_k = Linear(kv_dim, dim, bias=False)
        self.to_v = Linear(kv_dim, dim, bias=False)
        self.to_out = nn.ModuleList([Linear(dim, dim)])

    def prepare(self, self_attn):
        C = self.dim
        if self_attn:
            self.w_qkv = _stacked([self.to_q.weight.data, self.to_k.weight.data, self.to_v.weight.data])
            self.wt_qkv = K.transpose(self.w_qkv)  # [C][3C]
        else:
            self.w_kv = _stacked([self.to_k.weight.data, self.to_v.weight.data])
            self.to_q.prepare()
        self.to_out[0].prepare()


class BasicTransformerBlock(nn.Module):
    def __init__(self, dim, cross_dim):
        super().__init__()
        self.dim = dim
        self.norm1, self.norm2, self.norm3 = Norm(dim), Norm(dim), Norm(dim)
        self.attn1 = Attention(dim, dim)
        self.attn2 = Attention(dim, cross_dim)
        self.ff = SimpleFF(dim)

    def prepare(self):
        self.attn1.prepare(True)
        self.attn2.prepare(False)
        self.ff.prepare()

    def fwd(self, x, rt, path):
        """x [M, C] (M = B*S).  Returns h3 [M, C]."""
        C, M, B = self.dim, x.shape[0], rt.B
        S = M // B
        a1m, a2m = self.attn1, self.attn2
        lo = rt.lora_on
        L = rt.lora.blk[path] if lo else None
        r = rt.r
        # paired pass (policy images first, then their reference copies): the adapters act on the first Mp rows only
        Mp = M // 2 if rt.paired else M
        tr = Mp if rt.paired else 0
        pol = (lambda t: t[:t.shape[0] // 2]) if rt.paired else (lambda t: t)
        # --- self attention: fused q/k/v projection, the three LoRA up-projections as a grouped K-tail ---
        n1, st1 = K.layer_norm_fwd(x, self.norm1.weight, self.norm1.bias, 1e-5)
        f8 = rt.fp8  # fp8 forward (config 5): the LayerNorm-fed projections on e4m3 MFMA where the shapes allow
        # (the fp8 LoRA tail reads 16-B rows of the rank-r operands: r % 16 == 0)
        # ... and only where the e4m3 GEMM's 256 x 256 tiles make at least three quarters of a 256-CU round: below that
        # the product is latency-bound, not MFMA-bound, and the separate row quantisation makes it slower than the bf16
        # kernel (C5 at 1 + 1 images: the L2 cross-attention q, 2048 x 1280 -- 40 tiles -- 28 vs 21 us per launch)
        ok8 = lambda n_out, k_in, kind: (f8 is not None and kind in FP8_KINDS and n_out % 256 == 0 and
                                         k_in % 128 == 0 and (not lo or rt.r % 16 == 0) and
                                         ((M + 255) // 256) * (n_out // 256) >= FP8_MIN_TILES)
        ver = rt.lora.version if lo else 0
        if lo:
            u_qkv = K.gemm(pol(n1), L.A_qkv)                                # [Mp, 3r]
            if ok8(3 * C, C, "qkv") and "tail" not in FP8_KINDS:  # diagnostics: the LoRA term in bf16
                qkv = K.gemm_fp8(K.quant_rows_fp8(n1), f8((id(self), "qkv"), a1m.w_qkv))
                for j in range(3):
                    sl = qkv[:Mp, j * C:(j + 1) * C]
                    sl.copy_(K.gemm(u_qkv[:, j * r:(j + 1) * r], L.sB_qkv[j * C:(j + 1) * C], resid=sl))
            elif ok8(3 * C, C, "qkv"):
                qkv = K.gemm_fp8(K.quant_rows_fp8(n1), f8((id(self), "qkv"), a1m.w_qkv),
                                 a2=K.quant_rows_fp8(u_qkv), w2=f8((id(self), "sB_qkv"), L.sB_qkv, ver),
                                 tail_group_n=C, tail_rows=tr)
            else:
                qkv = _gemm_fwd(n1, a1m.w_qkv, a2=u_qkv, w2=L.sB_qkv, tail_group_n=C, tail_rows=tr)
        elif ok8(3 * C, C, "qkv"):
            qkv = K.gemm_fp8(K.quant_rows_fp8(n1), f8((id(self), "qkv"), a1m.w_qkv))
        else:
            qkv = K.gemm(n1, a1m.w_qkv)
        q3 = qkv.view(B, S, 3 * C)
        a1, lse1 = K.attention_fwd(q3[..., :C], q3[..., C:2 * C], q3[..., 2 * C:], a1m.heads)
        a1 = a1.view(M, C)
        o1 = a1m.to_out[0]
        if lo:
            u_o1 = K.gemm(pol(a1), L.A_o1)
            if ok8(C, C, "out"):  # (diagnostic kind, not in the default FP8_KINDS: DESIGN §7 #8 table)
                h1 = K.gemm_fp8(K.quant_rows_fp8(a1), f8((id(self), "o1"), o1.weight), a2=K.quant_rows_fp8(u_o1),
                                w2=f8((id(self), "sB_o1"), L.sB_o1, ver), bias=o1.bias, resid=x, tail_rows=tr)
            else:
                h1 = _gemm_fwd(a1, o1.weight, bias=o1.bias, resid=x, a2=u_o1, w2=L.sB_o1, tail_rows=tr)
        elif ok8(C, C, "out"):
            h1 = K.gemm_fp8(K.quant_rows_fp8(a1), f8((id(self), "o1"), o1.weight), bias=o1.bias, resid=x)
        else:
            h1 = K.gemm(a1, o1.weight, bias=o1.bias, resid=x)
        # --- cross attention over the 77 text tokens ---
        n2, st2 = K.layer_norm_fwd(h1, self.norm2.weight, self.norm2.bias, 1e-5)
        enc = rt.enc  # [B*77, Dc]
        Se = enc.shape[0] // B
        if lo:
            u_q2 = K.gemm(pol(n2), L.A_q2)
            if ok8(C, C, "q2") and "tail" not in FP8_KINDS:  # diagnostics: the LoRA term in bf16
                q2 = K.gemm_fp8(K.quant_rows_fp8(n2), f8((id(self), "q2"), a2m.to_q.weight))
                q2[:Mp].copy_(K.gemm(u_q2, L.sB_q2, resid=q2[:Mp]))
            elif ok8(C, C, "q2"):
                q2 = K.gemm_fp8(K.quant_rows_fp8(n2), f8((id(self), "q2"), a2m.to_q.weight),
                                a2=K.quant_rows_fp8(u_q2), w2=f8((id(self), "sB_q2"), L.sB_q2, ver), tail_rows=tr)
            else:
                q2 = _gemm_fwd(n2, a2m.to_q.weight, a2=u_q2, w2=L.sB_q2, tail_rows=tr)
        elif ok8(C, C, "q2"):
            q2 = K.gemm_fp8(K.quant_rows_fp8(n2), f8((id(self), "q2"), a2m.to_q.weight))
        else:
            q2 = K.gemm(n2, a2m.to_q.weight)
        # K/V of the text tokens: this block's columns of the width-batched projection (UNet2DConditionModel.kv_text)
        kv_all, u_all = rt.kv_text(C)
        j = self._kv_slot
        kv3 = kv_all.view(B, Se, -1)[..., j * 2 * C:(j + 1) * 2 * C]        # [B, 77, 2C] view
        u_kv2 = u_all[:, j * 2 * r:(j + 1) * 2 * r] if lo else None          # [Bp*77, 2r] view
        a2, lse2 = K.attention_fwd(q2.view(B, S, C), kv3[..., :C], kv3[..., C:], a2m.heads)
        a2 = a2.view(M, C)
        o2 = a2m.to_out[0]
        if lo:
            u_o2 = K.gemm(pol(a2), L.A_o2)
            if ok8(C, C, "out"):
                h2 = K.gemm_fp8(K.quant_rows_fp8(a2), f8((id(self), "o2"), o2.weight), a2=K.quant_rows_fp8(u_o2),
                                w2=f8((id(self), "sB_o2"), L.sB_o2, ver), bias=o2.bias, resid=h1, tail_rows=tr)
            else:
                h2 = _gemm_fwd(a2, o2.weight, bias=o2.bias, resid=h1, a2=u_o2, w2=L.sB_o2, tail_rows=tr)
        elif ok8(C, C, "out"):
            h2 = K.gemm_fp8(K.quant_rows_fp8(a2), f8((id(self), "o2"), o2.weight), bias=o2.bias, resid=h1)
        else:
            h2 = K.gemm(a2, o2.weight, bias=o2.bias, resid=h1)
        # --- GEGLU feed-forward ---
        n3, st3 = K.layer_norm_fwd(h2, self.norm3.weight, self.norm3.bias, 1e-5)
        ff = self.ff
        f = torch.empty((Mp, ff.w_int.shape[0]), device=x.device, dtype=BF16) if rt.save else None
        if ok8(ff.w_int.shape[0], C, "ff") and fp8_geglu_pays(M, ff.w_int.shape[0]):
            gg = K.gemm_fp8(K.quant_rows_fp8(n3), f8((id(self), "ff"), ff.w_int), bias=ff.b_int, geglu=True, out_pre=f,
                            pre_rows=Mp)
        else:
            gg = K.gemm_geglu(n3, ff.w_int, ff.b_int, out_pre=f, pre_rows=Mp)  # f: interleaved pre-activation (bwd)
        if ok8(C, ff.out.weight.shape[1], "ffout"):  # ff.net.2 (diagnostic kind: DESIGN §7 #8 table)
            h3 = K.gemm_fp8(K.quant_rows_fp8(gg), f8((id(self), "ffout"), ff.out.weight), bias=ff.out.bias, resid=h2)
        else:
            h3 = K.gemm(gg, ff.out.weight, bias=ff.out.bias, resid=h2)
        if rt.save:  # the backward runs on the policy images only
            sv = dict(x=pol(x), st1=pol(st1), n1=pol(n1), qkv=pol(qkv), a1=pol(a1), lse1=pol(lse1), h1=pol(h1),
                      st2=pol(st2), n2=pol(n2), q2=pol(q2), kv3=pol(kv3), a2=pol(a2), lse2=pol(lse2), h2=pol(h2),
                      st3=pol(st3), f=f)
            if lo:
                sv.update(u_qkv=u_qkv, u_o1=u_o1, u_q2=u_q2, u_kv2=u_kv2, u_o2=u_o2)
            if rt.fg is not None:  # full-UNet grads: the ff.proj / ff.out inputs too
                sv.update(n3=n3, gg=gg)
            rt.saved.append(sv)
        return h3

    def bwd(self, dh3, sv, rt, path, need_dx=True):
        C = self.dim
        B = rt.B
        M = dh3.shape[0]
        S = M // B
        r = rt.r
        lo = rt.lora_on
        st = rt.lora
        L = st.blk[path] if lo else None
        g = (lambda k: st.grad_seg(path, k)) if lo else None
        a1m, a2m = self.attn1, self.attn2
        # --- FF ---
        fg = rt.fg
        df = K.gemm_geglu_bwd(dh3, self.ff.out.wt, sv["f"])  # interleaved d[h | gate]
        if fg is not None:
            _lin_dw(fg, self.ff.out, dh3, sv["gg"], rt)
            n3 = sv["n3"]

            def ff_proj_dw():
                # df's columns are in the GEGLU interleave (per 32 outputs [h 32 | gate 32]): the weight gradient
                # lands in the natural row order from the TN epilogue, the bias sum through a strided view
                F2 = df.shape[1]
                if _GEGLU_TN:
                    K.gemm_tn_geglu(df, n3, fg.g(self.ff.proj.weight))
                else:  # benchmark knob PSO_GEGLU_TN=0: the transient interleaved matrix + index_add (round 3)
                    tmp = torch.zeros((F2, C), device=df.device, dtype=torch.float32)
                    K.gemm_tn(df, n3, tmp)
                    fg.g(self.ff.proj.weight).index_add_(0, K.geglu_interleave_index(F2 // 2, df.device), tmp)
                tb = torch.zeros((1, F2), device=df.device, dtype=torch.float32)
                K.colsum_acc(df, tb)
                fg.g(self.ff.proj.bias).view(2, F2 // 64, 32).add_(tb.view(F2 // 64, 2, 32).transpose(0, 1))
            rt.side.launch(ff_proj_dw, df, n3)
        dn3 = K.gemm(df, self.ff.wt_int)
        if fg is not None:
            h2s, st3 = sv["h2"], sv["st3"]
            rt.side.launch(lambda: K.layer_norm_dparam(h2s, dn3, st3, fg.g(self.norm3.weight), fg.g(self.norm3.bias)),
                           h2s, dn3, st3)
        dh2 = K.layer_norm_bwd(sv["h2"], dn3, sv["st3"], self.norm3.weight, dadd=dh3)
        # --- cross attention out-proj:  y = a W^T + (a A^T)(sB)^T ;  v = dy sB ; da = dy W + v A ---
        o2 = a2m.to_out[0]
        if lo:
            v_o2 = K.gemm(dh2, L.sBt_o2)
            da2 = K.gemm(dh2, o2.wt, a2=v_o2, w2=L.At_o2)
            a2s, uo2 = sv["a2"], sv["u_o2"]
            rt.side.launch(lambda: (rt.dw(v_o2, a2s, g("attn2.A_o")), rt.dw(dh2, uo2, g("attn2.B_o"), st.scale)),
                           v_o2, a2s, dh2, uo2)
        else:
            da2 = K.gemm(dh2, o2.wt)
        if fg is not None:
            _lin_dw(fg, o2, dh2, sv["a2"], rt)
        enc = rt.enc
        Se = enc.shape[0] // B
        kv3 = sv["kv3"]
        dkv2 = torch.empty((B * Se, 2 * C), device=dh3.device, dtype=BF16)
        dk3 = dkv2.view(B, Se, 2 * C)
        dq2, _, _ = K.attention_bwd(sv["q2"].view(B, S, C), kv3[..., :C], kv3[..., C:], sv["a2"].view(B, S, C),
                                    sv["lse2"], da2.view(B, S, C), a2m.heads, dk=dk3[..., :C], dv=dk3[..., C:])
        dq2 = dq2.view(M, C)
        if lo:
            v_q2 = K.gemm(dq2, L.sBt_q2)
            dn2 = K.gemm(dq2, a2m.to_q.wt, a2=v_q2, w2=L.At_q2)
            n2s, uq2, enc_, u_kv2 = sv["n2"], sv["u_q2"], rt.enc, sv["u_kv2"]
            # k/v adapters of the text tokens: v_kv = [dk sB_k | dv sB_v] on the compute stream -- the deferred
            # weight-gradient queue (rt.dw) is flushed there, so its operands must not come from the side stream
            v_kv = K.gemm_grouped_skinny(dkv2, L.sBt_kv2, 2)

            def dw_attn2():
                rt.dw(v_q2, n2s, g("attn2.A_q"))
                rt.dw(dq2, uq2, g("attn2.B_q"), st.scale)
                # dA_kv += v_kv^T enc; dB_kv += s dkv^T u
                rt.dw(v_kv, enc_, g("attn2.A_kv"))
                gB = g("attn2.B_kv")
                if r in K.TN_RANKS:
                    rt.dw(dkv2, u_kv2, gB, st.scale, group=C)
                else:
                    rt.dw(dkv2[:, :C], u_kv2[:, :r], gB[:C], st.scale)
                    rt.dw(dkv2[:, C:], u_kv2[:, r:], gB[C:], st.scale)
            rt.side.launch(dw_attn2, v_q2, n2s, dq2, uq2, dkv2, enc_, u_kv2, v_kv)
        else:
            dn2 = K.gemm(dq2, a2m.to_q.wt)
        if fg is not None:
            n2, h1s, st2 = sv["n2"], sv["h1"], sv["st2"]

            def attn2_dw():
                K.gemm_tn(dq2, n2, fg.g(a2m.to_q.weight))
                _tn_stacked(fg, (a2m.to_k, a2m.to_v), dkv2, enc)
                K.layer_norm_dparam(h1s, dn2, st2, fg.g(self.norm2.weight), fg.g(self.norm2.bias))
            rt.side.launch(attn2_dw, dq2, n2, dkv2, enc, h1s, dn2, st2)
        dh1 = K.layer_norm_bwd(sv["h1"], dn2, sv["st2"], self.norm2.weight, dadd=dh2)
        # --- self attention ---
        o1 = a1m.to_out[0]
        if lo:
            v_o1 = K.gemm(dh1, L.sBt_o1)
            da1 = K.gemm(dh1, o1.wt, a2=v_o1, w2=L.At_o1)
            a1s, uo1 = sv["a1"], sv["u_o1"]
            rt.side.launch(lambda: (rt.dw(v_o1, a1s, g("attn1.A_o")), rt.dw(dh1, uo1, g("attn1.B_o"), st.scale)),
                           v_o1, a1s, dh1, uo1)
        else:
            da1 = K.gemm(dh1, o1.wt)
        if fg is not None:
            _lin_dw(fg, o1, dh1, sv["a1"], rt)
        q3 = sv["qkv"].view(B, S, 3 * C)
        dqkv = torch.empty((M, 3 * C), device=dh3.device, dtype=BF16)
        d3 = dqkv.view(B, S, 3 * C)
        K.attention_bwd(q3[..., :C], q3[..., C:2 * C], q3[..., 2 * C:], sv["a1"].view(B, S, C), sv["lse1"],
                        da1.view(B, S, C), a1m.heads, dq=d3[..., :C], dk=d3[..., C:2 * C], dv=d3[..., 2 * C:])
        if lo:
            v_qkv = K.gemm_grouped_skinny(dqkv, L.sBt_qkv, 3)
            dn1 = K.gemm(dqkv, a1m.wt_qkv, a2=v_qkv, w2=L.At_qkv) if need_dx else None
            n1s, u_qkv = sv["n1"], sv["u_qkv"]

            def dw_attn1():
                rt.dw(v_qkv, n1s, g("attn1.A_qkv"))
                gB = g("attn1.B_qkv")
                if r in K.TN_RANKS:
                    rt.dw(dqkv, u_qkv, gB, st.scale, group=C)
                else:
                    for j in range(3):
                        rt.dw(dqkv[:, j * C:(j + 1) * C], u_qkv[:, j * r:(j + 1) * r], gB[j * C:(j + 1) * C],
                                  st.scale)
            rt.side.launch(dw_attn1, v_qkv, n1s, dqkv, u_qkv)
        else:
            dn1 = K.gemm(dqkv, a1m.wt_qkv) if need_dx else None
        if fg is not None:
            n1, xs, st1 = sv["n1"], sv["x"], sv["st1"]

            def attn1_dw():
                _tn_stacked(fg, (a1m.to_q, a1m.to_k, a1m.to_v), dqkv, n1)
                if dn1 is not None:
                    K.layer_norm_dparam(xs, dn1, st1, fg.g(self.norm1.weight), fg.g(self.norm1.bias))
            rt.side.launch(attn1_dw, dqkv, n1, xs, st1, *((dn1,) if dn1 is not None else ()))
        if not need_dx:  # first adapter block: nothing below it needs a gradient
            return None
        return K.layer_norm_bwd(sv["x"], dn1, sv["st1"], self.norm1.weight, dadd=dh1)


class SimpleFF(nn.Module):
    """diffusers FeedForward(dim, activation_fn="geglu"): net.0 = GEGLU(proj: dim -> 8*dim), net.2 = Linear(4dim->dim)."""

    def __init__(self, dim):
        super().__init__()
        self.proj = Linear(dim, 8 * dim)
        self.out = Linear(4 * dim, dim)

    def prepare(self):
        # rows interleaved per 32 outputs as [h 32 | gate 32] so the GEMM epilogue holds both halves of a GEGLU
        # output in one lane (pso_gemm_geglu); the pre-activation and its gradient live in that order internally
        F = self.out.in_features
        idx = K.geglu_interleave_index(F, self.proj.weight.device)
        self.w_int = self.proj.weight.data[idx].contiguous()
        self.b_int = self.proj.bias.data[idx].contiguous()
        self.wt_int = K.transpose(self.w_int)  # [dim][2F] for the input gradient
        self.out.prepare()

    def _remap(self):
        return {"net.0.proj": self.proj, "net.2": self.out}


class Transformer2DModel(nn.Module):
    """use_linear_projection=True: GN(eps 1e-6) -> proj_in -> blocks -> proj_out + residual."""

    def __init__(self, C, depth, cross_dim, groups):
        super().__init__()
        self.C, self.groups = C, groups
        self.norm = Norm(C)
        self.proj_in = Linear(C, C)
        self.transformer_blocks = nn.ModuleList([BasicTransformerBlock(C, cross_dim) for _ in range(depth)])
        self.proj_out = Linear(C, C)

    def prepare(self):
        self.proj_in.prepare()
        self.proj_out.prepare()
        for b in self.transformer_blocks:
            b.prepare()

    def fwd(self, x, rt, path):
        """x NHWC [B,H,W,C] -> same shape."""
        B, H, W, C = x.shape
        xn, st = K.group_norm_fwd(x, self.norm.weight, self.norm.bias, self.groups, 1e-6, False)
        h = K.gemm(xn.view(-1, C), self.proj_in.weight, bias=self.proj_in.bias)
        if rt.save:
            rt.saved.append({"x": rt.pol(x), "st": rt.pol(st), "xn": xn.view(-1, C) if rt.fg is not None else None})
        for i, blk in enumerate(self.transformer_blocks):
            h = blk.fwd(h, rt, f"{path}.transformer_blocks.{i}")
        if rt.save and rt.fg is not None:
            rt.saved.append({"hout": h})
        return K.gemm(h, self.proj_out.weight, bias=self.proj_out.bias, resid=x.view(-1, C)).view(B, H, W, C)

    def bwd(self, dy, rt, path, need_dx=True):
        B, H, W, C = dy.shape
        d2 = dy.view(-1, C)
        fg = rt.fg
        if fg is not None:
            _lin_dw(fg, self.proj_out, d2, rt.saved.pop()["hout"], rt)
        dh = K.gemm(d2, self.proj_out.wt)
        for i in reversed(range(len(self.transformer_blocks))):
            dh = self.transformer_blocks[i].bwd(dh, rt.saved.pop(), rt, f"{path}.transformer_blocks.{i}",
                                                need_dx=need_dx or i > 0)
        sv = rt.saved.pop()
        if not need_dx:
            return None
        dn = K.gemm(dh, self.proj_in.wt).view(B, H, W, C)
        if fg is not None:
            _lin_dw(fg, self.proj_in, dh, sv["xn"], rt)
            return K.group_norm_bwd(sv["x"], dn, sv["st"], self.norm.weight, self.norm.bias, False, dadd=dy,
                                    dgamma=fg.g(self.norm.weight), dbeta=fg.g(self.norm.bias), accumulate=True)
        return K.group_norm_bwd(sv["x"], dn, sv["st"], self.norm.weight, self.norm.bias, False, dadd=dy)


class ResnetBlock2D(nn.Module):
    def __init__(self, cin, cout, groups, eps, temb_dim):
        super().__init__()
        self.cin, self.cout, self.groups, self.eps = cin, cout, groups, eps
        self.norm1 = Norm(cin)
        self.conv1 = Conv2d(cin, cout, 3)
        self.time_emb_proj = Linear(temb_dim, cout) if temb_dim else None
        self.norm2 = Norm(cout)
        self.conv2 = Conv2d(cout, cout, 3)
        self.conv_shortcut = Conv2d(cin, cout, 1) if cin != cout else None

    def prepare(self):
        self.conv1.prepare()
        self.conv2.prepare()
        if self.conv_shortcut is not None:
            self.conv_shortcut.prepare()

    def fwd(self, x, rt, temb=None):
        """x NHWC [B,H,W,Ci]; temb [B, Co] row view (time_emb_proj output) or None."""
        h1, st1 = K.group_norm_fwd(x, self.norm1.weight, self.norm1.bias, self.groups, self.eps, True)
        c1 = K.conv2d(h1, self.conv1.w_nhwc, bias=self.conv1.bias, rowbias=temb)
        h2, st2 = K.group_norm_fwd(c1, self.norm2.weight, self.norm2.bias, self.groups, self.eps, True)
        if self.conv_shortcut is not None:
            B, H, W, _ = x.shape
            sc = K.gemm(x.view(-1, self.cin), self.conv_shortcut.w_mat, bias=self.conv_shortcut.bias)
            sc = sc.view(B, H, W, self.cout)
        else:
            sc = x
        out = K.conv2d(h2, self.conv2.w_nhwc, bias=self.conv2.bias, resid=sc)
        if rt.save:
            sv = {"x": rt.pol(x), "st1": rt.pol(st1), "c1": rt.pol(c1), "st2": rt.pol(st2)}
            if rt.fg is not None:  # conv inputs for the weight grads
                sv.update(h1=h1, h2=h2)
            rt.saved.append(sv)
        return out

    def bwd(self, dout, rt):
        sv = rt.saved.pop()
        fg = rt.fg
        B, H, W, _ = dout.shape
        dh2 = K.conv2d(dout, self.conv2.w_dx)
        if fg is not None:
            _conv_dw(fg, self.conv2, dout.view(-1, self.cout), sv["h2"], rt, K.im2col_conv)
            dc1 = K.group_norm_bwd(sv["c1"], dh2, sv["st2"], self.norm2.weight, self.norm2.bias, True,
                                   dgamma=fg.g(self.norm2.weight), dbeta=fg.g(self.norm2.bias), accumulate=True)
            dc2 = dc1.view(-1, self.cout)
            _conv_dw(fg, self.conv1, dc2, sv["h1"], rt, K.im2col_conv)
            # time-embedding row bias (one row per image): per-image column sums -> the time_emb_proj output grad
            K.colsum_acc(dc2, rt.dtemb[:, self._temb_off:self._temb_off + self.cout], rows_per_group=H * W)
        else:
            dc1 = K.group_norm_bwd(sv["c1"], dh2, sv["st2"], self.norm2.weight, self.norm2.bias, True)
        dh1 = K.conv2d(dc1, self.conv1.w_dx)
        if self.conv_shortcut is not None:
            dsc = K.gemm(dout.view(-1, self.cout), self.conv_shortcut.wt).view(B, H, W, self.cin)
            if fg is not None:
                d2, x2 = dout.view(-1, self.cout), sv["x"].view(-1, self.cin)
                sc = self.conv_shortcut

                def sc_dw():
                    K.gemm_tn(d2, x2, fg.g(sc.weight).view(self.cout, self.cin))
                    K.colsum_acc(d2, fg.g(sc.bias).view(1, -1))
                rt.side.launch(sc_dw, d2, x2)
        else:
            dsc = dout
        if fg is not None:
            return K.group_norm_bwd(sv["x"], dh1, sv["st1"], self.norm1.weight, self.norm1.bias, True, dadd=dsc,
                                    dgamma=fg.g(self.norm1.weight), dbeta=fg.g(self.norm1.bias), accumulate=True)
        return K.group_norm_bwd(sv["x"], dh1, sv["st1"], self.norm1.weight, self.norm1.bias, True, dadd=dsc)


class Downsample2D(nn.Module):
    def __init__(self, C):
        super().__init__()
        self.conv = Conv2d(C, C, 3, stride=2)

    def prepare(self):
        self.conv.prepare()

    def fwd(self, x, rt):
        if rt.save:
            rt.saved.append({"hw": x.shape[1:3], "x": x if rt.fg is not None else None})
        return K.conv2d(x, self.conv.w_nhwc, stride=2, bias=self.conv.bias)

    def bwd(self, dy, rt):
        sv = rt.saved.pop()
        if rt.fg is not None:
            _conv_dw(rt.fg, self.conv, dy.reshape(-1, self.conv.cout), sv["x"], rt,
                     lambda x: K.im2col_conv(x, stride=2))
        return K.conv2d(dy, self.conv.w_dx, mode=K.CONV_T2, out_hw=tuple(sv["hw"]))


class Upsample2D(nn.Module):
    def __init__(self, C):
        super().__init__()
        self.conv = Conv2d(C, C, 3)

    def prepare(self):
        self.conv.prepare()

    def fwd(self, x, rt):
        if rt.save and rt.fg is not None:
            rt.saved.append({"x": x})
        return K.conv2d(x, self.conv.w_nhwc, mode=K.CONV_UP2, bias=self.conv.bias)

    def bwd(self, dy, rt):
        if rt.fg is not None:
            _conv_dw(rt.fg, self.conv, dy.reshape(-1, self.conv.cout), rt.saved.pop()["x"], rt,
                     lambda x: K.im2col_conv(x, mode=K.CONV_UP2))
        du = K.conv2d(dy, self.conv.w_dx)  # input-gradient on the 2x grid
        return K.sumpool2(du)


class _Block(nn.Module):
    """down / up / mid block container with diffusers child names."""

    def __init__(self):
        super().__init__()


class TimestepEmbedding(nn.Module):
    def __init__(self, fin, dim):
        super().__init__()
        self.linear_1 = Linear(fin, dim)
        self.linear_2 = Linear(dim, dim)


# ======================================================================================================================
# the model
# ======================================================================================================================
class _Output(SimpleNamespace):
    pass


class UNet2DConditionModel(nn.Module):
    def __init__(self, config: UNetConfig = None):
        super().__init__()
        cfg = config or UNetConfig.sdxl()
        self.cfg = cfg
        self.config = SimpleNamespace(in_channels=cfg.in_channels, out_channels=cfg.out_channels,
                                      sample_size=cfg.sample_size, block_out_channels=cfg.block_out_channels,
                                      cross_attention_dim=cfg.cross_attention_dim,
                                      addition_time_embed_dim=cfg.addition_time_embed_dim,
                                      projection_class_embeddings_input_dim=cfg.projection_class_embeddings_input_dim)
        ch = cfg.block_out_channels
        G, eps, tdim = cfg.norm_num_groups, cfg.norm_eps, cfg.time_embed_dim
        self.conv_in = Conv2d(cfg.in_channels, ch[0], 3)
        self.time_embedding = TimestepEmbedding(cfg.time_proj_dim, tdim)
        self.add_embedding = TimestepEmbedding(cfg.projection_class_embeddings_input_dim, tdim)
        nlev = len(ch)
        self.down_blocks = nn.ModuleList()
        cin = ch[0]
        for i in range(nlev):
            blk = _Block()
            blk.resnets = nn.ModuleList()
            if cfg.down_has_attn[i]:
                blk.attentions = nn.ModuleList()
            for j in range(cfg.layers_per_block):
                blk.resnets.append(ResnetBlock2D(cin if j == 0 else ch[i], ch[i], G, eps, tdim))
                if cfg.down_has_attn[i]:
                    blk.attentions.append(Transformer2DModel(ch[i], cfg.transformer_layers_per_block[i],
                                                             cfg.cross_attention_dim, G))
            if i < nlev - 1:
                blk.downsamplers = nn.ModuleList([Downsample2D(ch[i])])
            cin = ch[i]
            self.down_blocks.append(blk)
        mid = _Block()
        mid.resnets = nn.ModuleList([ResnetBlock2D(ch[-1], ch[-1], G, eps, tdim),
                                     ResnetBlock2D(ch[-1], ch[-1], G, eps, tdim)])
        mid.attentions = nn.ModuleList([Transformer2DModel(ch[-1], cfg.transformer_layers_per_block[-1],
                                                           cfg.cross_attention_dim, G)])
        self.mid_block = mid
        self.up_blocks = nn.ModuleList()
        rch = list(reversed(ch))
        rattn = list(reversed(cfg.down_has_attn))
        rdepth = list(reversed(cfg.transformer_layers_per_block))
        prev = ch[-1]
        for i in range(nlev):
            out_c = rch[i]
            in_c = rch[min(i + 1, nlev - 1)]
            blk = _Block()
            blk.resnets = nn.ModuleList()
            if rattn[i]:
                blk.attentions = nn.ModuleList()
            n = cfg.layers_per_block + 1
            for j in range(n):
                skip_c = in_c if j == n - 1 else out_c
                res_in = prev if j == 0 else out_c
                blk.resnets.append(ResnetBlock2D(res_in + skip_c, out_c, G, eps, tdim))
                if rattn[i]:
                    blk.attentions.append(Transformer2DModel(out_c, rdepth[i], cfg.cross_attention_dim, G))
            if i < nlev - 1:
                blk.upsamplers = nn.ModuleList([Upsample2D(out_c)])
            prev = out_c
            self.up_blocks.append(blk)
        self.conv_norm_out = Norm(ch[0])
        self.conv_out = Conv2d(ch[0], cfg.out_channels, 3)
        self.lora = None
        self.full = None  # FullGradState when every parameter is trained (C3 / C4)
        self.fp8 = False  # fp8 forward of the LayerNorm-fed projections (enable_fp8_forward, config 5)
        self._fp8_cache = {}
        self._adapters_enabled = True
        self._prepared = False
        self.gradient_checkpointing = False

    # ---------------- parameter plumbing ----------------
    def _remap_key(self, k):
        return k.replace(".ff.net.0.proj.", ".ff.proj.").replace(".ff.net.2.", ".ff.out.")

    def _unmap_key(self, k):
        return k.replace(".ff.proj.", ".ff.net.0.proj.").replace(".ff.out.", ".ff.net.2.")

    def state_dict(self, *a, **kw):
        sd = super().state_dict(*a, **kw)
        return {self._unmap_key(k): v for k, v in sd.items()}

    def load_state_dict(self, sd, strict=True):
        sd = {self._remap_key(k): v for k, v in sd.items()}
        res = super().load_state_dict({k: v.to(BF16) for k, v in sd.items()}, strict=strict)
        self._prepared = False
        return res

    @classmethod
    def from_config(cls, config=None, **kw):
        """`UNet2DConditionModel.from_config(cfg)` (D:313-318): a UNetConfig, or a diffusers config dict (the keys of
        `unet/config.json`, validated against what the kernels implement: diffusers_io.unet_config_from_diffusers);
        None -> SDXL.  Weights are left uninitialised, as diffusers leaves them before load_state_dict."""
        from . import diffusers_io
        if config is None:
            config = UNetConfig.sdxl()
        elif isinstance(config, dict):
            config = diffusers_io.unet_config_from_diffusers(dict(config, **kw))
        elif not isinstance(config, UNetConfig):
            raise TypeError(f"from_config takes a UNetConfig or a diffusers config dict, not {type(config).__name__}")
        return cls(config)

    @classmethod
    def load_config(cls, path, subfolder=None, **kw):
        from . import diffusers_io
        return diffusers_io.load_config(path, subfolder)

    @classmethod
    def from_pretrained(cls, path, subfolder=None, torch_dtype=None, variant=None, revision=None, **kw):
        """`UNet2DConditionModel.from_pretrained(path, subfolder="unet")` (T:290) from a local diffusers directory:
        config.json + diffusion_pytorch_model[.variant].safetensors (bf16 weights; torch_dtype / revision are
        accepted for API parity -- the kernels compute in bf16)."""
        from . import diffusers_io
        model = cls.from_config(diffusers_io.load_config(path, subfolder))
        model.load_state_dict(diffusers_io.load_weights(path, subfolder, variant))
        return model

    def save_pretrained(self, path):
        from . import diffusers_io
        diffusers_io.save_pretrained(self, path, diffusers_io.unet_config_to_diffusers(self.cfg))

    def init_weights(self, seed=0):
        """PyTorch-default-style seeded init (the BASELINE synthetic-weights recipe); norms at identity."""
        g = torch.Generator(device=self.conv_in.weight.device).manual_seed(seed)
        for m in self.modules():
            if isinstance(m, (Linear, Conv2d, Norm)):
                m.reset(g)
        self._prepared = False
        return self

    def enable_gradient_checkpointing(self):
        self.gradient_checkpointing = True  # accepted for API parity; activations are kept (288 GB HBM)

    def _attn_modules(self):
        for name, m in self.named_modules():
            if isinstance(m, BasicTransformerBlock):
                yield name, m

    def add_adapter(self, lora_config):
        """peft LoraConfig(r, lora_alpha, init_lora_weights='gaussian', target_modules=[to_k,to_q,to_v,to_out.0])
        (T:338-345, D:361-366, DB:1319-1325).  The kernels implement exactly that adapter set: every LoraConfig field
        is checked (check_lora_config) and anything else raises instead of training other adapters than asked."""
        r, alpha = check_lora_config(lora_config)
        blocks = [(name, blk.dim, blk.attn2.kv_dim) for name, blk in self._attn_modules()]
        dev = self.conv_in.weight.device
        self.lora = LoraState(blocks, r, alpha, dev)
        if dev.type == "cuda":
            self.lora.init_gaussian(seed=getattr(lora_config, "seed", 0))
        self._adapters_enabled = True
        return self.lora

    def grad_units(self):
        """[(unit, [parameter names])] in the order backward_nhwc finishes them: conv_out / conv_norm_out, the up blocks
        (upsampler, then per layer its attention and resnet, last layer first), the mid block, the down blocks, and
        finally the embedding unit (conv_in, both embedding MLPs and every resnet's time_emb_proj, whose gradients
        are formed from the accumulated time-embedding gradient after the sweep).  backward_nhwc calls
        rt.unit_done(unit) at each of these points."""
        units = [("conv_out", ["conv_out.weight", "conv_out.bias", "conv_norm_out.weight", "conv_norm_out.bias"])]
        named = [n for n, _ in self.named_parameters()]

        def under(prefix):
            return [n for n in named if n.startswith(prefix + ".") and ".time_emb_proj." not in n]

        for i in reversed(range(len(self.up_blocks))):
            blk = self.up_blocks[i]
            if hasattr(blk, "upsamplers"):
                units.append((f"up_blocks.{i}.upsamplers.0", under(f"up_blocks.{i}.upsamplers.0")))
            for j in reversed(range(len(blk.resnets))):
                if hasattr(blk, "attentions"):
                    units.append((f"up_blocks.{i}.attentions.{j}", under(f"up_blocks.{i}.attentions.{j}")))
                units.append((f"up_blocks.{i}.resnets.{j}", under(f"up_blocks.{i}.resnets.{j}")))
        for u in ("mid_block.resnets.1", "mid_block.attentions.0", "mid_block.resnets.0"):
            units.append((u, under(u)))
        for i in reversed(range(len(self.down_blocks))):
            blk = self.down_blocks[i]
            if hasattr(blk, "downsamplers"):
                units.append((f"down_blocks.{i}.downsamplers.0", under(f"down_blocks.{i}.downsamplers.0")))
            for j in reversed(range(len(blk.resnets))):
                if hasattr(blk, "attentions"):
                    units.append((f"down_blocks.{i}.attentions.{j}", under(f"down_blocks.{i}.attentions.{j}")))
                units.append((f"down_blocks.{i}.resnets.{j}", under(f"down_blocks.{i}.resnets.{j}")))
        # the resnets' time_emb_proj weights, then their biases, each set back to back (the batched projection reads
        # them as one [sum Co][tdim] matrix / [sum Co] vector: zero-copy views of the full-UNet working copy)
        units.append(("embed", [n for n in named if n.startswith(("conv_in.", "time_embedding.", "add_embedding."))]
                      + [n for n in named if n.endswith(".time_emb_proj.weight")]
                      + [n for n in named if n.endswith(".time_emb_proj.bias")]))
        return units

    def grad_unit_ranges(self):
        """[(unit, offset, numel)] of the trained flat gradient (LoRA bucket or full-UNet grad) in backward completion
        order; every unit is one contiguous range (checked).  Units holding nothing trainable are dropped."""
        out = []
        if self.full is not None:
            for unit, names in self.grad_units():
                rs = sorted(self.full.offsets[n] for n in names if n in self.full.offsets)
                if rs:
                    out.append((unit, rs[0][0], sum(k for _, k in rs)))
        elif self.lora is not None:
            for unit, _ in self.grad_units():
                rs = sorted((seg[0], seg[1] * seg[2]) for path, segs in self.lora.layout.items()
                            if path.startswith(unit + ".") for seg in segs.values())
                if rs:
                    out.append((unit, rs[0][0], sum(k for _, k in rs)))
        for (_, o, k), (_, o2, _) in zip(out, out[1:]):
            assert o + k == o2, "gradient units must tile the flat buffer in completion order"
        return out

    def enable_full_grads(self):
        """Train every UNet parameter (BASELINE C3 / C4; the reference has no such path, App. A #4): flat fp32
        master + grad over named_parameters; backward_nhwc then accumulates every weight gradient into self.full.grad
        and runs down to conv_in.  Adapters, if any, must be absent."""
        if self.lora is not None:
            raise ValueError("full-UNet training and LoRA adapters are exclusive")
        self.full = FullGradState(self)
        return self.full

    def refresh_full(self, cast=True):
        """After an optimizer step on self.full.master: bf16 module weights + kernel-layout caches."""
        self.full.refresh(cast)
        self.prepare()

    def disable_adapters(self):
        self._adapters_enabled = False

    def enable_adapters(self):
        self._adapters_enabled = True

    def lora_parameters(self):
        return [self.lora.param] if self.lora is not None else []

    def prepare(self):
        """Derive kernel-layout weight caches (one-time after load; weights are frozen in LoRA training; the full-UNet
        step re-runs it after every optimizer step): every transposed weight in ONE batched launch."""
        with K.transpose_batch():
            self._prepare_caches()
        self._prepared = True
        if self.lora is not None:
            self.refresh_lora()

    def _prepare_caches(self):
        for m in self.modules():
            if isinstance(m, (Transformer2DModel, ResnetBlock2D, Downsample2D, Upsample2D)):
                m.prepare()
        # the time-embedding projections of all resnets as ONE GEMM
        res = [m for m in self.modules() if isinstance(m, ResnetBlock2D)]
        self._temb_w = _stacked([m.time_emb_proj.weight.data for m in res])
        self._temb_b = _stacked([m.time_emb_proj.bias.data for m in res])
        off = 0
        for m in res:
            m._temb_off = off
            off += m.cout
        self._temb_n = off
        # Cross-attention K/V: every transformer block projects the SAME 77 text tokens, so the blocks of one width run
        # their K/V projections as ONE GEMM (weights concatenated here, each block's w_kv a row view of them): 2 launches
        # per pass instead of 2 per block (the LoRA k/v down-projections likewise, see refresh_lora)
        groups = {}
        for _, blk in self._attn_modules():
            groups.setdefault(blk.dim, []).append(blk)
        self._kv_groups = {}
        for C, lst in groups.items():
            W = torch.cat([b.attn2.w_kv for b in lst], 0)
            for j, b in enumerate(lst):
                b.attn2.w_kv = W[j * 2 * C:(j + 1) * 2 * C]
                b._kv_slot = j
            self._kv_groups[C] = SimpleNamespace(W=W, blocks=lst)
        self.conv_in.prepare()
        self.conv_out.prepare()
        if self.full is not None:
            self._temb_wt = K.transpose(self._temb_w)  # [tdim][sum Co]: input gradient of the batched projection
            for lin in (self.time_embedding.linear_1, self.time_embedding.linear_2, self.add_embedding.linear_1,
                        self.add_embedding.linear_2):
                lin.prepare()
        self._fp8_cache = {}  # kernel-layout weights may have been rebuilt

    def refresh_lora(self, cast=True):
        self.lora.refresh(cast)

    # ---------------- fp8 forward (BASELINE config 5) ----------------
    def enable_fp8_forward(self, on=True):
        """Run the LayerNorm-fed projections of every transformer block named in FP8_KINDS -- the cross-attention q
        and the GEGLU ff.net.0.proj by default -- on fp8 e4m3 MFMA (pso_gemm_fp8: per-token activation scales,
        per-output-channel weight scales, the LoRA up-projection as an fp8 K-tail); everything else, and the whole
        backward, stays bf16 (BASELINE config 5: "fp8 MFMA UNet fwd + bf16 bwd").  The fused self-attention q/k/v
        ("qkv") is kept out by default: e4m3 q and k move the softmax logits, and on the C5 micro-step it alone
        carries a 7.5e-2 LoRA-gradient error (cross q 5.6e-3, GEGLU proj 3.5e-2; tools/diag_fp8_grads.py) while running
        slower than bf16.  Shapes the fp8 kernel does not take (N % 256 or K % 128 != 0) stay bf16.  LoRA training
        only (the base weights are quantised once and cached)."""
        if on and self.full is not None:
            raise ValueError("fp8 forward: LoRA training only (the full-UNet mode updates the base weights)")
        self.fp8 = bool(on)
        self._fp8_cache = {}
        return self

    def _fp8_weight(self, key, w, version=0):
        """(e4m3 [N, K], E8M0 [N]) of a weight, quantised per output channel.  Frozen base weights (version 0) are
        quantised once and cached.  The LoRA sB stacks (version > 0) change at every optimizer step: eager forwards
        re-quantise them once per LoRA version into buffers allocated once; under a hipGraph capture every forward
        re-quantises, so the capture records the quantisation kernel and each replay reads the current LoRA weights (a
        version-keyed cache hit would record nothing and replay the capture-time copies).  A quantisation recorded by
        a capture has not run yet, so its entry is marked stale (-1): the next eager forward re-quantises."""
        capturing = torch.cuda.is_current_stream_capturing()
        hit = self._fp8_cache.get(key)
        if hit is not None and hit[1][0].shape == w.shape:
            # a valid entry serves eager forwards, and captures of the frozen weights (computed eagerly before)
            if hit[0] == version and (version == 0 or not capturing):
                return hit[1]
            q, e = hit[1]
            K.quant_rows_fp8(w, q=q, e=e)
            buf = hit[1]
        else:
            buf = K.quant_rows_fp8(w)
        self._fp8_cache[key] = (-1 if capturing else version, buf)
        return buf

    def kv_text(self, rt, C):
        """K/V of the text tokens for every block of width C: ([rows, n*2C], LoRA down-projection [policy rows, n*2r]
        or None), computed on first use in a pass (rt.enc is then final: the paired duplication precedes every
        transformer block).  Output column group j (C columns: k or v of block j // 2) takes the LoRA tail
        u[:, j*r:(j+1)*r] (sB)^T -- the per-block grouped tail of the unbatched form, block after block."""
        hit = rt.kv_cache.get(C)
        if hit is not None:
            return hit
        grp = self._kv_groups[C]
        enc = rt.enc
        if rt.lora_on:
            A, sB = self.lora.kv_stacks[C][:2]  # same block order as grp.W (both follow _attn_modules)
            u = K.gemm(rt.pol(enc), A)
            kv = _gemm_fwd(enc, grp.W, a2=u, w2=sB, tail_group_n=C, tail_rows=enc.shape[0] // 2 if rt.paired else 0)
        else:
            u, kv = None, K.gemm(enc, grp.W)
        rt.kv_cache[C] = (kv, u)
        return kv, u

    # ---------------- forward / backward ----------------
    def _runtime(self, B, enc, save, lora_on):
        fg = self.full if save else None
        # full-UNet weight gradients run on the side stream beside the input-gradient GEMMs they do not feed (the
        # small-M dX and dW products each leave most CUs idle; GradBuckets joins it before each bucket's all-reduce)
        side = K.SideStream(enabled=True) if (fg is not None and _FULL_SIDE) else K.SideStream()
        rt = SimpleNamespace(B=B, enc=enc, save=save, saved=[], lora_on=lora_on, paired=False, side=side, fg=fg)
        rt.pol = lambda t: t[:t.shape[0] // 2] if rt.paired else t
        rt.kv_cache = {}
        rt.kv_text = lambda C: self.kv_text(rt, C)
        rt.lora = self.lora
        rt.r = self.lora.r if lora_on else 0
        rt.fp8 = self._fp8_weight if self.fp8 else None
        return rt

    def _embed(self, timestep, time_ids, text_embeds, B, dev):
        cfg = self.cfg
        t = torch.as_tensor(timestep, device=dev).float().reshape(-1)
        if t.numel() == 1:
            t = t.expand(B).contiguous()
        te = K.timestep_embedding(t, cfg.time_proj_dim)
        l1, l2 = self.time_embedding.linear_1, self.time_embedding.linear_2
        t1 = K.gemm(te, l1.weight, bias=l1.bias)
        s1 = K.silu(t1)
        emb = K.gemm(s1, l2.weight, bias=l2.bias)
        tid = K.timestep_embedding(time_ids.reshape(-1), cfg.addition_time_embed_dim).view(B, -1)
        add_in = K.concat_channels(text_embeds.to(BF16).contiguous(), tid)
        a1, a2 = self.add_embedding.linear_1, self.add_embedding.linear_2
        u1 = K.gemm(add_in, a1.weight, bias=a1.bias)
        s2 = K.silu(u1)
        emb = K.gemm(s2, a2.weight, bias=a2.bias, resid=emb)
        se = K.silu(emb)
        self._emb_saved = dict(te=te, t1=t1, s1=s1, add_in=add_in, u1=u1, s2=s2, emb=emb, se=se)
        return K.gemm(se, self._temb_w, bias=self._temb_b)  # [B, sum Co]

    def forward_nhwc(self, x, timestep, enc, text_embeds, time_ids, save=False, paired_ref=False):
        """Core forward.  x NHWC bf16 [B,h,w,4]; enc [B,77,Dc]; returns eps NHWC bf16 [B,h,w,4].

        paired_ref=True (the PSO micro-step, T:775-805): ONE pass yields the policy eps (adapters on) AND the reference
        eps (adapters disabled) of the same inputs, returned as [2B,h,w,4] = [policy; reference].  Everything below
        the first adapter-carrying attention is adapter-free, so it runs once on the B images and is then duplicated;
        from there on the batch is [policy; reference] and every adapter acts on the policy rows only (pso_gemm
        tail_rows).  save=True keeps the policy half of what the backward needs."""
        if not self._prepared:
            self.prepare()
        B = x.shape[0]
        lora_on = self.lora is not None and self._adapters_enabled
        encf = enc.to(BF16).reshape(B * enc.shape[1], enc.shape[2]).contiguous()
        rt = self._runtime(B, encf, save, lora_on)
        temb_all = self._embed(timestep, time_ids, text_embeds, B, x.device)
        tb = lambda m: temb_all[:, m._temb_off:m._temb_off + m.cout]
        # conv_in (C=4): im2col GEMM
        _, H, W, _ = x.shape
        cols = K.im2col3(x, self.conv_in.kp)
        h = K.gemm(cols, self.conv_in.w_col, bias=self.conv_in.bias).view(B, H, W, -1)
        skips = [h]
        i0, j0 = self._first_attn
        full = rt.fg is not None
        if full and paired_ref:
            raise ValueError("full-UNet training: the reference is a separate frozen UNet, not the adapter-free pass")
        if full:
            rt.emb = self._emb_saved
            rt.cols_in = cols
            i0, j0 = -1, -1  # everything is differentiated: no adapter-free prefix
        else:
            rt.save = False  # the prefix below the first adapter block is never differentiated (backward_nhwc)
        for i, blk in enumerate(self.down_blocks):
            for j, res in enumerate(blk.resnets):
                if (i, j) == (i0, j0):  # entering the adapter-carrying part
                    rt.save = save
                    if paired_ref:
                        dup = lambda t: torch.cat([t, t], 0)
                        h = dup(h)
                        skips = [dup(s_) for s_ in skips]
                        temb_all = dup(temb_all)
                        rt.enc = dup(rt.enc)
                        rt.B = 2 * B
                        rt.paired = True
                h = res.fwd(h, rt, tb(res))
                if hasattr(blk, "attentions"):
                    h = blk.attentions[j].fwd(h, rt, f"down_blocks.{i}.attentions.{j}")
                skips.append(h)
            if hasattr(blk, "downsamplers"):
                h = blk.downsamplers[0].fwd(h, rt)
                skips.append(h)
        m = self.mid_block
        h = m.resnets[0].fwd(h, rt, tb(m.resnets[0]))
        h = m.attentions[0].fwd(h, rt, "mid_block.attentions.0")
        h = m.resnets[1].fwd(h, rt, tb(m.resnets[1]))
        for i, blk in enumerate(self.up_blocks):
            for j, res in enumerate(blk.resnets):
                s = skips.pop()
                hc = K.concat_channels(h, s)
                if rt.save:
                    rt.saved.append({"c1": h.shape[-1]})
                h = res.fwd(hc, rt, tb(res))
                if hasattr(blk, "attentions"):
                    h = blk.attentions[j].fwd(h, rt, f"up_blocks.{i}.attentions.{j}")
            if hasattr(blk, "upsamplers"):
                h = blk.upsamplers[0].fwd(h, rt)
        hn, st = K.group_norm_fwd(h, self.conv_norm_out.weight, self.conv_norm_out.bias, self.cfg.norm_num_groups,
                                  self.cfg.norm_eps, True)
        out = K.conv2d(hn, self.conv_out.w_nhwc, bias=self.conv_out.bias)
        if save:
            rt.saved.append({"h": rt.pol(h), "st": rt.pol(st), "hn": hn if full else None})
        # the backward sees the policy half only
        rt.B = B
        rt.enc = rt.pol(rt.enc)
        rt.paired = False
        return out, rt

    def backward_nhwc(self, dout, rt):
        """Manual backward of forward_nhwc(save=True): accumulates LoRA grads into self.lora.grad.
        Returns None (no gradient w.r.t. the latent input is needed on the hot path)."""
        B = dout.shape[0]
        sv = rt.saved.pop()
        fg = rt.fg
        # conv_out input-gradient (C_out = 4): im2col of dout + GEMM with the rotated, transposed weights
        _, H, W, _ = dout.shape
        cols = K.im2col3(dout.contiguous(), self.conv_out.kp_dx)
        dhn = K.gemm(cols, self.conv_out.w_dx_col).view(B, H, W, -1)
        if fg is not None:
            rt.dtemb = torch.zeros((B, self._temb_n), device=dout.device, dtype=torch.float32)
            co = self.conv_out.cout
            dy8 = torch.zeros((B * H * W, 8), device=dout.device, dtype=BF16)  # TN operands need 8 | width
            dy8[:, :co] = dout.reshape(-1, co)
            _conv_dw(fg, self.conv_out, dy8, sv["hn"], rt, K.im2col_conv)
            dh = K.group_norm_bwd(sv["h"], dhn, sv["st"], self.conv_norm_out.weight, self.conv_norm_out.bias, True,
                                  dgamma=fg.g(self.conv_norm_out.weight), dbeta=fg.g(self.conv_norm_out.bias),
                                  accumulate=True)
        else:
            dh = K.group_norm_bwd(sv["h"], dhn, sv["st"], self.conv_norm_out.weight, self.conv_norm_out.bias, True)
        unit_done = getattr(rt, "unit_done", None) or (lambda unit: None)  # overlapped gradient sync (GradBuckets)
        # LoRA weight gradients are deferred per gradient unit and issued as one batched launch per rank / orientation
        # (K.TnRankQueue) right before the unit is reported done -- its all-reduce bucket may be issued next
        dwq = K.TnRankQueue() if TN_BATCH else None
        rt.dw = dwq.add if dwq is not None else K.gemm_tn

        def done(unit):
            if dwq is not None:
                dwq.flush()
            unit_done(unit)

        done("conv_out")
        skip_grads = []
        for i in reversed(range(len(self.up_blocks))):
            blk = self.up_blocks[i]
            if hasattr(blk, "upsamplers"):
                dh = blk.upsamplers[0].bwd(dh, rt)
                done(f"up_blocks.{i}.upsamplers.0")
            for j in reversed(range(len(blk.resnets))):
                if hasattr(blk, "attentions"):
                    dh = blk.attentions[j].bwd(dh, rt, f"up_blocks.{i}.attentions.{j}")
                    done(f"up_blocks.{i}.attentions.{j}")
                dhc = blk.resnets[j].bwd(dh, rt)
                done(f"up_blocks.{i}.resnets.{j}")
                c1 = rt.saved.pop()["c1"]
                dh, ds = K.split_channels(dhc, c1)
                skip_grads.append(ds)
        m = self.mid_block
        dh = m.resnets[1].bwd(dh, rt)
        done("mid_block.resnets.1")
        dh = m.attentions[0].bwd(dh, rt, "mid_block.attentions.0")
        done("mid_block.attentions.0")
        dh = m.resnets[0].bwd(dh, rt)
        done("mid_block.resnets.0")
        # the up-block backward visits skips in forward-push order, so the down-block backward takes them from the end.
        # Below the first adapter-carrying attention (down_blocks.1.attentions.0) nothing has a trainable parameter and
        # the latent needs no gradient, so the backward stops there: down_blocks.0 (two 128^2 resnets + downsample),
        # down_blocks.1.resnets.0 and conv_in are never differentiated (the reference's autograd also runs them only
        # for the input gradient, which is then discarded).
        i0, j0 = self._first_attn if fg is None else (0, -1)
        for i in reversed(range(i0, len(self.down_blocks))):
            blk = self.down_blocks[i]
            if hasattr(blk, "downsamplers"):
                dh = K.add(dh, skip_grads.pop())
                dh = blk.downsamplers[0].bwd(dh, rt)
                done(f"down_blocks.{i}.downsamplers.0")
            for j in reversed(range(len(blk.resnets))):
                dh = K.add(dh, skip_grads.pop())
                if (i, j) == (i0, j0):
                    blk.attentions[j].bwd(dh, rt, f"down_blocks.{i}.attentions.{j}", need_dx=False)
                    done(f"down_blocks.{i}.attentions.{j}")
                    break
                if hasattr(blk, "attentions"):
                    dh = blk.attentions[j].bwd(dh, rt, f"down_blocks.{i}.attentions.{j}")
                    done(f"down_blocks.{i}.attentions.{j}")
                dh = blk.resnets[j].bwd(dh, rt)
                done(f"down_blocks.{i}.resnets.{j}")
        if fg is not None:
            dh = K.add(dh, skip_grads.pop())  # conv_in output (the first skip)
            self._conv_in_dw(fg, dh, rt)
            self._embed_bwd(fg, rt)
            done("embed")
        rt.saved.clear()  # activations of the never-differentiated prefix
        if dwq is not None:
            dwq.flush()
        rt.side.join()  # LoRA weight gradients complete before anything reads lora.grad
        return None

    def _conv_in_dw(self, fg, dh, rt):
        """conv_in (C = 4, im2col GEMM in the forward): dW = dh^T . cols on the saved patch matrix."""
        ci = self.conv_in
        tmp = torch.zeros((ci.cout, ci.kp), device=dh.device, dtype=torch.float32)
        d2 = dh.reshape(-1, ci.cout)
        K.gemm_tn(d2, rt.cols_in, tmp)
        fg.g(ci.weight).add_(tmp[:, :9 * ci.cin].view(ci.cout, 3, 3, ci.cin).permute(0, 3, 1, 2))
        K.colsum_acc(d2, fg.g(ci.bias).view(1, -1))

    def _embed_bwd(self, fg, rt):
        """Weight grads of the time / added-condition embeddings from the accumulated time_emb_proj output grads
        rt.dtemb [B, sum Co]: the batched projection, silu, add_embedding and time_embedding MLPs.  The [B, 1280]
        silu derivatives are torch element-wise ops (a few KB)."""
        e = rt.emb
        dt = K.cast_f32_bf16(rt.dtemb)
        res = [m for m in self.modules() if isinstance(m, ResnetBlock2D)]
        gw = _stacked([fg.g(m.time_emb_proj.weight) for m in res])
        gb = _stacked([fg.g(m.time_emb_proj.bias) for m in res])
        if gw.data_ptr() == fg.g(res[0].time_emb_proj.weight).data_ptr() and \
                gb.data_ptr() == fg.g(res[0].time_emb_proj.bias).data_ptr():  # adjacent grads: accumulate in place
            K.gemm_tn(dt, e["se"], gw)
            gb.add_(rt.dtemb.sum(0))
        else:
            tmp = torch.zeros((self._temb_n, e["se"].shape[1]), device=dt.device, dtype=torch.float32)
            K.gemm_tn(dt, e["se"], tmp)
            for m in res:
                fg.g(m.time_emb_proj.weight).add_(tmp[m._temb_off:m._temb_off + m.cout])
                fg.g(m.time_emb_proj.bias).add_(rt.dtemb[:, m._temb_off:m._temb_off + m.cout].sum(0))

        def silu_bwd(dy, x):
            xf = x.float()
            sg = torch.sigmoid(xf)
            return (dy.float() * sg * (1 + xf * (1 - sg))).to(BF16)

        demb = silu_bwd(K.gemm(dt, self._temb_wt), e["emb"])  # d emb (pre-silu), [B, tdim]
        a1, a2 = self.add_embedding.linear_1, self.add_embedding.linear_2
        _lin_dw(fg, a2, demb, e["s2"])
        du1 = silu_bwd(K.gemm(demb, a2.wt), e["u1"])
        _lin_dw(fg, a1, du1, e["add_in"])
        l1, l2 = self.time_embedding.linear_1, self.time_embedding.linear_2
        _lin_dw(fg, l2, demb, e["s1"])
        dt1 = silu_bwd(K.gemm(demb, l2.wt), e["t1"])
        _lin_dw(fg, l1, dt1, e["te"])

    @property
    def _first_attn(self):
        for i, blk in enumerate(self.down_blocks):
            if hasattr(blk, "attentions"):
                return i, 0
        raise ValueError("UNet without attention blocks has no adapter to train")

    # ---------------- diffusers call surface ----------------
    def forward(self, sample, timestep, encoder_hidden_states, added_cond_kwargs=None, return_dict=True, **kw):
        added = added_cond_kwargs or {}
        x = K.nchw_to_nhwc(sample)
        # autograd trigger: the flat LoRA parameter, or (full-UNet training) a 1-element stand-in for all weights
        trig = self.lora.param if (self.lora is not None and self._adapters_enabled) else (
            self.full.trigger if self.full is not None else None)
        need_grad = torch.is_grad_enabled() and trig is not None
        if need_grad:
            out = _UNetFn.apply(x, trig, self, timestep, encoder_hidden_states, added["text_embeds"],
                                added["time_ids"])
        else:
            with torch.no_grad():
                out, _ = self.forward_nhwc(x, timestep, encoder_hidden_states, added["text_embeds"],
                                           added["time_ids"], save=False)
        eps = _NHWC2NCHW.apply(out)
        return _Output(sample=eps) if return_dict else (eps,)

    __call__ = nn.Module.__call__


class _UNetFn(torch.autograd.Function):
    """The whole UNet as one autograd node; LoRA grads go straight into the flat grad buffer."""

    @staticmethod
    def forward(ctx, x, lora_param, unet, timestep, enc, text_embeds, time_ids):
        out, rt = unet.forward_nhwc(x, timestep, enc, text_embeds, time_ids, save=True)
        ctx.unet, ctx.rt = unet, rt
        return out

    @staticmethod
    def backward(ctx, dout):
        ctx.unet.backward_nhwc(dout.contiguous(), ctx.rt)
        ctx.rt = None
        return None, None, None, None, None, None, None


class _NHWC2NCHW(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        return K.nhwc_to_nchw(x, torch.float32)

    @staticmethod
    def backward(ctx, g):
        return K.nchw_to_nhwc(g.contiguous())
