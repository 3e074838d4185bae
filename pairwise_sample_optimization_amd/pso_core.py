"""Host-side scalar math of the PSO step (float32, the reference's operation order) + the autograd boundary of the
fused pairwise loss kernel.

`turbo_coef` restates the sigma lookup of `DP/turbo_inference_with_logprob.py:61-85`; `dmd_coef` the alphas_cumprod
lookups of `DP/distilled_inference_with_logprob.py:36-42,102-110`.  These are per-sample scalars (a few floats per
image) computed once per step on the host; the per-element work runs in libpso_amd (pso_step_logprob,
pso_pair_loss_fwd/bwd).  The per-sample `(_t == self.timesteps).nonzero()[0].item()` host sync of the reference
(`DP/turbo_inference_with_logprob.py:61-63`) becomes a host-side table lookup on CPU copies of the tables.
"""
import math

import torch

from . import kernels as K
from ._lib import MODE_TURBO, MODE_DMD, MODE_DMD_F16, MODE_DMD_BF16, COEF_STRIDE

LOG_SQRT_2PI = torch.log(torch.sqrt(2 * torch.as_tensor(math.pi))).item()  # same float as the reference's expression


def _f32(x):
    return torch.as_tensor(x, dtype=torch.float32).cpu()


def _sqrt(v):
    """IEEE-exact float32 sqrt on any host: the float64 sqrt rounded to float32 (exact for sqrt, p64 >= 2 p32 + 2).
    torch's float32 CPU sqrt is NOT exact on every host CPU (a vectorised path on one GPU box returned 0x3f599312 for
    sqrt(0.72233057), correct 0x3f599311), which would move the DMD2 replay x0 across a bf16 rounding tie."""
    return torch.sqrt(v.double()).to(v.dtype)


def turbo_coef(sigmas, timesteps, t):
    """Per-sample [sigma, sigma_up, sigma_down - sigma, 2 sigma_up^2, log sigma_up, log sqrt(2 pi), 0, 0] (float32)."""
    sigmas = _f32(sigmas)
    timesteps = _f32(timesteps)
    t = _f32(t).reshape(-1)
    idx = [int((tt == timesteps).nonzero()[0].item()) for tt in t]
    nxt = [i + 1 for i in idx]
    s_from = sigmas[idx]
    s_to = sigmas[nxt]
    # `** 2` / `** 0.5` of the reference as explicit x*x and IEEE sqrt: torch's CPU pow kernels differ by an ulp
    # between host CPUs (vectorised pow vs sqrt), sqrt is correctly rounded everywhere
    sq = lambda v: v * v
    s_up = _sqrt(sq(s_to) * (sq(s_from) - sq(s_to)) / sq(s_from))
    s_down = _sqrt(sq(s_to) - sq(s_up))
    c = torch.zeros(len(idx), COEF_STRIDE, dtype=torch.float32)
    c[:, 0] = s_from
    c[:, 1] = s_up
    c[:, 2] = s_down - s_from
    c[:, 3] = 2 * sq(s_up)
    c[:, 4] = torch.log(s_up)
    c[:, 5] = LOG_SQRT_2PI
    return c


DMD_REPLAY_MODES = {torch.float16: MODE_DMD_F16, torch.bfloat16: MODE_DMD_BF16}


def dmd_mode(latent_dtype=torch.float32):
    """Kernel mode of a DMD2 step on latents of `latent_dtype` (fp16 / bf16 -> the latent-dtype replay modes)."""
    return DMD_REPLAY_MODES.get(latent_dtype, MODE_DMD)


def dmd_coef(alphas_cumprod, t, t_prev, latent_dtype=torch.float32):
    """Per-sample [sqrt(a_t), sqrt(1-a_t), sqrt(a_prev), sqrt(1-a_prev), 2(1-a_prev), log sqrt(1-a_prev),
    log sqrt(2 pi), 0] (float32, the reference's `** 0.5` on the float32 table).  latent_dtype fp16 / bf16: entries
    2-5 are the reference's latent-dtype values (DP/distilled_inference_with_logprob.py:98-110 casts the table to the
    latent dtype, then every op rounds to it) -- the same torch CPU ops on the same dtype."""
    ac = _f32(alphas_cumprod)
    a_t = ac[torch.as_tensor(t).reshape(-1).long().cpu()]
    tp = torch.as_tensor(t_prev).reshape(-1).long().cpu()
    a_p = ac[tp]
    # `** 0.5` as IEEE sqrt (correctly rounded on every host; torch's CPU pow / sqrt may not be), and in the latent dtype
    # as the fp32 sqrt rounded once to it (what torch's reduced-precision pow computes)
    rsqrt = lambda v: _sqrt(v.float()).to(v.dtype)
    if latent_dtype in DMD_REPLAY_MODES:
        acl = ac.to(latent_dtype)
        sa_l = rsqrt(acl[tp])
        sb_l = rsqrt(1 - acl[tp])
        c = torch.zeros(a_t.shape[0], COEF_STRIDE, dtype=torch.float32)
        c[:, 0] = _sqrt(a_t)
        c[:, 1] = _sqrt(1 - a_t)
        c[:, 2] = sa_l.float()
        c[:, 3] = sb_l.float()
        c[:, 4] = (2 * (sb_l * sb_l)).float()
        c[:, 5] = torch.log(sb_l).float()
        # `- torch.log(torch.sqrt(2 * torch.as_tensor(math.pi)))` (:132): the fp32 0-dim tensor meets a latent-dtype
        # tensor and is cast to that dtype first
        c[:, 6] = torch.tensor(LOG_SQRT_2PI).to(latent_dtype).float()
        return c
    sbp = _sqrt(1 - a_p)
    c = torch.zeros(a_t.shape[0], COEF_STRIDE, dtype=torch.float32)
    c[:, 0] = _sqrt(a_t)
    c[:, 1] = _sqrt(1 - a_t)
    c[:, 2] = _sqrt(a_p)
    c[:, 3] = sbp
    c[:, 4] = 2 * (sbp * sbp)
    c[:, 5] = torch.log(sbp)
    c[:, 6] = LOG_SQRT_2PI
    return c


class PairLoss(torch.autograd.Function):
    """Autograd boundary of the fused kernel: forward = the 4 log-probs + loss of `T:810-850`; backward = dL/d eps_pol
    (the only differentiable input: the reference computes eps_ref under no_grad, `T:791-805`)."""

    @staticmethod
    def forward(ctx, eps_pol, eps_ref, x, x_prev, coef, pref, mode, beta, clip_eps):
        P = x.shape[0] // 2
        ws = K.pair_loss_ws(P, x[0].numel(), x.device)
        loss, lp = K.pair_loss_fwd(mode, x, x_prev, eps_pol.detach(), eps_ref, coef, pref, beta, clip_eps, ws)
        ctx.save_for_backward(eps_pol, x, x_prev, coef, pref, ws)
        ctx.cfg = (mode, beta, clip_eps)
        ctx.mark_non_differentiable(lp)
        return loss, lp

    @staticmethod
    def backward(ctx, g_loss, g_lp):
        eps_pol, x, x_prev, coef, pref, ws = ctx.saved_tensors
        mode, beta, clip_eps = ctx.cfg
        deps = K.pair_loss_bwd(mode, x, x_prev, eps_pol, coef, pref, beta, clip_eps, ws,
                               grad_out=g_loss.contiguous().float(), out_dtype=eps_pol.dtype)
        return deps, None, None, None, None, None, None, None, None


def pair_loss(eps_pol, eps_ref, x, x_prev, coef, pref, mode, beta, clip_eps):
    """Returns (loss scalar, lp [2P, 2]).  Image order 2p + k."""
    return PairLoss.apply(eps_pol.contiguous(), eps_ref.contiguous(), x.contiguous(), x_prev.contiguous(),
                          coef.to(x.device), pref.to(x.device).float().contiguous(), mode, beta, clip_eps)
