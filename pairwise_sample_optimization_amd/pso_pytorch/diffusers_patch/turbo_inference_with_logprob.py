"""Drop-in for `pso_pytorch.diffusers_patch.turbo_inference_with_logprob` (DP/turbo_inference_with_logprob.py:24-116).

Same signature, return values and semantics: one Euler-ancestral step x_t -> x_{t-1} and the Gaussian log-prob of
`prev_sample` under N(mean, sigma_up^2), averaged over C,H,W.  The per-sample scalars (sigma lookup, sigma_up,
sigma_down) are host float32 scalars in the reference's op order; every per-element operation runs in the fused HIP
kernel `pso_step_logprob` (no CPU fallback).
"""
from typing import Optional

import torch

from ... import kernels as K
from ... import pso_core
from ..._lib import MODE_TURBO


def turbo_step_with_logprob(
    self,
    model_output: torch.FloatTensor,
    timestep: torch.Tensor,
    sample: torch.FloatTensor,
    generator=None,
    prev_sample: Optional[torch.FloatTensor] = None,
    device=torch.device("cuda"),
):
    coef = pso_core.turbo_coef(self.sigmas, self.timesteps, timestep)
    coef = coef.expand(sample.shape[0], -1).contiguous().to(model_output.device)  # one timestep for the batch
    eps = model_output if model_output.dtype in (torch.float32, torch.bfloat16) else model_output.float()
    x = sample.to(torch.float32)
    if prev_sample is None:
        noise = torch.randn(model_output.shape, generator=generator, device=model_output.device,
                            dtype=torch.float32)
        prev, lp = K.step_logprob(MODE_TURBO, x, eps, coef, noise=noise)
    else:
        prev, lp = K.step_logprob(MODE_TURBO, x, eps, coef, prev=prev_sample.to(torch.float32))
    return prev.to(model_output.dtype), lp
