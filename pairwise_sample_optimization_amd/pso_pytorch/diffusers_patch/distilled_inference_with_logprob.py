"""Drop-in for `pso_pytorch.diffusers_patch.distilled_inference_with_logprob`
(DP/distilled_inference_with_logprob.py:45-137): DMD2 step x0 = (x - sqrt(1-a_t) eps)/sqrt(a_t), mean =
sqrt(a_prev) x0, std = sqrt(1-a_prev); sampling re-noises with ONE (1,C,H,W) draw shared across the batch
(:123-126); raises ValueError when both `generator` and `prev_sample` are given (:115-119).

Numerics: the reference computes in the latent dtype (fp16/bf16 when the latents are); this kernel
computes in fp32 (identical for fp32 latents, the parity target) and returns prev_sample in the sample's dtype.
"""
from typing import Optional

import torch

from ... import kernels as K
from ... import pso_core
from ..._lib import MODE_DMD


def _get_x0_from_noise(sample, model_output, alphas_cumprod, timestep):
    """DP/distilled_inference_with_logprob.py:36-42 (host helper kept for API parity; tiny tensors only)."""
    alpha_prod_t = alphas_cumprod[timestep.long()].reshape(-1, 1, 1, 1)
    beta_prod_t = 1 - alpha_prod_t
    return (sample - beta_prod_t ** 0.5 * model_output) / alpha_prod_t ** 0.5


def distilled_step_with_logprob(
    self,
    model_output: torch.FloatTensor,
    timestep: torch.Tensor,
    prev_timestep: torch.Tensor,
    sample: torch.FloatTensor,
    eta: float = 0.0,
    use_clipped_model_output: bool = False,
    generator=None,
    prev_sample: Optional[torch.FloatTensor] = None,
    device=torch.device("cuda"),
):
    if prev_sample is not None and generator is not None:
        raise ValueError(
            "Cannot pass both generator and prev_sample. Please make sure that either `generator` or"
            " `prev_sample` stays `None`.")
    coef = pso_core.dmd_coef(self.alphas_cumprod, timestep, prev_timestep)
    coef = coef.expand(sample.shape[0], -1).contiguous().to(model_output.device)
    eps = model_output if model_output.dtype in (torch.float32, torch.bfloat16) else model_output.float()
    x = sample.to(torch.float32)
    if prev_sample is None:
        noise = torch.randn((1,) + tuple(sample.shape[1:]), generator=generator, device=model_output.device,
                            dtype=torch.float32)
        prev, lp = K.step_logprob(MODE_DMD, x, eps, coef, noise=noise, noise_shared=True)
    else:
        prev, lp = K.step_logprob(MODE_DMD, x, eps, coef, prev=prev_sample.to(torch.float32))
    return prev.type(sample.dtype), lp
