"""Drop-in for `pso_pytorch.diffusers_patch.distilled_inference_with_logprob`
(DP/distilled_inference_with_logprob.py:45-137): DMD2 step x0 = (x - sqrt(1-a_t) eps)/sqrt(a_t), mean =
sqrt(a_prev) x0, std = sqrt(1-a_prev); sampling re-noises with ONE (1,C,H,W) draw shared across the batch
(:123-126); raises ValueError when both `generator` and `prev_sample` are given (:115-119).

Numerics: like the reference, the step runs in the latent dtype -- fp32 latents in fp32; fp16 / bf16 latents in the
kernel's replay mode (PSO_MODE_DMD_F16 / _BF16), which rounds x0 (:84-86), the latent-dtype table terms (:98-110),
the mean, the re-noised sample and every term of the log-density (:126-135) to that dtype.  log_prob is returned in
the latent dtype, as the reference's is.
"""
from typing import Optional

import torch

from ... import kernels as K
from ... import pso_core


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
    mode = pso_core.dmd_mode(sample.dtype)
    coef = pso_core.dmd_coef(self.alphas_cumprod, timestep, prev_timestep, latent_dtype=sample.dtype)
    coef = coef.expand(sample.shape[0], -1).contiguous().to(model_output.device)
    eps = model_output if model_output.dtype in (torch.float32, torch.bfloat16) else model_output.float()
    x = sample.to(torch.float32)
    if prev_sample is None:
        # randn_tensor((1, C, H, W), dtype=sample.dtype) (:123-124): drawn in the latent dtype
        noise = torch.randn((1,) + tuple(sample.shape[1:]), generator=generator, device=model_output.device,
                            dtype=sample.dtype if sample.dtype in pso_core.DMD_REPLAY_MODES else torch.float32)
        prev, lp = K.step_logprob(mode, x, eps, coef, noise=noise.float(), noise_shared=True)
    else:
        prev, lp = K.step_logprob(mode, x, eps, coef, prev=prev_sample.to(torch.float32))
    return prev.type(sample.dtype), lp.to(sample.dtype if sample.dtype in pso_core.DMD_REPLAY_MODES else lp.dtype)
