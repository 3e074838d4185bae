"""Drop-in for `pso_pytorch.diffusers_patch.sdxl_dmd_with_logprob.sdxl_dmd_pipeline_with_logprob`
(DP/sdxl_dmd_with_logprob.py:53-174): DMD2 sampling over fixed `timesteps` (x0-prediction re-noised to the next
timestep); the last step returns x0 (:154-162), then VAE decode.  Returns (image, all_latents, all_log_probs).
"""
from typing import Any, Callable, Dict, List, Optional, Union

import torch

from .distilled_inference_with_logprob import distilled_step_with_logprob, _get_x0_from_noise


def prepare_latents(scheduler, batch_size, num_channels_latents, height, width, dtype, device, generator,
                    latents=None):
    shape = (batch_size, num_channels_latents, height // 8, width // 8)
    if latents is None:
        latents = torch.randn(shape, generator=generator, device=device, dtype=torch.float32).to(dtype)
    else:
        latents = latents.to(device)
    return latents * scheduler.init_noise_sigma


@torch.no_grad()
def sdxl_dmd_pipeline_with_logprob(
    accelerator,
    vae,
    unet,
    timesteps,
    noise_scheduler,
    height,
    width,
    num_inference_steps: int = 4,
    guidance_scale: float = 0.0,
    negative_prompt: Optional[Union[str, List[str]]] = None,
    num_images_per_prompt: Optional[int] = 1,
    generator=None,
    latents: Optional[torch.FloatTensor] = None,
    prompt_embeds: Optional[torch.FloatTensor] = None,
    pooled_prompt_embeds: Optional[torch.FloatTensor] = None,
    add_time_ids: Optional[torch.FloatTensor] = None,
    negative_prompt_embeds: Optional[torch.FloatTensor] = None,
    output_type: Optional[str] = "pil",
    return_dict: bool = True,
    callback: Optional[Callable[[int, int, torch.FloatTensor], None]] = None,
    callback_steps: int = 1,
    cross_attention_kwargs: Optional[Dict[str, Any]] = None,
    guidance_rescale: float = 0.0,
):
    batch_size = prompt_embeds.shape[0]
    unwrap = accelerator.unwrap_model(unet) if accelerator is not None else unet
    latents = prepare_latents(noise_scheduler, batch_size * num_images_per_prompt, unwrap.config.in_channels,
                              height, width, prompt_embeds.dtype, prompt_embeds.device, generator, latents)
    cond = {"time_ids": add_time_ids, "text_embeds": pooled_prompt_embeds}
    all_latents, all_log_probs = [latents], []
    x0_pred = latents
    for i, t in enumerate(timesteps):
        cur = torch.ones(batch_size, device=prompt_embeds.device, dtype=torch.long) * t
        noise_pred = unet(latents, cur, prompt_embeds, added_cond_kwargs=cond).sample
        if i != timesteps.shape[0] - 1:
            prev_t = torch.ones(batch_size, device=prompt_embeds.device, dtype=torch.long) * timesteps[i + 1]
            latents, log_prob = distilled_step_with_logprob(noise_scheduler, noise_pred, cur, prev_t, latents,
                                                            generator=generator, device=latents.device)
            all_latents.append(latents)
            all_log_probs.append(log_prob)
        else:
            x0_pred = _get_x0_from_noise(latents, noise_pred, noise_scheduler.alphas_cumprod.to(latents.device), cur)
            all_latents.append(x0_pred)
    if output_type != "latent":
        image = vae.decode(x0_pred / vae.config.scaling_factor, return_dict=False)[0]
    else:
        image = x0_pred
    return image, all_latents, all_log_probs
