"""Drop-in for `pso_pytorch.diffusers_patch.sdxl_turbo_with_logprob.sdxl_turbo_pipeline_with_logprob`
(DP/sdxl_turbo_with_logprob.py:52-161): Euler-ancestral sampling through the distilled UNet recording all latents,
model inputs and step log-probs (the last, deterministic step is not recorded, :146-149), then VAE decode.

Returns (image, all_latents, all_log_probs, all_model_input_latents) like the reference.  The latent side is
height // 8 (the reference hard-codes 64, i.e. 512^2; BASELINE config 2 samples at 1024^2).
"""
from typing import Any, Callable, Dict, List, Optional, Union

import torch

from .turbo_inference_with_logprob import turbo_step_with_logprob


def prepare_latents(batch_size, num_channels_latents, height, width, dtype, device, generator, latents=None):
    shape = (batch_size, num_channels_latents, height // 8, width // 8)
    if latents is None:
        return torch.randn(shape, generator=generator, device=device, dtype=torch.float32).to(dtype)
    return latents.to(device)


def _unwrap(accelerator, m):
    return accelerator.unwrap_model(m) if accelerator is not None else m


@torch.no_grad()
def sdxl_turbo_pipeline_with_logprob(
    accelerator,
    vae,
    unet,
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
    num_channels_latents = _unwrap(accelerator, unet).config.in_channels
    latents = prepare_latents(batch_size * num_images_per_prompt, num_channels_latents, height, width,
                              prompt_embeds.dtype, prompt_embeds.device, generator, latents)
    latents = latents * noise_scheduler.init_noise_sigma.to(latents.device)
    noise_scheduler.set_timesteps(num_inference_steps, device=prompt_embeds.device)
    timesteps = noise_scheduler.timesteps
    cond = {"time_ids": add_time_ids, "text_embeds": pooled_prompt_embeds}
    all_latents, all_model_input_latents, all_log_probs = [latents], [], []
    for i, t in enumerate(timesteps):
        sigma = noise_scheduler.sigmas[i]
        latent_model_input = latents / ((sigma ** 2 + 1) ** 0.5)
        noise_pred = unet(latent_model_input, t, encoder_hidden_states=prompt_embeds, added_cond_kwargs=cond,
                          return_dict=False)[0]
        latents, log_prob = turbo_step_with_logprob(noise_scheduler, noise_pred, t.unsqueeze(0), latents,
                                                    generator=generator, device=latents.device)
        if i != num_inference_steps - 1:
            all_model_input_latents.append(latent_model_input)
            all_latents.append(latents)
            all_log_probs.append(log_prob)
    if output_type != "latent":
        image = vae.decode(latents / vae.config.scaling_factor, return_dict=False)[0]
    else:
        image = latents
    return image, all_latents, all_log_probs, all_model_input_latents
