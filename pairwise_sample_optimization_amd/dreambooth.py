"""DreamBooth PSO step for SDXL-Turbo (BASELINE config 5), MI355X-native.

Reference: DB = personalization/train_pso_sdxl_turbo_dreambooth.py, the micro-step DB:1720-1964 with the recipe of
personalization/scripts/pso_dog.sh (EDM-style epsilon training, loss "pso_db", beta 5, prior weight 0.5, rank 16):

  pixel_values = [instances; negatives]                                  DB:1731
  x0     = vae.encode(pixel_values).latent_dist.sample() * scaling       DB:1750-1753
  noise  = one draw shared by both halves                                DB:1763
  t      = stride * (randint % 4) + stride - 1  in {249,499,749,999}     DB:1769-1777 (turbo branch), same for both
  noisy  = x0 + noise * sigma(t) ; unet_in = noisy / sqrt(sigma^2 + 1)   DB:1787-1796
  eps    = unet(unet_in, t, prompt_embeds x2, {time_ids, text_embeds})   DB:1815-1825
  loss   = fused DreamBooth PSO loss (csrc/db_loss.hip)                  DB:1847-1935
  backward -> LoRA grads ; every gradient_accumulation_steps: clip + AdamW   DB:1953-1964

Here the VAE encoder, the UNet forward/backward and the loss all run on libpso_amd; for loss_type "pso" the reference
eps (adapters disabled, DB:1894-1920) comes from the same paired UNet pass as the policy eps.  No host sync.
"""

import torch

from . import kernels as K
from .schedulers import EulerDiscreteScheduler, db_distill_timesteps
from .trainer import lora_optimizer_step



class DreamBoothPSOTrainer:
    def __init__(self, unet, vae, loss_type="pso_db", beta_pso=5.0, neg_defactor=0.1, prior_loss_weight=0.5,
                 distill_train_timesteps=4, learning_rate=2e-4, betas=(0.9, 0.999), adam_weight_decay=1e-4,
                 adam_epsilon=1e-8, max_grad_norm=1.0, gradient_accumulation_steps=4, process_group=None):
        """Defaults: DB argparse defaults (DB:636-674, 757-777) overridden by the recipe scripts/pso_dog.sh."""
        if loss_type not in ("pso", "pso_db"):
            raise ValueError(f"Unknown loss type {loss_type}")  # DB:1929
        self.unet, self.vae = unet, vae
        self.loss_type = loss_type
        self.lt = K.DB_SIGMOID if loss_type == "pso" else K.DB_HINGE
        self.beta, self.nd, self.prior_w = float(beta_pso), float(neg_defactor), float(prior_loss_weight)
        self.distill_steps = distill_train_timesteps
        self.lr, self.betas, self.wd, self.adam_eps = learning_rate, betas, adam_weight_decay, adam_epsilon
        self.max_grad_norm = max_grad_norm
        self.gas = gradient_accumulation_steps
        self.pg = process_group
        self.sched = EulerDiscreteScheduler()
        st = unet.lora
        self.exp_avg = torch.zeros_like(st.master)
        self.exp_avg_sq = torch.zeros_like(st.master)
        self.clip_buf = torch.zeros(2, device=st.master.device, dtype=torch.float32)
        self.opt_step = 0
        self.n_micro = 0
        self.loss_hist = []
        self.auto_step = True

    def prepare_inputs(self, pixel_values, generator=None):
        """DB:1731-1796 on device: latents, shared noise, distilled timesteps, EDM-preconditioned UNet input.
        pixel_values [2B,3,H,W] in [-1,1] (instances first).  Returns a dict of NHWC tensors."""
        dev = pixel_values.device
        B2 = pixel_values.shape[0]
        B = B2 // 2
        mo = self.vae.encode_nhwc(pixel_values)                                   # [2B,h,w,8] fp32
        L = self.vae.cfg.latent_channels
        mean, logvar = mo[..., :L], mo[..., L:].clamp(-30.0, 20.0)
        z = torch.randn(mean.shape, device=dev, generator=generator)
        x0 = ((mean + torch.exp(0.5 * logvar) * z) * self.vae.config.scaling_factor).contiguous()
        noise = torch.randn((B,) + tuple(x0.shape[1:]), device=dev, generator=generator).repeat(2, 1, 1, 1)
        raw = torch.randint(0, self.sched.num_train_timesteps, (B,), device=dev, generator=generator)
        t = db_distill_timesteps(raw, self.distill_steps, self.sched.num_train_timesteps).repeat(2)
        sigma = self.sched.sigma_at(t)
        s4 = sigma.view(-1, 1, 1, 1)
        noisy = (x0 + noise * s4).contiguous()
        unet_in = K.cast_f32_bf16(noisy / torch.sqrt(s4 * s4 + 1.0))
        return dict(x0=x0, noisy=noisy, sigma=sigma.contiguous(), t=t.float(), unet_in=unet_in)

    def micro_step(self, pixel_values, prompt_embeds, pooled, time_ids, generator=None):
        """One DreamBooth PSO micro-step (DB:1720-1964).  prompt_embeds [B,77,D], pooled [B,Dp], time_ids [B,6] are
        the instance prompt's; both halves use them (DB:1804, 1816-1818).  Returns the loss (device scalar)."""
        inp = self.prepare_inputs(pixel_values, generator)
        enc = prompt_embeds.repeat(2, 1, 1)
        pl = pooled.repeat(2, 1)
        tid = time_ids.repeat(2, 1)
        u = self.unet
        u.enable_adapters()
        paired = self.loss_type == "pso"
        eps, rt = u.forward_nhwc(inp["unet_in"], inp["t"], enc, pl, tid, save=True, paired_ref=paired)
        n = inp["unet_in"].shape[0]
        eps_pol = eps[:n]
        eps_ref = eps[n:] if paired else None
        ws = K.db_loss_ws(n // 2, eps_pol[0].numel(), eps.device)
        loss, _, _ = K.db_loss_fwd(self.lt, eps_pol, inp["noisy"], inp["x0"], inp["sigma"], self.beta, self.nd,
                                   self.prior_w, ws, eps_ref=eps_ref)
        # accelerator.backward divides by gradient_accumulation_steps
        deps = K.db_loss_bwd(self.lt, eps_pol, inp["noisy"], inp["x0"], inp["sigma"], self.beta, self.nd,
                             self.prior_w, ws, grad_scale=1.0 / self.gas)
        u.backward_nhwc(deps, rt)
        self.loss_hist.append(loss)
        self.n_micro += 1
        if self.auto_step and self.n_micro % self.gas == 0:
            self.optimizer_step()
        return loss

    def optimizer_step(self):
        lora_optimizer_step(self)
