"""Scheduler state the PSO hot path reads (host-side float32 tables), restating diffusers 0.27.0:

* `EulerAncestralDiscreteScheduler` (SDXL-Turbo, T:264-268): `.timesteps`, `.sigmas`, `.init_noise_sigma`,
  `.set_timesteps(N)` with timestep_spacing="trailing"; read by DP/sdxl_turbo_with_logprob.py:99-103,120 and
  DP/turbo_inference_with_logprob.py:61-66.
* `LCMScheduler` (DMD2, D:285): `.alphas_cumprod`, `.init_noise_sigma` (1.0); read by
  DP/distilled_inference_with_logprob.py:36-42,84-112 and DP/sdxl_dmd_with_logprob.py:47-49.

SDXL "scaled_linear" betas, beta_start 0.00085, beta_end 0.012, 1000 training steps.
"""
import numpy as np
import torch


def _alphas_cumprod(num_train_timesteps=1000, beta_start=0.00085, beta_end=0.012):
    betas = torch.linspace(beta_start ** 0.5, beta_end ** 0.5, num_train_timesteps, dtype=torch.float32) ** 2
    return torch.cumprod(1.0 - betas, dim=0)


class EulerAncestralDiscreteScheduler:
    def __init__(self, num_train_timesteps=1000, beta_start=0.00085, beta_end=0.012, timestep_spacing="trailing"):
        assert timestep_spacing == "trailing", "SDXL-Turbo uses trailing spacing"
        self.num_train_timesteps = num_train_timesteps
        self.alphas_cumprod = _alphas_cumprod(num_train_timesteps, beta_start, beta_end)
        sig = (((1 - self.alphas_cumprod) / self.alphas_cumprod) ** 0.5).numpy()
        self.sigmas = torch.from_numpy(np.concatenate([sig[::-1], [0.0]]).astype(np.float32))
        self.timesteps = None
        self.num_inference_steps = None
        self.is_scale_input_called = False

    @classmethod
    def from_pretrained(cls, *a, **kw):
        return cls()

    @property
    def init_noise_sigma(self):
        return self.sigmas.max()

    def set_timesteps(self, num_inference_steps, device=None):
        self.num_inference_steps = num_inference_steps
        ratio = self.num_train_timesteps / num_inference_steps
        ts = np.arange(self.num_train_timesteps, 0, -ratio).round().copy().astype(np.float32) - 1
        sig = (((1 - self.alphas_cumprod) / self.alphas_cumprod) ** 0.5).numpy()
        sig = np.interp(ts, np.arange(0, len(sig)), sig)
        self.sigmas = torch.from_numpy(np.concatenate([sig, [0.0]]).astype(np.float32))
        self.timesteps = torch.from_numpy(ts)
        if device is not None:
            self.sigmas = self.sigmas.to(device)
            self.timesteps = self.timesteps.to(device)


class EulerDiscreteScheduler:
    """diffusers EulerDiscreteScheduler in its training configuration (no set_timesteps), as the DreamBooth trainer
    loads it for EDM-style training (DB:1234-1237): timesteps 999..0, sigmas sqrt((1-abar)/abar) reversed + [0];
    `add_noise(x0, noise, t) = x0 + noise * sigma(t)`; `get_sigmas` = DB:1675-1685."""

    def __init__(self, num_train_timesteps=1000, beta_start=0.00085, beta_end=0.012):
        self.num_train_timesteps = num_train_timesteps
        self.alphas_cumprod = _alphas_cumprod(num_train_timesteps, beta_start, beta_end)
        sig = (((1 - self.alphas_cumprod) / self.alphas_cumprod) ** 0.5).numpy()
        self.sigmas = torch.from_numpy(np.concatenate([sig[::-1], [0.0]]).astype(np.float32))
        self.timesteps = torch.from_numpy(np.linspace(0, num_train_timesteps - 1, num_train_timesteps,
                                                      dtype=np.float32)[::-1].copy())
        self.config = type("Cfg", (), {"num_train_timesteps": num_train_timesteps, "prediction_type": "epsilon"})()

    @classmethod
    def from_pretrained(cls, *a, **kw):
        return cls()

    def sigma_at(self, t):
        """sigma of integer timesteps t (any shape): sigmas[index of t in timesteps] = sigmas[999 - t].  Indexed on
        t's device (a device-resident copy of the table), so the DreamBooth micro-step never syncs the host."""
        t = torch.as_tensor(t).long()
        if self.sigmas.device != t.device:
            self._dev_sigmas = getattr(self, "_dev_sigmas", None)
            if self._dev_sigmas is None or self._dev_sigmas.device != t.device:
                self._dev_sigmas = self.sigmas.to(t.device)
            return self._dev_sigmas[(self.num_train_timesteps - 1) - t]
        return self.sigmas[(self.num_train_timesteps - 1) - t]


def db_distill_timesteps(raw, distill_train_timesteps=4, num_train_timesteps=1000):
    """DB:1769-1777: raw draws in [0, 1000) -> stride * (raw % steps) + stride - 1 ({249, 499, 749, 999} at 4)."""
    stride = num_train_timesteps // distill_train_timesteps
    return stride * (raw % distill_train_timesteps) + stride - 1


class LCMScheduler:
    def __init__(self, num_train_timesteps=1000, beta_start=0.00085, beta_end=0.012):
        self.alphas_cumprod = _alphas_cumprod(num_train_timesteps, beta_start, beta_end)
        self.final_alpha_cumprod = torch.tensor(1.0)
        self.init_noise_sigma = 1.0
        self.config = type("Cfg", (), {"num_train_timesteps": num_train_timesteps})()

    @classmethod
    def from_pretrained(cls, *a, **kw):
        return cls()


def dmd_distill_timesteps(num_steps):
    """D:542-548 in integer arithmetic: [999, 749, 499, 249] for 4 steps (the bf16 cast bug of App. A #3 avoided)."""
    step_ratio = 1000 // num_steps
    return torch.from_numpy((np.arange(num_steps, 0, -1) * step_ratio).astype(np.int64) - 1), step_ratio
