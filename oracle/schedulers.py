"""ORACLE (test infrastructure only) -- CPU restatement of the two noise-scheduler tables the PSO hot path reads.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module.

The reference never defines these tables itself: it reads them from diffusers==0.27.0 schedulers
(`environment.yml:15`), which are not vendored and not installed here.  This file restates the published
diffusers 0.27 algorithm for exactly the attributes the reference touches:

* EulerAncestralDiscreteScheduler (SDXL-Turbo, `train_online_pso_sdxl_turbo.py:264-268`):
  `.timesteps`, `.sigmas`, `.init_noise_sigma`, `.set_timesteps(N)` with `timestep_spacing="trailing"`
  (read by `DP/sdxl_turbo_with_logprob.py:99-103,120` and `DP/turbo_inference_with_logprob.py:61-66`).
* LCMScheduler (DMD2, `train_online_pso_sdxl_dmd2.py:285`): `.alphas_cumprod`
  (read by `DP/distilled_inference_with_logprob.py:36-42,84-112`).

Both use the SDXL "scaled_linear" beta schedule, beta_start=0.00085, beta_end=0.012, 1000 train steps
(SURVEY.md Appendix C).  All tables are float32, like diffusers'.
"""
import numpy as np
import torch

NUM_TRAIN_TIMESTEPS = 1000
BETA_START = 0.00085
BETA_END = 0.012


def alphas_cumprod_f32():
    """diffusers `betas = linspace(sqrt(b0), sqrt(b1), T, float32) ** 2; alphas_cumprod = cumprod(1 - betas)`."""
    betas = torch.linspace(BETA_START ** 0.5, BETA_END ** 0.5, NUM_TRAIN_TIMESTEPS, dtype=torch.float32) ** 2
    return torch.cumprod(1.0 - betas, dim=0)


class EulerAncestralTrailing:
    """Restated EulerAncestralDiscreteScheduler state (diffusers 0.27, trailing spacing)."""

    def __init__(self):
        self.alphas_cumprod = alphas_cumprod_f32()
        full = np.array(((1 - self.alphas_cumprod) / self.alphas_cumprod) ** 0.5)
        self.sigmas = torch.from_numpy(np.concatenate([full[::-1], [0.0]]).astype(np.float32))
        self.timesteps = None
        self.num_inference_steps = None

    @property
    def init_noise_sigma(self):
        # trailing/linspace spacing => max sigma (not sqrt(max^2+1))
        return self.sigmas.max()

    def set_timesteps(self, num_inference_steps, device=None):
        self.num_inference_steps = num_inference_steps
        step_ratio = NUM_TRAIN_TIMESTEPS / num_inference_steps
        timesteps = np.arange(NUM_TRAIN_TIMESTEPS, 0, -step_ratio).round().copy().astype(np.float32)
        timesteps -= 1
        sig = np.array(((1 - self.alphas_cumprod) / self.alphas_cumprod) ** 0.5)
        sig = np.interp(timesteps, np.arange(0, len(sig)), sig)
        sig = np.concatenate([sig, [0.0]]).astype(np.float32)
        self.sigmas = torch.from_numpy(sig)
        self.timesteps = torch.from_numpy(timesteps)
        if device is not None:
            self.sigmas = self.sigmas.to(device)
            self.timesteps = self.timesteps.to(device)


class LCMTable:
    """The only LCMScheduler attribute the DMD2 path reads: `.alphas_cumprod` (float32, length 1000)."""

    def __init__(self):
        self.alphas_cumprod = alphas_cumprod_f32()
        self.final_alpha_cumprod = torch.tensor(1.0)
        self.init_noise_sigma = 1.0


def dmd_distill_timesteps(num_steps):
    """`D:542-548` restated with integer arithmetic (the fp32/fp16 result; bf16 is the App. A #3 bug)."""
    step_ratio = 1000 // num_steps
    return (np.arange(num_steps, 0, -1) * step_ratio).round().astype(np.int64) - 1, step_ratio
