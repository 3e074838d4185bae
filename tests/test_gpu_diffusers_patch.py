"""The pso_pytorch.diffusers_patch drop-ins against the reference's golden vectors and the
numpy oracle: same signatures, return values and error behaviour as DP/*.py."""
import glob
import os
from types import SimpleNamespace

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
GOLD = sorted(glob.glob(os.path.join(os.path.dirname(__file__), "golden", "pso_*.npz")))


def _sched(d, dev):
    if int(d["mode"]) == 0:
        return SimpleNamespace(sigmas=torch.tensor(d["sigmas"]), timesteps=torch.tensor(d["timesteps"]))
    return SimpleNamespace(alphas_cumprod=torch.tensor(d["alphas_cumprod"]))


@pytest.mark.parametrize("path", GOLD, ids=[os.path.basename(p) for p in GOLD])
def test_step_with_logprob_vs_golden(cuda, path):
    from pairwise_sample_optimization_amd.pso_pytorch.diffusers_patch.turbo_inference_with_logprob import \
        turbo_step_with_logprob
    from pairwise_sample_optimization_amd.pso_pytorch.diffusers_patch.distilled_inference_with_logprob import \
        distilled_step_with_logprob
    d = np.load(path)
    T = lambda k: torch.tensor(d[k], device=cuda)
    sch = _sched(d, cuda)
    for k in range(2):
        for which, col in (("pol", 0), ("ref", 1)):
            eps = T(f"eps_{which}{k}")
            if int(d["mode"]) == 0:
                prev, lp = turbo_step_with_logprob(sch, eps, T("t"), T(f"x{k}"), prev_sample=T(f"prev{k}"))
            else:
                prev, lp = distilled_step_with_logprob(sch, eps, T("t"), T("t_prev"), T(f"x{k}"),
                                                       prev_sample=T(f"prev{k}"))
            assert prev.dtype == torch.float32 and lp.shape == (d["x0"].shape[0],)
            want = d["lp_pol" if which == "pol" else "lp_ref"][:, k]
            np.testing.assert_allclose(lp.cpu().numpy(), want, rtol=1e-6, atol=1e-6)


def test_distilled_step_rejects_generator_and_prev(cuda):
    from pairwise_sample_optimization_amd.pso_pytorch.diffusers_patch.distilled_inference_with_logprob import \
        distilled_step_with_logprob
    from pairwise_sample_optimization_amd.schedulers import LCMScheduler
    x = torch.randn(1, 4, 8, 8, device=cuda)
    t = torch.tensor([999], device=cuda)
    with pytest.raises(ValueError):
        distilled_step_with_logprob(LCMScheduler(), x, t, t - 250, x, generator=torch.Generator(device=cuda),
                                    prev_sample=x)


def test_distilled_step_shares_noise_across_batch(cuda):
    """DP/distilled_inference_with_logprob.py:123-126: one (1,C,H,W) draw re-noises every sample."""
    from pairwise_sample_optimization_amd.pso_pytorch.diffusers_patch.distilled_inference_with_logprob import \
        distilled_step_with_logprob
    from pairwise_sample_optimization_amd.schedulers import LCMScheduler
    sch = LCMScheduler()
    x = torch.randn(1, 4, 8, 8, device=cuda).expand(3, -1, -1, -1).contiguous()
    eps = torch.randn(1, 4, 8, 8, device=cuda).expand(3, -1, -1, -1).contiguous()
    t = torch.full((3,), 749, device=cuda, dtype=torch.long)
    prev, lp = distilled_step_with_logprob(sch, eps, t, t - 250, x)
    assert torch.equal(prev[0], prev[1]) and torch.equal(prev[1], prev[2])


@pytest.mark.parametrize("mode", ["turbo", "dmd"])
def test_pipeline_with_logprob_self_consistent(cuda, mode):
    """Run the sampling pipeline through the HIP UNet/VAE, then recompute every recorded log-prob with the numpy
    oracle from the recorded latents and a fresh UNet evaluation: the trajectory the trainer replays is the one
    that was sampled."""
    from oracle import pso_math
    from pairwise_sample_optimization_amd import schedulers
    from pairwise_sample_optimization_amd.pso_pytorch.diffusers_patch import sdxl_dmd_with_logprob as dmdp
    from pairwise_sample_optimization_amd.pso_pytorch.diffusers_patch import sdxl_turbo_with_logprob as tp
    from pairwise_sample_optimization_amd.unet import UNet2DConditionModel, UNetConfig
    from pairwise_sample_optimization_amd.vae import AutoencoderKL, VAEConfig
    torch.manual_seed(0)
    with torch.device(cuda):
        cfg = UNetConfig.tiny(16)
        unet = UNet2DConditionModel(cfg)
        vae = AutoencoderKL(VAEConfig.tiny())
    unet.init_weights(0)
    vae.init_weights(1)
    B, h = 2, 16
    emb = torch.randn(B, 77, cfg.cross_attention_dim, device=cuda)
    pooled = torch.randn(B, cfg.projection_class_embeddings_input_dim - 6 * cfg.addition_time_embed_dim,
                         device=cuda)
    tid = torch.tensor([[8 * h, 8 * h, 0, 0, 8 * h, 8 * h]], device=cuda, dtype=torch.float32).repeat(B, 1)
    gen = torch.Generator(device=cuda).manual_seed(3)
    if mode == "turbo":
        sch = schedulers.EulerAncestralDiscreteScheduler()
        img, lat, lps, inputs = tp.sdxl_turbo_pipeline_with_logprob(
            None, vae, unet, sch, 8 * h, 8 * h, num_inference_steps=4, generator=gen, prompt_embeds=emb,
            pooled_prompt_embeds=pooled, add_time_ids=tid)
        assert len(lat) == 4 and len(lps) == 3 and len(inputs) == 3
        for i in range(3):
            t = sch.timesteps[i]
            eps = unet(inputs[i], t, encoder_hidden_states=emb,
                       added_cond_kwargs={"time_ids": tid, "text_embeds": pooled}).sample.float()
            c = pso_math.turbo_coefs(sch.sigmas.cpu().numpy(), sch.timesteps.cpu().numpy(),
                                     np.full(B, t.item(), np.float32))
            _, lp = pso_math.turbo_step_logprob(lat[i].float().cpu().numpy(), eps.cpu().numpy(), *c,
                                                prev=lat[i + 1].float().cpu().numpy())
            np.testing.assert_allclose(lps[i].cpu().numpy(), lp, rtol=1e-4, atol=1e-4)
    else:
        sch = schedulers.LCMScheduler()
        ts, _ = schedulers.dmd_distill_timesteps(4)
        ts = ts.to(cuda)
        img, lat, lps = dmdp.sdxl_dmd_pipeline_with_logprob(
            None, vae, unet, ts, sch, 8 * h, 8 * h, num_inference_steps=4, prompt_embeds=emb,
            pooled_prompt_embeds=pooled, add_time_ids=tid)
        assert len(lat) == 5 and len(lps) == 3
        for i in range(3):
            tt = torch.full((B,), int(ts[i]), device=cuda, dtype=torch.long)
            eps = unet(lat[i], tt, emb, added_cond_kwargs={"time_ids": tid, "text_embeds": pooled}).sample.float()
            c = pso_math.dmd_coefs(sch.alphas_cumprod.numpy(), tt.cpu().numpy(), (tt - 250).cpu().numpy())
            _, lp = pso_math.dmd_step_logprob(lat[i].float().cpu().numpy(), eps.cpu().numpy(), *c,
                                              prev=lat[i + 1].float().cpu().numpy())
            np.testing.assert_allclose(lps[i].cpu().numpy(), lp, rtol=1e-4, atol=1e-4)
    assert img.shape == (B, 3, 8 * h, 8 * h) and torch.isfinite(img).all()
