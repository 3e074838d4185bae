"""GPU parity of the HIP SDXL VAE decoder against the fp32 torch oracle (same diffusers-layout weights)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("which,h", [("tiny", 16), ("sdxl", 32)])
def test_vae_decode_parity(cuda, which, h):
    from oracle import sdxl_ref
    from pairwise_sample_optimization_amd.vae import AutoencoderKL, VAEConfig
    cfg = VAEConfig.tiny() if which == "tiny" else VAEConfig()
    with torch.device(cuda):
        vae = AutoencoderKL(cfg)
    vae.init_weights(0)
    z = torch.randn(2, 4, h, h, device=cuda).bfloat16().float()
    img = vae.decode(z / vae.config.scaling_factor, return_dict=False)[0]
    sd = sdxl_ref.sd_to(vae.state_dict(), cuda)
    ref = sdxl_ref.vae_decode(sd, (z / vae.config.scaling_factor).bfloat16().float())
    rel = ((img - ref).norm() / ref.norm()).item()
    print(f"vae {which} h={h}: rel err {rel:.3e}")
    assert img.shape == (2, 3, 8 * h, 8 * h)
    assert rel < 3e-2


@pytest.mark.parametrize("which,hw", [("tiny", 64), ("sdxl", 128)])
def test_vae_encode_parity(cuda, which, hw):
    """Encoder (DB:1750 `vae.encode(pixel_values).latent_dist`): moments vs the fp32 oracle, incl. the (0,1,0,1)-padded
    stride-2 down-sampling convs."""
    from oracle import sdxl_ref
    from pairwise_sample_optimization_amd.vae import AutoencoderKL, VAEConfig
    cfg = VAEConfig.tiny() if which == "tiny" else VAEConfig()
    with torch.device(cuda):
        vae = AutoencoderKL(cfg)
    vae.init_weights(1)
    x = (torch.rand(2, 3, hw, hw, device=cuda) * 2 - 1).bfloat16().float()
    dist = vae.encode(x).latent_dist
    sd = sdxl_ref.sd_to(vae.state_dict(), cuda)
    mean, logvar = sdxl_ref.vae_encode_moments(sd, x)
    rm = ((dist.mean - mean).norm() / mean.norm()).item()
    rv = ((dist.logvar - logvar).norm() / logvar.norm()).item()
    print(f"vae encode {which} {hw}: mean rel {rm:.3e} logvar rel {rv:.3e}")
    assert dist.mean.shape == (2, cfg.latent_channels, hw // 8, hw // 8)
    assert rm < 3e-2 and rv < 3e-2
    g = torch.Generator(device="cuda").manual_seed(0)
    s = dist.sample(generator=g)
    assert torch.isfinite(s).all() and s.shape == dist.mean.shape


def test_epoch_sampling_decodes_and_scores(cuda):
    """The online epoch's sampling phase (T:554-673): trajectories -> VAE decode of the final latents (NHWC entry,
    DP/sdxl_turbo_with_logprob.py:154-155) -> reward; the NHWC decode equals the NCHW `vae.decode(z / sf)` path bit
    for bit, and the light reward is the per-image mean of that image (pso_pytorch/rewards.py:5-9)."""
    from types import SimpleNamespace
    from pairwise_sample_optimization_amd import kernels as K
    from pairwise_sample_optimization_amd.rewards import light_reward
    from pairwise_sample_optimization_amd.trainer import PSOTrainer, compute_time_ids
    from pairwise_sample_optimization_amd.unet import UNet2DConditionModel, UNetConfig
    from pairwise_sample_optimization_amd.vae import AutoencoderKL, VAEConfig
    h = 16
    with torch.device(cuda):
        unet = UNet2DConditionModel(UNetConfig.tiny(h))
        vae = AutoencoderKL(VAEConfig.tiny())
    unet.init_weights(0)
    unet.add_adapter(SimpleNamespace(r=8, lora_alpha=8))
    unet.prepare()
    vae.init_weights(1)
    tr = PSOTrainer(unet, mode="turbo", num_steps=2, train_batch_size=1)
    g = torch.Generator(device="cuda").manual_seed(3)
    B = 2
    cfg = unet.cfg
    enc = torch.randn(B, 77, cfg.cross_attention_dim, device=cuda, generator=g).bfloat16()
    pooled = torch.randn(B, cfg.text_embed_dim, device=cuda, generator=g).bfloat16()
    tid = compute_time_ids(8 * h, 0, cuda).repeat(B, 1)
    seen = {}

    def reward(img):
        seen["img"] = img
        return light_reward()(img)

    buf = tr.sample_pairs(enc, pooled, tid, h, generator=g, reward_fn=reward, decode_fn=vae.decode_latents_nhwc)
    img = seen["img"]
    assert tuple(img.shape) == (2 * B, 8 * h, 8 * h, 3)
    z = buf["x_final"].permute(0, 3, 1, 2)
    ref = vae.decode_nhwc(z, scale=1.0 / vae.config.scaling_factor)
    assert torch.equal(img, ref)
    assert tuple(buf["rewards"].shape) == (B, 2, 1)
    assert torch.allclose(buf["rewards"].reshape(-1), img.float().reshape(2 * B, -1).mean(1), rtol=1e-5, atol=1e-6)


def test_decode_chunks_at_1024_match_single_images(cuda):
    """8 latents at 1024^2 exceed the kernels' 32-bit per-operand offsets in one pass ([8, 1024, 1024, 256] at the
    last upsampler): the decode runs in chunks of 4 images; each chunk must equal the decode of the same images as
    one batch (bit for bit), and every image its single-image decode up to the batch-size-dependent reduction order."""
    from pairwise_sample_optimization_amd.vae import AutoencoderKL, VAEConfig
    with torch.device(cuda):
        vae = AutoencoderKL(VAEConfig())
    vae.init_weights(2)
    g = torch.Generator(device="cuda").manual_seed(8)
    x = torch.randn(6, 128, 128, 4, device=cuda, generator=g)
    img = vae.decode_latents_nhwc(x)
    assert tuple(img.shape) == (6, 1024, 1024, 3)
    assert torch.equal(img[:4], vae.decode_latents_nhwc(x[:4].contiguous()))
    assert torch.equal(img[4:], vae.decode_latents_nhwc(x[4:].contiguous()))
    for i in (0, 5):
        one = vae.decode_latents_nhwc(x[i:i + 1].contiguous())
        assert ((img[i:i + 1].float() - one.float()).norm() / one.float().norm()).item() < 3e-2  # bf16 bar
