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
