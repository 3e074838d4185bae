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
