"""CPU checks of the UNet host side: diffusers key layout / parameter count, and the oracle restatement runs on the
product model's state dict (tiny config)."""
import torch


def test_sdxl_param_count_and_keys():
    from pairwise_sample_optimization_amd.unet import UNet2DConditionModel, UNetConfig
    u = UNet2DConditionModel(UNetConfig.sdxl())
    n = sum(p.numel() for p in u.parameters())
    assert abs(n / 1e6 - 2567.46) < 0.1  # SDXL UNet, SURVEY §8a a5
    sd = u.state_dict()
    for k in ["conv_in.weight", "time_embedding.linear_1.weight", "add_embedding.linear_1.weight",
              "down_blocks.0.resnets.0.conv1.weight", "down_blocks.0.downsamplers.0.conv.weight",
              "down_blocks.1.attentions.0.transformer_blocks.1.ff.net.0.proj.weight",
              "down_blocks.2.attentions.1.transformer_blocks.9.attn2.to_k.weight",
              "mid_block.attentions.0.transformer_blocks.9.norm3.weight", "up_blocks.0.resnets.2.conv_shortcut.weight",
              "up_blocks.1.upsamplers.0.conv.weight", "conv_norm_out.weight", "conv_out.weight"]:
        assert k in sd, k
    assert sd["add_embedding.linear_1.weight"].shape == (1280, 2816)
    assert sd["up_blocks.0.resnets.0.conv1.weight"].shape == (1280, 2560, 3, 3)
    assert sd["up_blocks.2.resnets.0.conv1.weight"].shape == (320, 960, 3, 3)


def test_oracle_runs_on_tiny_state_dict():
    from oracle import sdxl_ref
    from pairwise_sample_optimization_amd.unet import UNet2DConditionModel, UNetConfig
    cfg = UNetConfig.tiny(16)
    u = UNet2DConditionModel(cfg).init_weights(0)
    sd = sdxl_ref.sd_to(u.state_dict(), "cpu")
    x = torch.randn(2, 4, 16, 16)
    out = sdxl_ref.unet_forward(sd, x, torch.tensor([999.0, 499.0]), torch.randn(2, 77, 128), torch.randn(2, 64),
                                torch.tensor([[128.0, 128, 0, 0, 128, 128]] * 2),
                                cfg=dict(time_proj_dim=64, addition_time_embed_dim=32))
    assert out.shape == x.shape and torch.isfinite(out).all()
