"""The diffusers / config boundary on CPU (no kernels run): from_config(dict) honours and validates the diffusers
config keys, save_pretrained -> from_pretrained(path, subfolder=...) round-trips a synthetic model directory
(config.json + safetensors), and the reference's own run configs load unchanged through the ml_collections
stand-in (when /root/reference is present: the build container only)."""
import json
import os

import pytest
import torch

REF_CFG = "/root/reference/human_preference_tuning/config"


def test_unet_from_config_diffusers_dict_roundtrip():
    from pairwise_sample_optimization_amd import diffusers_io
    from pairwise_sample_optimization_amd.unet import UNet2DConditionModel, UNetConfig
    for cfg in (UNetConfig.sdxl(128), UNetConfig.tiny(16)):
        d = diffusers_io.unet_config_to_diffusers(cfg)
        assert diffusers_io.unet_config_from_diffusers(d) == cfg
    sdxl = {"block_out_channels": [320, 640, 1280], "attention_head_dim": [5, 10, 20],
            "transformer_layers_per_block": [1, 2, 10], "cross_attention_dim": 2048, "addition_time_embed_dim": 256,
            "projection_class_embeddings_input_dim": 2816, "use_linear_projection": True, "sample_size": 128,
            "down_block_types": ["DownBlock2D", "CrossAttnDownBlock2D", "CrossAttnDownBlock2D"],
            "up_block_types": ["CrossAttnUpBlock2D", "CrossAttnUpBlock2D", "UpBlock2D"],
            "addition_embed_type": "text_time", "norm_num_groups": 32, "layers_per_block": 2}
    u = UNet2DConditionModel.from_config(sdxl)
    assert u.cfg == UNetConfig.sdxl(128)
    assert sum(p.numel() for p in u.parameters()) == 2_567_463_684  # diffusers SDXL UNet parameter count
    assert u.config.in_channels == 4
    with pytest.raises(ValueError):
        UNet2DConditionModel.from_config(dict(sdxl, use_linear_projection=False))
    with pytest.raises(ValueError):
        UNet2DConditionModel.from_config(dict(sdxl, attention_head_dim=[8, 8, 8]))


def test_unet_and_vae_save_from_pretrained_roundtrip(tmp_path):
    from pairwise_sample_optimization_amd.unet import UNet2DConditionModel, UNetConfig
    from pairwise_sample_optimization_amd.vae import AutoencoderKL, VAEConfig
    u = UNet2DConditionModel(UNetConfig.tiny(16)).init_weights(3)
    u.save_pretrained(str(tmp_path / "unet"))
    cfgj = json.load(open(tmp_path / "unet" / "config.json"))
    assert cfgj["_class_name"] == "UNet2DConditionModel" and "down_blocks.1.attentions.0.proj_in.weight" in \
        __import__("safetensors.torch", fromlist=["load_file"]).load_file(
            str(tmp_path / "unet" / "diffusion_pytorch_model.safetensors"))
    u2 = UNet2DConditionModel.from_pretrained(str(tmp_path), subfolder="unet")
    a, b = u.state_dict(), u2.state_dict()
    assert a.keys() == b.keys() and all(torch.equal(a[k], b[k]) for k in a)
    assert any(".ff.net.0.proj." in k for k in a)  # diffusers key layout
    v = AutoencoderKL(VAEConfig.tiny()).init_weights(4)
    v.save_pretrained(str(tmp_path / "vae"))
    v2 = AutoencoderKL.from_pretrained(str(tmp_path / "vae"))
    assert v2.config.scaling_factor == v.config.scaling_factor
    assert all(torch.equal(v.state_dict()[k], v2.state_dict()[k]) for k in v.state_dict())
    with pytest.raises(OSError):
        UNet2DConditionModel.from_pretrained("stabilityai/sdxl-turbo", subfolder="unet")  # a hub id: no network


@pytest.mark.skipif(not os.path.isdir(REF_CFG), reason="reference configs live in the build container only")
@pytest.mark.parametrize("name,ours", [("config_sdxl_turbo_dpo.py", "config_sdxl_turbo_dpo"),
                                       ("config_sdxl_dmd_dpo.py", "config_sdxl_dmd_dpo")])
def test_reference_run_configs_load_unchanged(name, ours):
    import importlib
    from pairwise_sample_optimization_amd.config import load_config_file, apply_overrides
    ref = load_config_file(os.path.join(REF_CFG, name))
    mine = importlib.import_module(f"pairwise_sample_optimization_amd.config.{ours}").get_config()
    # every key the trainers read has the reference's value in the package's own config module
    for k in ("seed", "num_epochs", "checkpointing_steps", "mixed_precision"):
        assert mine[k] == ref[k], k
    for k in ("num_steps", "batch_size", "num_batches_per_epoch"):
        assert mine.sample[k] == ref.sample[k], k
    for k in ("lora_rank", "distilled_train_steps", "batch_size", "use_8bit_adam", "learning_rate", "adam_beta1",
              "adam_beta2", "adam_weight_decay", "adam_epsilon", "gradient_accumulation_steps", "max_grad_norm",
              "num_inner_epochs", "beta", "eps"):
        assert mine.train[k] == ref.train[k], k
    apply_overrides(ref, ["--config.train.beta=5", "train.eps=0.2", "sample.num_steps=2"])
    assert ref.train.beta == 5 and ref.train.eps == 0.2 and ref.sample.num_steps == 2
    with pytest.raises(KeyError):
        apply_overrides(ref, ["train.not_a_key=1"])
