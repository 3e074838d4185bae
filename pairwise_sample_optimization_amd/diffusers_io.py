"""diffusers checkpoint boundary of the UNet / VAE drop-ins: `from_pretrained(path, subfolder=...)`,
`from_config(dict)` honouring the diffusers config keys, `save_pretrained(path)`.

Reference call sites: `UNet2DConditionModel.from_pretrained(config.pretrained.pretrained_model_name_or_path,
subfolder="unet", revision=...)` (T:290), `UNet2DConditionModel.from_config(UNet2DConditionModel.load_config(base,
subfolder="unet"))` + `load_state_dict(torch.load(hf_hub_download("tianweiy/DMD2", ...)))` (D:310-318),
`AutoencoderKL.from_pretrained(vae_path, subfolder=...)` (T:273-284).  A local diffusers directory is read directly
(`<path>/<subfolder>/config.json` + `diffusion_pytorch_model[.<variant>].safetensors`, or the `.bin` through
`torch.load(weights_only=True)`); there is no hub download (no network on this build), a hub id raises a clear
error.  Only what the SDXL / SDXL-VAE configurations use is accepted: an option the kernels do not implement
(another attention layout, time-embedding variant, activation ...) raises ValueError instead of silently loading a
different network.
"""
import json
import os

import torch

WEIGHTS = ("diffusion_pytorch_model.safetensors", "diffusion_pytorch_model.bin")


def _seq(v, n):
    return list(v) if isinstance(v, (list, tuple)) else [v] * n


def _check(cfg, key, allowed):
    v = cfg.get(key, allowed[0])
    if v not in allowed:
        raise ValueError(f"diffusers config {key}={v!r} is not supported by this build (supported: {allowed})")


def unet_config_from_diffusers(d):
    """diffusers UNet2DConditionModel config dict -> UNetConfig (SDXL topology family)."""
    from .unet import UNetConfig
    ch = tuple(d.get("block_out_channels", (320, 640, 1280)))
    n = len(ch)
    down = d.get("down_block_types", ["DownBlock2D"] + ["CrossAttnDownBlock2D"] * (n - 1))
    up = d.get("up_block_types", ["CrossAttnUpBlock2D"] * (n - 1) + ["UpBlock2D"])
    if len(down) != n or len(up) != n:
        raise ValueError("down_block_types / up_block_types must have one entry per block_out_channels level")
    has_attn = tuple(t.startswith("CrossAttn") for t in down)
    if tuple(t.startswith("CrossAttn") for t in reversed(up)) != has_attn:
        raise ValueError("up_block_types must mirror down_block_types (attention on the same levels)")
    for t in list(down) + list(up):
        if t not in ("DownBlock2D", "CrossAttnDownBlock2D", "UpBlock2D", "CrossAttnUpBlock2D"):
            raise ValueError(f"block type {t!r} is not supported by this build")
    _check(d, "mid_block_type", ["UNetMidBlock2DCrossAttn"])
    _check(d, "addition_embed_type", ["text_time"])
    _check(d, "use_linear_projection", [True])
    _check(d, "act_fn", ["silu"])
    _check(d, "flip_sin_to_cos", [True])
    _check(d, "freq_shift", [0])
    _check(d, "resnet_time_scale_shift", ["default"])
    _check(d, "time_embedding_type", ["positional"])
    _check(d, "conv_in_kernel", [3])
    _check(d, "conv_out_kernel", [3])
    _check(d, "upcast_attention", [None, False])
    _check(d, "class_embed_type", [None])
    _check(d, "encoder_hid_dim", [None])
    _check(d, "time_cond_proj_dim", [None])
    _check(d, "dual_cross_attention", [False])
    _check(d, "only_cross_attention", [False])
    heads = _seq(d.get("num_attention_heads") or d.get("attention_head_dim", [5, 10, 20]), n)
    for c, h in zip(ch, heads):  # diffusers' attention_head_dim of SDXL is really the head COUNT per level
        if c % h or c // h != 64:
            raise ValueError(f"attention head dim {c}/{h} != 64 (the flash-attention kernels are d = 64)")
    if not isinstance(d.get("layers_per_block", 2), int):
        raise ValueError("layers_per_block must be an int")
    tdim = d.get("addition_time_embed_dim", 256)
    proj_in = d.get("projection_class_embeddings_input_dim", 2816)
    return UNetConfig(in_channels=d.get("in_channels", 4), out_channels=d.get("out_channels", 4),
                      block_out_channels=ch, layers_per_block=int(d.get("layers_per_block", 2)),
                      transformer_layers_per_block=tuple(_seq(d.get("transformer_layers_per_block", 1), n)),
                      down_has_attn=has_attn, head_dim=64, cross_attention_dim=d.get("cross_attention_dim", 2048),
                      addition_time_embed_dim=tdim, text_embed_dim=proj_in - 6 * tdim,
                      norm_num_groups=d.get("norm_num_groups", 32), norm_eps=d.get("norm_eps", 1e-5),
                      time_proj_dim=ch[0], sample_size=d.get("sample_size", 128))


def unet_config_to_diffusers(c):
    """UNetConfig -> the diffusers config dict (the keys unet_config_from_diffusers reads)."""
    return {"_class_name": "UNet2DConditionModel", "_diffusers_version": "0.27.0", "act_fn": "silu",
            "addition_embed_type": "text_time", "addition_time_embed_dim": c.addition_time_embed_dim,
            "attention_head_dim": [ch // c.head_dim for ch in c.block_out_channels],
            "block_out_channels": list(c.block_out_channels), "cross_attention_dim": c.cross_attention_dim,
            "down_block_types": ["CrossAttnDownBlock2D" if a else "DownBlock2D" for a in c.down_has_attn],
            "up_block_types": ["CrossAttnUpBlock2D" if a else "UpBlock2D" for a in reversed(c.down_has_attn)],
            "mid_block_type": "UNetMidBlock2DCrossAttn", "flip_sin_to_cos": True, "freq_shift": 0,
            "in_channels": c.in_channels, "out_channels": c.out_channels, "layers_per_block": c.layers_per_block,
            "norm_eps": c.norm_eps, "norm_num_groups": c.norm_num_groups,
            "projection_class_embeddings_input_dim": c.projection_class_embeddings_input_dim,
            "sample_size": c.sample_size, "transformer_layers_per_block": list(c.transformer_layers_per_block),
            "use_linear_projection": True}


def vae_config_from_diffusers(d):
    from .vae import VAEConfig
    for t in d.get("down_block_types", []):
        if t != "DownEncoderBlock2D":
            raise ValueError(f"VAE block type {t!r} is not supported by this build")
    for t in d.get("up_block_types", []):
        if t != "UpDecoderBlock2D":
            raise ValueError(f"VAE block type {t!r} is not supported by this build")
    _check(d, "act_fn", ["silu"])
    _check(d, "in_channels", [3])
    _check(d, "out_channels", [3])
    return VAEConfig(latent_channels=d.get("latent_channels", 4), out_channels=3,
                     block_out_channels=tuple(d.get("block_out_channels", (128, 256, 512, 512))),
                     layers_per_block=d.get("layers_per_block", 2), norm_num_groups=d.get("norm_num_groups", 32),
                     scaling_factor=float(d.get("scaling_factor", 0.13025)))


def vae_config_to_diffusers(c):
    n = len(c.block_out_channels)
    return {"_class_name": "AutoencoderKL", "_diffusers_version": "0.27.0", "act_fn": "silu",
            "block_out_channels": list(c.block_out_channels), "down_block_types": ["DownEncoderBlock2D"] * n,
            "up_block_types": ["UpDecoderBlock2D"] * n, "in_channels": 3, "out_channels": 3,
            "latent_channels": c.latent_channels, "layers_per_block": c.layers_per_block,
            "norm_num_groups": c.norm_num_groups, "scaling_factor": c.scaling_factor}


def _resolve(path, subfolder):
    d = os.path.join(path, subfolder) if subfolder else path
    if not os.path.isdir(d):
        raise OSError(f"{d} is not a local diffusers model directory (hub ids cannot be fetched: no network)")
    return d


def load_config(path, subfolder=None):
    with open(os.path.join(_resolve(path, subfolder), "config.json")) as f:
        return json.load(f)


def load_weights(path, subfolder=None, variant=None):
    """The state dict of a diffusers model directory (safetensors preferred; .bin with weights_only=True)."""
    d = _resolve(path, subfolder)
    names = []
    for w in WEIGHTS:
        stem, ext = w.rsplit(".", 1)
        if variant:
            names.append(f"{stem}.{variant}.{ext}")
        names.append(w)
    for nm in names:
        p = os.path.join(d, nm)
        if os.path.exists(p):
            if p.endswith(".safetensors"):
                from safetensors.torch import load_file
                return load_file(p)
            return torch.load(p, map_location="cpu", weights_only=True)
    raise OSError(f"no {' / '.join(names)} in {d}")


def save_pretrained(model, path, config_dict):
    from safetensors.torch import save_file
    os.makedirs(path, exist_ok=True)
    with open(os.path.join(path, "config.json"), "w") as f:
        json.dump(config_dict, f, indent=2)
    sd = {k: v.detach().cpu().contiguous() for k, v in model.state_dict().items()}
    save_file(sd, os.path.join(path, WEIGHTS[0]))
