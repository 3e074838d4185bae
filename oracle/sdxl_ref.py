"""ORACLE (test infrastructure only) -- plain-PyTorch fp32 restatement of the diffusers 0.27.0 SDXL
UNet2DConditionModel forward (+ peft LoRA) and AutoencoderKL decoder / encoder, reading diffusers-layout state dicts.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module.  It is the checker (and
the CPU baseline), never the product.  diffusers/peft are not vendored in the reference and not installed here
("parity unpinned" at the UNet/VAE boundary), so this is an independent restatement of their published
algorithm written NCHW with torch.nn.functional ops, deliberately sharing no code with the HIP implementation.
"""
import math

import torch
import torch.nn.functional as F


def _lin(sd, p, x, lora=None, lora_scale=1.0):
    y = F.linear(x, sd[p + ".weight"], sd.get(p + ".bias"))
    if lora is not None and p + ".lora_A.weight" in lora:
        y = y + F.linear(F.linear(x, lora[p + ".lora_A.weight"]), lora[p + ".lora_B.weight"]) * lora_scale
    return y


def _conv(sd, p, x, stride=1):
    w = sd[p + ".weight"]
    return F.conv2d(x, w, sd.get(p + ".bias"), stride=stride, padding=w.shape[-1] // 2)


def _gn(sd, p, x, eps, groups=32):
    return F.group_norm(x, groups, sd[p + ".weight"], sd[p + ".bias"], eps)


def timestep_embedding(t, dim):
    """diffusers get_timestep_embedding(flip_sin_to_cos=True, downscale_freq_shift=0, max_period=10000)."""
    half = dim // 2
    ex = torch.exp(-math.log(10000) * torch.arange(half, dtype=torch.float32, device=t.device) / half)
    a = t[:, None].float() * ex[None]
    e = torch.cat([torch.sin(a), torch.cos(a)], -1)
    return torch.cat([e[:, half:], e[:, :half]], -1)


def resnet(sd, p, x, temb, eps=1e-5):
    h = F.silu(_gn(sd, p + ".norm1", x, eps))
    h = _conv(sd, p + ".conv1", h)
    if temb is not None:
        h = h + _lin(sd, p + ".time_emb_proj", F.silu(temb))[:, :, None, None]
    h = F.silu(_gn(sd, p + ".norm2", h, eps))
    h = _conv(sd, p + ".conv2", h)
    if p + ".conv_shortcut.weight" in sd:
        x = _conv(sd, p + ".conv_shortcut", x)
    return x + h


def attention(sd, p, x, ctx, lora, heads_dim=64, self_attn=True):
    q = _lin(sd, p + ".to_q", x, lora)
    kv_in = x if self_attn else ctx
    k = _lin(sd, p + ".to_k", kv_in, lora)
    v = _lin(sd, p + ".to_v", kv_in, lora)
    B, S, C = q.shape
    H = C // heads_dim
    sp = lambda t: t.reshape(B, t.shape[1], H, heads_dim).transpose(1, 2)
    o = F.scaled_dot_product_attention(sp(q), sp(k), sp(v)).transpose(1, 2).reshape(B, S, C)
    return _lin(sd, p + ".to_out.0", o, lora)


def transformer_block(sd, p, x, ctx, lora):
    C = x.shape[-1]
    ln = lambda n, t: F.layer_norm(t, (C,), sd[f"{p}.{n}.weight"], sd[f"{p}.{n}.bias"], 1e-5)
    x = attention(sd, p + ".attn1", ln("norm1", x), None, lora) + x
    x = attention(sd, p + ".attn2", ln("norm2", x), ctx, lora, self_attn=False) + x
    h, gate = _lin(sd, p + ".ff.net.0.proj", ln("norm3", x)).chunk(2, dim=-1)
    return _lin(sd, p + ".ff.net.2", h * F.gelu(gate)) + x


def transformer2d(sd, p, x, ctx, lora):
    B, C, H, W = x.shape
    res = x
    h = _gn(sd, p + ".norm", x, 1e-6).permute(0, 2, 3, 1).reshape(B, H * W, C)
    h = _lin(sd, p + ".proj_in", h)
    i = 0
    while f"{p}.transformer_blocks.{i}.norm1.weight" in sd:
        h = transformer_block(sd, f"{p}.transformer_blocks.{i}", h, ctx, lora)
        i += 1
    h = _lin(sd, p + ".proj_out", h)
    return h.reshape(B, H, W, C).permute(0, 3, 1, 2) + res


def unet_forward(sd, sample, timestep, ctx, text_embeds, time_ids, lora=None, cfg=None):
    """diffusers UNet2DConditionModel.forward for the SDXL configuration.  All tensors fp32 NCHW."""
    cfg = cfg or {}
    tp = cfg.get("time_proj_dim", 320)
    atd = cfg.get("addition_time_embed_dim", 256)
    B = sample.shape[0]
    t = timestep.float().reshape(-1)
    if t.numel() == 1:
        t = t.expand(B)
    emb = _lin(sd, "time_embedding.linear_2", F.silu(_lin(sd, "time_embedding.linear_1", timestep_embedding(t, tp))))
    te = timestep_embedding(time_ids.reshape(-1), atd).reshape(B, -1)
    add = torch.cat([text_embeds, te], -1)
    emb = emb + _lin(sd, "add_embedding.linear_2", F.silu(_lin(sd, "add_embedding.linear_1", add)))
    h = _conv(sd, "conv_in", sample)
    skips = [h]
    i = 0
    while f"down_blocks.{i}.resnets.0.norm1.weight" in sd:
        j = 0
        while f"down_blocks.{i}.resnets.{j}.norm1.weight" in sd:
            h = resnet(sd, f"down_blocks.{i}.resnets.{j}", h, emb)
            if f"down_blocks.{i}.attentions.{j}.norm.weight" in sd:
                h = transformer2d(sd, f"down_blocks.{i}.attentions.{j}", h, ctx, lora)
            skips.append(h)
            j += 1
        if f"down_blocks.{i}.downsamplers.0.conv.weight" in sd:
            h = _conv(sd, f"down_blocks.{i}.downsamplers.0.conv", h, stride=2)
            skips.append(h)
        i += 1
    h = resnet(sd, "mid_block.resnets.0", h, emb)
    h = transformer2d(sd, "mid_block.attentions.0", h, ctx, lora)
    h = resnet(sd, "mid_block.resnets.1", h, emb)
    i = 0
    while f"up_blocks.{i}.resnets.0.norm1.weight" in sd:
        j = 0
        while f"up_blocks.{i}.resnets.{j}.norm1.weight" in sd:
            h = torch.cat([h, skips.pop()], 1)
            h = resnet(sd, f"up_blocks.{i}.resnets.{j}", h, emb)
            if f"up_blocks.{i}.attentions.{j}.norm.weight" in sd:
                h = transformer2d(sd, f"up_blocks.{i}.attentions.{j}", h, ctx, lora)
            j += 1
        if f"up_blocks.{i}.upsamplers.0.conv.weight" in sd:
            h = _conv(sd, f"up_blocks.{i}.upsamplers.0.conv", F.interpolate(h, scale_factor=2.0, mode="nearest"))
        i += 1
    h = F.silu(_gn(sd, "conv_norm_out", h, 1e-5))
    return _conv(sd, "conv_out", h)


# ---------------------------------------------------------------------------------------------------------------------
# AutoencoderKL decoder (SDXL VAE: latent 4, channels 128/256/512/512, 3 resnets per up block, eps 1e-6)
# ---------------------------------------------------------------------------------------------------------------------
def vae_attention(sd, p, x):
    B, C, H, W = x.shape
    res = x
    h = _gn(sd, p + ".group_norm", x, 1e-6).reshape(B, C, H * W).transpose(1, 2)
    q, k, v = (_lin(sd, f"{p}.{n}", h) for n in ("to_q", "to_k", "to_v"))
    o = F.scaled_dot_product_attention(q[:, None], k[:, None], v[:, None])[:, 0]
    o = _lin(sd, p + ".to_out.0", o)
    return o.transpose(1, 2).reshape(B, C, H, W) + res


def vae_decode(sd, z):
    """AutoencoderKL.decode(z) with z already divided by scaling_factor: post_quant_conv -> decoder."""
    h = _conv(sd, "post_quant_conv", z)
    h = _conv(sd, "decoder.conv_in", h)
    h = resnet(sd, "decoder.mid_block.resnets.0", h, None, eps=1e-6)
    h = vae_attention(sd, "decoder.mid_block.attentions.0", h)
    h = resnet(sd, "decoder.mid_block.resnets.1", h, None, eps=1e-6)
    i = 0
    while f"decoder.up_blocks.{i}.resnets.0.norm1.weight" in sd:
        j = 0
        while f"decoder.up_blocks.{i}.resnets.{j}.norm1.weight" in sd:
            h = resnet(sd, f"decoder.up_blocks.{i}.resnets.{j}", h, None, eps=1e-6)
            j += 1
        if f"decoder.up_blocks.{i}.upsamplers.0.conv.weight" in sd:
            h = _conv(sd, f"decoder.up_blocks.{i}.upsamplers.0.conv", F.interpolate(h, scale_factor=2.0,
                                                                                    mode="nearest"))
        i += 1
    h = F.silu(_gn(sd, "decoder.conv_norm_out", h, 1e-6))
    return _conv(sd, "decoder.conv_out", h)


def vae_encode_moments(sd, x):
    """AutoencoderKL.encode(x).latent_dist parameters: encoder -> quant_conv -> (mean, logvar clamped to [-30, 20]).
    diffusers Encoder: the down-sampling convs pad (0, 1, 0, 1) then stride 2 with padding 0."""
    h = _conv(sd, "encoder.conv_in", x)
    i = 0
    while f"encoder.down_blocks.{i}.resnets.0.norm1.weight" in sd:
        j = 0
        while f"encoder.down_blocks.{i}.resnets.{j}.norm1.weight" in sd:
            h = resnet(sd, f"encoder.down_blocks.{i}.resnets.{j}", h, None, eps=1e-6)
            j += 1
        p = f"encoder.down_blocks.{i}.downsamplers.0.conv"
        if p + ".weight" in sd:
            h = F.conv2d(F.pad(h, (0, 1, 0, 1)), sd[p + ".weight"], sd[p + ".bias"], stride=2)
        i += 1
    h = resnet(sd, "encoder.mid_block.resnets.0", h, None, eps=1e-6)
    h = vae_attention(sd, "encoder.mid_block.attentions.0", h)
    h = resnet(sd, "encoder.mid_block.resnets.1", h, None, eps=1e-6)
    h = F.silu(_gn(sd, "encoder.conv_norm_out", h, 1e-6))
    h = _conv(sd, "encoder.conv_out", h)
    h = _conv(sd, "quant_conv", h)
    mean, logvar = h.chunk(2, dim=1)
    return mean, logvar.clamp(-30.0, 20.0)


def sd_to(sd, device, dtype=torch.float32):
    return {k: v.to(device=device, dtype=dtype) for k, v in sd.items()}
