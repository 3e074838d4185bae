"""SDXL AutoencoderKL decoder and encoder (forward only) on the libpso_amd HIP kernels -- the reward-image decode of the

Drop-in surface: `vae.decode(z, return_dict=False)[0]`, `vae.config.scaling_factor`, diffusers
state-dict keys (`post_quant_conv.*`, `decoder.*`; `encoder.*` / `quant_conv.*` of a full checkpoint are accepted and
ignored).  Called at DP/sdxl_turbo_with_logprob.py:154-155 and DP/sdxl_dmd_with_logprob.py:167-168 with the fp16-fix
SDXL VAE (config_sdxl_turbo_dpo.py:52).  Architecture restated from diffusers 0.27.0 Decoder: post_quant_conv (1x1)
-> conv_in (4->512) -> mid (resnet, single-head attention over H*W tokens, resnet) -> 4 UpDecoderBlock2D (3 resnets
each; channels 512,512,256,128; nearest-2x upsample + conv on the first three) -> GroupNorm+SiLU -> conv_out (3).
GroupNorm eps 1e-6, 32 groups, no time embedding.

All activations NHWC bf16.  The mid-block attention has head dim 512 (outside the d=64 flash kernel); its 16384 x 16384
score matrix per image is small next to 288 GB, so it runs as one batched GEMM (scores, bf16, every image) -> row
softmax -> one batched GEMM.

The encoder (the DreamBooth PSO step's `vae.encode(pixel_values).latent_dist.sample()`, DB:1750) is
restated from diffusers 0.27.0 Encoder: conv_in (3->128) -> 4 DownEncoderBlock2D (2 resnets each; channels
128,256,512,512; a stride-2 3x3 conv with (0,1,0,1) padding on the first three) -> mid (resnet, attention, resnet)
-> GroupNorm+SiLU -> conv_out (2*latent) -> quant_conv (1x1) -> DiagonalGaussianDistribution (logvar clamped to
[-30, 20]).
"""
import math
from dataclasses import dataclass
from types import SimpleNamespace

import torch
import torch.nn as nn

from . import kernels as K
from .unet import Conv2d, Linear, Norm, ResnetBlock2D, Upsample2D

BF16 = torch.bfloat16


@dataclass
class VAEConfig:
    latent_channels: int = 4
    out_channels: int = 3
    block_out_channels: tuple = (128, 256, 512, 512)
    layers_per_block: int = 2
    norm_num_groups: int = 32
    scaling_factor: float = 0.13025

    @staticmethod
    def tiny():
        return VAEConfig(block_out_channels=(64, 64, 128, 128))


class VAEAttention(nn.Module):
    def __init__(self, C, groups):
        super().__init__()
        self.C, self.groups = C, groups
        self.group_norm = Norm(C)
        self.to_q, self.to_k, self.to_v = Linear(C, C), Linear(C, C), Linear(C, C)
        self.to_out = nn.ModuleList([Linear(C, C)])

    def prepare(self):
        self.w_qkv = torch.cat([self.to_q.weight.data, self.to_k.weight.data, self.to_v.weight.data], 0)
        self.b_qkv = torch.cat([self.to_q.bias.data, self.to_k.bias.data, self.to_v.bias.data], 0)

    def fwd(self, x):
        B, H, W, C = x.shape
        S = H * W
        hn, _ = K.group_norm_fwd(x, self.group_norm.weight, self.group_norm.bias, self.groups, 1e-6, False)
        qkv = K.gemm(hn.view(-1, C), self.w_qkv, bias=self.b_qkv).view(B, S, 3 * C)
        scale = 1.0 / math.sqrt(C)
        # every image in one launch per product: S_b = Q_b K_b^T (bf16, B x 512 MB at 1024^2), row softmax,
        # O_b = P_b V_b with V_b transposed once for all images (one batched transpose)
        s = K.gemm_batched(qkv[:, :, :C], qkv[:, :, C:2 * C], alpha=scale)            # [B, S, S]
        K.softmax_rows(s.view(B * S, S))
        vt = K.transpose_batched(qkv[:, :, 2 * C:])                                    # [B, C, S]
        out = K.gemm_batched(s, vt)                                                    # [B, S, C]
        o = self.to_out[0]
        return K.gemm(out.view(B * S, C), o.weight, bias=o.bias, resid=x.view(-1, C)).view(B, H, W, C)


class _Blk(nn.Module):
    pass


class Decoder(nn.Module):
    def __init__(self, cfg: VAEConfig):
        super().__init__()
        ch = list(reversed(cfg.block_out_channels))
        G = cfg.norm_num_groups
        self.conv_in = Conv2d(cfg.latent_channels, ch[0], 3)
        mid = _Blk()
        mid.resnets = nn.ModuleList([ResnetBlock2D(ch[0], ch[0], G, 1e-6, 0), ResnetBlock2D(ch[0], ch[0], G, 1e-6, 0)])
        mid.attentions = nn.ModuleList([VAEAttention(ch[0], G)])
        self.mid_block = mid
        self.up_blocks = nn.ModuleList()
        prev = ch[0]
        for i, c in enumerate(ch):
            blk = _Blk()
            blk.resnets = nn.ModuleList([ResnetBlock2D(prev if j == 0 else c, c, G, 1e-6, 0)
                                         for j in range(cfg.layers_per_block + 1)])
            if i < len(ch) - 1:
                blk.upsamplers = nn.ModuleList([Upsample2D(c)])
            prev = c
            self.up_blocks.append(blk)
        self.conv_norm_out = Norm(ch[-1])
        self.conv_out = Conv2d(ch[-1], cfg.out_channels, 3)


class Downsample2DEnc(nn.Module):
    """diffusers Downsample2D(use_conv=True, padding=0) of the encoder: F.pad(x, (0, 1, 0, 1)) then a stride-2 3x3
    conv -- the bottom/right zero row/column are the conv gather's out-of-range taps."""

    def __init__(self, C):
        super().__init__()
        self.conv = Conv2d(C, C, 3, stride=2)

    def prepare(self):
        self.conv.prepare()

    def fwd(self, x):
        B, H, W, C = x.shape
        return K.conv2d(x, self.conv.w_nhwc, stride=2, pad=0, out_hw=(H // 2, W // 2), bias=self.conv.bias)


class Encoder(nn.Module):
    def __init__(self, cfg: VAEConfig):
        super().__init__()
        ch = list(cfg.block_out_channels)
        G = cfg.norm_num_groups
        self.conv_in = Conv2d(cfg.out_channels, ch[0], 3)
        self.down_blocks = nn.ModuleList()
        prev = ch[0]
        for i, c in enumerate(ch):
            blk = _Blk()
            blk.resnets = nn.ModuleList([ResnetBlock2D(prev if j == 0 else c, c, G, 1e-6, 0)
                                         for j in range(cfg.layers_per_block)])
            if i < len(ch) - 1:
                blk.downsamplers = nn.ModuleList([Downsample2DEnc(c)])
            prev = c
            self.down_blocks.append(blk)
        mid = _Blk()
        mid.resnets = nn.ModuleList([ResnetBlock2D(ch[-1], ch[-1], G, 1e-6, 0),
                                     ResnetBlock2D(ch[-1], ch[-1], G, 1e-6, 0)])
        mid.attentions = nn.ModuleList([VAEAttention(ch[-1], G)])
        self.mid_block = mid
        self.conv_norm_out = Norm(ch[-1])
        self.conv_out = Conv2d(ch[-1], 2 * cfg.latent_channels, 3)


class DiagonalGaussianDistribution:
    """diffusers DiagonalGaussianDistribution over NCHW moments [mean | logvar] (logvar clamped to [-30, 20])."""

    def __init__(self, mean, logvar):
        self.mean = mean
        self.logvar = logvar.clamp(-30.0, 20.0)
        self.std = torch.exp(0.5 * self.logvar)
        self.var = torch.exp(self.logvar)

    def sample(self, generator=None):
        noise = torch.randn(self.mean.shape, generator=generator, device=self.mean.device, dtype=self.mean.dtype)
        return self.mean + self.std * noise

    def mode(self):
        return self.mean


class AutoencoderKL(nn.Module):
    def __init__(self, config: VAEConfig = None):
        super().__init__()
        self.cfg = config or VAEConfig()
        self.config = SimpleNamespace(scaling_factor=self.cfg.scaling_factor,
                                      latent_channels=self.cfg.latent_channels)
        self.encoder = Encoder(self.cfg)
        self.quant_conv = Conv2d(2 * self.cfg.latent_channels, 2 * self.cfg.latent_channels, 1)
        self.post_quant_conv = Conv2d(self.cfg.latent_channels, self.cfg.latent_channels, 1)
        self.decoder = Decoder(self.cfg)
        self._prepared = False

    @classmethod
    def from_config(cls, config=None, **kw):
        """A VAEConfig or a diffusers AutoencoderKL config dict (validated: diffusers_io.vae_config_from_diffusers)."""
        from . import diffusers_io
        if isinstance(config, dict):
            config = diffusers_io.vae_config_from_diffusers(dict(config, **kw))
        return cls(config)

    @classmethod
    def from_pretrained(cls, path, subfolder=None, torch_dtype=None, variant=None, revision=None, **kw):
        """`AutoencoderKL.from_pretrained(vae_path, subfolder=...)` (T:273-284) from a local diffusers directory."""
        from . import diffusers_io
        model = cls.from_config(diffusers_io.load_config(path, subfolder))
        model.load_state_dict(diffusers_io.load_weights(path, subfolder, variant))
        return model

    def save_pretrained(self, path):
        from . import diffusers_io
        diffusers_io.save_pretrained(self, path, diffusers_io.vae_config_to_diffusers(self.cfg))

    def init_weights(self, seed=0):
        g = torch.Generator(device=self.post_quant_conv.weight.device).manual_seed(seed)
        for m in self.modules():
            if isinstance(m, (Linear, Conv2d, Norm)):
                m.reset(g)
        self._prepared = False
        return self

    def load_state_dict(self, sd, strict=True):
        """diffusers AutoencoderKL keys (encoder.*, quant_conv.*, post_quant_conv.*, decoder.*).  A decoder-only
        state dict loads with strict=False (the encoder keeps its init)."""
        sd = {k: v.to(BF16) for k, v in sd.items()}
        res = super().load_state_dict(sd, strict=strict)
        self._prepared = False
        return res

    def prepare(self):
        d = self.decoder
        for m in self.modules():
            if isinstance(m, (ResnetBlock2D, Upsample2D, VAEAttention, Downsample2DEnc)):
                m.prepare()
        e = self.encoder
        e.conv_in.prepare()
        e.conv_out.prepare()
        self._qc_w = self.quant_conv.weight.data.reshape(self.quant_conv.cout, self.quant_conv.cin).contiguous()
        d.conv_in.prepare()
        lc = self.cfg.latent_channels
        self._lc_pad = 8 * ((lc + 7) // 8)
        w = self.post_quant_conv.weight.data.reshape(lc, lc)
        self._pq_w = torch.zeros(lc, self._lc_pad, device=w.device, dtype=BF16)
        self._pq_w[:, :lc] = w
        d.conv_out.prepare()
        self._prepared = True

    @torch.no_grad()
    def decode_nhwc(self, z, scale=1.0):
        """z NCHW (fp32/bf16) -> image NHWC bf16 [B, 8h, 8w, 3] (values in about [-1, 1], unclamped)."""
        if not self._prepared:
            self.prepare()
        zp = K.nchw_to_nhwc(z, pad_to=self._lc_pad, scale=scale)                  # [B,h,w,8] (zero-padded C)
        return self._decode_padded(zp)

    def _decode_padded(self, zp):
        """Images in chunks whose largest activation stays within 2^30 elements (the kernels' per-operand 32-bit
        element offsets).  Up block j of the decoder ends in an upsampler whose output keeps its rev[j] channels at
        4^(j+1) times the latent pixels (rev = block_out_channels reversed); the largest of those, and of the mid
        block's [h, w, rev[0]], bounds every activation of an image: SDXL [n, 8h, 8w, 256] -> 4 images per chunk at
        1024^2."""
        B, h, w, _ = zp.shape
        rev = list(reversed(self.cfg.block_out_channels))
        per_img = max([h * w * rev[0]] + [4 ** (j + 1) * h * w * rev[j] for j in range(len(rev) - 1)])
        per = max(1, (1 << 30) // per_img)
        if B <= per:
            return self._decode_chunk(zp)
        out = torch.empty((B, 8 * h, 8 * w, self.cfg.out_channels), device=zp.device, dtype=BF16)
        for i in range(0, B, per):  # conv_out writes each chunk's rows of the batch output in place
            self._decode_chunk(zp[i:i + per], out=out[i:i + per])
        return out

    def _decode_chunk(self, zp, out=None):
        d = self.decoder
        B, h, w, _ = zp.shape
        C = self.cfg.latent_channels
        pq = K.gemm(zp.view(-1, self._lc_pad), self._pq_w, bias=self.post_quant_conv.bias).view(B, h, w, C)
        cols = K.im2col3(pq, d.conv_in.kp)
        x = K.gemm(cols, d.conv_in.w_col, bias=d.conv_in.bias).view(B, h, w, -1)
        rt = SimpleNamespace(save=False)
        x = d.mid_block.resnets[0].fwd(x, rt, None)
        x = d.mid_block.attentions[0].fwd(x)
        x = d.mid_block.resnets[1].fwd(x, rt, None)
        for blk in d.up_blocks:
            for res in blk.resnets:
                x = res.fwd(x, rt, None)
            if hasattr(blk, "upsamplers"):
                x = blk.upsamplers[0].fwd(x, rt)
        hn, _ = K.group_norm_fwd(x, d.conv_norm_out.weight, d.conv_norm_out.bias, self.cfg.norm_num_groups, 1e-6,
                                 True)
        return K.conv2d(hn, d.conv_out.w_nhwc, bias=d.conv_out.bias, out=out)

    @torch.no_grad()
    def decode_latents_nhwc(self, x, scale=None):
        """Trainer-side decode of the sampler's final latents, kept NHWC: x [B, h, w, C] fp32 (the trajectory buffer
        layout) -> image NHWC bf16 [B, 8h, 8w, 3].  `vae.decode(latents / scaling_factor)` of
        DP/sdxl_turbo_with_logprob.py:154-155 (scale defaults to 1 / scaling_factor)."""
        B, h, w, C = x.shape
        s = 1.0 / self.cfg.scaling_factor if scale is None else scale
        # NHWC rows are NCHW images of 1 x 1 pixels: the same pad / scale / cast kernel the NCHW path uses
        z = x.reshape(B * h * w, C, 1, 1)
        if not self._prepared:
            self.prepare()
        zp = K.nchw_to_nhwc(z, pad_to=self._lc_pad, scale=s).view(B, h, w, self._lc_pad)
        return self._decode_padded(zp)

    @torch.no_grad()
    def encode_nhwc(self, x):
        """x NCHW image in [-1, 1] (fp32 / bf16) -> moments NHWC fp32 [B, H/8, W/8, 2*latent] (mean | logvar)."""
        if not self._prepared:
            self.prepare()
        e = self.encoder
        B, _, H, W = x.shape
        xh = K.nchw_to_nhwc(x)                                                    # [B,H,W,3] bf16
        cols = K.im2col3(xh, e.conv_in.kp)
        h = K.gemm(cols, e.conv_in.w_col, bias=e.conv_in.bias).view(B, H, W, -1)
        rt = SimpleNamespace(save=False)
        for blk in e.down_blocks:
            for res in blk.resnets:
                h = res.fwd(h, rt, None)
            if hasattr(blk, "downsamplers"):
                h = blk.downsamplers[0].fwd(h)
        h = e.mid_block.resnets[0].fwd(h, rt, None)
        h = e.mid_block.attentions[0].fwd(h)
        h = e.mid_block.resnets[1].fwd(h, rt, None)
        hn, _ = K.group_norm_fwd(h, e.conv_norm_out.weight, e.conv_norm_out.bias, self.cfg.norm_num_groups, 1e-6,
                                 True)
        mo = K.conv2d(hn, e.conv_out.w_nhwc, bias=e.conv_out.bias)              # [B,h,w,2L] bf16
        _, h8, w8, L2 = mo.shape
        return K.gemm(mo.view(-1, L2), self._qc_w, bias=self.quant_conv.bias,
                      out_dtype=torch.float32).view(B, h8, w8, L2)

    def encode(self, x, return_dict=True):
        """diffusers `vae.encode(x).latent_dist` (DB:1750): NCHW fp32 moments in a DiagonalGaussianDistribution."""
        mo = self.encode_nhwc(x)
        L = self.cfg.latent_channels
        mom = mo.permute(0, 3, 1, 2)
        dist = DiagonalGaussianDistribution(mom[:, :L].contiguous(), mom[:, L:].contiguous())
        return SimpleNamespace(latent_dist=dist) if return_dict else (dist,)

    def decode(self, z, return_dict=True):
        img = K.nhwc_to_nchw(self.decode_nhwc(z), torch.float32)
        return SimpleNamespace(sample=img) if return_dict else (img,)
