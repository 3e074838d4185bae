"""CLIP text / vision towers on the libpso_amd HIP kernels: the SDXL prompt encoders and the
PickScore reward model, in the HuggingFace `transformers` CLIP key layout so their checkpoints load unchanged.

Reference call sites:
  * `encode_prompt(text_encoders, text_input_ids_list)` T:96-118 (D: same) -- CLIPTextModel (OpenAI ViT-L/14 text,
    quick-GELU) + CLIPTextModelWithProjection (OpenCLIP ViT-bigG/14 text, GELU), loaded by
    `text_encoder_cls.from_pretrained(path, subfolder="text_encoder[_2]")` (T:252-266).  prompt_embeds =
    concat(hidden_states[-2] of both) [B, 77, 768 + 1280]; pooled = text_embeds of the second.
  * PickScore `Selector.score` pso_pytorch/pickscore_utils.py:28-62 -- CLIPModel (ViT-H/14: vision 32 x 1280, patch
    14 @ 224^2, text 24 x 1024, projection 1024): `get_image_features`, `get_text_features`, cosine of matched rows.

Architecture restated from transformers (4.38.1 pinned by the reference, environment.yml:17) `modeling_clip.py`:
pre-LN encoder layers (layer_norm1 -> self_attn (q/k/v/out_proj with bias, q scaled by head_dim^-0.5) -> residual ->
layer_norm2 -> mlp.fc1 -> act -> mlp.fc2 -> residual); text: token + position embeddings, causal mask, final_layer_norm,
pooled row = argmax(input_ids) (eos_token_id == 2, the legacy configs) or the first eos_token_id; vision:
conv patch embedding (no bias) + class token + position embeddings, pre_layrnorm, post_layernorm on the class row,
visual_projection (no bias).

Layout: token rows [B * S][C] bf16; q/k/v fused into one GEMM per layer; attention by `pso_attention_small`
(short sequences, head dim 64 / 80); LayerNorm by `pso_layer_norm_fwd`; activations in place.  Forward only (frozen
towers: the reference runs them under torch.no_grad()).
"""
import math
from dataclasses import dataclass, fields
from types import SimpleNamespace

import torch
import torch.nn as nn

from . import kernels as K
from .unet import Linear, Norm, _param

BF16 = torch.bfloat16


@dataclass
class CLIPTextConfig:
    vocab_size: int = 49408
    hidden_size: int = 768
    intermediate_size: int = 3072
    num_hidden_layers: int = 12
    num_attention_heads: int = 12
    max_position_embeddings: int = 77
    hidden_act: str = "quick_gelu"
    layer_norm_eps: float = 1e-5
    projection_dim: int = 768
    eos_token_id: int = 2

    @staticmethod
    def sdxl_l():
        """SDXL text_encoder: OpenAI CLIP ViT-L/14 text tower."""
        return CLIPTextConfig()

    @staticmethod
    def sdxl_bigg():
        """SDXL text_encoder_2: OpenCLIP ViT-bigG/14 text tower (CLIPTextModelWithProjection)."""
        return CLIPTextConfig(hidden_size=1280, intermediate_size=5120, num_hidden_layers=32, num_attention_heads=20,
                              hidden_act="gelu", projection_dim=1280)

    @staticmethod
    def pickscore_h():
        """PickScore_v1 / CLIP ViT-H/14 text tower."""
        return CLIPTextConfig(hidden_size=1024, intermediate_size=4096, num_hidden_layers=24, num_attention_heads=16,
                              hidden_act="gelu", projection_dim=1024)


@dataclass
class CLIPVisionConfig:
    hidden_size: int = 1280
    intermediate_size: int = 5120
    num_hidden_layers: int = 32
    num_attention_heads: int = 16
    image_size: int = 224
    patch_size: int = 14
    num_channels: int = 3
    hidden_act: str = "gelu"
    layer_norm_eps: float = 1e-5
    projection_dim: int = 1024


def _from_dict(cls, d):
    names = {f.name for f in fields(cls)}
    return cls(**{k: v for k, v in d.items() if k in names})


_ACTS = {"gelu": K.ACT_GELU, "quick_gelu": K.ACT_QUICK_GELU}


def _act_code(name):
    if name not in _ACTS:
        raise ValueError(f"hidden_act {name!r} is not supported by this build (supported: {sorted(_ACTS)})")
    return _ACTS[name]


class Embedding(nn.Module):
    def __init__(self, n, c):
        super().__init__()
        self.weight = _param(n, c)


class _SelfAttn(nn.Module):
    def __init__(self, c):
        super().__init__()
        self.q_proj, self.k_proj, self.v_proj, self.out_proj = Linear(c, c), Linear(c, c), Linear(c, c), Linear(c, c)


class _MLP(nn.Module):
    def __init__(self, c, f):
        super().__init__()
        self.fc1, self.fc2 = Linear(c, f), Linear(f, c)


class CLIPEncoderLayer(nn.Module):
    def __init__(self, c, f, heads):
        super().__init__()
        self.heads = heads
        self.self_attn = _SelfAttn(c)
        self.layer_norm1 = Norm(c)
        self.mlp = _MLP(c, f)
        self.layer_norm2 = Norm(c)

    def prepare(self):
        a = self.self_attn
        self.w_qkv = torch.cat([a.q_proj.weight.data, a.k_proj.weight.data, a.v_proj.weight.data], 0).contiguous()
        self.b_qkv = torch.cat([a.q_proj.bias.data, a.k_proj.bias.data, a.v_proj.bias.data], 0).contiguous()

    def fwd(self, x, B, S, causal, act, eps):
        """x [B*S, C] bf16 -> [B*S, C] (pre-LN attention block + pre-LN MLP block, residuals fused into the GEMMs)."""
        C = x.shape[1]
        H = self.heads
        D = C // H
        hn, _ = K.layer_norm_fwd(x, self.layer_norm1.weight, self.layer_norm1.bias, eps)
        qkv = K.gemm(hn, self.w_qkv, bias=self.b_qkv)                               # [B*S, 3C]
        att = K.attention_small(qkv[:, :C], qkv[:, C:2 * C], qkv[:, 2 * C:], B, S, H, causal, D ** -0.5)
        o = self.self_attn.out_proj
        x = K.gemm(att, o.weight, bias=o.bias, resid=x)
        hn, _ = K.layer_norm_fwd(x, self.layer_norm2.weight, self.layer_norm2.bias, eps)
        f = K.gemm(hn, self.mlp.fc1.weight, bias=self.mlp.fc1.bias)
        K.activation_(f, act)
        return K.gemm(f, self.mlp.fc2.weight, bias=self.mlp.fc2.bias, resid=x)


class CLIPEncoder(nn.Module):
    def __init__(self, c, f, heads, n):
        super().__init__()
        self.layers = nn.ModuleList([CLIPEncoderLayer(c, f, heads) for _ in range(n)])


def _init_linear(lin, std, g):
    with torch.no_grad():
        lin.weight.copy_(torch.randn(lin.weight.shape, generator=g, device=lin.weight.device) * std)
        if lin.bias is not None:
            lin.bias.zero_()


def _init_encoder(enc, c, n, g):
    """transformers CLIPPreTrainedModel._init_weights (factor 1): q/k/v/out N(0, c^-0.5 (2n)^-0.5),
    fc1 N(0, (2c)^-0.5), fc2 N(0, c^-0.5 (2n)^-0.5), LayerNorm (1, 0)."""
    in_std = c ** -0.5 * (2 * n) ** -0.5
    for l in enc.layers:
        a = l.self_attn
        for lin in (a.q_proj, a.k_proj, a.v_proj):
            _init_linear(lin, in_std, g)
        _init_linear(a.out_proj, c ** -0.5, g)
        _init_linear(l.mlp.fc1, (2 * c) ** -0.5, g)
        _init_linear(l.mlp.fc2, in_std, g)
        for nm in (l.layer_norm1, l.layer_norm2):
            nm.reset(g)


class _TextEmbeddings(nn.Module):
    def __init__(self, cfg):
        super().__init__()
        self.token_embedding = Embedding(cfg.vocab_size, cfg.hidden_size)
        self.position_embedding = Embedding(cfg.max_position_embeddings, cfg.hidden_size)


class CLIPTextTransformer(nn.Module):
    def __init__(self, cfg: CLIPTextConfig):
        super().__init__()
        self.cfg = cfg
        self.embeddings = _TextEmbeddings(cfg)
        self.encoder = CLIPEncoder(cfg.hidden_size, cfg.intermediate_size, cfg.num_attention_heads,
                                   cfg.num_hidden_layers)
        self.final_layer_norm = Norm(cfg.hidden_size)
        self._act = _act_code(cfg.hidden_act)

    def init_weights(self, g):
        with torch.no_grad():
            e = self.embeddings
            e.token_embedding.weight.copy_(torch.randn(e.token_embedding.weight.shape, generator=g,
                                                       device=e.token_embedding.weight.device) * 0.02)
            e.position_embedding.weight.copy_(torch.randn(e.position_embedding.weight.shape, generator=g,
                                                          device=e.position_embedding.weight.device) * 0.02)
        _init_encoder(self.encoder, self.cfg.hidden_size, self.cfg.num_hidden_layers, g)
        self.final_layer_norm.reset(g)

    def prepare(self):
        for l in self.encoder.layers:
            l.prepare()

    def pooled_index(self, ids):
        """Row of the pooled token per sequence: argmax(ids) for eos_token_id == 2 (legacy CLIP configs), else the
        first occurrence of eos_token_id (transformers CLIPTextTransformer.forward)."""
        if self.cfg.eos_token_id == 2:
            return ids.to(torch.int32).argmax(dim=-1)
        return (ids == self.cfg.eos_token_id).int().argmax(dim=-1)

    def fwd(self, ids, hidden_layer=None):
        """ids [B, S] int64 -> (last_hidden_state after final LN [B*S, C], pooled [B, C], hidden [B*S, C] | None):
        hidden = output of encoder layer `hidden_layer` (1-based; hidden_states[hidden_layer] in transformers)."""
        c = self.cfg
        B, S = ids.shape
        dev = self.final_layer_norm.weight.device
        ids_d = ids.to(dev, torch.int64).contiguous()
        x = K.embed_tokens(ids_d, self.embeddings.token_embedding.weight, self.embeddings.position_embedding.weight)
        hid = x if hidden_layer == 0 else None
        for i, l in enumerate(self.encoder.layers):
            x = l.fwd(x, B, S, True, self._act, c.layer_norm_eps)
            if hidden_layer == i + 1:
                hid = x
        last, _ = K.layer_norm_fwd(x, self.final_layer_norm.weight, self.final_layer_norm.bias, c.layer_norm_eps)
        rows = torch.arange(B, device=dev) * S + self.pooled_index(ids_d)
        pooled = K.gather_rows(last, rows)
        return last, pooled, hid


class _TextModelBase(nn.Module):
    config_class = CLIPTextConfig

    @classmethod
    def from_config(cls, config=None, **kw):
        if isinstance(config, dict):
            config = _from_dict(CLIPTextConfig, dict(config, **kw))
        return cls(config or CLIPTextConfig())

    @classmethod
    def from_pretrained(cls, path, subfolder=None, torch_dtype=None, variant=None, revision=None, **kw):
        """`CLIPTextModel[WithProjection].from_pretrained(path, subfolder="text_encoder[_2]")` (T:252-266) from a
        local transformers directory (config.json + model.safetensors / pytorch_model.bin)."""
        from . import hf_io
        m = cls.from_config(hf_io.load_config(path, subfolder))
        m.load_state_dict(hf_io.load_weights(path, subfolder, variant))
        return m

    def load_state_dict(self, sd, strict=True):
        sd = {k: v.to(BF16) for k, v in sd.items() if not k.endswith("position_ids")}
        res = super().load_state_dict(sd, strict=strict)
        self._prepared = False
        return res

    def _ensure(self):
        if not getattr(self, "_prepared", False):
            self.text_model.prepare()
            self._prepared = True

    @property
    def device(self):
        return self.text_model.final_layer_norm.weight.device


class CLIPTextModel(_TextModelBase):
    """transformers CLIPTextModel (keys `text_model.*`).  Call: `enc(ids, output_hidden_states=True)` -> object with
    [0] / .last_hidden_state, [1] / .pooler_output and .hidden_states (a lazy list: only [-2] and [-1] are formed)."""

    def __init__(self, config: CLIPTextConfig = None):
        super().__init__()
        self.config = config or CLIPTextConfig()
        self.text_model = CLIPTextTransformer(self.config)
        self._prepared = False

    def init_weights(self, seed=0):
        g = torch.Generator(device=self.device).manual_seed(seed)
        self.text_model.init_weights(g)
        self._prepared = False
        return self

    @torch.no_grad()
    def forward(self, input_ids, output_hidden_states=False, attention_mask=None, return_dict=True):
        self._ensure()
        B, S = input_ids.shape
        C = self.config.hidden_size
        L = self.config.num_hidden_layers
        last, pooled, hid = self.text_model.fwd(input_ids, hidden_layer=L - 1 if output_hidden_states else None)
        last = last.view(B, S, C)
        out = _TextOutput(last, pooled)
        if output_hidden_states:
            out.hidden_states = _Hidden(L + 1, {L - 1: hid.view(B, S, C)})
        return out


class CLIPTextModelWithProjection(_TextModelBase):
    """transformers CLIPTextModelWithProjection (keys `text_model.*`, `text_projection.weight`): output [0] /
    .text_embeds = text_projection(pooled), .last_hidden_state, .hidden_states (lazy: [-2] formed)."""

    def __init__(self, config: CLIPTextConfig = None):
        super().__init__()
        self.config = config or CLIPTextConfig.sdxl_bigg()
        self.text_model = CLIPTextTransformer(self.config)
        self.text_projection = Linear(self.config.hidden_size, self.config.projection_dim, bias=False)
        self._prepared = False

    def init_weights(self, seed=0):
        g = torch.Generator(device=self.device).manual_seed(seed)
        self.text_model.init_weights(g)
        _init_linear(self.text_projection, self.config.hidden_size ** -0.5, g)
        self._prepared = False
        return self

    @torch.no_grad()
    def forward(self, input_ids, output_hidden_states=False, attention_mask=None, return_dict=True):
        self._ensure()
        B, S = input_ids.shape
        C = self.config.hidden_size
        L = self.config.num_hidden_layers
        last, pooled, hid = self.text_model.fwd(input_ids, hidden_layer=L - 1 if output_hidden_states else None)
        emb = K.gemm(pooled, self.text_projection.weight)
        out = _TextOutput(emb, last.view(B, S, C))
        out.text_embeds, out.last_hidden_state = emb, last.view(B, S, C)
        if output_hidden_states:
            out.hidden_states = _Hidden(L + 1, {L - 1: hid.view(B, S, C)})
        return out


class _TextOutput(tuple):
    def __new__(cls, a, b):
        o = super().__new__(cls, (a, b))
        o.last_hidden_state, o.pooler_output = a, b
        return o


class _Hidden:
    """transformers' hidden_states tuple, materialised only where the caller reads it (encode_prompt reads [-2])."""

    def __init__(self, n, have):
        self.n, self.have = n, have

    def __len__(self):
        return self.n

    def __getitem__(self, i):
        j = i % self.n
        if j not in self.have:
            raise IndexError(f"hidden_states[{i}] is not retained by this build (available: "
                             f"{sorted(k - self.n for k in self.have)})")
        return self.have[j]


# ---------------------------------------------------------------------------------------------------------------------
# vision tower + CLIPModel (PickScore)
# ---------------------------------------------------------------------------------------------------------------------
class _VisionEmbeddings(nn.Module):
    def __init__(self, cfg):
        super().__init__()
        self.class_embedding = _param(cfg.hidden_size)
        self.patch_embedding = _ConvNoBias(cfg.num_channels, cfg.hidden_size, cfg.patch_size)
        n = (cfg.image_size // cfg.patch_size) ** 2 + 1
        self.position_embedding = Embedding(n, cfg.hidden_size)


class _ConvNoBias(nn.Module):
    def __init__(self, cin, cout, k):
        super().__init__()
        self.weight = _param(cout, cin, k, k)


class CLIPVisionTransformer(nn.Module):
    def __init__(self, cfg: CLIPVisionConfig):
        super().__init__()
        self.cfg = cfg
        self.embeddings = _VisionEmbeddings(cfg)
        self.pre_layrnorm = Norm(cfg.hidden_size)
        self.encoder = CLIPEncoder(cfg.hidden_size, cfg.intermediate_size, cfg.num_attention_heads,
                                   cfg.num_hidden_layers)
        self.post_layernorm = Norm(cfg.hidden_size)
        self._act = _act_code(cfg.hidden_act)
        self.kpad = 8 * ((cfg.num_channels * cfg.patch_size ** 2 + 7) // 8)

    def init_weights(self, g):
        c = self.cfg
        e = self.embeddings
        with torch.no_grad():
            dev = e.class_embedding.device
            e.class_embedding.copy_(torch.randn(c.hidden_size, generator=g, device=dev) * c.hidden_size ** -0.5)
            e.patch_embedding.weight.copy_(torch.randn(e.patch_embedding.weight.shape, generator=g, device=dev) * 0.02)
            e.position_embedding.weight.copy_(torch.randn(e.position_embedding.weight.shape, generator=g,
                                                          device=dev) * 0.02)
        _init_encoder(self.encoder, c.hidden_size, c.num_hidden_layers, g)
        self.pre_layrnorm.reset(g)
        self.post_layernorm.reset(g)

    def prepare(self):
        c = self.cfg
        w = self.embeddings.patch_embedding.weight.data.reshape(c.hidden_size, -1)  # (channel, ky, kx) order
        self.w_patch = torch.zeros(c.hidden_size, self.kpad, device=w.device, dtype=BF16)
        self.w_patch[:, :w.shape[1]] = w
        for l in self.encoder.layers:
            l.prepare()

    def fwd_patches(self, patches, B):
        """patches [B * P, kpad] bf16 (pso_clip_preprocess) -> pooled (post_layernorm of the class row) [B, C]."""
        c = self.cfg
        P = (c.image_size // c.patch_size) ** 2
        S = P + 1
        pe = K.gemm(patches, self.w_patch)                                         # [B*P, C]
        x = K.embed_vision(pe, self.embeddings.class_embedding, self.embeddings.position_embedding.weight, B, P)
        x, _ = K.layer_norm_fwd(x, self.pre_layrnorm.weight, self.pre_layrnorm.bias, c.layer_norm_eps)
        for l in self.encoder.layers:
            x = l.fwd(x, B, S, False, self._act, c.layer_norm_eps)
        cls_rows = K.gather_rows(x, torch.arange(B, device=x.device) * S)
        pooled, _ = K.layer_norm_fwd(cls_rows, self.post_layernorm.weight, self.post_layernorm.bias, c.layer_norm_eps)
        return pooled


# CLIPImageProcessor defaults of the OpenAI / LAION CLIP checkpoints (processor of laion/CLIP-ViT-H-14-laion2B-s32B-b79K)
CLIP_MEAN = (0.48145466, 0.4578275, 0.40821073)
CLIP_STD = (0.26862954, 0.26130258, 0.27577711)


class CLIPModel(nn.Module):
    """transformers CLIPModel (keys `text_model.*`, `vision_model.*`, `visual_projection.weight`,
    `text_projection.weight`, `logit_scale`) with get_image_features / get_text_features, plus the GPU-resident
    image path `image_features_from_images` (pso_clip_preprocess -> patch GEMM -> tower -> projection)."""

    def __init__(self, text_config: CLIPTextConfig = None, vision_config: CLIPVisionConfig = None,
                 projection_dim=None):
        super().__init__()
        self.text_config = text_config or CLIPTextConfig.pickscore_h()
        self.vision_config = vision_config or CLIPVisionConfig()
        pd = projection_dim or self.vision_config.projection_dim
        self.config = SimpleNamespace(text_config=self.text_config, vision_config=self.vision_config,
                                      projection_dim=pd)
        self.text_model = CLIPTextTransformer(self.text_config)
        self.vision_model = CLIPVisionTransformer(self.vision_config)
        self.visual_projection = Linear(self.vision_config.hidden_size, pd, bias=False)
        self.text_projection = Linear(self.text_config.hidden_size, pd, bias=False)
        self.logit_scale = nn.Parameter(torch.tensor(math.log(1 / 0.07)), requires_grad=False)
        self._prepared = False

    @classmethod
    def from_config(cls, config):
        if isinstance(config, dict):
            pd = config.get("projection_dim")
            tc = _from_dict(CLIPTextConfig, dict(config.get("text_config", {}), projection_dim=pd or 512))
            vc = _from_dict(CLIPVisionConfig, dict(config.get("vision_config", {}), projection_dim=pd or 512))
            return cls(tc, vc, pd)
        return cls()

    @classmethod
    def from_pretrained(cls, path, subfolder=None, **kw):
        """`AutoModel.from_pretrained("yuvalkirstain/PickScore_v1")` (pickscore_utils.py:20-23) from a local dir."""
        from . import hf_io
        m = cls.from_config(hf_io.load_config(path, subfolder))
        m.load_state_dict(hf_io.load_weights(path, subfolder, None))
        return m

    def load_state_dict(self, sd, strict=True):
        sd = {k: (v.float() if k == "logit_scale" else v.to(BF16)) for k, v in sd.items()
              if not k.endswith("position_ids")}
        res = super().load_state_dict(sd, strict=strict)
        self._prepared = False
        return res

    @property
    def device(self):
        return self.visual_projection.weight.device

    def init_weights(self, seed=0):
        g = torch.Generator(device=self.device).manual_seed(seed)
        self.text_model.init_weights(g)
        self.vision_model.init_weights(g)
        _init_linear(self.visual_projection, self.vision_config.hidden_size ** -0.5, g)
        _init_linear(self.text_projection, self.text_config.hidden_size ** -0.5, g)
        self._prepared = False
        return self

    def _ensure(self):
        if not self._prepared:
            self.text_model.prepare()
            self.vision_model.prepare()
            self._prepared = True

    @torch.no_grad()
    def get_text_features(self, input_ids, attention_mask=None, **kw):
        """[B, projection_dim] fp32 = text_projection(pooled) (the causal mask makes the padding mask irrelevant to
        the pooled eos row)."""
        self._ensure()
        _, pooled, _ = self.text_model.fwd(input_ids)
        return K.gemm(pooled, self.text_projection.weight, out_dtype=torch.float32)

    @torch.no_grad()
    def get_image_features(self, pixel_values=None, patches=None, **kw):
        """pixel_values NCHW float [B, 3, S, S] (already processed) or patches [B * P, kpad] bf16 -> [B, proj] fp32."""
        self._ensure()
        vc = self.vision_config
        if patches is None:
            patches = K.patchify(pixel_values, vc.patch_size, self.vision_model.kpad)
            B = pixel_values.shape[0]
        else:
            B = patches.shape[0] // (vc.image_size // vc.patch_size) ** 2
        pooled = self.vision_model.fwd_patches(patches, B)
        return K.gemm(pooled, self.visual_projection.weight, out_dtype=torch.float32)

    @torch.no_grad()
    def image_features_from_images(self, img_nhwc, mean=CLIP_MEAN, std=CLIP_STD):
        """Decoded images NHWC bf16 in [-1, 1] -> image features, the whole T:632-640 + processor path on the GPU."""
        vc = self.vision_config
        patches = K.clip_preprocess(img_nhwc, vc.image_size, vc.patch_size, self.vision_model.kpad, mean, std)
        return self.get_image_features(patches=patches)
