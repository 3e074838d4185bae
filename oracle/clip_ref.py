"""ORACLE (test infrastructure only) -- the third-party arithmetic at the CLIP boundary of SURVEY §8f #2-#3, run as
the library itself where it is installed in this image, restated where it is not.

Only tests/ may import this module; it is the checker, never the product.

* CLIP towers: `transformers` CLIPTextModel / CLIPTextModelWithProjection / CLIPModel (the classes the reference
  instantiates: T:252-266 `text_encoder_cls.from_pretrained`, pso_pytorch/pickscore_utils.py:20-23
  `AutoModel.from_pretrained`), built from our config dataclasses and loaded with the SAME state dict, run in fp32.
  The reference pins transformers==4.38.1 (environment.yml:17); this image has 5.15 -- the CLIP forward arithmetic
  is unchanged between them (pre-LN layers, q * head_dim^-0.5, causal mask, argmax-eos pooling for eos_token_id 2).
* Image preprocessing: transformers 4.38 CLIPImageProcessor.preprocess restated on PIL + numpy exactly as that
  version executes it (resize the shortest edge with PIL BICUBIC on the uint8 image, centre crop, `image * (1/255)`
  in float64 -> float32, `(image - mean) / std` in float32), because 5.x may route through another backend.  The
  uint8 images come from the trainer's own line ((img + 1) * 127.5).clamp(0, 255).to(torch.uint8) (T:632-633),
  executed verbatim in torch on the image dtype.
"""
import numpy as np
import torch


def _text_cfg(cfg):
    from transformers import CLIPTextConfig as HFText
    return HFText(vocab_size=cfg.vocab_size, hidden_size=cfg.hidden_size, intermediate_size=cfg.intermediate_size,
                  num_hidden_layers=cfg.num_hidden_layers, num_attention_heads=cfg.num_attention_heads,
                  max_position_embeddings=cfg.max_position_embeddings, hidden_act=cfg.hidden_act,
                  layer_norm_eps=cfg.layer_norm_eps, projection_dim=cfg.projection_dim, eos_token_id=cfg.eos_token_id,
                  attn_implementation="eager")


def _vision_cfg(cfg):
    from transformers import CLIPVisionConfig as HFVision
    return HFVision(hidden_size=cfg.hidden_size, intermediate_size=cfg.intermediate_size,
                    num_hidden_layers=cfg.num_hidden_layers, num_attention_heads=cfg.num_attention_heads,
                    image_size=cfg.image_size, patch_size=cfg.patch_size, num_channels=cfg.num_channels,
                    hidden_act=cfg.hidden_act, layer_norm_eps=cfg.layer_norm_eps, projection_dim=cfg.projection_dim,
                    attn_implementation="eager")


def _load(model, sd, device):
    sd = {k: v.detach().float().to("cpu") for k, v in sd.items()}
    if not any(k.startswith("text_model.") for k in model.state_dict()):  # transformers 5.x CLIPTextModel layout
        sd = {k[len("text_model."):] if k.startswith("text_model.") else k: v for k, v in sd.items()}
    missing, unexpected = model.load_state_dict(sd, strict=False)
    missing = [k for k in missing if not k.endswith("position_ids")]
    assert not missing and not unexpected, (missing, unexpected)
    return model.float().to(device).eval()


def hf_text_model(cfg, sd, device="cpu", projection=False):
    from transformers import CLIPTextModel, CLIPTextModelWithProjection
    cls = CLIPTextModelWithProjection if projection else CLIPTextModel
    return _load(cls(_text_cfg(cfg)), sd, device)


def hf_clip_model(text_cfg, vision_cfg, projection_dim, sd, device="cpu"):
    from transformers import CLIPConfig, CLIPModel
    c = CLIPConfig(text_config=_text_cfg(text_cfg).to_dict(), vision_config=_vision_cfg(vision_cfg).to_dict(),
                   projection_dim=projection_dim)
    return _load(CLIPModel(c), sd, device)


def trainer_uint8(img_nchw):
    """T:632-633 verbatim: ((images + 1.0) * 127.5).clamp(0, 255).to(torch.uint8).permute(0, 2, 3, 1) (CPU)."""
    return ((img_nchw + 1.0) * 127.5).clamp(0, 255).to(torch.uint8).permute(0, 2, 3, 1).cpu().numpy()


def clip_image_processor(images_u8, size=224, mean=(0.48145466, 0.4578275, 0.40821073),
                         std=(0.26862954, 0.26130258, 0.27577711)):
    """transformers 4.38 CLIPImageProcessor(do_resize shortest_edge=size BICUBIC, do_center_crop size, do_rescale
    1/255, do_normalize mean/std) on uint8 HWC images -> pixel_values float32 [B, 3, size, size]."""
    from PIL import Image
    out = []
    for a in images_u8:
        h, w = a.shape[:2]
        short, long = (h, w) if h <= w else (w, h)
        new_long = int(size * long / short)
        nh, nw = (size, new_long) if h <= w else (new_long, size)
        r = np.asarray(Image.fromarray(a).resize((nw, nh), resample=Image.BICUBIC))
        top, left = (nh - size) // 2, (nw - size) // 2
        r = r[top:top + size, left:left + size]
        x = (r * (1 / 255)).astype(np.float32)
        x = (x - np.array(mean, dtype=np.float32)) / np.array(std, dtype=np.float32)
        out.append(x.transpose(2, 0, 1))
    return np.stack(out).astype(np.float32)
