"""Prompt conditioning of the online PSO trainers: tokenizers, `tokenize_captions` (T:81-94) and
`encode_prompt` (T:96-118) over the HIP CLIP text towers (clip.py).

Tokenizers are the transformers CLIPTokenizer the reference loads with `AutoTokenizer.from_pretrained(path,
subfolder="tokenizer[_2]")` (T:242-251): host-side BPE over the checkpoint's vocab.json / merges.txt, read from a
local directory.  The ids go to the GPU once; everything after that (embedding lookup, 12 + 32 encoder layers, final
norm, projection) runs on the HIP kernels."""
import torch

from .clip import CLIPTextModel, CLIPTextModelWithProjection, CLIPTextConfig


def load_tokenizer(path, subfolder=None):
    import os
    from transformers import CLIPTokenizer
    d = os.path.join(path, subfolder) if subfolder else path
    if not os.path.isdir(d):
        raise OSError(f"{d} is not a local tokenizer directory (hub ids cannot be fetched: no network)")
    return CLIPTokenizer.from_pretrained(d)


def tokenize_captions(tokenizers, examples):
    """T:81-94: both tokenizers, padding="max_length", truncation, max_length = model_max_length."""
    captions = list(examples["caption"])
    ids = [t(captions, truncation=True, padding="max_length", max_length=t.model_max_length,
             return_tensors="pt").input_ids for t in tokenizers]
    return ids[0], ids[1]


@torch.no_grad()
def encode_prompt(text_encoders, text_input_ids_list):
    """T:96-118: prompt_embeds = concat over encoders of hidden_states[-2] ([B, 77, 768 + 1280] for SDXL);
    pooled = output[0] of the LAST encoder (CLIPTextModelWithProjection.text_embeds, [B, 1280])."""
    embeds = []
    pooled = None
    for enc, ids in zip(text_encoders, text_input_ids_list):
        out = enc(ids.to(enc.device), output_hidden_states=True)
        pooled = out[0]
        h = out.hidden_states[-2]
        embeds.append(h.reshape(h.shape[0], h.shape[1], -1))
    from . import kernels as K
    B = embeds[0].shape[0]
    cat = embeds[0]
    for e in embeds[1:]:  # channel concat (one copy kernel per extra encoder)
        cat = K.concat_channels(cat, e)
    return cat, pooled.reshape(B, -1)


def sdxl_text_encoders(device, seed=0, configs=(None, None)):
    """Random-init SDXL text encoders (CLIP ViT-L/14 text + OpenCLIP bigG/14 text with projection), synthetic
    weights in the transformers layout (no checkpoints on this build)."""
    c1 = configs[0] or CLIPTextConfig.sdxl_l()
    c2 = configs[1] or CLIPTextConfig.sdxl_bigg()
    with torch.device(device):
        e1, e2 = CLIPTextModel(c1), CLIPTextModelWithProjection(c2)
    return e1.init_weights(seed), e2.init_weights(seed + 1)
