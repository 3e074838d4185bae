"""transformers checkpoint boundary of the CLIP towers: `<path>/<subfolder>/config.json` + `model.safetensors`
(or `pytorch_model.bin` through `torch.load(weights_only=True)`), the layout `CLIPTextModel.from_pretrained(path,
subfolder="text_encoder")` (T:252-266) and `AutoModel.from_pretrained("yuvalkirstain/PickScore_v1")`
(pso_pytorch/pickscore_utils.py:20-23) read.  Local directories only (no network on this build)."""
import json
import os

import torch

from .diffusers_io import _resolve

WEIGHTS = ("model.safetensors", "pytorch_model.bin")


def load_config(path, subfolder=None):
    with open(os.path.join(_resolve(path, subfolder), "config.json")) as f:
        return json.load(f)


def load_weights(path, subfolder=None, variant=None):
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
