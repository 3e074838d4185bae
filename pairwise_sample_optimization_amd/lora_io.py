"""LoRA checkpoint interchange in the diffusers format the reference writes and reads.

* `save_lora_weights(output_dir, unet_lora_layers)` -- `StableDiffusionXLLoraLoaderMixin.save_lora_weights`
  as used by the save hook `T:361-379`: `pytorch_lora_weights.safetensors`, keys `unet.<module>.lora.{down,up}.weight`
  (peft `lora_A/lora_B` renamed by `convert_state_dict_to_diffusers`).
* `lora_state_dict(input_dir)` / `load_lora_into_unet(sd, network_alphas, unet)` -- the load hook `T:381-395`
  (and the consumers `T:138`, `evaluate_sdxl_dmd2.py:194`); accepts diffusers (`lora.down/up`) or peft
  (`lora_A/lora_B`) naming, with or without the `unet.` prefix.
* `save_state(trainer, dir)` / `load_state(trainer, dir)` -- resume (`T:886-890`, `accelerator.save_state`): the
  LoRA file plus the AdamW moments and step count (`optimizer.safetensors`).  8-bit AdamW checkpoints carry the
  per-tensor block table (round 4 on); an older checkpoint without one (uniform 2048-element blocks over the flat
  buffer) is re-quantised into the per-tensor layout on load, with a warning.
"""
import json
import os
import warnings

import torch
from safetensors.torch import load_file, save_file

LORA_WEIGHT_NAME = "pytorch_lora_weights.safetensors"
OPT_NAME = "optimizer.safetensors"


def peft_to_diffusers(sd):
    """convert_state_dict_to_diffusers for a peft LoRA state dict: `.lora_A.` -> `.lora.down.`, `.lora_B.` -> `.lora.up.`"""
    out = {}
    for k, v in sd.items():
        out[k.replace(".lora_A.", ".lora.down.").replace(".lora_B.", ".lora.up.")] = v
    return out


def diffusers_to_peft(sd):
    out = {}
    for k, v in sd.items():
        if k.startswith("unet."):
            k = k[len("unet."):]
        out[k.replace(".lora.down.", ".lora_A.").replace(".lora.up.", ".lora_B.")] = v
    return out


def get_peft_model_state_dict(unet):
    return unet.lora.state_dict_peft()


def save_lora_weights(output_dir, unet_lora_layers, weight_name=LORA_WEIGHT_NAME):
    os.makedirs(output_dir, exist_ok=True)
    packed = {f"unet.{k}": v.detach().float().contiguous().cpu() for k, v in unet_lora_layers.items()}
    save_file(packed, os.path.join(output_dir, weight_name), metadata={"format": "pt"})


def lora_state_dict(input_dir, weight_name=LORA_WEIGHT_NAME):
    path = input_dir if input_dir.endswith(".safetensors") else os.path.join(input_dir, weight_name)
    return load_file(path), None


def load_lora_into_unet(state_dict, network_alphas, unet):
    """Copy a LoRA state dict into the unet's adapter (ranks must match; network_alphas other than None/rank are
    folded into B as alpha/r, like peft's scaling)."""
    sd = diffusers_to_peft(state_dict)
    st = unet.lora
    missing = [n for n in st.adapter_names() if f"{n}.lora_A.weight" not in sd or f"{n}.lora_B.weight" not in sd]
    if missing:
        raise KeyError(f"LoRA state dict lacks {len(missing)} adapters, e.g. {missing[0]}")
    dev = st.master.device
    st.load_peft({k: v.to(dev, torch.float32) for k, v in sd.items()})


def save_state(trainer, output_dir):
    unet = trainer.unet
    save_lora_weights(output_dir, peft_to_diffusers(get_peft_model_state_dict(unet)))
    a8 = getattr(trainer, "adam8", None)
    if a8 is not None:  # 8-bit AdamW state as it stands (codes + block absmax): a resume continues bit for bit
        opt = {k: v.cpu() for k, v in a8.tensors().items()}
    else:
        opt = {"exp_avg": trainer.exp_avg.cpu(), "exp_avg_sq": trainer.exp_avg_sq.cpu()}
    save_file(opt, os.path.join(output_dir, OPT_NAME),
              metadata={"step": str(trainer.opt_step), "n_micro": str(trainer.n_micro)})
    with open(os.path.join(output_dir, "pso_state.json"), "w") as f:
        json.dump({"opt_step": trainer.opt_step, "n_micro": trainer.n_micro, "rank": unet.lora.r}, f)


def load_state(trainer, input_dir):
    sd, alphas = lora_state_dict(input_dir)
    load_lora_into_unet(sd, alphas, trainer.unet)
    opt = load_file(os.path.join(input_dir, OPT_NAME))
    a8 = getattr(trainer, "adam8", None)
    if a8 is not None:
        if "exp_avg_q" not in opt:
            raise KeyError("checkpoint holds fp32 AdamW state; this trainer runs the 8-bit AdamW (use_8bit_adam)")
        mine = a8.tensors()
        if "block_table" in mine and "block_table" not in opt:
            # a checkpoint of rounds <= 3: uniform 2048-element blocks over the whole flat buffer.  Its moments are
            # dequantised in that layout and re-quantised into the per-tensor blocks (lossy only in the code
            # rounding of the new blocks)
            warnings.warn("8-bit AdamW checkpoint without a block table (uniform blocks, older format): its moments "
                          "are re-quantised into the per-tensor block layout")
            from . import kernels as K
            old = K.Adam8State(a8.n, a8.qm.device)
            for k, t in old.tensors().items():
                t.copy_(opt[k])
            a8.load_dense(*old.dequant())
        elif ("block_table" in mine) != ("block_table" in opt) or (
                "block_table" in opt and not torch.equal(opt["block_table"], mine["block_table"].cpu())):
            raise KeyError("checkpoint's 8-bit AdamW block layout differs from this trainer's parameter tensors")
        else:
            for k, t in mine.items():
                if k != "block_table":
                    t.copy_(opt[k])
    else:
        if "exp_avg" not in opt:
            raise KeyError("checkpoint holds 8-bit AdamW state; this trainer runs fp32 AdamW")
        trainer.exp_avg.copy_(opt["exp_avg"])
        trainer.exp_avg_sq.copy_(opt["exp_avg_sq"])
    with open(os.path.join(input_dir, "pso_state.json")) as f:
        meta = json.load(f)
    trainer.opt_step, trainer.n_micro = int(meta["opt_step"]), int(meta["n_micro"])
