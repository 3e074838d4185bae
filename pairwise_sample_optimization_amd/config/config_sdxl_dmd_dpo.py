"""`config/config_sdxl_dmd_dpo.py` values (DMD2 on SDXL-base, 1024^2, 4 steps, LoRA r=16, PickScore+ImageReward)."""
from . import ConfigDict, _common


def get_config():
    c = ConfigDict(_common())
    c.azure_run_id = ""
    c.num_epochs = 5000
    c.cache_val_dir = None
    c.pretrained.pretrained_model_name_or_path = "stabilityai/stable-diffusion-xl-base-1.0"
    c.sample.batch_size = 1
    c.sample.num_batches_per_epoch = 16
    c.train.lora_rank = 16
    c.train.batch_size = 1
    c.train.gradient_accumulation_steps = 4
    c.reward_fn = "pickscore+imagereward"
    return c
