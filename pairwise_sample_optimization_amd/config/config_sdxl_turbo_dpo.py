"""`config/config_sdxl_turbo_dpo.py` values (SDXL-Turbo, 512^2, 4 steps, LoRA r=32, PickScore)."""
from . import ConfigDict, _common


def get_config():
    c = ConfigDict(_common())
    c.num_epochs = 10000
    c.cache_dir_val = None
    c.pretrained.pretrained_model_name_or_path = "stabilityai/sdxl-turbo"
    c.reward_fn = "pick_score"
    return c
