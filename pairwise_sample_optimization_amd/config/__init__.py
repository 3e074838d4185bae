"""Run configs of the two online-PSO trainers (reference `config/config_sdxl_{turbo,dmd}_dpo.py`), exposed as a
minimal attribute dict so code written against `ml_collections.ConfigDict` (absent here) reads them unchanged."""


class ConfigDict(dict):
    """`cfg.a.b` attribute access over nested dicts; unknown attributes raise AttributeError like ml_collections."""

    def __init__(self, d=None, **kw):
        super().__init__()
        for k, v in dict(d or {}, **kw).items():
            self[k] = v

    def __setitem__(self, k, v):
        super().__setitem__(k, ConfigDict(v) if isinstance(v, dict) and not isinstance(v, ConfigDict) else v)

    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError:
            raise AttributeError(k) from None

    def __setattr__(self, k, v):
        self[k] = v

    def to_dict(self):
        return {k: v.to_dict() if isinstance(v, ConfigDict) else v for k, v in self.items()}


def _common():
    return {
        "run_name": "", "seed": 0, "logdir": "logging", "output_dir": "output", "cache_dir": None,
        "general_cache_dir": None, "checkpointing_steps": 100, "num_checkpoint_limit": 10,
        "mixed_precision": "fp16", "allow_tf32": True, "resume_from": "", "use_lora": True, "use_xformers": False,
        "val_dataset": "yuvalkirstain/pickapic_v1_no_images", "val_split_name": "test_unique",
        "pretrained": {"pretrained_model_name_or_path": "", "revision": "main",
                       "pretrained_vae_model_name_or_path": "madebyollin/sdxl-vae-fp16-fix"},
        "sample": {"num_steps": 4, "eta": 1.0, "guidance_scale": 0.0, "batch_size": 4, "num_batches_per_epoch": 4,
                   "save_interval": 100, "eval_batch_size": 10, "eval_epoch": 10},
        "train": {"lora_rank": 32, "distilled_train_steps": 3, "batch_size": 4, "use_8bit_adam": True,
                  "learning_rate": 1e-5, "adam_beta1": 0.9, "adam_beta2": 0.999, "adam_weight_decay": 1e-6,
                  "adam_epsilon": 1e-8, "gradient_accumulation_steps": 2, "max_grad_norm": 1.0,
                  "num_inner_epochs": 1, "activation_checkpoint": True, "cfg": True, "adv_clip_max": 5,
                  "timestep_fraction": 1.0, "beta": 50, "eps": 0.1, "save_interval": 100, "sample_path": "",
                  "json_path": "", "clip_range": 1e-4},
        "per_prompt_stat_tracking": {"buffer_size": 16, "min_count": 16},
        "kl_ratio": 0.01, "prompt_fn": "simple_animals", "prompt_fn_kwargs": {},
    }


def load_config_file(path):
    """Execute a run config in the reference's own format -- e.g. the reference's
    `human_preference_tuning/config/config_sdxl_turbo_dpo.py` unchanged (`import ml_collections`,
    `config = ml_collections.ConfigDict()`, nested `config.sample = ml_collections.ConfigDict()`, `get_config()`) --
    with this module's ConfigDict standing in for the absent ml_collections package (T:55-56 loads it through absl's
    config_flags.DEFINE_config_file).  Returns the ConfigDict."""
    import importlib.util
    import sys
    import types
    stub = types.ModuleType("ml_collections")
    stub.ConfigDict = ConfigDict
    saved = sys.modules.get("ml_collections")
    sys.modules["ml_collections"] = stub
    try:
        spec = importlib.util.spec_from_file_location("_pso_run_config", path)
        mod = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(mod)
        return mod.get_config()
    finally:
        if saved is None:
            del sys.modules["ml_collections"]
        else:
            sys.modules["ml_collections"] = saved


def apply_overrides(cfg, overrides):
    """absl config_flags overrides as the launch scripts pass them (`--config.train.beta=50`,
    online_pso_sdxl_turbo.sh:4-15): each item "a.b.c=value" (a leading "--config." is stripped); values are Python
    literals where they parse as one, else strings."""
    import ast
    for item in overrides:
        key, _, val = item.partition("=")
        key = key[len("--config."):] if key.startswith("--config.") else key
        try:
            v = ast.literal_eval(val)
        except (ValueError, SyntaxError):
            v = val
        node = cfg
        parts = key.split(".")
        for p in parts[:-1]:
            node = getattr(node, p)
        if parts[-1] not in node:
            raise KeyError(f"config has no field {key!r}")
        node[parts[-1]] = v
    return cfg
