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
