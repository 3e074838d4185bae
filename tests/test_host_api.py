"""CPU checks of the host-side mirrors of the reference surface: run configs, LoRA key layout / checkpoint format,
trainer construction rules.  No GPU compute."""
from types import SimpleNamespace

import pytest
import torch


def test_configs_match_reference_values():
    from pairwise_sample_optimization_amd.config import config_sdxl_dmd_dpo, config_sdxl_turbo_dpo
    t = config_sdxl_turbo_dpo.get_config()
    d = config_sdxl_dmd_dpo.get_config()
    # config_sdxl_turbo_dpo.py:64-119 / config_sdxl_dmd_dpo.py
    assert (t.sample.num_steps, t.train.distilled_train_steps, t.train.beta, t.train.eps) == (4, 3, 50, 0.1)
    assert (t.train.lora_rank, t.train.batch_size, t.train.gradient_accumulation_steps) == (32, 4, 2)
    assert (d.train.lora_rank, d.train.batch_size, d.train.gradient_accumulation_steps) == (16, 1, 4)
    assert t.pretrained.pretrained_model_name_or_path == "stabilityai/sdxl-turbo"
    assert d.reward_fn == "pickscore+imagereward" and t.reward_fn == "pick_score"
    with pytest.raises(AttributeError):
        t.train.no_such_key
    t.train.learning_rate = 3e-5
    assert t.to_dict()["train"]["learning_rate"] == 3e-5


def test_trainer_from_config_enforces_T():
    from pairwise_sample_optimization_amd.config import config_sdxl_turbo_dpo
    from pairwise_sample_optimization_amd.trainer import PSOTrainer
    c = config_sdxl_turbo_dpo.get_config()
    c.train.distilled_train_steps = 2  # T:221 assert: must be num_steps - 1
    with pytest.raises(AssertionError):
        PSOTrainer.from_config(None, c)


def test_sdxl_lora_adapter_layout_and_diffusers_keys():
    from pairwise_sample_optimization_amd import lora_io
    from pairwise_sample_optimization_amd.unet import UNet2DConditionModel, UNetConfig
    with torch.device("meta"):
        u = UNet2DConditionModel(UNetConfig.sdxl())
    st = u.add_adapter(SimpleNamespace(r=32, lora_alpha=32))
    names = list(st.adapter_names())
    assert len(names) == 70 * 2 * 4          # 70 transformer blocks x (attn1, attn2) x (q, k, v, out.0)
    assert st.master.numel() == 46_448_640   # 46.45 M LoRA params at r=32
    sd = st.state_dict_peft()
    diff = lora_io.peft_to_diffusers(sd)
    k = "mid_block.attentions.0.transformer_blocks.9.attn2.to_out.0.lora.up.weight"
    assert k in diff and diff[k].shape == (1280, 32)
    assert diff["down_blocks.1.attentions.0.transformer_blocks.0.attn2.to_k.lora.down.weight"].shape == (32, 2048)
    back = lora_io.diffusers_to_peft({f"unet.{kk}": v for kk, v in diff.items()})
    assert set(back) == set(sd)


def test_lora_safetensors_format(tmp_path):
    from safetensors.torch import load_file
    from pairwise_sample_optimization_amd import lora_io
    sd = {"a.attn1.to_q.lora_A.weight": torch.randn(4, 8), "a.attn1.to_q.lora_B.weight": torch.randn(8, 4)}
    lora_io.save_lora_weights(str(tmp_path), lora_io.peft_to_diffusers(sd))
    raw = load_file(str(tmp_path / lora_io.LORA_WEIGHT_NAME))
    assert set(raw) == {"unet.a.attn1.to_q.lora.down.weight", "unet.a.attn1.to_q.lora.up.weight"}
    got, alphas = lora_io.lora_state_dict(str(tmp_path))
    assert alphas is None
    assert torch.equal(lora_io.diffusers_to_peft(got)["a.attn1.to_q.lora_B.weight"], sd["a.attn1.to_q.lora_B.weight"])


def test_trainer_from_config_latent_dtype_follows_mixed_precision():
    """DMD2 from the reference config: latents (and so the step / log-prob arithmetic) in weight_dtype, as D:329-333
    and DP/sdxl_dmd_with_logprob.py:91-101 make them; turbo always fp32 (DP/turbo_inference_with_logprob.py:69)."""
    import warnings
    from pairwise_sample_optimization_amd.config import config_sdxl_dmd_dpo
    from pairwise_sample_optimization_amd.trainer import PSOTrainer
    seen = {}

    class Probe(PSOTrainer):
        def __init__(self, unet, **kw):  # capture what from_config resolves, build nothing
            seen.update(kw)

    c = config_sdxl_dmd_dpo.get_config()
    for mp, want in (("fp16", torch.float16), ("bf16", torch.bfloat16), ("no", torch.float32)):
        c.mixed_precision = mp
        Probe.from_config(None, c, mode="dmd")
        assert seen["latent_dtype"] == want, (mp, seen["latent_dtype"])
        Probe.from_config(None, c, mode="turbo")
        assert seen["latent_dtype"] == torch.float32
    c.mixed_precision = "fp16"
    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter("always")
        Probe.from_config(None, c, mode="dmd", latent_dtype=torch.float32)
    assert seen["latent_dtype"] == torch.float32 and any("mixed_precision" in str(x.message) for x in w)


def test_add_adapter_honours_or_rejects_lora_config():
    """The reference's LoraConfig (T:338-343: r, lora_alpha = r, init 'gaussian', to_k / to_q / to_v / to_out.0) is
    accepted in peft's own form; any field that would make peft train other adapters raises instead of being ignored."""
    from pairwise_sample_optimization_amd.unet import LoraConfig, UNet2DConditionModel, UNetConfig
    with torch.device("meta"):
        u = UNet2DConditionModel(UNetConfig.sdxl())
    ref = dict(r=16, lora_alpha=16, init_lora_weights="gaussian", target_modules=["to_k", "to_q", "to_v", "to_out.0"])
    st = u.add_adapter(LoraConfig(**ref))
    assert (st.r, st.scale) == (16, 1.0)
    st = u.add_adapter(LoraConfig(**dict(ref, lora_alpha=32, target_modules=("to_out.0", "to_v", "to_q", "to_k"),
                                         task_type=None, inference_mode=False)))
    assert (st.r, st.scale) == (16, 2.0)
    bad = [dict(target_modules=["to_q", "to_v"]), dict(target_modules=["to_k", "to_q", "to_v", "to_out.0", "proj_in"]),
           dict(target_modules="to_q|to_k|to_v|to_out.0"), dict(target_modules=None), dict(init_lora_weights=True),
           dict(init_lora_weights="pissa"), dict(use_dora=True), dict(use_rslora=True), dict(lora_dropout=0.1),
           dict(bias="all"), dict(rank_pattern={"to_q": 4}), dict(alpha_pattern={"to_q": 4}),
           dict(modules_to_save=["conv_in"]), dict(layers_to_transform=[0]), dict(r=12), dict(r=0), dict(lora_alpha=0)]
    for b in bad:
        with pytest.raises(ValueError):
            u.add_adapter(LoraConfig(**dict(ref, **b)))
    # namespace configs: absent fields are the reference's, present ones are checked the same way
    assert u.add_adapter(SimpleNamespace(r=8, lora_alpha=8)).r == 8
    with pytest.raises(ValueError):
        u.add_adapter(SimpleNamespace(r=8, lora_alpha=8, target_modules=["to_q"]))
    # peft's default (init True, no target_modules) is not the reference's adapter either
    with pytest.raises(ValueError):
        u.add_adapter(LoraConfig(r=8, lora_alpha=8))
