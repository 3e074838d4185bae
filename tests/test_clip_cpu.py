"""CPU checks of the CLIP / prompt boundary: checkpoint key layout against transformers, the
PromptDataset drop-in and the tokenizer collate path."""
import json

import pytest
import torch

from pairwise_sample_optimization_amd.clip import (CLIPModel, CLIPTextConfig, CLIPTextModel,
                                                   CLIPTextModelWithProjection, CLIPVisionConfig)


def _shapes(sd):
    """key -> shape in the transformers 4.x checkpoint layout (5.x's CLIPTextModel drops the `text_model.` prefix
    of its own modules; checkpoints keep it)."""
    out = {}
    for k, v in sd.items():
        if k.endswith("position_ids"):
            continue
        if k.startswith(("embeddings.", "encoder.", "final_layer_norm.")):
            k = "text_model." + k
        out[k] = tuple(v.shape)
    return out


@pytest.mark.parametrize("which", ["sdxl_l", "sdxl_bigg", "pickscore_h"])
def test_text_keys_match_transformers(which):
    from oracle.clip_ref import _text_cfg
    from transformers import CLIPTextModel as HT, CLIPTextModelWithProjection as HTP
    cfg = getattr(CLIPTextConfig, which)()
    with torch.device("meta"):
        ours = CLIPTextModel(cfg)
        ours_p = CLIPTextModelWithProjection(cfg)
        hf = HT(_text_cfg(cfg))
        hf_p = HTP(_text_cfg(cfg))
    assert _shapes(ours.state_dict()) == _shapes(hf.state_dict())
    assert _shapes(ours_p.state_dict()) == _shapes(hf_p.state_dict())


def test_clip_model_keys_match_transformers():
    from oracle.clip_ref import _text_cfg, _vision_cfg
    from transformers import CLIPConfig, CLIPModel as HM
    tc, vc = CLIPTextConfig.pickscore_h(), CLIPVisionConfig()
    with torch.device("meta"):
        ours = CLIPModel(tc, vc, 1024)
        hf = HM(CLIPConfig(text_config=_text_cfg(tc).to_dict(), vision_config=_vision_cfg(vc).to_dict(),
                           projection_dim=1024))
    assert _shapes(ours.state_dict()) == _shapes(hf.state_dict())


def test_from_config_dict_honours_transformers_keys():
    d = {"hidden_size": 64, "intermediate_size": 128, "num_hidden_layers": 2, "num_attention_heads": 2,
         "hidden_act": "gelu", "projection_dim": 32, "vocab_size": 1000, "architectures": ["CLIPTextModel"]}
    with torch.device("meta"):
        m = CLIPTextModelWithProjection.from_config(d)
    assert m.config.hidden_size == 64 and m.config.num_hidden_layers == 2 and m.config.hidden_act == "gelu"
    assert tuple(m.text_projection.weight.shape) == (32, 64)
    with pytest.raises(ValueError):
        with torch.device("meta"):
            CLIPTextModel.from_config(dict(d, hidden_act="relu"))


def _tiny_tokenizer_dir(tmp_path):
    """A minimal CLIP BPE vocabulary (byte-level base alphabet + a few merges) in the transformers file layout."""
    bs = list(range(ord("!"), ord("~") + 1)) + list(range(ord("\u00a1"), ord("\u00ac") + 1)) + \
        list(range(ord("\u00ae"), ord("\u00ff") + 1))
    cs, n = bs[:], 0
    for b in range(256):  # the GPT-2 / CLIP byte -> printable-unicode alphabet
        if b not in bs:
            bs.append(b)
            cs.append(256 + n)
            n += 1
    base = [chr(c) for c in cs]
    vocab = base + [b + "</w>" for b in base]
    merges = [("c", "a"), ("ca", "t</w>"), ("d", "o"), ("do", "g</w>")]
    vocab += ["".join(m) for m in merges] + ["<|startoftext|>", "<|endoftext|>"]
    d = tmp_path / "tokenizer"
    d.mkdir()
    (d / "vocab.json").write_text(json.dumps({t: i for i, t in enumerate(vocab)}))
    (d / "merges.txt").write_text("#version: 0.2\n" + "\n".join(" ".join(m) for m in merges) + "\n")
    (d / "tokenizer_config.json").write_text(json.dumps({"model_max_length": 77, "pad_token": "<|endoftext|>"}))
    (d / "special_tokens_map.json").write_text(json.dumps({"bos_token": "<|startoftext|>",
                                                           "eos_token": "<|endoftext|>",
                                                           "unk_token": "<|endoftext|>",
                                                           "pad_token": "<|endoftext|>"}))
    return d


def test_prompt_dataset_and_collate(tmp_path):
    from pairwise_sample_optimization_amd.prompts import load_tokenizer, tokenize_captions
    from pairwise_sample_optimization_amd.pso_pytorch.prompt_dataset import PromptDataset
    p = tmp_path / "prompts.json"
    p.write_text(json.dumps([{"caption": "a cat"}, {"caption": "a dog"}, {"caption": "cat dog"}]))
    ds = PromptDataset(str(p))
    assert len(ds) == 3 and ds[1] == {"prompt": "a dog"}
    tok = load_tokenizer(str(_tiny_tokenizer_dir(tmp_path)))
    b = PromptDataset.sdxl_collate_fn([ds[0], ds[2]], tok, tok)
    assert b["prompts"] == ["a cat", "cat dog"]
    for k in ("input_ids_one", "input_ids_two"):
        ids = b[k]
        assert tuple(ids.shape) == (2, 77) and ids.dtype == torch.int64
        ref = tok(["a cat", "cat dog"], padding="max_length", truncation=True, max_length=77,
                  return_tensors="pt").input_ids
        assert torch.equal(ids, ref)
    bos, eos = tok.convert_tokens_to_ids("<|startoftext|>"), tok.convert_tokens_to_ids("<|endoftext|>")
    assert int(ids[0, 0]) == bos and int(ids[0].max()) == eos   # eos = the argmax the pooled row is taken at
    one, two = tokenize_captions([tok, tok], {"caption": ["a cat"]})
    assert torch.equal(one, two) and one.shape == (1, 77)
    s = PromptDataset.sd_collate_fn([ds[0]], tok)
    assert tuple(s["input_ids"].shape) == (1, 77)
    with pytest.raises(ValueError):
        PromptDataset()
