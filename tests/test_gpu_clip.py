"""GPU parity of the CLIP towers and the reward image path against transformers (fp32, same
weights) and PIL (the CLIPImageProcessor's resize), through the HIP kernels of clip.hip / gemm.hip / norm.hip."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


@pytest.mark.parametrize("S,D,H,causal", [(77, 64, 12, True), (77, 64, 20, True), (257, 80, 16, False),
                                          (50, 80, 2, True), (130, 128, 3, False)])
def test_attention_small_vs_fp32(cuda, S, D, H, causal):
    from pairwise_sample_optimization_amd import kernels as K
    B = 3
    g = torch.Generator(device="cuda").manual_seed(S + D)
    qkv = torch.randn(B * S, 3 * H * D, device=cuda, generator=g).bfloat16()
    C = H * D
    o = K.attention_small(qkv[:, :C], qkv[:, C:2 * C], qkv[:, 2 * C:], B, S, H, causal, D ** -0.5)
    f = lambda t: t.float().reshape(B, S, H, D).transpose(1, 2)
    q, k, v = f(qkv[:, :C]), f(qkv[:, C:2 * C]), f(qkv[:, 2 * C:])
    s = q @ k.transpose(-1, -2) * D ** -0.5
    if causal:
        s = s.masked_fill(torch.triu(torch.ones(S, S, dtype=torch.bool, device=cuda), 1), float("-inf"))
    ref = (torch.softmax(s, -1) @ v).transpose(1, 2).reshape(B * S, C)
    assert _rel(o, ref) < 8e-3


def _ids(B, S, vocab, g, cuda):
    """random prompts: bos, tokens, eos (the max id: the legacy argmax pooling row), eos padding."""
    ids = torch.randint(1, vocab - 2, (B, S), generator=g, device=cuda)
    ids[:, 0] = vocab - 2
    for b in range(B):
        n = 5 + 17 * b
        ids[b, n] = vocab - 1
        ids[b, n + 1:] = vocab - 1
    return ids


@pytest.mark.parametrize("which", ["sdxl_l", "sdxl_bigg"])
def test_text_encoder_vs_transformers(cuda, which):
    """Full-size SDXL text encoder (random weights) vs transformers fp32: the hidden_states[-2] encode_prompt reads,
    the final hidden state, and the pooled / projected output."""
    from oracle.clip_ref import hf_text_model
    from pairwise_sample_optimization_amd.clip import CLIPTextConfig, CLIPTextModel, CLIPTextModelWithProjection
    cfg = getattr(CLIPTextConfig, which)()
    proj = which == "sdxl_bigg"
    with torch.device(cuda):
        m = (CLIPTextModelWithProjection if proj else CLIPTextModel)(cfg)
    m.init_weights(3)
    hf = hf_text_model(cfg, m.state_dict(), cuda, projection=proj)
    g = torch.Generator(device="cuda").manual_seed(5)
    ids = _ids(3, 77, cfg.vocab_size, g, cuda)
    out = m(ids, output_hidden_states=True)
    with torch.no_grad():
        ref = hf(ids, output_hidden_states=True)
    e_h2 = _rel(out.hidden_states[-2], ref.hidden_states[-2])
    e_last = _rel(out.last_hidden_state, ref.last_hidden_state)
    e0 = _rel(out[0], ref[0])
    print(f"{which}: hidden[-2] {e_h2:.2e} last {e_last:.2e} out[0] {e0:.2e}")
    assert e_h2 < 2e-2 and e_last < 2e-2 and e0 < 2e-2


def test_encode_prompt_sdxl(cuda):
    """T:96-118 on both SDXL encoders: prompt_embeds [B, 77, 2048] = concat(hidden[-2]), pooled = text_embeds."""
    from oracle.clip_ref import hf_text_model
    from pairwise_sample_optimization_amd.prompts import encode_prompt, sdxl_text_encoders
    e1, e2 = sdxl_text_encoders(cuda, seed=1)
    g = torch.Generator(device="cuda").manual_seed(9)
    ids1, ids2 = _ids(2, 77, 49408, g, cuda), _ids(2, 77, 49408, g, cuda)
    pe, pooled = encode_prompt([e1, e2], [ids1, ids2])
    assert tuple(pe.shape) == (2, 77, 2048) and tuple(pooled.shape) == (2, 1280)
    h1 = hf_text_model(e1.config, e1.state_dict(), cuda)
    h2 = hf_text_model(e2.config, e2.state_dict(), cuda, projection=True)
    with torch.no_grad():
        r1, r2 = h1(ids1, output_hidden_states=True), h2(ids2, output_hidden_states=True)
    ref = torch.cat([r1.hidden_states[-2], r2.hidden_states[-2]], -1)
    assert _rel(pe, ref) < 2e-2
    assert _rel(pooled, r2[0]) < 2e-2


def test_clip_preprocess_bit_exact_vs_pil(cuda):
    """Decoded bf16 images at 1024^2 and 512^2: the trainer's uint8 quantisation (T:632-633, executed verbatim) ->
    CLIPImageProcessor (PIL bicubic) -> pixel values; ours must equal the bf16 rounding of the reference's values
    exactly (one uint8 step moves a value by >= 1/(255 std) > 1 bf16 ulp, so equality pins every resized byte)."""
    from oracle.clip_ref import clip_image_processor, trainer_uint8
    from pairwise_sample_optimization_amd import kernels as K
    from pairwise_sample_optimization_amd.clip import CLIP_MEAN, CLIP_STD
    for B, Hs in ((2, 1024), (3, 512)):
        g = torch.Generator(device="cuda").manual_seed(Hs)
        # smooth structure + noise + out-of-range values (clamped by the quantisation)
        yy = torch.linspace(-1.2, 1.2, Hs, device=cuda)
        img = (yy[None, :, None, None] * yy[None, None, :, None] * torch.randn(B, 1, 1, 3, device=cuda, generator=g)
               + 0.3 * torch.randn(B, Hs, Hs, 3, device=cuda, generator=g)).bfloat16().contiguous()
        patches = K.clip_preprocess(img, 224, 14, 592, CLIP_MEAN, CLIP_STD)
        u8 = trainer_uint8(img.permute(0, 3, 1, 2).cpu())
        pv = torch.from_numpy(clip_image_processor(u8)).to(cuda)
        ref = K.patchify(pv, 14, 592)
        assert torch.equal(patches, ref), (patches.float() - ref.float()).abs().max().item()
        # uint8 input path (the reference's PIL-image form of `score`)
        p2 = K.clip_preprocess(torch.from_numpy(np.ascontiguousarray(u8)).to(cuda), 224, 14, 592, CLIP_MEAN,
                               CLIP_STD)
        assert torch.equal(p2, ref)


def test_pickscore_vs_transformers(cuda):
    """PickScore (ViT-H/14 CLIPModel, random weights): score_tensor on decoded bf16 images vs transformers fp32 on the
    PIL-processed pixels of the same images, matched prompts (diag of text_n @ image_n^T)."""
    from oracle.clip_ref import clip_image_processor, hf_clip_model, trainer_uint8
    from pairwise_sample_optimization_amd.pso_pytorch.pickscore_utils import Selector
    sel = Selector(cuda, seed=4)
    m = sel.model
    hf = hf_clip_model(m.text_config, m.vision_config, m.config.projection_dim, m.state_dict(), cuda)
    g = torch.Generator(device="cuda").manual_seed(13)
    B = 4
    img = (0.6 * torch.randn(B, 512, 512, 3, device=cuda, generator=g)).clamp(-1, 1).bfloat16().contiguous()
    ids = _ids(B, 77, m.text_config.vocab_size, g, cuda)
    s = sel.score_tensor(img, ids)
    pv = torch.from_numpy(clip_image_processor(trainer_uint8(img.permute(0, 3, 1, 2).cpu()))).to(cuda)
    with torch.no_grad():
        ie = hf.get_image_features(pixel_values=pv)
        te = hf.get_text_features(input_ids=ids)
        ie = getattr(ie, "image_embeds", getattr(ie, "pooler_output", ie)) if not torch.is_tensor(ie) else ie
        te = getattr(te, "text_embeds", getattr(te, "pooler_output", te)) if not torch.is_tensor(te) else te
        ref = torch.nn.functional.cosine_similarity(te, ie, dim=-1)
        ours_ie = m.image_features_from_images(img)
    print(f"pickscore: ours {s.tolist()} ref {ref.tolist()} image-feature rel {_rel(ours_ie, ie):.2e}")
    assert _rel(ours_ie, ie) < 3e-2
    assert (s - ref).abs().max().item() < 2e-3
    # numpy-returning reference signature on uint8 images (the PIL-image form)
    u8 = trainer_uint8(img.permute(0, 3, 1, 2).cpu())
    s2 = sel.score(list(u8), None, input_ids=ids)
    assert np.abs(s2 - s.cpu().numpy()).max() < 1e-6


def test_light_reward_row_mean(cuda):
    from pairwise_sample_optimization_amd import kernels as K
    x = torch.randn(5, 64, 64, 3, device=cuda).bfloat16()
    assert _rel(K.row_mean(x), x.float().reshape(5, -1).mean(1)) < 1e-5
