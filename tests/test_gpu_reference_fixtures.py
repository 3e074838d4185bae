"""GPU parity of the HIP kernels against fixtures made by EXECUTING the reference's own source lines
(tools/make_golden.py): the loss scalar stage at the clamp bounds / ties (T:844-850, D:848-854), the preference
kernel (sample_compare T:401-416, compare D:420-434), the shuffle gather (T:733-745, D:737-749), the DreamBooth loss
(DB:1846-1935) and the DMD2 step + loss on fp16 / bf16 latents (DP/distilled_inference_with_logprob.py replay)."""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
G = os.path.join(os.path.dirname(__file__), "golden")
load = lambda name: np.load(os.path.join(G, name))


@pytest.mark.parametrize("tag,mode", [("turbo", 0), ("dmd", 1)])
def test_loss_scalar_stage_at_clamp_bounds(cuda, tag, mode):
    from pairwise_sample_optimization_amd import kernels as K
    d = load("loss_boundary.npz")
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(cuda)
    loss, dlp = K.pair_loss_from_lp(mode, T(d["lp_pol"]), T(d["lp_ref"]), T(d[f"pref_{tag}"]), float(d["beta"]),
                                    float(d["clip_eps"]))
    np.testing.assert_allclose(loss.item(), d[f"loss_{tag}"], rtol=2e-6)
    g = dlp.cpu().numpy()
    np.testing.assert_allclose(g, d[f"dlp_{tag}"], rtol=2e-5, atol=1e-9)
    assert (g[0] != 0).all()  # exp(Δ) exactly 1 -/+ eps: the gradient passes (torch.clamp semantics)


def test_preference_kernel_vs_executed_reference(cuda):
    from pairwise_sample_optimization_amd import kernels as K
    d = load("preferences.npz")
    for m in (1, 3):
        rw = torch.stack([torch.from_numpy(d[f"sc_a_m{m}"]), torch.from_numpy(d[f"sc_b_m{m}"])], 1).to(cuda)
        idx = torch.from_numpy(d[f"sc_idx_m{m}"]).to(cuda)
        c = K.preference(rw, 0, reward_idx=idx)
        np.testing.assert_array_equal(c.cpu().numpy(), d[f"sc_c_m{m}"])
    for m in (1, 2):
        a, b = torch.from_numpy(d[f"cmp_a_m{m}"]), torch.from_numpy(d[f"cmp_b_m{m}"])
        if a.dim() == 1:
            a, b = a[:, None], b[:, None]
        c = K.preference(torch.stack([a, b], 1).to(cuda), 1)
        np.testing.assert_array_equal(c.cpu().numpy(), d[f"cmp_c_m{m}"])


@pytest.mark.parametrize("name", ["shuffle_turbo.npz", "shuffle_dmd.npz"])
@pytest.mark.parametrize("P", [1, 2])
def test_shuffle_gather_vs_executed_reference(cuda, name, P):
    """pso_gather_rows with the trainer's index on the reference's perm / perms: bit-exact rows."""
    from pairwise_sample_optimization_amd import kernels as K
    from pairwise_sample_optimization_amd.trainer import shuffle_index
    d = load(name)
    perm, perms = torch.from_numpy(d["perm"]).to(cuda), torch.from_numpy(d["perms"]).to(cuda)
    Bp, T = d["perms"].shape
    nb = Bp // P
    img_idx, pair_img, tsel = shuffle_index(perm, perms, P)
    for key in [k[3:] for k in d.files if k.startswith("in_") and d[k].ndim == 6]:
        src = torch.from_numpy(d["in_" + key]).to(cuda)
        flat = src.reshape((Bp * 2 * T,) + src.shape[3:])
        got = K.gather_rows(flat, img_idx).reshape((nb, T, P, 2) + flat.shape[1:])
        want = torch.from_numpy(d["out_" + key][:nb * P]).reshape((nb, P, 2, T) + flat.shape[1:]).permute(
            0, 3, 1, 2, 4, 5, 6)
        assert torch.equal(got.cpu(), want)
    pe = torch.from_numpy(d["in_prompt_embeds"]).to(cuda).reshape(Bp * 2, -1)  # per-image rows 2p + k
    got = K.gather_rows(pe, pair_img).reshape(nb, T, P, 2, -1)[:, 0].reshape(nb * P, 2, *d["in_prompt_embeds"].shape[2:])
    assert torch.equal(got.cpu(), torch.from_numpy(d["out_prompt_embeds"][:nb * P]))


@pytest.mark.parametrize("name", ["db_loss_pso.npz", "db_loss_pso_db.npz"])
def test_db_loss_kernels_vs_executed_reference(cuda, name):
    from pairwise_sample_optimization_amd import kernels as K
    d = load(name)
    lt = int(d["loss_type"])
    T = lambda a: torch.from_numpy(a).to(cuda)
    eps = T(d["eps"]).bfloat16()  # bf16-valued in the fixture: exact
    er = T(d["eps_ref"]).bfloat16() if lt == K.DB_SIGMOID else None
    B = d["eps"].shape[0] // 2
    ws = K.db_loss_ws(B, d["eps"][0].size, cuda)
    args = (float(d["beta"]), float(d["neg_defactor"]), float(d["prior_w"]))
    loss, losses, _ = K.db_loss_fwd(lt, eps, T(d["noisy"]), T(d["x0"]), T(d["sigma"]), *args, ws, eps_ref=er)
    np.testing.assert_allclose(losses[:2 * B].cpu().numpy(), d["model_losses"], rtol=2e-6)
    np.testing.assert_allclose(loss.item(), d["loss"], rtol=2e-5)
    g = K.db_loss_bwd(lt, eps, T(d["noisy"]), T(d["x0"]), T(d["sigma"]), *args, ws,
                      out_dtype=torch.float32).cpu().numpy()
    ref = d["grad_eps"]
    assert np.abs(g - ref).max() <= 1e-4 * np.abs(ref).max()


REPLAY = ["dmd_replay_fp16_P2_h16_t999.npz", "dmd_replay_fp16_P3_h16_t749.npz", "dmd_replay_bf16_P2_h16_t499.npz"]


@pytest.mark.parametrize("name", REPLAY)
def test_dmd_latent_dtype_replay_vs_reference(cuda, name):
    """The reference's DMD2 step on fp16 / bf16 latents (x0, mean, re-noise and log-density in the latent dtype) and
    D:848-854 on those latent-dtype log-probs: prev bit-exact, log-probs within one latent-dtype ulp (summation
    order of the mean), loss rtol 1e-5; the drop-in distilled_step_with_logprob returns the latent dtype."""
    from pairwise_sample_optimization_amd import kernels as K, pso_core
    from pairwise_sample_optimization_amd.pso_pytorch.diffusers_patch.distilled_inference_with_logprob import \
        distilled_step_with_logprob
    from types import SimpleNamespace
    d = load(name)
    lat = torch.float16 if str(d["latent"]) == "fp16" else torch.bfloat16
    mode = pso_core.dmd_mode(lat)
    ulp = 2.0 ** -10 if lat == torch.float16 else 2.0 ** -7
    P = d["x0"].shape[0]
    coef = pso_core.dmd_coef(torch.from_numpy(d["alphas_cumprod"]), torch.from_numpy(d["t"]),
                             torch.from_numpy(d["t_prev"]), latent_dtype=lat).to(cuda)
    T = lambda k: torch.from_numpy(d[k]).to(cuda)
    sched = SimpleNamespace(alphas_cumprod=torch.from_numpy(d["alphas_cumprod"]))
    for k in range(2):
        prev, lp = K.step_logprob(mode, T(f"x{k}"), T(f"eps_ref{k}"), coef, noise=T(f"noise{k}"), noise_shared=P > 1)
        np.testing.assert_array_equal(prev.cpu().numpy(), d[f"prev{k}"])
        np.testing.assert_allclose(lp.cpu().numpy(), d[f"lp_sample{k}"], rtol=ulp)
        # drop-in surface with latent-dtype tensors, prev_sample given
        _, lpd = distilled_step_with_logprob(sched, T(f"eps_pol{k}"), torch.from_numpy(d["t"]).to(cuda),
                                             torch.from_numpy(d["t_prev"]).to(cuda), T(f"x{k}").to(lat),
                                             prev_sample=T(f"prev{k}").to(lat))
        assert lpd.dtype == lat
        np.testing.assert_allclose(lpd.float().cpu().numpy(), d[f"lp_pol{k}"], rtol=ulp)
    inter = lambda a, b: torch.stack([T(a), T(b)], 1).reshape((2 * P,) + d["x0"].shape[1:]).contiguous()
    x, xp = inter("x0", "x1"), inter("prev0", "prev1")
    ep, er = inter("eps_pol0", "eps_pol1"), inter("eps_ref0", "eps_ref1")
    coef2 = torch.stack([coef, coef], 1).reshape(2 * P, -1).contiguous()
    ws = K.pair_loss_ws(P, x[0].numel(), cuda)
    loss, lp = K.pair_loss_fwd(mode, x, xp, ep, er, coef2, T("pref"), float(d["beta"]), float(d["clip_eps"]), ws)
    lp = lp.cpu().numpy().reshape(P, 2, 2)
    for k in range(2):
        np.testing.assert_allclose(lp[:, k, 0], d[f"lp_pol{k}"], rtol=ulp)
        np.testing.assert_allclose(lp[:, k, 1], d[f"lp_ref{k}"], rtol=ulp)
    np.testing.assert_allclose(loss.item(), d["loss"], rtol=1e-5)
