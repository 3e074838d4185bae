"""Pin the oracle (and the product's host-side index math) to fixtures produced by EXECUTING the reference's own
source lines (tools/make_golden.py `exec_ref`): the loss at the clamp bounds and ties (T:844-850, D:848-854),
sample_compare (T:401-416), compare (D:420-434), the per-epoch shuffle (T:733-745, D:737-749), the DreamBooth loss
(DB:1846-1935) and the DMD2 step on fp16 / bf16 latents (DP/distilled_inference_with_logprob.py).  CPU only."""
import os

import numpy as np
import pytest
import torch

from oracle import pso_math as pm
from oracle.shuffle import reference_shuffle

G = os.path.join(os.path.dirname(__file__), "golden")
load = lambda name: np.load(os.path.join(G, name))


@pytest.mark.parametrize("tag", ["turbo", "dmd"])
def test_oracle_loss_at_clamp_bounds_and_ties(tag):
    d = load("loss_boundary.npz")
    loss, _, inside = pm.pair_loss(d["lp_pol"], d["lp_ref"], d[f"pref_{tag}"], d["beta"], d["clip_eps"])
    np.testing.assert_allclose(loss, d[f"loss_{tag}"], rtol=2e-6)
    # rows 0, 2, 6, 7 sit exactly at exp(Δ) = 1 -/+ eps: torch.clamp passes the gradient there
    assert inside[0].all() and inside[2, 1] and inside[6, 0] and inside[7, 1]
    g = pm.pair_loss_dlp(d["lp_pol"], d["lp_ref"], d[f"pref_{tag}"], d["beta"], d["clip_eps"])
    np.testing.assert_allclose(g, d[f"dlp_{tag}"], rtol=2e-5, atol=1e-9)
    assert (g[0] != 0).all()


def test_oracle_preferences_vs_executed_reference():
    d = load("preferences.npz")
    for m in (1, 3):
        c = pm.sample_compare(d[f"sc_a_m{m}"], d[f"sc_b_m{m}"], d[f"sc_idx_m{m}"])
        np.testing.assert_array_equal(c, d[f"sc_c_m{m}"])
    for m in (1, 2):
        np.testing.assert_array_equal(pm.compare(d[f"cmp_a_m{m}"], d[f"cmp_b_m{m}"]), d[f"cmp_c_m{m}"])
    assert (d["cmp_c_m1"] == 0).all(axis=1).any()  # the fixture holds DMD2 ties


@pytest.mark.parametrize("name", ["shuffle_turbo.npz", "shuffle_dmd.npz"])
@pytest.mark.parametrize("P", [1, 2, 3])
def test_shuffle_oracle_and_product_index_vs_executed_reference(name, P):
    """The reference's shuffled `samples` (before re-batching) vs (a) the numpy restatement and (b) the trainer's
    micro-step-ordered gather index on the same perm / perms.  Bit-exact."""
    from pairwise_sample_optimization_amd.trainer import shuffle_index
    d = load(name)
    perm, perms = d["perm"], d["perms"]
    Bp, T = perms.shape
    keys = [k[3:] for k in d.files if k.startswith("in_") and d[k].ndim == 6]  # latents [Bp, 2, T, C, h, w]
    ref_out = {k: d["out_" + k] for k in keys}
    # (a) oracle restatement of T:733-745 (per micro-step members)
    steps = reference_shuffle({k: d["in_" + k] for k in keys}, perm, perms, P)
    for s, ms in enumerate(steps):
        b, j = divmod(s, T)
        for k in keys:
            np.testing.assert_array_equal(ms[k][0], ref_out[k][b * P:(b + 1) * P, 0, j])
            np.testing.assert_array_equal(ms[k][1], ref_out[k][b * P:(b + 1) * P, 1, j])
    # (b) product index math: row ((b*T + j)*P + p)*2 + k of the gathered stream = reference [b*P + p, k, j]
    img_idx, pair_img, tsel = shuffle_index(torch.from_numpy(perm), torch.from_numpy(perms), P)
    nb = Bp // P
    for k in keys:
        flat = torch.from_numpy(d["in_" + k]).reshape((Bp * 2 * T,) + d["in_" + k].shape[3:])
        got = flat[img_idx].reshape((nb, T, P, 2) + flat.shape[1:])
        want = torch.from_numpy(ref_out[k][:nb * P]).reshape((nb, P, 2, T) + flat.shape[1:]).permute(
            0, 3, 1, 2, 4, 5, 6)
        assert torch.equal(got, want)
    ts_in = torch.from_numpy(d["in_timesteps"])          # [Bp, T]
    got_t = ts_in[pair_img // 2, tsel].reshape(nb, T, P, 2)
    want_t = torch.from_numpy(d["out_timesteps"][:nb * P]).reshape(nb, P, 2, T).permute(0, 3, 1, 2)
    assert torch.equal(got_t, want_t)
    lp_in = torch.from_numpy(d["in_log_probs"]).reshape(Bp * 2, T)  # [Bp, 2, T] -> rows 2p + k
    got_lp = lp_in[pair_img, tsel].reshape(nb, T, P, 2)
    want_lp = torch.from_numpy(d["out_log_probs"][:nb * P]).reshape(nb, P, 2, T).permute(0, 3, 1, 2)
    assert torch.equal(got_lp, want_lp)
    # per-pair tensors (rewards, prompt embeds) follow the pair permutation only
    pair_ids = (pair_img // 2).reshape(nb, T, P, 2)[:, 0, :, 0].reshape(-1)
    for key in ("rewards", "prompt_embeds"):
        assert torch.equal(torch.from_numpy(d["in_" + key])[pair_ids], torch.from_numpy(d["out_" + key][:nb * P]))


@pytest.mark.parametrize("name", ["db_loss_pso.npz", "db_loss_pso_db.npz"])
def test_oracle_db_loss_vs_executed_reference(name):
    d = load(name)
    lt = "pso" if int(d["loss_type"]) == 0 else "pso_db"
    args = (d["eps"], d["noisy"], d["x0"], d["sigma"], float(d["beta"]), float(d["neg_defactor"]), float(d["prior_w"]),
            lt, d["eps_ref"] if lt == "pso" else None)
    loss, l, _ = pm.db_loss(*args)
    np.testing.assert_allclose(l, d["model_losses"], rtol=2e-6)
    np.testing.assert_allclose(loss, d["loss"], rtol=2e-6)
    g = pm.db_loss_deps(*args)
    ref = d["grad_eps"]
    assert np.abs(g - ref).max() <= 1e-5 * np.abs(ref).max()


REPLAY = ["dmd_replay_fp16_P2_h16_t999.npz", "dmd_replay_fp16_P3_h16_t749.npz", "dmd_replay_bf16_P2_h16_t499.npz"]


@pytest.mark.parametrize("name", REPLAY)
def test_oracle_dmd_latent_dtype_replay(name):
    """DP/distilled_inference_with_logprob.py on fp16 / bf16 latents: the element-wise chain is reproduced exactly;
    the mean differs from torch's fp32 cascade sum only in summation order, so the latent-dtype log-prob may move by
    one ulp of that dtype (none does in these fixtures)."""
    d = load(name)
    lat = str(d["latent"])
    sa, sb, _, _ = pm.dmd_coefs(d["alphas_cumprod"], d["t"], d["t_prev"])
    ulp = 2.0 ** -10 if lat == "fp16" else 2.0 ** -7
    lp = {}
    for k in range(2):
        prev, lps = pm.dmd_step_logprob_latent(d[f"x{k}"], d[f"eps_ref{k}"], sa, sb, d["alphas_cumprod"],
                                               d["t_prev"], lat, noise=d[f"noise{k}"])
        np.testing.assert_array_equal(prev, d[f"prev{k}"])
        np.testing.assert_allclose(lps, d[f"lp_sample{k}"], rtol=ulp)
        for w in ("pol", "ref"):
            _, lp[w + str(k)] = pm.dmd_step_logprob_latent(d[f"x{k}"], d[f"eps_{w}{k}"], sa, sb, d["alphas_cumprod"],
                                                           d["t_prev"], lat, prev=d[f"prev{k}"])
            np.testing.assert_allclose(lp[w + str(k)], d[f"lp_{w}{k}"], rtol=ulp)
    lpp = np.stack([lp["pol0"], lp["pol1"]], 1)
    lpr = np.stack([lp["ref0"], lp["ref1"]], 1)
    loss, _, _ = pm.pair_loss(lpp, lpr, d["pref"], d["beta"], d["clip_eps"], latent=lat)
    np.testing.assert_allclose(loss, d["loss"], rtol=1e-5)
