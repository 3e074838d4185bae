"""Pin the numpy oracle (oracle/pso_math.py) against golden vectors produced by the REFERENCE step functions
(tools/make_golden.py).  CPU only."""
import glob
import os

import numpy as np
import pytest

from oracle import pso_math as pm

GOLD = sorted(glob.glob(os.path.join(os.path.dirname(__file__), "golden", "pso_*.npz")))


def _coefs(d):
    if int(d["mode"]) == 0:
        s, su, dt = pm.turbo_coefs(d["sigmas"], d["timesteps"], d["t"])
        return dict(sigma=s, s_up=su, dt=dt)
    sa, sb, sap, sbp = pm.dmd_coefs(d["alphas_cumprod"], d["t"], d["t_prev"])
    return dict(sa_t=sa, sb_t=sb, sa_prev=sap, sb_prev=sbp)


def _step(d, c, k, eps, prev=None, noise=None):
    x = d[f"x{k}"]
    if int(d["mode"]) == 0:
        return pm.turbo_step_logprob(x, eps, c["sigma"], c["s_up"], c["dt"], prev=prev, noise=noise)
    return pm.dmd_step_logprob(x, eps, c["sa_t"], c["sb_t"], c["sa_prev"], c["sb_prev"], prev=prev, noise=noise)


def test_golden_present():
    assert len(GOLD) >= 8


@pytest.mark.parametrize("path", GOLD, ids=[os.path.basename(p) for p in GOLD])
def test_oracle_matches_reference(path):
    d = np.load(path)
    c = _coefs(d)
    for k in range(2):
        # sampling branch: prev_sample = mean + noise*std is element-wise -> near bit-exact
        prev, lp_s = _step(d, c, k, d[f"eps_ref{k}"], noise=d[f"noise{k}"])
        np.testing.assert_allclose(prev, d[f"prev{k}"], rtol=2e-6, atol=2e-6)
        np.testing.assert_allclose(lp_s, d[f"lp_sample{k}"], rtol=1e-6)
        _, lp_p = _step(d, c, k, d[f"eps_pol{k}"], prev=d[f"prev{k}"])
        _, lp_r = _step(d, c, k, d[f"eps_ref{k}"], prev=d[f"prev{k}"])
        np.testing.assert_allclose(lp_p, d["lp_pol"][:, k], rtol=1e-6)
        np.testing.assert_allclose(lp_r, d["lp_ref"][:, k], rtol=1e-6)
    loss, _, _ = pm.pair_loss(d["lp_pol"], d["lp_ref"], d["pref"], d["beta"], d["clip_eps"])
    np.testing.assert_allclose(loss, d["loss"], rtol=1e-5)  # lp rounding x beta amplification
    g = pm.pair_loss_dlp(d["lp_pol"], d["lp_ref"], d["pref"], d["beta"], d["clip_eps"])
    for k in range(2):
        if int(d["mode"]) == 0:
            dl = pm.dlp_deps_turbo(d[f"x{k}"], d[f"eps_pol{k}"], d[f"prev{k}"], c["sigma"], c["s_up"], c["dt"])
        else:
            dl = pm.dlp_deps_dmd(d[f"x{k}"], d[f"eps_pol{k}"], d[f"prev{k}"], c["sa_t"], c["sb_t"],
                                 c["sa_prev"], c["sb_prev"])
        grad = g[:, k].reshape(-1, 1, 1, 1) * dl
        ref = d[f"grad_eps_pol{k}"]
        scale = max(np.abs(ref).max(), 1e-30)
        assert np.abs(grad - ref).max() <= 1e-5 * scale + 1e-12


def test_schedulers_match_survey_appendix_c():
    from oracle.schedulers import EulerAncestralTrailing, LCMTable
    s = EulerAncestralTrailing()
    s.set_timesteps(4)
    assert s.timesteps.tolist() == [999.0, 749.0, 499.0, 249.0]
    np.testing.assert_allclose(s.sigmas.numpy(), [14.614647, 4.081731, 1.612887, 0.693205, 0.0], rtol=2e-6)
    assert abs(float(s.init_noise_sigma) - 14.6146) < 1e-3
    _, su, dt = pm.turbo_coefs(s.sigmas.numpy(), s.timesteps.numpy(), [999.0, 749.0, 499.0])
    np.testing.assert_allclose(su, [3.919305, 1.481626, 0.625915], rtol=2e-6)
    s.set_timesteps(2)
    _, su, dt = pm.turbo_coefs(s.sigmas.numpy(), s.timesteps.numpy(), [999.0])
    np.testing.assert_allclose(su, [1.603035], rtol=2e-6)
    ac = LCMTable().alphas_cumprod.numpy()
    np.testing.assert_allclose(ac[[999, 749, 499, 249]], [0.0046601, 0.0566235, 0.2776694, 0.6754321], rtol=2e-5)


def test_compare_rules():
    a = np.array([[0.1], [0.5], [0.3]], np.float32)
    b = np.array([[0.2], [0.4], [0.3]], np.float32)
    # turbo: ties -> member 0 loses
    np.testing.assert_array_equal(pm.sample_compare(a, b, np.zeros(3, int)), [[-1, 1], [1, -1], [-1, 1]])
    # dmd: strict pareto, ties -> (0, 0)
    np.testing.assert_array_equal(pm.compare(a, b), [[-1, 1], [1, -1], [0, 0]])


def test_adam8bit_dynamic_maps():
    """bitsandbytes' dynamic quantisation maps (oracle/adam8bit.py): 256 sorted codes, signed map symmetric with one
    zero and 1.0 at the top, unsigned map on [0, 1]."""
    import numpy as np
    from oracle.adam8bit import create_dynamic_map, quantize_nearest
    s, u = create_dynamic_map(True), create_dynamic_map(False)
    assert s.shape == (256,) and u.shape == (256,)
    assert (np.diff(s) >= 0).all() and (np.diff(u) >= 0).all()
    assert s[-1] == 1.0 and u[-1] == 1.0 and u[0] == 0.0 and (u >= 0).all()
    assert (s == 0).sum() == 1 and np.allclose(np.sort(-s[s < 0]), np.sort(s[(s > 0) & (s < 1)]))
    assert s.min() > -1.0 and abs(s[s > 0].min() - 5.5e-7) < 1e-7
    x = np.array([0.0, 1.0, -0.3, 0.31, 1e-7], dtype=np.float32)
    q = quantize_nearest(x, s)
    assert s[q[0]] == 0.0 and s[q[1]] == 1.0 and abs(s[q[2]] + 0.3) < 0.02 and abs(s[q[3]] - 0.31) < 0.02
