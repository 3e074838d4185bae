"""GPU parity of the fused PSO step/loss kernels against the golden vectors of the reference (tests/golden)."""
import glob
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
GOLD = sorted(glob.glob(os.path.join(os.path.dirname(__file__), "golden", "pso_*.npz")))


def _coef(d):
    from pairwise_sample_optimization_amd import pso_core
    P = d["x0"].shape[0]
    if int(d["mode"]) == 0:
        return pso_core.turbo_coef(torch.tensor(d["sigmas"]), torch.tensor(d["timesteps"]), torch.tensor(d["t"]))
    return pso_core.dmd_coef(torch.tensor(d["alphas_cumprod"]), torch.tensor(d["t"]), torch.tensor(d["t_prev"]))


@pytest.mark.parametrize("path", GOLD, ids=[os.path.basename(p) for p in GOLD])
def test_step_and_pair_loss_vs_golden(cuda, path):
    from pairwise_sample_optimization_amd import kernels as K_
    d = np.load(path)
    mode = int(d["mode"])
    coef = _coef(d).to(cuda)
    T = lambda k: torch.tensor(d[k], device=cuda)
    for k in range(2):
        noise = T(f"noise{k}")
        prev, lp = K_.step_logprob(mode, T(f"x{k}"), T(f"eps_ref{k}"), coef, noise=noise,
                                   noise_shared=(noise.shape[0] == 1 and d[f"x{k}"].shape[0] > 1))
        np.testing.assert_allclose(prev.cpu().numpy(), d[f"prev{k}"], rtol=2e-6, atol=2e-6)
        np.testing.assert_allclose(lp.cpu().numpy(), d[f"lp_sample{k}"], rtol=1e-6)
    P = d["x0"].shape[0]
    inter = lambda a, b: torch.stack([T(a), T(b)], 1).reshape((2 * P,) + d["x0"].shape[1:])
    x = inter("x0", "x1")
    xp = inter("prev0", "prev1")
    ep = inter("eps_pol0", "eps_pol1").bfloat16()  # bf16-valued in the fixture: exact
    er = inter("eps_ref0", "eps_ref1").bfloat16()
    coef2 = torch.stack([coef, coef], 1).reshape(2 * P, -1)
    pref = T("pref")
    ws = K_.pair_loss_ws(P, x[0].numel(), cuda)
    loss, lp = K_.pair_loss_fwd(mode, x, xp, ep, er, coef2, pref, float(d["beta"]), float(d["clip_eps"]), ws)
    lp = lp.cpu().numpy().reshape(P, 2, 2)
    np.testing.assert_allclose(lp[:, :, 0], d["lp_pol"], rtol=1e-6)
    np.testing.assert_allclose(lp[:, :, 1], d["lp_ref"], rtol=1e-6)
    # loss: lp rounding (1 ulp) is amplified by beta=50 through the small log-ratio (the reference's own noise level)
    np.testing.assert_allclose(loss.item(), d["loss"], rtol=5e-5)
    go = torch.full((), 2.0, device=cuda)
    g = K_.pair_loss_bwd(mode, x, xp, ep, coef2, pref, float(d["beta"]), float(d["clip_eps"]), ws, grad_out=go,
                         grad_scale=0.5, out_dtype=torch.float32)
    g = g.reshape((P, 2) + d["x0"].shape[1:]).cpu().numpy()
    # fp32 kernel vs torch autograd through the reference step: agree to a few 1e-6 of the largest entry; the DMD2
    # t = 999 case multiplies the mean's rounding by sqrt(abar_prev) sqrt(1-abar_t) / sqrt(abar_t) = 3.4 (measured
    # 1.01e-5 of max once the step's products were made contraction-free), hence 2e-5
    for k in range(2):
        ref = d[f"grad_eps_pol{k}"]
        scale = max(np.abs(ref).max(), 1e-30)
        assert np.abs(g[:, k] - ref).max() <= 2e-5 * scale + 1e-12
