"""smoke(): one tiny PSO micro-step on cuda:0 checked against the oracle (oracle/ is the checker only)."""
import numpy as np
import torch


def run():
    assert torch.cuda.is_available(), "smoke() needs cuda:0"
    from oracle import pso_math as pm
    from oracle.schedulers import EulerAncestralTrailing
    from pairwise_sample_optimization_amd import pso_core
    dev = torch.device("cuda:0")
    s = EulerAncestralTrailing()
    s.set_timesteps(4)
    P, n_hw = 2, 16
    g = torch.Generator().manual_seed(0)
    shape = (2 * P, 4, n_hw, n_hw)
    x = torch.randn(shape, generator=g) * 14.6
    e_ref = torch.randn(shape, generator=g).bfloat16()
    e_pol = (e_ref.float() + 0.01 * torch.randn(shape, generator=g)).bfloat16()
    xp = torch.randn(shape, generator=g)
    t = torch.full((2 * P,), 999.0)
    coef = pso_core.turbo_coef(s.sigmas, s.timesteps, t)
    pref = torch.tensor([[1.0, -1.0], [-1.0, 1.0]])
    ep = e_pol.to(dev).requires_grad_(True)
    loss, lp = pso_core.pair_loss(ep, e_ref.to(dev), x.to(dev), xp.to(dev), coef, pref, 0, 50.0, 0.1)
    loss.backward()
    sig, su, dt = pm.turbo_coefs(s.sigmas.numpy(), s.timesteps.numpy(), t.numpy())
    lpp = pm.turbo_step_logprob(x.numpy(), e_pol.float().numpy(), sig, su, dt, prev=xp.numpy())[1]
    lpr = pm.turbo_step_logprob(x.numpy(), e_ref.float().numpy(), sig, su, dt, prev=xp.numpy())[1]
    L, _, _ = pm.pair_loss(lpp.reshape(P, 2), lpr.reshape(P, 2), pref.numpy(), 50.0, 0.1)
    np.testing.assert_allclose(lp[:, 0].cpu().numpy(), lpp, rtol=1e-6)
    np.testing.assert_allclose(loss.item(), L, rtol=1e-5)
    assert torch.isfinite(ep.grad.float()).all()
    print(f"smoke OK: loss={loss.item():.6f} oracle={L:.6f}")
