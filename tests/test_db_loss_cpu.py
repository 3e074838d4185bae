"""CPU checks of the DreamBooth PSO loss restatement (oracle/pso_math.py, DB:1847-1935) and its scheduler plumbing:
the analytic eps-gradient the HIP kernel implements against torch autograd of the same restated loss (float64), and
the Euler training sigmas / distilled timestep draw against SURVEY Appendix C."""
import numpy as np
import pytest
import torch

from oracle import pso_math


def _inputs(B, seed, spread=1.0):
    rng = np.random.default_rng(seed)
    shape = (2 * B, 4, 8, 8)
    sigma = rng.choice([14.614647, 4.081731, 1.612887, 0.693205], size=B).astype(np.float32)
    sigma = np.concatenate([sigma, sigma])  # instance and negative share the timestep (DB:1777 repeat(2))
    x0 = rng.standard_normal(shape).astype(np.float32)
    noise = rng.standard_normal(shape[:1 + 0] + shape[1:]).astype(np.float32)
    noisy = x0 + noise * sigma[:, None, None, None]
    eps = (noise + spread * 0.05 * rng.standard_normal(shape)).astype(np.float32)
    eps_ref = (noise + 0.05 * rng.standard_normal(shape)).astype(np.float32)
    return eps, eps_ref, noisy, x0, sigma


def _torch_loss(eps, eps_ref, noisy, x0, sigma, beta, nd, pw, loss_type):
    e = torch.tensor(eps, dtype=torch.float64, requires_grad=True)
    s = torch.tensor(sigma, dtype=torch.float64)[:, None, None, None]
    nz, t = torch.tensor(noisy, dtype=torch.float64), torch.tensor(x0, dtype=torch.float64)
    per = lambda pred: ((s ** -2.0) * (pred - t) ** 2).reshape(len(pred), -1).mean(1)
    lw, ll = per(e * (-s) + nz).chunk(2)
    md = lw - nd * ll
    if loss_type == "pso":
        rw, rl = per(torch.tensor(eps_ref, dtype=torch.float64) * (-s) + nz).chunk(2)
        logits = (rw - nd * rl) - md
        loss = -torch.nn.functional.logsigmoid(beta * logits).mean()
    else:
        logits = -md
        loss = torch.relu(1 - beta * logits).mean()
    loss = loss + pw * ll.mean()
    (g,) = torch.autograd.grad(loss, e)
    return loss.item(), g.numpy()


@pytest.mark.parametrize("loss_type", ["pso", "pso_db"])
@pytest.mark.parametrize("B,seed,spread", [(1, 0, 1.0), (3, 1, 4.0), (4, 2, 0.2)])
def test_db_loss_grad_matches_autograd(loss_type, B, seed, spread):
    eps, eps_ref, noisy, x0, sigma = _inputs(B, seed, spread)
    beta, nd, pw = (5.0, 0.1, 0.5) if loss_type == "pso_db" else (200.0, 0.1, 1.0)  # recipe / argparse defaults
    loss, _, logits = pso_math.db_loss(eps, noisy, x0, sigma, beta, nd, pw, loss_type, eps_ref)
    g = pso_math.db_loss_deps(eps, noisy, x0, sigma, beta, nd, pw, loss_type, eps_ref)
    tl, tg = _torch_loss(eps, eps_ref, noisy, x0, sigma, beta, nd, pw, loss_type)
    assert abs(loss - tl) <= 1e-6 * abs(tl) + 1e-9
    np.testing.assert_allclose(g, tg, rtol=1e-5, atol=1e-9 * np.abs(tg).max())
    if loss_type == "pso_db":  # the test data exercises both sides of the hinge somewhere in the sweep
        assert logits.shape == (B,)


def test_euler_training_sigmas_and_distilled_timesteps():
    from pairwise_sample_optimization_amd.schedulers import EulerDiscreteScheduler, db_distill_timesteps
    sch = EulerDiscreteScheduler()
    t = torch.tensor([999, 749, 499, 249])
    np.testing.assert_allclose(sch.sigma_at(t).numpy(), [14.614647, 4.081731, 1.612887, 0.693205], rtol=2e-6)
    assert float(sch.timesteps[0]) == 999.0 and float(sch.timesteps[-1]) == 0.0
    raw = torch.arange(0, 1000, 37)
    ts = db_distill_timesteps(raw)
    assert set(ts.tolist()) <= {249, 499, 749, 999}
    assert ts.tolist()[:4] == [249 + 250 * (r % 4) for r in raw.tolist()[:4]]
