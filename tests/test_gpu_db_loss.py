"""GPU parity of the fused DreamBooth PSO loss kernels (csrc/db_loss.hip) against the oracle restatement of
DB:1847-1935 (oracle/pso_math.py; parity unpinned beyond that restatement -- the DreamBooth trainer cannot be
imported here and ships no golden vectors)."""
import numpy as np
import pytest
import torch

from oracle import pso_math

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("loss_type", ["pso", "pso_db"])
@pytest.mark.parametrize("B,h,eps_bf16", [(1, 64, True), (2, 32, False), (3, 16, True)])
def test_db_loss_fwd_bwd_vs_oracle(cuda, loss_type, B, h, eps_bf16):
    from pairwise_sample_optimization_amd import kernels as K
    rng = np.random.default_rng(B * 100 + h)
    shape = (2 * B, 4, h, h)
    sig = rng.choice([14.614647, 4.081731, 1.612887, 0.693205], size=B).astype(np.float32)
    sigma = np.concatenate([sig, sig])
    x0 = rng.standard_normal(shape).astype(np.float32)
    noise = rng.standard_normal(shape).astype(np.float32)
    noisy = (x0 + noise * sigma[:, None, None, None]).astype(np.float32)
    eps = (noise + 0.05 * rng.standard_normal(shape)).astype(np.float32)
    eps_ref = (noise + 0.05 * rng.standard_normal(shape)).astype(np.float32)
    if eps_bf16:  # the kernel reads the UNet's bf16 output; give the oracle the same rounded values
        eps = torch.from_numpy(eps).bfloat16().float().numpy()
        eps_ref = torch.from_numpy(eps_ref).bfloat16().float().numpy()
    beta, nd, pw = (5.0, 0.1, 0.5) if loss_type == "pso_db" else (20.0, 0.1, 1.0)
    lt = K.DB_HINGE if loss_type == "pso_db" else K.DB_SIGMOID
    dt = torch.bfloat16 if eps_bf16 else torch.float32
    e = torch.from_numpy(eps).to(cuda, dt)
    er = torch.from_numpy(eps_ref).to(cuda, dt) if loss_type == "pso" else None
    nz, t, s = (torch.from_numpy(a).to(cuda) for a in (noisy, x0, sigma))
    ws = K.db_loss_ws(B, eps[0].size, cuda)
    loss, losses, logits = K.db_loss_fwd(lt, e, nz, t, s, beta, nd, pw, ws, eps_ref=er)
    deps = K.db_loss_bwd(lt, e, nz, t, s, beta, nd, pw, ws, grad_scale=0.5, out_dtype=torch.float32)
    rloss, rl, rlog = pso_math.db_loss(eps, noisy, x0, sigma, beta, nd, pw, loss_type, eps_ref)
    rg = 0.5 * pso_math.db_loss_deps(eps, noisy, x0, sigma, beta, nd, pw, loss_type, eps_ref)
    np.testing.assert_allclose(losses[:2 * B].cpu().numpy(), rl, rtol=2e-6)
    np.testing.assert_allclose(logits.cpu().numpy(), rlog, rtol=1e-4, atol=1e-6)
    assert abs(loss.item() - rloss) <= 2e-5 * abs(rloss) + 1e-7
    g = deps.cpu().numpy()
    assert np.abs(g - rg).max() <= 1e-4 * np.abs(rg).max() + 1e-12
