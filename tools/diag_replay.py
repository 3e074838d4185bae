"""Diagnostic (GPU): element-level comparison of the DMD2 bf16 replay step kernel with the numpy oracle on the
golden fixture, printing the intermediates of every mismatching element."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import pso_math as pm  # noqa: E402
from pairwise_sample_optimization_amd import kernels as K, pso_core  # noqa: E402

d = np.load("tests/golden/dmd_replay_bf16_P2_h16_t499.npz")
lat = torch.bfloat16
dev = torch.device("cuda")
coef = pso_core.dmd_coef(torch.from_numpy(d["alphas_cumprod"]), torch.from_numpy(d["t"]), torch.from_numpy(d["t_prev"]),
                         latent_dtype=lat).to(dev)
print("coef", coef.cpu().numpy(), [hex(v) for v in coef.cpu().numpy().view(np.uint32)[0, :4]])
print("np  ", [hex(v) for v in np.array([np.sqrt(np.float32(d["alphas_cumprod"][499])),
                                          np.sqrt(np.float32(1) - np.float32(d["alphas_cumprod"][499]))],
                                         np.float32).view(np.uint32)])
print("torch", torch.__version__, [hex(v) for v in torch.sqrt(1 - torch.tensor([d["alphas_cumprod"][499]])).numpy().view(np.uint32)],
      [hex(v) for v in ((1 - torch.tensor([d["alphas_cumprod"][499]])) ** 0.5).numpy().view(np.uint32)])
sa, sb, _, _ = pm.dmd_coefs(d["alphas_cumprod"], d["t"], d["t_prev"])
sa_p, sb_p, den, lstd = pm.dmd_coefs_latent(d["alphas_cumprod"], d["t_prev"], "bf16")
print("oracle", sa, sb, sa_p, sb_p, den, lstd)
rl = lambda v: pm.round_latent(v, "bf16")
for k in range(2):
    x = torch.from_numpy(d[f"x{k}"]).to(dev)
    e = torch.from_numpy(d[f"eps_ref{k}"]).to(dev)
    z = torch.from_numpy(d[f"noise{k}"]).to(dev)
    prev, lp = K.step_logprob(pso_core.dmd_mode(lat), x, e, coef, noise=z, noise_shared=True)
    g = prev.cpu().numpy()
    bad = np.argwhere(g != d[f"prev{k}"])
    print(k, "mismatches", len(bad))
    for idx in bad[:5]:
        i = tuple(idx)
        X, E, Z = d[f"x{k}"][i], d[f"eps_ref{k}"][i], d[f"noise{k}"][(0,) + i[1:]]
        b = i[0]
        x0f = (np.float32(X) - np.float32(sb[b]) * np.float32(E)) / np.float32(sa[b])
        x0 = rl(x0f)
        mean = rl(np.float32(sa_p[b]) * x0)
        pr = rl(mean + rl(np.float32(sb_p[b]) * np.float32(Z)))
        print(" idx", i, "x", X, "eps", E, "z", Z, "x0f", x0f, "x0", x0, "mean", mean, "oracle prev", pr,
              "ref prev", d[f"prev{k}"][i], "gpu prev", g[i])

# fp32 x0 of the failing element straight from the kernel: DMD mode, c2 = 1, zero noise -> prev = x0 (unrounded)
c = coef.clone()
c[:, 2] = 1.0
for k in range(2):
    x = torch.from_numpy(d[f"x{k}"]).to(dev)
    e = torch.from_numpy(d[f"eps_ref{k}"]).to(dev)
    prev, _ = K.step_logprob(1, x, e, c, noise=torch.zeros_like(x[:1]), noise_shared=True)
    g = prev.cpu().numpy()
    x0f = (d[f"x{k}"] - sb.reshape(-1, 1, 1, 1) * d[f"eps_ref{k}"]) / sa.reshape(-1, 1, 1, 1)
    bad = np.argwhere(g != x0f)
    print("fp32 x0 mismatches", k, len(bad), [(tuple(i), g[tuple(i)], x0f[tuple(i)]) for i in bad[:4]])
