"""Generate the PSO-math golden vectors in tests/golden/ from the REFERENCE's own step functions.

Runs only in the build container (needs /root/reference; never on the GPU box).  The two reference modules
`DP/turbo_inference_with_logprob.py` and `DP/distilled_inference_with_logprob.py` import diffusers only for type
hints and `randn_tensor`; diffusers is not installed, so a minimal in-process stub provides those names
(`randn_tensor` returns the pre-drawn noise tensor recorded in the fixture, so the sampling branch is pinned too).
The scheduler state they read (`.timesteps`, `.sigmas`, `.alphas_cumprod`) comes from oracle/schedulers.py.

The loss is inline in the trainers' main() (`T:844-850`, `D:848-854`) and cannot be imported; it is restated below
verbatim in torch and differentiated with autograd to give dL/d eps_theta through the reference step functions.

Output: tests/golden/pso_*.npz (allow_pickle=False loadable).
"""
import importlib.util
import os
import sys
import types

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from oracle.schedulers import EulerAncestralTrailing, LCMTable  # noqa: E402

REF_DP = "/root/reference/human_preference_tuning/pso_pytorch/diffusers_patch"
OUT = os.path.join(REPO, "tests", "golden")

_NOISE = {"t": None}


def _install_stub():
    def randn_tensor(shape, generator=None, device=None, dtype=None, layout=None):
        n = _NOISE["t"]
        assert n is not None and tuple(n.shape) == tuple(shape), (shape, None if n is None else n.shape)
        return n.to(dtype=dtype)

    class _Dummy:  # type-hint-only names
        pass

    mods = {
        "diffusers": {"DDPMScheduler": _Dummy},
        "diffusers.utils": {},
        "diffusers.utils.torch_utils": {"randn_tensor": randn_tensor},
        "diffusers.schedulers": {},
        "diffusers.schedulers.scheduling_euler_ancestral_discrete": {"EulerAncestralDiscreteScheduler": _Dummy},
        "diffusers.schedulers.scheduling_ddim": {"DDIMSchedulerOutput": _Dummy, "DDIMScheduler": _Dummy},
    }
    for name, attrs in mods.items():
        m = types.ModuleType(name)
        for k, v in attrs.items():
            setattr(m, k, v)
        sys.modules[name] = m


def _load(fname, modname):
    spec = importlib.util.spec_from_file_location(modname, os.path.join(REF_DP, fname))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def ref_loss(lp0, lpr0, lp1, lpr1, pref, beta, eps):
    """Verbatim restatement of `T:844-850` (identical text in `D:848-854`)."""
    ratio_0 = torch.clamp(torch.exp(lp0 - lpr0), 1 - eps, 1 + eps)
    ratio_1 = torch.clamp(torch.exp(lp1 - lpr1), 1 - eps, 1 + eps)
    return -torch.log(torch.sigmoid(
        beta * (torch.log(ratio_0)) * pref[:, 0] +
        beta * (torch.log(ratio_1)) * pref[:, 1]
    )).mean()


def bf16_round(x):
    return x.to(torch.bfloat16).to(torch.float32)


def make_turbo(mod, N, P, hw, seed, step, beta=50.0, eps=0.1, scale_eps=1.0):
    g = torch.Generator().manual_seed(seed)
    sch = EulerAncestralTrailing()
    sch.set_timesteps(N)
    shape = (P, 4, hw, hw)
    t = sch.timesteps[step].repeat(P)
    sig = sch.sigmas[step]
    out = {"mode": np.int32(0), "N": np.int32(N), "step": np.int32(step), "beta": np.float32(beta),
           "clip_eps": np.float32(eps), "timesteps": sch.timesteps.numpy(), "sigmas": sch.sigmas.numpy(),
           "t": t.numpy()}
    # member k in {0,1}: sample x, eps_theta (bf16-valued fp32), eps_ref, prev
    for k in range(2):
        x = torch.randn(shape, generator=g) * float(sig)
        e_ref = bf16_round(torch.randn(shape, generator=g))
        e_pol = bf16_round(e_ref + scale_eps * 0.004 * torch.randn(shape, generator=g))
        noise = torch.randn(shape, generator=g)
        # sampling branch through the reference (records prev_sample = mean + noise * sigma_up)
        _NOISE["t"] = noise
        prev, lp_sample = mod.turbo_step_with_logprob(sch, e_ref, t, x, generator=None, device=torch.device("cpu"))
        _NOISE["t"] = None
        out.update({f"x{k}": x.numpy(), f"eps_pol{k}": e_pol.numpy(), f"eps_ref{k}": e_ref.numpy(),
                    f"noise{k}": noise.numpy(), f"prev{k}": prev.numpy(), f"lp_sample{k}": lp_sample.numpy()})
    return out, sch, t


def finish_loss_turbo(mod, out, sch, t, P):
    beta, eps = float(out["beta"]), float(out["clip_eps"])
    lps = {}
    grads = {}
    ep = [torch.tensor(out[f"eps_pol{k}"], requires_grad=True) for k in range(2)]
    for k in range(2):
        x = torch.tensor(out[f"x{k}"])
        prev = torch.tensor(out[f"prev{k}"])
        _, lps[f"pol{k}"] = mod.turbo_step_with_logprob(sch, model_output=ep[k], timestep=t, sample=x,
                                                        prev_sample=prev)
        _, lps[f"ref{k}"] = mod.turbo_step_with_logprob(sch, model_output=torch.tensor(out[f"eps_ref{k}"]),
                                                        timestep=t, sample=x, prev_sample=prev)
    return lps, ep


def emit_loss(out, lps, ep, P, rng):
    beta, eps = float(out["beta"]), float(out["clip_eps"])
    # preferences from rewards via the trainers' own rules (restated in oracle; here just +-1 choices)
    pref = torch.tensor(rng.choice([-1.0, 1.0], size=P).astype(np.float32))
    pref = torch.stack([pref, -pref], 1)
    loss = ref_loss(lps["pol0"], lps["ref0"], lps["pol1"], lps["ref1"], pref, beta, eps)
    loss.backward()
    out.update({"pref": pref.numpy(), "loss": np.float32(loss.item()),
                "lp_pol": torch.stack([lps["pol0"], lps["pol1"]], 1).detach().numpy(),
                "lp_ref": torch.stack([lps["ref0"], lps["ref1"]], 1).detach().numpy(),
                "grad_eps_pol0": ep[0].grad.numpy(), "grad_eps_pol1": ep[1].grad.numpy()})


def make_dmd(mod, P, hw, seed, t_int, beta=50.0, eps=0.1, scale_eps=1.0):
    g = torch.Generator().manual_seed(seed)
    sch = LCMTable()
    shape = (P, 4, hw, hw)
    t = torch.full((P,), t_int, dtype=torch.long)
    tp = t - 250
    out = {"mode": np.int32(1), "beta": np.float32(beta), "clip_eps": np.float32(eps),
           "alphas_cumprod": sch.alphas_cumprod.numpy(), "t": t.numpy(), "t_prev": tp.numpy()}
    ep = []
    lps = {}
    for k in range(2):
        x = torch.randn(shape, generator=g)
        e_ref = bf16_round(torch.randn(shape, generator=g))
        e_pol = bf16_round(e_ref + scale_eps * 0.004 * torch.randn(shape, generator=g))
        noise = torch.randn((1,) + shape[1:], generator=g)  # batch-shared noise, DP/distilled...:123-126
        _NOISE["t"] = noise
        prev, lp_sample = mod.distilled_step_with_logprob(sch, e_ref, t, tp, x, device=torch.device("cpu"))
        _NOISE["t"] = None
        out.update({f"x{k}": x.numpy(), f"eps_pol{k}": e_pol.numpy(), f"eps_ref{k}": e_ref.numpy(),
                    f"noise{k}": noise.numpy(), f"prev{k}": prev.numpy(), f"lp_sample{k}": lp_sample.numpy()})
        e = torch.tensor(e_pol.numpy(), requires_grad=True)
        ep.append(e)
        _, lps[f"pol{k}"] = mod.distilled_step_with_logprob(sch, e, t, tp, x, prev_sample=prev,
                                                            device=torch.device("cpu"))
        _, lps[f"ref{k}"] = mod.distilled_step_with_logprob(sch, e_ref, t, tp, x, prev_sample=prev,
                                                            device=torch.device("cpu"))
    return out, lps, ep


def main():
    _install_stub()
    turbo = _load("turbo_inference_with_logprob.py", "ref_turbo_step")
    dmd = _load("distilled_inference_with_logprob.py", "ref_dmd_step")
    os.makedirs(OUT, exist_ok=True)
    rng = np.random.default_rng(1234)
    cases = []
    for (N, P, hw, seed, step, scale) in [(4, 1, 16, 0, 0, 1.0), (4, 2, 16, 1, 1, 1.0), (4, 2, 16, 2, 2, 1.0),
                                          (2, 2, 32, 3, 0, 1.0), (4, 2, 16, 4, 0, 40.0)]:
        out, sch, t = make_turbo(turbo, N, P, hw, seed, step, scale_eps=scale)
        lps, ep = finish_loss_turbo(turbo, out, sch, t, P)
        emit_loss(out, lps, ep, P, rng)
        name = f"pso_turbo_N{N}_P{P}_h{hw}_s{step}_seed{seed}.npz"
        np.savez_compressed(os.path.join(OUT, name), **out)
        cases.append(name)
    for (P, hw, seed, tt, scale) in [(1, 16, 10, 999, 1.0), (2, 16, 11, 749, 1.0), (2, 32, 12, 499, 1.0),
                                      (2, 16, 13, 749, 40.0)]:
        out, lps, ep = make_dmd(dmd, P, hw, seed, tt, scale_eps=scale)
        emit_loss(out, lps, ep, P, rng)
        name = f"pso_dmd_P{P}_h{hw}_t{tt}_seed{seed}.npz"
        np.savez_compressed(os.path.join(OUT, name), **out)
        cases.append(name)
    print("\n".join(cases))


if __name__ == "__main__":
    main()
