"""Generate the PSO-math golden vectors in tests/golden/ from the REFERENCE's own step functions.

Runs only in the build container (needs /root/reference; never on the GPU box).  The two reference modules
`DP/turbo_inference_with_logprob.py` and `DP/distilled_inference_with_logprob.py` import diffusers only for type
hints and `randn_tensor`; diffusers is not installed, so a minimal in-process stub provides those names
(`randn_tensor` returns the pre-drawn noise tensor recorded in the fixture, so the sampling branch is pinned too).
The scheduler state they read (`.timesteps`, `.sigmas`, `.alphas_cumprod`) comes from oracle/schedulers.py.

Code that is inline in the trainers' main() cannot be imported; it is EXECUTED from the reference's own source lines
instead (`exec_ref`: the line range is read from the file, checked against an anchor string, dedented and run in a
namespace holding the names it reads -- plain torch, plus tiny stand-ins for `accelerator.device`, `config.train`,
`args` and the adapter toggles).  That covers the loss (`T:844-850`, `D:848-854`, differentiated with autograd),
`sample_compare` (`T:401-416`), `compare` (`D:420-434`), the per-epoch shuffle (`T:733-745`, `D:737-749`) and the
DreamBooth loss (`DB:1846-1935`).

Output: tests/golden/*.npz (allow_pickle=False loadable).
"""
import importlib.util
import os
import sys
import textwrap
import types

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from oracle.schedulers import EulerAncestralTrailing, LCMTable  # noqa: E402

REF = "/root/reference"
REF_DP = REF + "/human_preference_tuning/pso_pytorch/diffusers_patch"
REF_T = REF + "/human_preference_tuning/train_online_pso_sdxl_turbo.py"
REF_D = REF + "/human_preference_tuning/train_online_pso_sdxl_dmd2.py"
REF_DB = REF + "/personalization/train_pso_sdxl_turbo_dreambooth.py"
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


def exec_ref(path, first, last, anchor, ns):
    """Execute lines [first, last] (1-based, inclusive) of a reference source file in namespace ns and return ns.
    `anchor` must occur in the first line (guards against a moved range)."""
    with open(path) as f:
        lines = f.read().split("\n")[first - 1:last]
    assert anchor in lines[0], (path, first, lines[0])
    exec(compile(textwrap.dedent("\n".join(lines)), f"{path}:{first}-{last}", "exec"), ns)
    return ns


def _cfg(beta, eps):
    return types.SimpleNamespace(train=types.SimpleNamespace(beta=beta, eps=eps))


def ref_loss(lp0, lpr0, lp1, lpr1, pref, beta, eps, trainer="T"):
    """The reference's own loss lines, executed: `T:844-850` (turbo) or `D:848-854` (DMD2)."""
    path, first = (REF_T, 844) if trainer == "T" else (REF_D, 848)
    ns = dict(torch=torch, total_prob_0=lp0, total_ref_prob_0=lpr0, total_prob_1=lp1, total_ref_prob_1=lpr1,
              human_prefer=pref, config=_cfg(beta, eps))
    return exec_ref(path, first, first + 6, "ratio_0 = torch.clamp", ns)["loss"]


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


def emit_loss(out, lps, ep, P, rng, trainer="T"):
    beta, eps = float(out["beta"]), float(out["clip_eps"])
    # preferences from rewards via the trainers' own rules (fixtures of their own below); here just +-1 choices
    pref = torch.tensor(rng.choice([-1.0, 1.0], size=P).astype(np.float32))
    pref = torch.stack([pref, -pref], 1)
    loss = ref_loss(lps["pol0"], lps["ref0"], lps["pol1"], lps["ref1"], pref, beta, eps, trainer)
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


# ----------------------------------------------------------------------------------------------------------------------
# loss scalar stage at the clamp bounds / ties (T:844-850, D:848-854 executed)
# ----------------------------------------------------------------------------------------------------------------------
def _lp_hitting(ratio, lp_ref):
    """A float32 lp_pol near lp_ref + log(ratio) whose reference Δ = lp_pol - lp_ref gives torch.exp(Δ) == ratio (as
    float32) EXACTLY -- the median of every such float in the window, so a 1-ulp different exp still lands on it."""
    target = torch.tensor(ratio, dtype=torch.float32)
    c = torch.tensor(lp_ref + float(np.log(ratio)), dtype=torch.float32)
    hits = []
    x = c.clone()
    for _ in range(200):
        x = torch.nextafter(x, torch.tensor(-np.inf))
    for _ in range(400):
        d = x - torch.tensor(lp_ref, dtype=torch.float32)
        if torch.exp(d) == target:
            hits.append(float(x))
        x = torch.nextafter(x, torch.tensor(np.inf))
    assert hits, ratio
    return hits[len(hits) // 2]


def make_loss_boundary():
    """P = 8 pairs whose members sit exactly at exp(Δ) = 0.9f / 1.1f, at Δ = 0, inside, and beyond the bounds, with
    turbo (+-1) and DMD2 (including the (0, 0) tie) preferences; loss and dL/d lp_pol by autograd through the
    reference's own lines."""
    beta, eps = 50.0, 0.1
    # |lp| < 0.5: a float32 Δ grid fine enough (3e-8) that some Δ maps exactly onto 0.9f / 1.1f under exp
    lp_ref = np.array([[-0.38, -0.41], [-0.39, -0.40], [-0.37, -0.42], [-0.385, -0.395],
                       [-0.36, -0.43], [-0.38, -0.38], [-0.40, -0.39], [-0.41, -0.37]], np.float32)
    lo, hi = float(np.float32(1 - eps)), float(np.float32(1 + eps))
    lp_pol = lp_ref.copy()
    lp_pol[0, 0] = _lp_hitting(lo, float(lp_ref[0, 0]))      # exactly at 1 - eps
    lp_pol[0, 1] = _lp_hitting(hi, float(lp_ref[0, 1]))      # exactly at 1 + eps
    lp_pol[1, 0] = _lp_hitting(hi, float(lp_ref[1, 0]))
    lp_pol[1, 1] = lp_ref[1, 1] + np.float32(0.01)            # inside
    lp_pol[2, 0] = lp_ref[2, 0] - np.float32(0.3)             # below the clip
    lp_pol[2, 1] = _lp_hitting(lo, float(lp_ref[2, 1]))
    lp_pol[3] = lp_ref[3] + np.float32(0.2)                   # above the clip
    lp_pol[4, 0] = lp_ref[4, 0] + np.float32(-0.02)
    # row 5: Δ = 0 (policy == reference, the first step of a run: loss log 2)
    lp_pol[6, 0] = _lp_hitting(lo, float(lp_ref[6, 0]))
    lp_pol[6, 1] = lp_ref[6, 1] + np.float32(0.05)
    lp_pol[7, 1] = _lp_hitting(hi, float(lp_ref[7, 1]))
    out = {"beta": np.float32(beta), "clip_eps": np.float32(eps), "lp_pol": lp_pol, "lp_ref": lp_ref}
    pref_t = np.array([[-1, 1], [1, -1], [-1, 1], [1, -1], [-1, 1], [1, -1], [-1, 1], [1, -1]], np.float32)
    pref_d = pref_t.copy()
    pref_d[[1, 4]] = 0.0                                      # DMD2 strict-Pareto ties -> (0, 0)
    for tag, pref, trainer in (("turbo", pref_t, "T"), ("dmd", pref_d, "D")):
        lp = torch.tensor(lp_pol, requires_grad=True)
        lr = torch.tensor(lp_ref)
        loss = ref_loss(lp[:, 0], lr[:, 0], lp[:, 1], lr[:, 1], torch.tensor(pref), beta, eps, trainer)
        loss.backward()
        out[f"pref_{tag}"] = pref
        out[f"loss_{tag}"] = np.float32(loss.item())
        out[f"dlp_{tag}"] = lp.grad.numpy()
    return out


# ----------------------------------------------------------------------------------------------------------------------
# preferences: sample_compare (T:401-416) and compare (D:420-434) executed
# ----------------------------------------------------------------------------------------------------------------------
class _RecordingTorch(types.ModuleType):
    """`torch` for the executed sample_compare: records the reward indices its torch.randint draws."""

    def __init__(self):
        super().__init__("torch")
        self.drawn = []

    def __getattr__(self, k):
        return getattr(torch, k)

    def randint(self, *a, **kw):
        r = torch.randint(*a, **kw)
        self.drawn.append(r.clone())
        return r


def make_preferences():
    g = torch.Generator().manual_seed(7)
    out = {}
    rt = _RecordingTorch()
    ns = exec_ref(REF_T, 401, 416, "def sample_compare", {"torch": rt})
    for m in (1, 3):
        a = torch.rand((16, m), generator=g)
        b = torch.rand((16, m), generator=g)
        b[:4] = a[:4]                                         # ties: member 0 loses (a <= b)
        torch.manual_seed(100 + m)
        c = ns["sample_compare"](a, b)
        out[f"sc_a_m{m}"], out[f"sc_b_m{m}"] = a.numpy(), b.numpy()
        out[f"sc_idx_m{m}"] = rt.drawn[-1].numpy().astype(np.int64)
        out[f"sc_c_m{m}"] = c.numpy()
    nsd = exec_ref(REF_D, 420, 434, "def compare", {"torch": torch})
    for m in (1, 2):
        a = torch.randint(0, 3, (24, m), generator=g).float() / 2
        b = torch.randint(0, 3, (24, m), generator=g).float() / 2
        a_in, b_in = (a[:, 0], b[:, 0]) if m == 1 else (a, b)  # the 1-D branch (:422-424) for m = 1
        out[f"cmp_a_m{m}"], out[f"cmp_b_m{m}"] = a_in.numpy(), b_in.numpy()
        out[f"cmp_c_m{m}"] = nsd["compare"](a_in, b_in).numpy()
    return out


# ----------------------------------------------------------------------------------------------------------------------
# per-epoch shuffle (T:733-745 turbo, D:737-749 DMD2) executed
# ----------------------------------------------------------------------------------------------------------------------
def make_shuffle(trainer, Bp=6, T=3, hw=4, seed=21):
    g = torch.Generator().manual_seed(seed)
    lat = lambda: torch.randn((Bp, 2, T, 4, hw, hw), generator=g)
    orig = {"latents": lat(), "next_latents": lat(), "timesteps": torch.randint(0, 1000, (Bp, T), generator=g),
            "log_probs": torch.randn((Bp, 2, T), generator=g), "rewards": torch.rand((Bp, 2, 1), generator=g),
            "prompt_embeds": torch.randn((Bp, 2, 3, 5), generator=g)}
    if trainer == "T":
        orig["input_latents"] = lat()
    path, first, last = (REF_T, 733, 745) if trainer == "T" else (REF_D, 737, 749)
    torch.manual_seed(seed)
    ns = dict(torch=torch, accelerator=types.SimpleNamespace(device=torch.device("cpu")), total_batch_size=Bp,
              num_timesteps=T, orig_sample={k: v.clone() for k, v in orig.items()})
    exec_ref(path, first, last, "perm = torch.randperm", ns)
    out = {"perm": ns["perm"].numpy(), "perms": ns["perms"].numpy()}
    for k, v in orig.items():
        out["in_" + k] = v.numpy()
        out["out_" + k] = ns["samples"][k].numpy()
    return out


# ----------------------------------------------------------------------------------------------------------------------
# DreamBooth loss (DB:1846-1935) executed, for both loss types, with the EDM branch the scripts use
# ----------------------------------------------------------------------------------------------------------------------
def make_db_loss(loss_type, B=2, hw=8, seed=31, beta=5.0, neg=1.0, prior=1.0):
    g = torch.Generator().manual_seed(seed)
    shape = (2 * B, 4, hw, hw)
    model_input = torch.randn(shape, generator=g)             # the clean latents [instance; negative]
    sigmas = torch.tensor([14.6146, 4.0817, 1.6129, 0.6932][:2 * B], dtype=torch.float32).view(-1, 1, 1, 1)
    noise = torch.randn(shape, generator=g)
    noisy = model_input + noise * sigmas
    eps = bf16_round(torch.randn(shape, generator=g)).requires_grad_(True)
    eps_ref = bf16_round(eps.detach() + 0.05 * torch.randn(shape, generator=g))
    toggles = types.SimpleNamespace(disable_adapters=lambda: None, enable_adapters=lambda: None)
    ns = dict(torch=torch, F=torch.nn.functional, model_pred=eps, noisy_model_input=noisy, sigmas=sigmas,
              model_input=model_input, noise=noise, timesteps=None, prompt_embeds_input=None,
              unet_added_conditions=None, inp_noisy_latents=None, scheduler_type="EulerDiscreteScheduler",
              noise_scheduler=types.SimpleNamespace(config=types.SimpleNamespace(prediction_type="epsilon")),
              args=types.SimpleNamespace(do_edm_style_training=True, neg_defactor=neg, loss_type=loss_type,
                                         beta_pso=beta, prior_loss_weight=prior),
              accelerator=types.SimpleNamespace(unwrap_model=lambda m: toggles),
              unet=lambda *a, **kw: (eps_ref.clone(),))
    exec_ref(REF_DB, 1846, 1935, "weighting = None", ns)
    ns["loss"].backward()
    return {"loss_type": np.int32(0 if loss_type == "pso" else 1), "beta": np.float32(beta),
            "neg_defactor": np.float32(neg), "prior_w": np.float32(prior), "eps": eps.detach().numpy(),
            "eps_ref": eps_ref.numpy(), "noisy": noisy.numpy(), "x0": model_input.numpy(),
            "sigma": sigmas.reshape(-1).numpy(), "loss": np.float32(ns["loss"].item()),
            "model_losses": ns["model_losses"].detach().numpy(), "grad_eps": eps.grad.numpy()}


# ----------------------------------------------------------------------------------------------------------------------
# DMD2 latent-dtype replay (DP/distilled_inference_with_logprob.py on fp16 / bf16 latents) + the D:848-854 loss
# ----------------------------------------------------------------------------------------------------------------------
def make_dmd_replay(mod, dtype, P, hw, seed, t_int, beta=50.0, eps=0.1):
    g = torch.Generator().manual_seed(seed)
    sch = LCMTable()
    shape = (P, 4, hw, hw)
    t = torch.full((P,), t_int, dtype=torch.long)
    tp = t - 250
    out = {"latent": np.array("fp16" if dtype == torch.float16 else "bf16"), "beta": np.float32(beta),
           "clip_eps": np.float32(eps), "alphas_cumprod": sch.alphas_cumprod.numpy(), "t": t.numpy(),
           "t_prev": tp.numpy()}
    lps = {}
    for k in range(2):
        x = torch.randn(shape, generator=g).to(dtype)
        # accelerate's convert_outputs_to_fp32: fp32 eps holding reduced-precision values
        e_ref = torch.randn(shape, generator=g).to(dtype).float()
        e_pol = (e_ref + 0.02 * torch.randn(shape, generator=g)).to(dtype).float()
        noise = torch.randn((1,) + shape[1:], generator=g).to(dtype)
        _NOISE["t"] = noise
        prev, lp_sample = mod.distilled_step_with_logprob(sch, e_ref, t, tp, x, device=torch.device("cpu"))
        _NOISE["t"] = None
        assert prev.dtype == dtype and lp_sample.dtype == dtype
        _, lps[f"pol{k}"] = mod.distilled_step_with_logprob(sch, e_pol, t, tp, x, prev_sample=prev,
                                                            device=torch.device("cpu"))
        _, lps[f"ref{k}"] = mod.distilled_step_with_logprob(sch, e_ref, t, tp, x, prev_sample=prev,
                                                            device=torch.device("cpu"))
        out.update({f"x{k}": x.float().numpy(), f"eps_pol{k}": e_pol.numpy(), f"eps_ref{k}": e_ref.numpy(),
                    f"noise{k}": noise.float().numpy(), f"prev{k}": prev.float().numpy(),
                    f"lp_sample{k}": lp_sample.float().numpy(), f"lp_pol{k}": lps[f"pol{k}"].float().numpy(),
                    f"lp_ref{k}": lps[f"ref{k}"].float().numpy()})
    pref = torch.tensor([[-1.0, 1.0], [1.0, -1.0], [0.0, 0.0]][:P])
    loss = ref_loss(lps["pol0"], lps["ref0"], lps["pol1"], lps["ref1"], pref, beta, eps, "D")
    out.update({"pref": pref.numpy(), "loss": np.float32(loss.item())})
    return out


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
        emit_loss(out, lps, ep, P, rng, trainer="D")
        name = f"pso_dmd_P{P}_h{hw}_t{tt}_seed{seed}.npz"
        np.savez_compressed(os.path.join(OUT, name), **out)
        cases.append(name)
    extra = {"loss_boundary.npz": make_loss_boundary(), "preferences.npz": make_preferences(),
             "shuffle_turbo.npz": make_shuffle("T"), "shuffle_dmd.npz": make_shuffle("D"),
             "db_loss_pso.npz": make_db_loss("pso"), "db_loss_pso_db.npz": make_db_loss("pso_db"),
             "dmd_replay_fp16_P2_h16_t999.npz": make_dmd_replay(dmd, torch.float16, 2, 16, 41, 999),
             "dmd_replay_fp16_P3_h16_t749.npz": make_dmd_replay(dmd, torch.float16, 3, 16, 42, 749),
             "dmd_replay_bf16_P2_h16_t499.npz": make_dmd_replay(dmd, torch.bfloat16, 2, 16, 43, 499)}
    for name, out in extra.items():
        np.savez_compressed(os.path.join(OUT, name), **out)
        cases.append(name)
    print("\n".join(cases))


if __name__ == "__main__":
    main()
