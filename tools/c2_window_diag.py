"""Conditioning of the C2 window loss at 1024^2 (BASELINE configs[1]: turbo, N = 2, P = 2, gas 2, LoRA r = 32): how far
does ANY bf16 UNet forward move the window loss (T:844-850, beta = 50) from the fp32 one, per window and per choice of
the step inputs?

For each seeded window: our paired pass, the fp32 oracle and the torch-bf16 autocast oracle give eps_pol / eps_ref of
the 16 images once (forward only); the loss is then a cheap function of (x, x_next, eps, rewards), evaluated here for

  * the sampled window itself (x_next from our sampler, random rewards) -- tests/test_gpu_fullsize.py's window;
  * constructed transitions x_next = x + dt (eps_ref^X + a_k (eps_pol^X - eps_ref^X)) + s sigma_up xi per member k,
    X = the sampling path (ours / fp32), with the rewards random or favouring one member.

Prints per design the per-window loss rel error of ours and torch-bf16, their means, the Delta range and clip count.
usage (GPU): python tools/c2_window_diag.py [windows] [b_std]"""
import itertools
import math
import os
import sys
from types import SimpleNamespace

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import sdxl_ref  # noqa: E402
from pairwise_sample_optimization_amd import kernels as K  # noqa: E402
from pairwise_sample_optimization_amd.trainer import PSOTrainer, compute_time_ids  # noqa: E402
from pairwise_sample_optimization_amd.unet import UNet2DConditionModel, UNetConfig  # noqa: E402

LOG_SQRT_2PI = math.log(math.sqrt(2 * math.pi))


def lp_turbo(x, eps, prev, c):
    """DP/turbo_inference_with_logprob.py:69-114 per image, batched: x / eps / prev [n, ...], c [n, 8]."""
    sig, su, dt = c[:, 0], c[:, 1], c[:, 2]
    shp = (-1,) + (1,) * (x.dim() - 1)
    mean = x + eps * dt.view(shp)  # x + (x - (x - sig eps)) / sig * dt
    lp = -((prev - mean) ** 2) / (2 * su.view(shp) ** 2) - torch.log(su.view(shp)) - LOG_SQRT_2PI
    return lp.flatten(1).mean(1)


def pair_loss(lpp, lpr, pref, beta=50.0, eps=0.1):
    """T:844-850 on [P, 2] log-probs."""
    ratio = torch.clamp(torch.exp(lpp - lpr), 1 - eps, 1 + eps)
    return -torch.log(torch.sigmoid(beta * torch.log(ratio[:, 0]) * pref[:, 0] +
                                    beta * torch.log(ratio[:, 1]) * pref[:, 1])).mean()


def main():
    W = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    b_std = float(sys.argv[2]) if len(sys.argv) > 2 else 1.5e-2
    cuda = torch.device("cuda", 0)
    h, P, gas, N, r = 128, 2, 2, 2, 32
    cfg = UNetConfig.sdxl(h)
    with torch.device(cuda):
        unet = UNet2DConditionModel(cfg)
    unet.init_weights(0)
    unet.add_adapter(SimpleNamespace(r=r, lora_alpha=r))
    unet.lora.init_gaussian(seed=0, b_std=b_std)
    unet.prepare()
    tr = PSOTrainer(unet, mode="turbo", num_steps=N, gradient_accumulation_steps=gas, train_batch_size=P)
    tr.auto_step = False
    sd = sdxl_ref.sd_to(unet.state_dict(), cuda)
    lora = {k: v.float() for k, v in unet.lora.state_dict_peft().items()}
    sd16 = {k: v.bfloat16() for k, v in sd.items()}
    ocfg = dict(time_proj_dim=cfg.time_proj_dim, addition_time_embed_dim=cfg.addition_time_embed_dim)
    wins = []
    for w in range(W):
        g = torch.Generator(device="cuda").manual_seed(1000 + 17 * w)
        Bp = P * gas
        enc = torch.randn(Bp, 77, 2048, device=cuda, generator=g).bfloat16()
        pooled = torch.randn(Bp, 1280, device=cuda, generator=g).bfloat16()
        tid = compute_time_ids(1024, 0, cuda).repeat(Bp, 1)
        buf = tr.sample_pairs(enc, pooled, tid, h, generator=g,
                              reward_fn=lambda img: torch.rand(img.shape[0], device=cuda, generator=g))
        sb = tr.shuffle(buf, generator=g)
        mb = tr.micro_batch(sb, 0, sb.n_micro)
        n = mb.unet_in.shape[0]
        with torch.no_grad():
            eb, _ = unet.forward_nhwc(mb.unet_in, mb.t, mb.enc, mb.pooled, mb.tid, save=False, paired_ref=True)
            x_in = K.nhwc_to_nchw(mb.unet_in).float()

            def fwd(i, wts, lo):
                return sdxl_ref.unet_forward(wts, x_in[i:i + 1], mb.t[i:i + 1], mb.enc[i:i + 1].float(),
                                             mb.pooled[i:i + 1].float(), mb.tid[i:i + 1], lora=lo, cfg=ocfg)
            ep = torch.cat([fwd(i, sd, lora) for i in range(n)])
            er = torch.cat([fwd(i, sd, None) for i in range(n)])
            with torch.autocast("cuda", dtype=torch.bfloat16):
                ep16 = torch.cat([fwd(i, sd16, lora).float() for i in range(n)])
                er16 = torch.cat([fwd(i, sd16, None).float() for i in range(n)])
        q = lambda t: t.bfloat16().float()  # the step functions see fp32 eps holding bf16 values
        wins.append(SimpleNamespace(
            x=mb.x.permute(0, 3, 1, 2).contiguous(), xn=mb.x_next.permute(0, 3, 1, 2).contiguous(), c=mb.coef,
            rewards=mb.rewards,
            eps=dict(ours=(K.nhwc_to_nchw(eb[:n]), K.nhwc_to_nchw(eb[n:])), fp32=(q(ep), q(er)),
                     bf16=(q(ep16), q(er16)))))
        e_o = wins[-1].eps["ours"]
        print(f"window {w}: eps rel ours {((e_o[0] - q(ep)).norm() / ep.norm()).item():.2e} bf16 "
              f"{((q(ep16) - q(ep)).norm() / ep.norm()).item():.2e}; |delta|/|eps| "
              f"{((q(ep) - q(er)).norm() / ep.norm()).item():.3e}", flush=True)

    def evaluate(name, make_prev, orient):
        rows = []
        for wi, wd in enumerate(wins):
            prev = make_prev(wd, wi)
            n = wd.x.shape[0]
            if orient == "random":
                rw = wd.rewards
            else:
                rw = torch.zeros(n // 2, 2, 1, device=cuda)
                rw[:, 1 if orient == "m1" else 0] = 1.0
            pref = K.preference(rw, 0)
            res = {}
            for path, (e_p, e_r) in wd.eps.items():
                lpp = lp_turbo(wd.x, e_p, prev, wd.c).view(-1, 2)
                lpr = lp_turbo(wd.x, e_r, prev, wd.c).view(-1, 2)
                res[path] = (pair_loss(lpp, lpr, pref).item(), (lpp - lpr).reshape(-1))
            L32, D32 = res["fp32"]
            rows.append((abs(res["ours"][0] - L32) / abs(L32), abs(res["bf16"][0] - L32) / abs(L32), L32,
                         (res["ours"][1] - D32).norm().item() / max(D32.norm().item(), 1e-30),
                         (res["bf16"][1] - D32).norm().item() / max(D32.norm().item(), 1e-30),
                         D32.min().item(), D32.max().item(),
                         int(((D32 > math.log(1.1)) | (D32 < math.log(0.9))).sum().item())))
        ro = [r_[0] for r_ in rows]
        rb = [r_[1] for r_ in rows]
        print(f"{name:44s} loss rel ours mean {sum(ro) / len(ro):.2e} max {max(ro):.2e} | bf16 mean "
              f"{sum(rb) / len(rb):.2e} max {max(rb):.2e} | L32 {[round(r_[2], 4) for r_ in rows]} | Delta rel ours "
              f"{sum(r_[3] for r_ in rows) / len(rows):.2e} bf16 {sum(r_[4] for r_ in rows) / len(rows):.2e} | "
              f"Delta [{min(r_[5] for r_ in rows):.4f}, {max(r_[6] for r_ in rows):.4f}] clipped "
              f"{sum(r_[7] for r_ in rows)}", flush=True)
        print("    per window ours " + " ".join(f"{v:.2e}" for v in ro) + " | bf16 " +
              " ".join(f"{v:.2e}" for v in rb) + " | LoRA-off |log2 - L32| / L32 min " +
              f"{min(abs(math.log(2) - r_[2]) / r_[2] for r_ in rows):.2e}", flush=True)

    evaluate("sampled window (test design)", lambda wd, wi: wd.xn, "random")

    def split(name, make_prev):
        """lp errors of each path split by side (policy E_t / reference E_r) and by pair mode: the loss sees only the
        within-pair difference (member 0 - member 1) of E_t - E_r."""
        acc = {}
        for wi, wd in enumerate(wins):
            prev = make_prev(wd, wi)
            lp32 = [lp_turbo(wd.x, e, prev, wd.c) for e in wd.eps["fp32"]]
            for path in ("ours", "bf16"):
                lpP = [lp_turbo(wd.x, e, prev, wd.c) for e in wd.eps[path]]
                Et, Er = (lpP[0] - lp32[0]).view(-1, 2), (lpP[1] - lp32[1]).view(-1, 2)
                for nm, E in (("E_pol", Et), ("E_ref", Er), ("E_Delta", Et - Er)):
                    d = (E[:, 0] - E[:, 1]) / 2
                    cm = (E[:, 0] + E[:, 1]) / 2
                    a = acc.setdefault((path, nm), [0.0, 0.0, 0])
                    a[0] += (d ** 2).sum().item()
                    a[1] += (cm ** 2).sum().item()
                    a[2] += d.numel()
        print(f"  lp error split ({name}): " + "; ".join(
            f"{p_} {nm} diff {(v[0] / v[2]) ** 0.5:.2e} common {(v[1] / v[2]) ** 0.5:.2e}"
            for (p_, nm), v in sorted(acc.items())), flush=True)

    split("sampled window", lambda wd, wi: wd.xn)
    xi_cache = {}

    def constructed(a0, a1, s, X):
        def mk(wd, wi):
            if wi not in xi_cache:
                xi_cache[wi] = torch.randn(wd.x.shape, device=cuda,
                                           generator=torch.Generator(device="cuda").manual_seed(77 + wi))
            e_p, e_r = wd.eps[X]
            n = wd.x.shape[0]
            a = torch.tensor([a0, a1] * (n // 2), device=cuda).view(-1, 1, 1, 1)
            dt, su = wd.c[:, 2].view(-1, 1, 1, 1), wd.c[:, 1].view(-1, 1, 1, 1)
            return wd.x + dt * (e_r + a * (e_p - e_r)) + s * su * xi_cache[wi]
        return mk

    grid = itertools.product(("ours", "fp32"), ((1, 1), (1, 0), (0, 1), (1.5, -0.5), (2, -1), (1, -1), (0.5, 0.5)),
                             (1.0, 0.5, 0.25, 0.0), ("random", "m1", "m0"))
    if os.environ.get("C2_GRID") == "sat":  # member 0 saturates the clip, member 1 inside it
        grid = itertools.product(("fp32", "ours"), ((2.5, -0.5), (3, -0.5), (2.5, -0.25), (2.5, 0), (3, 0.25)),
                                 (0.0, 0.25, 0.5), ("m1",))
    if os.environ.get("C2_GRID") == "small":
        grid = itertools.product(("fp32",), ((1, 0), (1, -1), (1.5, -0.5)), (1.0, 0.5, 0.25, 0.0), ("m1", "m0"))
    split("X=fp32 a=(1,1) s=1", constructed(1, 1, 1.0, "fp32"))
    split("X=fp32 a=(1,1) s=0", constructed(1, 1, 0.0, "fp32"))
    if os.environ.get("C2_GRID") == "split":
        return
    for X, (a0, a1), s, orient in grid:
        evaluate(f"X={X} a=({a0},{a1}) s={s} {orient}", constructed(a0, a1, s, X), orient)


if __name__ == "__main__":
    main()
