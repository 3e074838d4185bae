"""PSO train-step throughput on MI355X (BASELINE.json metric: "PSO train-step imgs/sec (paired 1024^2 SDXL)").

Workload (BASELINE.json configs[1]): SDXL-Turbo PSO, bf16, 1024x1024 (128x128 latents), 2-step
sampler (T = 1 trained transition; a literal 1-step sampler trains nothing), LoRA r=32 grads only,
2 pairs per micro-step per GPU, gradient_accumulation_steps 2 (the turbo config default).  One bench "step" = one
optimizer step = gas*T micro-steps (+ the per-inner-epoch buffer shuffle, RCCL all-reduce, clip, and the 8-bit
AdamW of the reference default config -- --adam32 for fp32 AdamW); each micro-step trains 2P images (2P policy UNet
fwd+bwd + 2P reference fwd + fused loss).  Synthetic data: random-init
SDXL weights (seeded), N(0,1) text embeddings, trajectories from this build's own sampler (untimed), U(0,1)
rewards.  Multi-GPU: one process per GPU, pure data parallel (weak scaling); the LoRA gradient is all-reduced over RCCL in
~32 MB buckets issued during the backward of the window's last micro-step (GradBuckets), overlapped with it.

Secondary objects on the same JSON line (never the headline value):
  "c3"        BASELINE configs[2] on this GPU: SDXL-DMD2 PSO, 4-step sampler (T = 3), full-UNet grads against a frozen
              reference UNet, 1 pair per micro-step -- its own warmed-up, timed steps + dominant-kernel roofline;
  "lora_bs1"  the north-star operating point "bs = 1 / GPU": the C2 LoRA step at 1 pair, gas 1 (one micro-step =
              2 policy + 2 reference images in one paired pass);
  "dmd_lora"  the reference's own DMD2 recipe (config_sdxl_dmd_dpo.py: LoRA r=16, T=3, gas 4) at 1024^2;
  "turbo_ref" the reference's own Turbo recipe (config_sdxl_turbo_dpo.py: LoRA r=32, T=3, 4 pairs, gas 2) at 512^2;
  "c5"        BASELINE configs[4] on this GPU: the DreamBooth PSO micro-step (1 instance + 1 negative, r = 16, VAE
              encode in the step), bf16 and with the fp8 forward, and their ratio;
  "vae"       the reward-image VAE decode (8 latents -> 8 images at 1024^2) alone: ms, TF/s, GEMM-family roofline;
  "dist"      (N > 1) the backend and world size torch.distributed really runs, every rank's ms/step, and the
              bucketed all-reduce: bytes on the wire, its time alone, and the part of it left exposed after the
              backward (the rest ran under the backward).
  The config objects run at N = 1 only (--no-extra skips them).

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]
  Under torchrun (RANK / WORLD_SIZE / LOCAL_RANK set) every process is one rank.  Started directly with --gpus N > 1,
  bench.py launches `python -m torch.distributed.run --nproc-per-node N ... bench.py` as a child BEFORE any GPU call
  and exits with its code, so both launch forms measure N GPUs.
"""
import argparse
import glob
import json
import os
import socket
import subprocess
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PEAK_BF16_TFLOPS = 2500.0   # MI355X dense bf16 MFMA (MI355X_MICROARCH.md chip table)
SURVEY_TFLOP_PER_PAIR_MICRO = {32: 42.54, 16: 42.29}  # LoRA @1024^2, excludes checkpoint recompute


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--pairs", type=int, default=2)
    ap.add_argument("--gas", type=int, default=2)
    ap.add_argument("--res", type=int, default=1024)
    ap.add_argument("--rank", type=int, default=32)
    ap.add_argument("--num-steps", type=int, default=2)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-roofline", action="store_true")
    ap.add_argument("--epochs", type=int, default=2,
                    help="timed full epochs (sampling + VAE decode + PickScore + training) for the secondary metric; "
                         "0 skips it")
    ap.add_argument("--graph", action="store_true",
                    help="replay each epoch as one captured hipGraph (measured neutral: 31.32 vs 31.36 imgs/s eager)")
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--mode", default="turbo", choices=["turbo", "dmd"])
    ap.add_argument("--full-unet", action="store_true",
                    help="train every UNet parameter against a frozen reference UNet (BASELINE C3 / C4; use with "
                         "--mode dmd --num-steps 4 --pairs 1 --gas 1)")
    ap.add_argument("--adam32", action="store_true",
                    help="fp32 AdamW instead of the reference default 8-bit AdamW (config use_8bit_adam = True)")
    ap.add_argument("--allreduce", default="fp32", choices=["auto", "fp32", "bf16"],
                    help="gradient all-reduce wire dtype (fp32 accumulation and optimizer either way): auto = bf16 for "
                         "the full-UNet gradient (C3 / C4), fp32 for the LoRA bucket (DESIGN.md §6)")
    ap.add_argument("--allreduce-bf16", action="store_true", help="alias of --allreduce bf16")
    ap.add_argument("--cpu-timed", type=int, default=3, help="timed CPU-baseline samples after one warm-up")
    ap.add_argument("--no-extra", action="store_true", help="skip the c3 / lora_bs1 / c5 secondary objects")
    ap.add_argument("--extra-steps", type=int, default=3)
    return ap.parse_args()


def log(*a):
    if int(os.environ.get("RANK", "0")) == 0:
        print(*a, file=sys.stderr, flush=True)


def build(args, dev):
    from types import SimpleNamespace
    from pairwise_sample_optimization_amd.unet import UNet2DConditionModel, UNetConfig
    from pairwise_sample_optimization_amd.trainer import PSOTrainer, compute_time_ids
    h = args.res // 8
    with torch.device(dev):
        unet = UNet2DConditionModel(UNetConfig.sdxl(h))
    unet.init_weights(0)  # same frozen weights on every rank
    ref_unet = None
    if args.full_unet:  # C3 / C4: every parameter trained, the reference is a frozen copy of the initial UNet
        with torch.device(dev):
            ref_unet = UNet2DConditionModel(UNetConfig.sdxl(h))
        ref_unet.init_weights(0)
        ref_unet.prepare()
        unet.enable_full_grads()
    else:
        unet.add_adapter(SimpleNamespace(r=args.rank, lora_alpha=args.rank))
        unet.lora.init_gaussian(seed=0, b_std=1e-3)  # non-zero B so policy != reference
    unet.prepare()
    tr = PSOTrainer(unet, mode=args.mode, num_steps=args.num_steps, gradient_accumulation_steps=args.gas,
                    train_batch_size=args.pairs, num_reward=1, ref_unet=ref_unet,
                    allreduce_dtype=wire_dtype(args),
                    use_8bit_adam=not getattr(args, "adam32", False))  # the reference default (T:427-435)
    g = torch.Generator(device=dev).manual_seed(1000 + int(os.environ.get("RANK", "0")))
    Bp = args.pairs * args.gas  # pairs sampled per epoch per GPU
    enc = torch.randn(Bp, 77, 2048, device=dev, generator=g).bfloat16()
    pooled = torch.randn(Bp, 1280, device=dev, generator=g).bfloat16()
    tid = compute_time_ids(args.res, 0, dev).repeat(Bp, 1)
    reward = lambda img: torch.rand(img.shape[0], device=dev, generator=g)
    buf = tr.sample_pairs(enc, pooled, tid, h, generator=g, reward_fn=reward)
    return unet, tr, buf, g


def wire_dtype(args):
    if getattr(args, "allreduce_bf16", False):
        return torch.bfloat16
    return {"auto": "auto", "fp32": torch.float32, "bf16": torch.bfloat16}[getattr(args, "allreduce", "fp32")]


def one_step(tr, buf, g, graph=False):
    """shuffle (eager: a few gathers) + one epoch; graph=True replays the epoch's captured hipGraph."""
    sb = tr.shuffle(buf, generator=g)
    if graph:
        tr.train_epoch_graph(sb)
    else:
        tr.train_epoch(sb)


def src_hash():
    """Hash of the HIP sources the library is built from: a PMC traffic file is used only for the code it measured."""
    import hashlib
    h = hashlib.sha256()
    for f in sorted(glob.glob(os.path.join(ROOT, "pairwise_sample_optimization_amd", "csrc", "*.hip")) +
                    glob.glob(os.path.join(ROOT, "pairwise_sample_optimization_amd", "csrc", "*.h"))):
        h.update(open(f, "rb").read())
    return h.hexdigest()[:16]


def roofline(tr, buf, g):
    """One extra profiled step with HIP events around every GEMM-family launch (on torch's current stream = the
    launch stream), grouped by the launched kernel (pso_last_kernel).  The roofline is the DOMINANT kernel's (most
    time per step): achieved = its algorithmic 2*M*N*K flop per launch / its average launch duration.  The whole
    family is reported beside it.  traffic = HBM bytes per launch of that kernel from the two PMC passes
    (tools/gpu_full.sh -> tools/parse_prof.py), used only when they were collected on these exact sources."""
    return family_roofline(lambda: one_step(tr, buf, g))


def family_roofline(fn):
    """roofline() of any callable: fn runs once with every GEMM-family launch timed by its own HIP event pair."""
    from collections import defaultdict
    from pairwise_sample_optimization_amd import kernels as K
    K.PROFILE = []
    side, K.SideStream.enabled_any = K.SideStream.enabled_any, False  # serial launches: each event pair times one kernel
    fn()
    torch.cuda.synchronize()
    rec, K.PROFILE = K.PROFILE, None
    K.SideStream.enabled_any = side
    per = defaultdict(lambda: [0, 0.0, 0.0, 0.0])  # kernel -> launches, flop, bytes, ms
    for fl, nb, e0, e1, _tag, kname in rec:
        a = per[kname]
        a[0] += 1
        a[1] += fl
        a[2] += nb
        a[3] += e0.elapsed_time(e1)
    dom, (n, fl, nb, ms) = max(per.items(), key=lambda kv: kv[1][3])
    achieved = fl / (ms * 1e-3) / 1e12
    n_all, fl_all, ms_all = len(rec), sum(v[1] for v in per.values()), sum(v[3] for v in per.values())
    out = {"bound": "mfma", "kernel": dom, "achieved": round(achieved, 1), "peak": PEAK_BF16_TFLOPS,
           "unit": "TFLOP/s", "frac": round(achieved / PEAK_BF16_TFLOPS, 4), "traffic": None,
           "launches_per_step": n, "flop_per_launch": fl / n, "bytes_per_launch": nb / n,
           "avg_launch_us": round(ms * 1e3 / n, 2), "share_of_family_time": round(ms / ms_all, 3),
           "family": {"kernels": "every GEMM / implicit-GEMM conv / LoRA rank-product launch of one train step",
                      "launches_per_step": n_all, "achieved": round(fl_all / (ms_all * 1e-3) / 1e12, 1),
                      "frac": round(fl_all / (ms_all * 1e-3) / 1e12 / PEAK_BF16_TFLOPS, 4),
                      "ms_per_step": round(ms_all, 2)}}
    sh = src_hash()
    for tp in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_traffic.json")), reverse=True):
        t = json.load(open(tp))
        if t.get("src_hash") == sh and t.get("kernel") == dom:
            out["traffic"] = round(t["traffic_bytes_per_launch"])
            out["traffic_unit"] = "bytes/launch (PMC FETCH_SIZE*2 + WRITE_SIZE, gfx950 correction)"
            out["traffic_source"] = os.path.relpath(tp, ROOT)
            break
    else:
        out["traffic_note"] = f"no PMC pass on these sources (src {sh}) for {dom}"
    out["src_hash"] = sh
    return out


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform
    return platform.processor() or "unknown"


def cpu_baseline(args, unet):
    """Oracle (plain torch fp32 CPU restatement, oracle/sdxl_ref.py) on a bounded sample of the same workload: the
    per-image share of one micro-step at 1024^2 = 1 policy forward + LoRA backward + 1 reference forward (BASELINE.md
    §3: one warm-up, then >= 3 timed samples; the median is the value, the CPU model and thread count beside it)."""
    from oracle import sdxl_ref
    torch.set_num_threads(args.cpu_threads)
    sd = {k: v.float().cpu() for k, v in unet.state_dict().items()}
    lora = {k: v.float().cpu().requires_grad_(True) for k, v in unet.lora.state_dict_peft().items()}
    h = args.res // 8
    gen = torch.Generator().manual_seed(0)
    x = torch.randn(1, 4, h, h, generator=gen)
    t = torch.tensor([999.0])
    enc = torch.randn(1, 77, 2048, generator=gen)
    pooled = torch.randn(1, 1280, generator=gen)
    tid = torch.tensor([[args.res, args.res, 0, 0, args.res, args.res]], dtype=torch.float32)

    def share():
        out = sdxl_ref.unet_forward(sd, x, t, enc, pooled, tid, lora=lora)
        out.sum().backward()
        with torch.no_grad():
            sdxl_ref.unet_forward(sd, x, t, enc, pooled, tid, lora=None)
        for v in lora.values():
            v.grad = None

    t0 = time.perf_counter()
    share()  # warm-up: allocator, thread pool, first-touch of the fp32 weights
    warm = time.perf_counter() - t0
    times = []
    for _ in range(max(1, args.cpu_timed)):
        t0 = time.perf_counter()
        share()
        times.append(time.perf_counter() - t0)
    del sd, lora
    med = sorted(times)[len(times) // 2]
    return {"value": round(1.0 / med, 5), "unit": "imgs/s", "cores": args.cpu_threads, "kind": "port",
            "cpu_model": cpu_model(), "host_cpus": os.cpu_count(), "warmup_s": round(warm, 2),
            "timed_s": [round(v, 2) for v in times],
            "sample": f"1 image at {args.res}^2: policy fwd + LoRA bwd + reference fwd, fp32 torch oracle "
                      f"(oracle/sdxl_ref.py); 1 warm-up + {len(times)} timed, median {med:.1f} s"}


def skipped_ref_prefix_tflop(h):
    """TFLOP per reference image the paired pass never executes: the adapter-free prefix (conv_in, down_blocks.0's
    two resnets and downsampler) runs once on the policy images and is duplicated."""
    m0, m1 = h * h, (h // 2) * (h // 2)
    c = 320
    fl = 2 * m0 * c * 4 * 9 + 4 * 2 * m0 * c * c * 9 + 2 * m1 * c * c * 9
    return fl / 1e12


SDXL_FWD_TFLOP_PER_IMG = 6.765   # one UNet forward at 1024^2
SURVEY_TFLOP_FULL_UNET = 54.10   # one pair-micro-step with full-UNet grads at 1024^2
VAE_DEC_TFLOP_PER_IMG = 10.49    # AutoencoderKL.decode at 1024^2


def epoch_metric(args, dev, tr, buf, g, n_epochs):
    """Secondary metric (SURVEY §8d "epoch imgs/s"): one full online epoch = paired sampling of P*gas prompts (N UNet
    forwards over both trajectories of every prompt, batched) -> VAE decode of the final latents -> PickScore reward
    (ViT-H/14 on the GPU-preprocessed images; random-init weights, random prompt ids) -> shuffle -> training epoch
    (the timed step above).  value = trained images / wall time of the whole epoch."""
    from pairwise_sample_optimization_amd.vae import AutoencoderKL, VAEConfig
    from pairwise_sample_optimization_amd.pso_pytorch.pickscore_utils import Selector
    from pairwise_sample_optimization_amd.rewards import pickscore_reward
    h = args.res // 8
    with torch.device(dev):
        vae = AutoencoderKL(VAEConfig())
    vae.init_weights(0)
    vae.prepare()
    sel = Selector(dev, seed=0)
    Bp = args.pairs * args.gas
    ids = torch.randint(1, 49406, (Bp, 77), device=dev, generator=g)
    ids[:, 0], ids[:, 20:] = 49406, 49407
    reward = pickscore_reward(sel, ids.repeat_interleave(2, 0))
    enc, pooled, tid = buf["enc"][::2].contiguous(), buf["pooled"][::2].contiguous(), buf["tid"][::2].contiguous()

    def epoch():
        b = tr.sample_pairs(enc, pooled, tid, h, generator=g, reward_fn=reward, decode_fn=vae.decode_latents_nhwc)
        one_step(tr, b, g)

    epoch()
    torch.cuda.synchronize()
    if dist.is_initialized():
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(n_epochs):
        epoch()
    torch.cuda.synchronize()
    if dist.is_initialized():
        dist.barrier()
    dt = max_over_ranks(time.perf_counter() - t0, dev) / n_epochs
    world = dist.get_world_size() if dist.is_initialized() else 1
    n_img = 2 * Bp
    trained = n_img * (args.num_steps - 1)
    tf = None
    if args.res == 1024 and not args.full_unet and args.rank in SURVEY_TFLOP_PER_PAIR_MICRO:
        tf = (args.num_steps * n_img * SDXL_FWD_TFLOP_PER_IMG + n_img * VAE_DEC_TFLOP_PER_IMG
              + SURVEY_TFLOP_PER_PAIR_MICRO[args.rank] * Bp * (args.num_steps - 1))
    out = {"imgs_per_s": round(trained * world / dt, 3), "ms_per_epoch": round(dt * 1e3, 1), "epochs": n_epochs,
           "sampled_images": n_img * world, "reward": "PickScore ViT-H/14 (random-init weights, random prompt ids)"}
    if tf:
        out["tflop_per_epoch_per_gpu"] = round(tf, 1)
        out["mfma_frac"] = round(tf / dt / PEAK_BF16_TFLOPS, 4)
    del vae, sel
    return out


def sub_config(args, dev, name, steps, warmup=1, **over):
    """One secondary configuration on this GPU (a fresh model / trainer / buffer; the headline's objects must be freed
    by the caller first): warmup, `steps` timed train steps, its dominant-kernel roofline."""
    import copy
    a = copy.copy(args)
    for k, v in over.items():
        setattr(a, k, v)
    unet, tr, buf, g = build(a, dev)
    for _ in range(warmup):
        one_step(tr, buf, g)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        one_step(tr, buf, g)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    imgs = 2 * a.pairs * a.gas * (a.num_steps - 1)
    out = {"imgs_per_s": round(imgs / dt, 3), "ms_per_step": round(dt * 1e3, 2), "steps": steps, "warmup": warmup,
           "imgs_per_step": imgs, "loss": round(torch.stack(tr.loss_hist[-2:]).mean().item(), 6)}
    pair_micro = a.pairs * a.gas * (a.num_steps - 1)
    tf = SURVEY_TFLOP_FULL_UNET if a.full_unet else SURVEY_TFLOP_PER_PAIR_MICRO.get(a.rank)
    if a.res == 1024 and tf:
        skip = 0.0 if a.full_unet else 2 * pair_micro * skipped_ref_prefix_tflop(a.res // 8)
        out["tflop_per_step"] = round(tf * pair_micro, 2)
        out["skipped_ref_prefix_tflop_per_step"] = round(skip, 3)
        out["step_mfma_frac"] = round((tf * pair_micro - skip) / dt / PEAK_BF16_TFLOPS, 4)
    if not a.no_roofline:
        rf = roofline(tr, buf, g)
        out["roofline"] = {k: rf[k] for k in ("bound", "kernel", "achieved", "peak", "unit", "frac", "avg_launch_us",
                                              "launches_per_step", "share_of_family_time", "family")}
    del unet, tr, buf
    torch.cuda.empty_cache()
    log(f"[bench] {name}: {out['imgs_per_s']} imgs/s ({out['ms_per_step']} ms/step)")
    return out


def c5_metric(dev, steps=8, warmup=2):
    """BASELINE configs[4] on this GPU: the DreamBooth PSO micro-step (pso_db, LoRA r = 16, 1 instance + 1 negative
    image, VAE encode inside the step, gas 4 -- the recipe's batch) at 1024^2, bf16 and with the fp8 forward of the
    cross-attention q / GEGLU proj (enable_fp8_forward), same model, same inputs."""
    from types import SimpleNamespace
    from pairwise_sample_optimization_amd.dreambooth import DreamBoothPSOTrainer
    from pairwise_sample_optimization_amd.trainer import compute_time_ids
    from pairwise_sample_optimization_amd.unet import UNet2DConditionModel, UNetConfig
    from pairwise_sample_optimization_amd.vae import AutoencoderKL
    with torch.device(dev):
        unet = UNet2DConditionModel(UNetConfig.sdxl(128))
        vae = AutoencoderKL()
    unet.init_weights(0)
    vae.init_weights(1)
    unet.add_adapter(SimpleNamespace(r=16, lora_alpha=16))
    unet.lora.init_gaussian(seed=0, b_std=1e-3)
    unet.prepare()
    tr = DreamBoothPSOTrainer(unet, vae, loss_type="pso_db", beta_pso=5.0, gradient_accumulation_steps=4)
    g = torch.Generator(device=dev).manual_seed(0)
    pix = torch.rand(2, 3, 1024, 1024, device=dev, generator=g) * 2 - 1
    enc = torch.randn(1, 77, 2048, device=dev, generator=g).bfloat16()
    pooled = torch.randn(1, 1280, device=dev, generator=g).bfloat16()
    tid = compute_time_ids(1024, 0, dev)
    out = {}
    for fp8 in (False, True):
        unet.enable_fp8_forward(fp8)
        for _ in range(warmup):
            tr.micro_step(pix, enc, pooled, tid, generator=g)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            tr.micro_step(pix, enc, pooled, tid, generator=g)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / steps
        out["fp8" if fp8 else "bf16"] = {"imgs_per_s": round(2 / dt, 3), "ms_per_micro_step": round(dt * 1e3, 2)}
    unet.enable_fp8_forward(False)
    out["fp8_over_bf16"] = round(out["fp8"]["imgs_per_s"] / out["bf16"]["imgs_per_s"], 4)
    out["workload"] = ("C5 (1 GPU): DreamBooth PSO pso_db, SDXL-Turbo UNet + VAE encoder, LoRA r=16, 1 instance + 1 "
                       "negative per micro-step, gas 4, 1024^2; fp8 = e4m3 cross-attention q and GEGLU proj, bf16 backward")
    del unet, vae, tr
    torch.cuda.empty_cache()
    log(f"[bench] c5: bf16 {out['bf16']['imgs_per_s']} / fp8 {out['fp8']['imgs_per_s']} imgs/s")
    return out


def vae_metric(dev, n_img=8, steps=5, warmup=1):
    """SURVEY §8a a7 on this GPU: the reward-image VAE decode of one epoch's sampled latents (2 P gas = 8 images at
    1024^2, DP/sdxl_turbo_with_logprob.py:154-155: decode of latents / scaling_factor; random-init weights), timed alone
    with HIP events over `steps` decodes; its GEMM-family roofline from one profiled decode.  10.49 TFLOP per image
     -> mfma_frac."""
    from pairwise_sample_optimization_amd.vae import AutoencoderKL, VAEConfig
    with torch.device(dev):
        vae = AutoencoderKL(VAEConfig())
    vae.init_weights(0)
    vae.prepare()
    g = torch.Generator(device=dev).manual_seed(7)
    lat = torch.randn(n_img, 128, 128, 4, device=dev, generator=g)   # the trajectory buffer's NHWC fp32 latents
    for _ in range(warmup):
        vae.decode_latents_nhwc(lat)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(steps):
        vae.decode_latents_nhwc(lat)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / steps
    tf = VAE_DEC_TFLOP_PER_IMG * n_img
    rf = family_roofline(lambda: vae.decode_latents_nhwc(lat))
    out = {"images": n_img, "ms_per_decode": round(ms, 2), "ms_per_image": round(ms / n_img, 3),
           "tflop_per_decode": round(tf, 2), "achieved_tflops": round(tf / (ms * 1e-3), 1),
           "mfma_frac": round(tf / (ms * 1e-3) / PEAK_BF16_TFLOPS, 4),
           "roofline": {k: rf[k] for k in ("bound", "kernel", "achieved", "peak", "unit", "frac", "avg_launch_us",
                                           "launches_per_step", "share_of_family_time", "family")},
           "workload": "VAE decode (SDXL AutoencoderKL decoder, random-init) of 8 latents 128x128 -> 8 images 1024^2, "
                       "bf16, one launch sequence per call"}
    del vae, lat
    torch.cuda.empty_cache()
    log(f"[bench] vae: {out['ms_per_decode']} ms per {n_img}-image decode ({out['achieved_tflops']} TF/s)")
    return out


def dist_report(tr, dev, dt_rank, steps):
    """What torch.distributed really ran (backend, world) and the overlap of the gradient all-reduce with the
    backward: exposed = the compute stream's wait for RCCL after the window's last backward (GradBuckets.finish,
    HIP events on the compute stream); alone = the same buckets all-reduced with nothing beside them."""
    world = dist.get_world_size()
    per = torch.tensor([dt_rank / steps * 1e3], dtype=torch.float64, device=dev)
    allp = [torch.zeros_like(per) for _ in range(world)]
    dist.all_gather(allp, per)
    out = {"backend": dist.get_backend(), "world_size": world,
           "rank_ms_per_step": [round(t.item(), 2) for t in allp]}
    gb = tr.buckets
    if gb is not None:
        exp = [a.elapsed_time(b) for a, b in gb.exposed_ms]
        gb.exposed_ms = []
        alone = gb.alone_ms()
        from pairwise_sample_optimization_amd import kernels as K
        K.zero_(gb.flat)
        out["allreduce"] = {"buckets": len(gb.buckets), "bytes_on_wire": gb.bytes_on_wire(),
                            "wire_dtype": str(gb.wire_dtype or gb.flat.dtype).replace("torch.", ""),
                            "alone_ms": round(alone, 3) if alone is not None else None,
                            "exposed_ms_per_step": round(sum(exp) / max(len(exp), 1), 3) if exp else None}
        if exp and alone:
            out["allreduce"]["hidden_frac"] = round(max(0.0, 1.0 - (sum(exp) / len(exp)) / alone), 3)
    return out


def max_over_ranks(dt, dev):
    """The slowest rank sets the job time (barrier-bracketed timed region, MAX over ranks)."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return dt
    tt = torch.tensor([dt], dtype=torch.float64, device=dev)
    dist.all_reduce(tt, op=dist.ReduceOp.MAX)
    return tt.item()


def spawn_ranks(n):
    """--gpus N without a launcher: run N ranks under torch.distributed.run (127.0.0.1 rendezvous) as a child
    process -- no GPU call has happened in this process -- and return its exit code."""
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd, env=env)


def main():
    args = parse()
    if os.environ.get("PSO_BENCH_GEMM_VARIANT") or os.environ.get("PSO_BENCH_ATTN_VARIANT"):
        os.environ["PSO_LIB"] = "knobs"  # A/B knobs exist in the tools build only (include/pso_amd_knobs.h)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        log(f"[bench] note: WORLD_SIZE={world} but --gpus {args.gpus}; measuring the {world} launched ranks")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)
    torch.manual_seed(rank)
    if os.environ.get("PSO_BENCH_GEMM_VARIANT"):  # A/B knob of the GEMM dispatch (tools/_ab.sh)
        from pairwise_sample_optimization_amd import kernels as K
        K.gemm_set_variant(int(os.environ["PSO_BENCH_GEMM_VARIANT"]))
    if os.environ.get("PSO_BENCH_ATTN_VARIANT"):  # A/B knob of the attention kernels
        from pairwise_sample_optimization_amd import kernels as K
        K.lib().pso_attention_set_variant(int(os.environ["PSO_BENCH_ATTN_VARIANT"]))
    t_build = time.time()
    unet, tr, buf, g = build(args, dev)
    log(f"[bench] built + sampled in {time.time() - t_build:.1f}s; warmup {args.warmup}")
    for _ in range(args.warmup):
        one_step(tr, buf, g, graph=args.graph)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    if tr.buckets is not None:
        tr.buckets.timing = True
        tr.buckets.exposed_ms = []
    t0 = time.perf_counter()
    for i in range(args.steps):
        one_step(tr, buf, g, graph=args.graph)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    dt_rank = time.perf_counter() - t0
    dt = max_over_ranks(dt_rank, dev)
    if tr.buckets is not None:
        tr.buckets.timing = False
    imgs_per_step_gpu = 2 * args.pairs * args.gas * (args.num_steps - 1)
    value = imgs_per_step_gpu * world * args.steps / dt
    ms = dt / args.steps * 1e3
    loss = torch.stack(tr.loss_hist[-4:]).mean().item()
    res = {
        "metric": "PSO train-step imgs/sec (paired 1024² SDXL) at 1/2/4/8 MI355X",
        "value": round(value, 3), "unit": "imgs/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(ms, 2), "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "bf16", "data": "synthetic (random-init SDXL weights, N(0,1) text embeds, own-sampler trajectories)",
        "config": {"workload": ("C3/C4: SDXL-%s PSO train step, full-UNet grads vs a frozen reference UNet, %d "
                                "pairs/GPU/micro-step, gas %d, %d-step sampler (T=%d)"
                                % ("DMD2" if args.mode == "dmd" else "Turbo", args.pairs, args.gas, args.num_steps,
                                   args.num_steps - 1)) if args.full_unet else
                               ("C2: SDXL-Turbo PSO train step, LoRA r=%d grads, %d pairs/GPU/micro-step, gas %d, "
                                "%d-step sampler (T=%d)" % (args.rank, args.pairs, args.gas, args.num_steps,
                                                            args.num_steps - 1)),
                   "global_batch": 2 * args.pairs * world, "seq_len": (args.res // 16) ** 2, "resolution": args.res,
                   "parallelism": f"dp{world}", "launch": "hipgraph-epoch" if args.graph else "eager"},
        "loss": round(loss, 6),
    }
    tf = SURVEY_TFLOP_PER_PAIR_MICRO.get(args.rank) if (args.res == 1024 and not args.full_unet) else None
    if tf:
        pair_micro = args.pairs * args.gas * (args.num_steps - 1)
        # executed work: the SURVEY count minus the reference images' adapter-free prefix the paired pass shares
        skip = 2 * pair_micro * skipped_ref_prefix_tflop(args.res // 8)
        step_tf = tf * pair_micro - skip
        res["step_mfma_frac"] = round(step_tf / (ms * 1e-3) / PEAK_BF16_TFLOPS, 4)
        res["step_tflop_executed"] = round(step_tf, 2)
        res["skipped_ref_prefix_tflop_per_step"] = round(skip, 3)
    if world > 1:
        res["dist"] = dist_report(tr, dev, dt_rank, args.steps)
    if not args.no_roofline:
        res["roofline"] = roofline(tr, buf, g)
    if args.epochs > 0:
        log("[bench] epoch metric ...")
        res["epoch"] = epoch_metric(args, dev, tr, buf, g, args.epochs)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        log("[bench] cpu baseline ...")
        res["cpu_baseline"] = cpu_baseline(args, unet)
    if world == 1 and not args.no_extra and not args.full_unet and args.res == 1024:
        del unet, tr, buf
        torch.cuda.empty_cache()
        log("[bench] lora_bs1 ...")
        res["lora_bs1"] = dict(sub_config(args, dev, "lora_bs1", args.extra_steps + 2, warmup=2, pairs=1, gas=1),
                               workload="C2 LoRA r=%d step at 1 pair / GPU, gas 1: 2 policy + 2 reference images per "
                                        "paired pass (north-star bs=1/GPU)" % args.rank)
        log("[bench] c3 ...")
        res["c3"] = dict(sub_config(args, dev, "c3", args.extra_steps, warmup=1, mode="dmd", num_steps=4, pairs=1,
                                    gas=1, full_unet=True),
                         workload="C3: SDXL-DMD2 PSO, 4-step sampler (T=3), full-UNet grads vs a frozen reference UNet, "
                                  "1 pair / micro-step, gas 1, bf16, 1024^2")
        log("[bench] dmd_lora ...")
        res["dmd_lora"] = dict(sub_config(args, dev, "dmd_lora", max(1, args.extra_steps - 1), warmup=1, mode="dmd",
                                          num_steps=4, pairs=1, gas=4, rank=16, full_unet=False),
                               workload="the reference's own DMD2 recipe (config_sdxl_dmd_dpo.py): LoRA r=16, 4-step "
                                        "sampler (T=3), 1 pair / micro-step, gas 4 (12 micro-steps = 24 images per "
                                        "optimizer step, passes of <= 16 images), 8-bit AdamW, bf16, 1024^2")
        log("[bench] turbo_ref ...")
        res["turbo_ref"] = dict(sub_config(args, dev, "turbo_ref", max(1, args.extra_steps - 1), warmup=1,
                                           mode="turbo", num_steps=4, pairs=4, gas=2, rank=32, res=512,
                                           full_unet=False),
                                workload="the reference's own Turbo recipe (online_pso_sdxl_turbo.sh, "
                                         "config_sdxl_turbo_dpo.py): LoRA r=32, 4-step sampler (T=3), 4 pairs / "
                                         "micro-step, gas 2 (6 micro-steps = 48 images per optimizer step, passes of "
                                         "<= 16 images), 8-bit AdamW, bf16, 512^2 (T:324-332)")
        log("[bench] c5 ...")
        res["c5"] = c5_metric(dev)
        log("[bench] vae ...")
        res["vae"] = vae_metric(dev)
    if rank == 0:
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
