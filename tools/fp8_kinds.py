"""Per-kind gain of the fp8 forward on BASELINE config 5 (the DreamBooth PSO micro-step at 1024^2, pso_db, r = 16,
1 instance + 1 negative, the recipe's batch): each LayerNorm-fed / attention-fed projection kind on e4m3 alone --
qkv (self-attention q/k/v), q2 (cross-attention q), out (both to_out.0, separate row quantisation), ff (GEGLU proj),
ffout (ff.net.2, separate quantisation) -- and the default set, each with and without the occupancy rule
(unet.FP8_MIN_TILES: 192 tiles of 256 x 256), against the bf16 forward: micro-step time (median of alternated
rounds), loss and LoRA-gradient distance.  usage (GPU): python tools/fp8_kinds.py"""
import os
import sys
import time
from types import SimpleNamespace

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pairwise_sample_optimization_amd import unet as U  # noqa: E402
from pairwise_sample_optimization_amd.dreambooth import DreamBoothPSOTrainer  # noqa: E402
from pairwise_sample_optimization_amd.trainer import compute_time_ids  # noqa: E402
from pairwise_sample_optimization_amd.vae import AutoencoderKL, VAEConfig  # noqa: E402


def main():
    cuda = torch.device("cuda", 0)
    with torch.device(cuda):
        unet = U.UNet2DConditionModel(U.UNetConfig.sdxl(128))
        vae = AutoencoderKL(VAEConfig())
    unet.init_weights(0)
    vae.init_weights(2)
    unet.add_adapter(SimpleNamespace(r=16, lora_alpha=16))
    unet.lora.init_gaussian(seed=1, b_std=5e-3)
    unet.prepare()
    tr = DreamBoothPSOTrainer(unet, vae, loss_type="pso_db", beta_pso=5.0, gradient_accumulation_steps=1)
    tr.auto_step = False
    g = torch.Generator(device="cuda").manual_seed(4)
    pix = torch.rand(2, 3, 1024, 1024, device=cuda, generator=g) * 2 - 1
    enc = torch.randn(1, 77, 2048, device=cuda, generator=g).bfloat16()
    pooled = torch.randn(1, 1280, device=cuda, generator=g).bfloat16()
    tid = compute_time_ids(1024, 0, cuda)
    st = unet.lora

    def step():
        st.grad.zero_()
        return tr.micro_step(pix, enc, pooled, tid, generator=torch.Generator(device="cuda").manual_seed(11))

    def setup(cfg):
        kinds, tiles = cfg
        U.FP8_KINDS = set(kinds) | {"tail"}
        U.FP8_MIN_TILES = tiles
        unet.enable_fp8_forward(bool(kinds))

    configs = [((), 192), (("q2", "ff"), 192), (("q2", "ff"), 0)]
    for kind in ("qkv", "q2", "out", "ff", "ffout"):
        configs += [((kind,), 192), ((kind,), 0)]
    configs += [(("qkv", "q2", "out", "ff", "ffout"), 192), (("qkv", "q2", "out", "ff", "ffout"), 0)]
    res = {}
    for c in configs:  # loss / gradients once per configuration
        setup(c)
        loss = step().item()
        torch.cuda.synchronize()
        res[c] = [loss, {k: v.clone() for k, v in st.grad_dict_peft().items()}, []]
    for _ in range(5):  # alternated timing rounds
        for c in configs:
            setup(c)
            step()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(3):
                step()
            torch.cuda.synchronize()
            res[c][2].append((time.perf_counter() - t0) / 3 * 1e3)
    l0, g0, t0s = res[configs[0]]
    den = sum((v.float() ** 2).sum().item() for v in g0.values())
    med = lambda v: sorted(v)[len(v) // 2]
    print(f"bf16: {med(t0s):.2f} ms/micro-step (rounds {[round(x, 2) for x in t0s]})", flush=True)
    for c in configs[1:]:
        l1, g1, ts = res[c]
        grel = (sum(((g1[k].float() - v.float()) ** 2).sum().item() for k, v in g0.items()) / den) ** 0.5
        print(f"fp8 {'+'.join(c[0]):26s} min_tiles {c[1]:3d}: {med(ts):.2f} ms (x{med(t0s) / med(ts):.3f} vs bf16)  "
              f"loss rel {abs(l1 - l0) / abs(l0):.2e}  LoRA grad rel {grel:.3e}", flush=True)
    U.FP8_KINDS = {"q2", "ff", "tail"}
    U.FP8_MIN_TILES = 192
    unet.enable_fp8_forward(False)


if __name__ == "__main__":
    main()
