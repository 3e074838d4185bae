"""Which fp8 projections carry the fp8 forward's LoRA-gradient error (BASELINE config 5)?  The DreamBooth micro-step of
tests/test_gpu_dreambooth.py::test_dreambooth_micro_step_fp8_at_1024 (1024^2, pso_db, r = 16, 1 instance + 1 negative)
with the e4m3 kernel on a subset of the LayerNorm-fed projections (unet.FP8_KINDS: qkv, q2, ff, and "tail" = the
LoRA up-projection as an e4m3 K-tail instead of a bf16 add), each against the bf16 forward: loss and LoRA-gradient
relative distance, plus the micro-step time.
usage (GPU): python tools/diag_fp8_grads.py"""
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
    cfg = U.UNetConfig.sdxl(128)
    with torch.device(cuda):
        unet = U.UNet2DConditionModel(cfg)
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

    def run(fp8, kinds):
        U.FP8_KINDS = set(kinds)
        unet.enable_fp8_forward(fp8)
        st.grad.zero_()
        loss = tr.micro_step(pix, enc, pooled, tid, generator=torch.Generator(device="cuda").manual_seed(11)).item()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(3):
            st.grad.zero_()
            tr.micro_step(pix, enc, pooled, tid, generator=torch.Generator(device="cuda").manual_seed(11))
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / 3 * 1e3
        st.grad.zero_()
        tr.micro_step(pix, enc, pooled, tid, generator=torch.Generator(device="cuda").manual_seed(11))
        return loss, {k: v.clone() for k, v in st.grad_dict_peft().items()}, ms

    l0, g0, ms0 = run(False, ())
    den = sum((v.float() ** 2).sum().item() for v in g0.values())
    print(f"bf16: loss {l0:.6f}  {ms0:.1f} ms/micro-step", flush=True)
    for kinds in [("q2", "ff", "tail"), ("qkv", "q2", "ff", "tail"), ("qkv", "q2", "ff"), ("qkv", "tail"), ("qkv",),
                  ("q2", "tail"), ("q2",), ("ff",)]:
        l1, g1, ms1 = run(True, kinds)
        grel = (sum(((g1[k].float() - v.float()) ** 2).sum().item() for k, v in g0.items()) / den) ** 0.5
        # per module kind: which adapters' gradients moved most
        part = {}
        for k, v in g0.items():
            key = next((t for t in ("to_q", "to_k", "to_v", "to_out") if t in k), "other")
            a = part.setdefault(key, [0.0, 0.0])
            a[0] += ((g1[k].float() - v.float()) ** 2).sum().item()
            a[1] += (v.float() ** 2).sum().item()
        parts = " ".join(f"{t} {(a[0] / max(a[1], 1e-30)) ** 0.5:.3e}" for t, a in sorted(part.items()))
        print(f"fp8 {'+'.join(kinds):22s}: loss rel {abs(l1 - l0) / abs(l0):.2e}  LoRA grad rel vs bf16 {grel:.3e}  "
              f"[{parts}]  {ms1:.1f} ms/micro-step", flush=True)
    U.FP8_KINDS = {"q2", "ff", "tail"}
    unet.enable_fp8_forward(False)


if __name__ == "__main__":
    main()
