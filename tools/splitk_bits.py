"""Split-K (pso_gemm_ws) products of the bs = 1 pass: a digest of the outputs and the per-call time, so two builds can be
compared bit for bit (PSO_LIB_PATH selects the library: same-box A/B only).
usage (GPU): PSO_LIB_PATH=prev/libpso_old.so python tools/splitk_bits.py; python tools/splitk_bits.py"""
import hashlib
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pairwise_sample_optimization_amd import kernels as K  # noqa: E402

# (M, N, K, bias, resid, LoRA tail rank)
SHAPES = [(2048, 1280, 10240, False, False, 0), (2048, 1280, 5120, True, True, 0), (4096, 1280, 5120, True, True, 32),
          (2048, 640, 2560, True, False, 32), (8192, 640, 5120, False, False, 0), (1024, 1280, 10240, True, True, 0)]


def main():
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    print(f"PSO_LIB_PATH={os.environ.get('PSO_LIB_PATH', '(default)')}", flush=True)
    for M, N, Kd, bias, resid, r in SHAPES:
        rnd = lambda *s: torch.randn(*s, device=dev, generator=g).bfloat16()
        a, w = rnd(M, Kd), rnd(N, Kd) * 0.02
        kw = dict(bias=rnd(N) if bias else None, resid=rnd(M, N) if resid else None)
        if r:
            kw.update(a2=rnd(M, r), w2=rnd(N, r) * 0.1)
        f = lambda: K.gemm(a, w, **kw)
        out = f()
        torch.cuda.synchronize()
        dig = hashlib.sha1(out.view(torch.int16).cpu().numpy().tobytes()).hexdigest()[:16]
        for _ in range(5):
            f()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(50):
            f()
        e1.record()
        torch.cuda.synchronize()
        print(f"M={M} N={N} K={Kd} bias={bias} resid={resid} r={r}: {e0.elapsed_time(e1) / 50 * 1e3:.1f} us  "
              f"digest {dig}", flush=True)


if __name__ == "__main__":
    main()
