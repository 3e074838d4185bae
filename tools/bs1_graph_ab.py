"""Same-process A/B of eager launches vs the hipGraph-captured epoch at the north-star bs = 1 / GPU point (the
lora_bs1 sub-bench: C2 LoRA step at 1 pair, gas 1), alternating arms.  usage (GPU): python tools/bs1_graph_ab.py [rounds]"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    sys.argv = [sys.argv[0], "--no-cpu-baseline"]
    args = bench.parse()
    args.pairs, args.gas = 1, 1
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    unet, tr, buf, g = bench.build(args, dev)
    imgs = 2 * args.pairs * args.gas * (args.num_steps - 1)
    for r in range(rounds):
        for graph in (False, True):
            for _ in range(2):
                bench.one_step(tr, buf, g, graph=graph)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            n = 10
            for _ in range(n):
                bench.one_step(tr, buf, g, graph=graph)
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / n
            print(f"round {r} {'graph' if graph else 'eager'}: {dt * 1e3:.2f} ms/step  {imgs / dt:.2f} imgs/s", flush=True)


if __name__ == "__main__":
    main()
