"""One rank of the world-2 data-parallel trainer check (tests/test_gpu_dist.py launches two under
torch.distributed.run, both on cuda:0, gloo backend).  Each rank trains its OWN pairs (seed 1000 + rank, T:238) from
the same initial weights:
  1. the window's backward with the overlapped bucketed all-reduce (GradBuckets) -> synced gradient A;
  2. the same window with the flat post-backward all-reduce -> synced gradient B;  A == B up to the dW kernels'
     float-atomic rounding, and A is bitwise identical on both ranks;
  3. a real optimizer step: LoRA masters bitwise identical on both ranks afterwards.
With --full, the C4 path (BASELINE configs[3], D:777-864 under DDP, T:228-233,857): DMD2 (N = 4, T = 3), every UNet
parameter trained against a frozen reference UNet, the per-tensor 8-bit AdamW, the full-UNet gradient on the bf16
wire (the trainer's default for full-UNet mode):
  1. the window's backward with the overlapped bucketed all-reduce -> synced gradient A (every bucket issued during
     the backward);
  2. the same window once more without a sync -> the local gradient L; the bucketed sync of L (GradBuckets.finish
     issuing every bucket) and the flat sync of L (allreduce_grads) give the same bits; A matches them up to the
     full-UNet backward's f32-atomic order (bias / norm parameter sums);
  3. a real optimizer step from A: every rank holds the same fp32 masters and bf16 working weights afterwards, and
     the whole gradient buffer -- the pads between parameter tensors included -- is zero (the 8-bit step zeroes what
     it reads, no kernel writes a pad).
Writes rank<r>.json into the --out directory."""
import argparse
import json
import os
import sys
from types import SimpleNamespace

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    ap.add_argument("--full", action="store_true")
    args = ap.parse_args()
    if args.full:
        return main_full(args)
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from pairwise_sample_optimization_amd.trainer import PSOTrainer, compute_time_ids, allreduce_grads
    from pairwise_sample_optimization_amd.unet import UNet2DConditionModel, UNetConfig
    cfg = UNetConfig.tiny(16)
    with torch.device(dev):
        unet = UNet2DConditionModel(cfg)
    unet.init_weights(0)
    unet.add_adapter(SimpleNamespace(r=8, lora_alpha=8))
    unet.lora.init_gaussian(seed=1, b_std=0.05)
    unet.prepare()
    P, gas = 2, 2
    tr = PSOTrainer(unet, mode="turbo", num_steps=2, gradient_accumulation_steps=gas, train_batch_size=P, lr=1e-3)
    assert tr.world == world and tr.buckets is not None and len(tr.buckets.buckets) >= 1
    tr.buckets.__init__(unet, unet.lora.grad, bucket_mb=0.05)  # several buckets even at the tiny size
    g = torch.Generator(device="cuda").manual_seed(1000 + rank)
    Bp = P * gas
    enc = torch.randn(Bp, 77, cfg.cross_attention_dim, device=dev, generator=g).bfloat16()
    pooled = torch.randn(Bp, cfg.text_embed_dim, device=dev, generator=g).bfloat16()
    tid = compute_time_ids(128, 0, dev).repeat(Bp, 1)
    buf = tr.sample_pairs(enc, pooled, tid, 16, generator=g,
                          reward_fn=lambda x: torch.rand(x.shape[0], device=dev, generator=g))
    sb = tr.shuffle(buf, generator=torch.Generator(device="cuda").manual_seed(77 + rank))
    mb = tr.micro_batch(sb, 0, sb.n_micro)
    st = unet.lora
    # 1. overlapped bucketed sync: the window's last (here: only) backward issues the buckets
    step = tr.optimizer_step
    tr.optimizer_step = lambda: None
    st.grad.zero_()
    tr.micro_step(mb)
    armed = tr.sync_armed
    issued = sum(w is not None for w in tr.buckets.works)
    scale = tr.buckets.finish()
    tr.sync_armed = False
    ga = st.grad.clone()
    # 2. flat sync of the same window
    tr.overlap_sync = False
    tr.n_micro = 0
    st.grad.zero_()
    tr.micro_step(mb)
    allreduce_grads(st.grad)
    gb = st.grad.clone()
    rel = ((ga - gb).norm() / gb.norm()).item()
    gathered = [torch.empty_like(ga) for _ in range(world)]
    dist.all_gather(gathered, ga)
    ranks_equal = all(torch.equal(gathered[0], x) for x in gathered)
    # 3. a real optimizer step from the synced gradient
    tr.optimizer_step = step
    st.grad.copy_(ga)
    tr.optimizer_step()
    torch.cuda.synchronize()
    mg = [torch.empty_like(st.master) for _ in range(world)]
    dist.all_gather(mg, st.master)
    with open(os.path.join(args.out, f"rank{rank}.json"), "w") as f:
        json.dump({"armed": armed, "issued_before_finish": issued, "buckets": len(tr.buckets.buckets),
                   "scale": scale, "bucketed_vs_flat_rel": rel, "synced_equal_across_ranks": ranks_equal,
                   "masters_equal_across_ranks": all(torch.equal(mg[0], x) for x in mg),
                   "grad_norm": gb.norm().item()}, f)
    dist.destroy_process_group()


def main_full(args):
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from pairwise_sample_optimization_amd.trainer import PSOTrainer, compute_time_ids, allreduce_grads, GradBuckets
    from pairwise_sample_optimization_amd.unet import UNet2DConditionModel, UNetConfig
    cfg = UNetConfig.tiny(16)

    def make():
        with torch.device(dev):
            u = UNet2DConditionModel(cfg)
        u.init_weights(0)  # the same initial weights on every rank
        return u

    unet, ref_unet = make(), make()
    fg = unet.enable_full_grads()
    ref_unet.prepare()
    unet.prepare()
    P = 1
    tr = PSOTrainer(unet, mode="dmd", num_steps=4, gradient_accumulation_steps=1, train_batch_size=P,
                    ref_unet=ref_unet, use_8bit_adam=True, lr=1e-4, allreduce_dtype="auto")
    assert tr.world == world and tr.buckets is not None
    assert tr.allreduce_dtype == torch.bfloat16  # "auto" (opt-in): the full-UNet gradient on a bf16 wire
    tr.buckets = GradBuckets(unet, fg.grad, bucket_mb=0.5, wire_dtype=tr.allreduce_dtype)  # several buckets
    g = torch.Generator(device="cuda").manual_seed(1000 + rank)
    enc = torch.randn(P, 77, cfg.cross_attention_dim, device=dev, generator=g).bfloat16()
    pooled = torch.randn(P, cfg.text_embed_dim, device=dev, generator=g).bfloat16()
    tid = compute_time_ids(128, 0, dev).repeat(P, 1)
    buf = tr.sample_pairs(enc, pooled, tid, 16, generator=g,
                          reward_fn=lambda x: torch.rand(x.shape[0], device=dev, generator=g))
    sb = tr.shuffle(buf, generator=torch.Generator(device="cuda").manual_seed(77 + rank))
    assert sb.n_micro == tr.gas_total == 3
    mb = tr.micro_batch(sb, 0, sb.n_micro)
    # 1. overlapped bucketed sync on the bf16 wire
    step = tr.optimizer_step
    tr.optimizer_step = lambda: None
    fg.grad.zero_()
    loss = tr.micro_step(mb)
    armed = tr.sync_armed
    issued = sum(w is not None for w in tr.buckets.works)
    scale = tr.buckets.finish()
    tr.sync_armed = False
    ga = fg.grad.clone()
    # 2. the local gradient of the same window, then its bucketed and flat syncs
    tr.overlap_sync = False
    tr.n_micro = 0
    fg.grad.zero_()
    tr.micro_step(mb)
    local = fg.grad.clone()
    fg.grad.zero_()
    tr.n_micro = 0
    tr.micro_step(mb)
    local_repeat = torch.equal(fg.grad, local)  # every gradient sum of the full-UNet backward is ordered
    fg.grad.copy_(local)
    for b in range(len(tr.buckets.buckets)):
        assert tr.buckets.works[b] is None
    tr.buckets.finish()  # issues every bucket of the local gradient, waits, casts the bf16 wire back
    gc_ = fg.grad.clone()
    fg.grad.copy_(local)
    allreduce_grads(fg.grad, wire_dtype=torch.bfloat16)
    gb = fg.grad.clone()
    gathered = [torch.empty_like(ga) for _ in range(world)]
    dist.all_gather(gathered, ga)
    ranks_equal = all(torch.equal(gathered[0], x) for x in gathered)
    # 3. a real optimizer step from the overlapped sync
    tr.overlap_sync = True
    tr.optimizer_step = step
    fg.grad.copy_(ga)
    w0 = unet.conv_out.weight.detach().clone()
    tr.optimizer_step()
    torch.cuda.synchronize()
    mg = [torch.empty_like(fg.master) for _ in range(world)]
    dist.all_gather(mg, fg.master)
    wk = [torch.empty_like(fg.work) for _ in range(world)]
    dist.all_gather(wk, fg.work)
    with open(os.path.join(args.out, f"rank{rank}.json"), "w") as f:
        json.dump({"armed": armed, "issued_before_finish": issued, "buckets": len(tr.buckets.buckets),
                   "wire": str(tr.allreduce_dtype), "scale": scale, "loss": loss.item(),
                   "numel": fg.grad.numel(), "bucketed_equals_flat": torch.equal(gc_, gb),
                   "overlapped_vs_flat_rel": ((ga - gb).norm() / gb.norm()).item(),
                   "overlapped_equals_flat": torch.equal(ga, gb), "local_run_to_run_equal": local_repeat,
                   "synced_equal_across_ranks": ranks_equal,
                   "masters_equal_across_ranks": all(torch.equal(mg[0], x) for x in mg),
                   "work_equal_across_ranks": all(torch.equal(wk[0], x) for x in wk),
                   "weights_moved": not torch.equal(unet.conv_out.weight, w0),
                   "grad_max_after_step": fg.grad.abs().max().item(),
                   "grad_norm": gb.norm().item()}, f)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
