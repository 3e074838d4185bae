"""World-1 RCCL rank of tests/test_gpu_dist.py::test_rccl_world1_bucketed_overlap_on_comm_stream (launched under
torch.distributed.run, backend "nccl" = RCCL on ROCm, the backend bench.py uses).  Reference: the DDP gradient sync
of accelerator.backward (T:228-233,491-493,857).

The SDXL-topology UNet at 32^2 latents with LoRA r = 32, the LoRA weight-gradient products NOT batched and launched on
the side stream (PSO_SIDE_STREAM path), small buckets so a dozen all-reduces leave during the backward:
  1. overlapped bucketed sync (GradBuckets: side.join() -> async all_reduce on RCCL's stream -> finish() stream
     waits) -> gradient A;
  2. the same window with the flat post-backward all_reduce -> gradient B;  A == B bit for bit (world 1: the sum is
     the identity, and every reduction of the backward is ordered);
  3. bf16 on the wire: the synced gradient is exactly bf16(A);
  4. one optimizer step from each: identical LoRA masters.
Writes rank0.json into --out."""
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
    args = ap.parse_args()
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
    from pairwise_sample_optimization_amd import kernels as K
    from pairwise_sample_optimization_amd import unet as unet_mod
    from pairwise_sample_optimization_amd.trainer import PSOTrainer, compute_time_ids, allreduce_grads
    from pairwise_sample_optimization_amd.unet import UNet2DConditionModel, UNetConfig
    K.SideStream.enabled = True   # LoRA dW closures on the side stream ...
    unet_mod.TN_BATCH = False     # ... each product launched there at once (not deferred to the compute stream)
    cfg = UNetConfig.sdxl(32)

    def make(wire=None):
        with torch.device(dev):
            u = UNet2DConditionModel(cfg)
        u.init_weights(0)
        u.add_adapter(SimpleNamespace(r=32, lora_alpha=32))
        u.lora.init_gaussian(seed=1, b_std=3e-3)
        u.prepare()
        t = PSOTrainer(u, mode="turbo", num_steps=2, gradient_accumulation_steps=2, train_batch_size=2, lr=1e-4,
                       overlap_sync=True, bucket_mb=1.0, allreduce_dtype=wire)
        return u, t

    unet, tr = make()
    g = torch.Generator(device="cuda").manual_seed(1000 + rank)
    enc = torch.randn(4, 77, 2048, device=dev, generator=g).bfloat16()
    pooled = torch.randn(4, 1280, device=dev, generator=g).bfloat16()
    tid = compute_time_ids(256, 0, dev).repeat(4, 1)
    buf = tr.sample_pairs(enc, pooled, tid, 32, generator=g,
                          reward_fn=lambda x: torch.rand(x.shape[0], device=dev, generator=g))
    sb = tr.shuffle(buf, generator=torch.Generator(device="cuda").manual_seed(77))
    mb = tr.micro_batch(sb, 0, sb.n_micro)
    st = unet.lora

    side_pending = [0]

    def spy(bk):
        orig = bk._issue

        def issue(b, side=None):
            if side is not None and side.pending:
                side_pending[0] += 1
            orig(b, side)
        bk._issue = issue

    spy(tr.buckets)
    # 1. overlapped bucketed sync, then the optimizer step (auto_step at the window's end)
    st.grad.zero_()
    step = tr.optimizer_step
    grads = {}

    def grab_then_step():
        issued = sum(w is not None for w in tr.buckets.works)
        grads["issued"] = issued
        tr.buckets.finish()
        tr.sync_armed = False
        grads["a"] = st.grad.clone()
        step()
    tr.optimizer_step = grab_then_step
    tr.micro_step(mb)
    torch.cuda.synchronize()
    ma = st.master.clone()
    # 2. flat sync of the same window from the same initial weights
    unet2, tr2 = make()
    tr2.overlap_sync = False
    st2 = unet2.lora
    step2 = tr2.optimizer_step

    def grab_flat_then_step():
        allreduce_grads(st2.grad)
        grads["b"] = st2.grad.clone()
        step2()
    tr2.optimizer_step = grab_flat_then_step
    tr2.micro_step(mb)
    torch.cuda.synchronize()
    mb_ = st2.master.clone()
    # 3. bf16 on the wire
    unet3, tr3 = make(wire=torch.bfloat16)

    def grab_wire():
        tr3.buckets.finish()
        tr3.sync_armed = False
        grads["c"] = unet3.lora.grad.clone()
    tr3.optimizer_step = grab_wire
    tr3.micro_step(mb)
    torch.cuda.synchronize()
    ga, gb, gc = grads["a"], grads["b"], grads["c"]
    res = dict(backend=dist.get_backend(), world=dist.get_world_size(), buckets=len(tr.buckets.buckets),
               issued_before_finish=grads["issued"], side_pending_at_issue=side_pending[0],
               grad_norm=ga.norm().item(), bucketed_equals_flat=bool(torch.equal(ga, gb)),
               wire_bf16_equals_cast=bool(torch.equal(gc, ga.bfloat16().float())),
               masters_equal=bool(torch.equal(ma, mb_)))
    with open(os.path.join(args.out, f"rank{rank}.json"), "w") as f:
        json.dump(res, f)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
