"""The online PSO epoch for timestep-distilled SDXL, MI355X-native: paired on-policy sampling, trajectory buffer +
shuffles, the (pair-batch, transition) micro-step and the optimizer step.

Reference loop (`T` = human_preference_tuning/train_online_pso_sdxl_turbo.py, `D` = ..._dmd2.py):
  SAMPLING  T:554-673 / D:557-679  two independent trajectories per prompt through the distilled UNet, rewards
  BUFFER    T:610-666,714-749       stack (B, 2, T, ...); per inner epoch permute pairs and, independently per pair,
                                    the transition order (same for both members)
  MICRO     T:771-861 / D:773-864   2 policy UNet fwd (LoRA on) + 2 reference fwd (adapters off) + 4 step log-probs
                                    + clipped pairwise loss + backward; grads accumulate over gas*T micro-steps
  SYNC      T:857-861               DDP all-reduce, clip_grad_norm_(1.0), optimizer.step, zero_grad

Here every per-element operation runs in libpso_amd; the micro-step issues no host synchronisation (the reference
syncs 4x in turbo_step_with_logprob's `.item()` lookups and once in `accelerator.gather(loss).item()`).  The two
members of every pair ride in ONE UNet batch (image order 2p + k), policy and reference forwards share the frozen
weights, the loss kernel consumes the bf16 NHWC eps directly and emits d loss / d eps for the hand-written UNet
backward, which accumulates LoRA grads into the flat all-reduce bucket.
"""
import gc
import math
from types import SimpleNamespace

import torch
import torch.distributed as dist

import os

from . import kernels as K
from . import pso_core
from ._lib import MODE_TURBO, MODE_DMD
from .schedulers import EulerAncestralDiscreteScheduler, LCMScheduler, dmd_distill_timesteps

# full-UNet mode: the frozen reference pass on a stream of its own (PSO_REF_STREAM=0 keeps it in line, A/B knob)
_REF_STREAM = os.environ.get("PSO_REF_STREAM", "1") == "1"
_GC_PAUSE = os.environ.get("PSO_GC_PAUSE", "1") == "1"  # train_epoch: cyclic GC paused (A/B knob)
_REF_STREAMS = {}


def _ref_stream():
    """ONE reference-pass stream per device for the process (the caching allocator keeps freed blocks per stream)."""
    dev = torch.cuda.current_device()
    st = _REF_STREAMS.get(dev)
    if st is None:
        st = _REF_STREAMS[dev] = torch.cuda.Stream(device=dev)
    return st


BF16 = torch.bfloat16


def compute_time_ids(size, crop=0, device=None):
    """T:324-332 (512) / D:347-355 (1024): [orig_h, orig_w, crop_top, crop_left, target_h, target_w]."""
    return torch.tensor([[size, size, crop, crop, size, size]], dtype=torch.float32, device=device)


def shuffle_index(perm, perms, P):
    """Row indices of the shuffled, re-batched training stream (T:733-760 / D:719-753).

    perm [Bp] pair permutation, perms [Bp, T] per-row time permutation.  The reference applies `perms` after
    `samples = samples[perm]`, so shuffled row i = old pair perm[i] with time order perms[i].  Micro-step s = (batch b, step j) holds, for p < P and
    member k, buffer row ((perm[bP+p]*2 + k)*T + perms[bP+p, j]) of the [2Bp*T] latent stream.
    Returns (img_idx [nb*T*P*2], pair_img [same] rows of per-pair tensors, tsel [same] transition index)."""
    Bp, T = perms.shape
    nb = Bp // P
    dev = perm.device
    pb = torch.arange(nb, device=dev).view(nb, 1, 1, 1)
    jj = torch.arange(T, device=dev).view(1, T, 1, 1)
    pp = torch.arange(P, device=dev).view(1, 1, P, 1)
    kk = torch.arange(2, device=dev).view(1, 1, 1, 2)
    row = pb * P + pp                                         # new (shuffled) position  [nb,1,P,1]
    pair = perm[row]                                          # old pair id
    tsel = perms[row, jj]                                     # [nb,T,P,1]
    img_idx = ((pair * 2 + kk) * T + tsel).reshape(-1)
    pair_img = (pair * 2 + kk).expand(nb, T, P, 2).reshape(-1)
    tsel_i = tsel.expand(nb, T, P, 2).reshape(-1)
    return img_idx, pair_img, tsel_i


def allreduce_grads(flat, process_group=None, wire_dtype=None):
    """DDP gradient sync of the flat trained gradient in one collective (T:857 under accelerate: all-reduce SUM, then
    the mean) -- the path when no overlapped GradBuckets sync was armed (hipGraph epochs).  The 1/world factor is
    returned, not applied: the clip and AdamW kernels fold it into their gradient read.  wire_dtype=torch.bfloat16
    reduces a bf16 copy and casts the sum back (half the bytes; fp32 accumulation stays local)."""
    if not (dist.is_available() and dist.is_initialized()):
        return 1.0
    world = dist.get_world_size(process_group)
    if world == 1:
        return 1.0
    if wire_dtype is not None and wire_dtype != flat.dtype:
        t = flat.to(wire_dtype)
        dist.all_reduce(t, group=process_group)
        flat.copy_(t)
    else:
        dist.all_reduce(flat, group=process_group)
    return 1.0 / world


class GradBuckets:
    """DDP-style gradient sync overlapped with the backward (what accelerator.backward's DDP bucket hooks do on a sync
    micro-step, T:228-233,857): the flat trained gradient is cut into ~bucket_mb contiguous buckets
    along the backward's completion order (UNet2DConditionModel.grad_unit_ranges); backward_nhwc reports every
    finished unit through rt.unit_done and, as soon as a bucket's last unit is done, its all-reduce (SUM) is issued
    asynchronously -- with RCCL it runs on the communicator's own stream, ordered after the compute stream's work so
    far, beside the rest of the backward.  finish() issues whatever is left and makes the compute stream wait for
    every bucket before the clip / AdamW read the gradient.  The 1/world mean is folded into those kernels."""

    def __init__(self, unet, flat, bucket_mb=32.0, process_group=None, wire_dtype=None):
        self.flat = flat
        self.pg = process_group
        self.world = dist.get_world_size(process_group)
        # wire_dtype=torch.bfloat16: every bucket is cast to bf16 for the all-reduce and cast back into the fp32 flat
        # gradient afterwards (what DDP's bf16_compress_hook does): half the xGMI bytes -- 5.1 instead of 10.3 GB per
        # full-UNet step (C4) -- while the local accumulation over the window's micro-steps stays fp32
        self.wire_dtype = wire_dtype
        self.timing = False      # record the compute-stream stall on the outstanding buckets (bench diagnostics)
        self.exposed_ms = []     # per finish(): ms the compute stream waited for RCCL after the backward
        self._ev = None
        cap = int(bucket_mb * 1e6 / flat.element_size())
        self.buckets = []        # [(offset, numel, last unit)]
        self.unit_bucket = {}    # unit -> bucket index (every unit of the bucket)
        units = unet.grad_unit_ranges()
        cur_off, cur_n, cur_units = None, 0, []
        for unit, off, n in units:
            if cur_off is None:
                cur_off = off
            cur_n += n
            cur_units.append(unit)
            if cur_n >= cap:
                self._close(cur_off, cur_n, cur_units)
                cur_off, cur_n, cur_units = None, 0, []
        if cur_units:
            self._close(cur_off, cur_n, cur_units)
        covered = sum(n for _, n, _ in self.buckets)
        assert covered == flat.numel(), f"buckets cover {covered} of {flat.numel()} gradient elements"
        self.reset()

    def _close(self, off, n, units):
        b = len(self.buckets)
        self.buckets.append((off, n, tuple(units)))
        for u in units:
            self.unit_bucket[u] = b

    def reset(self):
        self.pending = [set(u) for _, _, u in self.buckets]
        self.works = [None] * len(self.buckets)
        self.wire = [None] * len(self.buckets)

    def _issue(self, b, side=None):
        if self.works[b] is not None:
            return
        if side is not None:
            side.join()  # LoRA dW launches on the side stream belong to this bucket
        off, n, _ = self.buckets[b]
        t = self.flat[off:off + n]
        if self.wire_dtype is not None and self.wire_dtype != t.dtype:
            t = t.to(self.wire_dtype)  # cast on the compute stream; the collective is ordered after it
            self.wire[b] = t
        self.works[b] = dist.all_reduce(t, group=self.pg, async_op=True)

    def bytes_on_wire(self):
        es = torch.empty((), dtype=self.wire_dtype or self.flat.dtype).element_size()
        return sum(n for _, n, _ in self.buckets) * es

    def hook(self, rt):
        """rt.unit_done for one backward pass (the pass that ends an accumulation window)."""
        side = getattr(rt, "side", None)

        def unit_done(unit):
            b = self.unit_bucket.get(unit)
            if b is None:
                return
            self.pending[b].discard(unit)
            if not self.pending[b]:
                self._issue(b, side)
        return unit_done

    def finish(self):
        """Issue the buckets not reported (none on the normal path), then wait for all of them; returns 1/world.
        With RCCL the waits are stream waits: the compute stream (clip / AdamW next) queues behind each bucket's
        collective, the host does not block.  bf16 wire buckets are cast back into the fp32 gradient here."""
        for b in range(len(self.buckets)):
            self._issue(b)
        if self.timing and torch.cuda.is_available() and self.flat.is_cuda:
            e0 = torch.cuda.Event(enable_timing=True)
            e0.record()
        else:
            e0 = None
        for b, w in enumerate(self.works):
            w.wait()
            if self.wire[b] is not None:
                off, n, _ = self.buckets[b]
                self.flat[off:off + n].copy_(self.wire[b])
        if e0 is not None:
            e1 = torch.cuda.Event(enable_timing=True)
            e1.record()
            self.exposed_ms.append((e0, e1))
        self.reset()
        return 1.0 / self.world

    def alone_ms(self, reps=3):
        """Time the window's all-reduces with nothing beside them (every bucket issued back to back, then waited):
        the denominator of the hidden-under-backward fraction.  Sums into the gradient: callers zero it after."""
        dev_ev = self.flat.is_cuda
        times = []
        for _ in range(reps):
            if dev_ev:
                torch.cuda.synchronize()
            dist.barrier(group=self.pg)
            t0 = torch.cuda.Event(enable_timing=True) if dev_ev else None
            if dev_ev:
                t0.record()
            for b in range(len(self.buckets)):
                self._issue(b)
            for b, w in enumerate(self.works):
                w.wait()
            if dev_ev:
                t1 = torch.cuda.Event(enable_timing=True)
                t1.record()
                torch.cuda.synchronize()
                times.append(t0.elapsed_time(t1))
            self.reset()
        return min(times) if times else None


def trainable(unet):
    """(master, grad, refresh) of what the step trains: the flat LoRA bucket (the reference's recipe), or every UNet
    parameter when unet.enable_full_grads() was called (BASELINE C3 / C4, build-only).  refresh(cast=True)."""
    if getattr(unet, "full", None) is not None:
        return unet.full.master, unet.full.grad, unet.refresh_full
    st = unet.lora
    return st.master, st.grad, st.refresh


def trainable_segments(unet):
    """[(offset, numel)] of the parameter tensors inside the flat trained buffer -- what the reference hands its
    optimizer (T:428-448: the peft lora_A / lora_B weights, or every UNet parameter in full-UNet mode); the 8-bit
    AdamW quantises each of them on its own (K.Adam8State)."""
    if getattr(unet, "full", None) is not None:
        fg = unet.full
        return [(fg.offsets[nm][0], p.numel()) for nm, p in zip(fg.names, fg.params)]
    st = unet.lora
    base = st.master.data_ptr()
    segs = []
    for name in st.adapter_names():
        for t in st.adapter_views(st.master, name):
            segs.append(((t.data_ptr() - base) // st.master.element_size(), t.numel()))
    return segs


def _work_copy(unet, master):
    """The flat bf16 working copy that refresh() casts the master into (the optimizer can write it directly)."""
    st = unet.full if getattr(unet, "full", None) is not None else unet.lora
    w = getattr(st, "work", None)
    ok = (w is not None and w.dtype == torch.bfloat16 and w.numel() == master.numel() and w.is_contiguous()
          and w.data_ptr() % 16 == 0)
    return w if ok else None


def lora_optimizer_step(tr):
    """accelerator.backward's sync step + clip_grad_norm_ + optimizer.step + zero_grad (T:857-861, DB:1953-1964) on
    the flat LoRA bucket of tr.unet: RCCL all-reduce -> global-norm clip coefficient -> fused AdamW (clip and 1/world
    folded into the gradient read) -> zero -> refresh the bf16 working copies.  tr carries exp_avg, exp_avg_sq,
    opt_step, clip_buf, lr, betas, adam_eps, wd, max_grad_norm, pg and, when the last backward of the window already
    issued the bucketed all-reduce (tr.sync_armed), the GradBuckets to finish."""
    master, grad, refresh = trainable(tr.unet)
    if getattr(tr, "sync_armed", False):
        scale = tr.buckets.finish()
        tr.sync_armed = False
    else:
        scale = allreduce_grads(grad, tr.pg, getattr(tr, "allreduce_dtype", None))
    K.grad_clip_coef(grad, tr.max_grad_norm, grad_scale=scale, out=tr.clip_buf)
    tr.opt_step += 1
    cast = True
    if getattr(tr, "adam8", None) is not None:  # train.use_8bit_adam: bitsandbytes AdamW8bit (T:427-435)
        work = _work_copy(tr.unet, master)  # the step also writes the bf16 working copy (no separate cast pass)
        # with a per-tensor block table the step also zeroes the gradient it reads (the pads between tensors are
        # zero from allocation and no kernel writes them)
        zeroed = K.adamw8bit_step(master, grad, tr.adam8, tr.lr, tr.betas, tr.adam_eps, tr.wd, tr.opt_step,
                                  grad_scale=scale, clip=tr.clip_buf, out_bf16=work, zero_grad=True)
        cast = work is None
    else:
        zeroed = False
        K.adamw_step(master, grad, tr.exp_avg, tr.exp_avg_sq, tr.lr, tr.betas, tr.adam_eps, tr.wd, tr.opt_step,
                     grad_scale=scale, clip=tr.clip_buf)
    if not zeroed:
        K.zero_(grad)
    refresh(cast=cast)


class PSOTrainer:
    def __init__(self, unet, mode="turbo", num_steps=2, beta=50.0, clip_eps=0.1, lr=1e-5, betas=(0.9, 0.999),
                 weight_decay=1e-6, adam_eps=1e-8, max_grad_norm=1.0, gradient_accumulation_steps=1,
                 train_batch_size=1, num_reward=1, process_group=None, max_pass_images=16, ref_unet=None,
                 latent_dtype=torch.float32, allreduce_dtype=None, use_8bit_adam=False, overlap_sync=None,
                 bucket_mb=32.0):
        self.unet = unet
        if mode not in ("turbo", "dmd"):
            raise ValueError(f"mode must be 'turbo' or 'dmd', got {mode!r}")
        # DMD2 with fp16 / bf16 latents: the reference's latent-dtype step / log-prob arithmetic (replay modes,
        # DP/distilled_inference_with_logprob.py:84-135); turbo upcasts to fp32 in the reference, so it stays fp32
        self.latent_dtype = latent_dtype if mode == "dmd" else torch.float32
        self.mode = MODE_TURBO if mode == "turbo" else pso_core.dmd_mode(self.latent_dtype)
        self.num_steps = num_steps
        self.T = num_steps - 1                       # the last (deterministic) step is never trained (T:218-221)
        self.beta, self.clip_eps = beta, clip_eps
        self.lr, self.betas, self.wd, self.adam_eps = lr, betas, weight_decay, adam_eps
        self.max_grad_norm = max_grad_norm
        self.gas = gradient_accumulation_steps
        self.gas_total = gradient_accumulation_steps * self.T  # Accelerator(gradient_accumulation_steps=gas*T) T:232
        self.P = train_batch_size
        self.m = num_reward
        self.pg = process_group
        self.world = dist.get_world_size(process_group) if (dist.is_available() and dist.is_initialized()) else 1
        master, _, _ = trainable(unet)
        # optimizer state: fp32 AdamW moments, or -- train.use_8bit_adam, the reference default (T:427-435) -- the
        # blockwise 8-bit AdamW of bitsandbytes (uint8 codes + per-2048-block absmax, blocks restarting at every
        # parameter tensor, 32-bit state under 4096 elements: K.Adam8State)
        self.adam8 = K.Adam8State(master.numel(), master.device, segments=trainable_segments(unet)) \
            if use_8bit_adam else None
        self.exp_avg = None if use_8bit_adam else torch.zeros_like(master)
        self.exp_avg_sq = None if use_8bit_adam else torch.zeros_like(master)
        self.opt_step = 0
        self.n_micro = 0
        self.clip_buf = torch.zeros(2, device=master.device, dtype=torch.float32)
        # full-UNet training (C3 / C4): the reference model is a frozen copy of the initial UNet (App. A #4), run as
        # its own forward instead of the adapter-free half of a paired pass
        self.ref_unet = ref_unet
        if getattr(unet, "full", None) is not None and ref_unet is None:
            raise ValueError("full-UNet training needs ref_unet (a frozen copy of the initial weights)")
        self.loss_hist = []
        # overlapped bucketed all-reduce on multi-GPU runs (GradBuckets); off inside hipGraph capture.  overlap_sync
        # forces it on (or off) whatever the world size: a world-1 RCCL group still runs every collective (tests)
        self.overlap_sync = (self.world > 1) if overlap_sync is None else bool(overlap_sync)
        if self.overlap_sync and not (dist.is_available() and dist.is_initialized()):
            raise ValueError("overlap_sync needs an initialised process group")
        # The default (None / torch.float32) is the reference's wire: DDP's fp32 all-reduce (T:228-233).  Opt-in:
        # torch.bfloat16 puts the gradient on a bf16 wire (fp32 accumulation and optimizer, GradBuckets); "auto" does
        # that for the full-UNet gradient only (C3 / C4: 10.3 GB fp32 per sync, 18 GB of ring traffic per rank at 8
        # ranks) and keeps the LoRA bucket fp32.  RCCL's ring re-rounds every partial sum on a bf16 wire, so its error
        # grows with the world size
        if isinstance(allreduce_dtype, str):
            if allreduce_dtype != "auto":
                raise ValueError(f"allreduce_dtype must be a torch dtype, None or 'auto', got {allreduce_dtype!r}")
            allreduce_dtype = torch.bfloat16 if getattr(unet, "full", None) is not None else None
        elif allreduce_dtype == torch.float32:
            allreduce_dtype = None
        self.allreduce_dtype = allreduce_dtype
        self.buckets = GradBuckets(unet, trainable(unet)[1], bucket_mb=bucket_mb, process_group=process_group,
                                   wire_dtype=allreduce_dtype) if self.overlap_sync else None
        self.sync_armed = False
        self.max_pass_images = max_pass_images  # images per batched UNet pass (HBM budget: ~5 GB saved each @1024^2)
        self.auto_step = True  # run the optimizer every gas*T micro-steps (tests may inspect raw grads)
        if self.mode == MODE_TURBO:
            self.sched = EulerAncestralDiscreteScheduler()
            self.sched.set_timesteps(num_steps)
            self.timesteps = self.sched.timesteps.clone()  # float32 [N]
        else:
            self.sched = LCMScheduler()
            ts, self.step_ratio = dmd_distill_timesteps(num_steps)
            self.timesteps = ts.float()
        dev = master.device
        self.timesteps_dev = self.timesteps.to(dev)
        # per-transition step coefficients [T, 8], host-computed once, device resident
        self.coef_dev = torch.stack([self.coef_for_step(j, 1)[0] for j in range(self.T)], 0).to(dev) \
            if self.T > 0 else torch.zeros(0, 8, device=dev)

    @classmethod
    def from_config(cls, unet, config, mode="turbo", num_reward=1, process_group=None, ref_unet=None,
                    latent_dtype=None):
        """Build from a reference run config (`config_sdxl_{turbo,dmd}_dpo.get_config()`): sample.num_steps,
        train.{beta, eps, learning_rate, adam_*, max_grad_norm, gradient_accumulation_steps, batch_size}.
        Both trainers require `distilled_train_steps == num_steps - 1` (turbo asserts it at T:221; DMD2 asserts
        `<=` at D:225 and the trajectory length `==` at D:719-720).
        latent_dtype (DMD2 only): None follows `config.mixed_precision` as the reference does -- its latents are
        weight_dtype (D:329-333; drawn in prompt_embeds.dtype, DP/sdxl_dmd_with_logprob.py:91-101), so its step /
        log-prob arithmetic runs in that dtype (DP/distilled_inference_with_logprob.py:84-135) -> the replay mode of
        that dtype; pass torch.float32 to train on the fp32 step math instead.  A value that disagrees with the
        config is honoured with a warning."""
        tr = config.train
        if tr.distilled_train_steps != config.sample.num_steps - 1:
            raise AssertionError("train.distilled_train_steps must equal sample.num_steps - 1 "
                                 f"({tr.distilled_train_steps} vs {config.sample.num_steps - 1})")
        mp = getattr(config, "mixed_precision", "no")
        cfg_dtype = {"fp16": torch.float16, "bf16": torch.bfloat16}.get(mp, torch.float32)
        if latent_dtype is None:
            latent_dtype = cfg_dtype if mode == "dmd" else torch.float32
        elif mode == "dmd" and latent_dtype != cfg_dtype:
            import warnings
            warnings.warn(f"PSOTrainer.from_config: latent_dtype {latent_dtype} differs from the config's "
                          f"mixed_precision={mp!r} (reference latents: {cfg_dtype})")
        return cls(unet, mode=mode, num_steps=config.sample.num_steps, beta=float(tr.beta), clip_eps=float(tr.eps),
                   lr=tr.learning_rate, betas=(tr.adam_beta1, tr.adam_beta2), weight_decay=tr.adam_weight_decay,
                   adam_eps=tr.adam_epsilon, max_grad_norm=tr.max_grad_norm,
                   gradient_accumulation_steps=tr.gradient_accumulation_steps, train_batch_size=tr.batch_size,
                   num_reward=num_reward, process_group=process_group, ref_unet=ref_unet, latent_dtype=latent_dtype,
                   use_8bit_adam=bool(getattr(tr, "use_8bit_adam", False)))

    # ------------------------------------------------------------------------------------------------------------
    # coefficients of transition j (host float32 scalars, the reference's operation order)
    # ------------------------------------------------------------------------------------------------------------
    def coef_for_step(self, j, n):
        if self.mode == MODE_TURBO:
            t = self.timesteps[j].repeat(n)
            return pso_core.turbo_coef(self.sched.sigmas, self.sched.timesteps, t)
        t = self.timesteps[j].long().repeat(n)
        return pso_core.dmd_coef(self.sched.alphas_cumprod, t, t - self.step_ratio, latent_dtype=self.latent_dtype)

    # ------------------------------------------------------------------------------------------------------------
    # SAMPLING: B prompts -> 2 trajectories each (independent x_T, T:572-608) -> buffer rows
    # ------------------------------------------------------------------------------------------------------------
    @torch.no_grad()
    def sample_pairs(self, enc, pooled, time_ids, h, generator=None, reward_fn=None, decode_fn=None):
        """enc [B,77,Dc] bf16, pooled [B,Dp], time_ids [B,6].  Returns a dict of NHWC buffer tensors.
        Both trajectories of a prompt are sampled in ONE UNet batch (image order 2b + k)."""
        dev = enc.device
        B = enc.shape[0]
        n_img = 2 * B
        N, T = self.num_steps, self.T
        enc2 = enc.repeat_interleave(2, 0).contiguous()
        pooled2 = pooled.repeat_interleave(2, 0).contiguous()
        tid2 = time_ids.repeat_interleave(2, 0).contiguous()
        shape = (n_img, h, h, 4)
        x = torch.randn(shape, device=dev, generator=generator, dtype=torch.float32)
        if self.mode == MODE_TURBO:
            x = x * float(self.sched.init_noise_sigma)
        elif self.latent_dtype != torch.float32:  # x_T drawn in the latent dtype (DP/sdxl_dmd_with_logprob.py:91-101)
            x = x.to(self.latent_dtype).float()
        member = torch.arange(n_img, device=dev) % 2
        xs, ins, lps = [x], [], []
        for i in range(N):
            t = self.timesteps_dev[i].repeat(n_img)
            if self.mode == MODE_TURBO:
                sig = float(self.sched.sigmas[i])
                model_in = K.cast_f32_bf16(x, scale=1.0 / math.sqrt(sig * sig + 1.0))  # DP/sdxl_turbo...:120-122
            else:
                model_in = K.cast_f32_bf16(x)
            eps, _ = self.unet.forward_nhwc(model_in, t, enc2, pooled2, tid2, save=False)
            if i < N - 1:
                coef = self.coef_for_step(i, n_img).to(dev)
                if self.mode == MODE_TURBO:
                    noise = torch.randn(shape, device=dev, generator=generator)
                    x, lp = K.step_logprob(self.mode, x, eps, coef, noise=noise)
                else:
                    # DMD2: each trajectory is its own sdxl_dmd_pipeline_with_logprob call (D:585-618) whose step
                    # re-noises with ONE (1,C,H,W) draw shared by that call's batch (DP/distilled_...:123-126): one
                    # draw per pair member k, shared by the prompts, never by the two members of a pair
                    noise = torch.randn((2,) + shape[1:], device=dev, generator=generator)
                    if self.latent_dtype != torch.float32:
                        noise = noise.to(self.latent_dtype).float()
                    x, lp = K.step_logprob(self.mode, x, eps, coef, noise=noise[member].contiguous())
                xs.append(x)
                ins.append(model_in)
                lps.append(lp)
            else:
                x_final = self._final_step(x, eps, n_img)
        x_stack = torch.stack(xs[:T + 1], 1)                    # [2B, T+1, h, h, 4]
        buf = dict(x=x_stack[:, :T].contiguous(), x_next=x_stack[:, 1:T + 1].contiguous(),
                   unet_in=torch.stack(ins, 1).contiguous(), lp=torch.stack(lps, 1), enc=enc2, pooled=pooled2,
                   tid=tid2)
        buf["x_final"] = x_final
        if reward_fn is not None:
            img = decode_fn(x_final) if decode_fn is not None else x_final
            buf["rewards"] = reward_fn(img).reshape(B, 2, -1).float()
        return buf

    def _final_step(self, x, eps, n):
        """Last sampler step (never trained): turbo sigma_to = 0 -> x + eps*(0 - sigma) (T:218-221); DMD2 returns
        x0 = (x - sqrt(1-a_t) eps) / sqrt(a_t) (DP/sdxl_dmd_with_logprob.py:154-162)."""
        dev = x.device
        zero = torch.zeros((1,) + tuple(x.shape[1:]), device=dev)
        if self.mode == MODE_TURBO:
            c = self.coef_for_step(self.num_steps - 1, n)
        else:
            t = self.timesteps[-1].long().repeat(n)
            c = pso_core.dmd_coef(self.sched.alphas_cumprod, t, t)
            c[:, 2] = 1.0  # sqrt(abar_prev) -> 1: mean = x0
            c[:, 3] = 1.0
        xf, _ = K.step_logprob(self.mode, x, eps, c.to(dev), noise=zero, noise_shared=True)
        return xf

    # ------------------------------------------------------------------------------------------------------------
    # BUFFER shuffle (T:733-749): pair permutation + independent per-pair transition permutation, written out in
    # micro-step order so every micro-step reads contiguous [2P] slices.
    # ------------------------------------------------------------------------------------------------------------
    def shuffle(self, buf, generator=None):
        dev = buf["x"].device
        n_img = buf["x"].shape[0]
        Bp = n_img // 2
        T, P = self.T, self.P
        assert Bp % P == 0, "samples per epoch must be a multiple of train.batch_size (T:521-523)"
        perm = torch.randperm(Bp, device=dev, generator=generator)
        perms = torch.argsort(torch.rand((Bp, T), device=dev, generator=generator), dim=1)  # per-pair time perm
        nb = Bp // P
        img_idx, pair_img, tsel_i = shuffle_index(perm, perms, P)
        tt = self.timesteps_dev[tsel_i]
        out = SimpleNamespace(n_micro=nb * T, P=P)
        flat = lambda t: t.reshape((n_img * T,) + tuple(t.shape[2:]))
        out.x = K.gather_rows(flat(buf["x"]), img_idx)
        out.x_next = K.gather_rows(flat(buf["x_next"]), img_idx)
        out.unet_in = K.gather_rows(flat(buf["unet_in"]), img_idx)
        out.enc = K.gather_rows(buf["enc"], pair_img)
        out.pooled = K.gather_rows(buf["pooled"], pair_img)
        out.tid = K.gather_rows(buf["tid"], pair_img)
        out.t = tt.float().contiguous()
        out.coef = K.gather_rows(self.coef_dev, tsel_i)               # per-image step coefficients
        rw = buf["rewards"]                                       # [Bp, 2, m]
        out.rewards = rw[perm[(torch.arange(nb, device=dev)[:, None] * P + torch.arange(P, device=dev)[None])]]
        out.rewards = out.rewards.reshape(nb, 1, P, 2, -1).expand(nb, T, P, 2, rw.shape[-1]).reshape(-1, 2,
                                                                                                   rw.shape[-1])
        out.rewards = out.rewards.contiguous()
        return out

    def micro_batch(self, sb, s, count=1):
        """Micro-steps [s, s + count) of the shuffled stream (contiguous rows: 2P images per micro-step)."""
        n = 2 * self.P
        sl = slice(s * n, (s + count) * n)
        return SimpleNamespace(x=sb.x[sl], x_next=sb.x_next[sl], unet_in=sb.unet_in[sl], enc=sb.enc[sl],
                               pooled=sb.pooled[sl], tid=sb.tid[sl], t=sb.t[sl], coef=sb.coef[sl],
                               rewards=sb.rewards[s * self.P:(s + count) * self.P], count=count)

    # ------------------------------------------------------------------------------------------------------------
    # MICRO-STEP (T:773-861) -- no host synchronisation
    # ------------------------------------------------------------------------------------------------------------
    def micro_step(self, mb, generator=None):
        """One micro-step, or -- when mb holds `count` consecutive micro-steps of ONE accumulation window -- all of
        them in a single batched pass.  Inside a window the LoRA weights do not change (the optimizer steps only at
        the window end, T:857-861), so the batched pass produces the sum of the per-micro-step gradients: every
        pair's loss term keeps its weight 1 / (P * gas * T) (the per-micro-step mean over P pairs, divided by the
        accumulation count as accelerate does).  Larger batches keep the MFMA GEMMs fed (M = images * tokens)."""
        count = getattr(mb, "count", 1)
        if self.n_micro // self.gas_total != (self.n_micro + count - 1) // self.gas_total:
            raise ValueError("a batched pass must not cross an optimizer step")
        P = self.P * count
        u = self.unet
        if self.ref_unet is not None:  # full-UNet training: policy pass + the frozen reference UNet's pass
            rs = _ref_stream() if _REF_STREAM and mb.unet_in.is_cuda else None
            if rs is not None:
                # the reference pass (different weights, same inputs, no saved state) on its own stream, beside the
                # policy pass: two grids of the small-M (6 images) GEMMs / attention fill the chip together
                main = torch.cuda.current_stream()
                rs.wait_stream(main)
                with torch.cuda.stream(rs), torch.no_grad():
                    eps_ref, _ = self.ref_unet.forward_nhwc(mb.unet_in, mb.t, mb.enc, mb.pooled, mb.tid, save=False)
                eps_pol, rt = u.forward_nhwc(mb.unet_in, mb.t, mb.enc, mb.pooled, mb.tid, save=True)
                main.wait_stream(rs)
                eps_ref.record_stream(main)
            else:
                eps_pol, rt = u.forward_nhwc(mb.unet_in, mb.t, mb.enc, mb.pooled, mb.tid, save=True)
                with torch.no_grad():
                    eps_ref, _ = self.ref_unet.forward_nhwc(mb.unet_in, mb.t, mb.enc, mb.pooled, mb.tid, save=False)
        else:
            u.enable_adapters()
            # policy (LoRA on, T:775-787) and reference (adapters disabled, T:790-805) eps of the same inputs in ONE pass
            eps_both, rt = u.forward_nhwc(mb.unet_in, mb.t, mb.enc, mb.pooled, mb.tid, save=True, paired_ref=True)
            n = mb.unet_in.shape[0]
            eps_pol, eps_ref = eps_both[:n], eps_both[n:]
        idx = None
        if self.mode == MODE_TURBO and self.m > 1:  # sample_compare draws a reward column per pair (T:405)
            idx = torch.randint(0, self.m, (P,), device=mb.x.device, generator=generator)
        pref = K.preference(mb.rewards, 0 if self.mode == MODE_TURBO else 1, reward_idx=idx)
        ws = K.pair_loss_ws(P, mb.x[0].numel(), mb.x.device)
        loss, lp = K.pair_loss_fwd(self.mode, mb.x, mb.x_next, eps_pol, eps_ref, mb.coef, pref, self.beta,
                                   self.clip_eps, ws)
        # accelerator.backward divides by gradient_accumulation_steps (accelerate accelerator.py:2840)
        deps = K.pair_loss_bwd(self.mode, mb.x, mb.x_next, eps_pol, mb.coef, pref, self.beta, self.clip_eps, ws,
                               grad_scale=count / self.gas_total)
        if self.overlap_sync and self.auto_step and (self.n_micro + count) % self.gas_total == 0:
            rt.unit_done = self.buckets.hook(rt)  # the window's last backward: overlap the gradient all-reduce
            self.sync_armed = True
        u.backward_nhwc(deps, rt)
        self.loss_hist.append(loss)  # mean over the pass's pairs = mean of its micro-step losses
        self.n_micro += count
        if self.auto_step and self.n_micro % self.gas_total == 0:
            self.optimizer_step()
        return loss

    # ------------------------------------------------------------------------------------------------------------
    # SYNC (T:857-861): all-reduce (RCCL) -> clip -> AdamW -> zero -> refresh bf16 working copies
    # ------------------------------------------------------------------------------------------------------------
    def optimizer_step(self):
        lora_optimizer_step(self)

    _SB_TENSORS = ("x", "x_next", "unet_in", "enc", "pooled", "tid", "t", "coef", "rewards")

    def train_epoch_graph(self, sb, generator=None):
        """train_epoch as ONE hipGraph replay (torch.cuda.CUDAGraph over the HIP runtime): the epoch's micro-steps --
        paired UNet pass, fused loss, backward into the flat LoRA grad bucket -- are captured on the first call and
        replayed afterwards, so the ~7k kernel launches of an epoch cost one graph launch instead of one host call
        each.  The shuffled buffer is copied into the graph's static input buffers first; the optimizer step (its
        AdamW step count is a host scalar) runs eagerly after the replay.  Requires: the epoch is exactly one
        accumulation window starting at a window boundary, and the turbo sampler draws no reward column (m = 1);
        otherwise this is train_epoch."""
        if (sb.n_micro != self.gas_total or self.n_micro % self.gas_total or not self.auto_step
                or (self.mode == MODE_TURBO and self.m > 1)):
            return self.train_epoch(sb, generator)
        if getattr(self.unet, "full", None) is not None:
            # full-UNet training: the optimizer step rebuilds the kernel-layout weight caches as new tensors
            # (refresh_full -> prepare), which a captured graph would keep reading at their old addresses
            return self.train_epoch(sb, generator)
        key = tuple((k, tuple(getattr(sb, k).shape)) for k in self._SB_TENSORS)
        g = getattr(self, "_graph", None)
        if g is None or self._graph_key != key:
            self._graph = None
            # no collective inside the captured region: the step's all-reduce is eager.  Only the warm-up and the
            # capture run without the overlapped bucketed sync; eager epochs afterwards get it back (finally below).
            overlap0, self.overlap_sync = self.overlap_sync, False
            self._gsb = SimpleNamespace(n_micro=sb.n_micro, P=sb.P,
                                        **{k: getattr(sb, k).clone() for k in self._SB_TENSORS})
            _, st_grad, _ = trainable(self.unet)
            saved = st_grad.clone()
            self.auto_step = False
            n0, h0 = self.n_micro, len(self.loss_hist)
            try:
                self.train_epoch(self._gsb)  # eager warm-up of everything the capture will launch
                torch.cuda.synchronize()
                h1 = len(self.loss_hist)
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g):
                    self.train_epoch(self._gsb)
                self._gloss = self.loss_hist[h1:]
            finally:
                self.auto_step = True
                self.overlap_sync = overlap0
                self.n_micro = n0
                del self.loss_hist[h0:]
                st_grad.copy_(saved)
            self._graph, self._graph_key = g, key
        for k in self._SB_TENSORS:
            getattr(self._gsb, k).copy_(getattr(sb, k))
        self._graph.replay()
        self.loss_hist.extend(l.clone() for l in self._gloss)
        self.n_micro += sb.n_micro
        self.optimizer_step()

    def train_epoch(self, sb, generator=None):
        """One inner epoch over a shuffled buffer: every micro-step in order (T:755-861), batched per accumulation
        window up to `max_pass_images` images per UNet pass.  Python's cyclic garbage collector is paused for the
        epoch (PSO_GC_PAUSE=0 keeps it running): the ~3k kernel launches of a step allocate enough small objects to
        trigger collections in the middle of launch-bound stretches."""
        gc_on = _GC_PAUSE and gc.isenabled()
        if gc_on:
            gc.disable()
        try:
            self._train_epoch(sb, generator)
        finally:
            if gc_on:
                gc.enable()

    def _train_epoch(self, sb, generator=None):
        s = 0
        per_pass = max(1, self.max_pass_images // (2 * self.P))
        while s < sb.n_micro:
            left_in_window = self.gas_total - self.n_micro % self.gas_total
            c = min(per_pass, left_in_window, sb.n_micro - s)
            self.micro_step(self.micro_batch(sb, s, c), generator=generator)
            s += c
