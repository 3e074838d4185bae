"""TEST INFRASTRUCTURE ONLY (oracle): numpy restatement of bitsandbytes' blockwise 8-bit AdamW (`bnb.optim.AdamW8bit`,
the reference's default optimizer: `config.train.use_8bit_adam = True`, config_sdxl_turbo_dpo.py:86, selected at
T:427-435 / D:451-459).  Imported only by tests/.

PARITY UNPINNED: bitsandbytes is not installed in this image (and the reference pins no version of it, nor holds any
fixture of its optimizer); this restates the published algorithm (bitsandbytes `functional.create_dynamic_map` and the
`kOptimizerStatic8bit2StateBlockwise` ADAM update) from its documentation and source as the builder knows it:

  * state: m and v as uint8 codes into two 256-entry "dynamic" quantisation maps (signed for m, unsigned for v) plus
    one fp32 absmax per block of 2048 elements per state; zero-initialised (every code -> 0.0 after dequantisation);
  * step t (g already scaled):  m = map_s[qm] * absmax_m ;  v = map_u[qv] * absmax_v   (the previous step's absmax)
                                m = b1 m + (1 - b1) g ;     v = b2 v + (1 - b2) g^2
                                c1 = 1 - b1^t ; c2 = sqrt(1 - b2^t)
                                p = p - lr * c2 / c1 * m / (sqrt(v) + c2 * eps)      then   p *= (1 - lr * wd)
                                absmax' = max over the block of |m| (|v|);  q = nearest code of m / absmax' (v / ...)
  * bitsandbytes quantises every parameter tensor on its own: the 2048-blocks restart at each tensor (the last one
    partial), and tensors below 4096 elements (`min_8bit_size`) keep 32-bit m / v with the same update
    (kOptimizer32bit2State) -- `adamw8bit_step_tensors` restates that over a flat buffer and its tensor list;
  * non-finite gradient elements: bitsandbytes skips their parameter update; here they leave p, m and v unchanged
    (what bitsandbytes does to their state is not restated);
  * the 2048-element block follows bitsandbytes' BLOCKSIZE_2STATE of the releases of the reference's time (the
    reference pins no version; later releases may use other block sizes).
"""
import numpy as np

BLOCK = 2048


def create_dynamic_map(signed=True, max_exponent_bits=7, total_bits=8):
    """bitsandbytes.functional.create_dynamic_map: an exponent of 10 that shrinks the fraction's bits as it grows,
    the fraction's codes at the midpoints of a linear grid on [0.1, 1]; plus 0 and 1.0; sorted (float32)."""
    data = []
    non_sign_bits = total_bits - 1
    additional_items = 2 ** (non_sign_bits - max_exponent_bits) - 1
    i = 0
    for i in range(max_exponent_bits):
        n = int(2 ** (i + non_sign_bits - max_exponent_bits) + 1 if signed
                else 2 ** (i + non_sign_bits - max_exponent_bits + 1) + 1)
        b = np.linspace(0.1, 1, n, dtype=np.float32)
        means = (b[:-1] + b[1:]) / np.float32(2.0)
        data += (np.float32(10 ** (-(max_exponent_bits - 1) + i)) * means).tolist()
        if signed:
            data += (-np.float32(10 ** (-(max_exponent_bits - 1) + i)) * means).tolist()
    if additional_items > 0:
        b = np.linspace(0.1, 1, additional_items + 1, dtype=np.float32)
        means = (b[:-1] + b[1:]) / np.float32(2.0)
        data += (np.float32(10 ** (-(max_exponent_bits - 1) + i)) * means).tolist()
        if signed:
            data += (-np.float32(10 ** (-(max_exponent_bits - 1) + i)) * means).tolist()
    data.append(0.0)
    data.append(1.0)
    assert len(data) == 2 ** total_bits
    data += [0.0] * (256 - len(data))
    return np.array(sorted(data), dtype=np.float32)


def quantize_nearest(x, code):
    """Index of the nearest code (ties to the lower index); x already divided by the block absmax."""
    idx = np.searchsorted(code, x, side="left")
    idx = np.clip(idx, 1, len(code) - 1)
    lo, hi = code[idx - 1], code[idx]
    return np.where(np.abs(x - lo) <= np.abs(hi - x), idx - 1, idx).astype(np.uint8)


def adamw8bit_step(p, g, qm, qv, am, av, lr, b1, b2, eps, wd, step):
    """One blockwise 8-bit AdamW step on flat fp32 arrays (n % BLOCK == 0).  Returns new (p, qm, qv, am, av)."""
    cs, cu = create_dynamic_map(True), create_dynamic_map(False)
    n = p.size
    nb = n // BLOCK
    p, g = p.astype(np.float32), g.astype(np.float32)
    m = cs[qm].reshape(nb, BLOCK) * am[:, None]
    v = cu[qv].reshape(nb, BLOCK) * av[:, None]
    gb = g.reshape(nb, BLOCK)
    m = np.float32(b1) * m + np.float32(1 - b1) * gb
    v = np.float32(b2) * v + np.float32(1 - b2) * gb * gb
    c1 = np.float32(1 - b1 ** step)
    c2 = np.float32(np.sqrt(1 - b2 ** step))
    step_size = np.float32(-lr) * c2 / c1
    pb = p.reshape(nb, BLOCK) + step_size * (m / (np.sqrt(v) + c2 * np.float32(eps)))
    pb = pb * np.float32(1 - lr * wd)
    am2 = np.abs(m).max(1).astype(np.float32)
    av2 = np.abs(v).max(1).astype(np.float32)
    sm = np.where(am2[:, None] > 0, m / np.where(am2 > 0, am2, 1)[:, None], 0)
    sv = np.where(av2[:, None] > 0, v / np.where(av2 > 0, av2, 1)[:, None], 0)
    qm2 = quantize_nearest(sm.reshape(-1), cs)
    qv2 = quantize_nearest(sv.reshape(-1), cu)
    return pb.reshape(-1), qm2, qv2, am2, av2


def _adam_update(p, m, v, g, lr, b1, b2, eps, wd, step):
    """The element update of both bitsandbytes kernels (fp32), where g is finite; returns (p, m, v)."""
    f = np.float32
    ok = np.isfinite(g)
    gz = np.where(ok, g, f(0))
    m2 = f(b1) * m + f(1 - b1) * gz
    v2 = f(b2) * v + f(1 - b2) * gz * gz
    c1 = f(1 - b1 ** step)
    c2 = f(np.sqrt(1 - b2 ** step))
    step_size = f(-lr) * c2 / c1
    p2 = (p + step_size * (m2 / (np.sqrt(v2) + c2 * f(eps)))) * f(1 - lr * wd)
    return np.where(ok, p2, p).astype(f), np.where(ok, m2, m).astype(f), np.where(ok, v2, v).astype(f)


MIN_8BIT_SIZE = 4096


def adamw8bit_step_tensors(p, g, segments, state, lr, b1, b2, eps, wd, step):
    """One AdamW8bit step over the parameter tensors segments = [(offset, numel)] of the flat fp32 buffers p / g, as
    bitsandbytes runs it on a list of tensors (T:428-448).  state: dict offset -> per-tensor state, created on the
    first call ({"m32", "v32"} under MIN_8BIT_SIZE, else {"qm", "qv", "am", "av"} with ceil(numel / BLOCK) blocks, the
    last one partial).  Returns the new p (state updated in place)."""
    cs, cu = create_dynamic_map(True), create_dynamic_map(False)
    p = p.astype(np.float32).copy()
    g = g.astype(np.float32)
    for off, k in segments:
        pt, gt = p[off:off + k], g[off:off + k]
        if k < MIN_8BIT_SIZE:
            st = state.setdefault(off, {"m32": np.zeros(k, np.float32), "v32": np.zeros(k, np.float32)})
            p[off:off + k], st["m32"], st["v32"] = _adam_update(pt, st["m32"], st["v32"], gt, lr, b1, b2, eps, wd, step)
            continue
        nb = -(-k // BLOCK)
        st = state.setdefault(off, {"qm": np.zeros(k, np.uint8), "qv": np.zeros(k, np.uint8),
                                    "am": np.zeros(nb, np.float32), "av": np.zeros(nb, np.float32)})
        for b in range(nb):
            sl = slice(b * BLOCK, min(k, (b + 1) * BLOCK))
            m = cs[st["qm"][sl]] * st["am"][b]
            v = cu[st["qv"][sl]] * st["av"][b]
            pb, m, v = _adam_update(pt[sl], m, v, gt[sl], lr, b1, b2, eps, wd, step)
            p[off + sl.start:off + sl.stop] = pb
            am, av = np.float32(np.abs(m).max()), np.float32(np.abs(v).max())
            st["am"][b], st["av"][b] = am, av
            st["qm"][sl] = quantize_nearest(m / am if am > 0 else np.zeros_like(m), cs)
            st["qv"][sl] = quantize_nearest(v / av if av > 0 else np.zeros_like(v), cu)
    return p
