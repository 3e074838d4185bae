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
  * tensors below 4096 elements keep 32-bit state in bitsandbytes (`min_8bit_size`); every LoRA tensor of the SDXL
    UNet is larger (r * 640 >= 10240) and a multiple of 2048, so blocks of the flat LoRA buffer never straddle two
    tensors.
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
