"""CPU checks of the AdamW8bit restatement (oracle/adam8bit.py) and of the host-side block table of K.Adam8State's
per-tensor form (bitsandbytes semantics, T:428-448).  Parity unpinned: bitsandbytes is not installed."""
import numpy as np

from oracle import adam8bit as O


def _f32(x):
    return float(np.float32(x))


def test_per_tensor_restatement_equals_uniform_on_whole_blocks():
    """One tensor whose size is a multiple of 2048: the per-tensor restatement is the uniform-block one."""
    n = 2048 * 6
    rng = np.random.default_rng(0)
    p = (rng.standard_normal(n) * 0.02).astype(np.float32)
    qm, qv = np.zeros(n, np.uint8), np.zeros(n, np.uint8)
    am, av = np.zeros(n // 2048, np.float32), np.zeros(n // 2048, np.float32)
    pt, st = p.copy(), {}
    hp = dict(lr=_f32(1e-3), b1=_f32(0.9), b2=_f32(0.999), eps=_f32(1e-8), wd=_f32(1e-2))
    for step in range(1, 4):
        g = (rng.standard_normal(n) * 1e-2).astype(np.float32)
        p, qm, qv, am, av = O.adamw8bit_step(p, g, qm, qv, am, av, step=step, **hp)
        pt = O.adamw8bit_step_tensors(pt, g, [(0, n)], st, step=step, **hp)
    assert np.array_equal(p, pt)
    assert np.array_equal(qm, st[0]["qm"]) and np.array_equal(am, st[0]["am"])


def test_small_tensor_keeps_32bit_state_and_nonfinite_is_skipped():
    rng = np.random.default_rng(1)
    k = 1000
    p = (rng.standard_normal(k) * 0.02).astype(np.float32)
    st = {}
    hp = dict(lr=_f32(1e-3), b1=_f32(0.9), b2=_f32(0.999), eps=_f32(1e-8), wd=_f32(1e-2))
    g = (rng.standard_normal(k) * 1e-3).astype(np.float32)
    g[7] = np.nan
    p1 = O.adamw8bit_step_tensors(p, g, [(0, k)], st, step=1, **hp)
    assert set(st[0]) == {"m32", "v32"}
    assert p1[7] == p[7] and st[0]["m32"][7] == 0 and st[0]["v32"][7] == 0
    # the first Adam step moves every other parameter by ~lr (m / sqrt(v) = sign(g))
    moved = np.abs(p1 - p * np.float32(1 - 1e-5))
    assert np.all(np.delete(moved, 7) > 0.5e-3)


def test_block_table_follows_tensors():
    """K.Adam8State(segments=...) builds the per-tensor block table on the host (no GPU call)."""
    import torch
    from pairwise_sample_optimization_amd import kernels as K
    segs = [(0, 5000), (5056, 1000), (6080, 4096)]
    st = K.Adam8State(10176, torch.device("cpu"), segments=segs)
    assert st.rows == [(0, 2048, -1, 0), (2048, 2048, -1, 0), (4096, 904, -1, 0), (5056, 1000, 0, 0),
                       (6080, 2048, -1, 0), (8128, 2048, -1, 0)]
    assert st.nblk == 6 and st.m32.numel() == 1000
