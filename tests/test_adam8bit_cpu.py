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


def _filled_state(segs, n, seed):
    """A per-tensor Adam8State with random codes, block absmax and 32-bit moments (host tensors)."""
    import torch
    from pairwise_sample_optimization_amd import kernels as K
    st = K.Adam8State(n, torch.device("cpu"), segments=segs)
    g = torch.Generator().manual_seed(seed)
    st.qm.copy_(torch.randint(0, 256, (n,), generator=g, dtype=torch.uint8))
    st.qv.copy_(torch.randint(0, 256, (n,), generator=g, dtype=torch.uint8))
    st.am.copy_(torch.rand(st.am.shape, generator=g) + 0.1)
    st.av.copy_(torch.rand(st.av.shape, generator=g) + 0.1)
    st.m32.copy_(torch.randn(st.m32.shape, generator=g))
    st.v32.copy_(torch.rand(st.v32.shape, generator=g))
    return st


def test_dequant_vectorised_equals_row_loop_and_load_dense_roundtrips():
    """Adam8State.dequant is vectorised over slices of the block table (full-UNet mode: ~1.25M rows).  It
    equals the per-row definition; elements outside every tensor read 0; quantising the dequantised moments back
    (load_dense: per-block absmax, nearest code) returns the same 32-bit moments and, for every block whose largest
    code is +-1 (the kernel's invariant after an update), the same absmax and codes."""
    import torch
    from pairwise_sample_optimization_amd import kernels as K
    sizes = [5000, 1000, 4096, 4095, 20480, 64, 2049, 320]
    segs, off = [], 0
    for k in sizes:
        segs.append((off, k))
        off += -(-k // 64) * 64
    n = off
    st = _filled_state(segs, n, 0)
    K.Adam8State._CHUNK_ROWS = 3  # several slices even at this size
    try:
        m, v = st.dequant()
        cs, cu = K.Adam8State.maps(torch.device("cpu"))
        m_ref, v_ref = torch.zeros(n), torch.zeros(n)
        for b, (o, k, so, _) in enumerate(st.rows):
            if so >= 0:
                m_ref[o:o + k], v_ref[o:o + k] = st.m32[so:so + k], st.v32[so:so + k]
            else:
                m_ref[o:o + k] = cs[st.qm[o:o + k].long()] * st.am[b]
                v_ref[o:o + k] = cu[st.qv[o:o + k].long()] * st.av[b]
        assert torch.equal(m, m_ref) and torch.equal(v, v_ref)
        # the kernel's invariant: each 8-bit block's largest |code| is 1 (its absmax element)
        for b, (o, k, so, _) in enumerate(st.rows):
            if so < 0:
                st.qm[o] = int(torch.argmax(cs))
                st.qv[o] = int(torch.argmax(cu))
        m, v = st.dequant()
        st2 = K.Adam8State(n, torch.device("cpu"), segments=segs)
        st2.load_dense(m, v)
        m2, v2 = st2.dequant()
        for (o, k, so, _) in st.rows:
            if so >= 0:  # the used 32-bit slots (the 8-aligned slot tails are never read)
                assert torch.equal(st2.m32[so:so + k], st.m32[so:so + k])
                assert torch.equal(st2.v32[so:so + k], st.v32[so:so + k])
        eight = torch.tensor([so < 0 for (_, _, so, _) in st.rows])
        assert torch.equal(st2.am[eight], st.am[eight]) and torch.equal(st2.av[eight], st.av[eight])
        assert torch.equal(m2, m) and torch.equal(v2, v)
    finally:
        K.Adam8State._CHUNK_ROWS = 16384


def test_legacy_uniform_checkpoint_requantised_on_load(tmp_path, monkeypatch):
    """an 8-bit AdamW checkpoint of the uniform-block format (no block_table) loads into a per-tensor
    trainer with a warning, its moments re-quantised into the per-tensor blocks (within the 8-bit code spacing)."""
    import json
    import os
    import warnings
    from types import SimpleNamespace
    import torch
    from safetensors.torch import save_file
    from pairwise_sample_optimization_amd import kernels as K, lora_io
    sizes = [5000, 4096, 20480]
    segs, off = [], 0
    for k in sizes:
        segs.append((off, k))
        off += -(-k // 64) * 64
    n = off
    old = K.Adam8State(n, torch.device("cpu"))
    g = torch.Generator().manual_seed(1)
    old.qm.copy_(torch.randint(0, 256, (n,), generator=g, dtype=torch.uint8))
    old.qv.copy_(torch.randint(0, 256, (n,), generator=g, dtype=torch.uint8))
    old.am.copy_(torch.rand(old.am.shape, generator=g) + 0.1)
    old.av.copy_(torch.rand(old.av.shape, generator=g) + 0.1)
    pads = torch.ones(n, dtype=torch.bool)
    for o, k in segs:
        pads[o:o + k] = False
    old.qm[pads] = 127  # the pads of an old checkpoint hold zero moments (code of 0.0)
    save_file({k: v for k, v in old.tensors().items()}, os.path.join(tmp_path, lora_io.OPT_NAME))
    with open(os.path.join(tmp_path, "pso_state.json"), "w") as f:
        json.dump({"opt_step": 7, "n_micro": 14, "rank": 8}, f)
    tr = SimpleNamespace(adam8=K.Adam8State(n, torch.device("cpu"), segments=segs), unet=None, opt_step=0, n_micro=0)
    monkeypatch.setattr(lora_io, "load_lora_into_unet", lambda *a, **k: None)  # the LoRA file is not tested here
    monkeypatch.setattr(lora_io, "lora_state_dict", lambda d: ({}, None))
    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter("always")
        lora_io.load_state(tr, str(tmp_path))
    assert any("block table" in str(x.message) for x in w)
    assert tr.opt_step == 7 and tr.n_micro == 14
    m0, v0 = old.dequant()
    m1, v1 = tr.adam8.dequant()
    keep = ~pads
    assert (m1[keep] - m0[keep]).abs().max() <= 0.1 * m0[keep].abs().max()
    assert ((m1[keep] - m0[keep]).norm() / m0[keep].norm()).item() < 0.05
    assert ((v1[keep] - v0[keep]).norm() / v0[keep].norm()).item() < 0.05
