"""Bit-compare the GroupNorm passes of two builds of the library (e.g. the in-tree one and a previous norm.hip linked
into prev/libpso_amd_prev.so): same inputs, every output (y, stats, dx, dgamma, dbeta) must be byte-identical.
usage (GPU): python tools/norm_bits_check.py [other_lib]"""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from pairwise_sample_optimization_amd import _lib  # noqa: E402


def bind(path):
    lib = ctypes.CDLL(path)
    vp, ci, cf, sz = ctypes.c_void_p, ctypes.c_int, ctypes.c_float, ctypes.c_size_t
    lib.pso_group_norm_ws_bytes.restype = sz
    lib.pso_group_norm_ws_bytes.argtypes = [ci, ci, ci]
    lib.pso_group_norm_fwd.argtypes = [ci, ci, ci, ci, cf, vp, vp, vp, ci, vp, vp, vp, sz, vp]
    lib.pso_group_norm_bwd.argtypes = [ci, ci, ci, ci, vp, vp, vp, vp, vp, ci, vp, vp, vp, vp, ci, vp, sz, vp]
    return lib


def run(lib, x, gm, bt, dy, dadd, silu, dparam):
    B, H, W, C = x.shape
    HW, G = H * W, 32
    s = torch.cuda.current_stream().cuda_stream
    wsb = lib.pso_group_norm_ws_bytes(B, HW, C)
    ws = torch.zeros(wsb, device=x.device, dtype=torch.uint8)
    y = torch.empty_like(x)
    st = torch.empty((B, G, 2), device=x.device, dtype=torch.float32)
    assert lib.pso_group_norm_fwd(B, HW, C, G, 1e-5, x.data_ptr(), gm.data_ptr(), bt.data_ptr(), int(silu),
                                  y.data_ptr(), st.data_ptr(), ws.data_ptr(), wsb, s) == 0
    dx = torch.empty_like(x)
    dg = torch.zeros(C, device=x.device) if dparam else None
    db = torch.zeros(C, device=x.device) if dparam else None
    assert lib.pso_group_norm_bwd(B, HW, C, G, x.data_ptr(), dy.data_ptr(), st.data_ptr(), gm.data_ptr(), bt.data_ptr(),
                                  int(silu), dadd.data_ptr() if dadd is not None else None, dx.data_ptr(),
                                  dg.data_ptr() if dparam else None, db.data_ptr() if dparam else None, 0,
                                  ws.data_ptr(), wsb, s) == 0
    torch.cuda.synchronize()
    return [y, st, dx] + ([dg, db] if dparam else [])


def main():
    other = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "prev", "libpso_amd_prev.so")
    a, b = bind(_lib.LIB_PATH), bind(other)
    dev = torch.device("cuda")
    bad = 0
    for (B, H, C, silu, dadd, dparam) in [(16, 128, 320, True, False, False), (16, 64, 640, True, True, False),
                                          (16, 32, 1280, True, False, True), (8, 64, 640, True, True, True),
                                          (16, 64, 640, False, False, False), (8, 128, 640, True, False, False),
                                          (2, 16, 2560, True, True, True), (1, 256, 128, True, False, True),
                                          (3, 20, 320, False, True, False)]:
        g = torch.Generator(device="cuda").manual_seed(B * 1000 + H + C)
        x = (torch.randn(B, H, H, C, device=dev, generator=g) * 2 + 0.3).bfloat16()
        gm = (1 + 0.1 * torch.randn(C, device=dev, generator=g)).bfloat16()
        bt = (0.1 * torch.randn(C, device=dev, generator=g)).bfloat16()
        dy = torch.randn(B, H, H, C, device=dev, generator=g).bfloat16()
        da = torch.randn(B, H, H, C, device=dev, generator=g).bfloat16() if dadd else None
        ra = run(a, x, gm, bt, dy, da, silu, dparam)
        rb = run(b, x, gm, bt, dy, da, silu, dparam)
        same = [torch.equal(p, q) for p, q in zip(ra, rb)]
        bad += not all(same)
        print(f"B{B} {H}x{H}x{C} silu={int(silu)} dadd={int(dadd)} dparam={int(dparam)}: "
              f"{'identical' if all(same) else 'DIFFER ' + str(same)}", flush=True)
    print("ALL IDENTICAL" if bad == 0 else f"{bad} shapes differ")
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
