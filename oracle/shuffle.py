"""TEST INFRASTRUCTURE ONLY (imported by tests/, never by the product path).

numpy restatement of the reference's per-epoch shuffle and re-batching, `T:733-760` (turbo) / `D:719-753` (DMD2):
pair permutation along the batch, an independent time permutation per (shuffled) sample shared by both members, then
micro-steps in order (batch i, then transition j).  perm / perms are inputs so the product's index math can be
compared on identical permutations (the RNG streams cannot match).
"""
import numpy as np


def reference_shuffle(samples, perm, perms, batch_size):
    """samples: dict of arrays shaped [Bp, 2, T, ...] (latents/next_latents/input_latents) or [Bp, 2, T]
    (timesteps, log_probs).  Returns a list over micro-steps of {key: (member0 [P,...], member1 [P,...])}."""
    Bp = perm.shape[0]
    T = perms.shape[1]
    s = {k: v[perm] for k, v in samples.items()}                          # T:734-735
    rows = np.arange(Bp)[:, None]
    for k in list(s):
        v = s[k]
        moved = np.moveaxis(v, 1, -1)                                      # [Bp, T, ..., 2]
        s[k] = np.moveaxis(moved[rows, perms], -1, 1)                      # T:738-745
    out = []
    for i in range(0, Bp, batch_size):                                     # T:755-
        for j in range(T):
            out.append({k: (v[i:i + batch_size, 0, j], v[i:i + batch_size, 1, j]) for k, v in s.items()})
    return out
