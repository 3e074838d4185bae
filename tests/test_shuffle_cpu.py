"""The trainer's shuffle index math (one gather per tensor on device) against the numpy restatement of the
reference shuffle T:733-760, on identical permutations."""
import numpy as np
import pytest
import torch


@pytest.mark.parametrize("Bp,T,P", [(4, 3, 1), (8, 3, 2), (6, 1, 2), (16, 3, 4)])
def test_shuffle_index_matches_reference(Bp, T, P):
    from oracle.shuffle import reference_shuffle
    from pairwise_sample_optimization_amd.trainer import shuffle_index
    g = torch.Generator().manual_seed(Bp * 100 + T * 10 + P)
    perm = torch.randperm(Bp, generator=g)
    perms = torch.stack([torch.randperm(T, generator=g) for _ in range(Bp)])
    lat = torch.randn(Bp, 2, T, 4, 3, 3, generator=g)   # buffer layout [pair, member, transition, C, h, w]
    ts = torch.arange(T, dtype=torch.float32).view(1, 1, T).expand(Bp, 2, T).contiguous()
    ref = reference_shuffle({"latents": lat.numpy(), "timesteps": ts.numpy()}, perm.numpy(), perms.numpy(), P)
    img_idx, pair_img, tsel = shuffle_index(perm, perms, P)
    flat = lat.reshape(Bp * 2 * T, 4, 3, 3)
    n = 2 * P
    assert len(ref) == (Bp // P) * T
    for s, mstep in enumerate(ref):
        rows = img_idx[s * n:(s + 1) * n].view(P, 2)
        got = flat[rows]                               # [P, 2, C, h, w]
        np.testing.assert_array_equal(got[:, 0].numpy(), mstep["latents"][0])
        np.testing.assert_array_equal(got[:, 1].numpy(), mstep["latents"][1])
        np.testing.assert_array_equal(tsel[s * n:(s + 1) * n].view(P, 2)[:, 0].float().numpy(), mstep["timesteps"][0])
        # per-pair tensors (prompt embeds) follow the pair permutation
        assert torch.equal(pair_img[s * n:(s + 1) * n].view(P, 2) // 2, rows // (2 * T))
