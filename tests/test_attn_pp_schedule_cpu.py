"""Model check of the ping-pong dK/dV kernel's barrier / ring protocol (attention.hip, attn_bwd_dkv_pp_kernel).

The kernel's two wave groups run the same loop one barrier apart; a mismatch in their s_barrier counts hangs the GPU,
and an early slot re-stage or a short vmcnt silently corrupts dK / dV.  This restates the loop's control flow (issue
points, counted waits, segment reads) as data and checks, for the ring depths the kernel allows (3, 4) and every
tile count up to 16:
  * both groups execute the same number of barriers;
  * every tile's LDS-DMA pieces are waited for (by every wave) at or before the barrier that opens the first segment
    in which either group reads that tile;
  * a slot is re-staged only after the last segment that reads its previous tile;
  * the vmcnt tile count the kernel passes to att_wait_barrier equals the tiles issued after the awaited one
    (and stays within the 3 the helper encodes);
  * every tile is issued by both groups.
"""
import pytest


def program(grp, n, stg):
    """The loop of attn_bwd_dkv_pp_kernel for one group: a list of events ('issue', t) / ('bar', awaited tile or None,
    newer-tile count passed to att_wait_barrier or None) / ('read', t)."""
    ev = [("issue", t) for t in range(min(stg, n))]
    if grp:
        ev.append(("bar", 0 if n > 0 else None, min(n - 1, stg - 1) if n > 0 else None))
    t = 0
    while True:
        if not grp and t < n:
            ev.append(("bar", t, min(n - 1, max(stg - 1, t + stg - 3)) - t))
        else:
            ev.append(("bar", None, None))
        if not grp and t >= 2 and t + stg - 2 < n:
            ev.append(("issue", t + stg - 2))
        if t > 0:
            ev.append(("read", t - 1))  # dV / dK of the previous tile (transposed reads issued in its B segment)
        if t == n:
            break
        ev.append(("read", t))  # S / dP: row and delta reads
        if grp:
            ev.append(("bar", t + 1 if t + 1 < n else None,
                       min(n - 1, max(stg - 1, t + stg - 2)) - (t + 1) if t + 1 < n else None))
        else:
            ev.append(("bar", None, None))
        if grp and t >= 1 and t + stg - 1 < n:
            ev.append(("issue", t + stg - 1))
        ev.append(("read", t))  # LSE reads + the transposed reads of tile t for the next A segment
        t += 1
    if not grp:
        ev.append(("bar", None, None))
    return ev


@pytest.mark.parametrize("stg", [3, 4])
def test_pp_protocol(stg):
    for n in range(0, 17):
        progs = [program(0, n, stg), program(1, n, stg)]
        nbar = [sum(1 for e in p if e[0] == "bar") for p in progs]
        assert nbar[0] == nbar[1], (stg, n, nbar)
        waited, issued_at, first_read, last_read = {}, {}, {}, {}
        for gi, p in enumerate(progs):
            k = -1  # segment index = number of barriers passed - 1 (global: both groups count the same barriers)
            issued = []
            waited[gi], issued_at[gi] = {}, {}
            for e in p:
                if e[0] == "bar":
                    k += 1
                    if e[1] is not None:
                        newer = sum(1 for x in issued if x > e[1])
                        assert newer == e[2], (stg, n, gi, e, newer)
                        assert 0 <= e[2] <= 3
                        for tt in range(e[1] + 1):  # in-order completion: everything up to the awaited tile
                            waited[gi].setdefault(tt, k)
                elif e[0] == "issue":
                    issued.append(e[1])
                    issued_at[gi][e[1]] = k
                else:
                    first_read[e[1]] = min(first_read.get(e[1], 10 ** 9), k)
                    last_read[e[1]] = max(last_read.get(e[1], -1), k)
            assert sorted(issued) == list(range(n)), (stg, n, gi)
        for tt in range(n):
            for gi in (0, 1):
                assert waited[gi][tt] <= first_read[tt], (stg, n, tt, gi)
        for tt in range(n - stg):
            for gi in (0, 1):
                assert issued_at[gi][tt + stg] > last_read[tt], (stg, n, tt, gi)
