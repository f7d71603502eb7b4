"""The fused plan launch's workgroup map (fsst.hip fsst_k1g_kernel, launch_fsst_k1g), restated
on the host: the T FSST decode tiles are spread evenly over the first M = T + G * pct / 100
workgroups of a T + G grid (workgroup b < M is tile floor(b T / M) where that floor steps at b),
the other workgroups are the K1g workgroups in order.  Every tile and every K1g workgroup must
be covered exactly once, for every VXG_FUSED_MIX percentage and edge size (no GPU needed)."""
import pytest


def fused_map(b, T, M):
    if b < M:
        d0, d1 = b * T // M, (b + 1) * T // M
        if d1 > d0:
            return "tile", d0
        return "k1g", b - d1
    return "k1g", b - T


@pytest.mark.parametrize("T,G", [(1, 0), (5, 0), (1, 1), (3, 7), (2930, 915), (23443, 7325), (7, 3), (1000, 1)])
@pytest.mark.parametrize("pct", [0, 1, 50, 100])
def test_fused_map_covers_every_tile_and_job_once(T, G, pct):
    M = T + G * pct // 100
    tiles, jobs = [], []
    for b in range(T + G):
        kind, i = fused_map(b, T, M)
        (tiles if kind == "tile" else jobs).append(i)
    assert sorted(tiles) == list(range(T))
    assert sorted(jobs) == list(range(G))
    # tiles in increasing order of workgroup (their records are read in dispatch order)
    assert tiles == sorted(tiles)
