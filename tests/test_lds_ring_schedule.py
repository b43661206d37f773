"""The coarse-plane LDS ring of mz_prolong_sweep_lds_kernel (csrc/amg_kernels.hip),
emulated on the host: with the kernel's schedule -- coarse planes (k0 >> 1) - 1
.. (k0 >> 1) + 1 + (k0 & 1) loaded before the march, plane (k >> 1) + 2 fetched
at every even step k and stored at its end, published by the barrier of the
next even step -- every coarse plane a fine plane's prolongation reads (the own
lines' plane k + 2, the halo lines' plane k, the initial planes k0 - 1 .. k0 + 1)
sits in its slot (c & 3) when read, and no store overwrites a slot a step still
reads.  Chunk lengths 2..64 from odd and even chunk starts."""
import pytest


def coarse_planes(z, ncz):
    """coarse planes fine plane z reads (geo_prolong_pair's z candidates)"""
    if z & 1:
        return [(z - 1) >> 1]
    out = []
    if z >= 2:
        out.append((z >> 1) - 1)
    if (z >> 1) < ncz:
        out.append(z >> 1)
    return out


@pytest.mark.parametrize("nz", [4, 6, 10, 16, 64])
@pytest.mark.parametrize("zc", [2, 3, 4, 5, 8, 64])
def test_lds_ring_schedule(nz, zc):
    ncz = nz // 2
    for k0 in range(0, nz, zc):
        k1 = min(k0 + zc, nz)
        vis, pend = {}, {}
        for c in range((k0 >> 1) - 1, (k0 >> 1) + 2 + (k0 & 1)):
            vis[c & 3] = c

        def read(z):
            if 0 <= z < nz:
                for c in coarse_planes(z, ncz):
                    assert vis.get(c & 3) == c, (nz, zc, k0, z, c)

        for z in (k0 - 1, k0, k0 + 1):
            read(z)
        fetch = None
        for k in range(k0, k1):
            if k % 2 == 0:
                if k != k0:
                    vis.update(pend)
                    pend = {}
                fetch = (k >> 1) + 2
            if k + 2 < nz and k + 1 < k1:
                read(k + 2)
            read(k)
            if k % 2 == 0:
                slot = fetch & 3
                for kk in (k, k + 1):  # steps that may still read when the store lands
                    for z in (kk, kk + 2):
                        if 0 <= z < nz:
                            assert all(c & 3 != slot or c == fetch for c in coarse_planes(z, ncz))
                pend[slot] = fetch
