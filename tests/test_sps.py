"""Stochastic parallel Southwell gating (-smoother async_sps) host pieces: the
RandDouble stream the decisions draw from (Misc.cpp:282-285 over glibc rand()
after srand(seed)) pinned against this host's own libc, and the update
probability (DMEM_Smooth.cpp:548-572) restated for the GPU tests."""
import ctypes
import math

import numpy as np
import pytest


@pytest.mark.parametrize("seed", [0, 1, 7, 12345, 2 ** 31 - 2])
def test_rand_stream_matches_libc(amg, seed):
    libc = ctypes.CDLL("libc.so.6")
    libc.rand.restype = ctypes.c_int
    libc.srand(ctypes.c_uint(seed))
    n = 2000
    ref = np.array([libc.rand() for _ in range(n)], dtype=np.float64) / 2147483647.0
    got = amg.rand_double_stream(seed, n)
    assert np.array_equal(got, ref)
    lo, hi = -3.0, 5.0
    got2 = amg.rand_double_stream(seed, 10, lo, hi)
    np.testing.assert_array_equal(got2, lo + (hi - lo) * ref[:10])


def update_probability(kind, alpha, mine, theirs):
    """StochasticParallelSouthwellUpdateProbability (DMEM_Smooth.cpp:548-572)."""
    x = 0.0 if kind == 2 else float(sum(1 for t in theirs if mine < t))
    if kind == 1:
        return math.inf if x == 0 else (1.0 / x) * (1.0 / alpha)
    if kind == 0:
        return math.exp(-x * alpha)
    return alpha


def test_sps_defaults(amg):
    o = amg.default_opts()
    assert o.sps_probability_type == amg.AMG_SPS_EXPONENTIAL
    assert o.sps_alpha == 1.0 and o.sps_min_prob == 0.0
    # the largest residual among its neighbours always relaxes; the others less often
    assert update_probability(0, 1.0, 5.0, [1.0, 2.0]) == 1.0
    assert update_probability(0, 1.0, 1.0, [2.0, 3.0]) == math.exp(-2.0)
