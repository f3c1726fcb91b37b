"""256-bit all-pairs Hamming matching (BASELINE config 4).  CPU: the oracle against a numpy statement of
the specification.  GPU: the device matcher against the oracle, bit-exact (indices and distances), at the
full 10k x 10k size and on the edge cases (ties, empty / single-row train sets, ragged sizes)."""
import os
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "oracle"))
import oracle  # noqa: E402
from slamgpu.matcher import HammingMatcher, make_descriptor_sets  # noqa: E402


def _numpy_match(q, t):
    d = np.bitwise_count(q[:, None, :] ^ t[None, :, :]).sum(-1).astype(np.int64)
    bi = d.argmin(1)                       # first (lowest) index on ties
    bd = d[np.arange(len(q)), bi]
    d2 = d.copy()
    d2[np.arange(len(q)), bi] = 1 << 30
    return bi, bd, d2.min(1)


def test_oracle_matches_numpy_specification():
    rng = np.random.default_rng(0)
    q = rng.integers(0, 2 ** 64, (300, 4), dtype=np.uint64, endpoint=False)
    t = rng.integers(0, 2 ** 64, (700, 4), dtype=np.uint64, endpoint=False)
    t[500] = t[100]                        # duplicate train rows: ties resolve to the lower index
    q[7] = t[100]
    bi, bd, sd = oracle.hamming_match(q, t, nthreads=4)
    ri, rd, rs = _numpy_match(q, t)
    np.testing.assert_array_equal(bi, ri)
    np.testing.assert_array_equal(bd, rd)
    np.testing.assert_array_equal(sd, rs)
    assert bi[7] == 100 and bd[7] == 0 and sd[7] == 0


def test_descriptor_sets_recover_most_true_matches():
    A, B, truth = make_descriptor_sets(2000)
    bi, bd, sd = oracle.hamming_match(B, A, nthreads=4)
    kept = truth >= 0
    assert (bi[kept] == truth[kept]).mean() > 0.99
    assert np.median(bd[kept]) < 16 and np.median(bd[~kept]) > 90


@pytest.mark.gpu
def test_device_full_size_bit_exact(gpu_lib):
    A, B, truth = make_descriptor_sets(10000)
    m = HammingMatcher()
    bi, bd, sd = m.match(B, A)
    ri, rd, rs = oracle.hamming_match(B, A, nthreads=8)
    np.testing.assert_array_equal(bi, ri)
    np.testing.assert_array_equal(bd, rd)
    np.testing.assert_array_equal(sd, rs)


@pytest.mark.gpu
@pytest.mark.parametrize("nq,nt", [(1, 1), (5, 0), (257, 255), (1000, 513), (3, 70000)])
def test_device_edge_sizes_and_ties(gpu_lib, nq, nt):
    rng = np.random.default_rng(nq + nt)
    q = rng.integers(0, 2 ** 64, (nq, 4), dtype=np.uint64, endpoint=False)
    t = rng.integers(0, 2 ** 64, (nt, 4), dtype=np.uint64, endpoint=False)
    if nt > 10:
        t[nt - 1] = t[3]                   # tie across slices: lowest index wins
        q[0] = t[3]
    m = HammingMatcher()
    bi, bd, sd = m.match(q, t)
    ri, rd, rs = oracle.hamming_match(q, t, nthreads=8)
    np.testing.assert_array_equal(bi, ri)
    np.testing.assert_array_equal(bd, rd)
    np.testing.assert_array_equal(sd, rs)
