"""All-pairs 256-bit descriptor matching on the device (sg_matcher_* / sg_hamming_*), and the synthetic
descriptor sets of BASELINE config 4 (10k random 256-bit descriptors, seed 4; B = a
permutation of A with Binomial(256, 0.03) bit flips on 70 % of the rows and fresh random rows on 30 %)."""
from __future__ import annotations

import ctypes as C

import numpy as np

from .capi import SgDeviceOptions, check, load_library

_ip = C.POINTER(C.c_int32)
_u64p = C.POINTER(C.c_uint64)


def make_descriptor_sets(n: int = 10000, seed: int = 4, flip_p: float = 0.03, keep: float = 0.7):
    """Returns (A, B, truth) with truth[i] = row of A that B[i] was derived from, or -1 for fresh rows."""
    rng = np.random.default_rng(seed)
    A = rng.integers(0, 2 ** 64, size=(n, 4), dtype=np.uint64, endpoint=False)
    perm = rng.permutation(n)
    B = A[perm].copy()
    truth = perm.astype(np.int64)
    fresh = rng.random(n) >= keep
    B[fresh] = rng.integers(0, 2 ** 64, size=(int(fresh.sum()), 4), dtype=np.uint64, endpoint=False)
    truth[fresh] = -1
    flips = rng.random((n, 256)) < flip_p
    flips[fresh] = False
    bits = np.packbits(flips, axis=1, bitorder="little").view(np.uint64).reshape(n, 4)
    B ^= bits
    return A, B, truth


class HammingMatcher:
    def __init__(self, device: int = 0):
        self.lib = load_library()
        self.h = C.c_void_p()
        dev = SgDeviceOptions(device=device, precision=0, rank=0, nranks=1)
        check(self.lib.sg_matcher_create(C.byref(self.h), C.byref(dev)), "sg_matcher_create")

    def close(self):
        if self.h:
            self.lib.sg_matcher_destroy(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def match(self, query: np.ndarray, train: np.ndarray):
        """(best_idx, best_dist, second_dist) per query row."""
        q = np.ascontiguousarray(query, dtype=np.uint64).reshape(-1, 4)
        t = np.ascontiguousarray(train, dtype=np.uint64).reshape(-1, 4)
        n = q.shape[0]
        bi, bd, sd = (np.zeros(n, np.int32) for _ in range(3))
        check(self.lib.sg_hamming_match(self.h, q.ctypes.data_as(_u64p), n, t.ctypes.data_as(_u64p), t.shape[0],
                                        bi.ctypes.data_as(_ip), bd.ctypes.data_as(_ip), sd.ctypes.data_as(_ip)),
              "sg_hamming_match")
        return bi, bd, sd

    def load(self, query, train):
        self._q = np.ascontiguousarray(query, dtype=np.uint64).reshape(-1, 4)
        self._t = np.ascontiguousarray(train, dtype=np.uint64).reshape(-1, 4)
        check(self.lib.sg_hamming_load(self.h, self._q.ctypes.data_as(_u64p), self._q.shape[0],
                                       self._t.ctypes.data_as(_u64p), self._t.shape[0]), "sg_hamming_load")

    def run(self, repeats: int = 1):
        check(self.lib.sg_hamming_run(self.h, repeats), "sg_hamming_run")

    def results(self):
        n = self._q.shape[0]
        bi, bd, sd = (np.zeros(n, np.int32) for _ in range(3))
        ms = C.c_double()
        check(self.lib.sg_hamming_results(self.h, bi.ctypes.data_as(_ip), bd.ctypes.data_as(_ip),
                                          sd.ctypes.data_as(_ip), C.byref(ms)), "sg_hamming_results")
        return bi, bd, sd, ms.value
