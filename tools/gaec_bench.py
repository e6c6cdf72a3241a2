"""Host GAEC timing without a GPU: pemp_pose_cluster (host C++ in libpemp.so) on C3-shaped inputs.
Fully graphs of B images x n nodes, person-structured edge probabilities as bench.py::person_structured_probs
(node i -> person i mod P; sigmoid(+-2.5 + N(0, 1.5)) per direction), weights w = p(s,d) + p(d,s) on the upper
edges as pose_edge_weights_kernel writes them, every image averaged (flags bit 0).
usage: python tools/gaec_bench.py [B n persons threads reps]"""
import ctypes
import sys
import time

import numpy as np

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from pemp_amd import _lib  # noqa: E402


def inputs(B, n, P, seed=7):
    rng = np.random.default_rng(seed)
    src, dst = np.meshgrid(np.arange(n), np.arange(n), indexing="ij")
    keep = src != dst
    s1, d1 = src[keep], dst[keep]
    E1 = s1.size
    ei = np.empty((2, B * E1), dtype=np.int64)
    w = np.empty(B * E1, dtype=np.float32)
    for b in range(B):
        same = (s1 % P) == (d1 % P)
        p = 1 / (1 + np.exp(-(np.where(same, 2.5, -2.5) + 1.5 * rng.standard_normal(E1)))).astype(np.float32)
        pm = np.zeros((n, n), np.float32)
        pm[s1, d1] = p
        wt = np.where(s1 < d1, pm[s1, d1] + pm[d1, s1], np.float32(np.nan)).astype(np.float32)
        ei[0, b * E1:(b + 1) * E1] = s1 + b * n
        ei[1, b * E1:(b + 1) * E1] = d1 + b * n
        w[b * E1:(b + 1) * E1] = wt
    node_off = np.arange(B + 1, dtype=np.int64) * n
    flags = np.ones(B + 1, dtype=np.int32) | 2
    flags[B] = 0
    return node_off, ei, w, flags


def cluster(L, node_off, ei, w, flags, threads):
    B = len(node_off) - 1
    N = int(node_off[-1])
    labels = np.empty(N, np.int32)
    ncomp = np.empty(B, np.int32)
    _lib.check(L.pemp_pose_cluster(B, node_off.ctypes.data, ei.ctypes.data, ei.shape[1], w.ctypes.data,
                                   flags.ctypes.data, 0, threads, labels.ctypes.data, ncomp.ctypes.data), L)
    return labels, ncomp


def main():
    a = [int(x) for x in sys.argv[1:]] + [8, 153, 9, 8, 20][len(sys.argv) - 1:]
    B, n, P, threads, reps = a[:5]
    L = _lib.load_cdll()
    args = inputs(B, n, P)
    lab, nc = cluster(L, *args, threads)
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        cluster(L, *args, threads)
        ts.append(time.perf_counter() - t0)
    print(f"B={B} n={n} persons={P} threads={threads}: median {np.median(ts) * 1e3:.3f} ms, min "
          f"{min(ts) * 1e3:.3f} ms; components {nc.tolist()}")


if __name__ == "__main__":
    main()
