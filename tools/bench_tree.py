#!/usr/bin/env python3
"""Note-commitment tree windows on the GPU, measured.

Workload: a window of 1,024 blocks x 64 Sapling outputs (65,536 note commitments) appended to a
Sapling tree (H32) whose frontier already holds ~2^30 leaves, with the root after every block
(BlockSaplingRoot, accept_block.rs:290-320) and the final state; the same shape for the Sprout
tree (H29). Leaves are resident in HBM (zg_tree_roots_device); the timed call includes the
frontier upload, the 32 level launches, the roots' and state's download.

    python tools/bench_tree.py [--reps K] [--leaves N] [--per-block B]

Prints one JSON object: per tree, leaves/s, roots/s, hashes/s (n + HEIGHT x roots + level
overhang), wall ms per window, the level kernels' device ms (HIP events), and the CPU baseline:
the reference's sequential algorithm restated in C++ (oracle/cpu/merkle_cpu.cpp, one core; the
reference's own Rust is not buildable here) on windows of the same shape.
"""
import argparse
import json
import os
import random
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def frontier(rnd, kind, height, s0):
    from oracle import merkle as M
    t = M.TreeState(kind, height)
    c = (s0 - 1) >> 1
    t.left = rnd.randbytes(32)
    t.right = rnd.randbytes(32) if s0 % 2 == 0 else None
    t.parents = [rnd.randbytes(32) if (c >> i) & 1 else None for i in range(height - 1)]
    t.is_empty = False
    return t


def hashes_in_window(height, s0, n, nroots):
    """the hashes zg_tree_roots performs: per level the completed-node build + one per root"""
    tot = 0
    s1 = s0 + n
    for lv in range(1, height):
        base = (s0 - 1) >> lv if s0 else 0
        tot += ((s1 - 1) >> lv) - base + 1
    return tot + height * nroots


def run(ctx, kind, height, n, per, reps, warm=2, seed=1):
    import torch
    rnd = random.Random(seed + kind)
    s0 = (1 << 30) + rnd.randrange(1 << 20)
    st = frontier(rnd, kind, height, s0).serialize()
    leaves = torch.randint(0, 256, (n, 32), dtype=torch.uint8, device="cuda:0")
    leaves[:, 31] &= 0x7F
    marks = list(range(per, n + 1, per))
    for _ in range(warm):
        ctx.tree_roots(kind, height, st, n, marks, device_leaves=leaves.data_ptr())
    torch.cuda.synchronize()
    kms = []
    t = time.perf_counter()
    for _ in range(reps):
        _, _, ms = ctx.tree_roots(kind, height, st, n, marks, device_leaves=leaves.data_ptr(), with_time=True)
        kms.append(ms)
    dt = (time.perf_counter() - t) / reps
    h = hashes_in_window(height, s0, n, len(marks))
    kmean = sum(kms) / len(kms)
    return {"height": height, "leaves": n, "roots": len(marks), "frontier_leaves": s0, "hashes": h,
            "ms_per_window": dt * 1e3, "kernel_ms": kmean, "leaves_per_s": n / dt, "roots_per_s": len(marks) / dt,
            "hashes_per_s": h / dt, "kernel_hashes_per_s": h / (kmean * 1e-3)}


def cpu_window(kind, height, per, seconds=6.0, threads=1):
    """the reference's sequential path (oracle/cpu/merkle_cpu.cpp: TreeState append + root per
    block, sapling-crypto's Pedersen algorithm) over windows of the same shape (a root per `per`
    leaves) from the same kind of deep frontier, for about `seconds`. With threads > 1, that many
    independent windows (own frontier each) run concurrently, one per thread: the reference
    appends ONE tree sequentially, so this is the aggregate rate of the host's cores, an upper
    bound on what its CPU path reaches for a single tree."""
    import threading
    from tests import cpulib
    L = cpulib.load_merkle()
    n = 16 * per
    marks = list(range(per, n + 1, per))
    jobs = []
    for t_ in range(max(1, threads)):
        rnd = random.Random(5 + kind + 101 * t_)
        s0 = (1 << 30) + rnd.randrange(1 << 20)
        jobs.append((frontier(rnd, kind, height, s0).serialize(), [rnd.randbytes(31) + b"\x00" for _ in range(n)]))
    assert cpulib.merkle_window(L, kind, height, jobs[0][0], jobs[0][1], marks)[0] == 0   # lazy tables, one thread
    done = [0] * len(jobs)
    stop = time.perf_counter() + seconds

    def work(j):
        st, leaves = jobs[j]
        while time.perf_counter() < stop:
            rc, _ = cpulib.merkle_window(L, kind, height, st, leaves, marks)
            assert rc == 0
            done[j] += 1
    t = time.perf_counter()
    ths = [threading.Thread(target=work, args=(j,)) for j in range(len(jobs))]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    dt = time.perf_counter() - t
    k = sum(done)
    return {"leaves_per_s": k * n / dt, "roots_per_s": k * len(marks) / dt, "cores": len(jobs), "kind": "port",
            "sample": "%d windows of %d leaves, a root per %d, from 2^30-leaf frontiers, %d concurrent independent "
                      "windows (one per thread) (%.1f s)" % (k, n, per, len(jobs), dt)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--leaves", type=int, default=65536)
    ap.add_argument("--per-block", type=int, default=64)
    ap.add_argument("--no-cpu", action="store_true")
    a = ap.parse_args()
    import torch
    torch.cuda.set_device(0)   # torch's HIP runtime first, then the library's context
    torch.zeros(1, device="cuda:0")
    from zebra_amd import Context
    from zebra_amd import zg
    ctx = Context(device=0, max_batch=64, load_builtin=False)
    out = {"workload": "window of %d leaves, a root per %d" % (a.leaves, a.per_block)}
    out["sapling_h32"] = run(ctx, zg.TREE_SAPLING, 32, a.leaves, a.per_block, a.reps)
    out["sprout_h29"] = run(ctx, zg.TREE_SPROUT, 29, a.leaves, a.per_block, a.reps)
    if not a.no_cpu:
        out["sapling_h32"]["cpu_baseline"] = cpu_window(zg.TREE_SAPLING, 32, a.per_block)
        out["sprout_h29"]["cpu_baseline"] = cpu_window(zg.TREE_SPROUT, 29, a.per_block)
    ctx.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
