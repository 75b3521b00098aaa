#!/usr/bin/env python3
"""PGHR13 Sprout proofs on BN254, measured.

Workload: n proofs (default 65,536) cycling through the nine valid PHGR statements of the
reference's fixtures (crypto/src/pghr13.rs verification / verification2, sprout.rs smoky_pghr and
the six JoinSplits of mainnet block 522; tests/golden/pghr13.json), every one verified
(decode + G2 subgroup check + the five equalities folded with random weights + one final
exponentiation), packed host buffers through zg_pghr13_verify (upload included in the wall time;
the kernels' device time reported beside it). CPU baseline: the compiled C++ restatement
(oracle/cpu/pghr13_cpu.cpp, the reference's five separate pairing equalities) on a bounded sample.

    python tools/bench_pghr13.py [--n N] [--reps K]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def workload(n):
    g = json.load(open(os.path.join(ROOT, "tests", "golden", "pghr13.json")))
    valid = [c for c in g["cases"] if c["status"] == 0]
    proofs = [bytes.fromhex(valid[i % len(valid)]["proof"]) for i in range(n)]
    inputs = [[bytes.fromhex(x) for x in valid[i % len(valid)]["inputs"]] for i in range(n)]
    return proofs, inputs


def run(ctx, n=65536, reps=3):
    proofs, inputs = workload(n)
    ctx.pghr13_verify(proofs[:64], inputs[:64])   # key, tables, first launch
    # the ABI's packed host buffers (a caller's block window), built once outside the clock
    pblob = b"".join(proofs)
    iblob = b"".join(b"".join(r) + bytes(32 * (9 - len(r))) for r in inputs)
    cnt = bytes(len(r) for r in inputs)
    ctx.pghr13_verify(pblob, iblob, cnt)          # the arena at this size
    kms, t = [], time.perf_counter()
    for _ in range(reps):
        st, ms = ctx.pghr13_verify(pblob, iblob, cnt, with_time=True)
        kms.append(ms)
    dt = (time.perf_counter() - t) / reps
    assert st == [0] * n
    km = sum(kms) / len(kms)
    return {"proofs": n, "ms_per_batch": dt * 1e3, "kernel_ms": km, "proofs_per_s": n / dt,
            "kernel_proofs_per_s": n / (km * 1e-3), "all_ok": True}


def cpu_baseline(seconds=6.0, threads=1):
    """the reference's PGHR13 check restated in C++ (oracle/cpu/pghr13_cpu.cpp: Proof::from_raw +
    pghr13::verify's five equalities as 12 separate pairings, crypto/src/pghr13.rs:69-105), one
    proof per task on `threads` std::threads, over the same 9 statements, for about `seconds`"""
    from tests import cpulib
    L = cpulib.load_pghr13()
    proofs, inputs = workload(9)
    m = 9 * max(1, threads)
    t = time.perf_counter()
    assert cpulib.pg_verify(L, proofs * (m // 9), inputs * (m // 9), threads) == [0] * m
    rate = m / (time.perf_counter() - t)
    m = max(m, 9 * int(rate * seconds / 9))
    t = time.perf_counter()
    assert cpulib.pg_verify(L, proofs * (m // 9), inputs * (m // 9), threads) == [0] * (9 * (m // 9))
    dt = time.perf_counter() - t
    n = 9 * (m // 9)
    return {"proofs_per_s": n / dt, "cores": threads, "kind": "port",
            "ms_per_proof_per_core": 1e3 * dt * threads / n,
            "sample": "%d proofs (the 9 valid statements, repeated) in %.1f s on %d threads: C++ restatement of "
                      "crypto/src/pghr13.rs:69-105 (oracle/cpu/pghr13_cpu.cpp, 12 pairings per valid proof)"
                      % (n, dt, threads)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=65536)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--no-cpu", action="store_true")
    a = ap.parse_args()
    import torch
    torch.cuda.set_device(0)
    torch.zeros(1, device="cuda:0")
    from zebra_amd import Context
    ctx = Context(device=0, max_batch=64, load_builtin=False)
    out = run(ctx, a.n, a.reps)
    if not a.no_cpu:
        out["cpu_baseline"] = cpu_baseline()
        out["gpu_over_cpu"] = out["proofs_per_s"] / out["cpu_baseline"]["proofs_per_s"]
    ctx.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
