#!/usr/bin/env python3
"""PGHR13 Sprout proofs on BN254, measured.

Workload: n proofs (default 65,536) cycling through the nine valid PHGR statements of the
reference's fixtures (crypto/src/pghr13.rs verification / verification2, sprout.rs smoky_pghr and
the six JoinSplits of mainnet block 522; tests/golden/pghr13.json), every one verified
(decode + G2 subgroup check + the five equalities folded with random weights + one final
exponentiation), host buffers through zg_pghr13_verify (upload included in the wall time; the
kernels' device time reported beside it). CPU baseline: the Python oracle (oracle/pghr13.py,
the reference's five separate pairing equalities) on a bounded sample, one core.

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
    kms, t = [], time.perf_counter()
    for _ in range(reps):
        st, ms = ctx.pghr13_verify(proofs, inputs, with_time=True)
        kms.append(ms)
    dt = (time.perf_counter() - t) / reps
    assert st == [0] * n
    km = sum(kms) / len(kms)
    return {"proofs": n, "ms_per_batch": dt * 1e3, "kernel_ms": km, "proofs_per_s": n / dt,
            "kernel_proofs_per_s": n / (km * 1e-3), "all_ok": True}


def cpu_baseline(seconds=6.0):
    from oracle import pghr13 as PG
    vk = PG.load_vk_json(open(os.path.join(ROOT, "zebra_amd", "res", "sprout-verifying-key.json")).read())
    proofs, inputs = workload(9)
    k, t = 0, time.perf_counter()
    while time.perf_counter() - t < seconds:
        xs = [int.from_bytes(x, "little") for x in inputs[k % 9]]
        assert PG.verify_raw(vk, proofs[k % 9], xs) == PG.OK
        k += 1
    dt = time.perf_counter() - t
    return {"proofs_per_s": k / dt, "cores": 1, "kind": "port (Python oracle, 5 pairing equalities)",
            "sample": "%d proofs in %.1f s" % (k, dt)}


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
