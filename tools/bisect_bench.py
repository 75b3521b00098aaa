#!/usr/bin/env python3
"""Config 4 (4,096 proofs, 41 corrupted -> exact reject set via bisection) against a clean
4,096-proof batch, both through zg_verify_batch; prints ms per batch and the context counters.
Run it under rocprofv3 --kernel-trace --stats to see where the bisection time goes.
Usage: python tools/bisect_bench.py [reps]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    from tests.test_gpu_parity import corrupted_4096
    from zebra_amd import Context
    ctx = Context(device=0, max_batch=4096)
    proofs, kinds, inputs, want = corrupted_4096(ctx)
    clean = ctx.synth_rerandomize(*_sources(), [i % 9 for i in range(4096)], 3)
    res = {}
    for name, pr in (("clean_4096", clean), ("config4_4096_41_bad", proofs)):
        sts, _ = ctx.verify_batch(pr, kinds, inputs if name != "clean_4096" else _clean_inputs())
        t = time.perf_counter()
        for _ in range(reps):
            sts, _ = ctx.verify_batch(pr, kinds, inputs if name != "clean_4096" else _clean_inputs())
        res[name] = {"ms_per_batch": (time.perf_counter() - t) / reps * 1e3}
        if name != "clean_4096":
            assert sts == want, "reject set differs"
        else:
            assert sts == [0] * 4096
    res["ratio"] = res["config4_4096_41_bad"]["ms_per_batch"] / res["clean_4096"]["ms_per_batch"]
    res["stats"] = ctx.stats()
    print(json.dumps(res))
    ctx.close()


def _sources():
    from tests.conftest import load_golden
    real = load_golden("real_proofs.json")["proofs"]
    return b"".join(bytes.fromhex(e["proof"]) for e in real), bytes(e["kind"] for e in real)


_ci = None


def _clean_inputs():
    global _ci
    if _ci is None:
        from tests.conftest import load_golden
        from zebra_amd import pack_inputs
        real = load_golden("real_proofs.json")["proofs"]
        _ci = pack_inputs([[bytes.fromhex(x) for x in real[i % 9]["inputs"]] for i in range(4096)])
    return _ci


if __name__ == "__main__":
    main()
