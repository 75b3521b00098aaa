#!/usr/bin/env python3
"""Config 2 alone (1,024 spends, one batch, host buffers) repeated, for a rocprofv3 kernel trace of
a small batch's critical path (tools/timeline.py). Usage: python tools/config2_trace.py [reps]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    import bench
    from zebra_amd import Context, pack_inputs
    src_proofs, src_kinds, *_ = bench.workload(0, 1, 64)
    ctx = Context(device=0, max_batch=1024)
    real = {e["name"]: e for e in json.load(open(os.path.join(ROOT, "tests", "golden", "real_proofs.json")))["proofs"]}
    rows = {s: [bytes.fromhex(x) for x in real[s]["inputs"]] for s in ("S1", "S2")}
    idx = [i % 2 for i in range(1024)]
    proofs = ctx.synth_rerandomize(src_proofs, src_kinds, idx, 1)
    kinds = bytes(src_kinds[j] for j in idx)
    inputs = pack_inputs([rows[("S1", "S2")[j]] for j in idx])
    ms = []
    for _ in range(reps):
        t = time.perf_counter()
        sts, _ = ctx.verify_batch(proofs, kinds, inputs)
        ms.append((time.perf_counter() - t) * 1e3)
        assert sts == [0] * 1024
    print(json.dumps({"ms_per_batch": ms, "phase_ms": dict(zip(Context.PHASES, ctx.last_timings()))}))


if __name__ == "__main__":
    main()
