#!/usr/bin/env python3
"""Configs 2 and 4 (bench.py other_configs: 1,024 spends; 4,096 with 41 corrupted) on a context
sized for the headline (max_batch 65,536) and on one sized for the batch, plus a clean 4,096
batch and the per-phase HIP-event timings of each. Run it under rocprofv3 --kernel-trace --stats
to see where a small batch's time goes.  Usage: python tools/small_batch.py [reps]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    import bench
    from zebra_amd import Context
    src_proofs, src_kinds, *_ = bench.workload(0, 1, 64)
    out = {}
    for cap in (65536, 4096):
        ctx = Context(device=0, max_batch=cap)
        t = time.perf_counter()
        res = bench.other_configs(ctx, src_proofs, src_kinds, reps)
        res["wall_s"] = time.perf_counter() - t
        res["last_phase_ms"] = dict(zip(Context.PHASES, ctx.last_timings()))
        res["stats"] = ctx.stats()
        # a clean 4,096-proof batch (config 4 without the corruptions)
        idx = [i % 5 for i in range(4096)]
        pr = ctx.synth_rerandomize(src_proofs, src_kinds, idx, 5)
        _, kinds, _, _, inputs, _ = bench.workload(0, 1, 4096)
        kinds = bytes(src_kinds[j] for j in idx)
        real = {e["name"]: e for e in json.load(open(os.path.join(ROOT, "tests", "golden", "real_proofs.json")))["proofs"]}
        from zebra_amd import pack_inputs
        srcs = ["S1", "S2", "O1", "O2", "O3"]
        inputs = pack_inputs([[bytes.fromhex(x) for x in real[srcs[j]]["inputs"]] for j in idx])
        ctx.verify_batch(pr, kinds, inputs)
        t = time.perf_counter()
        for _ in range(reps):
            sts, _ = ctx.verify_batch(pr, kinds, inputs)
        res["clean_4096_ms"] = (time.perf_counter() - t) / reps * 1e3
        res["clean_4096_phase_ms"] = dict(zip(Context.PHASES, ctx.last_timings()))
        assert sts == [0] * 4096
        out["cap%d" % cap] = res
        ctx.close()
        print(json.dumps({"cap": cap, **res}), flush=True)


if __name__ == "__main__":
    main()
