#!/usr/bin/env python3
"""Headline benchmark: Sapling Groth16 proofs verified/s, batch 64k (BASELINE.json metric,
config 3: 65,536 mixed spend/output proofs), on N MI355X, one process per GPU.

  python bench.py [--gpus N --steps K --warmup W]        (N > 1 under torch.distributed.run)

A step = one batch verification of the whole 65,536-proof workload: every rank verifies its
contiguous shard (decode + subgroup checks + batch algebra + per-proof Miller loops + product
tree) from HBM-resident inputs, emits one 576-byte Miller partial; at N > 1 (or with --dist at
N = 1) the partials are gathered over RCCL (one all-gather) -- at N = 1 without --dist no
collective runs and config.collective says so -- every rank runs the ONE final exponentiation of
their product on the same gathered bytes (same verdict, no second collective) and finalises its
per-proof statuses. The host->HBM input copies are outside the timed region; h2d_ms_per_batch
reports them. Inputs: real mainnet proofs from the reference's fixtures,
re-randomized on the GPU (synthetic, all valid; verified OK after the timed region).
Batch scalars r_i come from the OS RNG inside the timed region (production mode).
Batches in flight (--inflight; default 6, 8 for shards of at most 8,192 proofs): each GPU keeps that many
consecutive batches on the device, one context (buffers + streams) each. The host reads the
oldest batch's partial and statuses and relaunches its context at once; the batch's verdict
runs off that loop: the exchange (gather) on a worker thread in batch order, the final
exponentiations on one coalescing verdict thread that checks every gathered batch waiting for it in
one launch (Context.gt_check_many; --checkers N: N verdict threads with a checker context each), so
consecutive verdicts overlap (--sync-verdict: before the relaunch). Every batch is fully verified and its verdict is in
inside the timed region (pipeline fill and drain included); a false verdict re-runs the batch
with bisection. A batch's own latency is phase_ms.device_pipeline plus the final exponentiation.
"""
import argparse
import json
import os
import queue
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# frozen algorithmic work per proof (Fq-mul-equivalents), attributed to the
# kernel that performs it (the G2 subgroup check of B rides on the R-chain kernel).
W_DECODE = 2679 + 2 * 507 + 1593 + 3         # point decode (2 Fq + 1 Fq2 sqrt), 2 G1 checks, r_i A_i, Fr
W_K4 = 264                                   # Pippenger sum r_i C_i share (K4, side stream)
W_LINES = 1634 + 1189                        # G2 line coefficients (R-chain) + G2 subgroup check
W_FCHAIN = 5192                              # Miller f-chain (sparse line products + squarings)
W_TREE = 54                                  # tree-product Fq12 multiply
W_TOTAL = 13622
assert W_DECODE + W_K4 + W_LINES + W_FCHAIN + W_TREE == W_TOTAL
# K4 bucket phase, algorithmic HBM bytes: per entry the 4-byte bucket entry and the 100-byte
# affine C_i it names (G1A), plus the bucket offsets read and the (T, U) segment sums written
# (Jacobian, 144 B each) -- zg_msm.h msm_shape: c = 11 from 32k padded proofs, 10 from 8k, 9 below
# K4's bucket phase per entry: the 4-B entry + its C_i operands as lazy digits (x or beta x, y:
# 2 x 14 x 4 B, written once per proof by k_msm_count); per segment the (T, U) pair written as
# G1D (3 x 14 words each); the isolated pass runs a lone batch, so P = 4 (2 below 8k) lanes per bucket
K4_ENTRY_BYTES = 4 + 2 * 56


def k4_fixed_bytes(npad):
    c, w, nb, parts = (11, 6, 1024, 4) if npad >= 32768 else (10, 7, 512, 4) if npad >= 8192 else (9, 8, 256, 2)
    ncount = 3 * w * nb
    return ncount * 4 + (ncount // (64 // parts)) * 2 * 168
NOMINAL_LANES = 256 * 4 * 16                        # MI355X: CUs x SIMDs x lanes per clock
MACS_PER_FQMUL = 288                                # 2 * 12^2 32x32->64 MACs (product + CIOS reduction)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def workload(rank, world, n_total):
    """config 3: even i -> spend S[(i/2) mod 2], odd i -> output O[(i/2) mod 3]; contiguous shards."""
    real = {e["name"]: e for e in json.load(open(os.path.join(ROOT, "tests", "golden", "real_proofs.json")))["proofs"]}
    srcs = ["S1", "S2", "O1", "O2", "O3"]
    shard = n_total // world
    lo = rank * shard
    idx = []
    for i in range(lo, lo + shard):
        idx.append((i // 2) % 2 if i % 2 == 0 else 2 + (i // 2) % 3)
    src_proofs = b"".join(bytes.fromhex(real[s]["proof"]) for s in srcs)
    src_kinds = bytes(real[s]["kind"] for s in srcs)
    inputs_by_src = []
    for s in srcs:
        row = bytearray(288)
        for j, x in enumerate(real[s]["inputs"]):
            row[32 * j:32 * j + 32] = bytes.fromhex(x)
        inputs_by_src.append(bytes(row))
    kinds = bytes(src_kinds[j] for j in idx)
    inputs = b"".join(inputs_by_src[j] for j in idx)
    return src_proofs, src_kinds, idx, kinds, inputs, shard


def host_cpu():
    """the host the CPU baseline runs on: nproc, the CPUs this process may use, the model"""
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    try:
        usable = len(os.sched_getaffinity(0))
    except AttributeError:
        usable = os.cpu_count() or 1
    return {"nproc": os.cpu_count() or 1, "usable": usable, "cpu_model": model,
            "omp_num_threads": os.environ.get("OMP_NUM_THREADS")}


def cpu_threads(requested=0):
    """every core this process may use (the rayon fan-out of accept_chain.rs:76-81 uses all
    logical CPUs), capped by OMP_NUM_THREADS where the box sets this process's CPU share"""
    h = host_cpu()
    n = h["usable"]
    if h["omp_num_threads"] and h["omp_num_threads"].isdigit():
        n = min(n, int(h["omp_num_threads"]))
    if requested > 0:
        n = min(n, requested)
    return max(1, n)


def cpu_baseline(proofs, kinds, inputs, seconds, threads):
    """the oracle's C++ restatement of bellman's per-proof verify, on host cores, on a bounded
    sample of the same workload. `threads` is this job's CPU share on the box (OMP_NUM_THREADS;
    the pool's rules keep a one-GPU job's worker pools to that share), so the all-core figure of
    SURVEY.md 8(d) is reported beside it as a projection: the measured per-thread rate x every
    usable CPU, with the measured 1 -> `threads` scaling efficiency that justifies it."""
    from tests import cpulib
    L = cpulib.load()
    n = len(kinds)
    m0 = min(n, 4 * threads)
    t = time.perf_counter()
    sts, _ = cpulib.verify(L, proofs[:192 * m0], kinds[:m0], inputs[:288 * m0], threads=threads)
    rate = m0 / (time.perf_counter() - t)
    m = int(min(n, max(m0, rate * seconds)))
    t = time.perf_counter()
    sts, _ = cpulib.verify(L, proofs[:192 * m], kinds[:m], inputs[:288 * m], threads=threads)
    dt = time.perf_counter() - t
    assert all(s == 0 for s in sts), "cpu baseline rejected a valid proof"
    # one thread on a short sample: the scaling efficiency of the threaded figure
    m1 = max(8, int(m / threads / 6))
    t = time.perf_counter()
    cpulib.verify(L, proofs[:192 * m1], kinds[:m1], inputs[:288 * m1], threads=1)
    rate1 = m1 / (time.perf_counter() - t)
    h = host_cpu()
    value = m / dt
    # calibration: the port's building blocks on one thread, set against SURVEY.md
    # 8(a) row a13's analytical bellman estimate (~69 k Fq-mul-eq per spend proof at 30-50 ns each)
    calib = None
    try:
        real = {e["name"]: e for e in json.load(open(os.path.join(ROOT, "tests", "golden", "real_proofs.json")))["proofs"]}
        e = real["S1"]
        row = bytearray(288)
        for j, x in enumerate(e["inputs"]):
            row[32 * j:32 * j + 32] = bytes.fromhex(x)
        ops = cpulib.bench_ops(L, e["kind"], bytes.fromhex(e["proof"]), bytes(row), len(e["inputs"]), reps=10)
        calib = {k: round(v, 2) for k, v in ops.items()}
        calib["verify_one_fq_mul_eq"] = round(1e3 * ops["verify_one_us"] / ops["fq_mul_ns"])
        calib["survey_estimate"] = {"fq_mul_ns": [30, 50], "ms_per_proof": [2.0, 3.5], "fq_mul_eq_per_spend_proof": 69000,
                                    "source": "SURVEY.md 8(a) row a13 (analytical)"}
        calib["ratio_to_estimate_upper"] = round(1e-3 * ops["verify_one_us"] / 3.5, 3)
        calib["note"] = ("one spend proof (real_proofs.json S1) on one thread: Fq product and squaring chains, one "
                         "G2Prepared, the 3-pair Miller loop and the final exponentiation of verify_proof, a 255-bit "
                         "G1 product (one IC term; the naive [r]P subgroup check has the same cost), the naive G2 "
                         "[r]Q check, and the whole verify_one")
    except Exception as ex:  # the calibration is informative only
        calib = {"error": repr(ex)}
    return {"value": value, "unit": "proofs/s", "cores": threads, "kind": "port", "calibration": calib,
            "nproc": h["nproc"], "usable_cpus": h["usable"], "cpu_model": h["cpu_model"],
            "ms_per_proof_per_core": 1e3 * dt * threads / m,
            "one_thread_proofs_per_s": rate1, "scaling_efficiency": value / (threads * rate1),
            "projected_all_usable_cpus": {
                "value": value / threads * h["usable"], "cpus": h["usable"],
                "note": "measured per-thread rate x usable CPUs (linear scaling, the one-proof-per-task "
                        "fan-out has no shared state); not measured: the box grants a one-GPU job %d of "
                        "its CPUs (OMP_NUM_THREADS) and its worker pools are kept to that share" % threads},
            "sample": "first %d proofs of the same re-randomized 65,536-proof workload, bellman-restatement "
                      "per-proof verify_proof (oracle/cpu/bellman_cpu.cpp), one proof per std::thread task on "
                      "%d threads, %.1f s; one thread: %d proofs" % (m, threads, dt, m1)}


def h2d_copy_ms(proofs, kinds, inputs, dev, reps=5):
    """what the headline excludes: one shard's host -> HBM copies (192-B proofs, kinds, 288-B
    input rows), from pageable host memory (what zg_verify_batch's host-buffer call copies) and
    from pinned memory; measured after the timed region"""
    import torch
    bufs = [torch.frombuffer(bytearray(b), dtype=torch.uint8) for b in (proofs, kinds, inputs)]
    pinned = [b.pin_memory() for b in bufs]
    out = {"bytes": sum(b.numel() for b in bufs)}
    for name, src in (("pageable", bufs), ("pinned", pinned)):
        dst = [torch.empty_like(b, device=dev) for b in src]
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(reps):
            for d, b in zip(dst, src):
                d.copy_(b, non_blocking=(name == "pinned"))
        torch.cuda.synchronize()
        out[name + "_ms"] = 1e3 * (time.perf_counter() - t) / reps
    out["note"] = ("excluded from value (inputs already resident in HBM when the clock starts); the "
                   "PCIe-inclusive rate adds pageable_ms per batch unless the copy overlaps other batches")
    return out


# PGHR13 batch path, BN254 Fq products per proof: 7 G1 decompressions (Fq sqrt ~315);
# b's decode (norm-method Fq2 sqrt ~700 + the 63-bit G2 membership ~1,870); 9 input combs x 32 mixed
# additions (11) + acc; the Straus sums (9 families: 64 shared doublings / B=2 + ~48 mixed additions +
# q + phi(q)); P_i7 (one GLV product + 4 byte combs); b's 102 lines (64 doublings x 28 + 38 additions x
# 40 in Fq); the segment loops (64 Fq12 squarings shared by K=8 proofs + 102 sparse products x 43)
PGHR13_FQ_PER_PROOF = {"g1_decode": 2205, "g2_decode": 2570, "input_combs": 3312, "straus_sums": 7443,
                       "p7": 1470, "b_lines": 3312, "segment_loops": 4674}


def other_configs(ctx, src_proofs, src_kinds, cpu_threads=0, reps=5):
    """SURVEY.md 8(d) configs 2 and 4 through the host-buffer API zg_verify_batch (PCIe copies,
    OS-RNG scalars and the exact per-proof statuses included), the clean 4,096 batch config 4 is set
    against, and config 5 through the block collector (tools/bench_config5.py, with the C++
    restatement on the same blocks when cpu_threads): not the headline metric."""
    import random
    real = {e["name"]: e for e in json.load(open(os.path.join(ROOT, "tests", "golden", "real_proofs.json")))["proofs"]}
    pts = json.load(open(os.path.join(ROOT, "tests", "golden", "points.json")))
    srcs = ["S1", "S2", "O1", "O2", "O3"]
    rows = {s: [bytes.fromhex(x) for x in real[s]["inputs"]] for s in srcs}
    from zebra_amd import pack_inputs
    res = {}
    # config 2: 1,024 spends, proof i = S[i mod 2] re-randomized with seed 1
    idx = [i % 2 for i in range(1024)]
    proofs = ctx.synth_rerandomize(src_proofs, src_kinds, idx, 1)
    kinds = bytes(src_kinds[j] for j in idx)
    inputs = pack_inputs([rows[srcs[j]] for j in idx])
    ctx.verify_batch(proofs, kinds, inputs)
    t = time.perf_counter()
    for _ in range(reps):
        sts, _ = ctx.verify_batch(proofs, kinds, inputs)
    dt = (time.perf_counter() - t) / reps
    assert sts == [0] * 1024
    res["config2_1024_spends"] = {"proofs_per_s": 1024 / dt, "ms_per_batch": dt * 1e3, "all_ok": True}
    # config 4: 4,096 mixed, 41 corrupted (seed 3) -> exact reject set via bisection
    n = 4096
    idx = [i % 5 for i in range(n)]
    proofs = bytearray(ctx.synth_rerandomize(src_proofs, src_kinds, idx, 3))
    rowsl = [list(rows[srcs[j]]) for j in idx]
    rng = random.Random(3)
    bad = sorted(rng.sample(range(n), 41))
    want = [0] * n
    for q, i in enumerate(bad):
        if q % 3 == 0:
            x = bytearray(rowsl[i][0])
            x[0] ^= 1
            rowsl[i][0] = bytes(x)
            want[i] = 3
        elif q % 3 == 1:
            p = proofs[192 * i:192 * i + 192]
            proofs[192 * i:192 * i + 192] = p[144:] + p[48:144] + p[:48]
            want[i] = 3
        else:
            proofs[192 * i + 48:192 * i + 144] = bytes.fromhex(pts["g2_not_in_subgroup"])
            want[i] = 1
    kinds = bytes(src_kinds[j] for j in idx)
    inputs = pack_inputs(rowsl)
    ctx.verify_batch(bytes(proofs), kinds, inputs)
    t = time.perf_counter()
    for _ in range(reps):
        sts, _ = ctx.verify_batch(bytes(proofs), kinds, inputs)
    dt = (time.perf_counter() - t) / reps
    assert sts == want, "config 4 reject set differs"
    res["config4_4096_1pct_corrupted"] = {"proofs_per_s": n / dt, "ms_per_batch": dt * 1e3, "rejected": len(bad),
                                          "exact_reject_set": True}
    # the same 4,096 proofs uncorrupted: what config 4's bisection is set against
    clean = ctx.synth_rerandomize(src_proofs, src_kinds, idx, 3)
    cin = pack_inputs([rows[srcs[j]] for j in idx])
    ctx.verify_batch(clean, kinds, cin)
    t = time.perf_counter()
    for _ in range(reps):
        sts, _ = ctx.verify_batch(clean, kinds, cin)
    dt4 = (time.perf_counter() - t) / reps
    assert sts == [0] * n
    res["clean_4096_ms"] = dt4 * 1e3
    res["config4_over_clean_4096"] = dt / dt4
    from tools import bench_config5
    res["config5_replay"] = bench_config5.run(ctx, cpu_threads)
    return res


def lineprod_parts(m, ncu, ncoeff=68, pmax=8):
    """the step-part bounds zg.hip lineprod_parts chooses by default (wave-aligned parts) for m groups"""
    bps = (m + 63) // 64
    first, spw = 2 * max(1, ncu // bps), max(1, (ncu - bps) // bps)
    ln = 2 * spw
    while 1 + (ncoeff - min(first, ncoeff) + ln - 1) // ln > pmax:
        ln += spw
    b, n = [], 0
    while n < ncoeff:
        b.append(n)
        n += first if len(b) == 1 else ln
    return b + [ncoeff]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--proofs", "--n", dest="n", type=int, default=65536, help="total proofs per step (all ranks)")
    ap.add_argument("--inflight", type=int, default=0,
                    help="batches in flight per GPU, one context each (0: the default, 6)")
    ap.add_argument("--sync-verdict", action="store_true",
                    help="take each batch's verdict (gather + final exponentiation) before relaunching its context")
    # (round 6) 0 = auto: two checkers in a single process (8k, 8 in flight: 2.36 vs 2.51 ms per batch with one),
    # one under RCCL, where a second checker's high-priority stream pair beside RCCL's costs 6-13 % (8k 2.57 vs
    # 2.79, 32k 6.69 vs 7.60 ms; profiles/r06w_rccl_priority.txt, r06y)
    ap.add_argument("--checkers", type=int, default=0,
                    help="verdict threads, one checker context each (final exponentiations of consecutive batches "
                         "overlap), instead of the coalescing thread; 0: the coalescing thread, or with --coalesce "
                         "off 2, or 1 under torch.distributed")
    # (round 6) the coalescing checker is the default: under RCCL it beats the single checker (8k shards
    # 2.38-2.39 vs 2.51-2.55 ms per batch, 64k 12.12-12.21 vs 12.25-12.32) without a second high-priority
    # stream pair beside RCCL's; in a single process it ties the two-checker pool (six alternating repeats on
    # two boxes: 8k 2.332 vs 2.343, 64k 12.246 vs 12.243 mean ms) with one checker context instead of two;
    # at the default stream priority it is slower (8k 2.341, 64k 12.300). profiles/r06zc_coalesce.txt,
    # r06zh_coalesce_priority.txt
    ap.add_argument("--coalesce", choices=["auto", "on", "off"], default="auto",
                    help="one verdict thread that checks every gathered batch waiting for it in one launch "
                         "(Context.gt_check_many, one final exponentiation per batch side by side) instead of "
                         "--checkers threads; auto: on unless --checkers is given")
    ap.add_argument("--no-priority", action="store_true",
                    help="default-priority streams for the checker context and RCCL")
    ap.add_argument("--rccl-priority", choices=["high", "normal"], default="high",
                    help="RCCL's stream priority (the checkers keep theirs unless --no-priority)")
    ap.add_argument("--dist", action="store_true", help="use torch.distributed (RCCL) even at world size 1")
    ap.add_argument("--no-iso", action="store_true", help="skip the isolated-launch pass (profiling the timed launches)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-configs", action="store_true", help="skip the config 2 / config 4 side measurements")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="0: every CPU this process may use, capped by OMP_NUM_THREADS (the box's share)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # --dist: the RCCL path even at world size 1 (a 1-GPU rehearsal of the multi-GPU protocol)
    use_dist = world > 1 or args.dist
    if args.inflight <= 0:
        # small shards need more batches on the device to fill it (8k-proof shards, round 2:
        # 4 -> 3.54, 5 -> 3.28, 6 -> 3.20, 8 -> 3.25, 10 -> 3.63 ms per batch; profiles/r02l_inflight_sweep.txt);
        # the slots share the device's fixed stream pool, so the round-1 limit of
        # 6 contexts per process no longer applies
        # (65,536-proof shards, r02v: 2 -> 15.95, 3 -> 16.01, 4 -> 15.67, 5 -> 15.83 ms per batch; on the
        # round-4 kernels, 5 alternating repeats: 4 -> 14.02, 6 -> 13.78, 8 -> 13.91 mean ms per batch,
        # 6 the fastest in every repeat, profiles/r04y_inflight_64k.txt)
        # (round 6, profiles/r06m_depths.txt, one box: 8k shards 6 -> 2.60, 8 -> 2.40, 10 -> 2.53, 12 -> 2.98 ms
        # per batch; 16k 6 -> 4.01, 8 -> 4.02; 32k 6 -> 6.80, 8 -> 6.90; 64k 6 -> 12.21, 8 -> 12.28)
        args.inflight = 8 if (args.n + world - 1) // world <= 8192 else 6
    # two streams per context (main + side): give each its own hardware queue (set before the
    # HIP runtime starts; measured: 8k-proof shards 6 in flight 6.4 ms/batch on 4 queues, 5.0 on 12)
    # (RCCL's own streams want queues too: 8k shard over RCCL 5.58 ms/batch at 12 queues, 4.70 at 24)
    # (round 6) a stream pair per batch context (ZG_STREAM_PAIRS, the device pool: deeper pipelines than
    # its default 8 would otherwise share pairs), two hardware queues per pair + the checkers' pairs
    os.environ.setdefault("ZG_STREAM_PAIRS", str(min(16, max(8, args.inflight))))
    hwq = min(32, max(int(os.environ.get("GPU_MAX_HW_QUEUES", "4")), 24, 2 * args.inflight + 8))
    if os.environ.get("ZG_BENCH_HWQ"):   # (tooling: an exact queue count for the sweeps in tools/gpu_r05.sh)
        hwq = min(32, int(os.environ["ZG_BENCH_HWQ"]))
    os.environ["GPU_MAX_HW_QUEUES"] = str(hwq)
    import torch
    import torch.distributed as dist
    if use_dist and "RANK" not in os.environ:  # --dist outside torch.distributed.run: a world of one
        os.environ.update({"RANK": "0", "WORLD_SIZE": "1", "LOCAL_RANK": "0", "MASTER_ADDR": "127.0.0.1",
                           "MASTER_PORT": os.environ.get("MASTER_PORT", str(29500 + os.getpid() % 1000))})
    if use_dist:
        # RCCL prints its version banner on stdout while it initialises: keep stdout for the one
        # JSON line (fd-level, the banner comes from C)
        sys.stdout.flush()
        saved = os.dup(1)
        os.dup2(2, 1)
        try:
            opts = None
            if not args.no_priority and args.rccl_priority == "high":   # the 576-B gathers jump the queue
                opts = dist.ProcessGroupNCCL.Options()
                opts.is_high_priority_stream = True
            dist.init_process_group("nccl", device_id=torch.device("cuda", local), pg_options=opts)
            dist.barrier()
        finally:
            sys.stdout.flush()
            os.dup2(saved, 1)
            os.close(saved)
    torch.cuda.set_device(local)

    from zebra_amd import Context
    from zebra_amd.dist import combine_partials, gather_partials, run_pipelined, run_pipelined_deferred
    src_proofs, src_kinds, idx, kinds, inputs, shard = workload(rank, world, args.n)
    ctx = Context(device=local, max_batch=shard)
    # batches in flight per GPU: each has its own context (buffers + streams); while the host
    # waits on the oldest batch's partial / verdict, the next one is already on the device
    ctxs = [ctx] + [Context(device=local, max_batch=shard) for _ in range(args.inflight - 1)]
    # the verdicts (gather + final exponentiation) run on a checker context of their own, on a
    # worker thread in batch order, so a batch context is relaunched as soon as its partial and
    # statuses are read (zebra_amd.dist.run_pipelined_deferred)
    # (round 6) --checkers contexts, one per verdict thread: consecutive batches' final exponentiations
    # overlap (zebra_amd.dist.run_pipelined_deferred gather / checks)
    coalesce = (args.coalesce == "on" or (args.coalesce == "auto" and args.checkers <= 0)) \
        and not args.sync_verdict
    nck = 1 if coalesce else args.checkers if args.checkers > 0 else (1 if use_dist else 2)
    checkers = [] if args.sync_verdict else [Context(device=local, max_batch=64) for _ in range(nck)]
    for chk in checkers:
        if not args.no_priority:
            chk.set_priority(True)
    free_checkers = queue.SimpleQueue()
    for chk in checkers:
        free_checkers.put(chk)
    t0 = time.perf_counter()
    proofs = ctx.synth_rerandomize(src_proofs, src_kinds, idx, 2 + 1000003 * rank)
    log("rank %d: generated %d re-randomized proofs in %.1f s" % (rank, shard, time.perf_counter() - t0))
    peak, clock_hz = ctx.bench_mad_rate(with_clock=True)

    dev = torch.device("cuda", local)
    d_proofs = torch.frombuffer(bytearray(proofs), dtype=torch.uint8).to(dev)
    d_kinds = torch.frombuffer(bytearray(kinds), dtype=torch.uint8).to(dev)
    d_inputs = torch.frombuffer(bytearray(inputs), dtype=torch.uint8).to(dev)
    timings = []

    ltime = []   # host seconds per batch in zg_batch_begin_device (the pipeline's launches)

    def launch(c):
        t0 = time.perf_counter()
        c.batch_begin_device(shard, d_proofs.data_ptr(), d_kinds.data_ptr(), d_inputs.data_ptr())
        ltime.append(time.perf_counter() - t0)

    host = []   # per batch: host seconds waiting for the partial, in the exchange + check, in finish

    def check(part, on):
        if use_dist:   # RCCL over xGMI: 576 B per GPU, the final exponentiation of their product
            return combine_partials(part, on.gt_check, world, rank, dev)
        return on.gt_check([part])

    def complete(c):
        t0 = time.perf_counter()
        part = c.batch_partial()
        timings.append(c.last_timings())
        t1 = time.perf_counter()
        ok = check(part, c)
        t2 = time.perf_counter()
        sts = c.batch_finish(ok, shard)
        host.append((t1 - t0, t2 - t1, time.perf_counter() - t2))
        return ok, sts

    def harvest(c):
        t0 = time.perf_counter()
        part = c.batch_partial()
        timings.append(c.last_timings())
        t1 = time.perf_counter()
        sts = c.batch_finish(True, shard)   # provisional: a false verdict re-runs the batch (redo)
        host.append((t1 - t0, 0.0, time.perf_counter() - t1))
        return part, sts

    def gather(part):   # ordered stage: the exchange (RCCL all-gather at world > 1)
        return gather_partials(part, world, rank, dev) if use_dist else [part]

    def verdict(parts):  # pooled stage: ONE final exponentiation of the gathered partials' product
        t0 = time.perf_counter()
        chk = free_checkers.get()
        try:
            ok = chk.gt_check(parts)
        finally:
            free_checkers.put(chk)
        vtime.append(time.perf_counter() - t0)
        return ok

    vsets = []   # coalescing checker: batches per gt_check_many call

    def verdict_many(sets):   # the coalescing checker: every waiting batch's final exponentiation at once
        t0 = time.perf_counter()
        oks = checkers[0].gt_check_many(sets)
        dt = time.perf_counter() - t0
        vtime.extend([dt / len(sets)] * len(sets))
        vsets.append(len(sets))
        return oks

    def redo(_s):
        launch(ctx)
        return complete(ctx)[1]

    vtime = []

    def run(k):
        if args.sync_verdict:
            return run_pipelined(ctxs, k, launch, complete)
        return run_pipelined_deferred(ctxs, k, launch, harvest, verdict, redo, ready=lambda c: c.batch_ready(),
                                      gather=gather, checks=len(checkers),
                                      verdict_many=verdict_many if coalesce else None)

    def barrier():
        if use_dist:
            dist.barrier()
        torch.cuda.synchronize()

    run(args.warmup)
    timings.clear()
    host.clear()
    vtime.clear()
    vsets.clear()
    ltime.clear()
    barrier()
    import resource
    ru0 = resource.getrusage(resource.RUSAGE_SELF)
    t0 = time.perf_counter()
    results = run(args.steps)
    torch.cuda.synchronize()
    barrier()
    dt = time.perf_counter() - t0
    ru1 = resource.getrusage(resource.RUSAGE_SELF)
    cpu_busy = (ru1.ru_utime - ru0.ru_utime + ru1.ru_stime - ru0.ru_stime) / dt   # CPUs busy on average
    if use_dist:
        tt = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
    for ok, sts in results:
        assert ok and all(s == 0 for s in sts), "valid synthetic batch rejected"

    host_ms = [1e3 * sum(h[i] for h in host) / len(host) for i in range(3)]
    if vtime:   # deferred verdicts: the worker thread's time per batch (overlaps the next batches)
        host_ms[1] = 1e3 * sum(vtime) / len(vtime)
    # isolated launches (one batch in flight, after the timed region): the kernels' own roofline
    # (ZG_SERIAL_SIDE: this context runs the side-stream work -- K4 and the root's VK pairs -- on
    # its main stream after the product tree, so the Miller kernels are alone on the device)
    iso, k4_entries = [], None
    if not args.no_iso:
        os.environ["ZG_SERIAL_SIDE"] = "1"
        try:
            ictx = Context(device=local, max_batch=shard)
        finally:
            del os.environ["ZG_SERIAL_SIDE"]
        for _ in range(3):
            launch(ictx)
            ok_, sts_ = complete(ictx)
            iso.append(timings.pop())
            assert ok_ and all(x == 0 for x in sts_)
        k4_entries = ictx.stats()["k4_entries"]
        ictx.close()

    h2d = h2d_copy_ms(proofs, kinds, inputs, dev)
    total = shard * world
    value = total * args.steps / dt
    names = list(Context.PHASES)
    NP = len(names)
    # phases = HIP events around launch groups; decode = k_decode_sqrt + k_decode_points + k_decode_finish
    avg = [sum(t[i] for t in timings) / len(timings) for i in range(NP)]
    # roofline of the dominant single kernel: the f-chain (the R-chain + f-chain launch when the
    # shard runs them fused -- its lines phase is then empty), algorithmic MACs per launch over
    # its mean launch duration (HIP events, timed region; with batches in flight a launch shares
    # the device with the other batch's kernels)
    if not iso:
        iso = timings
    fused = iso[0][1] < 0.05   # the fused launch leaves the lines phase empty (isolated pass)
    st0 = ctx.stats()
    quads = st0.get("quad_fchain_launches", 0) > 0  # four proofs per lane (k_batch_fchain4)
    # group line products (k_line_prod) + one chain per group (k_batch_fchaing): the f-chain phase
    # is the two launches back to back; the work stays the frozen per-proof Miller-loop count
    lprod = st0.get("line_product_batches", 0) > 0
    rk, wk = ("k_lines_fchain", W_LINES + W_FCHAIN) if fused else \
        ("k_line_prod+k_batch_fchaing" if lprod else "k_batch_fchain4" if quads else "k_batch_fchain", W_FCHAIN)
    achieved = wk * MACS_PER_FQMUL * shard / (avg[2] * 1e-3)
    iso_avg = [sum(t[i] for t in iso) / len(iso) for i in range(NP)]
    iso_achieved = wk * MACS_PER_FQMUL * shard / (iso_avg[2] * 1e-3)
    phase_frac = {names[i]: w * MACS_PER_FQMUL * shard / (iso_avg[i] * 1e-3) / peak
                  for i, w in ((0, W_DECODE), (1, W_LINES), (2, W_FCHAIN), (7, W_K4)) if iso_avg[i] >= 0.05}
    traffic = k4_traffic = None
    pmc = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if os.path.exists(pmc) and shard == 65536 and not fused:   # the PMC passes run the default 64k bench
        pt = json.load(open(pmc))
        traffic, k4_traffic = pt.get(rk), pt.get("k_msm_bucket")
        if "+" in rk:  # the line-product phase: each kernel runs once per step part
            parts = int(os.environ.get("ZG_LINE_PROD_PARTS", "0")) or len(lineprod_parts(
                shard // 32, torch.cuda.get_device_properties(dev).multi_processor_count)) - 1
            got = [pt.get(k) for k in rk.split("+")]
            traffic = parts * sum(got) if all(g is not None for g in got) else None
    k4 = None
    if k4_entries is not None and iso_avg[8] > 0:
        npad = 1 << max(1, (shard - 1).bit_length())
        k4_bytes = k4_entries * K4_ENTRY_BYTES + k4_fixed_bytes(npad)
        k4 = {"kernel": "k_msm_bucket", "bound": "hbm", "entries": k4_entries, "algorithmic_bytes": k4_bytes,
              "ms": iso_avg[8], "achieved_gbs": k4_bytes / (iso_avg[8] * 1e-3) / 1e9, "peak_gbs": 8000.0,
              "frac": k4_bytes / (iso_avg[8] * 1e-3) / 8e12, "traffic": k4_traffic,
              "k4_total_ms": iso_avg[7],
              "note": "HBM GB/s of the Pippenger bucket phase (isolated pass, HIP events around "
                      "k_msm_bucket): entries x (4-B entry + 112-B digit operands of C_i) + segment sums written; "
                      "the phase is VALU-bound (mixed additions), not HBM-bound"}
    out = {
        "metric": "Sapling Groth16 proofs verified/sec (batch 64k) at 1/2/4/8 MI355X",
        "value": value, "unit": "proofs/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": dt / args.steps * 1e3, "higher_is_better": True, "scaling": "strong",
        "vs_baseline": None, "dtype": "u32", "data": "synthetic: real mainnet proofs (reference fixtures) "
        "re-randomized on GPU, all valid",
        "config": {"workload": "config 3: 65,536 mixed Sapling spend/output Groth16 proofs, contiguous shard per "
                               "GPU, one final exponentiation per batch; inputs HBM-resident (H2D copies excluded, "
                               "see h2d_ms_per_batch)",
                   "collective": ("RCCL all-gather of the %d ranks' 576-B Miller partials (torch.distributed nccl)"
                                  % world) if use_dist else
                                 "none (dp1: the one 576-B partial goes straight to the final exponentiation)",
                   "global_batch": total, "shard": shard, "parallelism": "dp%d" % world,
                   "batches_in_flight_per_gpu": len(ctxs), "hw_queues": hwq},
        # headline: the dominant kernel ALONE on the GPU (isolated pass); the in-flight launch
        # shares the device with the other batches' kernels, which stretches its duration
        "roofline": {"bound": "valu-int (v_mad_u64_u32)", "kernel": rk, "achieved": iso_achieved / 1e12,
                     "peak": peak / 1e12, "unit": "T u32-MAC/s", "frac": iso_achieved / peak, "traffic": traffic,
                     "work_per_proof_fq_mul_eq": wk, "kernel_ms": iso_avg[2],
                     "peak_probe": {"clock_ghz": clock_hz / 1e9, "macs_per_clock": peak / clock_hz if clock_hz else None,
                                    "nominal_peak_2p4ghz": NOMINAL_LANES * 2.4e9 / 1e12,
                                    "frac_of_nominal": iso_achieved / (NOMINAL_LANES * 2.4e9),
                                    "note": "peak = measured v_mad_u64_u32 chains (k_mad_rate, full occupancy) "
                                            "at the clock the chip held (s_memtime / s_memrealtime); nominal = "
                                            "256 CU x 4 SIMD x 16 lanes x 2.4 GHz, one MAC per lane per clock"},
                     "phase_ms": dict(zip(names, iso_avg)), "phase_frac": phase_frac,
                     "note": "no isolated pass (--no-iso): same launches as roofline_inflight" if args.no_iso else
                             "3 batches with one in flight after the timed region, side-stream work serialised "
                             "after the product tree (ZG_SERIAL_SIDE): the kernels alone on the GPU"},
        "roofline_inflight": {"kernel": rk, "achieved": achieved / 1e12, "frac": achieved / peak,
                              "kernel_ms": avg[2], "note": "mean launch duration inside the timed region, "
                              "sharing the GPU with the other batches in flight"},
        "k4_msm_bucket_phase": k4,
        "job_roofline_frac": value * W_TOTAL * MACS_PER_FQMUL / peak,
        "phase_ms": dict(zip(names, avg)),
        "h2d_ms_per_batch": h2d,
        "host_ms_per_batch": {"launch": 1e3 * sum(ltime) / max(1, len(ltime)), "wait_partial": host_ms[0],
                              "exchange_and_final_exp": host_ms[1], "statuses": host_ms[2],
                              "process_cpus_busy": cpu_busy,
                              "verdict": "sync" if args.sync_verdict else
                              ("deferred (ordered gather thread, one coalescing verdict thread: %.2f batches per "
                               "gt_check_many launch)" % (sum(vsets) / max(1, len(vsets))) if coalesce else
                               "deferred (ordered gather thread, %d verdict threads with a checker context each)"
                               % len(checkers))},
    }
    if rank == 0 and world == 1 and not args.no_configs:
        out["other_configs"] = other_configs(ctx, src_proofs, src_kinds, 0 if args.no_cpu else cpu_threads(args.cpu_threads))
        # note-commitment tree windows (tools/bench_tree.py), not the headline
        from tools import bench_tree
        from zebra_amd import zg as _zg
        trees = {"workload": "1,024 blocks x 64 commitments (65,536 leaves, a root per block) onto a "
                             "2^30-leaf frontier, leaves HBM-resident (zg_tree_roots_device)"}
        for name, kind, h in (("sapling_h32", _zg.TREE_SAPLING, 32), ("sprout_h29", _zg.TREE_SPROUT, 29)):
            trees[name] = bench_tree.run(ctx, kind, h, 65536, 64, 10)
            if not args.no_cpu:
                trees[name]["cpu_baseline"] = bench_tree.cpu_window(kind, h, 64, 4.0, cpu_threads(args.cpu_threads))
                trees[name]["gpu_over_cpu"] = trees[name]["leaves_per_s"] / trees[name]["cpu_baseline"]["leaves_per_s"]
        out["note_commitment_trees"] = trees
        # PGHR13 Sprout proofs on BN254 (tools/bench_pghr13.py), not the headline
        from tools import bench_pghr13
        pg = bench_pghr13.run(ctx, 65536, 2)
        pg["workload"] = ("65,536 PHGR JoinSplit proofs cycling through the 9 valid reference / block-522 "
                          "statements; host buffers (zg_pghr13_verify)")
        if not args.no_cpu:
            pg["cpu_baseline"] = bench_pghr13.cpu_baseline(4.0, cpu_threads(args.cpu_threads))
            pg["gpu_over_cpu"] = pg["proofs_per_s"] / pg["cpu_baseline"]["proofs_per_s"]
        # roofline ESTIMATE for the side line: BN254 Fq products per proof of the batch path counted from
        # its operations (2 x 8^2 u32 MACs each, the word-form unit like the headline's
        # 2 x 12^2), over the call's kernel time, against the same measured v_mad_u64_u32 peak
        w = PGHR13_FQ_PER_PROOF
        ach = sum(w.values()) * 128 * pg["proofs"] / (max(pg["kernel_ms"], 1e-6) * 1e-3) / 1e12
        pg["roofline_est"] = {"bound": "valu-int (v_mad_u64_u32)", "achieved": ach, "peak": peak / 1e12,
                              "unit": "T u32-MAC/s", "frac": ach / (peak / 1e12), "traffic": None,
                              "work_per_proof_bn_fq_mul": w,
                              "note": "estimate: per-proof operation counts of the batch path (one check per call; "
                                      "the per-segment trees and the one final exponentiation per call are not "
                                      "counted), not measured instruction counts"}
        out["pghr13_sprout_proofs"] = pg
    if rank == 0 and world == 1 and not args.no_cpu:
        out["cpu_baseline"] = cpu_baseline(proofs, kinds, inputs, args.cpu_seconds, cpu_threads(args.cpu_threads))
        out["gpu_over_cpu"] = value / out["cpu_baseline"]["value"]
        out["gpu_over_cpu_all_usable_projected"] = value / out["cpu_baseline"]["projected_all_usable_cpus"]["value"]
    st = {}
    for c in ctxs:
        for k, v in c.stats().items():
            st[k] = st.get(k, 0) + v
    out["context_stats"] = st
    if rank == 0:
        print(json.dumps(out), flush=True)
    for c in ctxs + checkers:
        c.close()
    if use_dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
