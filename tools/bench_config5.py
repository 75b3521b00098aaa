"""Config 5: a replayed block import mixing Sprout-Groth16 JoinSplits and Sapling
spends / outputs, timed through the block-level collector (zebra_amd/collector.py verify_block, the
caller side of accept_chain.rs:76-81) -- not the headline metric; bench.py's other_configs.

Blocks are built like tests/test_collector.py::test_config5_replay_block_stream: the reference's real
transactions (tests/golden/input_prep.json tx fields, real_proofs.json proofs), their Groth16 proofs
re-randomized on the GPU per block, Sprout-Groth16 : Sapling = 1 : 4 by proof count. Measured:

  * import windows: consecutive blocks verified with ONE verify_block call per window (the f2 import
    window, blocks_writer.rs:63-90 batched), proofs/s at window sizes of 1 and all blocks;
  * lone blocks: the median verify_block latency of one block alone, at the replay's block size and
    at a small block of one transaction per source;
  * the oracle's C++ bellman restatement (oracle/cpu/bellman_cpu.cpp, checker / CPU baseline only)
    through the same collector on the same blocks, on the job's CPU threads.

Every proof goes to the GPU, whatever the block size (the product has no CPU verification path,
DESIGN.md §5). The public-input preparation of a window from 64 descriptions runs as one
zg_prep_batch call (Sapling descriptions on the GPU), below that on the host functions, as the
reference prepares them on the host (collector._GPU_PREP_MIN).
"""
import json
import os
import random
import statistics
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SRC_TX = {"bd4fe81c": ["S1", "O1"], "smoky": ["J1"], "991edf59": ["S2", "O3"], "56afac11": ["O2"],
          "53cf8971": ["J2"], "a2a2fe38": ["J3"], "70abe357": ["J4"]}
NAMES = ["S1", "S2", "O1", "O2", "O3", "J1", "J2", "J3", "J4"]


def _golden(name):
    return json.load(open(os.path.join(ROOT, "tests", "golden", name)))


def _fields():
    tf = _golden("input_prep.json")["tx_fields"]
    return {e["name"]: e for kind in ("spends", "outputs", "joinsplits") for e in tf[kind]}


def _tx(names, F, proof):
    from zebra_amd.collector import JoinSplit, Output, Spend, Tx
    h = bytes.fromhex
    tx = Tx()
    for nm in names:
        e = F[nm]
        if nm[0] == "J":
            tx.js_pubkey = h(e["pubkey"])
            tx.joinsplits.append(JoinSplit(h(e["anchor"]), h(e["random_seed"]), [h(x) for x in e["nullifiers"]],
                                           [h(x) for x in e["macs"]], [h(x) for x in e["commitments"]],
                                           e["vpub_old"], e["vpub_new"], proof[nm]))
        elif nm[0] == "S":
            tx.spends.append(Spend(h(e["cv"]), h(e["anchor"]), h(e["nullifier"]), h(e["rk"]), proof[nm]))
        else:
            tx.outputs.append(Output(h(e["cv"]), h(e["cmu"]), h(e["epk"]), proof[nm]))
    return tx


def build_blocks(ctx, nblocks, per_block, seed):
    """nblocks blocks of about per_block proofs each (lists of collector.Tx), Sprout : Sapling 1 : 4"""
    F = _fields()
    real = {e["name"]: e for e in _golden("real_proofs.json")["proofs"]}
    src = b"".join(bytes.fromhex(real[n]["proof"]) for n in NAMES)
    kinds = bytes(real[n]["kind"] for n in NAMES)
    rng = random.Random(seed)
    sap = [v for v in SRC_TX.values() if v[0][0] != "J"]
    spr = [v for v in SRC_TX.values() if v[0][0] == "J"]
    blocks = []
    for bi in range(nblocks):
        names, nsap, nspr = [], 0, 0
        while nsap + nspr < per_block:
            if nspr * 4 < nsap:
                pick = rng.choice(spr)
                nspr += len(pick)
            else:
                pick = rng.choice(sap)
                nsap += len(pick)
            names.append(pick)
        flat = [n for t in names for n in t]
        rr = ctx.synth_rerandomize(src, kinds, [NAMES.index(n) for n in flat], seed * 1000 + bi)
        k, txs = 0, []
        for t in names:
            cur = {}
            for n in t:
                cur[n] = rr[192 * k:192 * k + 192]
                k += 1
            txs.append(_tx(t, F, cur))
        blocks.append((txs, len(flat)))
    return blocks


def _windows(blocks, w):
    return [blocks[i:i + w] for i in range(0, len(blocks), w)]


def run(ctx, cpu_threads, nblocks=24, per_block=400, reps=3, cpu_blocks=3):
    from zebra_amd.collector import verify_block
    blocks = build_blocks(ctx, nblocks, per_block, 5)
    small = build_blocks(ctx, 8, 9, 6)   # one transaction per source: ~9 proofs
    total = sum(n for _, n in blocks)
    out = {"workload": "%d replayed blocks of ~%d proofs (Sprout-Groth16 : Sapling = 1 : 4 by proof count, "
                       "re-randomized reference transactions), %d proofs; collector.verify_block" % (nblocks, per_block, total)}
    for txs, _ in blocks[:2]:  # warm-up
        assert verify_block(txs, ctx=ctx) is None
    win = {}
    for w in (1, nblocks):
        best = None
        for _ in range(reps):
            t = time.perf_counter()
            for group in _windows(blocks, w):
                assert verify_block([tx for txs, _ in group for tx in txs], ctx=ctx) is None
            dt = time.perf_counter() - t
            best = dt if best is None else min(best, dt)
        win["window_%d_blocks" % w] = {"proofs_per_window": total // len(_windows(blocks, w)),
                                       "proofs_per_s": total / best, "ms_per_window": 1e3 * best / len(_windows(blocks, w))}
    out["import_windows"] = win

    def lone(bl, fn):
        ms = []
        for txs, _ in bl:
            t = time.perf_counter()
            assert fn(txs) is None
            ms.append(1e3 * (time.perf_counter() - t))
        return statistics.median(ms)
    gpu = lambda txs: verify_block(txs, ctx=ctx)
    out["lone_block_ms"] = {"block_%d_proofs" % blocks[0][1]: lone(blocks[:8], gpu),
                            "block_%d_proofs" % small[0][1]: lone(small, gpu)}
    if not cpu_threads:
        return out
    # the C++ bellman restatement through the same collector (checker code: CPU baseline only)
    from tests import cpulib
    L = cpulib.load()

    def cpu(txs):
        return verify_block(txs, verify=lambda p, k, i, n: cpulib.verify(L, p, k, i, n, threads=cpu_threads)[0])
    t = time.perf_counter()
    for txs, _ in blocks[:cpu_blocks]:
        assert cpu(txs) is None
    dt = time.perf_counter() - t
    ncpu = sum(n for _, n in blocks[:cpu_blocks])
    out["cpu_restatement"] = {"threads": cpu_threads, "proofs_per_s": ncpu / dt, "sample_blocks": cpu_blocks,
                              "lone_block_ms": {"block_%d_proofs" % blocks[0][1]: 1e3 * dt / cpu_blocks,
                                                "block_%d_proofs" % small[0][1]: lone(small[:4], cpu)},
                              "kind": "port (oracle/cpu/bellman_cpu.cpp, one proof per task)"}
    out["gpu_over_cpu_window"] = win["window_%d_blocks" % nblocks]["proofs_per_s"] / out["cpu_restatement"]["proofs_per_s"]
    return out
