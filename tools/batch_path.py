#!/usr/bin/env python3
"""Per-batch critical path of a pipelined run (tooling), from a rocprofv3 rocpd .db.

A batch starts with k_chacha20 on its context's main stream; the context's side stream is the
next stream id (zg.hip: a slot uses one (main, side) pair). For every batch, each kernel's
start / end relative to the batch's k_chacha20 start, main and side stream; printed as the
mean over the batches (excluding the first and last two per stream), in time order, with the
gap each kernel waited on its stream. Usage: batch_path.py run_results.db [out.txt]"""
import sqlite3
import sys


def main():
    db = sqlite3.connect(sys.argv[1])
    cols = [r[1] for r in db.execute("pragma table_info(kernels)").fetchall()]
    sid = next((c for c in ("stream_id", "queue_id", "stream", "queue") if c in cols), None)
    rows = db.execute("select name, start, end, %s from kernels order by start" % sid).fetchall()
    short = lambda n: n.split("(")[0].replace("zg::", "").replace("void ", "")
    mains = sorted({r[3] for r in rows if "k_chacha20" in r[0]})
    acc = {}
    nb = 0
    for m in mains:
        ks = [r for r in rows if r[3] == m]
        side = [r for r in rows if r[3] == m + 1]
        starts = [r[1] for r in ks if "k_chacha20" in r[0]]
        for bi in range(1, len(starts) - 2):
            t0, t1 = starts[bi], starts[bi + 1]
            nb += 1
            seen = {}
            for tag, lst in (("M", ks), ("S", side)):
                prev = None
                for n, s, e, _ in lst:
                    if s < t0 or s >= t1:
                        if s < t0:
                            prev = e
                        continue
                    key = (tag, short(n))
                    c = seen.get(key, 0)
                    seen[key] = c + 1
                    k2 = (tag, short(n), c)
                    a = acc.setdefault(k2, [0, 0.0, 0.0, 0.0])
                    a[0] += 1
                    a[1] += (s - t0) / 1e3
                    a[2] += (e - t0) / 1e3
                    a[3] += max(0, s - prev) / 1e3 if prev is not None else 0
                    prev = e
    out = ["%d batches (mean over batches; us from the batch's k_chacha20 start)" % nb,
           "%-3s %-32s %4s %9s %9s %8s %8s" % ("st", "kernel", "#", "start", "end", "dur", "gap")]
    items = sorted(acc.items(), key=lambda kv: kv[1][1] / kv[1][0])
    for (tag, n, c), (k, s, e, g) in items:
        if k < nb // 2:
            continue
        out.append("%-3s %-32s %4d %9.0f %9.0f %8.0f %8.0f" % (tag, n[:32], c, s / k, e / k, (e - s) / k, g / k))
    text = "\n".join(out)
    if len(sys.argv) > 2:
        open(sys.argv[2], "w").write(text + "\n")
    print(text)


if __name__ == "__main__":
    main()
