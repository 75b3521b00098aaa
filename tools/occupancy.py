#!/usr/bin/env python3
"""Device occupancy and stream gaps of a pipelined run (tooling), from a rocprofv3 rocpd .db.

Over the span of the Groth16 batches (first to last k_chacha20 launch):
  * resident waves over time: the sum over running kernels of their grid's waves, capped at the
    chip's wave slots (2 per SIMD for the ~256-VGPR kernels: 2,048) -- the share of time spent
    below 25 / 50 / 75 / 100 % of the slots;
  * per stream: busy time (union of its kernels) and the gaps between consecutive kernels
    (dispatch + dependency + host waits), with the largest gaps named by the kernel that follows.
Usage: occupancy.py run_results.db [out.txt]"""
import sqlite3
import sys

SLOTS = 2048


def main():
    db = sqlite3.connect(sys.argv[1])
    cols = [r[1] for r in db.execute("pragma table_info(kernels)").fetchall()]
    sid = next((c for c in ("stream_id", "queue_id", "stream", "queue") if c in cols), None)
    if "stream_id" in cols and "queue_id" in cols:  # which hardware queue serves each stream
        pairs = db.execute("select stream_id, queue_id, count(*) from kernels group by stream_id, queue_id").fetchall()
        print("stream -> queue (kernels): " + ", ".join("%s->%s (%d)" % p for p in sorted(pairs)))
    rows = db.execute("select name, start, end, grid_x * grid_y * grid_z%s from kernels order by start"
                      % (", " + sid if sid else ", 0")).fetchall()
    marks = [r[1] for r in rows if "k_chacha20" in r[0]]
    t0, t1 = min(marks), max(marks)
    rows = [r for r in rows if t0 <= r[1] <= t1]
    out = ["span %.3f ms, %d dispatches, %d batches (k_chacha20 launches)" % ((t1 - t0) / 1e6, len(rows), len(marks) - 1)]
    # resident waves over time (event sweep)
    ev = []
    for name, s, e, thr, _ in rows:
        w = (thr + 63) // 64
        ev.append((s, w))
        ev.append((min(e, t1), -w))
    ev.sort()
    cur, last, hist, area = 0, t0, [0.0] * 5, 0.0
    for t, d in ev:
        if t > last:
            occ = min(cur, SLOTS)
            hist[min(4, occ * 4 // SLOTS)] += t - last
            area += occ * (t - last)
            last = t
        cur += d
    span = t1 - t0
    out.append("resident waves (capped at %d): mean %.0f (%.1f %%)" % (SLOTS, area / span, 100 * area / span / SLOTS))
    for i, lab in enumerate(["<25%", "25-50%", "50-75%", "75-100%", "full"]):
        out.append("  %-8s of slots: %5.1f %% of the time" % (lab, 100 * hist[i] / span))
    # per stream busy / gaps
    by = {}
    for name, s, e, thr, q in rows:
        by.setdefault(q, []).append((s, e, name.split("(")[0].replace("zg::", "").replace("void ", "")))
    out.append("%-8s %6s %9s %9s %9s  largest gaps (us, next kernel)" % ("stream", "kerns", "busy_ms", "gap_ms", "gap/k_us"))
    for q, ks in sorted(by.items(), key=lambda kv: -len(kv[1])):
        busy, gaps, prev_end = 0.0, [], None
        for s, e, n in ks:
            if prev_end is not None:
                gaps.append((max(0, s - prev_end), n))
            busy += e - s
            prev_end = max(prev_end or 0, e)
        g = sum(x for x, _ in gaps)
        top = sorted(gaps, reverse=True)[:3]
        out.append("%-8s %6d %9.2f %9.2f %9.1f  %s" % (q, len(ks), busy / 1e6, g / 1e6, g / max(1, len(gaps)) / 1e3,
                                                       ", ".join("%.0f %s" % (x / 1e3, n[:24]) for x, n in top)))
    # gap distribution between dependent kernels (same stream), by the kernel that follows
    agg = {}
    for q, ks in by.items():
        prev_end = None
        for s, e, n in ks:
            if prev_end is not None:
                a = agg.setdefault(n, [0, 0.0])
                a[0] += 1
                a[1] += max(0, s - prev_end)
            prev_end = max(prev_end or 0, e)
    out.append("mean gap before each kernel (same stream):")
    for n, (c, g) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:16]:
        out.append("  %-34s %6d x %8.1f us = %8.2f ms" % (n[:34], c, g / c / 1e3, g / 1e6))
    text = "\n".join(out)
    if len(sys.argv) > 2:
        open(sys.argv[2], "w").write(text + "\n")
    print(text)


if __name__ == "__main__":
    main()
