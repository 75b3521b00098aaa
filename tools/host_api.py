#!/usr/bin/env python3
"""Host-side HIP API time of a pipelined run (tooling), from a rocprofv3 rocpd .db recorded with
--hip-trace: over the span of the Groth16 batches (first to last k_chacha20 launch), per host
thread, the API calls by total time (count, total ms, mean / max us), and the longest single
calls with their start relative to the span. Shows whether a thread sits inside a blocking call
(synchronize, pageable copies) while the device waits for it.
Usage: host_api.py run_results.db [out.txt]"""
import sqlite3
import sys


def main():
    db = sqlite3.connect(sys.argv[1])
    marks = [r[0] for r in db.execute("select start from kernels where name like '%k_chacha20%' order by start")]
    t0, t1 = marks[0], marks[-1]
    rows = db.execute("select tid, name, start, end from regions where start >= ? and start <= ? order by start",
                      (t0, t1)).fetchall()
    out = ["span %.3f ms, %d API calls" % ((t1 - t0) / 1e6, len(rows))]
    by = {}
    for tid, name, s, e in rows:
        a = by.setdefault(tid, {}).setdefault(name, [0, 0.0, 0.0])
        a[0] += 1
        a[1] += (e - s) / 1e6
        a[2] = max(a[2], (e - s) / 1e3)
    for tid, calls in sorted(by.items(), key=lambda kv: -sum(v[1] for v in kv[1].values())):
        tot = sum(v[1] for v in calls.values())
        out.append("thread %s: %.2f ms inside the API (%.1f %% of the span)" % (tid, tot, 100 * tot * 1e6 / (t1 - t0)))
        for name, (c, ms, mx) in sorted(calls.items(), key=lambda kv: -kv[1][1])[:10]:
            out.append("  %-32s %6d x  %9.3f ms  mean %8.1f us  max %8.1f us" % (name[:32], c, ms, 1e3 * ms / c, mx))
    longest = sorted(rows, key=lambda r: r[2] - r[3])[:15]
    out.append("longest calls:")
    for tid, name, s, e in longest:
        out.append("  thread %s %-32s at %9.3f ms  %8.1f us" % (tid, name[:32], (s - t0) / 1e6, (e - s) / 1e3))
    text = "\n".join(out)
    if len(sys.argv) > 2:
        open(sys.argv[2], "w").write(text + "\n")
    print(text)


if __name__ == "__main__":
    main()
