#!/usr/bin/env python3
"""Where a pipelined run's device time goes: per kernel, launches, mean duration and WAVE-TIME
(duration x waves of the grid, in wave-ms) from a rocprofv3 rocpd .db, plus the share of the
total and the span of the traced dispatches. When every kernel of a batch is resident at once
(small shards, batches in flight) the wave-time share is the kernel's share of the device.
Usage: wavetime.py run_results.db [out.txt] [--skip-name SUBSTR ...]"""
import sqlite3
import sys


def main():
    args = sys.argv[1:]
    skip = [args[i + 1] for i, a in enumerate(args) if a == "--skip-name"]
    pos = [a for i, a in enumerate(args) if not a.startswith("--") and (i == 0 or args[i - 1] != "--skip-name")]
    db = sqlite3.connect(pos[0])
    rows = db.execute("select name, start, end, grid_x, grid_y, grid_z, workgroup_x, workgroup_y, workgroup_z "
                      "from kernels").fetchall()
    agg = {}
    lo, hi = None, None
    for name, s, e, gx, gy, gz, wx, wy, wz in rows:
        short = name.split("(")[0].replace("zg::", "").replace("void ", "")
        if any(k in short for k in skip):
            continue
        threads = gx * gy * gz  # rocprofv3 reports the grid in work-items
        waves = (threads + 63) // 64
        a = agg.setdefault(short, [0, 0.0, 0.0, waves])
        a[0] += 1
        a[1] += (e - s) / 1e6
        a[2] += (e - s) / 1e6 * waves
        lo = s if lo is None else min(lo, s)
        hi = e if hi is None else max(hi, e)
    tot = sum(a[2] for a in agg.values()) or 1.0
    lines = ["span of the traced dispatches: %.3f ms; total wave-time %.1f wave-ms (%.0f resident waves on average)"
             % ((hi - lo) / 1e6, tot, tot / ((hi - lo) / 1e6)),
             "%-28s %6s %10s %12s %7s %7s" % ("kernel", "calls", "avg ms", "wave-ms", "share", "waves")]
    for k, (n, d, wt, waves) in sorted(agg.items(), key=lambda kv: -kv[1][2]):
        lines.append("%-28s %6d %10.3f %12.1f %6.1f%% %7d" % (k, n, d / n, wt, 100 * wt / tot, waves))
    out = "\n".join(lines)
    print(out)
    if len(pos) > 1:
        open(pos[1], "w").write(out + "\n")


if __name__ == "__main__":
    main()
