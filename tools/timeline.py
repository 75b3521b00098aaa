#!/usr/bin/env python3
"""Kernel timeline of the LAST batch in a rocprofv3 rocpd .db (tooling): every kernel from the last
launch of MARK (default k_chacha20, the first kernel of a Groth16 batch) on, with its start / end
relative to that launch, duration and stream. Usage: timeline.py run_results.db [MARK] [out.txt]"""
import sqlite3
import sys


def main():
    db = sqlite3.connect(sys.argv[1])
    mark = sys.argv[2] if len(sys.argv) > 2 else "k_chacha20"
    cols = [r[1] for r in db.execute("pragma table_info(kernels)").fetchall()]
    sid = next((c for c in ("stream_id", "queue_id", "stream", "queue") if c in cols), None)
    q = "select name, start, end%s from kernels order by start" % (", " + sid if sid else "")
    rows = db.execute(q).fetchall()
    t0 = max(r[1] for r in rows if mark in r[0])
    out = ["columns: %s (stream column: %s)" % (",".join(cols), sid),
           "%9s %9s %9s  %-8s %s" % ("start_us", "end_us", "dur_us", "stream", "kernel")]
    for r in rows:
        if r[1] < t0:
            continue
        name = r[0].split("(")[0].replace("zg::", "")
        out.append("%9.1f %9.1f %9.1f  %-8s %s" % ((r[1] - t0) / 1e3, (r[2] - t0) / 1e3, (r[2] - r[1]) / 1e3,
                                                  r[3] if sid else "-", name[:70]))
    text = "\n".join(out)
    if len(sys.argv) > 3:
        open(sys.argv[3], "w").write(text + "\n")
    print(text)


if __name__ == "__main__":
    main()
