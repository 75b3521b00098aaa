"""config 5 alone (tooling): tools/bench_config5.run on one context, the JSON on stdout"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from zebra_amd import Context
    from tools import bench_config5
    ctx = Context(device=0, max_batch=65536)
    threads = int(os.environ.get("OMP_NUM_THREADS", "16"))
    print(json.dumps(bench_config5.run(ctx, threads if "--cpu" in sys.argv else 0)))
    ctx.close()


if __name__ == "__main__":
    main()
