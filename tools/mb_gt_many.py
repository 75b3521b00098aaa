"""Idle-device timing of zg_gt_check_many: k batches' verdicts in one launch vs k zg_gt_check calls
(does a launch of k final exponentiations take the time of one?)."""
import time

from zebra_amd import Context
from tests.conftest import load_golden
from tests.test_gpu_parity import fx_batch


def main():
    c = Context(device=0, max_batch=64)
    good = [e for e in load_golden("batch64.json")["items"] if e["status"] == 0]
    parts = []
    for shard in (good[:20], good[20:]):
        c.batch_begin(*fx_batch(shard))
        parts.append(c.batch_partial())
        c.batch_finish(True, len(shard))
    for k in (1, 2, 4, 8, 16):
        sets = [parts] * k
        c.gt_check_many(sets)
        t0 = time.perf_counter()
        for _ in range(5):
            assert c.gt_check_many(sets) == [True] * k
        many = (time.perf_counter() - t0) / 5
        t0 = time.perf_counter()
        for _ in range(5):
            for s in sets:
                assert c.gt_check(s)
        each = (time.perf_counter() - t0) / 5
        print("sets %2d: one gt_check_many %.3f ms, %d gt_check calls %.3f ms" % (k, 1e3 * many, k, 1e3 * each))
    c.close()


if __name__ == "__main__":
    main()
