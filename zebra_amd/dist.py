"""Multi-GPU protocol (one process per GPU, torch.distributed; backend "nccl" is RCCL on
ROCm): contiguous shards, one 576-byte Miller partial per rank, all-gather, the final
exponentiation of their product on every rank (same inputs, same verdict). SURVEY.md 8(e);
DESIGN.md section 6."""

import os

GT_BYTES = 576


def shard_range(n, world, rank):
    """contiguous shard [lo, hi) of n items for `rank` (sizes differ by at most one)."""
    base, extra = divmod(n, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


_xbufs = {}


def _exchange_buffers(world, device, k):
    """per (device, world, k): the staging buffers of combine_partials, allocated once (pinned
    host memory and a high-priority stream on a GPU, so the k x 576-B copies are DMA enqueues
    that do not wait behind in-flight batches)"""
    import torch
    key = (str(device), world, k)
    if key not in _xbufs:
        gpu = torch.device(device).type == "cuda"
        # (ZG_XSTREAM_PRIO=0: a default-priority stream; tooling for the priority A/B of DESIGN §4d)
        prio = -1 if os.environ.get("ZG_XSTREAM_PRIO", "1") != "0" else 0
        stream = torch.cuda.Stream(device=device, priority=prio) if gpu else None
        _xbufs[key] = (torch.empty(k * GT_BYTES, dtype=torch.uint8, pin_memory=gpu),
                       torch.empty(k * GT_BYTES, dtype=torch.uint8, device=device),
                       torch.empty(world * k * GT_BYTES, dtype=torch.uint8, device=device),
                       torch.empty(world * k * GT_BYTES, dtype=torch.uint8, pin_memory=gpu), stream)
    return _xbufs[key]


def combine_partials(partial, check, world, rank, device, group=None):
    """All-gather every rank's 576-byte partial (one RCCL all-gather into one tensor, one copy
    back) and run `check(list_of_partials) -> bool` -- ONE final exponentiation of their
    product -- on every rank: all ranks hold the same partials, so they reach the same verdict
    without a second collective (ncclAllGather when every rank needs the result).
    Keeping the exchange to one collective matters with batches in flight: every extra device
    op queues behind the other batches' kernels. Calls must not overlap (the staging buffers are
    reused; run_pipelined* issue them from one thread, in batch order).

    `partial` is one 576-B partial, or a list of k of them when a rank verifies k shards of the
    batch (every rank must pass the same k): the gather then moves world x k partials in the
    same single collective, ordered rank-major (rank 0's k shards first)."""
    return check(gather_partials(partial, world, rank, device, group))


def gather_partials(partial, world, rank, device, group=None):
    """The exchange step of combine_partials alone: every rank's partial(s), rank-major, as a list
    of 576-B bytes (same on every rank). Calls must not overlap and must run in the same order on
    every rank (run_pipelined_deferred's ordered gather stage). device "cpu" with a gloo `group`
    exchanges the host-resident partials without a device round trip (bench.py --exchange gloo)."""
    import contextlib
    import numpy as np
    import torch
    import torch.distributed as dist
    parts = [partial] if isinstance(partial, (bytes, bytearray)) else list(partial)
    k = len(parts)
    assert k >= 1 and all(len(p) == GT_BYTES for p in parts)
    host, mine, flat, back, stream = _exchange_buffers(world, device, k)
    with torch.cuda.stream(stream) if stream is not None else contextlib.nullcontext():
        host.numpy()[:] = np.frombuffer(b"".join(parts), dtype=np.uint8)
        mine.copy_(host, non_blocking=True)
        dist.all_gather_into_tensor(flat, mine, group=group)
        back.copy_(flat)
    if stream is not None:
        stream.synchronize()
    allb = back.numpy().tobytes()
    return [allb[GT_BYTES * j:GT_BYTES * (j + 1)] for j in range(world * k)]


def run_pipelined(ctxs, k, launch, complete):
    """k batches with up to len(ctxs) in flight (one context each, round-robin): a context is
    relaunched only after its previous batch completed, and batches complete in launch order
    on every rank, so the per-batch collectives of `complete` (combine_partials) line up across
    ranks. Returns the k results of complete(ctx) in batch order."""
    out, q = [], []
    for s in range(k):
        if len(q) == len(ctxs):
            out.append(complete(q.pop(0)))
        c = ctxs[s % len(ctxs)]
        launch(c)
        q.append(c)
    while q:
        out.append(complete(q.pop(0)))
    return out


def run_pipelined_deferred(ctxs, k, launch, harvest, verdict, redo, ready=None, gather=None, checks=1,
                           verdict_many=None, max_sets=16):
    """run_pipelined with the verdict taken off the context's critical path.

    harvest(ctx) -> (partial, statuses) waits for a batch's Miller partial and reads its
    per-proof statuses as if the batch verdict were true (decode rejects and input-count
    errors are final either way); the context is then free and is relaunched at once.
    ready(ctx) -> bool (optional; Context.batch_ready, never blocks): batches in flight finish out
    of launch order (they share the device), so the loop harvests whichever batch is done first
    and relaunches its context, instead of idling finished contexts behind the oldest batch
    (without `ready`: strictly the oldest). verdict(partial) -> bool (the all-gather + ONE final
    exponentiation, on a checker context of its own) runs on a single worker thread in BATCH order
    whatever the harvest order, so the per-batch collectives line up across ranks exactly as in
    run_pipelined. A batch whose verdict is false is re-verified by redo(batch_index) -> statuses
    (bisection on a fresh pass: per-proof results do not depend on the batch scalars) after the
    pipeline has drained. Returns the k (verdict, statuses) pairs in batch order; all verdicts are
    in before it returns.

    gather / checks (round 6): with gather(partial) -> partials given, the worker thread runs only
    that exchange (the collective) in batch order and hands verdict(partials) -- the final
    exponentiation, a lone wave on the device for ~2 ms -- to a pool of `checks` threads, so the
    verdicts of consecutive batches overlap instead of bounding the batch rate (8k shards, 6 in
    flight: one verdict thread was busy 2.16 of every 2.61 ms). verdict must then be thread-safe
    (e.g. one checker context per thread).

    verdict_many (round 6, with gather): instead of the pool, ONE checker thread takes every
    gathered set waiting for it (up to max_sets) and checks them together, verdict_many([partials,
    ...]) -> [bool, ...] (Context.gt_check_many: one final exponentiation per set, side by side in one
    launch) -- the overlap of the pool's concurrent verdicts on a single checker context."""
    import queue
    import threading
    import time
    from concurrent.futures import Future, ThreadPoolExecutor
    free, inflight = list(ctxs), []   # inflight: (batch index, ctx) in launch order
    done, res = {}, {}                # harvested, verdict not yet submitted / submitted
    nxt = launched = 0
    pool = coalesce = None
    if gather is not None and verdict_many is not None:
        coalesce = queue.SimpleQueue()   # (gathered partials, Future); None ends the checker

        def checker():
            stop = False
            while not stop:
                item = coalesce.get()
                if item is None:
                    return
                items = [item]
                while len(items) < max_sets:
                    try:
                        more = coalesce.get_nowait()
                    except queue.Empty:
                        break
                    if more is None:
                        stop = True
                        break
                    items.append(more)
                try:
                    oks = verdict_many([p for p, _ in items])
                    for (_, f), ok in zip(items, oks):
                        f.set_result(ok)
                except BaseException as e:   # every waiting batch sees the failure
                    for _, f in items:
                        f.set_exception(e)
        th = threading.Thread(target=checker, daemon=True)
        th.start()
    elif gather is not None:
        pool = ThreadPoolExecutor(max_workers=max(1, checks))

    def staged(part):                 # ordered worker: the exchange, then the check on the pool
        if coalesce is not None:
            f = Future()
            coalesce.put((gather(part), f))
            return f
        return pool.submit(verdict, gather(part))

    def result(f):
        r = f.result()
        return r.result() if gather is not None else r
    try:
        with ThreadPoolExecutor(max_workers=1) as ex:
            while launched < k or inflight:
                while free and launched < k:
                    c = free.pop(0)
                    launch(c)
                    inflight.append((launched, c))
                    launched += 1
                i = 0
                if ready is not None:
                    i = next((j for j, (_, c) in enumerate(inflight) if ready(c)), None)
                    if i is None:          # nothing finished yet: poll again shortly
                        time.sleep(2e-5)
                        continue
                s, c = inflight.pop(i)
                done[s] = harvest(c)
                free.append(c)
                while nxt in done:         # verdicts (collectives) strictly in batch order
                    part, sts = done.pop(nxt)
                    res[nxt] = (sts, ex.submit(staged if gather is not None else verdict, part))
                    nxt += 1
            oks = [result(res[s][1]) for s in range(k)]
    finally:
        if pool is not None:
            pool.shutdown()
        if coalesce is not None:
            coalesce.put(None)
            th.join()
    return [(ok, res[s][0] if ok else redo(s)) for s, ok in enumerate(oks)]
