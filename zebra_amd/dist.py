"""Multi-GPU protocol (one process per GPU, torch.distributed; backend "nccl" is RCCL on
ROCm): contiguous shards, one 576-byte Miller partial per rank, all-gather, ONE final
exponentiation on rank 0, verdict broadcast. SURVEY.md 8(e); DESIGN.md section 6."""

GT_BYTES = 576


def shard_range(n, world, rank):
    """contiguous shard [lo, hi) of n items for `rank` (sizes differ by at most one)."""
    base, extra = divmod(n, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def combine_partials(partial, check, world, rank, device):
    """All-gather every rank's 576-byte partial; rank 0 runs `check(list_of_partials) -> bool`
    (one final exponentiation of their product); the verdict is broadcast to every rank."""
    import torch
    import torch.distributed as dist
    assert len(partial) == GT_BYTES
    mine = torch.frombuffer(bytearray(partial), dtype=torch.uint8).to(device)
    parts = [torch.empty(GT_BYTES, dtype=torch.uint8, device=device) for _ in range(world)]
    dist.all_gather(parts, mine)
    okt = torch.zeros(1, dtype=torch.int32, device=device)
    if rank == 0:
        okt.fill_(1 if check([bytes(p.cpu().numpy().tobytes()) for p in parts]) else 0)
    dist.broadcast(okt, 0)
    return bool(okt.item())


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
