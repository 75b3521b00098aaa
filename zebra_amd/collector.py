"""Block-level Groth16 collector -- the caller side of the boundary.

Restates how the reference's chain acceptor reaches the proof checks, so that a whole block
(or import window) is verified with ONE batch call while the reported error stays exactly the
reference's:

  ChainAcceptor::check_transactions   verification/src/accept_chain.rs:76-81
      rayon fold/reduce over transactions: the LOWEST failing tx index wins
  TransactionAcceptor::check          verification/src/accept_transaction.rs:68-84
      ... -> eval (sighash) -> join_split.check -> sapling.check
  JoinSplitVerification::check        accept_transaction.rs:649-657
      ed25519 JoinSplit signature -> JoinSplitProof::check -> JoinSplit nullifiers
  JoinSplitProof::check               accept_transaction.rs:575-596
      per description i: sprout::verify (-> InvalidJoinSplit(i)), then tree_cache.continue_root
  SaplingVerification                 accept_transaction.rs:700-714 (SaplingProof::check)
      accept_sapling (sapling.rs:75-98): per spend (cv, anchor, rk, spend_auth_sig, proof),
      per output (cv, cmu, epk, proof), binding signature -> any failure is InvalidSapling;
      then Sapling nullifiers

The checks that are not proofs or Sapling signatures (JoinSplit ed25519 signature, tree
roots, nullifiers, the transparent checks before the shielded stages) are evaluated by the
caller exactly as today and handed in as outcomes; the collector prepares every public input of
the window in one zg_prep_batch call (the Sapling descriptions' Jubjub decodes on the GPU, the
JoinSplits on host threads; without a context, the per-description zg_prep_* host functions),
verifies all Groth16 proofs of the window in
one zg_verify_batch call and all PGHR13 proofs of pre-Sapling JoinSplits (sprout.rs:61-67,
inputs Input::into_bn_frs via zg_prep_joinsplit_bn) in one zg_pghr13_verify call, and
re-injects the per-proof statuses in reference order: a PHGR description that fails to decode
(InvalidEncoding) or to verify (InvalidPGHRProof) is InvalidJoinSplit(index), at its place among
the transaction's descriptions, before its tree_cache.continue_root (accept_transaction.rs:575-592).
"""
from dataclasses import dataclass, field
from typing import List, Optional

from . import zg

OK = zg.STATUS_OK


@dataclass
class JoinSplit:
    """one JoinSplit description (chain/src/join_split.rs:169-186)"""
    anchor: bytes
    random_seed: bytes
    nullifiers: List[bytes]
    macs: List[bytes]
    commitments: List[bytes]
    vpub_old: int
    vpub_new: int
    zkproof: bytes                    # 192 B Groth16 (v4+) or 296 B PGHR13
    groth: bool = True
    pghr_ok: Optional[bool] = None    # a PGHR13 verdict the caller already holds (None: the GPU
                                      # verifies the description in the window's PGHR13 call)
    tree_error: Optional[str] = None  # caller's tree_cache.continue_root outcome (None = ok)


@dataclass
class Spend:
    cv: bytes
    anchor: bytes
    nullifier: bytes
    rk: bytes
    zkproof: bytes
    sig_ok: bool = True               # caller's spend_auth_sig (RedJubjub) verdict, used when
    spend_auth_sig: Optional[bytes] = None   # ... this is None; else verified on the GPU


@dataclass
class Output:
    cv: bytes
    cmu: bytes
    epk: bytes
    zkproof: bytes


@dataclass
class Tx:
    """the shielded-proof view of one transaction, with the caller's non-Groth16 outcomes"""
    pre_error: Optional[str] = None           # first failing check before the JoinSplit stage
    js_pubkey: Optional[bytes] = None
    js_sig_ok: bool = True
    joinsplits: List[JoinSplit] = field(default_factory=list)
    js_nullifier_error: Optional[str] = None
    spends: List[Spend] = field(default_factory=list)
    outputs: List[Output] = field(default_factory=list)
    binding_ok: bool = True                   # caller's binding_sig verdict, used when binding_sig is None
    sapling_nullifier_error: Optional[str] = None
    # the Sapling signature checks on the GPU: the no-input ZIP-243 sighash the
    # acceptor computes (accept_transaction.rs:374-386), valueBalance and the binding signature
    sighash: Optional[bytes] = None
    value_balance: int = 0
    binding_sig: Optional[bytes] = None


_POOL = None
_PAR_MIN = 32   # prep jobs below this run inline (a pool round trip costs more than they do)
# windows from this many descriptions go through zg_prep_batch (the GPU); below, the host functions:
# a lone 9-description block took 6.6 ms with host prep and 8.6 ms with the batched call (its copies
# and launch), a 401-description block 12.1 -> 9.8 ms, a 9,609-description window 383 -> 35 ms
# (tools/bench_config5.py; profiles/r06q_config5.txt)
_GPU_PREP_MIN = 64


def _prep_pool():
    """host threads for the public-input preparation (Jubjub point decodes, small-order checks,
    multipacking: ~0.35 ms of C per Sapling description); the prep functions are ctypes calls into
    libzg.so, which release the GIL, so a window's descriptions decode in parallel like the
    reference's rayon fan-out over transactions (accept_chain.rs:76-81). Sized like the bench's
    CPU share: OMP_NUM_THREADS when set, else every usable CPU (at most 64)."""
    global _POOL
    if _POOL is None:
        import concurrent.futures
        import os
        try:
            n = len(os.sched_getaffinity(0))
        except AttributeError:
            n = os.cpu_count() or 1
        omp = os.environ.get("OMP_NUM_THREADS", "")
        if omp.isdigit() and int(omp) > 0:
            n = min(n, int(omp))
        _POOL = concurrent.futures.ThreadPoolExecutor(max_workers=max(1, min(64, n)))
    return _POOL


def _run_prep(job):
    fn, args = job
    try:
        return fn(*args)
    except zg.PrepError as e:
        return e


def _jobs(txs):
    """the window's preparation jobs in reference order: (PREP_KIND_*, arguments of the prep function)"""
    jobs = []
    for tx in txs:
        for d in tx.joinsplits:
            if tx.js_pubkey is None or (not d.groth and d.pghr_ok is not None):
                continue
            jobs.append((zg.PREP_KIND_JOINSPLIT if d.groth else zg.PREP_KIND_JOINSPLIT_BN,
                         (d.anchor, d.random_seed, d.nullifiers, d.macs, d.commitments, d.vpub_old, d.vpub_new,
                          tx.js_pubkey)))
        for s in tx.spends:
            jobs.append((zg.PREP_KIND_SPEND, (s.cv, s.anchor, s.nullifier, s.rk)))
        for o in tx.outputs:
            jobs.append((zg.PREP_KIND_OUTPUT, (o.cv, o.cmu, o.epk)))
    return jobs


_PREP_FN = {zg.PREP_KIND_SPEND: zg.prep_spend, zg.PREP_KIND_OUTPUT: zg.prep_output,
            zg.PREP_KIND_JOINSPLIT: zg.prep_joinsplit, zg.PREP_KIND_JOINSPLIT_BN: zg.prep_joinsplit_bn}


_PAD = {zg.PREP_KIND_SPEND: bytes(zg.PREP_FIELD_BYTES - 128), zg.PREP_KIND_OUTPUT: bytes(zg.PREP_FIELD_BYTES - 96)}


def _fields(jobs):
    """the window's zg_prep_batch field rows: the Sapling descriptions' 32-byte fields joined as they are
    (one join for the window), the JoinSplits through zg.prep_fields; a field of the wrong size is
    reported by zg.prep_fields"""
    out = []
    for k, a in jobs:
        if k == zg.PREP_KIND_SPEND or k == zg.PREP_KIND_OUTPUT:
            out.extend(a)
            out.append(_PAD[k])
        else:
            out.append(zg.prep_fields(k, *a))
    f = b"".join(out)
    if len(f) != zg.PREP_FIELD_BYTES * len(jobs):
        f = b"".join(zg.prep_fields(k, *a) for k, a in jobs)   # raises on the malformed description
    return f


def _prepare(jobs, ctx):
    """-> per job: the packed 288-byte input row, or a PrepError. With a context: ONE zg_prep_batch call
    for the window (Sapling descriptions on the GPU, JoinSplits on host threads); without: the
    per-description host functions (in parallel for a large window)."""
    if ctx is not None and len(jobs) >= _GPU_PREP_MIN:
        kinds = bytes(k for k, _ in jobs)
        fields = _fields(jobs)
        rows, codes = ctx.prep_batch(kinds, fields)
        return [zg.PrepError(c) if c else rows[zg.INPUT_STRIDE * i:zg.INPUT_STRIDE * (i + 1)]
                for i, c in enumerate(codes)]
    calls = [(_PREP_FN[k], a) for k, a in jobs]
    if len(calls) >= _PAR_MIN:
        done = list(_prep_pool().map(_run_prep, calls, chunksize=16))
    else:
        done = [_run_prep(c) for c in calls]
    return [d if isinstance(d, zg.PrepError) else zg.pack_inputs([d]) for d in done]


def _queue(txs, ctx=None):
    """prepare inputs; returns (Groth16 items (kind, proof, 288-byte input row, n inputs), PGHR13 items
    (proof, inputs), per-tx plans). A plan entry refers to a queued proof by index ("proof" / "pghr"),
    or carries a prep error or a caller verdict. The window's preparation runs first (_prepare), then
    the items and plans are assembled in reference order."""
    res = iter(_prepare(_jobs(txs), ctx))
    items, pghr, plans = [], [], []
    for tx in txs:
        js_plan, sp_plan, out_plan = [], [], []
        for d in tx.joinsplits:
            if tx.js_pubkey is None or (not d.groth and d.pghr_ok is not None):
                js_plan.append(("caller", bool(d.pghr_ok)))
                continue
            row = next(res)
            if isinstance(row, zg.PrepError):   # (the JoinSplit preps raise no PrepError)
                raise row
            if not d.groth:
                js_plan.append(("pghr", len(pghr)))
                pghr.append((bytes(d.zkproof), [row[32 * j:32 * j + 32] for j in range(9)]))
                continue
            js_plan.append(("proof", len(items)))
            items.append((zg.KIND_SPROUT, bytes(d.zkproof), row, 9))
        for s in tx.spends:
            row = next(res)
            if isinstance(row, zg.PrepError):
                sp_plan.append(("prep", row.name))
                continue
            sp_plan.append(("proof", len(items)))
            items.append((zg.KIND_SPEND, bytes(s.zkproof), row, 7))
        for o in tx.outputs:
            row = next(res)
            if isinstance(row, zg.PrepError):
                out_plan.append(("prep", row.name))
                continue
            out_plan.append(("proof", len(items)))
            items.append((zg.KIND_OUTPUT, bytes(o.zkproof), row, 5))
        plans.append((js_plan, sp_plan, out_plan))
    return items, pghr, plans


def _sig_verdicts(txs, ctx, verify_sigs, sapling_bvk):
    """spend_auth_sig and binding_sig verdicts of the transactions that carry a sighash (the rest
    keep the caller's booleans): the binding verification keys in one zg_sapling_bvk call, every
    signature of the window in ONE zg_redjubjub_verify call (accept_spend sapling.rs:119-137,
    accept_sapling_final :216-244). Returns (per-tx spend sig oks, per-tx binding ok)."""
    if verify_sigs is None:
        verify_sigs = ctx.redjubjub_verify if ctx is not None else None
    if sapling_bvk is None:
        sapling_bvk = ctx.sapling_bvk if ctx is not None else None
    sp_ok = [[s.sig_ok for s in tx.spends] for tx in txs]
    bind_ok = [tx.binding_ok for tx in txs]
    need = [i for i, tx in enumerate(txs) if tx.sighash is not None and (tx.spends or tx.outputs)]
    if not need:
        return sp_ok, bind_ok
    if verify_sigs is None or sapling_bvk is None:
        raise zg.ZgError(-1, "transactions carry a sighash but no signature backend was given "
                             "(pass ctx=, or verify_sigs= and sapling_bvk=)")
    bvks = sapling_bvk([([s.cv for s in txs[i].spends], [o.cv for o in txs[i].outputs], txs[i].value_balance)
                        for i in need])
    items, where = [], []
    for i, (st, bvk) in zip(need, bvks):
        tx = txs[i]
        for j, s in enumerate(tx.spends):
            if s.spend_auth_sig is not None:
                items.append((s.rk, s.spend_auth_sig, bytes(s.rk) + bytes(tx.sighash), zg.GEN_SPEND_AUTH))
                where.append((i, j))
        if tx.binding_sig is not None:
            if st == 0:
                items.append((bvk, tx.binding_sig, bvk + bytes(tx.sighash), zg.GEN_BINDING))
                where.append((i, None))
            else:   # a cv that does not decode fails its own description first; i64::MIN: InvalidBalanceValue
                bind_ok[i] = False
    if items:
        oks = verify_sigs(*[list(x) for x in zip(*items)])
        for (i, j), ok in zip(where, oks):
            if j is None:
                bind_ok[i] = ok
            else:
                sp_ok[i][j] = ok
    return sp_ok, bind_ok


def _tx_error(tx, plan, status, sp_ok=None, bind_ok=None, pghr_status=()):
    """the reference's first error of one transaction, given the proof statuses"""
    js_plan, sp_plan, out_plan = plan
    if sp_ok is None:
        sp_ok = [s.sig_ok for s in tx.spends]
    if bind_ok is None:
        bind_ok = tx.binding_ok
    if tx.pre_error:
        return tx.pre_error
    if tx.joinsplits:
        if not tx.js_sig_ok:
            return "JoinSplitSignature"
        for i, (d, (how, v)) in enumerate(zip(tx.joinsplits, js_plan)):
            ok = v if how == "caller" else (pghr_status[v] if how == "pghr" else status[v]) == OK
            if not ok:
                return ("InvalidJoinSplit", i)
            if d.tree_error:
                return d.tree_error
        if tx.js_nullifier_error:
            return tx.js_nullifier_error
    if tx.spends or tx.outputs:
        for ok, (how, v) in zip(sp_ok, sp_plan):
            if how == "prep" or not ok or status[v] != OK:
                return "InvalidSapling"
        for how, v in out_plan:
            if how == "prep" or status[v] != OK:
                return "InvalidSapling"
        if not bind_ok:
            return "InvalidSapling"
        if tx.sapling_nullifier_error:
            return tx.sapling_nullifier_error
    return None


def _chunked(verify, cap):
    """an import window larger than one batch (the context's max_batch) is verified as
    consecutive batches of at most `cap` proofs; statuses are joined in order (per-proof
    statuses do not depend on how proofs are grouped into batches)"""
    if not cap:
        return verify

    def run(proofs, kinds, inputs, n_inputs):
        n = len(kinds)
        out = []
        for lo in range(0, n, cap):
            hi = min(n, lo + cap)
            out += list(verify(proofs[192 * lo:192 * hi], kinds[lo:hi], inputs[zg.INPUT_STRIDE * lo:zg.INPUT_STRIDE * hi],
                               n_inputs[lo:hi]))
        return out
    return run


def verify_block(txs, verify=None, ctx=None, verify_sigs=None, sapling_bvk=None, verify_pghr=None):
    """Check the shielded proofs of a block (or an import window: a flat list of Tx in chain
    order). Returns None if every transaction passes, else (tx_index, error) with the error the
    reference reports (accept_chain.rs:79-80: the lowest failing index wins).

    verify(proofs, kinds, inputs, n_inputs) -> statuses; default: ctx.verify_batch (ONE GPU
    batch for the whole block, exact per-proof statuses via bisection). A window larger than
    the context's max_batch (or a `verify.max_batch` attribute) is split into consecutive
    batches. Transactions that carry their sighash get their RedJubjub signatures verified on
    the GPU too (verify_sigs / sapling_bvk default to ctx.redjubjub_verify / ctx.sapling_bvk).
    PHGR JoinSplit proofs go through verify_pghr(proofs, inputs) -> statuses, default
    ctx.pghr13_verify (ONE zg_pghr13_verify call for the window)."""
    items, pghr, plans = _queue(txs, ctx)
    if verify is None:
        def verify(proofs, kinds, inputs, n_inputs):
            return ctx.verify_batch(proofs, kinds, inputs, n_inputs)[0]
        cap = getattr(ctx, "max_batch", None)
    else:
        cap = getattr(verify, "max_batch", None)
    verify = _chunked(verify, cap)
    status = []
    if items:
        proofs = b"".join(p for _, p, _, _ in items)
        kinds = bytes(k for k, _, _, _ in items)
        inputs = b"".join(row for _, _, row, _ in items)
        n_inputs = bytes(nin for _, _, _, nin in items)
        status = list(verify(proofs, kinds, inputs, n_inputs))
    pghr_status = []
    if pghr:
        if verify_pghr is None:
            if ctx is None:
                raise zg.ZgError(-1, "PHGR JoinSplits in the window but no PGHR13 backend (pass ctx= or verify_pghr=)")
            verify_pghr = ctx.pghr13_verify
        pghr_status = list(verify_pghr([p for p, _ in pghr], [inp for _, inp in pghr]))
    sp_ok, bind_ok = _sig_verdicts(txs, ctx, verify_sigs, sapling_bvk)
    for idx, (tx, plan) in enumerate(zip(txs, plans)):
        err = _tx_error(tx, plan, status, sp_ok[idx], bind_ok[idx], pghr_status)
        if err is not None:
            return idx, err
    return None
