"""GPU tier: the two launch shapes of the R-chain + f-chain (zg_kernels.h k_lines_fchain vs
k_batch_lines then k_batch_fchain), forced through ZG_LINES_FCHAIN (read by zg_create), give
the same statuses, GT bytes and 576-byte Miller partials. The fused shape is the default for
shards whose two grids fit on the device at once (the 8-GPU run's 8,192-proof ranks); forcing
it on a 16,384-proof batch puts more blocks in flight than there are CUs."""
import os

import pytest

from tests.conftest import load_golden
from tests.test_gpu_parity import corrupted_4096, fx_batch

pytestmark = pytest.mark.gpu


def make_ctx(mode, max_batch=16384):
    from zebra_amd import Context
    old = os.environ.get("ZG_LINES_FCHAIN")
    os.environ["ZG_LINES_FCHAIN"] = mode
    try:
        return Context(device=0, max_batch=max_batch, seed=7)
    finally:
        if old is None:
            del os.environ["ZG_LINES_FCHAIN"]
        else:
            os.environ["ZG_LINES_FCHAIN"] = old


@pytest.fixture(scope="module")
def ctxs():
    cs = {m: make_ctx(m) for m in ("0", "1")}
    yield cs
    for c in cs.values():
        c.close()


@pytest.mark.parametrize("mode", ["0", "1"])
def test_batch64_statuses_and_gt(ctxs, mode):
    b = load_golden("batch64.json")
    items = b["items"]
    proofs, kinds, inputs, nin = fx_batch(items)
    r = b"".join(bytes.fromhex(e["r"]) for e in items)
    sts, gt = ctxs[mode].verify_batch(proofs, kinds, inputs, nin, r=r, want_gt=True)
    assert sts == [e["status"] for e in items]
    assert gt.hex() == b["gt_out"]


@pytest.mark.parametrize("mode", ["0", "1"])
def test_corrupted_4096(ctxs, mode):
    """non-subgroup B among them: the fused launch's gated f-chain re-run (bfail) path"""
    proofs, kinds, inputs, want = corrupted_4096(ctxs[mode])
    sts, _ = ctxs[mode].verify_batch(proofs, kinds, inputs)
    assert sts == want


@pytest.mark.parametrize("n", [128, 4096, 16384])
def test_partials_equal(ctxs, n):
    """same seeded r_i, same proofs: the two shapes produce the same Miller partial bytes"""
    from zebra_amd import pack_inputs
    real = load_golden("real_proofs.json")["proofs"]
    src_proofs = b"".join(bytes.fromhex(e["proof"]) for e in real)
    src_kinds = bytes(e["kind"] for e in real)
    idx = [i % len(real) for i in range(n)]
    proofs = ctxs["0"].synth_rerandomize(src_proofs, src_kinds, idx, 5)
    kinds = bytes(src_kinds[j] for j in idx)
    inputs = pack_inputs([[bytes.fromhex(x) for x in real[j]["inputs"]] for j in idx])
    parts = []
    for mode in ("0", "1"):
        c = ctxs[mode]
        c.batch_begin(proofs, kinds, inputs)
        parts.append(c.batch_partial())
        assert c.gt_check([parts[-1]])
        assert c.batch_finish(True, n) == [0] * n
    assert parts[0] == parts[1]


def test_batches_in_flight_match_sequential():
    """three contexts with batches queued together on one GPU (bench.py's batches in flight)
    give the same Miller partials and statuses as one batch at a time"""
    from zebra_amd import Context, pack_inputs
    real = load_golden("real_proofs.json")["proofs"]
    src_proofs = b"".join(bytes.fromhex(e["proof"]) for e in real)
    src_kinds = bytes(e["kind"] for e in real)
    n = 2048
    cs = [Context(device=0, max_batch=n, seed=11) for _ in range(3)]
    try:
        batches = []
        for b in range(3):
            idx = [(i + b) % len(real) for i in range(n)]
            proofs = cs[0].synth_rerandomize(src_proofs, src_kinds, idx, 20 + b)
            kinds = bytes(src_kinds[j] for j in idx)
            inputs = pack_inputs([[bytes.fromhex(x) for x in real[j]["inputs"]] for j in idx])
            batches.append((proofs, kinds, inputs))
        seq = []
        for b in range(3):
            cs[0].batch_begin(*batches[b])
            seq.append(cs[0].batch_partial())
            assert cs[0].batch_finish(True, n) == [0] * n
        for b in range(3):
            cs[b].batch_begin(*batches[b])
        for b in range(3):
            assert cs[b].batch_partial() == seq[b]
            assert cs[b].gt_check([seq[b]])
            assert cs[b].batch_finish(True, n) == [0] * n
    finally:
        for c in cs:
            c.close()


# ---- the two R-chain kernels: the staged program (k_batch_lines) and the straight-line
# lane-per-proof kernel (zg_lines.hip k_batch_lines_lane, the default from 32k padded proofs),
# forced through ZG_LINES_LANE at small sizes; ZG_LINES_FCHAIN=0 keeps the split launches
def make_lines_ctx(lane):
    from zebra_amd import Context
    saved = {k: os.environ.get(k) for k in ("ZG_LINES_LANE", "ZG_LINES_FCHAIN")}
    os.environ["ZG_LINES_LANE"] = lane
    os.environ["ZG_LINES_FCHAIN"] = "0"
    try:
        return Context(device=0, max_batch=4096, seed=7)
    finally:
        for k, v in saved.items():
            if v is None:
                del os.environ[k]
            else:
                os.environ[k] = v


@pytest.fixture(scope="module")
def lctxs():
    cs = {m: make_lines_ctx(m) for m in ("0", "1", "2")}
    yield cs
    for c in cs.values():
        c.close()


@pytest.mark.parametrize("lane", ["1", "2"])
def test_lines_lane_batch64_and_corruptions(lctxs, lane):
    """the straight-line R-chain (both register budgets): batch64's statuses and GT bytes, the
    corrupted 4,096 (non-subgroup B: its G2 check and the gated recompute), and the same 576-byte
    Miller partial as the staged program"""
    b = load_golden("batch64.json")
    items = b["items"]
    proofs, kinds, inputs, nin = fx_batch(items)
    r = b"".join(bytes.fromhex(e["r"]) for e in items)
    sts, gt = lctxs[lane].verify_batch(proofs, kinds, inputs, nin, r=r, want_gt=True)
    assert sts == [e["status"] for e in items]
    assert gt.hex() == b["gt_out"]
    cp, ck, cx, want = corrupted_4096(lctxs[lane])
    assert lctxs[lane].verify_batch(cp, ck, cx)[0] == want
    parts = []
    for m in ("0", lane):
        lctxs[m].batch_begin(cp, ck, cx, r=r * 64)
        parts.append(lctxs[m].batch_partial())
        lctxs[m].batch_finish(True, len(ck))
    assert parts[0] == parts[1]
