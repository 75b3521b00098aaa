"""ctypes binding of the C ABI (include/zg.h) -- the same calls a Rust `verification/gpu`
module makes over `extern "C"`. Loads the in-tree zebra_amd/libzg.so and
fails loudly if it is missing: there is no CPU fallback in the product path.
"""
import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libzg.so")
# A/B experiments (tooling): ZG_LIB_VARIANT=name loads zebra_amd/libzg_<name>.so, a build of the same
# sources with other compile-time switches (tools/build_variant.py); never set in production
if os.environ.get("ZG_LIB_VARIANT"):
    LIB_PATH = os.path.join(HERE, "libzg_%s.so" % os.environ["ZG_LIB_VARIANT"])

KIND_SPEND, KIND_OUTPUT, KIND_SPROUT = 0, 1, 2
GEN_SPEND_AUTH, GEN_BINDING = 0, 1   # include/zg.h ZG_GEN_*
TREE_SPROUT, TREE_SAPLING = 0, 1     # include/zg.h ZG_TREE_*
SPROUT_HEIGHT, SAPLING_HEIGHT = 29, 32   # storage/src/tree_state.rs H29 / H32
E_TREE_FULL = -7
E_DEBUG = -8     # ZG_DEBUG_EACH=1: batch statuses differ from the per-proof re-check
KIND_NINPUTS = {KIND_SPEND: 7, KIND_OUTPUT: 5, KIND_SPROUT: 9}
STATUS_OK, STATUS_DECODE_INVALID, STATUS_MALFORMED_VK, STATUS_VERIFY_FAILED, STATUS_INPUT_NONCANONICAL = 0, 1, 2, 3, 4
STATUS_NAMES = {0: "OK", 1: "DECODE_INVALID", 2: "MALFORMED_VK", 3: "VERIFY_FAILED", 4: "INPUT_NONCANONICAL"}
PROOF_BYTES, INPUT_STRIDE, GT_BYTES, R_BYTES = 192, 288, 576, 16
PREP_KIND_SPEND, PREP_KIND_OUTPUT, PREP_KIND_JOINSPLIT, PREP_KIND_JOINSPLIT_BN = 0, 1, 2, 3   # include/zg.h
PREP_FIELD_BYTES = 304

_lib = None


class ZgError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__("zg error %d: %s" % (code, msg))
        self.code = code


class _Config(ctypes.Structure):
    _fields_ = [("device", ctypes.c_int), ("max_batch", ctypes.c_uint32), ("seeded", ctypes.c_int),
                ("seed", ctypes.c_uint64)]


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError("zebra_amd/libzg.so is not built (run __graft_entry__.build()); "
                              "the GPU path has no fallback")
        L = ctypes.CDLL(LIB_PATH)
        vp, u8p, sz, i = ctypes.c_void_p, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_int
        L.zg_create.restype = vp
        L.zg_create.argtypes = [ctypes.POINTER(_Config)]
        L.zg_set_priority.argtypes = [vp, i]
        L.zg_destroy.argtypes = [vp]
        L.zg_last_error.restype = ctypes.c_char_p
        L.zg_last_error.argtypes = [vp]
        L.zg_version.restype = ctypes.c_char_p
        L.zg_vk_load_builtin.argtypes = [vp, i]
        L.zg_vk_load_json.argtypes = [vp, i, u8p, sz]
        L.zg_vk_load_uncompressed.argtypes = [vp, i, u8p, u8p, u8p, u8p, u8p, u8p, sz, u8p]
        L.zg_vk_alpha_beta.argtypes = [vp, i, u8p]
        L.zg_verify_one_gt.argtypes = [vp, i, u8p, u8p, sz, u8p, u8p]
        L.zg_verify_each.argtypes = [vp, sz, u8p, u8p, u8p, u8p, u8p, u8p]
        L.zg_verify_batch.argtypes = [vp, sz, u8p, u8p, u8p, u8p, u8p, u8p, u8p]
        L.zg_batch_begin.argtypes = [vp, sz, u8p, u8p, u8p, u8p, u8p]
        L.zg_batch_begin_device.argtypes = [vp, sz, vp, vp, vp, vp, vp]
        L.zg_batch_partial.argtypes = [vp, u8p]
        L.zg_batch_ready.argtypes = [vp]
        L.zg_gt_check.argtypes = [vp, sz, u8p, ctypes.POINTER(i)]
        L.zg_gt_check_many.argtypes = [vp, sz, ctypes.POINTER(sz), u8p, ctypes.POINTER(i)]
        L.zg_batch_finish.argtypes = [vp, i, u8p]
        L.zg_synth_rerandomize.argtypes = [vp, sz, u8p, u8p, sz, ctypes.POINTER(ctypes.c_uint32), ctypes.c_uint64, u8p]
        L.zg_last_timings.argtypes = [vp, ctypes.POINTER(ctypes.c_float)]
        L.zg_last_phase_ms.argtypes = [vp, ctypes.POINTER(ctypes.c_float), sz]
        L.zg_stats.argtypes = [vp, ctypes.POINTER(ctypes.c_uint64), sz]
        L.zg_bench_mad_rate.argtypes = [vp, ctypes.POINTER(ctypes.c_double)]
        L.zg_bench_mad_rate_clock.argtypes = [vp, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double)]
        L.zg_chacha20_blocks.argtypes = [vp, u8p, u8p, ctypes.c_uint32, ctypes.c_size_t, u8p]
        L.zg_redjubjub_verify.argtypes = [vp, sz, u8p, u8p, u8p, u8p, u8p]
        L.zg_sapling_bvk.argtypes = [vp, sz, ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_uint32), u8p,
                                     ctypes.POINTER(ctypes.c_int64), u8p, u8p]
        L.zg_jubjub_decode.argtypes = [vp, sz, u8p, u8p, u8p]
        L.zg_prep_batch.argtypes = [vp, sz, u8p, u8p, u8p, u8p]
        L.zg_merkle_combine.argtypes = [vp, i, sz, u8p, u8p, u8p, u8p]
        L.zg_pghr13_vk_load_builtin.argtypes = [vp]
        L.zg_pghr13_vk_load_json.argtypes = [vp, u8p, sz]
        L.zg_pghr13_verify.argtypes = [vp, sz, u8p, u8p, u8p, u8p, ctypes.POINTER(ctypes.c_float)]
        L.zg_bn254_pairing.argtypes = [vp, sz, u8p, u8p, u8p]
        L.zg_tree_empty_roots.argtypes = [vp, i, sz, u8p]
        L.zg_tree_state_max_bytes.restype = sz
        L.zg_tree_state_max_bytes.argtypes = [i]
        u64p = ctypes.POINTER(ctypes.c_uint64)
        L.zg_tree_roots.argtypes = [vp, i, i, u8p, sz, sz, u8p, sz, u64p, u8p, u8p, ctypes.POINTER(sz)]
        L.zg_tree_roots_device.argtypes = [vp, i, i, u8p, sz, sz, vp, sz, u64p, u8p, u8p, ctypes.POINTER(sz),
                                           ctypes.POINTER(ctypes.c_float)]
        L.zg_prep_spend.argtypes = [u8p, u8p, u8p, u8p, u8p]
        L.zg_prep_output.argtypes = [u8p, u8p, u8p, u8p]
        L.zg_prep_joinsplit.argtypes = [u8p, u8p, u8p, u8p, u8p, ctypes.c_uint64, ctypes.c_uint64, u8p, u8p]
        L.zg_prep_joinsplit_bn.argtypes = [u8p, u8p, u8p, u8p, u8p, ctypes.c_uint64, ctypes.c_uint64, u8p, u8p]
        L.zg_hsig.argtypes = [u8p, u8p, u8p, u8p, u8p]
        L.zg_debug_field_mul.argtypes = [i, i, sz, u8p, u8p, u8p]
        _lib = L
    return _lib


# ---- host-side public-input preparation (include/zg.h zg_prep_*; CPU, no GPU needed)
PREP_ERRORS = {1: "ValueCommitment(Invalid)", 2: "ValueCommitment(SmallOrder)", 3: "Anchor",
               4: "RandomizedKey(Invalid)", 5: "RandomizedKey(SmallOrder)", 6: "NoteCommitment",
               7: "EphemeralKey(Invalid)", 8: "EphemeralKey(SmallOrder)"}


class PrepError(ValueError):
    """a description's public input failed the reference's checks (SpendError/OutputError class)"""

    def __init__(self, code):
        super().__init__(PREP_ERRORS.get(code, str(code)))
        self.code = code
        self.name = PREP_ERRORS.get(code, str(code))


def _prep(rc, out, n):
    if rc < 0:
        raise ZgError(rc, "bad argument")
    if rc:
        raise PrepError(rc)
    return [out.raw[32 * j:32 * j + 32] for j in range(n)]


def prep_fields(kind, *args):
    """one description's ZG_PREP_FIELD_BYTES row for zg_prep_batch: SPEND (cv, anchor, nullifier, rk),
    OUTPUT (cv, cmu, epk), JOINSPLIT[_BN] (anchor, random_seed, nullifiers, macs, commitments, vpub_old,
    vpub_new, pubkey) -- the arguments of prep_spend / prep_output / prep_joinsplit[_bn]"""
    if kind in (PREP_KIND_SPEND, PREP_KIND_OUTPUT):
        parts = [bytes(a) for a in args]
        if len(parts) != (4 if kind == PREP_KIND_SPEND else 3) or any(len(x) != 32 for x in parts):
            raise ZgError(-1, "bad Sapling description fields")
        row = b"".join(parts)
    else:
        anchor, seed, nfs, macs, cms, vo, vn, pk = args
        if any(len(bytes(x)) != 32 for x in [anchor, seed, pk, *nfs, *macs, *cms]) or not (
                len(nfs) == len(macs) == len(cms) == 2):
            raise ZgError(-1, "bad JoinSplit description fields")
        row = (bytes(anchor) + bytes(seed) + b"".join(map(bytes, nfs)) + b"".join(map(bytes, macs)) +
               b"".join(map(bytes, cms)) + bytes(pk) + int(vo).to_bytes(8, "little") + int(vn).to_bytes(8, "little"))
    return row.ljust(PREP_FIELD_BYTES, b"\0")


def prep_spend(cv, anchor, nullifier, rk):
    """accept_spend (verification/src/sapling.rs:101-155) -> 7 x 32-byte LE Fr"""
    out = ctypes.create_string_buffer(7 * 32)
    return _prep(lib().zg_prep_spend(bytes(cv), bytes(anchor), bytes(nullifier), bytes(rk), out), out, 7)


def prep_output(cv, cmu, epk):
    """accept_output (verification/src/sapling.rs:171-200) -> 5 x 32-byte LE Fr"""
    out = ctypes.create_string_buffer(5 * 32)
    return _prep(lib().zg_prep_output(bytes(cv), bytes(cmu), bytes(epk), out), out, 5)


def prep_joinsplit(anchor, random_seed, nullifiers, macs, commitments, vpub_old, vpub_new, pubkey):
    """sprout::verify input (verification/src/sprout.rs:34-58,86-153) -> 9 x 32-byte LE Fr"""
    out = ctypes.create_string_buffer(9 * 32)
    return _prep(lib().zg_prep_joinsplit(bytes(anchor), bytes(random_seed), b"".join(map(bytes, nullifiers)),
                                         b"".join(map(bytes, macs)), b"".join(map(bytes, commitments)),
                                         vpub_old, vpub_new, bytes(pubkey), out), out, 9)


def prep_joinsplit_bn(anchor, random_seed, nullifiers, macs, commitments, vpub_old, vpub_new, pubkey):
    """the PHGR branch's input (sprout.rs:34-67, Input::into_bn_frs: 253-bit chunks) -> 9 x
    32-byte LE BN254 Fr"""
    out = ctypes.create_string_buffer(9 * 32)
    return _prep(lib().zg_prep_joinsplit_bn(bytes(anchor), bytes(random_seed), b"".join(map(bytes, nullifiers)),
                                            b"".join(map(bytes, macs)), b"".join(map(bytes, commitments)),
                                            vpub_old, vpub_new, bytes(pubkey), out), out, 9)


def hsig(random_seed, nf0, nf1, pubkey):
    out = ctypes.create_string_buffer(32)
    rc = lib().zg_hsig(bytes(random_seed), bytes(nf0), bytes(nf1), bytes(pubkey), out)
    if rc:
        raise ZgError(rc, "bad argument")
    return out.raw


FIELD_BYTES = {0: 48, 1: 48, 2: 96, 3: 32, 4: 32}   # zg_debug_field_mul operand sizes


def debug_field_mul(field, a, b, device=0):
    """zg_debug_field_mul: the device's Montgomery product for each pair (lists of LE bytes)"""
    w = FIELD_BYTES[field]
    n = len(a)
    assert len(b) == n and all(len(x) == w for x in a) and all(len(x) == w for x in b)
    out = ctypes.create_string_buffer(max(1, w * n))
    rc = lib().zg_debug_field_mul(device, field, n, b"".join(a), b"".join(b), out)
    if rc:
        raise ZgError(rc, "zg_debug_field_mul")
    return [out.raw[w * i:w * i + w] for i in range(n)]


def pack_inputs(rows):
    """list (per proof) of lists of ints / 32-byte LE values -> n x 288 bytes"""
    out = bytearray(INPUT_STRIDE * len(rows))
    for i, row in enumerate(rows):
        for j, x in enumerate(row):
            b = x if isinstance(x, (bytes, bytearray)) else int(x).to_bytes(32, "little")
            out[INPUT_STRIDE * i + 32 * j:INPUT_STRIDE * i + 32 * j + 32] = b
    return bytes(out)


class Context:
    """One zg_ctx: a HIP stream, device buffers and the prepared VKs of one GPU."""

    def __init__(self, device=0, max_batch=65536, seed=None, load_builtin=True):
        L = lib()
        self.max_batch = max_batch
        cfg = _Config(device, max_batch, 1 if seed is not None else 0, seed or 0)
        self._p = L.zg_create(ctypes.byref(cfg))
        if not self._p:
            raise ZgError(-2, "zg_create failed: %s" % (L.zg_last_error(None) or b"no GPU / HIP error").decode())
        if load_builtin:
            for k in (KIND_SPEND, KIND_OUTPUT, KIND_SPROUT):
                self.vk_load_builtin(k)

    def close(self):
        if self._p:
            lib().zg_destroy(self._p)
            self._p = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _chk(self, rc):
        if rc != 0:
            raise ZgError(rc, lib().zg_last_error(self._p).decode())

    def vk_load_builtin(self, kind):
        self._chk(lib().zg_vk_load_builtin(self._p, kind))

    def vk_load_json(self, kind, text):
        b = text.encode() if isinstance(text, str) else text
        self._chk(lib().zg_vk_load_json(self._p, kind, b, len(b)))

    def vk_load_uncompressed(self, kind, alpha_g1, beta_g1, beta_g2, gamma_g2, delta_g1, delta_g2, ic):
        self._chk(lib().zg_vk_load_uncompressed(self._p, kind, alpha_g1, beta_g1, beta_g2, gamma_g2, delta_g1,
                                                delta_g2, len(ic), b"".join(ic) if ic else None))

    def alpha_beta(self, kind):
        out = ctypes.create_string_buffer(GT_BYTES)
        self._chk(lib().zg_vk_alpha_beta(self._p, kind, out))
        return out.raw

    def verify_one_gt(self, kind, proof, inputs):
        """bellman verify_proof for one proof -> (status, GT bytes | None)."""
        inp = pack_inputs([inputs])[:32 * len(inputs)] if inputs else b""
        st = ctypes.create_string_buffer(1)
        gt = ctypes.create_string_buffer(GT_BYTES)
        self._chk(lib().zg_verify_one_gt(self._p, kind, bytes(proof), inp or None, len(inputs), st, gt))
        s = st.raw[0]
        return s, (gt.raw if s in (STATUS_OK, STATUS_VERIFY_FAILED) else None)

    def verify_each(self, proofs, kinds, inputs, n_inputs=None, want_gt=True):
        """per-proof bellman-exact verification -> (statuses, list of GT bytes | None)"""
        n = len(kinds)
        st = ctypes.create_string_buffer(max(n, 1))
        gts = ctypes.create_string_buffer(max(GT_BYTES * n, 1)) if want_gt else None
        self._chk(lib().zg_verify_each(self._p, n, bytes(proofs), bytes(kinds), bytes(inputs),
                                       bytes(n_inputs) if n_inputs is not None else None, st, gts))
        sts = list(st.raw[:n])
        if not want_gt:
            return sts, None
        return sts, [gts.raw[GT_BYTES * i:GT_BYTES * (i + 1)] if sts[i] in (0, 3) else None for i in range(n)]

    def verify_batch(self, proofs, kinds, inputs, n_inputs=None, r=None, want_gt=False):
        """-> (list of statuses, accumulated GT bytes | None)"""
        n = len(kinds)
        st = ctypes.create_string_buffer(max(n, 1))
        gt = ctypes.create_string_buffer(GT_BYTES) if want_gt else None
        self._chk(lib().zg_verify_batch(self._p, n, bytes(proofs), bytes(kinds), bytes(inputs),
                                        bytes(n_inputs) if n_inputs is not None else None,
                                        bytes(r) if r is not None else None, st, gt))
        return list(st.raw[:n]), (gt.raw if want_gt else None)

    def batch_begin(self, proofs, kinds, inputs, n_inputs=None, r=None):
        self._chk(lib().zg_batch_begin(self._p, len(kinds), bytes(proofs), bytes(kinds), bytes(inputs),
                                       bytes(n_inputs) if n_inputs is not None else None,
                                       bytes(r) if r is not None else None))

    def batch_begin_device(self, n, d_proofs, d_kinds, d_inputs, d_n_inputs=None, d_r=None):
        """device pointers (ints, e.g. torch tensor data_ptr()) of HBM-resident inputs"""
        self._chk(lib().zg_batch_begin_device(self._p, n, d_proofs, d_kinds, d_inputs, d_n_inputs, d_r))

    def batch_partial(self):
        out = ctypes.create_string_buffer(GT_BYTES)
        self._chk(lib().zg_batch_partial(self._p, out))
        return out.raw

    def batch_ready(self):
        """True once the batch's device work is done (never blocks; zg_batch_ready)"""
        r = lib().zg_batch_ready(self._p)
        if r < 0:
            self._chk(r)
        return r == 1

    def gt_check(self, partials):
        ok = ctypes.c_int(0)
        self._chk(lib().zg_gt_check(self._p, len(partials), b"".join(partials), ctypes.byref(ok)))
        return bool(ok.value)

    GT_SETS_MAX = 16

    def gt_check_many(self, sets):
        """verdicts of several batches in one launch (zg_gt_check_many): sets = [[partial, ...], ...]
        (1..16 sets), one final exponentiation each, side by side -> [bool, ...]"""
        n = len(sets)
        if not 0 < n <= self.GT_SETS_MAX or any(len(p) == 0 for p in sets):
            raise ValueError("gt_check_many: 1..%d non-empty sets" % self.GT_SETS_MAX)
        counts = (ctypes.c_size_t * n)(*[len(p) for p in sets])
        ok = (ctypes.c_int * n)()
        self._chk(lib().zg_gt_check_many(self._p, n, counts, b"".join(b"".join(p) for p in sets), ok))
        return [bool(v) for v in ok]

    def set_priority(self, high):
        """recreate this context's streams at the highest (True) or default priority"""
        self._chk(lib().zg_set_priority(self._p, 1 if high else 0))

    def batch_finish(self, batch_ok, n):
        st = ctypes.create_string_buffer(max(n, 1))
        self._chk(lib().zg_batch_finish(self._p, 1 if batch_ok else 0, st))
        return list(st.raw[:n])

    PHASES = ("decode", "k_batch_lines", "k_batch_fchain", "k_tree_f", "root_partial", "side_stream_vk",
              "device_pipeline", "k4_msm", "k4_bucket_phase")

    def last_timings(self):
        """[decode, lines, fchain, tree, root_partial, side_stream, device_pipeline, K4, K4 bucket
        phase] in ms (include/zg.h zg_last_phase_ms)"""
        a = (ctypes.c_float * len(self.PHASES))()
        self._chk(lib().zg_last_phase_ms(self._p, a, len(self.PHASES)))
        return list(a)

    STAT_NAMES = ("batches", "fused_launches", "fused_wait_failures", "b_subgroup_recomputes", "bisections",
                  "bisect_nodes", "k4_entries", "quad_fchain_launches", "pghr13_calls", "pghr13_batch_failures",
                  "glv_csum_batches", "line_product_batches", "affine_line_batches")

    def stats(self):
        """cumulative counters (include/zg.h zg_stats) as a dict"""
        a = (ctypes.c_uint64 * len(self.STAT_NAMES))()
        self._chk(lib().zg_stats(self._p, a, len(self.STAT_NAMES)))
        return dict(zip(self.STAT_NAMES, list(a)))

    def synth_rerandomize(self, src_proofs, src_kinds, src_index, seed):
        n = len(src_index)
        idx = (ctypes.c_uint32 * max(n, 1))(*src_index)
        out = ctypes.create_string_buffer(max(192 * n, 1))
        self._chk(lib().zg_synth_rerandomize(self._p, len(src_kinds), bytes(src_proofs), bytes(src_kinds), n, idx,
                                             seed, out))
        return out.raw[:192 * n]

    # ---- Sapling signatures / Jubjub points on the GPU (include/zg.h zg_redjubjub_verify, ...)
    def redjubjub_verify(self, vks, sigs, msgs, gens):
        """per item: redjubjub PublicKey::read(vk) + verify(msg, sig, generator) -> list of bool"""
        n = len(vks)
        assert len(sigs) == len(msgs) == len(gens) == n
        ok = ctypes.create_string_buffer(max(n, 1))
        self._chk(lib().zg_redjubjub_verify(self._p, n, b"".join(map(bytes, vks)), b"".join(map(bytes, sigs)),
                                            b"".join(map(bytes, msgs)), bytes(gens), ok))
        return [b == 1 for b in ok.raw[:n]]

    def sapling_bvk(self, txs):
        """txs: list of (spend cvs, output cvs, value_balance) -> list of (status, bvk bytes)"""
        n = len(txs)
        ns = (ctypes.c_uint32 * max(n, 1))(*[len(t[0]) for t in txs])
        no = (ctypes.c_uint32 * max(n, 1))(*[len(t[1]) for t in txs])
        vb = (ctypes.c_int64 * max(n, 1))(*[t[2] for t in txs])
        cvs = b"".join(b"".join(map(bytes, t[0])) + b"".join(map(bytes, t[1])) for t in txs)
        bvk = ctypes.create_string_buffer(max(32 * n, 1))
        st = ctypes.create_string_buffer(max(n, 1))
        self._chk(lib().zg_sapling_bvk(self._p, n, ns, no, cvs or None, vb, bvk, st))
        return [(st.raw[i], bvk.raw[32 * i:32 * i + 32]) for i in range(n)]

    def prep_batch(self, kinds, fields):
        """zg_prep_batch: a window's public-input preparation in one call. kinds: bytes (PREP_KIND_*),
        fields: n x PREP_FIELD_BYTES (prep_fields) -> (inputs n x 288 bytes, codes bytes: ZG_PREP_*)"""
        n = len(kinds)
        if len(fields) != PREP_FIELD_BYTES * n:
            raise ZgError(-1, "fields must be n x %d bytes" % PREP_FIELD_BYTES)
        inp = ctypes.create_string_buffer(max(INPUT_STRIDE * n, 1))
        codes = ctypes.create_string_buffer(max(n, 1))
        self._chk(lib().zg_prep_batch(self._p, n, bytes(kinds), bytes(fields), inp, codes))
        return inp.raw[:INPUT_STRIDE * n], codes.raw[:n]

    def jubjub_decode(self, points):
        """edwards::Point::read + small-order check -> list of (status 0/1/2, x, y ints)"""
        n = len(points)
        st = ctypes.create_string_buffer(max(n, 1))
        xy = ctypes.create_string_buffer(max(64 * n, 1))
        self._chk(lib().zg_jubjub_decode(self._p, n, b"".join(map(bytes, points)), st, xy))
        return [(st.raw[i], int.from_bytes(xy.raw[64 * i:64 * i + 32], "little"),
                 int.from_bytes(xy.raw[64 * i + 32:64 * i + 64], "little")) for i in range(n)]

    # ---- PGHR13 Sprout proofs on BN254 (include/zg.h zg_pghr13_* / zg_bn254_pairing)
    def pghr13_vk_load_json(self, text):
        """this context's PGHR13 key (other contexts keep theirs; a failed load keeps the old one)"""
        b = text.encode() if isinstance(text, str) else bytes(text)
        self._chk(lib().zg_pghr13_vk_load_json(self._p, b, len(b)))

    def pghr13_vk_load_builtin(self):
        self._chk(lib().zg_pghr13_vk_load_builtin(self._p))

    def pghr13_verify(self, proofs, inputs, n_inputs=None, with_time=False):
        """proofs: 296-byte PHGR proofs; inputs: per proof a list of <= 9 32-byte LE BN254 Fr
        (Input::into_bn_frs) -> statuses (STATUS_*). Packed form (the ABI's own buffers): proofs a
        bytes of n * 296, inputs a bytes of n * 288 (9 slots of 32 per proof) and n_inputs given."""
        if isinstance(proofs, (bytes, bytearray)):
            n = len(proofs) // 296
            assert len(proofs) == 296 * n and len(inputs) == 288 * n and n_inputs is not None and len(n_inputs) == n
            pblob, iblob, cnt = proofs, inputs, bytes(n_inputs)
        else:
            n = len(proofs)
            rows = []
            for r in inputs:
                r = [bytes(x) for x in r]
                assert len(r) <= 9
                rows.append(b"".join(r) + bytes(32 * (9 - len(r))))
            cnt = bytes(len(r) for r in inputs) if n_inputs is None else bytes(n_inputs)
            pblob, iblob = b"".join(map(bytes, proofs)), b"".join(rows)
        st = ctypes.create_string_buffer(max(n, 1))
        ms = ctypes.c_float(0)
        self._chk(lib().zg_pghr13_verify(self._p, n, pblob, iblob, cnt, st, ctypes.byref(ms)))
        out = list(st.raw[:n])
        return (out, ms.value) if with_time else out

    def bn254_pairing(self, g1s, g2s):
        """device pairing (tests): g1 (x, y) ints, g2 ((x0, x1), (y0, y1)) -> 12 ints per GT"""
        n = len(g1s)
        a = b"".join(x.to_bytes(32, "little") + y.to_bytes(32, "little") for x, y in g1s)
        b = b"".join(q[0][0].to_bytes(32, "little") + q[0][1].to_bytes(32, "little") +
                     q[1][0].to_bytes(32, "little") + q[1][1].to_bytes(32, "little") for q in g2s)
        out = ctypes.create_string_buffer(max(384 * n, 1))
        self._chk(lib().zg_bn254_pairing(self._p, n, a, b, out))
        return [[int.from_bytes(out.raw[384 * i + 32 * k:384 * i + 32 * k + 32], "little") for k in range(12)]
                for i in range(n)]

    # ---- note-commitment trees (include/zg.h zg_merkle_combine / zg_tree_*)
    def merkle_combine(self, kind, lefts, rights, depths=None):
        """TreeHash::combine on the GPU: [combine(l, r, depth)] as 32-byte strings"""
        n = len(lefts)
        assert len(rights) == n and (depths is None or len(depths) == n)
        out = ctypes.create_string_buffer(max(32 * n, 1))
        d = None if depths is None else bytes(depths)
        self._chk(lib().zg_merkle_combine(self._p, kind, n, b"".join(map(bytes, lefts)),
                                          b"".join(map(bytes, rights)), d, out))
        return [out.raw[32 * j:32 * j + 32] for j in range(n)]

    def tree_empty_roots(self, kind, levels=64):
        """H::empty()[0..levels)"""
        out = ctypes.create_string_buffer(32 * levels)
        self._chk(lib().zg_tree_empty_roots(self._p, kind, levels, out))
        return [out.raw[32 * j:32 * j + 32] for j in range(levels)]

    def tree_roots(self, kind, height, state, leaves, marks, want_state=True, device_leaves=None,
                   with_time=False):
        """(roots after each marks[k] appended leaves, serialized final state or None).
        state: the reference's serialized TreeState (b"" = new tree). device_leaves: a device
        pointer holding the leaves (len(leaves) is then the count, an int). Raises ZgError
        with code E_TREE_FULL past the capacity (the partial roots are on the exception)."""
        state = bytes(state or b"")
        nm = len(marks)
        mk = (ctypes.c_uint64 * max(nm, 1))(*marks)
        roots = ctypes.create_string_buffer(max(32 * nm, 1))
        cap = lib().zg_tree_state_max_bytes(height)
        so = ctypes.create_string_buffer(cap) if want_state else None
        slen = ctypes.c_size_t(cap)
        ms = ctypes.c_float(0)
        if device_leaves is None:
            n = len(leaves)
            rc = lib().zg_tree_roots(self._p, kind, height, state, len(state), n, b"".join(map(bytes, leaves)),
                                     nm, mk, roots, so, ctypes.byref(slen))
        else:
            n = int(leaves)
            rc = lib().zg_tree_roots_device(self._p, kind, height, state, len(state), n,
                                            ctypes.c_void_p(device_leaves), nm, mk, roots, so,
                                            ctypes.byref(slen), ctypes.byref(ms))
        rl = [roots.raw[32 * j:32 * j + 32] for j in range(nm)]
        if rc:
            e = ZgError(rc, lib().zg_last_error(self._p).decode(errors="replace"))
            e.roots = rl
            raise e
        st = so.raw[:slen.value] if want_state else None
        return (rl, st, ms.value) if with_time else (rl, st)

    def chacha20_blocks(self, key, nonce, counter, nblocks):
        """the device ChaCha20 keystream (the batch-scalar CSPRNG), nblocks x 64 bytes"""
        assert len(key) == 32 and len(nonce) == 12
        out = ctypes.create_string_buffer(64 * max(nblocks, 1))
        self._chk(lib().zg_chacha20_blocks(self._p, bytes(key), bytes(nonce), counter, nblocks, out))
        return out.raw[:64 * nblocks]

    def bench_mad_rate(self, with_clock=False):
        """v_mad_u64_u32 MACs/s of the probe; with_clock: (rate, shader clock in Hz)"""
        v, hz = ctypes.c_double(0), ctypes.c_double(0)
        self._chk(lib().zg_bench_mad_rate_clock(self._p, ctypes.byref(v), ctypes.byref(hz)))
        return (v.value, hz.value) if with_clock else v.value
