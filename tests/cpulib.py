"""ctypes loader for oracle/_build/libzgcpu.so -- the C++ restatement of bellman's per-proof
path (checker and bench cpu_baseline only)."""
import ctypes
import json
import os
import runpy

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
VK_FILES = {0: "sapling-spend-verifying-key.json", 1: "sapling-output-verifying-key.json",
            2: "sprout-groth16-key.json"}


def vk_fields(kind):
    d = json.load(open(os.path.join(ROOT, "zebra_amd", "res", VK_FILES[kind])))
    h = lambda s: bytes.fromhex(s[2:] if s.startswith("0x") else s)  # noqa: E731
    return (b"".join(h(d[k]) for k in ("alphaG1", "betaG1", "betaG2", "gammaG2", "deltaG1", "deltaG2")),
            [h(x) for x in d["ic"]])


def load():
    lib = runpy.run_path(os.path.join(ROOT, "oracle", "cpu", "build.py"))["build"]()
    L = ctypes.CDLL(lib)
    L.zgcpu_vk_load.argtypes = [ctypes.c_int, ctypes.c_char_p, ctypes.c_int, ctypes.c_char_p, ctypes.c_char_p]
    L.zgcpu_verify.argtypes = [ctypes.c_size_t] + [ctypes.c_char_p] * 6 + [ctypes.c_int]
    for k in VK_FILES:
        f, ic = vk_fields(k)
        ab = ctypes.create_string_buffer(576)
        assert L.zgcpu_vk_load(k, f, len(ic), b"".join(ic), ab) == 0
    return L


def verify(L, proofs, kinds, inputs, n_inputs=None, threads=1, want_gt=False):
    n = len(kinds)
    st = ctypes.create_string_buffer(max(n, 1))
    gts = ctypes.create_string_buffer(576 * n) if want_gt else None
    assert L.zgcpu_verify(n, bytes(proofs), bytes(kinds), bytes(inputs),
                          bytes(n_inputs) if n_inputs is not None else None, st, gts, threads) == 0
    sts = list(st.raw[:n])
    return sts, ([gts.raw[576 * i:576 * i + 576] for i in range(n)] if want_gt else None)


OPS = ("fq_mul_ns", "fq_sqr_ns", "miller_loop_3pair_us", "final_exp_us", "g2_prepare_us", "g1_mul255_us",
       "g2_subgroup_us", "verify_one_us")


def bench_ops(L, kind, proof, inputs, k, reps=20):
    """single-thread timings of the port's building blocks (zgcpu_bench_ops), a dict over OPS"""
    L.zgcpu_bench_ops.argtypes = [ctypes.c_int, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int, ctypes.c_int,
                                  ctypes.POINTER(ctypes.c_double)]
    out = (ctypes.c_double * 8)()
    assert L.zgcpu_bench_ops(kind, bytes(proof), bytes(inputs), k, reps, out) == 0
    return dict(zip(OPS, list(out)))


def load_merkle():
    """oracle/_build/libzgmerkle.so (merkle_cpu.cpp), initialised with the Pedersen generators of
    the Python oracle"""
    from oracle import merkle as M
    from oracle.sapling_sig import aff
    lib = runpy.run_path(os.path.join(ROOT, "oracle", "cpu", "build.py"))["build_merkle"]()
    L = ctypes.CDLL(lib)
    L.mc_init.argtypes = [ctypes.c_char_p]
    L.mc_combine.argtypes = [ctypes.c_int, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int, ctypes.c_char_p]
    L.mc_window.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_size_t,
                            ctypes.c_char_p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_uint64), ctypes.c_char_p]
    gens = b""
    for j in range(3):
        x, y = aff(M.pedersen_generator(j))
        gens += x.to_bytes(32, "little") + y.to_bytes(32, "little")
    assert L.mc_init(gens) == 0
    return L


def merkle_window(L, kind, height, state, leaves, marks):
    """mc_window: the reference's sequential appends + roots (marks sorted)"""
    nm = len(marks)
    mk = (ctypes.c_uint64 * max(nm, 1))(*marks)
    out = ctypes.create_string_buffer(max(32 * nm, 1))
    rc = L.mc_window(kind, height, bytes(state), len(state), len(leaves), b"".join(leaves), nm, mk, out)
    return rc, [out.raw[32 * k:32 * k + 32] for k in range(nm)]


def load_pghr13():
    """oracle/_build/libpghr13cpu.so (pghr13_cpu.cpp, the reference's PGHR13 check restated in
    C++), with the key of res/sprout-verifying-key.json (parsed and point-checked by
    oracle.pghr13.load_vk_json)"""
    from oracle import pghr13 as PG
    lib = runpy.run_path(os.path.join(ROOT, "oracle", "cpu", "build.py"))["build_pghr13"]()
    L = ctypes.CDLL(lib)
    L.pg_vk_load.argtypes = [ctypes.c_char_p, ctypes.c_int]
    L.pg_pairing.argtypes = [ctypes.c_size_t, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p]
    L.pg_verify.argtypes = [ctypes.c_size_t] + [ctypes.c_char_p] * 4 + [ctypes.c_int]
    vk = PG.load_vk_json(open(os.path.join(ROOT, "zebra_amd", "res", "sprout-verifying-key.json")).read())
    le = lambda x: x.to_bytes(32, "little")  # noqa: E731
    g1 = lambda p: le(p[0]) + le(p[1])  # noqa: E731
    g2 = lambda q: le(q[0][0]) + le(q[0][1]) + le(q[1][0]) + le(q[1][1])  # noqa: E731
    blob = b"".join(g2(vk[k]) for k in ("a", "c", "z", "gamma", "gamma_beta_2"))
    blob += g1(vk["b"]) + g1(vk["gamma_beta_1"]) + b"".join(g1(p) for p in vk["ic"])
    assert L.pg_vk_load(blob, len(vk["ic"])) == 0
    return L


def pg_verify(L, proofs, inputs, threads=1):
    """proofs: 296-byte PHGR proofs; inputs: per proof a list of <= 9 32-byte LE BN254 Fr"""
    n = len(proofs)
    rows = b"".join(b"".join(bytes(x) for x in r) + bytes(32 * (9 - len(r))) for r in inputs)
    st = ctypes.create_string_buffer(max(n, 1))
    assert L.pg_verify(n, b"".join(map(bytes, proofs)), rows, bytes(len(r) for r in inputs), st, threads) == 0
    return list(st.raw[:n])


def pg_pairing(L, ps, qs):
    """e(P, Q) per pair (affine integer points) -> GT as 12 integers (oracle.bn254.gt_ints order)"""
    le = lambda x: x.to_bytes(32, "little")  # noqa: E731
    g1 = b"".join(le(p[0]) + le(p[1]) for p in ps)
    g2 = b"".join(le(q[0][0]) + le(q[0][1]) + le(q[1][0]) + le(q[1][1]) for q in qs)
    out = ctypes.create_string_buffer(384 * len(ps))
    L.pg_pairing(len(ps), g1, g2, out)
    return [[int.from_bytes(out.raw[384 * i + 32 * k:384 * i + 32 * k + 32], "little") for k in range(12)]
            for i in range(len(ps))]
