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
