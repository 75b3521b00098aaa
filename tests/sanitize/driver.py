"""Runs host-code checks against the AddressSanitizer + UndefinedBehaviorSanitizer builds made by
tests/test_sanitizers.py (never imported by the product; a child process with the sanitizer
runtime preloaded):

  * tests/native/zg_san.hip (the input preparation of zg_prep.h and the 29-bit-digit field
    products of zg_fq29_gen.h, host-compiled): every test function of tests/test_input_prep.py
    and tests/test_host_arith.py::test_field_products_host_edges, called with the instrumented
    library;
  * the oracle's C++ restatement of bellman (oracle/cpu/bellman_cpu.cpp): the golden accept /
    reject fixtures, single-threaded and on 4 threads.

argv: <harness .so> <oracle .so>. Exit 0 when every check passes; the sanitizers abort the
process on the first report (halt_on_error)."""
import ctypes
import inspect
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


class _PrepShim:
    """the zg_prep_* entry points of zebra_amd.zg, served by the instrumented harness"""

    def __init__(self, L):
        c, sz = ctypes.c_char_p, ctypes.c_uint64
        self.zg_prep_spend = L.zgt_prep_spend
        self.zg_prep_spend.argtypes = [c] * 5
        self.zg_prep_output = L.zgt_prep_output
        self.zg_prep_output.argtypes = [c] * 4
        self.zg_hsig = L.zgt_hsig
        self.zg_hsig.argtypes = [c] * 5
        self.zg_prep_joinsplit = L.zgt_prep_joinsplit
        self.zg_prep_joinsplit.argtypes = [c] * 5 + [sz, sz, c, c]


def _run_module(mod, arg):
    n = 0
    for name, fn in sorted(vars(mod).items()):
        if name.startswith("test_") and callable(fn) and list(inspect.signature(fn).parameters) == ["Z"]:
            fn(arg)
            n += 1
    return n


def main():
    harness, oracle_lib = sys.argv[1], sys.argv[2]
    L = ctypes.CDLL(harness)
    from tests import test_host_arith, test_input_prep
    for f in range(5):
        test_host_arith.test_field_products_host_edges(L, f)
    n = 1
    from zebra_amd import zg
    zg._lib = _PrepShim(L)
    n += _run_module(test_input_prep, zg)
    # the oracle restatement on the golden fixtures
    from tests import cpulib
    from tests.conftest import load_golden
    C = ctypes.CDLL(oracle_lib)
    C.zgcpu_vk_load.argtypes = [ctypes.c_int, ctypes.c_char_p, ctypes.c_int, ctypes.c_char_p, ctypes.c_char_p]
    C.zgcpu_verify.argtypes = [ctypes.c_size_t] + [ctypes.c_char_p] * 6 + [ctypes.c_int]
    for k in cpulib.VK_FILES:
        f, ic = cpulib.vk_fields(k)
        assert C.zgcpu_vk_load(k, f, len(ic), b"".join(ic), ctypes.create_string_buffer(576)) == 0
    items = load_golden("batch64.json")["items"]
    proofs = b"".join(bytes.fromhex(e["proof"]) for e in items)
    kinds = bytes(e["kind"] for e in items)
    rows = bytearray(288 * len(items))
    for i, e in enumerate(items):
        for j, x in enumerate(e["inputs"]):
            rows[288 * i + 32 * j:288 * i + 32 * j + 32] = bytes.fromhex(x)
    want = [e["status"] for e in items]
    for threads in (1, 4):
        sts, _ = cpulib.verify(C, proofs, kinds, bytes(rows), threads=threads, want_gt=True)
        assert sts == want, (threads, sts, want)
    n += 1
    print("sanitized host checks passed: %d test functions + oracle fixtures" % n)


if __name__ == "__main__":
    main()
