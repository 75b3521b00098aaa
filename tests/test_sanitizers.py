"""CPU tier: AddressSanitizer + UndefinedBehaviorSanitizer over the host C++.

Builds, with the clang of the ROCm toolchain and sanitizers on the HOST code only:
  * tests/native/zg_san.hip -> the product's host input preparation (zebra_amd/csrc/zg_prep.h:
    Jubjub decode, small-order checks, multipacking, hSig, Sprout packing) and the 29-bit-digit
    field products every kernel uses (zg_fq29_gen.h), compiled for the CPU (--offload-host-only);
  * oracle/cpu/bellman_cpu.cpp -> the C++ restatement of bellman used as checker and baseline;
then runs tests/sanitize/driver.py in a child process with the sanitizer runtime preloaded:
every test function of tests/test_input_prep.py and the field-product edge cases of
tests/test_host_arith.py against the instrumented harness, and the golden batch64 fixtures through the instrumented oracle on 1 and
4 threads. Any sanitizer report aborts the child. The GPU code is not instrumented (GPU
sanitizers are not available on the pool); the device side is covered by the GPU parity tests."""
import os
import subprocess
import sys

import pytest

from tests.conftest import ROOT

LLVM = "/opt/rocm/lib/llvm/bin"
OUT = os.path.join(ROOT, "tests", "native", "_san")
HARNESS_SRC = os.path.join(ROOT, "tests", "native", "zg_san.hip")
ORACLE_SRC = os.path.join(ROOT, "oracle", "cpu", "bellman_cpu.cpp")
CSRC = os.path.join(ROOT, "zebra_amd", "csrc")
SAN = ["-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fsanitize=undefined",
       "-Xarch_host", "-fno-sanitize-recover=all", "-shared-libsan"]


def _stale(lib, deps):
    return not os.path.exists(lib) or any(os.path.getmtime(d) > os.path.getmtime(lib) for d in deps)


def _build():
    os.makedirs(OUT, exist_ok=True)
    harness = os.path.join(OUT, "libzg_san.so")
    deps = [HARNESS_SRC] + [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")]
    if _stale(harness, deps):
        subprocess.check_call(["hipcc", "-x", "hip", "--offload-host-only", "-O1", "-g", "-fno-omit-frame-pointer",
                               "-fPIC", "-shared", "-std=c++17", "-Wno-psabi"] + SAN +
                              [HARNESS_SRC, "-o", harness + ".tmp"])
        os.replace(harness + ".tmp", harness)
    oracle = os.path.join(OUT, "libzgcpu_san.so")
    if _stale(oracle, [ORACLE_SRC]):
        subprocess.check_call([os.path.join(LLVM, "clang++"), "-O1", "-g", "-fno-omit-frame-pointer", "-std=c++17",
                               "-fPIC", "-shared", "-pthread"] + SAN + [ORACLE_SRC, "-o", oracle + ".tmp"])
        os.replace(oracle + ".tmp", oracle)
    return harness, oracle


@pytest.mark.timeout(1800)
def test_host_code_under_asan_ubsan():
    harness, oracle = _build()
    rt = subprocess.run([os.path.join(LLVM, "clang++"), "-print-file-name=libclang_rt.asan-x86_64.so"],
                        capture_output=True, text=True, check=True).stdout.strip()
    assert os.path.exists(rt), rt
    env = dict(os.environ, LD_PRELOAD=rt,
               ASAN_OPTIONS="detect_leaks=0:halt_on_error=1:abort_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "sanitize", "driver.py"), harness, oracle],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=1700)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert "ERROR: AddressSanitizer" not in out and "runtime error:" not in out, out[-4000:]
    assert "sanitized host checks passed" in r.stdout
