"""ctypes loader for tests/native/libzg_hosttest.so (the product's arithmetic compiled for
the CPU; test harness only). Built on demand with hipcc --offload-host-only."""
import ctypes
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
SRC = os.path.join(HERE, "native", "zg_hosttest.hip")
LIB = os.path.join(HERE, "native", "libzg_hosttest.so")
CSRC = os.path.join(ROOT, "zebra_amd", "csrc")


def _stale():
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    deps = [SRC] + [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")]
    return any(os.path.getmtime(d) > t for d in deps)


def build():
    if _stale():
        subprocess.check_call(["hipcc", "-x", "hip", "--offload-host-only", "-O2", "-fPIC", "-shared",
                               "-std=c++17", "-Wno-psabi", SRC, "-o", LIB])
    return LIB


_lib = None


def lib():
    global _lib
    if _lib is None:
        _lib = ctypes.CDLL(build())
    return _lib


def buf(n):
    return ctypes.create_string_buffer(n)
