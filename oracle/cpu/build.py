#!/usr/bin/env python3
"""Build oracle/_build/libzgcpu.so (the CPU restatement of bellman's per-proof path) and
oracle/_build/libzgmerkle.so (the reference's note-commitment tree path, merkle_cpu.cpp) and
oracle/_build/libpghr13cpu.so (the reference's PGHR13 check on BN254, pghr13_cpu.cpp) with
g++ -O3. Test/bench infrastructure only."""
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(os.path.dirname(HERE), "_build")
SRC = os.path.join(HERE, "bellman_cpu.cpp")
LIB = os.path.join(OUT, "libzgcpu.so")


MERKLE_SRC = os.path.join(HERE, "merkle_cpu.cpp")
MERKLE_LIB = os.path.join(OUT, "libzgmerkle.so")


def _gxx(src, lib):
    os.makedirs(OUT, exist_ok=True)
    if not os.path.exists(lib) or os.path.getmtime(lib) < os.path.getmtime(src):
        subprocess.check_call(["g++", "-O3", "-march=x86-64-v3", "-std=c++17", "-fPIC", "-shared", "-pthread",
                               src, "-o", lib + ".tmp"])
        os.replace(lib + ".tmp", lib)
    return lib


PGHR13_SRC = os.path.join(HERE, "pghr13_cpu.cpp")
PGHR13_LIB = os.path.join(OUT, "libpghr13cpu.so")


def build():
    _gxx(MERKLE_SRC, MERKLE_LIB)
    _gxx(PGHR13_SRC, PGHR13_LIB)
    return _gxx(SRC, LIB)


def build_pghr13():
    return _gxx(PGHR13_SRC, PGHR13_LIB)


def build_merkle():
    return _gxx(MERKLE_SRC, MERKLE_LIB)


if __name__ == "__main__":
    print(build())
