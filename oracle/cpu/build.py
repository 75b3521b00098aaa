#!/usr/bin/env python3
"""Build oracle/_build/libzgcpu.so (the CPU restatement of bellman's per-proof path) with
g++ -O3. Test/bench infrastructure only."""
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(os.path.dirname(HERE), "_build")
SRC = os.path.join(HERE, "bellman_cpu.cpp")
LIB = os.path.join(OUT, "libzgcpu.so")


def build():
    os.makedirs(OUT, exist_ok=True)
    if not os.path.exists(LIB) or os.path.getmtime(LIB) < os.path.getmtime(SRC):
        subprocess.check_call(["g++", "-O3", "-march=x86-64-v3", "-std=c++17", "-fPIC", "-shared", "-pthread",
                               SRC, "-o", LIB + ".tmp"])
        os.replace(LIB + ".tmp", LIB)
    return LIB


if __name__ == "__main__":
    print(build())
