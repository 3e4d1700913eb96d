"""Builds the HIP library in-tree (``lib/libpt.so``) for gfx950.

    python -m compute_path_tracer_amd.build
"""
from __future__ import annotations

import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "compute_path_tracer_amd")
CSRC = os.path.join(PKG, "csrc")
LIB = os.path.join(PKG, "lib", "libpt.so")
SOURCES = ["pt_kernel.hip", "pt_runtime.hip", "pt_scene.cpp"]
HEADERS = ["pt_math.h", "pt_device.h", os.path.join("..", "..", "include", "pt_abi.h")]

# -ffp-contract=off + correctly rounded f32 divide/sqrt: the semantics
# contract of DESIGN.md 3 (no FMA contraction; IEEE-rounded / and sqrt).
FLAGS = ["-O3", "--offload-arch=gfx950", "-std=c++17", "-fPIC", "-shared", "-ffp-contract=off",
         "-fhip-fp32-correctly-rounded-divide-sqrt", "-fno-fast-math", "-Wall", "-Wno-unused-function"]


def _stale() -> bool:
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    deps = [os.path.join(CSRC, s) for s in SOURCES + HEADERS] + [os.path.abspath(__file__)]
    return any(os.path.getmtime(d) > t for d in deps)


def build(force: bool = False, verbose: bool = True) -> str:
    if not force and not _stale():
        return LIB
    os.makedirs(os.path.dirname(LIB), exist_ok=True)
    tmp = LIB + ".tmp"
    cmd = ["hipcc", *FLAGS, "-I" + os.path.join(ROOT, "include"), "-o", tmp,
           *[os.path.join(CSRC, s) for s in SOURCES], "-lrccl"]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(tmp, LIB)
    return LIB


def build_oracle(verbose: bool = True) -> str:
    """Test infrastructure: the C restatement used as parity checker."""
    d = os.path.join(ROOT, "oracle")
    subprocess.run(["make", "-s", "-C", d], check=True)
    return os.path.join(d, "libpt_oracle.so")


if __name__ == "__main__":
    build(force="--force" in sys.argv)
    build_oracle()
