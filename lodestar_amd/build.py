"""In-tree build of the native pieces (run on the CPU container; the .so files travel to
the GPU box with the tree).  hipcc cross-compiles gfx950 without a GPU.

  * lodestar_amd/liblodestar_bls.so   the product: HIP kernels + C ABI (include/lodestar_bls.h)
  * build/lb_harness.so               test infrastructure: the same arithmetic headers
                                      compiled for x86, checked against oracle/ on CPU
  * build/lb_cpu_pool                 CPU baseline pool (oracle/cpu_pool.cpp)
"""
from __future__ import annotations

import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "lodestar_amd", "csrc")
INC = os.path.join(ROOT, "include")
LIB = os.path.join(ROOT, "lodestar_amd", "liblodestar_bls.so")
HARNESS = os.path.join(ROOT, "build", "lb_harness.so")
CPU_POOL = os.path.join(ROOT, "build", "lb_cpu_pool.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


def _sources(*names):
    return [os.path.join(CSRC, n) for n in names]


def _stale(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _deps():
    hdrs = [os.path.join(CSRC, f) for f in os.listdir(CSRC)]
    return hdrs + [os.path.join(INC, "lodestar_bls.h")]


def build_lib(force=False, verbose=True):
    if not force and not _stale(LIB, _deps()):
        return LIB
    cmd = [HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
           "-Wno-unused-result", "-Wno-unused-value", "-I" + INC, "-I" + CSRC,
           *_sources("lb_engine.hip"), "-o", LIB + ".tmp"]
    if verbose:
        print("[build]", " ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(LIB + ".tmp", LIB)
    return LIB


def build_harness(force=False, verbose=True):
    src = os.path.join(ROOT, "tests", "harness", "lb_harness.cpp")
    os.makedirs(os.path.dirname(HARNESS), exist_ok=True)
    if not force and not _stale(HARNESS, _deps() + [src]):
        return HARNESS
    cmd = ["g++", "-O2", "-shared", "-fPIC", "-I" + INC, "-I" + CSRC, src, "-o", HARNESS + ".tmp"]
    if verbose:
        print("[build]", " ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(HARNESS + ".tmp", HARNESS)
    return HARNESS


def build_cpu_pool(force=False, verbose=True):
    src = os.path.join(ROOT, "oracle", "cpu_pool.cpp")
    if not os.path.exists(src):
        return None
    os.makedirs(os.path.dirname(CPU_POOL), exist_ok=True)
    if not force and not _stale(CPU_POOL, _deps() + [src]):
        return CPU_POOL
    cmd = ["g++", "-O3", "-shared", "-fPIC", "-pthread", "-I" + INC, "-I" + CSRC, src,
           "-o", CPU_POOL + ".tmp"]
    if verbose:
        print("[build]", " ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(CPU_POOL + ".tmp", CPU_POOL)
    return CPU_POOL


UBENCH = ["fpmul_asm"]  # tools/ubench programs the GPU tests run (correctness of the asm Fp multiply)


def build_ubench(force=False, verbose=True):
    out = []
    for name in UBENCH:
        src = os.path.join(ROOT, "tools", "ubench", name + ".hip")
        dst = os.path.join(ROOT, "tools", "ubench", name)
        if force or _stale(dst, _deps() + [src]):
            cmd = [HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-Wno-unused-result", "-Wno-unused-value",
                   "-I" + INC, "-I" + CSRC, src, "-o", dst]
            if verbose:
                print("[build]", " ".join(cmd), flush=True)
            subprocess.run(cmd, check=True)
        out.append(dst)
    return out


NAPI = os.path.join(ROOT, "lodestar_amd", "napi", "lodestar_bls.node")


def build_napi(force=False, verbose=True):
    """N-API addon (plain C against the system node_api.h) linked to liblodestar_bls.so."""
    src = os.path.join(ROOT, "lodestar_amd", "napi", "lb_napi.c")
    hdr = "/usr/include/node/node_api.h"
    if not os.path.exists(hdr):
        return None
    if not force and not _stale(NAPI, [src, LIB, os.path.join(INC, "lodestar_bls.h")]):
        return NAPI
    cmd = ["gcc", "-O2", "-shared", "-fPIC", "-I/usr/include/node", "-I" + INC, src, "-o", NAPI + ".tmp",
           "-L" + os.path.dirname(LIB), "-llodestar_bls", "-Wl,-rpath,$ORIGIN/.."]
    if verbose:
        print("[build]", " ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(NAPI + ".tmp", NAPI)
    return NAPI


def build_all(force=False):
    build_lib(force)
    build_napi(force)
    build_harness(force)
    build_cpu_pool(force)
    build_ubench(force)


if __name__ == "__main__":
    build_all(force="--force" in sys.argv)
