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
import time

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


def _jobs():
    """parallel compiles: the host's CPUs, at most 16 (the GPU box's share), at most one per group"""
    n = os.cpu_count() or 4
    try:
        n = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        pass
    return max(1, min(16, n, int(os.environ.get("MAX_JOBS", "16") or 16)))


def build_lib(force=False, verbose=True, extra_flags=(), out=None):
    """The split build (tools/gen_kdecls.py): lb_kgroup.hip once per kernel group (-DLB_KGROUP=g)
    and lb_engine.hip (host code + launches, -DLB_KGROUP=99), compiled in parallel, linked into
    one shared library."""
    out = out or LIB
    if not force and not extra_flags and not _stale(out, _deps()):
        return out
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import gen_kdecls
    cur = open(gen_kdecls.OUT).read() if os.path.exists(gen_kdecls.OUT) else ""
    if cur != gen_kdecls.render():
        with open(gen_kdecls.OUT, "w") as f:
            f.write(gen_kdecls.render())
    odir = os.path.join(ROOT, "build", "obj" + ("" if out == LIB else "_" + os.path.basename(out)))
    os.makedirs(odir, exist_ok=True)
    base = [HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-Wno-unused-result",
            "-Wno-unused-value", "-I" + INC, "-I" + CSRC, *extra_flags]
    units = [(os.path.join(CSRC, "lb_engine.hip"), "99", os.path.join(odir, "engine.o"))]
    units += [(os.path.join(CSRC, "lb_kgroup.hip"), str(g), os.path.join(odir, f"kgroup{g}.o"))
              for g in range(gen_kdecls.N_GROUPS)]
    # the slowest units first
    order = [u for u in units if u[1] in ("3", "6", "8", "9", "7")] + [u for u in units if u[1] not in ("3", "6", "8", "9", "7")]
    running, failed = [], []
    t0 = time.time()
    # per-unit staleness: the kernel groups do not include lb_engine.hip (host code + launches)
    kdeps = [d for d in _deps() if os.path.basename(d) != "lb_engine.hip"]
    pend = [u for u in order if force or extra_flags or _stale(u[2], _deps() if u[1] == "99" else kdeps)]
    while pend or running:
        while pend and len(running) < _jobs():
            src, g, obj = pend.pop(0)
            cmd = base + ["-DLB_KGROUP=" + g, "-c", src, "-o", obj]
            if verbose:
                print("[build]", " ".join(cmd[-5:]), flush=True)
            running.append((subprocess.Popen(cmd), g, time.time()))
        time.sleep(0.2)
        for r in list(running):
            rc = r[0].poll()
            if rc is not None:
                running.remove(r)
                if verbose:
                    print(f"[build] group {r[1]} done in {time.time() - r[2]:.0f} s (rc {rc})", flush=True)
                if rc != 0:
                    failed.append(r[1])
    if failed:
        raise subprocess.CalledProcessError(1, f"hipcc (groups {failed})")
    cmd = [HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", *[u[2] for u in units], "-o", out + ".tmp"]
    subprocess.run(cmd, check=True)
    os.replace(out + ".tmp", out)
    if verbose:
        print(f"[build] {out} in {time.time() - t0:.0f} s", flush=True)
    return out


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
    cmd = ["gcc", "-O2", "-shared", "-fPIC", "-pthread", "-I/usr/include/node", "-I" + INC, src, "-o", NAPI + ".tmp",
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
