"""Build libuthot.so (gfx950 HIP kernels + C ABI) in-tree.

    python -m uptune_amd.build            # incremental
    python -m uptune_amd.build --force

The shared library lands next to this file (uptune_amd/libuthot.so) so it
travels with the repository snapshot to the GPU box.  hipcc cross-compiles
for gfx950 without a GPU present.

Also builds libuthot_hostcheck.so (g++) -- the host build of ut_core.h used
only by tests/test_core_host.py.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OBJ = os.path.join(HERE, "_build")
LIB = os.path.join(HERE, "libuthot.so")
HOSTLIB = os.path.join(HERE, "libuthot_hostcheck.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("UT_OFFLOAD_ARCH", "gfx950")

SOURCES = ["api.hip", "propose.hip", "hash.hip", "dedup.hip", "gp.hip", "gp_gemm.hip", "gp_i8.hip", "gp_kq.hip", "topk.hip", "forest.hip", "comm.hip"]
HEADERS = ["ut_core.h", "ut_internal.h", "ut_param.h", "ut_perm.h", "ryu_tables.h", "libm_log_data.h", os.path.join("..", "..", "include", "uthot.h")]

# RCCL for the multi-GPU exchange (comm.hip); the soname (librccl.so.1) is the
# one torch loads too, so a process that imported torch first shares its copy
LINK_LIBS = ["-L/opt/rocm/lib", "-lrccl", "-Wl,-rpath,/opt/rocm/lib"]

HIP_FLAGS = [
    "-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}",
    # bit-exact parameter arithmetic: no FMA contraction anywhere
    "-ffp-contract=off",
    "-Wno-unused-result",
]


def _mtime(p: str) -> float:
    try:
        return os.path.getmtime(p)
    except OSError:
        return 0.0


def _ensure_tables() -> None:
    tbl = os.path.join(CSRC, "ryu_tables.h")
    gen = os.path.join(CSRC, "gen_ryu_tables.py")
    if _mtime(tbl) < _mtime(gen):
        subprocess.check_call([sys.executable, gen, tbl])


def _compile(src: str, force: bool) -> str:
    obj = os.path.join(OBJ, os.path.splitext(src)[0] + ".o")
    srcp = os.path.join(CSRC, src)
    newest_dep = max([_mtime(srcp)] + [_mtime(os.path.join(CSRC, h)) for h in HEADERS])
    if not force and _mtime(obj) > newest_dep:
        return obj
    cmd = [HIPCC, *HIP_FLAGS, "-c", srcp, "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src}:\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return obj


def build(force: bool = False, verbose: bool = False) -> str:
    os.makedirs(OBJ, exist_ok=True)
    _ensure_tables()
    jobs = min(len(SOURCES), int(os.environ.get("MAX_JOBS", "8")))
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        objs = list(ex.map(lambda s: _compile(s, force), SOURCES))
    if force or _mtime(LIB) < max(_mtime(o) for o in objs):
        tmp = LIB + ".tmp"
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", *objs, "-o", tmp, *LINK_LIBS]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
        os.replace(tmp, LIB)
    hsrc = os.path.join(CSRC, "hostcheck.cpp")
    if force or _mtime(HOSTLIB) < max(_mtime(hsrc), *[_mtime(os.path.join(CSRC, h)) for h in HEADERS]):
        cmd = ["g++", "-O2", "-std=c++17", "-shared", "-fPIC", "-ffp-contract=off", hsrc, "-o", HOSTLIB]
        subprocess.check_call(cmd)
    if verbose:
        print(LIB)
    return LIB


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    a = ap.parse_args()
    build(force=a.force, verbose=True)
