"""Build libsrpde_hip.so (gfx950) in-tree with hipcc.

    python -m superresolution_for_pdes_amd.build [--force]

The .so lands in superresolution_for_pdes_amd/lib/ (git-ignored, but it travels to the
GPU box with the gpurun snapshot).  Objects are compiled in parallel and the build is
skipped when the library is newer than every source.
"""
from __future__ import annotations

import concurrent.futures as cf
import glob
import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
LIBDIR = os.path.join(PKG, "lib")
LIB = os.path.join(LIBDIR, "libsrpde_hip.so")
# SRPDE_BUILD_OUT: build to another path (an A/B baseline for tools/gpu/conv_ab.sh)
if os.environ.get("SRPDE_BUILD_OUT"):
    LIB = os.path.abspath(os.environ["SRPDE_BUILD_OUT"])
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("SRPDE_ARCH", "gfx950")
# no packed-FP32 VALU ops (v_pk_fma/mul/add_f32) anywhere: on the MI355X boxes their results on lanes
# 48-63 come out wrong while MFMA work runs beside them on the chip (another stream or process;
# DESIGN.md 7.4, tools/race_up.py); the host compile ignores the feature (one warning per file)
NO_PK = ["-Xclang", "-target-feature", "-Xclang", "-packed-fp32-ops"]
FLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-Wall", "-Wno-unused-function"] + NO_PK
# SRPDE_EXTRA_FLAGS: extra compile flags (e.g. -DBNAS_U=8) for an A/B variant built with SRPDE_BUILD_OUT
FLAGS += os.environ.get("SRPDE_EXTRA_FLAGS", "").split()


def sources():
    return sorted(glob.glob(os.path.join(CSRC, "*.hip")) + glob.glob(os.path.join(CSRC, "*.cpp")))


def _deps():
    return sources() + glob.glob(os.path.join(CSRC, "*.h")) + [os.path.join(ROOT, "include", "srpde.h")]


def up_to_date() -> bool:
    if not os.path.exists(LIB):
        return False
    t = os.path.getmtime(LIB)
    return all(os.path.getmtime(d) <= t for d in _deps())


def build(force: bool = False, verbose: bool = False) -> str:
    if not force and up_to_date():
        return LIB
    objdir = os.path.join(os.path.dirname(LIB), "obj" if LIB.startswith(LIBDIR) else "obj_" + os.path.basename(LIB))
    os.makedirs(objdir, exist_ok=True)

    def compile_one(src):
        obj = os.path.join(objdir, os.path.basename(src) + ".o")
        cmd = [HIPCC] + FLAGS + ["-c", src, "-o", obj]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed for {src}:\n{r.stderr}")
        if verbose and r.stderr:
            print(r.stderr, file=sys.stderr)
        return obj

    jobs = min(8, int(os.environ.get("MAX_JOBS", "8")))
    with cf.ThreadPoolExecutor(jobs) as ex:
        objs = list(ex.map(compile_one, sources()))
    tmp = LIB + ".tmp"
    cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp] + objs
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{r.stderr}")
    os.replace(tmp, LIB)
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
