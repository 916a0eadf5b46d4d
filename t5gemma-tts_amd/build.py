"""Build libt5gtts.so (HIP C++ for gfx950) in-tree with hipcc.

``python t5gemma-tts_amd/build.py`` or ``t5gemma_tts_amd.build.build()``.
Objects go to ``t5gemma-tts_amd/build/``, the library to ``t5gemma-tts_amd/lib/``
(git-ignored, shipped to the GPU box by gpurun's snapshot).
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
OBJ = os.path.join(PKG, "build")
LIB = os.path.join(PKG, "lib", "libt5gtts.so")
SOURCES = ["gemm.hip", "gemv.hip", "norm.hip", "attn.hip", "sampler.hip", "engine.hip", "fused.hip", "exact.hip", "xmm.hip", "xattn.hip", "xlayer.hip", "eager.hip", "noise.hip", "xc2.hip", "xc2enc.hip", "whisper.hip", "host_sampler.cpp"]
HEADERS = ["common.h", "t5g_kernels.h", "xc2_common.h", "exact_math.h", "exact_dev.h", "ref_ksplit.h", "sort_emu.h"]
ARCH = os.environ.get("T5G_ARCH", "gfx950")
# -ffp-contract=off: HIP's default (fast-honor-pragmas) fuses a*b+c into one fma even
# through __fmul_rn / __fsub_rn, which changes roundings the reference's CPU kernels keep
# separate (e.g. aten's fast exp: x*log2e is rounded before floor / subtract). Every fma
# the kernels want is written explicitly (fmaf, MFMA).
FLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-Wno-unused-result", "-ffp-contract=off",
         "-I", os.path.join(REPO, "include")]


def _hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", "hipcc"):
        if c and (os.path.isabs(c) and os.path.exists(c) or not os.path.isabs(c)):
            return c
    raise RuntimeError("hipcc not found")


def _newest_dep() -> float:
    deps = [os.path.join(CSRC, h) for h in HEADERS] + [os.path.join(REPO, "include", h) for h in ("t5gtts.h", "xc2.h", "whisper.h")]
    return max(os.path.getmtime(p) for p in deps if os.path.exists(p))


def _compile(src: str, force: bool, dbg: bool = False) -> str:
    s = os.path.join(CSRC, src)
    o = os.path.join(OBJ, ("dbg_" if dbg else "") + os.path.splitext(src)[0] + ".o")
    if not force and os.path.exists(o) and os.path.getmtime(o) >= max(os.path.getmtime(s), _newest_dep()):
        return o
    cmd = [_hipcc()] + FLAGS + (["-DT5G_DBG_TS=1"] if dbg else []) + ["-c", s, "-o", o]
    if src.endswith(".cpp"):
        # host-only C++ (the parity host sampler, the host build of csrc/sort_emu.h): g++
        cmd = ["g++", "-O3", "-std=c++17", "-fPIC", "-Wno-unused-result", "-I",
               os.path.join(REPO, "include"), "-I", CSRC, "-c", s, "-o", o]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src}:\n{r.stderr[-4000:]}")
    return o


def build(force: bool = False, verbose: bool = True, dbg: bool = False) -> str:
    """dbg=True builds the diagnostic variant lib/libt5gtts_dbg.so (per-block timestamps,
    common.h T5G_TS; used only by tools/micro_timeline.cpp, never by the product)."""
    os.makedirs(OBJ, exist_ok=True)
    os.makedirs(os.path.dirname(LIB), exist_ok=True)
    lib = LIB.replace(".so", "_dbg.so") if dbg else LIB
    srcs = [s for s in SOURCES if os.path.exists(os.path.join(CSRC, s))]
    with cf.ThreadPoolExecutor(max_workers=min(8, len(srcs))) as ex:
        objs = list(ex.map(lambda s: _compile(s, force, dbg), srcs))
    if force or not os.path.exists(lib) or os.path.getmtime(lib) < max(os.path.getmtime(o) for o in objs):
        cmd = [_hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", lib] + objs
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stderr[-4000:]}")
        if verbose:
            print(f"[t5gtts] built {lib}")
    return lib


ORACLE_SRC = os.path.join(REPO, "oracle", "sort_order.cpp")
ORACLE_LIB = os.path.join(REPO, "oracle", "lib", "liboracle_sort.so")
ORACLE_EXPF_SRC = os.path.join(REPO, "oracle", "glibc_expf.c")
ORACLE_EXPF_LIB = os.path.join(REPO, "oracle", "lib", "liboracle_expf.so")


def _build_one(src: str, lib: str, cmd: list, force: bool) -> str:
    os.makedirs(os.path.dirname(lib), exist_ok=True)
    if force or not os.path.exists(lib) or os.path.getmtime(lib) < os.path.getmtime(src):
        r = subprocess.run(cmd + ["-o", lib, src], capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"oracle build failed:\n{r.stderr[-4000:]}")
    return lib


def build_oracle(force: bool = False) -> str:
    """Compile the oracle's C / C++ restatements (test infrastructure: the std::sort tie
    order, glibc's expf) into oracle/lib/. Returns the sort library's path."""
    # -ffp-contract=off: the expf restatement's fused multiply-adds are explicit fma() calls
    _build_one(ORACLE_EXPF_SRC, ORACLE_EXPF_LIB, ["gcc", "-O2", "-ffp-contract=off", "-shared", "-fPIC"], force)
    return _build_one(ORACLE_SRC, ORACLE_LIB, ["g++", "-O2", "-std=c++17", "-shared", "-fPIC"], force)


if __name__ == "__main__":
    build(force="--force" in sys.argv, dbg="--dbg" in sys.argv)
