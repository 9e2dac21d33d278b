"""Build libpfm_hip.so (the C-ABI HIP library) in-tree for gfx950 with hipcc.

    python -m funasr_amd.build        # or funasr_amd.build.build()

Each csrc/*.hip is compiled to an object in parallel, then linked into
funasr_amd/_lib/libpfm_hip.so. Objects are rebuilt only when a source or header is newer.
"""
from __future__ import annotations

import glob
import os
import shutil
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
OUT_DIR = os.path.join(HERE, "_lib")
OBJ_DIR = os.path.join(HERE, "_lib", "obj")
LIB = os.path.join(OUT_DIR, "libpfm_hip.so")
ARCH = os.environ.get("PFM_OFFLOAD_ARCH", "gfx950")

# bit-exact host-order arithmetic (CIF / LayerNorm / fbank): no FMA contraction
NO_CONTRACT = {"k_elem.hip", "k_fbank.hip", "k_stream.hip"}


def hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found (ROCm required to build the HIP extension)")


def _flags(src: str):
    f = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-Wall", "-Wno-unused-function",
         "-Wno-unused-variable", "-Wno-unused-lambda-capture", "-I", os.path.join(ROOT, "include")]
    if os.path.basename(src) in NO_CONTRACT:
        f.append("-ffp-contract=off")
    return f


def _headers():
    return glob.glob(os.path.join(CSRC, "*.h")) + glob.glob(os.path.join(ROOT, "include", "*.h"))


def _stale(obj: str, deps) -> bool:
    if not os.path.exists(obj):
        return True
    t = os.path.getmtime(obj)
    return any(os.path.getmtime(d) > t for d in deps)


def build(verbose: bool = False, jobs: int = 8) -> str:
    os.makedirs(OBJ_DIR, exist_ok=True)
    cc = hipcc()
    srcs = sorted(glob.glob(os.path.join(CSRC, "*.hip")))
    hdrs = _headers()
    todo = []
    objs = []
    for s in srcs:
        o = os.path.join(OBJ_DIR, os.path.basename(s) + ".o")
        objs.append(o)
        if _stale(o, [s] + hdrs):
            todo.append((s, o))

    def compile_one(so):
        s, o = so
        cmd = [cc] + _flags(s) + ["-c", s, "-o", o]
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed on {os.path.basename(s)}:\n{r.stdout}\n{r.stderr}")
        if r.stderr.strip() and verbose:
            print(r.stderr)
        return o

    if todo:
        with ThreadPoolExecutor(max_workers=max(1, min(jobs, len(todo)))) as ex:
            list(ex.map(compile_one, todo))
    if todo or not os.path.exists(LIB) or _stale(LIB, objs):
        tmp = LIB + ".tmp"
        cmd = [cc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp] + objs
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stdout}\n{r.stderr}")
        os.replace(tmp, LIB)
    return LIB


if __name__ == "__main__":
    print(build(verbose="-v" in sys.argv))
