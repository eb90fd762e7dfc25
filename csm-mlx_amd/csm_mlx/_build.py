"""Build libcsm_hip.so in-tree with hipcc for gfx950 (no torch, no JIT cache).

Every ``*.hip`` / ``*.cpp`` under csm-mlx_amd/csrc is compiled to an object
under csm-mlx_amd/build/ and linked into csm-mlx_amd/csm_mlx/libcsm_hip.so, so
the shared library travels with the repo snapshot to the GPU box.
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)                     # csm-mlx_amd/
CSRC = os.path.join(ROOT, "csrc")
BUILD = os.path.join(ROOT, "build")
LIB = os.path.join(PKG, "libcsm_hip.so")
ARCH = os.environ.get("CSM_HIP_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-Wno-unused-result"]
# per-source flags: the persistent kernels hold weight prefetches in registers across hand-off
# waits at 256 VGPRs; the AMDGPU scheduler's own register-pressure trackers keep it from spilling
# them (55 -> 5 spilled VGPRs; a spill store waits for its load, draining the prefetch).
SRC_FLAGS = {"dec_frame.hip": ["-mllvm", "-amdgpu-use-amdgpu-trackers=1"],
             "bb_step.hip": ["-mllvm", "-amdgpu-use-amdgpu-trackers=1"],
             "dec_step_xs.hip": ["-mllvm", "-amdgpu-use-amdgpu-trackers=1"]}


def _sources():
    return sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith((".hip", ".cpp")))


def _headers_mtime():
    hs = [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")]
    hs += [os.path.join(os.path.dirname(ROOT), "include", h) for h in ("csm_hip.h", "csm_hip_prof.h")]
    return max(os.path.getmtime(h) for h in hs if os.path.exists(h))


def _compile(src, hdr_mtime, verbose):
    obj = os.path.join(BUILD, os.path.basename(src) + ".o")
    if os.path.exists(obj) and os.path.getmtime(obj) >= max(os.path.getmtime(src), hdr_mtime):
        return obj
    lang = ["-x", "hip"] if src.endswith(".hip") else []
    cmd = [HIPCC, *FLAGS, *SRC_FLAGS.get(os.path.basename(src), []), *lang, "-c", src, "-o", obj]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src}:\n{r.stderr[-6000:]}")
    return obj


def build(verbose: bool = False, jobs: int = 8) -> str:
    os.makedirs(BUILD, exist_ok=True)
    srcs = _sources()
    hm = _headers_mtime()
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        objs = list(ex.map(lambda s: _compile(s, hm, verbose), srcs))
    if not os.path.exists(LIB) or os.path.getmtime(LIB) < max(os.path.getmtime(o) for o in objs):
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", LIB, *objs]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stderr[-6000:]}")
    return LIB


if __name__ == "__main__":
    print(build(verbose=True))
