"""Builds libdrnmi.so (the C-ABI library of HIP kernels) in-tree for gfx950.

Plain hipcc, one object per .hip source compiled in parallel, then one shared
link.  The .so lands next to this file so it travels to the GPU box with the
repository snapshot (it is git-ignored, not gpurun-ignored).
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import subprocess
import sys

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG_DIR)                 # video-seg-model-compress_amd/
REPO = os.path.dirname(ROOT)
CSRC = os.path.join(ROOT, "csrc")
INCLUDE = os.path.join(REPO, "include")
LIB_PATH = os.path.join(PKG_DIR, "libdrnmi.so")
OBJ_DIR = os.path.join(ROOT, "build")

HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"
CFLAGS = ["-O3", "-fPIC", "-std=c++17", f"--offload-arch={ARCH}", "-I", INCLUDE, "-Wall",
          "-Wno-unused-function"]


# per-source extra flags.  front.hip: MFMA results in VGPRs (the weights are pinned to AGPRs in the
# source), so the epilogues read the accumulators without v_accvgpr_read copies
EXTRA = {"front.hip": ["-mllvm", "-amdgpu-mfma-vgpr-form=1"], "block64.hip": ["-mllvm", "-amdgpu-mfma-vgpr-form=1"],
         "conv_s2row.hip": ["-mllvm", "-amdgpu-mfma-vgpr-form=1"]}


def sources():
    return sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith((".hip", ".cpp")))


def _headers_mtime():
    hs = [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")]
    hs += [os.path.join(INCLUDE, f) for f in os.listdir(INCLUDE) if f.endswith(".h")]
    return max(os.path.getmtime(h) for h in hs) if hs else 0.0


def _compile(src: str, obj: str) -> None:
    cmd = [HIPCC, *CFLAGS, *EXTRA.get(os.path.basename(src), []), "-c", src, "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src}:\n{r.stdout}\n{r.stderr}")


def build(force: bool = False, jobs: int = 8, verbose: bool = True) -> str:
    os.makedirs(OBJ_DIR, exist_ok=True)
    hdr_t = _headers_mtime()
    todo, objs = [], []
    for src in sources():
        obj = os.path.join(OBJ_DIR, os.path.basename(src) + ".o")
        objs.append(obj)
        if force or not os.path.exists(obj) or os.path.getmtime(obj) < max(os.path.getmtime(src), hdr_t):
            todo.append((src, obj))
    if todo:
        if verbose:
            print(f"[drnmi.build] hipcc {len(todo)} source(s) for {ARCH}", file=sys.stderr)
        with cf.ThreadPoolExecutor(max_workers=min(jobs, len(todo))) as ex:
            list(ex.map(lambda a: _compile(*a), todo))
    newest_obj = max(os.path.getmtime(o) for o in objs)
    if force or todo or not os.path.exists(LIB_PATH) or os.path.getmtime(LIB_PATH) < newest_obj:
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", *objs, "-o", LIB_PATH]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stdout}\n{r.stderr}")
        if verbose:
            print(f"[drnmi.build] linked {LIB_PATH}", file=sys.stderr)
    return LIB_PATH


if __name__ == "__main__":
    build(force="--force" in sys.argv)
