"""Build the gfx950 kernel library in-tree: ``iit_amd/_native/libiit_hip.so``.

Compiled directly with ``hipcc --offload-arch=gfx950`` (no hipify, no torch
extension machinery): the library exposes a plain C ABI that
:mod:`iit_amd.ops.hip_kernels` binds with ``ctypes`` and launches on the current
torch stream, so every launch is capturable in HIP graphs.  A source hash stamp
avoids rebuilding an up-to-date library (the built ``.so`` travels to the GPU box
with the repository snapshot).
"""
from __future__ import annotations

import hashlib
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
CSRC = os.path.join(ROOT, "csrc")
OUT_DIR = os.path.join(ROOT, "iit_amd", "_native")
LIB = os.path.join(OUT_DIR, "libiit_hip.so")
OBJ_CACHE = os.path.join(ROOT, "build", "objcache")  # git-ignored; not shipped to the GPU box
SOURCES = ["gemm.hip", "gemm_glds.hip", "gemm_dual.hip", "gemm_8ph.hip", "gemm_4w.hip", "conv_nhwc.hip", "kernels.hip", "attn_mfma.hip", "flash_attn.hip", "llama_ops.hip",
           "splice.hip", "ioi_hl.hip", "bn_nhwc.hip"]
# per-source compiler flags: the pipelined LDS-DMA GEMM keeps its accumulators in VGPRs (MFMA VGPR form), which
# avoids the AGPR shuffles hipcc otherwise emits around its register double buffer
EXTRA_FLAGS = {"gemm_glds.hip": ["-mllvm", "-amdgpu-mfma-vgpr-form"], "conv_nhwc.hip": ["-mllvm", "-amdgpu-mfma-vgpr-form"], "gemm_dual.hip": ["-mllvm", "-amdgpu-mfma-vgpr-form"],
               "gemm_8ph.hip": ["-mllvm", "-amdgpu-mfma-vgpr-form"]}
HEADERS = ["common.h", "gemm_glds_body.h", "gemm_w4.h", "splice_spec.h"]
ARCH = os.environ.get("IIT_OFFLOAD_ARCH", "gfx950")


def _hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc"):
        if c and os.path.exists(c):
            return c
    return "hipcc"


def sources():
    return [os.path.join(CSRC, s) for s in SOURCES if os.path.exists(os.path.join(CSRC, s))]


def source_hash() -> str:
    h = hashlib.sha256()
    for p in sources() + [os.path.join(CSRC, h) for h in HEADERS]:
        with open(p, "rb") as f:
            h.update(f.read())
    h.update(ARCH.encode())
    h.update(repr(sorted(EXTRA_FLAGS.items())).encode())
    return h.hexdigest()[:16]


def is_up_to_date() -> bool:
    stamp = LIB + ".stamp"
    return os.path.exists(LIB) and os.path.exists(stamp) and open(stamp).read().strip() == source_hash()


def _obj_key(src: str) -> str:
    """Object-cache key of one source: its text, every shared header, the arch and its flags."""
    h = hashlib.sha256()
    for p in [src] + [os.path.join(CSRC, x) for x in HEADERS]:
        with open(p, "rb") as f:
            h.update(f.read())
    h.update(ARCH.encode())
    h.update(repr(EXTRA_FLAGS.get(os.path.basename(src), [])).encode())
    return h.hexdigest()[:16]


def build(force: bool = False, verbose: bool = False) -> str:
    if not force and is_up_to_date():
        return LIB
    os.makedirs(OBJ_CACHE, exist_ok=True)
    objs = []
    procs = []
    for src in sources():
        # per-source object cache: only the sources (or shared headers) that changed are recompiled
        obj = os.path.join(OBJ_CACHE, f"{os.path.basename(src)}.{_obj_key(src)}.o")
        objs.append(obj)
        if os.path.exists(obj) and not force:
            continue
        cmd = [_hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-munsafe-fp-atomics",
               "-I", CSRC, "-c", src, "-o", obj + ".tmp"] + EXTRA_FLAGS.get(os.path.basename(src), [])
        procs.append((cmd, obj, subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)))
    for cmd, obj, p in procs:
        out, _ = p.communicate()
        if p.returncode != 0:
            raise RuntimeError(f"hipcc failed: {' '.join(cmd)}\n{out.decode(errors='replace')}")
        os.replace(obj + ".tmp", obj)
        if verbose and out:
            print(out.decode(errors="replace"))
    tmp = LIB + ".tmp"
    cmd = [_hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp] + objs
    res = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
    if res.returncode != 0:
        raise RuntimeError(f"link failed: {res.stdout.decode(errors='replace')}")
    os.replace(tmp, LIB)
    keep = set(objs)
    for f in os.listdir(OBJ_CACHE):  # drop stale objects of earlier source versions
        if os.path.join(OBJ_CACHE, f) not in keep:
            os.remove(os.path.join(OBJ_CACHE, f))
    with open(LIB + ".stamp", "w") as f:
        f.write(source_hash())
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
