"""Build recipe for the gfx950 HIP library ``lib/libhashnerf_amd.so``.

Plain ``hipcc`` (no cmake, no torch extension machinery): each ``csrc/*.hip``
is compiled to an object with ``--offload-arch=gfx950 -ffp-contract=off``
(fp32 expressions round exactly like the reference's eager torch ops), then
linked into one C-ABI shared library.  Objects are rebuilt only when a source
or header is newer.
"""
from __future__ import annotations

import glob
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
LIBDIR = os.path.join(HERE, "lib")
OBJDIR = os.path.join(HERE, "build")
LIB = os.path.join(LIBDIR, "libhashnerf_amd.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"
# -amdgpu-mfma-vgpr-form: MFMA accumulators are allocated as VGPRs where the
# registers allow (the MLP backward's dW accumulators stay in AGPRs); its
# data-path MFMA results then need no v_accvgpr_read before their ReLU/split
# VALU (~300 -> ~150 accvgpr moves per tile; MLP-backward launch -0.5 to -1%,
# r03h; the forward is unchanged: it uses no AGPRs at 4 waves per SIMD).
CFLAGS = ["-O3", f"--offload-arch={ARCH}", "-std=c++17", "-fPIC", "-ffp-contract=off",
          "-munsafe-fp-atomics", "-mllvm", "-amdgpu-mfma-vgpr-form=1",
          "-Wall", "-Wno-unused-function", "-I", os.path.join(ROOT, "include")]


def _newest(paths):
    return max((os.path.getmtime(p) for p in paths), default=0.0)


def sources():
    return sorted(glob.glob(os.path.join(CSRC, "*.hip")))


def build_variant(defines, out_lib, verbose=False) -> str:
    """Diagnostic build (e.g. ``["-DHN_ABLATE=1"]``) into its own .so and objects."""
    objdir = out_lib + ".objs"
    os.makedirs(objdir, exist_ok=True)
    objs = []
    for src in sources():
        obj = os.path.join(objdir, os.path.basename(src).replace(".hip", ".o"))
        subprocess.run([HIPCC, *CFLAGS, *defines, "-c", src, "-o", obj], check=True)
        objs.append(obj)
    subprocess.run([HIPCC, "-shared", f"--offload-arch={ARCH}", "-fPIC", *objs, "-o", out_lib], check=True)
    return out_lib


def build(verbose: bool = False, force: bool = False) -> str:
    os.makedirs(LIBDIR, exist_ok=True)
    os.makedirs(OBJDIR, exist_ok=True)
    headers = glob.glob(os.path.join(CSRC, "*.h")) + glob.glob(os.path.join(ROOT, "include", "*.h"))
    hdr_t = _newest(headers)
    objs = []
    for src in sources():
        obj = os.path.join(OBJDIR, os.path.basename(src).replace(".hip", ".o"))
        objs.append(obj)
        if force or not os.path.exists(obj) or os.path.getmtime(obj) < max(os.path.getmtime(src), hdr_t):
            cmd = [HIPCC, *CFLAGS, "-c", src, "-o", obj]
            if verbose:
                print(" ".join(cmd), file=sys.stderr)
            subprocess.run(cmd, check=True)
    if force or not os.path.exists(LIB) or os.path.getmtime(LIB) < _newest(objs):
        cmd = [HIPCC, "-shared", f"--offload-arch={ARCH}", "-fPIC", *objs, "-o", LIB]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        subprocess.run(cmd, check=True)
    return LIB


if __name__ == "__main__":
    print(build(verbose=True, force="--force" in sys.argv))
