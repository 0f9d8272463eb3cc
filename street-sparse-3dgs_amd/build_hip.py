"""Build the gfx950 HIP library libgsr_hip.so in-tree (hipcc cross-compiles without a GPU).

    python street-sparse-3dgs_amd/build_hip.py [--force] [--jobs N]

Each csrc/*.hip is compiled to an object with `hipcc --offload-arch=gfx950 -O3
-ffp-contract=off` (fp contraction off keeps the index-producing maths bit-reproducible by
the CPU oracle) and the objects are linked into
street-sparse-3dgs_amd/diff_gaussian_rasterization/libgsr_hip.so.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import glob
import os
import subprocess
import sys

PKG_ROOT = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(PKG_ROOT)
CSRC = os.path.join(PKG_ROOT, "csrc")
OBJ = os.path.join(PKG_ROOT, "build", "obj")
LIB = os.path.join(PKG_ROOT, "diff_gaussian_rasterization", "libgsr_hip.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("GSR_OFFLOAD_ARCH", "gfx950")
CFLAGS = ["--offload-arch=" + ARCH, "-O3", "-fPIC", "-std=c++17", "-ffp-contract=off", "-Wall",
          "-Wno-unused-result", "-I", CSRC, "-I", os.path.join(REPO, "include")]


# Per-file extra flags.  render.hip: the SLP vectoriser pairs the backward's per-pixel
# accumulations into v_pk_fma/add_f32 fed by v_mov_b32 shuffles -- packed fp32 has no throughput
# gain on gfx950, so the moves (4 per pixel, 16 per instance) are pure overhead: render_bwd
# 0.260 -> 0.246 ms.  train.hip (the SSIM passes): train step -1%.
FILE_FLAGS = {"render.hip": ["-fno-slp-vectorize"], "train.hip": ["-fno-slp-vectorize"]}
for _f in filter(None, os.environ.get("GSR_NOSLP_FILES", "").split(",")):  # measurement variants
    FILE_FLAGS[_f] = ["-fno-slp-vectorize"]
if os.environ.get("GSR_RENDER_FLAGS"):  # measurement variants: extra flags for render.hip
    FILE_FLAGS["render.hip"] = FILE_FLAGS["render.hip"] + os.environ["GSR_RENDER_FLAGS"].split()


def _headers():
    return glob.glob(os.path.join(CSRC, "*.h")) + glob.glob(os.path.join(REPO, "include", "*.h"))


def _stale(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _compile(src, force, objdir=OBJ, defines=()):
    obj = os.path.join(objdir, os.path.basename(src) + ".o")
    if force or _stale(obj, [src] + _headers()):
        cmd = [HIPCC] + CFLAGS + FILE_FLAGS.get(os.path.basename(src), []) + ["-D" + d for d in defines] + \
            ["-c", src, "-o", obj + ".tmp"]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed for {src}:\n{r.stdout}\n{r.stderr}")
        os.replace(obj + ".tmp", obj)
    return obj


HOST_SRC = os.path.join(PKG_ROOT, "host", "rasterize_host.cpp")
HOST_EXT = os.path.join(PKG_ROOT, "diff_gaussian_rasterization", "_gsr_host.so")


def build_host(force: bool = False, out: str = HOST_EXT) -> str:
    """The rasterizer's per-call host path (host/rasterize_host.cpp): a CPython extension against
    torch's C++ API that calls libgsr_hip.so's C ABI.  Plain g++ -- host code only, no device code --
    with torch's include paths and C++ ABI."""
    import sysconfig

    import torch
    import torch.utils.cpp_extension as ce
    if not force and not _stale(out, [HOST_SRC, os.path.join(REPO, "include", "gsr.h")]):
        return out
    tlib = os.path.join(os.path.dirname(torch.__file__), "lib")
    cmd = ["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-w", "-DTORCH_EXTENSION_NAME=_gsr_host",
           "-DTORCH_API_INCLUDE_EXTENSION_H", f"-D_GLIBCXX_USE_CXX11_ABI={int(torch._C._GLIBCXX_USE_CXX11_ABI)}",
           "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1"]
    for inc in ce.include_paths() + [sysconfig.get_paths()["include"], "/opt/rocm/include",
                                     os.path.join(REPO, "include")]:
        cmd += ["-I", inc]
    # libgsr_hip.so is not linked: bind(path) dlopens the file the ctypes layer loaded (GSR_LIBRARY too)
    cmd += [HOST_SRC, "-o", out + ".tmp", "-L", tlib, "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_python",
            "-ldl", "-Wl,-rpath," + tlib]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"host extension build failed:\n{r.stdout}\n{r.stderr}")
    os.replace(out + ".tmp", out)
    return out


def build(force: bool = False, jobs: int = 4, defines=(), lib: str = LIB) -> str:
    """Build the library; `defines` (NAME or NAME=VALUE) with a different `lib` path builds a
    measurement variant in its own object directory (load it with GSR_LIBRARY=path)."""
    tag = [d.replace("=", "-") for d in defines]
    if os.environ.get("GSR_NOSLP_FILES"):
        tag.append("noslp-" + os.environ["GSR_NOSLP_FILES"].replace(",", "-"))
    if os.environ.get("GSR_RENDER_FLAGS"):
        tag.append("rf" + "".join(c for c in os.environ["GSR_RENDER_FLAGS"] if c.isalnum()))
    objdir = OBJ if not tag else os.path.join(PKG_ROOT, "build", "obj_" + "_".join(tag))
    os.makedirs(objdir, exist_ok=True)
    srcs = sorted(glob.glob(os.path.join(CSRC, "*.hip")))
    with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        objs = list(ex.map(lambda s: _compile(s, force, objdir, tuple(defines)), srcs))
    if force or _stale(lib, objs):
        os.makedirs(os.path.dirname(lib), exist_ok=True)
        cmd = [HIPCC, "--offload-arch=" + ARCH, "-shared", "-fPIC", "-o", lib + ".tmp"] + objs
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stdout}\n{r.stderr}")
        os.replace(lib + ".tmp", lib)
    return lib


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--jobs", type=int, default=4)
    ap.add_argument("--define", action="append", default=[], help="extra -D for a measurement variant")
    ap.add_argument("--out", default=LIB, help="library path (variants: anywhere outside the package)")
    a = ap.parse_args()
    print(build(a.force, a.jobs, a.define, a.out))
    if a.out == LIB:
        print(build_host(a.force))
    sys.exit(0)
