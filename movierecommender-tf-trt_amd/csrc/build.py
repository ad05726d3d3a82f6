"""Build libmovierec_ncf.so for gfx950 with hipcc (no cmake, no JIT cache).

Output goes in-tree (``movierec/_lib/``) so it travels with the repo snapshot
to the GPU box.  Usage: ``python csrc/build.py [--force]``.
"""

import concurrent.futures as cf
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.dirname(HERE)
ROOT = os.path.dirname(PKG)
INCLUDE = os.path.join(ROOT, "include")
OUT_DIR = os.path.join(PKG, "movierec", "_lib")
LIB = os.path.join(OUT_DIR, "libmovierec_ncf.so")
SOURCES = ["ncf_index.hip", "ncf_update.hip", "ncf_generic.hip", "ncf_fused.hip", "ncf_capi.hip"]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"
CFLAGS = ["--offload-arch=" + ARCH, "-O3", "-fPIC", "-std=c++17", "-I" + INCLUDE, "-I" + HERE,
          "-Wno-unused-result"]


def _deps_mtime():
    files = [os.path.join(HERE, f) for f in os.listdir(HERE) if f.endswith((".hip", ".h"))]
    files.append(os.path.join(INCLUDE, "movierec_ncf.h"))
    return max(os.path.getmtime(f) for f in files)


def build(force=False, verbose=False):
    os.makedirs(OUT_DIR, exist_ok=True)
    if not force and os.path.exists(LIB) and os.path.getmtime(LIB) >= _deps_mtime():
        return LIB
    obj_dir = os.path.join(OUT_DIR, "obj")
    os.makedirs(obj_dir, exist_ok=True)

    def compile_one(src):
        obj = os.path.join(obj_dir, src.replace(".hip", ".o"))
        cmd = [HIPCC] + CFLAGS + ["-c", os.path.join(HERE, src), "-o", obj]
        if verbose:
            print(" ".join(cmd))
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError("hipcc failed on %s:\n%s\n%s" % (src, r.stdout, r.stderr))
        return obj

    with cf.ThreadPoolExecutor(max_workers=min(8, len(SOURCES))) as ex:
        objs = list(ex.map(compile_one, SOURCES))
    tmp = LIB + ".tmp"
    cmd = [HIPCC, "--offload-arch=" + ARCH, "-shared", "-o", tmp] + objs
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("link failed:\n%s\n%s" % (r.stdout, r.stderr))
    os.replace(tmp, LIB)
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
