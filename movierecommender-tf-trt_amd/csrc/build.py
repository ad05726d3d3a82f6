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
SOURCES = ["ncf_index.hip", "ncf_update.hip", "ncf_generic.hip", "ncf_fused.hip", "ncf_unit.hip", "ncf_wave.hip", "ncf_layered.hip", "ncf_layer1.hip", "ncf_laymid.hip", "ncf_score.hip", "ncf_sample.hip", "ncf_comm.hip", "ncf_capi.hip"]
# per-source extra flags: the scorer keeps its MFMA accumulators in VGPRs (no v_accvgpr_read
# before every epilogue op; its 226 registers fit the unified file at 2 waves/SIMD)
EXTRA = {"ncf_score.hip": ["-mllvm", "-amdgpu-mfma-vgpr-form"]}
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"
CFLAGS = ["--offload-arch=" + ARCH, "-O3", "-fPIC", "-std=c++17", "-I" + INCLUDE, "-I" + HERE,
          "-Wno-unused-result"]


def _deps_mtime():
    files = [os.path.join(HERE, f) for f in os.listdir(HERE) if f.endswith((".hip", ".h"))]
    files.append(os.path.join(INCLUDE, "movierec_ncf.h"))
    return max(os.path.getmtime(f) for f in files)


def build(force=False, verbose=False, defines=(), out=None):
    """Compile and link; ``defines``/``out`` build an experiment variant elsewhere."""
    lib_path = out or LIB
    os.makedirs(os.path.dirname(lib_path), exist_ok=True)
    if not force and os.path.exists(lib_path) and os.path.getmtime(lib_path) >= _deps_mtime():
        return lib_path
    obj_dir = os.path.join(os.path.dirname(lib_path), "obj" + ("_" + os.path.basename(lib_path) if out else ""))
    os.makedirs(obj_dir, exist_ok=True)

    def compile_one(src):
        obj = os.path.join(obj_dir, src.replace(".hip", ".o"))
        # NCF_EXTRA_<SOURCE STEM>: extra compiler flags of one source (experiment variants)
        env_extra = os.environ.get("NCF_EXTRA_" + src.replace(".hip", "").upper(), "").split()
        cmd = ([HIPCC] + CFLAGS + EXTRA.get(src, []) + env_extra + ["-D" + d for d in defines] +
               ["-c", os.path.join(HERE, src), "-o", obj])
        if verbose:
            print(" ".join(cmd))
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError("hipcc failed on %s:\n%s\n%s" % (src, r.stdout, r.stderr))
        return obj

    with cf.ThreadPoolExecutor(max_workers=min(8, len(SOURCES))) as ex:
        objs = list(ex.map(compile_one, SOURCES))
    tmp = lib_path + ".tmp"
    # rocBLAS (plain fp32 GEMMs of the layered path): same soname as the copy torch loads, so one
    # rocBLAS serves the process
    # RCCL (the data-parallel step's all-reduce, ncf_comm.hip): librccl.so.1, the soname torch loads too
    cmd = [HIPCC, "--offload-arch=" + ARCH, "-shared", "-o", tmp] + objs + ["-L/opt/rocm/lib", "-lrocblas", "-lrccl"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("link failed:\n%s\n%s" % (r.stdout, r.stderr))
    os.replace(tmp, lib_path)
    return lib_path


if __name__ == "__main__":
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-D", dest="defines", action="append", default=[])
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    print(build(force=a.force, verbose=True, defines=a.defines, out=a.out))
