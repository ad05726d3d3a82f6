"""Build libmovierec_ncf.so for gfx950 with hipcc (no cmake, no JIT cache).

Output goes in-tree (``movierec/_lib/``) so it travels with the repo snapshot
to the GPU box.  Usage: ``python csrc/build.py [--force]``.
"""

import concurrent.futures as cf
import hashlib
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


HASH_MARK = b"NCF_SRC_SHA256="


def source_hash(defines=()):
    """SHA-256 of what the library is compiled from: every csrc .hip/.h source and the ABI header
    (name order, name + content), the compiler flags and the -D defines.  Embedded in the binary
    (ncf_build_info) so a library can be matched to the tree it came from."""
    files = sorted(f for f in os.listdir(HERE) if f.endswith((".hip", ".h")))
    h = hashlib.sha256()
    for f in files:
        h.update(f.encode() + b"\0")
        with open(os.path.join(HERE, f), "rb") as fh:
            h.update(fh.read())
    with open(os.path.join(INCLUDE, "movierec_ncf.h"), "rb") as fh:
        h.update(b"movierec_ncf.h\0" + fh.read())
    h.update(repr(([f for f in CFLAGS if not f.startswith("-I")], sorted(EXTRA.items()), list(defines), _env_extras())).encode())
    return h.hexdigest()


def _env_extras():
    """NCF_EXTRA_<SOURCE STEM> compiler flags in the environment (experiment variants)."""
    return sorted((k, v) for k, v in os.environ.items() if k.startswith("NCF_EXTRA_") and v.strip())


def embedded_hash(lib_path):
    """The source hash a built library carries (None if absent or unreadable)."""
    try:
        with open(lib_path, "rb") as fh:
            data = fh.read()
    except OSError:
        return None
    i = data.find(HASH_MARK)
    if i < 0:
        return None
    return data[i + len(HASH_MARK):i + len(HASH_MARK) + 64].decode("ascii", "replace")


def build(force=False, verbose=False, defines=(), out=None):
    """Compile and link; ``defines``/``out`` build an experiment variant elsewhere.  An existing
    library is reused only when its embedded source hash equals the tree's (no mtime trust)."""
    lib_path = out or LIB
    os.makedirs(os.path.dirname(lib_path), exist_ok=True)
    want = source_hash(defines)
    if not force and embedded_hash(lib_path) == want:
        return lib_path
    variant = " ".join(["-D" + d for d in defines] + ["%s=%s" % kv for kv in _env_extras()])
    info = ["-DNCF_BUILD_HASH=\"%s\"" % want, "-DNCF_BUILD_DEFINES=\"%s\"" % variant.replace('"', "'")]
    obj_dir = os.path.join(os.path.dirname(lib_path), "obj" + ("_" + os.path.basename(lib_path) if out else ""))
    os.makedirs(obj_dir, exist_ok=True)

    def compile_one(src):
        obj = os.path.join(obj_dir, src.replace(".hip", ".o"))
        # NCF_EXTRA_<SOURCE STEM>: extra compiler flags of one source (experiment variants)
        env_extra = os.environ.get("NCF_EXTRA_" + src.replace(".hip", "").upper(), "").split()
        cmd = ([HIPCC] + CFLAGS + EXTRA.get(src, []) + env_extra + ["-D" + d for d in defines] +
               (info if src == "ncf_capi.hip" else []) + ["-c", os.path.join(HERE, src), "-o", obj])
        if verbose:
            print(" ".join(cmd))
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError("hipcc failed on %s:\n%s\n%s" % (src, r.stdout, r.stderr))
        return obj

    with cf.ThreadPoolExecutor(max_workers=min(8, len(SOURCES))) as ex:
        objs = list(ex.map(compile_one, SOURCES))
    tmp = lib_path + ".tmp"
    # RCCL (the data-parallel step's collectives, ncf_comm.hip): librccl.so.1, the soname torch loads
    # too.  No vendor BLAS: every matrix product is a hand-written MFMA kernel.
    cmd = [HIPCC, "--offload-arch=" + ARCH, "-shared", "-o", tmp] + objs + ["-L/opt/rocm/lib", "-lrccl"]
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
