"""Build librn.so (the C-ABI HIP runtime) in-tree for gfx950.

Each csrc/*.hip is compiled to an object in parallel with hipcc, then linked into
resnet.mxnet_amd/rn/librn.so. The .so is git-ignored but travels to the GPU box with the
gpurun snapshot. Rebuilds only when a source or header is newer than the library.
"""
import concurrent.futures as cf
import os
import subprocess
import sys

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG_DIR)                      # resnet.mxnet_amd/
REPO = os.path.dirname(ROOT)
CSRC = os.path.join(ROOT, "csrc")
INCLUDE = os.path.join(REPO, "include")
# RN_DIAG=1: the diagnostic build (wrong-result isolation modes of rn_set_tuning 3 / 6 / 7 and
# rn_sgd_mom_update_pack_checked compiled in) as a separate library; the product loads librn.so
DIAG = os.environ.get("RN_DIAG", "0") == "1"
BUILD_DIR = os.path.join(ROOT, "build_diag" if DIAG else "build")
LIB_PATH = os.path.join(PKG_DIR, "librn_diag.so" if DIAG else "librn.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"
CXXFLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-I", INCLUDE, "-I", CSRC,
            "-Wno-unused-result", "-munsafe-fp-atomics",
            "-mllvm", "-disable-promote-alloca-to-lds"]  # keep per-thread arrays out of the staging LDS
if DIAG:
    CXXFLAGS.append("-DRN_DIAG=1")


def _sources():
    return sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".hip"))


def _deps():
    deps = [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith((".h", ".hip"))]
    deps += [os.path.join(INCLUDE, f) for f in os.listdir(INCLUDE) if f.endswith(".h")]
    deps.append(os.path.abspath(__file__))
    return deps


def needs_build():
    if not os.path.exists(LIB_PATH):
        return True
    t = os.path.getmtime(LIB_PATH)
    return any(os.path.getmtime(d) > t for d in _deps())


def _compile(src, extra):
    obj = os.path.join(BUILD_DIR, os.path.basename(src) + ".o")
    cmd = [HIPCC] + CXXFLAGS + extra + ["-c", src, "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src}:\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return obj


def build(force=False, verbose=True, extra=()):
    if not force and not needs_build():
        return LIB_PATH
    os.makedirs(BUILD_DIR, exist_ok=True)
    srcs = _sources()
    jobs = min(len(srcs), int(os.environ.get("MAX_JOBS", "8")), 16)
    with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        objs = list(ex.map(lambda s: _compile(s, list(extra)), srcs))
    tmp = LIB_PATH + ".tmp"
    cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp] + objs
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{r.stdout}\n{r.stderr}")
    os.replace(tmp, LIB_PATH)
    if verbose:
        print(f"[rn] built {LIB_PATH}", file=sys.stderr)
    return LIB_PATH


if __name__ == "__main__":
    build(force="--force" in sys.argv)
