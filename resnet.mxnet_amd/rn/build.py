"""Build librn.so (the C-ABI HIP runtime) in-tree for gfx950.

Each csrc/*.hip is compiled to an object in parallel with hipcc, then linked into
resnet.mxnet_amd/rn/librn.so. The .so is git-ignored but travels to the GPU box with the
gpurun snapshot. The library carries a build id -- a hash of the sources, include/rn.h and the compiler
flags (source_hash) -- baked in with -DRN_BUILD_ID and exported as rn_build_id(); it is rebuilt whenever
that id differs from the tree's, and rn.lib.load() refuses a library whose id does not match (a stale
prebuilt after a checkout or copy fails loudly instead of being tested silently).
"""
import concurrent.futures as cf
import hashlib
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


def source_hash(diag=DIAG):
    """16 hex digits over the library's inputs: every csrc/*.hip / *.h and include/*.h (name + bytes) and
    the compile flags (the diagnostic build's -DRN_DIAG=1 included). Machine-independent: the same tree
    gives the same id here and on the GPU box."""
    h = hashlib.sha256()
    flags = [f for f in CXXFLAGS if f != "-DRN_DIAG=1"] + (["-DRN_DIAG=1"] if diag else [])
    h.update(" ".join(f for f in flags if f not in (INCLUDE, CSRC)).encode())
    for path in sorted(_deps()):
        if path == os.path.abspath(__file__):
            continue
        h.update(os.path.relpath(path, REPO).encode() + b"\0")
        with open(path, "rb") as f:
            h.update(f.read())
        h.update(b"\0")
    return h.hexdigest()[:16]


_MARKER = b"RN_BUILD_ID="


def library_build_id(path=None):
    """The build id baked into a built library file (read from its bytes, without loading it), or None."""
    path = path or LIB_PATH
    if not os.path.exists(path):
        return None
    with open(path, "rb") as f:
        data = f.read()
    i = data.find(_MARKER)
    return data[i + len(_MARKER):i + len(_MARKER) + 16].decode("ascii", "replace") if i >= 0 else None


def needs_build():
    return library_build_id(LIB_PATH) != source_hash()


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
    bid = [f'-DRN_BUILD_ID="{source_hash()}"'] if not extra else []  # (extra flags: an experiment, no id)
    with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        objs = list(ex.map(lambda s: _compile(s, bid + list(extra)), srcs))
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
