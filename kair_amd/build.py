"""Build libkair_hip.so (the C-ABI kernel library) for gfx950 with hipcc.

    python -m kair_amd.build [--force] [-j N]

Objects go to kair_amd/build/, the library to kair_amd/lib/libkair_hip.so (in-tree, so it travels
to the GPU box with the repo snapshot).  Rebuilds only when a source or header is newer.
"""
import argparse
import concurrent.futures as cf
import glob
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
OBJ = os.path.join(HERE, "build")
LIB = os.path.join(HERE, "lib", "libkair_hip.so")
INCLUDE = os.path.join(ROOT, "include")
ARCH = os.environ.get("KAIR_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-I", CSRC, "-I", INCLUDE,
         "-Wno-unused-result", "-munsafe-fp-atomics"]


def _newest_dep():
    deps = glob.glob(os.path.join(CSRC, "*.h")) + glob.glob(os.path.join(INCLUDE, "*.h"))
    return max(os.path.getmtime(p) for p in deps) if deps else 0.0


def _compile(src, force, dep_time):
    obj = os.path.join(OBJ, os.path.basename(src) + ".o")
    if not force and os.path.exists(obj) and os.path.getmtime(obj) >= max(os.path.getmtime(src), dep_time):
        return obj, None
    cmd = [HIPCC, *FLAGS, "-c", src, "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        return obj, f"$ {' '.join(cmd)}\n{r.stdout}\n{r.stderr}"
    return obj, None


def build(force=False, jobs=None, verbose=True, debug_ablations=False):
    """debug_ablations: compile the perf-investigation ablation switches (KAIR_*_DBG environment bits
    that drop stores / skip GEMMs) into the library -- never for training; the release build has none."""
    if debug_ablations:
        FLAGS.append("-DKAIR_DEBUG_ABLATIONS=1")
        force = True
    os.makedirs(OBJ, exist_ok=True)
    os.makedirs(os.path.dirname(LIB), exist_ok=True)
    srcs = sorted(glob.glob(os.path.join(CSRC, "*.hip")) + glob.glob(os.path.join(CSRC, "*.cpp")))
    dep_time = _newest_dep()
    jobs = jobs or min(8, len(srcs), os.cpu_count() or 1)
    with cf.ThreadPoolExecutor(jobs) as ex:
        results = list(ex.map(lambda s: _compile(s, force, dep_time), srcs))
    errs = [e for _, e in results if e]
    if errs:
        raise RuntimeError("hipcc failed:\n" + "\n".join(errs))
    objs = [o for o, _ in results]
    if force or not os.path.exists(LIB) or os.path.getmtime(LIB) < max(os.path.getmtime(o) for o in objs):
        cmd = [HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", *objs, "-o", LIB]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stdout}\n{r.stderr}")
        if verbose:
            print("built", LIB)
    return LIB


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", type=int, default=None)
    ap.add_argument("--debug-ablations", action="store_true")
    a = ap.parse_args()
    try:
        build(a.force, a.j, debug_ablations=a.debug_ablations)
    except RuntimeError as e:
        print(e, file=sys.stderr)
        sys.exit(1)
