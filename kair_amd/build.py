"""Build libkair_hip.so (the C-ABI kernel library) for gfx950 with hipcc.

    python -m kair_amd.build [--force] [-j N]

Objects go to kair_amd/build/, the library to kair_amd/lib/libkair_hip.so (in-tree, so it travels
to the GPU box with the repo snapshot).  An object is rebuilt when the content stamp of its source,
the headers and the compile flags changes (not by mtime: `git stash` round trips and debug builds
would otherwise leave stale objects behind), the library when any object's stamp changed.
"""
import argparse
import concurrent.futures as cf
import glob
import hashlib
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
OBJ = os.path.join(HERE, "build")
LIB = os.path.join(HERE, "lib", "libkair_hip.so")
# debug-ablation builds: their own objects and library (kair_amd._hip loads it only with KAIR_LIB=debug),
# so a release build() after a debug one in the same process or tree never ships the ablation switches
OBJ_DBG = os.path.join(HERE, "build_dbg")
LIB_DBG = os.path.join(HERE, "lib", "libkair_hip_dbg.so")
INCLUDE = os.path.join(ROOT, "include")
ARCH = os.environ.get("KAIR_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-I", CSRC, "-I", INCLUDE,
         "-Wno-unused-result", "-munsafe-fp-atomics"]


def _headers_digest():
    h = hashlib.sha256()
    for p in sorted(glob.glob(os.path.join(CSRC, "*.h")) + glob.glob(os.path.join(INCLUDE, "*.h"))):
        h.update(p.encode())
        with open(p, "rb") as f:
            h.update(f.read())
    return h.hexdigest()


def _read(p):
    try:
        with open(p) as f:
            return f.read().strip()
    except OSError:
        return None


def _compile(src, force, hdr, flags, objdir):
    obj = os.path.join(objdir, os.path.basename(src) + ".o")
    h = hashlib.sha256(" ".join([HIPCC, *flags, hdr]).encode())
    with open(src, "rb") as f:
        h.update(f.read())
    stamp = h.hexdigest()
    if not force and os.path.exists(obj) and _read(obj + ".stamp") == stamp:
        return obj, None, stamp
    if os.path.exists(obj + ".stamp"):
        os.remove(obj + ".stamp")
    cmd = [HIPCC, *flags, "-c", src, "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        return obj, f"$ {' '.join(cmd)}\n{r.stdout}\n{r.stderr}", stamp
    with open(obj + ".stamp", "w") as f:
        f.write(stamp)
    return obj, None, stamp


def build(force=False, jobs=None, verbose=True, debug_ablations=False):
    """debug_ablations: compile the perf-investigation ablation switches (KAIR_*_DBG environment bits
    that drop stores / skip GEMMs) into the library -- never for training; the release build has none."""
    flags = FLAGS + (["-DKAIR_DEBUG_ABLATIONS=1"] if debug_ablations else [])   # per call: FLAGS never changes
    objdir, lib = (OBJ_DBG, LIB_DBG) if debug_ablations else (OBJ, LIB)
    os.makedirs(objdir, exist_ok=True)
    os.makedirs(os.path.dirname(lib), exist_ok=True)
    srcs = sorted(glob.glob(os.path.join(CSRC, "*.hip")) + glob.glob(os.path.join(CSRC, "*.cpp")))
    hdr = _headers_digest()
    jobs = jobs or min(8, len(srcs), os.cpu_count() or 1)
    with cf.ThreadPoolExecutor(jobs) as ex:
        results = list(ex.map(lambda s: _compile(s, force, hdr, flags, objdir), srcs))
    errs = [e for _, e, _ in results if e]
    if errs:
        raise RuntimeError("hipcc failed:\n" + "\n".join(errs))
    objs = [o for o, _, _ in results]
    lib_stamp = hashlib.sha256("".join(st for _, _, st in results).encode()).hexdigest()
    if force or not os.path.exists(lib) or _read(lib + ".stamp") != lib_stamp:
        if os.path.exists(lib + ".stamp"):
            os.remove(lib + ".stamp")
        cmd = [HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", *objs, "-o", lib]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stdout}\n{r.stderr}")
        with open(lib + ".stamp", "w") as f:
            f.write(lib_stamp)
        if verbose:
            print("built", lib)
    return lib


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
