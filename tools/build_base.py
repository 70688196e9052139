"""A/B baseline library: kair_amd/lib/libkair_hip_base.so built from the kernel sources of a git revision
(loaded with KAIR_LIB=base; never shipped).  Sources identical to the working tree reuse its objects
(kair_amd/build/), so a one-file change rebuilds one object.

    python tools/build_base.py REV      e.g. HEAD, HEAD~1
"""
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from kair_amd import build as B  # noqa: E402


def main():
    rev = sys.argv[1] if len(sys.argv) > 1 else "HEAD"
    B.build(verbose=False)   # the working tree's objects, to reuse
    tmp = tempfile.mkdtemp(prefix="kair_base_")
    arch = subprocess.run(["git", "-C", ROOT, "archive", rev, "kair_amd/csrc", "include"], check=True, capture_output=True).stdout
    subprocess.run(["tar", "-x", "-C", tmp], input=arch, check=True)
    csrc, inc = os.path.join(tmp, "kair_amd", "csrc"), os.path.join(tmp, "include")
    same_hdr = all(open(os.path.join(d, f), "rb").read() == open(os.path.join(dt, f), "rb").read()
                   for d, dt in ((csrc, B.CSRC), (inc, B.INCLUDE)) for f in os.listdir(d) if f.endswith(".h")
                   if os.path.exists(os.path.join(dt, f)))
    flags = [f if f not in (B.CSRC, B.INCLUDE) else (csrc if f == B.CSRC else inc) for f in B.FLAGS]
    objs = []
    for f in sorted(os.listdir(csrc)):
        if not f.endswith((".hip", ".cpp")):
            continue
        src, cur = os.path.join(csrc, f), os.path.join(B.CSRC, f)
        if same_hdr and os.path.exists(cur) and open(src, "rb").read() == open(cur, "rb").read():
            objs.append(os.path.join(B.OBJ, f + ".o"))
            continue
        obj = os.path.join(tmp, f + ".o")
        print("compiling", f, flush=True)
        subprocess.run([B.HIPCC, *flags, "-c", src, "-o", obj], check=True)
        objs.append(obj)
    out = os.path.join(ROOT, "kair_amd", "lib", "libkair_hip_base.so")
    subprocess.run([B.HIPCC, "-shared", "-fPIC", f"--offload-arch={B.ARCH}", *objs, "-o", out], check=True)
    print("built", out, "from", rev)


if __name__ == "__main__":
    main()
