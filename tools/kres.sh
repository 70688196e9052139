#!/bin/bash
# Per-kernel register / LDS / scratch usage of a built object: tools/kres.sh kair_amd/build/gemm.hip.o [regex]
set -e
T=$(mktemp -d)
/opt/rocm/lib/llvm/bin/llvm-objcopy --dump-section=.hip_fatbin=$T/fat.bin "$1"
/opt/rocm/lib/llvm/bin/clang-offload-bundler --unbundle --type=o --input=$T/fat.bin \
  --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output=$T/k.co
/opt/rocm/lib/llvm/bin/llvm-readelf --notes $T/k.co | python3 -c '
import sys, re
txt = sys.stdin.read(); pat = sys.argv[1] if len(sys.argv) > 1 else ""
for blk in txt.split("- .agpr_count")[1:]:
    g = lambda k: (re.search(r"\.%s:\s+(\S+)" % k, blk) or [None, "?"])[1]
    name = g("name")
    if pat and not re.search(pat, name): continue
    print("%-90s vgpr %4s agpr %4s sgpr %3s lds %6s scratch %4s" % (name[:90], g("vgpr_count"), blk.split()[1] if blk.split() else "?",
          g("sgpr_count"), g("group_segment_fixed_size"), g("private_segment_fixed_size")))
' "${2:-}"
rm -rf $T
