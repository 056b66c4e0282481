#!/bin/bash
# register / spill metadata of every step-kernel instantiation in a built library: bash tools/kmeta.sh LIB.so
set -e
T=$(mktemp -d)
/opt/rocm/lib/llvm/bin/llvm-objcopy --dump-section=.hip_fatbin=$T/fb.bin "$1"
/opt/rocm/lib/llvm/bin/clang-offload-bundler --unbundle --type=o --input=$T/fb.bin --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output=$T/dev.o
/opt/rocm/lib/llvm/bin/llvm-readelf --notes $T/dev.o | python3 -c '
import sys, re
cur = {}; out = []
for l in sys.stdin:
    m = re.match(r"\s*-?\s*\.(\w+):\s+(\S+)", l)
    if not m: continue
    k, v = m.groups()
    if k == "agpr_count" and cur: out.append(cur); cur = {}
    cur[k] = v
out.append(cur)
for b in out:
    if "step_kernel" in b.get("name", ""):
        print(b["name"][:48], "vgpr", b.get("vgpr_count"), "agpr", b.get("agpr_count"), "spill", b.get("vgpr_spill_count"), "scratch", b.get("private_segment_fixed_size"), "lds", b.get("group_segment_fixed_size"))
'
/opt/rocm/lib/llvm/bin/llvm-readelf -S $T/dev.o | grep " .text" | awk '{print "text bytes", strtonum("0x"$6)}'
rm -rf $T
