#!/bin/bash
# Per-kernel VGPR/AGPR/SGPR/scratch/LDS of the gfx950 code object in pa_kernels.o
# (read from the AMDGPU metadata notes; no GPU needed).  Usage: profiles/kernel_resources.sh [regex]
set -euo pipefail
OBJ=${OBJ:-$(dirname "$0")/../cardiac-ablation-ecm2_amd/build/pa_kernels.o}
T=$(mktemp -d)
/opt/rocm/lib/llvm/bin/llvm-objcopy --dump-section=.hip_fatbin="$T/fat.bin" "$OBJ"
/opt/rocm/lib/llvm/bin/clang-offload-bundler --unbundle --type=o --input="$T/fat.bin" \
  --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output="$T/k.co"
/opt/rocm/lib/llvm/bin/llvm-readelf --notes "$T/k.co" | python3 -c '
import sys, re
pat = re.compile(sys.argv[1] if len(sys.argv) > 1 else ".")
cur = {}
rows = []
for line in sys.stdin:
    m = re.match(r"\s*-?\s*\.(\w+):\s*(.*)", line)
    if not m: continue
    k, v = m.group(1), m.group(2).strip()
    if k == "agpr_count": cur = {"agpr": v}
    elif k == "name": cur["name"] = v
    elif k == "vgpr_count": cur["vgpr"] = v
    elif k == "sgpr_count": cur["sgpr"] = v
    elif k == "private_segment_fixed_size": cur["scratch"] = v
    elif k == "group_segment_fixed_size": cur["lds"] = v
    elif k == "vgpr_spill_count":
        cur["vspill"] = v
        if "name" in cur: rows.append(dict(cur))
for r in rows:
    if pat.search(r.get("name", "")):
        print("%-90s v=%s a=%s s=%s scratch=%s lds=%s vspill=%s" % (r.get("name", "")[:90], r.get("vgpr"), r.get("agpr"), r.get("sgpr"), r.get("scratch"), r.get("lds"), r.get("vspill")))
' "${1:-.}"
rm -rf "$T"
