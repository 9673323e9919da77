#!/bin/bash
# VGPR / SGPR / LDS / scratch of the kernels in a built object whose name
# matches PATTERN, from the gfx950 code object's metadata (no recompile):
#   bash tools/kernel_regs.sh [OBJ] PATTERN
set -eu
OBJ=${2:+$1}; OBJ=${OBJ:-apex-camera-models_amd/build/acm.o}
PAT=${2:-$1}
B=/opt/rocm/lib/llvm/bin
T=$(mktemp -d)
$B/llvm-objcopy --dump-section=.hip_fatbin=$T/fat.bin "$OBJ" /dev/null
$B/clang-offload-bundler --unbundle --type=o --input=$T/fat.bin \
  --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output=$T/dev.co
$B/llvm-readelf --notes $T/dev.co > $T/notes.txt
python3 - "$T/notes.txt" "$PAT" <<'PY'
import re, sys
txt = open(sys.argv[1]).read()
for blk in txt.split("  - .agpr_count")[1:]:
    name = re.search(r"\.name:\s+(\S+)", blk).group(1)
    if not re.search(sys.argv[2], name):
        continue
    g = lambda k: (re.search(r"\." + k + r":\s+(\d+)", blk) or [None, "?"])[1]
    print(f"vgpr {g('vgpr_count'):>4} sgpr {g('sgpr_count'):>4} lds {g('group_segment_fixed_size'):>6} "
          f"scratch {g('private_segment_fixed_size'):>4} spill_v {g('vgpr_spill_count'):>3}  {name}")
PY
rm -rf $T
