#!/bin/bash
# Per-kernel register / spill / LDS usage of one source file (compiler view), filtered by a pattern.
#   tools/kres.sh pnp-pds_amd/csrc/ops.hip blur_rb
f=$1; pat=${2:-.}
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -mllvm -pragma-unroll-threshold=200000 $KFLAGS -c "$f" -o /tmp/kres.o \
  -Rpass-analysis=kernel-resource-usage 2>&1 | sed -n 's/.*remark: *//p' | awk -v pat="$pat" '
  /^Function Name:/ {name=$3; show = (name ~ pat)}
  show && /^VGPRs:/ {v=$2} show && /^AGPRs:/ {a=$2} show && /^VGPRs Spill:/ {sp=$3}
  show && /^Occupancy/ {o=$NF}
  show && /^LDS Size/ {printf "%-90s vgpr=%s agpr=%s spill=%s occ=%s lds=%s\n", substr(name,1,90), v, a, sp, o, $NF}'
