# Per-kernel VGPR / AGPR / spill / LDS / occupancy of a .hip file for gfx950.
# Usage: bash tools/kernel_resources.sh <file.hip> [name-filter]
f=$1; filt=${2:-.}
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 -I$(dirname $f) $EXTRA -c $f -o /tmp/_kr.o \
  -Rpass-analysis=kernel-resource-usage 2>&1 | sed -n 's/.*remark: *//p' | awk -v filt="$filt" '
  /Function Name:/ {name=$3}
  /^ *VGPRs:/ {v=$2}
  /^ *AGPRs:/ {ag=$2}
  /VGPRs Spill:/ {sp=$3}
  /Occupancy/ {occ=$3}
  /LDS Size/ {lds=$4; if (name ~ filt) printf "%-66s vgpr=%-4s agpr=%-4s spill=%-4s lds=%-6s occ=%s\n", substr(name,1,66), v, ag, sp, lds, occ}'
