#!/bin/bash
# gfx950 listing + loop opcode histogram of one dynamics_group_kernel instantiation (the headline
# dynamics_group_kernel<4, kModeStep, SED, false, 1> by default), with optional -D defines.
#   usage: bash tools/isa_dyn.sh <out dir> [-DNAME=val ...]
#   INST="<G>, kModeStepNR, 0, false, 4" picks another instantiation.
set -e -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
OUT=$1; shift
mkdir -p "$OUT"
INST=${INST:-"4, kModeStep, 0, false, 1"}
cat > "$OUT/dyn_inst.hip" <<EOF
#include "lbsim_internal.h"
#include "lbsim_dyn_group.h"
namespace lbk {
template __global__ void dynamics_group_kernel<$INST>(DevState, SimParams, const void*, int,
                                                     int32_t*, const uint8_t*);
}
EOF
/opt/rocm/bin/hipcc -O3 -std=c++17 -ffp-contract=off --offload-arch=gfx950 --cuda-device-only -S \
  -I"$R/marllb_amd/csrc" -I"$R/include" "$@" -o "$OUT/dyn_inst.s" "$OUT/dyn_inst.hip" 2>/dev/null
name=$(grep -o '^_Z[^ :]*' "$OUT/dyn_inst.s" | head -1)
grep -E '\.(vgpr|sgpr)_(count|spill_count):|private_segment_fixed_size|group_segment_fixed_size' \
  "$OUT/dyn_inst.s" > "$OUT/resources.txt"
python "$R/tools/isa_hist.py" "$OUT/dyn_inst.s" "$name" --out "$OUT" > /dev/null
rm -f "$OUT/dyn_inst.s"
cat "$OUT/resources.txt"
