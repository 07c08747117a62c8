#!/bin/bash
# Register / scratch / occupancy of the qp_step instantiations, with the library's own compile flags
# (developer tool, no GPU).  Extra arguments (e.g. -DQSP_MIN_WAVES=2) are appended.
cd "$(dirname "$0")/.." || exit 1
FLAGS=$(python3 -c "from uclv_qs_pushing_matlab_amd.build import FLAGS; print(' '.join(f for f in FLAGS if f not in ('-shared', '-fPIC')))")
/opt/rocm/bin/hipcc --offload-arch=gfx950 $FLAGS -I include "$@" \
  -c uclv_qs_pushing_matlab_amd/csrc/qsp_solver.hip -o /tmp/kres.o -Rpass-analysis=kernel-resource-usage 2>&1 |
  grep -A12 -E "Function Name: _ZN3qsp1(4qp_step|5sqp_loop)" | grep -E "Name|VGPRs:|AGPRs|Scratch|Occupancy" |
  sed -e 's/.*remark: *//' -e 's/ \[-Rpass.*//' | paste - - - - -
