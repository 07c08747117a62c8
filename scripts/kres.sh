#!/bin/bash
# Register / scratch / occupancy of the qp_step instantiations (developer tool, no GPU)
cd "$(dirname "$0")/.." && /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include $@ \
  -c uclv_qs_pushing_matlab_amd/csrc/qsp_solver.hip -o /tmp/kres.o -Rpass-analysis=kernel-resource-usage 2>&1 |
  grep -A12 -E "Function Name: _ZN3qsp1(4qp_step|5sqp_loop)" | grep -E "Name|VGPRs:|AGPRs|Scratch|Occupancy" |
  sed -e 's/.*remark: *//' -e 's/ \[-Rpass.*//' | paste - - - - -
