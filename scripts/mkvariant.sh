#!/bin/bash
# Build variants/NAME.so from the current sources with extra compiler flags (developer tool):
#   bash scripts/mkvariant.sh NAME -DFOO=1 ...
set -e
cd "$(dirname "$0")/.."
name=$1; shift
mkdir -p variants
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC -shared -mllvm -greedy-regclass-priority-trumps-globalness -mllvm -amdgpu-mfma-vgpr-form -I include "$@" \
  uclv_qs_pushing_matlab_amd/csrc/qsp_solver.hip uclv_qs_pushing_matlab_amd/csrc/qsp_capi.hip -o variants/$name.so
echo "variants/$name.so"
