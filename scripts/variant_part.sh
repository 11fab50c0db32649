#!/bin/bash
# Build an A/B variant library ppo-bipedalwalker_amd/libwk_<name>.so that recompiles one part
# of the physics source (WK_PHYS_PART, see wk_physics.hip) with extra flags and links the rest
# from build/:   bash scripts/variant_part.sh <name> "<flags>" <part>
set -eu
cd "$(dirname "$0")/../ppo-bipedalwalker_amd"
name=$1; flags=$2; part=$3
B=build_$name
rm -rf $B; mkdir -p $B; cp build/*.o $B/
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off \
  -fhip-fp32-correctly-rounded-divide-sqrt -Wall -Wno-unused-function \
  -mllvm -amdgpu-use-amdgpu-trackers -I../include -Icsrc -fno-slp-vectorize \
  -mllvm -amdgpu-sched-strategy=max-ilp $flags -DWK_PHYS_PART=$part -x hip -c csrc/wk_physics.hip \
  -o $B/wk_physics.hip.p$part.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o libwk_$name.so $B/*.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
echo built libwk_$name.so
