#!/bin/bash
# Build an A/B variant library ppo-bipedalwalker_amd/libwk_<name>.so that recompiles only the
# listed sources with extra flags and links the rest from build/:
#   bash scripts/variant.sh <name> "<-D flags>" wk_ppo_mfma.hip [wk_ppo.hip ...]
set -eu
cd "$(dirname "$0")/../ppo-bipedalwalker_amd"
name=$1; flags=$2; shift 2
B=build_$name
rm -rf $B; mkdir -p $B; cp build/*.o $B/
for src in "$@"; do
  extra=""
  # (the physics variant is one object with every part: drop the three part objects)
  case $src in wk_physics.hip) extra="-fno-slp-vectorize -mllvm -amdgpu-sched-strategy=max-ilp"; rm -f $B/wk_physics.hip.p*.o;; esac
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off \
    -fhip-fp32-correctly-rounded-divide-sqrt -Wall -Wno-unused-function \
    -mllvm -amdgpu-use-amdgpu-trackers -I../include -Icsrc $extra $flags -x hip -c csrc/$src -o $B/$src.o
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o libwk_$name.so $B/*.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
echo built libwk_$name.so
