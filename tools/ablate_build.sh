#!/bin/bash
# Diagnostic: build the library with -D<flag> variants (CPU, here) into psketch_amd/lib/abl_<name>.so;
# run tools/producer_bench.py against one with PSKETCH_CRAFT_LIB=... on the GPU box.
set -e
cd "$(dirname "$0")/.."
O=psketch_amd/lib/obj
mkdir -p psketch_amd/lib/obj_abl
for spec in "$@"; do
  name=${spec%%=*}; defs=${spec#*=}
  flags=""; for d in ${defs//,/ }; do flags="$flags -D$d"; done
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC $flags -c psketch_amd/csrc/craft_rollout_w3.hip -o psketch_amd/lib/obj_abl/w3_$name.o &
done
wait
for spec in "$@"; do
  name=${spec%%=*}
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o psketch_amd/lib/abl_$name.so $O/craft_sim.o $O/craft_tile.o psketch_amd/lib/obj_abl/w3_$name.o $O/craft_rollout_w5.o $O/craft_rollout_w7.o $O/craft_teacher.o $O/craft_scenarios.o $O/scenario_gen.o
done
