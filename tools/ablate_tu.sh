#!/bin/bash
# Diagnostic: rebuild ONE translation unit with -D<flag> variants (CPU, here) and link each
# into psketch_amd/lib/abl_<name>.so beside the product objects; time with
# PSKETCH_CRAFT_LIB=psketch_amd/lib/abl_<name>.so on the GPU box.  Never the product.
#   tools/ablate_tu.sh craft_tick_teach noteach=CRAFT_ABL_NOTEACH nobfs=CRAFT_ABL_NOBFS
set -e
cd "$(dirname "$0")/.."
O=psketch_amd/lib/obj
TU=$1; shift
mkdir -p psketch_amd/lib/obj_abl
for spec in "$@"; do
  name=${spec%%=*}; defs=${spec#*=}
  flags=""; for d in ${defs//,/ }; do flags="$flags -D$d"; done
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC $flags -c psketch_amd/csrc/$TU.hip -o psketch_amd/lib/obj_abl/${TU}_$name.o &
done
wait
for spec in "$@"; do
  name=${spec%%=*}
  objs=""
  for o in $O/*.o; do
    if [ "$(basename $o .o)" = "$TU" ]; then objs="$objs psketch_amd/lib/obj_abl/${TU}_$name.o"; else objs="$objs $o"; fi
  done
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o psketch_amd/lib/abl_$name.so $objs
done
