#!/bin/bash
# One gpurun call: the one-tick kernel with 4 / 8 / 16 stores in flight per lane in E
# (libpsketch_craft_tu{8,16}.so: -DCRAFT_TILE_U), w = 3 and w = 5, alternating (step_probe).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=${TAG:-r04_tileu}; OUT=gpurun_out/$T; mkdir -p $OUT
for pass in 1 2; do
  for spec in u4:libpsketch_craft.so u8:libpsketch_craft_tu8.so u16:libpsketch_craft_tu16.so; do
    IFS=: read name lib <<< "$spec"
    for w in craft_medium_12x12 craft_medium_12x12_w5; do
      PSKETCH_CRAFT_LIB=psketch_amd/lib/$lib timeout -k 10 120 python tools/step_probe.py --world $w --ring 16 1 \
          --obs-store 2 --iters 100 > "$OUT/${name}_${w}_pass${pass}.jsonl" 2> "$OUT/u.err" || exit $?
    done
  done
done
for f in $OUT/*.jsonl; do echo "$(basename $f) $(cat $f | tr '\n' ' ')"; done
