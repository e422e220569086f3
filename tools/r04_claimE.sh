#!/bin/bash
# One gpurun call: the GPU suite; the one-tile fused kernel with its E in claimed blocks that the
# teacher waves join, against the previous commit's library (libpsketch_craft_base.so),
# alternating: step_probe --teacher at w = 3 (its teach_tile column) and w = 5, config 5 at w = 5.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=${TAG:-r04_claimE}; OUT=gpurun_out/$T; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > "$OUT/pytest_gpu.log" 2>&1 || { tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
for pass in 1 2; do
  for spec in base:libpsketch_craft_base.so claim:libpsketch_craft.so; do
    IFS=: read name lib <<< "$spec"
    for w in craft_medium_12x12 craft_medium_12x12_w5; do
      PSKETCH_CRAFT_LIB=psketch_amd/lib/$lib timeout -k 10 150 python tools/step_probe.py --world $w --teacher \
          --ring 16 1 --obs-store 2 --iters 100 > "$OUT/${name}_${w}_pass${pass}.jsonl" 2> "$OUT/p.err" || exit $?
    done
  done
done
TAG=$T/config5_w5 REPS=2 STEPS=100 SPECS="base=PSKETCH_CRAFT_LIB=psketch_amd/lib/libpsketch_craft_base.so| claim=|" \
    BENCH_ARGS="--workload teacher --world craft_medium_12x12_w5" bash tools/ab.sh || exit $?
for f in $OUT/*.jsonl; do echo "$(basename $f) $(cat $f | tr '\n' ' ')"; done
