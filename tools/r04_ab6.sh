#!/bin/bash
# One gpurun call: the GPU suite; the fused teacher with 4 / 8 stores in flight per tick-wave lane
# (libpsketch_craft_u8.so: -DCRAFT_T2_U=8), alternating; 7x7 compact records against u8 rows.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=${TAG:-r04_ab6}; OUT=gpurun_out/$T; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > "$OUT/pytest_gpu.log" 2>&1 || { tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
for pass in 1 2; do
  for spec in u4:libpsketch_craft.so u8:libpsketch_craft_u8.so; do
    IFS=: read name lib <<< "$spec"
    PSKETCH_CRAFT_LIB=psketch_amd/lib/$lib timeout -k 10 120 python tools/step_probe.py --teacher \
        --ring 16 1 --obs-store 2 --iters 200 > "$OUT/teach_${name}_pass${pass}.jsonl" 2> "$OUT/teach.err" || exit $?
  done
done
for c in 1 0; do
  CRAFT_COMPACT=$c timeout -k 10 200 python tools/step_probe.py --world craft_16x16_w7 --ring 16 1 --obs-store 2 \
      --iters 100 --tiles 0 16 32 > $OUT/w7_compact$c.jsonl 2> $OUT/w7.err || exit $?
done
for f in $OUT/*.jsonl; do echo "$(basename $f) $(cat $f)"; done
