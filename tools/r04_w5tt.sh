#!/bin/bash
# One gpurun call: config 5 at w = 5 with teacher-table reads always on against auto (off on a
# fresh ring slot), alternating (tools/step_probe.py --teacher).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=${TAG:-r04_w5tt}; OUT=gpurun_out/$T; mkdir -p $OUT
for pass in 1 2; do
  for f in 2 1; do
    CRAFT_TT_FUSED=$f timeout -k 10 200 python tools/step_probe.py --world craft_medium_12x12_w5 --teacher \
        --ring 16 1 --obs-store 2 --iters 100 > $OUT/tt${f}_pass$pass.jsonl 2> $OUT/tt.err || exit $?
  done
done
for f in $OUT/*.jsonl; do echo "$(basename $f) $(cat $f)"; done
