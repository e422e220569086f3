#!/bin/bash
# One gpurun call: with the teacher waves joining D + E, teacher-table reads always (1) against
# auto (2: off on a fresh ring slot), alternating: step_probe and the config 5 line.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=${TAG:-r04_share_tt}; OUT=gpurun_out/$T; mkdir -p $OUT
for pass in 1 2; do
  for f in 2 1; do
    CRAFT_TT_FUSED=$f timeout -k 10 120 python tools/step_probe.py --teacher --ring 16 1 \
        --obs-store 2 --iters 200 > "$OUT/teach_tt${f}_pass${pass}.jsonl" 2> "$OUT/teach.err" || exit $?
  done
done
TAG=$T/config5 REPS=2 STEPS=200 SPECS="auto=| on=CRAFT_TT_FUSED=1|" BENCH_ARGS="--workload teacher" bash tools/ab.sh || exit $?
for f in $OUT/*.jsonl; do echo "$(basename $f) $(cat $f | tr '\n' ' ')"; done
