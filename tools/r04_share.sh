#!/bin/bash
# One gpurun call: the GPU suite; tick2 with the teacher waves joining D + E (tick2_share) against
# the previous commit's library (libpsketch_craft_base.so), alternating: step_probe at both
# buffers, the trainer line and config 5.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=${TAG:-r04_share}; OUT=gpurun_out/$T; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > "$OUT/pytest_gpu.log" 2>&1 || { tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
for pass in 1 2; do
  for spec in base:libpsketch_craft_base.so share:libpsketch_craft.so; do
    IFS=: read name lib <<< "$spec"
    PSKETCH_CRAFT_LIB=psketch_amd/lib/$lib timeout -k 10 120 python tools/step_probe.py --teacher --ring 16 1 \
        --obs-store 2 --iters 200 > "$OUT/teach_${name}_pass${pass}.jsonl" 2> "$OUT/teach.err" || exit $?
  done
done
TAG=$T/trainer REPS=2 STEPS=5 SPECS="base=PSKETCH_CRAFT_LIB=psketch_amd/lib/libpsketch_craft_base.so| share=|" \
    BENCH_ARGS="--workload trainer" bash tools/ab.sh || exit $?
TAG=$T/config5 REPS=2 STEPS=200 SPECS="base=PSKETCH_CRAFT_LIB=psketch_amd/lib/libpsketch_craft_base.so| share=|" \
    BENCH_ARGS="--workload teacher" bash tools/ab.sh || exit $?
for f in $OUT/*.jsonl; do echo "$(basename $f) $(cat $f | tr '\n' ' ')"; done
