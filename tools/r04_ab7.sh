#!/bin/bash
# One gpurun call: the fused teacher's table reads (CRAFT_TT_FUSED auto / on / off) on the trainer
# line and on config 5's 16-slot ring, alternating (tools/ab.sh), then the GPU suite.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=${TAG:-r04_ab7}; OUT=gpurun_out/$T; mkdir -p $OUT
TAG=$T/trainer REPS=2 STEPS=5 SPECS="auto=| on=CRAFT_TT_FUSED=1| off=CRAFT_TT_FUSED=0|" BENCH_ARGS="--workload trainer" \
    bash tools/ab.sh || exit $?
TAG=$T/config5 REPS=2 STEPS=200 SPECS="auto=| on=CRAFT_TT_FUSED=1| off=CRAFT_TT_FUSED=0|" BENCH_ARGS="--workload teacher" \
    bash tools/ab.sh || exit $?
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > "$OUT/pytest_gpu.log" 2>&1 || { tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
