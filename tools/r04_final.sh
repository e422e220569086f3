#!/bin/bash
# Round-4 final tree, one gpurun call: smoke, the GPU suite, every bench line
# (tools/bench_lines.sh), then rocprof kernel-trace + FETCH_SIZE / WRITE_SIZE passes of the lines
# whose kernels changed last (config 5, the trainer, config 5 at w = 5).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=${TAG:-r04_final}; OUT=gpurun_out/$T; mkdir -p $OUT
timeout -k 10 240 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { tail -20 "$OUT/smoke.log"; exit 1; }
tail -1 "$OUT/smoke.log"
timeout -k 10 300 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread \
    > "$OUT/pytest_gpu.log" 2>&1; rc=$?; tail -1 "$OUT/pytest_gpu.log"; [ $rc -le 1 ] || exit $rc
TAG=$T/lines CPU_SECONDS=${CPU_SECONDS:-8} bash tools/bench_lines.sh || exit $?
CONFIGS=$'config5|--workload teacher|200\ntrainer|--workload trainer|5\nconfig5_w5|--world craft_medium_12x12_w5 --workload teacher|100' \
  TAG=$T/prof CPU_SECONDS=2 bash tools/profile.sh || exit $?
