#!/bin/bash
# 5x5 one-tick A/B (one gpurun call): the compact and parity tests, compact records against u8
# rows (alternating passes), phase stamps of both.  JSON lines in $OUT.
set -u
REPO="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$REPO/gpurun_out/${TAG:-r04_w5}"
mkdir -p "$OUT"
cd "$REPO"
timeout -k 10 300 python -u -m pytest tests/test_gpu_compact.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 \
    --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -2 "$OUT/pytest_gpu.log"
for pass in 1 2; do
  for c in 1 0; do
    CRAFT_COMPACT=$c timeout -k 10 120 python tools/step_probe.py --world craft_medium_12x12_w5 --ring 16 1 --obs-store 2 \
        --iters 100 > "$OUT/w5_compact${c}_pass${pass}.jsonl" 2> "$OUT/w5_compact${c}.err" || exit $?
  done
done
for c in 1 0; do
  CRAFT_COMPACT=$c timeout -k 10 120 python tools/phase_stamps.py craft_medium_12x12_w5 \
      > "$OUT/w5_stamps_compact${c}.jsonl" 2> "$OUT/w5_stamps_compact${c}.err" || exit $?
done
for f in "$OUT"/*.jsonl; do echo "$(basename $f) $(cat $f)"; done
