#!/bin/bash
# Round-4 A/B pass 2 (one gpurun call): the GPU suite, then bit-string compact records against
# u8-row staging for the 5x5 one-tick kernel, the fused teacher with and without table reads
# (CRAFT_TT_FUSED), and phase stamps of both.  Alternating passes; JSON lines in $OUT.
set -u
REPO="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$REPO/gpurun_out/${TAG:-r04_ab2}"
mkdir -p "$OUT"
cd "$REPO"
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > "$OUT/pytest_gpu.log" 2>&1 || { tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -2 "$OUT/pytest_gpu.log"
for pass in 1 2; do
  for c in 1 0; do
    CRAFT_COMPACT=$c timeout -k 10 120 python tools/step_probe.py --world craft_medium_12x12_w5 --ring 16 1 --obs-store 2 \
        --iters 100 > "$OUT/w5_compact${c}_pass${pass}.jsonl" 2> "$OUT/w5_compact${c}.err" || exit $?
  done
  for f in 0 1; do
    CRAFT_TT_FUSED=$f timeout -k 10 120 python tools/step_probe.py --teacher --ring 16 1 \
        --obs-store 2 --iters 200 > "$OUT/teach_fused${f}_pass${pass}.jsonl" 2> "$OUT/teach.err" || exit $?
  done
done
for c in 1 0; do
  CRAFT_COMPACT=$c timeout -k 10 120 python tools/phase_stamps.py craft_medium_12x12_w5 \
      > "$OUT/w5_stamps_compact${c}.jsonl" 2> "$OUT/w5_stamps_compact${c}.err" || exit $?
done
timeout -k 10 120 python tools/tick2_stamps.py > "$OUT/tick2_stamps.jsonl" 2> "$OUT/tick2_stamps.err" || exit $?
cat "$OUT"/*.jsonl
