#!/bin/bash
# Round-4 A/B pass (one gpurun call): the teacher table on/off and the tick2 wave-priority knob
# on config 5's fused tick + teacher; compact against u8-row staging for the 5x5 one-tick
# kernel; phase stamps of both (diagnostic libraries).  Alternating passes; JSON lines in $OUT.
set -u
REPO="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$REPO/gpurun_out/${TAG:-r04_ab}"
mkdir -p "$OUT"
cd "$REPO"
for pass in 1 2; do
  for tt in 1 0; do
    for p in 0 1; do
      CRAFT_TEACH_TABLE=$tt CRAFT_T2_PRIO=$p timeout -k 10 120 python tools/step_probe.py --teacher --ring 16 1 \
          --obs-store 2 --iters 200 > "$OUT/teach_tt${tt}_prio${p}_pass${pass}.jsonl" 2> "$OUT/teach.err" || exit $?
    done
  done
  for c in 1 0; do
    CRAFT_COMPACT=$c timeout -k 10 120 python tools/step_probe.py --world craft_medium_12x12_w5 --ring 16 1 --obs-store 2 \
        --iters 100 > "$OUT/w5_compact${c}_pass${pass}.jsonl" 2> "$OUT/w5_compact${c}.err" || exit $?
  done
done
for c in 1 0; do
  CRAFT_COMPACT=$c timeout -k 10 120 python tools/phase_stamps.py craft_medium_12x12_w5 \
      > "$OUT/w5_stamps_compact${c}.jsonl" 2> "$OUT/w5_stamps_compact${c}.err" || exit $?
done
for tt in 1 0; do
  CRAFT_TEACH_TABLE=$tt timeout -k 10 120 python tools/tick2_stamps.py > "$OUT/tick2_stamps_tt${tt}.jsonl" \
      2> "$OUT/tick2_stamps.err" || exit $?
done
timeout -k 10 120 python tools/tick2_stamps.py --lib libpsketch_craft_diag_c.so --ring 16 \
    > "$OUT/tick2_stamps_c.jsonl" 2> "$OUT/tick2_stamps_c.err" || exit $?
cat "$OUT"/*.jsonl
