#!/bin/bash
# One gpurun call: the GPU suite; the K-tick launch with and without the readlane recipe loop
# (libpsketch_craft_base.so = the previous commit's library), alternating; the fused teacher
# (base / new, with and without teacher-table reads); its walk / dense-pass stamps; the 5x5 sweep.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=${TAG:-r04_ab5}; OUT=gpurun_out/$T; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > "$OUT/pytest_gpu.log" 2>&1 || { tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
TAG=$T/rollout REPS=3 SPECS="base=PSKETCH_CRAFT_LIB=psketch_amd/lib/libpsketch_craft_base.so| new=|" bash tools/ab.sh || exit $?
for pass in 1 2; do
  for spec in base0:libpsketch_craft_base.so:0 new0:libpsketch_craft.so:0 new1:libpsketch_craft.so:1; do
    IFS=: read name lib f <<< "$spec"
    PSKETCH_CRAFT_LIB=psketch_amd/lib/$lib CRAFT_TT_FUSED=$f timeout -k 10 120 python tools/step_probe.py --teacher \
        --ring 16 1 --obs-store 2 --iters 200 > "$OUT/teach_${name}_pass${pass}.jsonl" 2> "$OUT/teach.err" || exit $?
  done
done
for f in 0 1; do
  CRAFT_TT_FUSED=$f timeout -k 10 120 python tools/tick2_stamps.py --lib libpsketch_craft_diag_t.so \
      > $OUT/t2t_fused$f.jsonl 2> $OUT/t2t.err || exit $?
done
TAG=$T bash tools/w5_sweep.sh > /dev/null || exit $?
for f in $OUT/*.jsonl; do echo "$(basename $f) $(cat $f)"; done
