#!/bin/bash
# One gpurun call: the GPU suite, then config 5 at w = 5 (the one-tile fused tick + teacher) at
# 32- and 64-env tiles with 2 and 4 teacher lanes per env (tools/step_probe.py --teacher).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=${TAG:-r04_w5teach}; OUT=gpurun_out/$T; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > "$OUT/pytest_gpu.log" 2>&1 || { tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
for pass in 1 2; do
  for tl in 4 2; do
    CRAFT_TEACH_LANES=$tl timeout -k 10 200 python tools/step_probe.py --world craft_medium_12x12_w5 --teacher \
        --ring 16 1 --obs-store 2 --iters 100 --tiles 32 64 > $OUT/tl${tl}_pass$pass.jsonl 2> $OUT/w5t.err || exit $?
  done
done
for f in $OUT/*.jsonl; do echo "$(basename $f) $(cat $f)"; done
