#!/bin/bash
# 5x5 windows at 65,536 envs: the one-tick kernel over tile sizes and residency caps, and the
# fused tick + teacher, with compact records and with u8 rows (tools/step_probe.py).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-r04_sweep}; mkdir -p $OUT
CRAFT_COMPACT=1 timeout -k 10 200 python tools/step_probe.py --world craft_medium_12x12_w5 --ring 16 1 --obs-store 2 \
    --iters 100 --tiles 64 32 16 --caps 0 3 --teacher > $OUT/compact1.jsonl 2>$OUT/c1.err &&
CRAFT_COMPACT=0 timeout -k 10 200 python tools/step_probe.py --world craft_medium_12x12_w5 --ring 16 1 --obs-store 2 \
    --iters 100 --tiles 32 16 --caps 0 3 --teacher > $OUT/compact0.jsonl 2>$OUT/c0.err
cat $OUT/*.jsonl
