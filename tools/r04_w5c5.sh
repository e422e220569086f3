#!/bin/bash
# One gpurun call: config 5 at w = 5 (the one-tile fused tick + teacher), its bench line and its
# rocprof kernel-trace + FETCH_SIZE / WRITE_SIZE passes (tools/profile.sh).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=${TAG:-r04_w5c5}; OUT=gpurun_out/$T; mkdir -p $OUT
timeout -k 10 300 python bench.py --world craft_medium_12x12_w5 --workload teacher --steps 100 --warmup 10 \
    --cpu-seconds 8 > $OUT/config5_w5.json 2> $OUT/config5_w5.err || { tail -5 $OUT/config5_w5.err; exit 1; }
CONFIGS=$'config5_w5|--world craft_medium_12x12_w5 --workload teacher|100' TAG=$T CPU_SECONDS=2 bash tools/profile.sh
