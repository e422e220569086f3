#!/bin/bash
# One gpurun call: tick2 phase stamps on the final tree (CRAFT_STAMPS, then CRAFT_STAMPS_T),
# both buffers.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=${TAG:-r04_stamps_final}; OUT=gpurun_out/$T; mkdir -p $OUT
timeout -k 10 120 python tools/tick2_stamps.py > $OUT/t2.jsonl 2> $OUT/t2.err || exit $?
timeout -k 10 120 python tools/tick2_stamps.py --lib libpsketch_craft_diag_t.so > $OUT/t2t.jsonl 2> $OUT/t2t.err || exit $?
cat $OUT/*.jsonl
