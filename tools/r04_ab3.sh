#!/bin/bash
# One gpurun call: the 5x5 sweep (tools/w5_sweep.sh) and the fused teacher's walk / dense-pass
# stamps (CRAFT_STAMPS_T) with and without teacher-table reads.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-r04_ab3}; mkdir -p $OUT
TAG=${TAG:-r04_ab3} bash tools/w5_sweep.sh || exit $?
for f in 0 1; do
  CRAFT_TT_FUSED=$f timeout -k 10 120 python tools/tick2_stamps.py --lib libpsketch_craft_diag_t.so \
      > $OUT/t2t_fused$f.jsonl 2> $OUT/t2t.err || exit $?
done
for f in $OUT/t2t*.jsonl; do echo "$(basename $f) $(cat $f)"; done
