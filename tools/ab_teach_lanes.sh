#!/bin/bash
# Teacher lanes per query (1, 2, 4) for the fused tick + teacher kernel (CRAFT_TEACH_LANES) and
# the standalone teacher (CRAFT_TEACHER_LANES): the teacher parity tests under each, then
# tools/teacher_bench.py.  Stops at the first failing or abnormal step.
set -u
REPO="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$REPO/gpurun_out/${TAG:-abteach}"
mkdir -p "$OUT"
cd "$REPO"
for tl in ${LANES:-2 4 1}; do
  CRAFT_TEACH_LANES=$tl CRAFT_TEACHER_LANES=$tl timeout -k 10 300 python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread \
      tests/test_gpu_teach_fused.py tests/test_gpu_parity.py -k "teach" > "$OUT/pytest.$tl.log" 2>&1
  rc=$?; echo "lanes $tl pytest rc=$rc"; tail -2 "$OUT/pytest.$tl.log"; [ $rc -eq 0 ] || exit $rc
  CRAFT_TEACH_LANES=$tl CRAFT_TEACHER_LANES=$tl TEACHER_ENVS=${TEACHER_ENVS:-4096,32768,65536} timeout -k 10 200 python tools/teacher_bench.py > "$OUT/bench.$tl.json" 2> "$OUT/bench.$tl.err"
  rc=$?; echo "lanes $tl bench rc=$rc"; cat "$OUT/bench.$tl.json"; [ $rc -eq 0 ] || exit $rc
done
