#!/bin/bash
# The two-tile tick kernel (craft_tick2.h) against the one-tile kernel: the GPU tests on the
# default build, then tools/teacher_bench.py (tick, teacher, fused tick + teacher) under each.
set -u
REPO="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$REPO/gpurun_out/${TAG:-abtick2}"
mkdir -p "$OUT"
cd "$REPO"
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread tests > "$OUT/pytest.log" 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -5 "$OUT/pytest.log"; [ $rc -eq 0 ] || exit $rc
fi
for rep in 1 2; do
  for cfg in "tick2:TEACH_KERNEL=2" "tick2_tl4:TEACH_KERNEL=2,CRAFT_TEACH_LANES=4" "one_tile:TEACH_KERNEL=1"; do
    name=${cfg%%:*}; envs=""; [ "$name" != "$cfg" ] && envs=${cfg#*:}
    env ${envs//,/ } TEACHER_ENVS=${TEACHER_ENVS:-65536} timeout -k 10 200 python tools/teacher_bench.py > "$OUT/$name.$rep.json" 2> "$OUT/$name.$rep.err"
    rc=$?; [ $rc -eq 0 ] || { echo "$name rc=$rc"; tail -3 "$OUT/$name.$rep.err"; exit $rc; }
    python -c "import json,sys; d=list(json.load(open(sys.argv[1])).values())[0]; print(sys.argv[2], 'tick %.2f teacher %.2f fused %.2f us' % (d['tick_us'], d['teacher_us'], d['step_teach_us']))" "$OUT/$name.$rep.json" $name
  done
done
