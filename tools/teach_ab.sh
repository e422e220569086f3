#!/bin/bash
# Config-5 bench forms on one box: the fused tick + teacher launch (4 or 1 teacher
# lanes per env) against craft_teacher + craft_step, alternating.  One JSON line per run.
set -u
REPO="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$REPO/gpurun_out/${TAG:-teach}"
mkdir -p "$OUT"
cd "$REPO"
for rep in 1 2; do
  for mode in fused4 fused1 separate; do
    unset CRAFT_TEACH_LANES
    tm=fused
    case $mode in fused1) export CRAFT_TEACH_LANES=1;; separate) tm=separate;; esac
    timeout -k 10 120 python bench.py --workload teacher --teacher-mode $tm --steps ${STEPS:-200} --warmup 10 --no-cpu-baseline > "$OUT/$mode.$rep.json" 2> "$OUT/$mode.$rep.err"
    rc=$?; [ $rc -eq 0 ] || { echo "rc=$rc $mode"; tail -3 "$OUT/$mode.$rep.err"; exit $rc; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], 'value %.3fG' % (d['value']/1e9), 'us/step %.2f' % (1e3*d['ms_per_step']), 'kernel_us %.1f' % d['roofline']['kernel_us'], 'frac %.3f' % d['roofline']['frac'])" "$OUT/$mode.$rep.json" $mode
  done
done
