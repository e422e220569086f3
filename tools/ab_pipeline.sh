#!/bin/bash
# A/B of the rollout kernel's pipeline forms on one box: continuous (--rollout-chunk -1) vs
# one pipeline per tile (the default), alternating, at the driver's --steps 20
# and at 512 steps (16 launches of 32 ticks).  One JSON line per run in $OUT.
set -u
REPO="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$REPO/gpurun_out/${TAG:-ab}"
mkdir -p "$OUT"
cd "$REPO"
for rep in 1 2; do
  for mode in flat unit; do
    for steps in 20 512; do
      if [ $mode = unit ]; then CH=0; else CH=-1; fi
      timeout -k 10 120 python bench.py --steps $steps --warmup 5 --no-cpu-baseline --rollout-chunk $CH ${BENCH_ARGS:-} > "$OUT/$mode.$steps.$rep.json" 2> "$OUT/$mode.$steps.$rep.err"
      rc=$?; [ $rc -eq 0 ] || { echo "rc=$rc $mode $steps"; tail -3 "$OUT/$mode.$steps.$rep.err"; exit $rc; }
      python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], sys.argv[3], 'value %.3fG' % (d['value']/1e9), 'ms/step %.4f' % d['ms_per_step'], 'kernel_us %.1f' % d['roofline']['kernel_us'], 'frac %.3f' % d['roofline']['frac'])" "$OUT/$mode.$steps.$rep.json" $mode $steps
    done
  done
done
