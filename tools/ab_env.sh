#!/bin/bash
# A/B of a library knob read from the environment (VAR, values VALUES), alternating on one box,
# bench.py at STEPS (default: the driver's 20 and 512).  One JSON line per run in $OUT.
#   VAR=CRAFT_TEACH_LANES VALUES="2 4" STEPS=200 BENCH_ARGS="--workload teacher" bash tools/ab_env.sh
# (round 2 also ran it on a producer-priority knob since removed: profiles/r02/ab_prio/)
set -u
REPO="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$REPO/gpurun_out/${TAG:-ab_env}"
mkdir -p "$OUT"
cd "$REPO"
for rep in $(seq 1 ${REPS:-3}); do
  for val in ${VALUES}; do
    for steps in ${STEPS:-20 512}; do
      env "$VAR=$val" timeout -k 10 120 python bench.py --steps $steps --warmup 5 --no-cpu-baseline ${BENCH_ARGS:-} > "$OUT/$val.$steps.$rep.json" 2> "$OUT/$val.$steps.$rep.err"
      rc=$?; [ $rc -eq 0 ] || { echo "rc=$rc $VAR=$val $steps"; tail -3 "$OUT/$val.$steps.$rep.err"; exit $rc; }
      python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], 'steps', sys.argv[3], 'value %.3fG' % (d['value']/1e9), 'ms/step %.4f' % d['ms_per_step'], 'kernel_us %.1f' % d['roofline']['kernel_us'], 'frac %.3f' % d['roofline']['frac'])" "$OUT/$val.$steps.$rep.json" "$VAR=$val" $steps
    done
  done
done
