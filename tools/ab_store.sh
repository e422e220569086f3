#!/bin/bash
# A/B of the observation store cache policy for the rollout kernel (0 write-back, 1 nontemporal,
# 2 write-through), alternating, at the driver's --steps 20 and at 512 steps.
set -u
REPO="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$REPO/gpurun_out/${TAG:-abstore}"
mkdir -p "$OUT"
cd "$REPO"
for rep in 1 2; do
  for pol in 0 1 2; do
    for steps in 20 512; do
      timeout -k 10 120 python bench.py --steps $steps --warmup 5 --no-cpu-baseline --obs-store $pol ${BENCH_ARGS:-} > "$OUT/$pol.$steps.$rep.json" 2> "$OUT/$pol.$steps.$rep.err"
      rc=$?; [ $rc -eq 0 ] || { echo "rc=$rc $pol $steps"; tail -3 "$OUT/$pol.$steps.$rep.err"; exit $rc; }
      python -c "import json,sys; d=json.load(open(sys.argv[1])); print('policy', sys.argv[2], sys.argv[3], 'value %.3fG' % (d['value']/1e9), 'kernel_us %.1f' % d['roofline']['kernel_us'])" "$OUT/$pol.$steps.$rep.json" $pol $steps
    done
  done
done
