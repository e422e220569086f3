#!/bin/bash
# A/B of the split rollout kernel's role-to-wave map (CRAFT_ROLE_MAP: 0 = scatter on hardware
# wave 1, 1 = scatter on wave 2; tools/hwid_probe.hip), alternating on one box, at the driver's
# --steps 20 and at 512 steps.  One JSON line per run in $OUT.
set -u
REPO="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$REPO/gpurun_out/${TAG:-ab_roles}"
mkdir -p "$OUT"
cd "$REPO"
for rep in 1 2 3; do
  for map in ${MAPS:-0 1}; do
    for steps in ${STEPS:-20 512}; do
      CRAFT_ROLE_MAP=$map timeout -k 10 120 python bench.py --steps $steps --warmup 5 --no-cpu-baseline ${BENCH_ARGS:-} > "$OUT/$map.$steps.$rep.json" 2> "$OUT/$map.$steps.$rep.err"
      rc=$?; [ $rc -eq 0 ] || { echo "rc=$rc map $map $steps"; tail -3 "$OUT/$map.$steps.$rep.err"; exit $rc; }
      python -c "import json,sys; d=json.load(open(sys.argv[1])); print('map', sys.argv[2], 'steps', sys.argv[3], 'value %.3fG' % (d['value']/1e9), 'ms/step %.4f' % d['ms_per_step'], 'kernel_us %.1f' % d['roofline']['kernel_us'], 'frac %.3f' % d['roofline']['frac'])" "$OUT/$map.$steps.$rep.json" $map $steps
    done
  done
done
