#!/bin/bash
# A/B of bench.py variants, alternating on one box, REPS passes, one JSON line per run in $OUT.
# Each spec is "<name>=<env assignments separated by ','>|<extra bench.py args separated by ','>":
#   SPECS="base=| kernarg=HIP_FORCE_DEV_KERNARG=1| wpe5=PSKETCH_CRAFT_LIB=psketch_amd/lib/abl.so|--rollout-threads,384" \
#     STEPS="20 512" bash tools/ab.sh
# (round 2's knob and build A/Bs ran through this; their results are the table in DESIGN.md)
set -u
REPO="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$REPO/gpurun_out/${TAG:-ab}"
mkdir -p "$OUT"
cd "$REPO"
for rep in $(seq 1 ${REPS:-2}); do
  for spec in ${SPECS}; do
    name=${spec%%=*}; rest=${spec#*=}; envs=${rest%%|*}; args=${rest#*|}
    for steps in ${STEPS:-20 512}; do
      env ${envs//,/ } timeout -k 10 120 python bench.py --steps $steps --warmup 5 --no-cpu-baseline ${args//,/ } ${BENCH_ARGS:-} > "$OUT/$name.$steps.$rep.json" 2> "$OUT/$name.$steps.$rep.err"
      rc=$?; [ $rc -eq 0 ] || { echo "rc=$rc $name $steps"; tail -3 "$OUT/$name.$steps.$rep.err"; exit $rc; }
      python -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[2], 'steps', sys.argv[3], 'value %.3fG' % (d['value']/1e9), 'kernel_us %.1f' % r['kernel_us'], 'frac %.3f' % r['frac'], r['kernel'])" "$OUT/$name.$steps.$rep.json" "$name" $steps
    done
  done
done
