#!/bin/bash
# A/B of library builds (tools/ablate_tu.sh variants) and rollout shapes, alternating on one
# box: each spec is "<lib or default>:<rollout threads>", run at STEPS.
#   SPECS="default:512 psketch_amd/lib/abl_wpe5.so:384" bash tools/ab_lib.sh
set -u
REPO="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$REPO/gpurun_out/${TAG:-ab_lib}"
mkdir -p "$OUT"
cd "$REPO"
for rep in $(seq 1 ${REPS:-2}); do
  i=0
  for spec in ${SPECS}; do
    lib=${spec%%:*}; nt=${spec##*:}; i=$((i + 1))
    for steps in ${STEPS:-20 512}; do
      if [ "$lib" = default ]; then L=""; else L="$lib"; fi
      PSKETCH_CRAFT_LIB=${L:-$REPO/psketch_amd/lib/libpsketch_craft.so} timeout -k 10 120 python bench.py --steps $steps --warmup 5 --no-cpu-baseline --rollout-threads $nt ${BENCH_ARGS:-} > "$OUT/$i.$steps.$rep.json" 2> "$OUT/$i.$steps.$rep.err"
      rc=$?; [ $rc -eq 0 ] || { echo "rc=$rc $spec $steps"; tail -3 "$OUT/$i.$steps.$rep.err"; exit $rc; }
      python -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[2], 'steps', sys.argv[3], 'value %.3fG' % (d['value']/1e9), 'kernel_us %.1f' % r['kernel_us'], 'frac %.3f' % r['frac'], r['kernel'])" "$OUT/$i.$steps.$rep.json" "$spec" $steps
    done
  done
done
