#!/bin/bash
# Per-launch fixed cost of the rollout kernel: kernel time per launch at 20 and 32 ticks for
# 1, 2 and 4 tiles per workgroup (16384 / 32768 / 65536 envs; 512 workgroups of 32-env tiles).
set -u
REPO="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$REPO/gpurun_out/${TAG:-fixed}"
mkdir -p "$OUT"
cd "$REPO"
for n in 16384 32768 65536; do
  for k in 20 32; do
    timeout -k 10 120 python bench.py --envs $n --steps $((k * 8)) --warmup $k --ticks-per-launch $k --no-cpu-baseline ${BENCH_ARGS:-} > "$OUT/$n.$k.json" 2> "$OUT/$n.$k.err"
    rc=$?; [ $rc -eq 0 ] || { echo "rc=$rc $n $k"; tail -3 "$OUT/$n.$k.err"; exit $rc; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[2], sys.argv[3], 'kernel %.1f us/launch  %.2f us/tick  frac %.3f' % (r['kernel_us'], r['kernel_us']/r['ticks_per_launch'], r['frac']))" "$OUT/$n.$k.json" $n $k
  done
done
