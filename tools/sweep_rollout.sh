#!/bin/bash
# The rollout kernel's launch shapes at the driver's command (--steps 20 --warmup 5), two
# alternating passes: tile {16, 32} x threads {384, 512} x pipeline {per unit, continuous}.
set -u
REPO="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$REPO/gpurun_out/${TAG:-sweep_rollout}"
mkdir -p "$OUT"
cd "$REPO"
for rep in 1 2; do
  for tile in 32 16; do
    for thr in 512 384; do
      for chunk in 0 -1; do
        name="t${tile}_n${thr}_c${chunk}"
        timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --tile $tile --rollout-threads $thr --rollout-chunk $chunk > "$OUT/$name.$rep.json" 2> "$OUT/$name.$rep.err"
        rc=$?; [ $rc -eq 0 ] || { echo "rc=$rc $name"; tail -3 "$OUT/$name.$rep.err"; exit $rc; }
        python -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[2], 'value %.3fG kernel %.1f us %s' % (d['value']/1e9, r['kernel_us'], r['kernel']))" "$OUT/$name.$rep.json" $name
      done
    done
  done
done
