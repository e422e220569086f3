#!/bin/bash
# bench.py per observation format (f32 = the metric's line; bf16 / u8 hold the same exact
# values in 2 / 1 bytes), each with a 1.7 GB ring so the bytes written between two visits of
# a slot (~420 MB) stay above the 256 MB Infinity Cache.  One JSON line per run in $OUT.
set -u
REPO="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$REPO/gpurun_out/${TAG:-obs_formats}"
mkdir -p "$OUT"
cd "$REPO"
for rep in 1 2; do
  for fr in f32:16 bf16:32 u8:64; do
    f=${fr%%:*}; R=${fr##*:}
    for steps in 20 512; do
      timeout -k 10 120 python bench.py --steps $steps --warmup 5 --no-cpu-baseline --obs-format $f --ring $R > "$OUT/$f.$steps.$rep.json" 2> "$OUT/$f.$steps.$rep.err"
      rc=$?; [ $rc -eq 0 ] || { echo "rc=$rc $f $steps"; tail -3 "$OUT/$f.$steps.$rep.err"; exit $rc; }
      python -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[2], 'steps', sys.argv[3], 'value %.3fG' % (d['value']/1e9), 'ms/step %.4f' % d['ms_per_step'], 'kernel_us %.1f' % r['kernel_us'], 'B/step %d' % r['bytes_per_env_step'], 'frac %.3f' % r['frac'])" "$OUT/$f.$steps.$rep.json" $f $steps
    done
  done
done
