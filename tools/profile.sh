#!/bin/bash
# rocprofv3 evidence for bench lines: for each config line "name|bench.py args|steps", a
# kernel-trace --stats run of the bench (its JSON line kept beside the trace), then separate
# FETCH_SIZE and WRITE_SIZE passes of the same command without warmup or CPU baseline (counters
# are never combined with another trace domain).  Summarise with tools/pmc_summary.py.
#   CONFIGS=$'headline||20\nk1|--ticks-per-launch 1|200' TAG=prof bash tools/profile.sh
set -u
REPO="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$REPO/gpurun_out/${TAG:-prof}"
mkdir -p "$OUT"
cd /tmp
export TMPDIR=/tmp
while IFS='|' read -r name args steps; do
  [ -n "$name" ] || continue
  d="$OUT/$name"; mkdir -p "$d"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$d/trace" -o run -- \
      python3 "$REPO/bench.py" $args --steps $steps --warmup ${WARMUP:-5} --cpu-seconds ${CPU_SECONDS:-3} --no-kernel-profiler \
      < /dev/null > "$d/bench.json" 2> "$d/trace.err"
  rc=$?; echo "$name trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 300 rocprofv3 --pmc $C --output-format csv -d "$d/pmc_$C" -o run -- \
        python3 "$REPO/bench.py" $args --steps $steps --warmup 0 --no-cpu-baseline --no-kernel-profiler \
        < /dev/null > "$d/pmc_$C.json" 2> "$d/pmc_$C.err"
    rc=$?; echo "$name pmc $C rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
done <<< "$CONFIGS"
