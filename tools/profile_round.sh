#!/bin/bash
# rocprofv3 evidence for one round: kernel-trace stats of the bench command, then
# separate PMC passes (counters never combined with other trace domains).
set -u
REPO="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$REPO/gpurun_out/${TAG:-prof}"
mkdir -p "$OUT"
cd /tmp
export TMPDIR=/tmp
ARGS="--steps ${STEPS:-1024} --warmup 64 ${BENCH_ARGS:-}"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
    python3 "$REPO/bench.py" $ARGS > "$OUT/trace_bench.json" 2> "$OUT/trace.err"
rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $C --output-format csv -d "$OUT/pmc_$C" -o run -- \
      python3 "$REPO/bench.py" --steps 128 --warmup 32 --no-cpu-baseline ${BENCH_ARGS:-} > "$OUT/pmc_$C.json" 2> "$OUT/pmc_$C.err"
  rc=$?; echo "pmc $C rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
find "$OUT" -name '*.csv' | sort
