#!/bin/bash
# rocprofv3 evidence for one round: kernel-trace stats of the bench at the driver's command
# (--steps 20 --warmup 5: one 20-tick launch) and at 512 steps (32-tick launches), then
# separate PMC passes (counters never combined with other trace domains), with no warmup so
# that every traced launch has the same tick count.
set -u
REPO="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$REPO/gpurun_out/${TAG:-prof}"
mkdir -p "$OUT"
cd /tmp
export TMPDIR=/tmp
for S in 20 512; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_$S" -o run -- \
      python3 "$REPO/bench.py" --steps $S --warmup 5 ${BENCH_ARGS:-} > "$OUT/trace_bench_$S.json" 2> "$OUT/trace_$S.err"
  rc=$?; echo "trace $S rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
for S in 20 128; do
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --pmc $C --output-format csv -d "$OUT/pmc_${S}_$C" -o run -- \
        python3 "$REPO/bench.py" --steps $S --warmup 0 --no-cpu-baseline ${BENCH_ARGS:-} > "$OUT/pmc_${S}_$C.json" 2> "$OUT/pmc_${S}_$C.err"
    rc=$?; echo "pmc $S $C rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
done
find "$OUT" -name '*.csv' | sort
