#!/bin/bash
# rocprofv3 evidence for the config-5 bench line (bench.py --workload teacher: one fused tick +
# teacher launch per tick): kernel-trace stats, then separate FETCH_SIZE / WRITE_SIZE passes.
set -u
REPO="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$REPO/gpurun_out/${TAG:-prof_teach}"
mkdir -p "$OUT"
cd /tmp
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
    python3 "$REPO/bench.py" --workload teacher --steps 200 --warmup 10 > "$OUT/trace_bench.json" 2> "$OUT/trace.err"
rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $C --output-format csv -d "$OUT/pmc_$C" -o run -- \
      python3 "$REPO/bench.py" --workload teacher --steps 50 --warmup 0 --no-cpu-baseline > "$OUT/pmc_$C.json" 2> "$OUT/pmc_$C.err"
  rc=$?; echo "pmc $C rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
find "$OUT" -name '*.csv' | sort
