#!/bin/bash
# One gpurun call: smoke, GPU parity tests, a bench line, a rocprofv3 kernel-trace summary.
# Stops at the first step that ends abnormally (fault / abort / timeout); test
# assertion failures (rc 1) do not stop the later measurement steps.
set -u
REPO="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$REPO"
OUT="$REPO/gpurun_out/${TAG:-run}"
mkdir -p "$OUT"
export TMPDIR=/tmp
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }

timeout -k 10 240 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 "$OUT/smoke.log"; ok $rc || exit $rc

if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread ${PYTEST_ARGS:-} > "$OUT/pytest_gpu.log" 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -15 "$OUT/pytest_gpu.log"; ok $rc || exit $rc
fi

timeout -k 10 300 python bench.py ${BENCH_ARGS:-} > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?; echo "bench rc=$rc"; cat "$OUT/bench.json"; tail -5 "$OUT/bench.err"; [ $rc -eq 0 ] || exit $rc

if [ "${SKIP_PROF:-0}" != "1" ]; then
  cd /tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
      python "$REPO/bench.py" --steps 512 --warmup 64 --no-cpu-baseline > "$OUT/prof_bench.json" 2> "$OUT/prof.err"
  rc=$?; echo "rocprof rc=$rc"; tail -3 "$OUT/prof.err"; [ $rc -eq 0 ] || exit $rc
  find "$OUT/prof" -name '*stats*' | head
fi
