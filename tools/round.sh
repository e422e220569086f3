#!/bin/bash
# One gpurun call of round evidence.  STEPS picks the parts, in order (default all four):
#   smoke  __graft_entry__.smoke()
#   suite  pytest -m gpu (the parity suite)
#   lines  every bench line (tools/bench_lines.sh)
#   prof   rocprofv3 kernel-trace + separate FETCH_SIZE / WRITE_SIZE passes (tools/profile.sh) of
#          $CONFIGS ("name|bench.py args|steps" lines; default: the headline and config 5)
# Stops at the first part that ends abnormally; test failures (rc 1) do not stop the measurements.
#   TAG=r05_final bash tools/round.sh
#   TAG=r05_p STEPS="prof" CONFIGS=$'config5|--workload teacher --ticks-per-launch 20|20' bash tools/round.sh
set -u
REPO="${GRAFT_REPO_ROOT:-/root/repo}"
T=${TAG:-round}; OUT="$REPO/gpurun_out/$T"; mkdir -p "$OUT"
cd "$REPO"
for part in ${STEPS:-smoke suite lines prof}; do
  case $part in
    smoke)
      timeout -k 10 240 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
      rc=$?; echo "smoke rc=$rc"; tail -2 "$OUT/smoke.log"; [ $rc -eq 0 ] || exit $rc ;;
    suite)
      timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread \
          > "$OUT/pytest_gpu.log" 2>&1
      rc=$?; echo "suite rc=$rc"; tail -1 "$OUT/pytest_gpu.log"; [ $rc -le 1 ] || exit $rc ;;
    lines)
      TAG=$T/lines CPU_SECONDS=${CPU_SECONDS:-8} bash tools/bench_lines.sh || exit $? ;;
    prof)
      CONFIGS=${CONFIGS:-$'headline||20\nconfig5|--workload teacher --ticks-per-launch 20|20'} \
          TAG=$T/prof CPU_SECONDS=2 bash tools/profile.sh || exit $? ;;
    *) echo "unknown part $part"; exit 2 ;;
  esac
done
