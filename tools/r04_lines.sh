#!/bin/bash
# Round-4 evidence, call 1: smoke, the GPU suite, every bench line (tools/bench_lines.sh).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=${TAG:-r04_lines}; OUT=gpurun_out/$T; mkdir -p $OUT
timeout -k 10 240 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { tail -20 "$OUT/smoke.log"; exit 1; }
tail -2 "$OUT/smoke.log"
timeout -k 10 300 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread \
    > "$OUT/pytest_gpu.log" 2>&1; rc=$?; tail -1 "$OUT/pytest_gpu.log"; [ $rc -le 1 ] || exit $rc
TAG=$T/lines CPU_SECONDS=${CPU_SECONDS:-8} bash tools/bench_lines.sh || exit $?
for f in $OUT/lines/*.json; do python - "$f" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d.get("roofline", {})
print(sys.argv[1].split("/")[-1], "value %.3g" % d["value"], "frac", r.get("frac"), "kernel_us", r.get("kernel_us"),
      "ceiling_frac", r.get("frac_of_ceiling"), "cpu", (d.get("cpu_baseline") or {}).get("value"))
PY
done
