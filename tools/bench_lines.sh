#!/bin/bash
# Every bench line of the round on one box (no profiler attached), one JSON file each in $OUT:
# the driver's command, 512 steps, the one-tick kernel (16-slot ring and one reused buffer),
# config 5 (teacher-labelled K-tick launches at K = 32 and 20, and the one-tick fused kernel;
# K = 20 with every env acting on its label, and with half of them: demonstrations, DAgger's mix),
# the closed-loop trainer, the w = 5 rollout and one-tick lines, and config 5 at w = 5 (K-tick and
# one craft_step_teach per tick).
set -u
REPO="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$REPO/gpurun_out/${TAG:-lines}"
mkdir -p "$OUT"
cd "$REPO"
CS=${CPU_SECONDS:-3}
run() {
  name=$1; shift
  timeout -k 10 300 python bench.py "$@" --cpu-seconds $CS > "$OUT/$name.json" 2> "$OUT/$name.err"
  rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || { tail -3 "$OUT/$name.err"; exit $rc; }
}
run driver --steps 20 --warmup 5
run steps512 --steps 512 --warmup 5
run k1 --ticks-per-launch 1 --steps 200 --warmup 20
run k1_ring1 --ticks-per-launch 1 --ring 1 --steps 200 --warmup 20
run config5 --workload teacher --steps 200 --warmup 20
run config5_k20 --workload teacher --ticks-per-launch 20 --steps 200 --warmup 20
run config5_k1 --workload teacher --ticks-per-launch 1 --steps 200 --warmup 20
run config5_label --workload teacher --ticks-per-launch 20 --teacher-actions label --steps 200 --warmup 20
run config5_mix --workload teacher --ticks-per-launch 20 --teacher-actions mix --steps 200 --warmup 20
run trainer --workload trainer --steps 5 --warmup 2
run w5 --world craft_medium_12x12_w5 --steps 20 --warmup 5
run w5_k1 --world craft_medium_12x12_w5 --ticks-per-launch 1 --steps 100 --warmup 10
run config5_w5 --world craft_medium_12x12_w5 --workload teacher --ticks-per-launch 20 --steps 100 --warmup 10
run config5_w5_k1 --world craft_medium_12x12_w5 --workload teacher --ticks-per-launch 1 --steps 100 --warmup 10
