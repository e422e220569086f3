#!/bin/bash
# Round-4 evidence, call 2: rocprofv3 kernel-trace + FETCH_SIZE / WRITE_SIZE passes (tools/profile.sh)
# of the headline, config 5, the trainer, the w = 5 one-tick line and the one-tick reused-buffer line.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
CONFIGS=$'headline||20\nconfig5|--workload teacher|200\ntrainer|--workload trainer|5\nw5_k1|--world craft_medium_12x12_w5 --ticks-per-launch 1|100\nk1_ring1|--ticks-per-launch 1 --ring 1|200' \
  TAG=${TAG:-r04_prof} CPU_SECONDS=2 bash tools/profile.sh
