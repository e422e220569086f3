#!/bin/bash
# One gpurun call: the standalone teacher (craft_teacher) with and without the teacher table at
# 4,096 / 32,768 / 65,536 envs (tools/teacher_bench.py), alternating.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=${TAG:-r04_teacher}; OUT=gpurun_out/$T; mkdir -p $OUT
for pass in 1 2; do
  for tt in 1 0; do
    CRAFT_TEACH_TABLE=$tt TEACHER_ENVS=4096,32768,65536 timeout -k 10 200 python tools/teacher_bench.py \
        > $OUT/table${tt}_pass$pass.json 2> $OUT/t.err || exit $?
  done
done
for f in $OUT/*.json; do echo "$(basename $f) $(cat $f | tr '\n' ' ')"; done
