set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/exp9; mkdir -p $O
run() { local nm=$1; shift
  timeout -k 10 120 python bench.py --no-cpu-baseline --steps 1024 "$@" > $O/$nm.json 2>$O/$nm.err || exit $?
  python -c "import json;d=json.load(open('$O/$nm.json'));print('$nm',round(d['value']/1e9,3),round(d['roofline']['kernel_us']/32,2),round(d['roofline']['frac'],3))"
}
for i in 1 2; do
 for st in 0 1; do
  run t64_512_s${st}_$i --tile 64 --rollout-threads 512 --obs-store $st
  run t16_256_s${st}_$i --tile 16 --rollout-threads 256 --obs-store $st
  run t32_256_s${st}_$i --tile 32 --rollout-threads 256 --obs-store $st
 done
done
