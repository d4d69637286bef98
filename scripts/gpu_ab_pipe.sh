# A/B of the pipeline's GPU-side choices at the 8-way shard size (1.25e8):
# niceonly stream priority, slots rotated, one vs two contexts, depth.
set -e
cd /root/repo
mkdir -p gpurun_out
B="timeout -k 10 200 python3 bench.py --no-cpu-baseline --probe-lib --steps 40 --warmup 5 --field-size 1.25e8"
for rep in 1 2; do
for cfg in "1 3 0 1" "1 3 0 2" "0 3 0 1" "0 3 0 2" "1 2 0 1" "0 2 0 1" "0 2 1 1" "1 2 1 1" "0 3 1 2"; do
  set -- $cfg
  extra=""; [ $3 = 1 ] && extra="--two-ctx"
  NICE_NICE_PRIO=$1 NICE_SLOTS=$2 $B --depth $4 $extra > gpurun_out/ab.json
  python3 -c "import json; d=json.load(open('gpurun_out/ab.json')); print('prio=$1 slots=$2 twoctx=$3 depth=$4', round(d['ms_per_step'],4), round(d['roofline']['kernel_ms'],4))"
done
done > gpurun_out/ab_pipe.log 2>&1
