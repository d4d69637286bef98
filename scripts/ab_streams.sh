set -e -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for fs in 1e9 1.25e8; do
 for q in 4 8; do
  for sh in 0 1 3; do
   NICE_SHARED_STREAMS=$sh timeout -k 10 120 python3 bench.py --probe-lib --no-cpu-baseline --steps 100 --warmup 10 --field-size $fs --hw-queues $q > gpurun_out/ab_s${sh}_q${q}_f${fs}.json 2>/dev/null
   python3 -c "import json;d=json.load(open('gpurun_out/ab_s${sh}_q${q}_f${fs}.json'));print('$fs q$q shared$sh', round(d['ms_per_step'],4), round(d['roofline']['kernel_ms'],4), round(d['detailed_ms_per_step'],4), round(d['niceonly_ms_per_step'],4))"
  done
 done
done 2>&1 | tee gpurun_out/ab_streams.log
