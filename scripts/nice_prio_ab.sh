# niceonly stream at the highest priority (product) vs the detailed streams'
# (probe knob NICE_NICE_PRIO=0): the bench step at 1e9 and the 8-way dealt
# shares (scripts/shard_pipelined.py), probe library, two passes.
#   gpurun -- bash scripts/nice_prio_ab.sh
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/nice_prio.log
P=$PWD/nice_amd/libnice_hip_probe.so
for pass in 1 2; do
  for pr in 1 0; do
    NICE_NICE_PRIO=$pr timeout -k 10 120 python3 bench.py --probe-lib --steps 100 --warmup 20 --no-cpu-baseline > gpurun_out/np.json 2> gpurun_out/np.err
    python3 -c "import json; d=json.loads(open('gpurun_out/np.json').readline()); print('prio', $pr, '1e9', round(d['ms_per_step'],4), round(d['detailed_ms_per_step'],4), round(d['niceonly_ms_per_step'],4))" >> $out
    NICE_LIB_PATH=$P NICE_NICE_PRIO=$pr timeout -k 10 200 python3 scripts/shard_pipelined.py --worlds 8 --steps 300 > gpurun_out/np8.json 2> /dev/null
    python3 -c "import json; d=json.loads(open('gpurun_out/np8.json').readline()); print('prio', $pr, 'N8', d['max_rank_ms_per_step'], round(sum(d['ranks_ms_per_step'])/8, 5))" >> $out
  done
done
