# (Record of a round-6 A/B: the NICE_FD2_CHAIN probe was removed after it)
# Chained pipelined fields (probe NICE_FD2_CHAIN, per mille of a field's fd2
# part launched before the event the next field waits on; 0 = the product's
# concurrent fields): GPU tests through the probe library with chaining on,
# then the pipelined bench step at 1.25e8 / 2.5e8 / 1e9 and the 8-way dealt
# shares, two passes.
#   gpurun -- bash scripts/chain_ab.sh
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
P=$PWD/nice_amd/libnice_hip_probe.so
NICE_LIB_PATH=$P NICE_FD2_CHAIN=850 timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 \
    --timeout-method thread > gpurun_out/chain_tests.log 2>&1
out=gpurun_out/chain.log
for pass in 1 2; do
  for c in 0 700 850 950; do
    for fs in 1.25e8 2.5e8 1e9; do
      NICE_FD2_CHAIN=$c timeout -k 10 120 python3 bench.py --probe-lib --field-size $fs --steps 100 --warmup 20 \
          --no-cpu-baseline > gpurun_out/ch.json 2> gpurun_out/ch.err
      python3 -c "import json; d=json.loads(open('gpurun_out/ch.json').readline()); print('chain', $c, '$fs', round(d['ms_per_step'],4), round(d['detailed_ms_per_step'],4), d['verified_against_fixture'])" >> $out
    done
    NICE_LIB_PATH=$P NICE_FD2_CHAIN=$c timeout -k 10 200 python3 scripts/shard_pipelined.py --worlds 8 --steps 300 > gpurun_out/ch8.json 2> /dev/null
    python3 -c "import json; d=json.loads(open('gpurun_out/ch8.json').readline()); print('chain', $c, 'N8', d['max_rank_ms_per_step'], round(sum(d['ranks_ms_per_step'])/8, 5))" >> $out
  done
done
