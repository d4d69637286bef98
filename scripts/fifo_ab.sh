# Detailed fields back to back on ONE stream (probe NICE_SHARED_STREAMS=1)
# against one stream per slot (concurrent, the product), pipelined bench step
# at 1.25e8 / 2.5e8 / 1e9, detailed only and both modes, probe library, two passes.
#   gpurun -- bash scripts/fifo_ab.sh
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/fifo.log
for pass in 1 2; do
  for sh in 0 1; do
    for fs in 1.25e8 2.5e8 1e9; do
      NICE_SHARED_STREAMS=$sh timeout -k 10 120 python3 bench.py --probe-lib --field-size $fs --steps 100 --warmup 20 \
          --no-cpu-baseline > gpurun_out/ff.json 2> gpurun_out/ff.err
      python3 -c "import json; d=json.loads(open('gpurun_out/ff.json').readline()); print('shared', $sh, '$fs', round(d['ms_per_step'],4), round(d['detailed_ms_per_step'],4))" >> $out
    done
  done
done
