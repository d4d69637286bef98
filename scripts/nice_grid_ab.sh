# niceonly_kernel grid cap (probe knob NICE_NICE_GRID; product: 8 workgroups
# per CU) on the pipelined bench step: the 8-way shard (1.25e8) and the whole
# 1e9 field, probe library, two passes.
#   gpurun -- bash scripts/nice_grid_ab.sh
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/nice_grid.log
for pass in 1 2; do
  for g in 2048 1024 512 256 128; do
    for fs in 1.25e8 1e9; do
      NICE_NICE_GRID=$g timeout -k 10 120 python3 bench.py --probe-lib --field-size $fs --steps 100 --warmup 20 \
          --no-cpu-baseline > gpurun_out/ng.json 2> gpurun_out/ng.err
      python3 -c "import json; d=json.loads(open('gpurun_out/ng.json').readline()); print($g, '$fs', round(d['ms_per_step'],4), round(d['detailed_ms_per_step'],4), round(d['niceonly_ms_per_step'],4))" >> $out
    done
  done
done
