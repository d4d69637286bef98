# Fused MSD kernel at one wave per workgroup vs four (probe knob NICE_MSD_WG):
# the GPU tests through the probe library at 64, then the pipelined bench
# step (8-way shard 1.25e8 and the whole 1e9 field), two passes.
#   gpurun -- bash scripts/msd_wg_ab.sh
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
NICE_LIB_PATH=$PWD/nice_amd/libnice_hip_probe.so NICE_MSD_WG=64 timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q \
    --timeout 300 --timeout-method thread > gpurun_out/msd_wg_tests.log 2>&1
out=gpurun_out/msd_wg.log
for pass in 1 2; do
  for wg in 256 64; do
    for fs in 1.25e8 1e9; do
      NICE_MSD_WG=$wg timeout -k 10 120 python3 bench.py --probe-lib --field-size $fs --steps 100 --warmup 20 \
          --no-cpu-baseline > gpurun_out/mw.json 2> gpurun_out/mw.err
      python3 -c "import json; d=json.loads(open('gpurun_out/mw.json').readline()); print($wg, '$fs', round(d['ms_per_step'],4), round(d['detailed_ms_per_step'],4), round(d['niceonly_ms_per_step'],4))" >> $out
    done
  done
done
