# Round check: GPU parity tests, one default bench line, rocprofv3 kernel-trace
# summary of the same bench, and PMC passes over the detailed kernel.
set -e
cd /root/repo
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/t_gpu.log 2>&1
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /root/repo/gpurun_out/prof -o run -- python3 /root/repo/bench.py --no-cpu-baseline > /root/repo/gpurun_out/bench_prof.json 2>&1
bash /root/repo/scripts/gpu_pmc.sh bench
