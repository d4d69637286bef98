# Niceonly iteration: niceonly / massive GPU parity tests, the massive field's
# wall time (scripts/massive_1gpu.py) and its rocprofv3 kernel summary.
set -e
cd /root/repo
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread \
    -k "nice or massive or unique" > gpurun_out/t_nice.log 2>&1
timeout -k 10 120 python3 -u scripts/massive_1gpu.py 10 > gpurun_out/massive.log 2>&1
timeout -k 10 120 python3 -u scripts/massive_1gpu.py 10 >> gpurun_out/massive.log 2>&1
cd /tmp && export TMPDIR=/tmp
R=/root/repo
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_massive -o run -- python3 $R/scripts/massive_1gpu.py 10 > $R/gpurun_out/prof_massive.log 2>&1
rm -f $R/gpurun_out/prof_massive/run_kernel_trace.csv
