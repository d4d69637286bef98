# niceonly iteration: niceonly parity tests, bench (niceonly only) under a kernel trace.
set -e
cd /root/repo
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -k "niceonly or is_nice" > gpurun_out/t_nice.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /root/repo/gpurun_out/prof_nice -o run -- python3 /root/repo/bench.py --no-cpu-baseline --mode niceonly > /root/repo/gpurun_out/bench_nice.json 2>&1
