# FD kernel iteration: FD parity tests, probe timings, bench line + kernel trace.
set -e
cd /root/repo
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -k "fd_kernel or reference or full_fields_detailed or size_independent" > gpurun_out/t_fd2.log 2>&1
timeout -k 10 200 python -u scripts/probe_sweep.py > gpurun_out/probe.log 2>&1
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_fd2.json 2> gpurun_out/bench_fd2.err
