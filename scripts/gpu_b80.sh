# b80 kernel iteration: FD parity tests + b80 1e9 rep timings + fd sweep.
set -e
cd /root/repo
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -k "fd_kernel or reference or full_fields_detailed or size_independent" > gpurun_out/t_fd2.log 2>&1
timeout -k 10 120 python -u scripts/rep_times.py 80 1e9 6 > gpurun_out/rep80.log 2>&1
SWEEP_VARIANTS=0 timeout -k 10 300 python -u scripts/fd_sweep.py > gpurun_out/sweep_fd2.log 2>&1
