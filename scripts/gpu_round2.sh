# Round-2 GPU check: box CPU facts, GPU parity suite, a short bench line.
set -e
cd /root/repo
mkdir -p gpurun_out
{ nproc; python3 -c "import os; print('cpu_count', os.cpu_count(), 'affinity', len(os.sched_getaffinity(0)))"; cat /sys/fs/cgroup/cpu.max 2>/dev/null || true; env | grep -E "OMP_NUM|MAX_JOBS|GPU_MAX_HW" || true; } > gpurun_out/box_cpu.txt 2>&1
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_quick.json 2> gpurun_out/bench_quick.err
