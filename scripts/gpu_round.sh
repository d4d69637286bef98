set -e
cd /root/repo
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/t_all.log 2>&1
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /root/repo/gpurun_out/prof_r01b -o run -- python3 /root/repo/bench.py --no-cpu-baseline > /root/repo/gpurun_out/bench_prof.json 2>&1
