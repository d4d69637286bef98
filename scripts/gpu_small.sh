set -e
cd /root/repo
mkdir -p gpurun_out
timeout -k 10 300 python3 scripts/small_sweep.py > gpurun_out/small_sweep.log 2>&1
