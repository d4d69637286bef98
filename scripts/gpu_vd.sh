set -e
cd /root/repo
mkdir -p gpurun_out
timeout -k 10 500 python3 scripts/vd_sweep_all.py > gpurun_out/vd_sweep_all.log 2>&1
