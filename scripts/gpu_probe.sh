set -e
cd /root/repo
mkdir -p gpurun_out
timeout -k 10 200 python -u scripts/probe_sweep.py > gpurun_out/probe.log 2>&1
bash scripts/gpu_pmc.sh fd2
