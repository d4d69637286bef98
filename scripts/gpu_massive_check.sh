set -e
cd /root/repo
mkdir -p gpurun_out
L=gpurun_out/massive_probe.log
: > $L
timeout -k 10 60 python3 -u scripts/massive_probe.py >> $L 2>&1
NICE_MSD_CPB=656 timeout -k 10 60 python3 -u scripts/massive_probe.py >> $L 2>&1
NICE_MSD_CPB=1311 timeout -k 10 60 python3 -u scripts/massive_probe.py >> $L 2>&1
timeout -k 10 120 python3 -u scripts/massive_deal.py 8 3 > gpurun_out/massive_deal.log 2>&1
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_dist.py > gpurun_out/t_all.log 2>&1
