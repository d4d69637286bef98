set -e
cd /root/repo
mkdir -p gpurun_out
L=gpurun_out/latency_probe.log
: > $L
for i in 1 2; do
timeout -k 10 200 python3 -u scripts/latency_probe.py >> $L 2>&1
done
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_dist.py > gpurun_out/latency_tests.log 2>&1
