set -e
cd /root/repo
mkdir -p gpurun_out
L=gpurun_out/massive_probe.log
: > $L
for v in 82 164 328 656; do
  NICE_MSD_CPB=$v timeout -k 10 60 python3 -u scripts/massive_probe.py >> $L 2>&1
done
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 280 --timeout-method thread tests/test_gpu_parity.py -k fd_bases_whole > gpurun_out/fd_bases_test.log 2>&1
