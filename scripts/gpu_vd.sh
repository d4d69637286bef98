set -e
cd /root/repo
mkdir -p gpurun_out
VDS=101,356,357,358,0 timeout -k 10 500 python3 scripts/vd_sweep_all.py 59 60 62 63 64 65 67 68 80 > gpurun_out/vd_sweep_low.log 2>&1
