cd /root/repo && mkdir -p gpurun_out && timeout -k 10 600 python3 -u scripts/massive_deal.py 8 3 > gpurun_out/massive_deal.log 2>&1
