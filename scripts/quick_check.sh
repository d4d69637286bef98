# Env probe + default bench + 1-rank torchrun bench (no CPU baseline).
set -e
cd /root/repo
mkdir -p gpurun_out
echo "GPU_MAX_HW_QUEUES=${GPU_MAX_HW_QUEUES-unset} nproc=$(nproc)" > gpurun_out/env.log
timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/qb.json 2> gpurun_out/qb.err
timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 1 --no-cpu-baseline > gpurun_out/qb_tr1.json 2> gpurun_out/qb_tr1.err
