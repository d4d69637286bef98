set -e
cd /root/repo
TR="python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 1 --no-cpu-baseline"
timeout -k 10 200 $TR > gpurun_out/tr_default.json 2> gpurun_out/tr_default.err
timeout -k 10 200 $TR --sequential > gpurun_out/tr_seq.json 2> gpurun_out/tr_seq.err
GPU_MAX_HW_QUEUES=8 timeout -k 10 200 $TR > gpurun_out/tr_q8.json 2> gpurun_out/tr_q8.err
