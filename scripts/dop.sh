set -e
cd /root/repo
mkdir -p gpurun_out
P=scripts/dist_overlap_phases.py
timeout -k 10 120 python $P > gpurun_out/dop.log 2>&1
TORCH_CUDA=1 timeout -k 10 120 python $P >> gpurun_out/dop.log 2>&1
timeout -k 10 120 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 $P >> gpurun_out/dop.log 2>&1
