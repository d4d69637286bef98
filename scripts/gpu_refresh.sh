# Round refresh on the GPU box: full GPU test suite, the bench line (with the
# CPU baseline), a 1-rank torchrun bench, the rocprofv3 kernel-trace summary of
# the bench, and the PMC passes (traffic / VALU / LDS) of the detailed kernel.
set -e
cd /root/repo
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_all.log 2>&1
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 1 --no-cpu-baseline > gpurun_out/bench_tr1.json 2> gpurun_out/bench_tr1.err
bash scripts/gpu_prof.sh prof_latest
bash scripts/gpu_pmc.sh fd2
timeout -k 10 300 python -u scripts/bench_configs.py > gpurun_out/configs.jsonl 2> gpurun_out/configs.err
