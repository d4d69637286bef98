# New FD bases: GPU parity for them, then 1e9 detailed per base (configs).
set -e
cd /root/repo
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -k "production_bases or limb_count or fd_kernel_segments or reference_detailed or full_fields_detailed" > gpurun_out/gpu_bases.log 2>&1
timeout -k 10 300 python3 scripts/bench_configs.py --bases all --only-bases --reps 5 > gpurun_out/configs_bases.jsonl 2> gpurun_out/configs_bases.err
