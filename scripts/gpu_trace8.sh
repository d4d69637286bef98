set -e
cd /tmp && export TMPDIR=/tmp
R=/root/repo
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/prof_shard8 -o kt -- python3 $R/bench.py --no-cpu-baseline --steps 40 --warmup 5 --field-size 1.25e8 --depth 1 > $R/gpurun_out/prof_shard8.json 2>$R/gpurun_out/prof_shard8.err
