# rocprofv3 kernel-trace summary of one bench run (args: output dir name, bench args...)
set -e
name=$1; shift
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /root/repo/gpurun_out/$name -o run -- python3 /root/repo/bench.py --no-cpu-baseline "$@" > /root/repo/gpurun_out/$name.json 2>&1
