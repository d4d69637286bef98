# Lone (synchronous) b40 fields on the pipelined-walk layout: the launcher's
# pick (0: rounds-aware since round 6) against forced strides, isolated
# launches (scripts/knob_sweep.py, probe library), at several sizes and
# offsets; then the GPU tests and the default bench line with the product library.
#   gpurun -- bash scripts/lone_rounds_ab.sh
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
KNOB_ROUNDS=5 timeout -k 10 600 python3 scripts/knob_sweep.py NICE_FD2_SIBCHUNK 0,143,159,169 \
    40:1e9 40:1e9:0.1 40:1e9:0.2 40:5e8 40:7e8 40:4e8:0.25 > gpurun_out/lone_rounds.log 2>&1
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tests_lone.log 2>&1
bash scripts/gpu.sh bench lone_a
bash scripts/gpu.sh bench lone_b
