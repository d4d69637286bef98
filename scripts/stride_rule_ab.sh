# Stride-rule A/B on the b40 pipelined-walk layout: at four offsets into the
# range, the strides two picker rules choose (target 140 / tol 0.5 against
# target 120 / tol 2.5), pipelined, five repetitions.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
run() { timeout -k 10 300 python3 scripts/ubench/stride_sweep_pipe.py --base 40 --sizes 1e9,2.5e8,1.25e8 --lo 1 --hi 0 --extra $2 --reps 5 --numbers 6e9 --at $1 >> gpurun_out/rule_ab.log 2>> gpurun_out/rule_ab.err; }
run 0.0 143,159,119,115
run 0.1 133,139,117,123,115
run 0.2 131,121
run 0.25 153,165,131,119,117
