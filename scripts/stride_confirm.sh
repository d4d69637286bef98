# Confirmation of the sweep winners (scripts/stride_sweep_all.sh): fresh
# repetitions, a third field size and fields halfway into each base range.
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 300 python3 scripts/ubench/stride_sweep_pipe.py --base 40 --sizes 1e9,4e8,1.25e8 --lo 1 --hi 0 --extra 0,119,147,159,191 --reps 6 --numbers 8e9 --at 0.0 >> gpurun_out/confirm.log 2>> gpurun_out/confirm.err
timeout -k 10 300 python3 scripts/ubench/stride_sweep_pipe.py --base 40 --sizes 1e9,4e8,1.25e8 --lo 1 --hi 0 --extra 0,119,147,159,191 --reps 6 --numbers 8e9 --at 0.5 >> gpurun_out/confirm.log 2>> gpurun_out/confirm.err
timeout -k 10 300 python3 scripts/ubench/stride_sweep_pipe.py --base 42 --sizes 1e9,4e8,1.25e8 --lo 1 --hi 0 --extra 0,147,189,105 --reps 6 --numbers 8e9 --at 0.0 >> gpurun_out/confirm.log 2>> gpurun_out/confirm.err
timeout -k 10 300 python3 scripts/ubench/stride_sweep_pipe.py --base 42 --sizes 1e9,4e8,1.25e8 --lo 1 --hi 0 --extra 0,147,189,105 --reps 6 --numbers 8e9 --at 0.5 >> gpurun_out/confirm.log 2>> gpurun_out/confirm.err
timeout -k 10 300 python3 scripts/ubench/stride_sweep_pipe.py --base 43 --sizes 1e9,4e8,1.25e8 --lo 1 --hi 0 --extra 0,251,193,169 --reps 6 --numbers 8e9 --at 0.0 >> gpurun_out/confirm.log 2>> gpurun_out/confirm.err
timeout -k 10 300 python3 scripts/ubench/stride_sweep_pipe.py --base 43 --sizes 1e9,4e8,1.25e8 --lo 1 --hi 0 --extra 0,251,193,169 --reps 6 --numbers 8e9 --at 0.5 >> gpurun_out/confirm.log 2>> gpurun_out/confirm.err
timeout -k 10 300 python3 scripts/ubench/stride_sweep_pipe.py --base 44 --sizes 1e9,4e8,1.25e8 --lo 1 --hi 0 --extra 0,127,231,121 --reps 6 --numbers 8e9 --at 0.0 >> gpurun_out/confirm.log 2>> gpurun_out/confirm.err
timeout -k 10 300 python3 scripts/ubench/stride_sweep_pipe.py --base 44 --sizes 1e9,4e8,1.25e8 --lo 1 --hi 0 --extra 0,127,231,121 --reps 6 --numbers 8e9 --at 0.5 >> gpurun_out/confirm.log 2>> gpurun_out/confirm.err
timeout -k 10 300 python3 scripts/ubench/stride_sweep_pipe.py --base 45 --sizes 1e9,4e8,1.25e8 --lo 1 --hi 0 --extra 0,159,119,157 --reps 6 --numbers 8e9 --at 0.0 >> gpurun_out/confirm.log 2>> gpurun_out/confirm.err
timeout -k 10 300 python3 scripts/ubench/stride_sweep_pipe.py --base 45 --sizes 1e9,4e8,1.25e8 --lo 1 --hi 0 --extra 0,159,119,157 --reps 6 --numbers 8e9 --at 0.5 >> gpurun_out/confirm.log 2>> gpurun_out/confirm.err
timeout -k 10 300 python3 scripts/ubench/stride_sweep_pipe.py --base 47 --sizes 1e9,4e8,1.25e8 --lo 1 --hi 0 --extra 0,199,141,171 --reps 6 --numbers 8e9 --at 0.0 >> gpurun_out/confirm.log 2>> gpurun_out/confirm.err
timeout -k 10 300 python3 scripts/ubench/stride_sweep_pipe.py --base 47 --sizes 1e9,4e8,1.25e8 --lo 1 --hi 0 --extra 0,199,141,171 --reps 6 --numbers 8e9 --at 0.5 >> gpurun_out/confirm.log 2>> gpurun_out/confirm.err
timeout -k 10 300 python3 scripts/ubench/stride_sweep_pipe.py --base 48 --sizes 1e9,4e8,1.25e8 --lo 1 --hi 0 --extra 0,161,199,219 --reps 6 --numbers 8e9 --at 0.0 >> gpurun_out/confirm.log 2>> gpurun_out/confirm.err
timeout -k 10 300 python3 scripts/ubench/stride_sweep_pipe.py --base 48 --sizes 1e9,4e8,1.25e8 --lo 1 --hi 0 --extra 0,161,199,219 --reps 6 --numbers 8e9 --at 0.5 >> gpurun_out/confirm.log 2>> gpurun_out/confirm.err
timeout -k 10 300 python3 scripts/ubench/stride_sweep_pipe.py --base 49 --sizes 1e9,4e8,1.25e8 --lo 1 --hi 0 --extra 0,147,203,245 --reps 6 --numbers 8e9 --at 0.0 >> gpurun_out/confirm.log 2>> gpurun_out/confirm.err
timeout -k 10 300 python3 scripts/ubench/stride_sweep_pipe.py --base 49 --sizes 1e9,4e8,1.25e8 --lo 1 --hi 0 --extra 0,147,203,245 --reps 6 --numbers 8e9 --at 0.5 >> gpurun_out/confirm.log 2>> gpurun_out/confirm.err
timeout -k 10 300 python3 scripts/ubench/stride_sweep_pipe.py --base 50 --sizes 1e9,4e8,1.25e8 --lo 1 --hi 0 --extra 0,183,137,123 --reps 6 --numbers 8e9 --at 0.0 >> gpurun_out/confirm.log 2>> gpurun_out/confirm.err
timeout -k 10 300 python3 scripts/ubench/stride_sweep_pipe.py --base 50 --sizes 1e9,4e8,1.25e8 --lo 1 --hi 0 --extra 0,183,137,123 --reps 6 --numbers 8e9 --at 0.5 >> gpurun_out/confirm.log 2>> gpurun_out/confirm.err
timeout -k 10 300 python3 scripts/ubench/stride_sweep_pipe.py --base 52 --sizes 1e9,4e8,1.25e8 --lo 1 --hi 0 --extra 0,169,255,223 --reps 6 --numbers 8e9 --at 0.0 >> gpurun_out/confirm.log 2>> gpurun_out/confirm.err
timeout -k 10 300 python3 scripts/ubench/stride_sweep_pipe.py --base 52 --sizes 1e9,4e8,1.25e8 --lo 1 --hi 0 --extra 0,169,255,223 --reps 6 --numbers 8e9 --at 0.5 >> gpurun_out/confirm.log 2>> gpurun_out/confirm.err
timeout -k 10 300 python3 scripts/ubench/stride_sweep_pipe.py --base 53 --sizes 1e9,4e8,1.25e8 --lo 1 --hi 0 --extra 0,199,231,193 --reps 6 --numbers 8e9 --at 0.0 >> gpurun_out/confirm.log 2>> gpurun_out/confirm.err
timeout -k 10 300 python3 scripts/ubench/stride_sweep_pipe.py --base 53 --sizes 1e9,4e8,1.25e8 --lo 1 --hi 0 --extra 0,199,231,193 --reps 6 --numbers 8e9 --at 0.5 >> gpurun_out/confirm.log 2>> gpurun_out/confirm.err
timeout -k 10 300 python3 scripts/ubench/stride_sweep_pipe.py --base 54 --sizes 1e9,4e8,1.25e8 --lo 1 --hi 0 --extra 0,135,129,119 --reps 6 --numbers 8e9 --at 0.0 >> gpurun_out/confirm.log 2>> gpurun_out/confirm.err
timeout -k 10 300 python3 scripts/ubench/stride_sweep_pipe.py --base 54 --sizes 1e9,4e8,1.25e8 --lo 1 --hi 0 --extra 0,135,129,119 --reps 6 --numbers 8e9 --at 0.5 >> gpurun_out/confirm.log 2>> gpurun_out/confirm.err
timeout -k 10 300 python3 scripts/ubench/stride_sweep_pipe.py --base 55 --sizes 1e9,4e8,1.25e8 --lo 1 --hi 0 --extra 0,253,215,227 --reps 6 --numbers 8e9 --at 0.0 >> gpurun_out/confirm.log 2>> gpurun_out/confirm.err
timeout -k 10 300 python3 scripts/ubench/stride_sweep_pipe.py --base 55 --sizes 1e9,4e8,1.25e8 --lo 1 --hi 0 --extra 0,253,215,227 --reps 6 --numbers 8e9 --at 0.5 >> gpurun_out/confirm.log 2>> gpurun_out/confirm.err
