# Round-6 small-field variants: the GPU tests on the
# product library (tagged result words), then the probe build's small-field
# kernels (NICE_FD2_SMALLV 0 production / 1 no low-digit table / 2 same +
# limb 0 by VALU / 3 no table) and tagged vs untagged result words, kernel
# times interleaved (scripts/knob_sweep.py), and the phase stamps.
set -e -o pipefail
bash scripts/gpu.sh tests
export KNOB_ROUNDS=5
timeout -k 10 200 python3 scripts/knob_sweep.py NICE_FD2_SMALLV 0,1,2,3 40:1e6 80:1e6 40:1e5 40:9e6 80:9e6 40:1e6:0.5 80:1e6:0.5 > gpurun_out/small_v.log 2>&1
timeout -k 10 200 python3 scripts/knob_sweep.py NICE_FD2_UNTAGGED ,1 40:1e6 80:1e6 40:1e5 > gpurun_out/small_tag.log 2>&1
for v in 0 1 2 3; do NICE_FD2_SMALLV=$v timeout -k 10 120 python3 scripts/fd2_stamps.py 40:1e6 80:1e6 > gpurun_out/stamps_v$v.log 2>&1; done
