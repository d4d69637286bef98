#!/bin/bash
# b80 lane->n assignment on the hardware: the kernel's
# real index traces (S 1-8 + C 1-16) with a wave's lanes at stride 239 (the
# production chunk), 1 (interleaved lanes), 3, 241 and b^4 = 40 960 000
# (one lane per b^2-limb block: limbs 0-1 of n^2 / n^3 equal across lanes),
# each timed by scripts/ubench/lds_trace.hip -> gpurun_out/lds_stride.log
set -e
mkdir -p gpurun_out
hipcc --offload-arch=gfx950 -O3 -o gpurun_out/lds_trace scripts/ubench/lds_trace.hip
: > gpurun_out/lds_stride.log
for c in 239 1 3 241 40960000; do
    python3 scripts/ubench/lds_trace_gen.py 80 $c 8 16 gpurun_out/trace80_$c.bin
    echo "== b80 lane stride $c" >> gpurun_out/lds_stride.log
    timeout -k 10 120 gpurun_out/lds_trace gpurun_out/trace80_$c.bin >> gpurun_out/lds_stride.log 2>&1
    rm -f gpurun_out/trace80_$c.bin
done
rm -f gpurun_out/lds_trace
