#!/bin/bash
# Build the LDS trace microbenchmark on the box, write the kernel's real index
# traces (b80: S 1-8 + C 1-16 at chunk 239; b40: S 1-4 + C 1-8 at chunk 81)
# and time every layout / read style on them -> gpurun_out/lds_trace.log
set -e
mkdir -p gpurun_out
hipcc --offload-arch=gfx950 -O3 -o gpurun_out/lds_trace scripts/ubench/lds_trace.hip
python3 scripts/ubench/lds_trace_gen.py 80 239 8 16 gpurun_out/trace80.bin
python3 scripts/ubench/lds_trace_gen.py 40 81 4 8 gpurun_out/trace40.bin
for b in 80 40; do
    timeout -k 10 120 gpurun_out/lds_trace gpurun_out/trace$b.bin
done 2>&1 | tee gpurun_out/lds_trace.log
rm -f gpurun_out/trace80.bin gpurun_out/trace40.bin gpurun_out/lds_trace
