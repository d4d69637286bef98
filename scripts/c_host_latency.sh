# Wall time a native (C) caller sees per synchronous detailed call, on the
# two small BASELINE configs (default b40 1e6, hi-base b80 1e6): median and
# minimum of 300 calls of examples/nice_field (clock_gettime around the library
# call) next to the kernel's HIP-event time, then the same with the context's
# kernel timing off (no HIP events per field, nice_ctx_set_kernel_timing).
# Product library only: never load the probe build into a process linked
# against libnice_hip.so (the two builds' kernels share names but not
# argument layouts).
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for b in 40 80; do
    echo "== b$b 1e6 timed"
    timeout -k 10 60 examples/nice_field --gpu --repeat 300 detailed $b range 1000000 | tail -1
    echo "== b$b 1e6 kernel timing off"
    timeout -k 10 60 examples/nice_field --gpu --repeat 300 --no-timing detailed $b range 1000000 | tail -1
done
