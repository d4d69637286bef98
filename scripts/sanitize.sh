# Host-code sanitizer runs (CPU only, this container): the CPU API
# (cpu_path.cpp), the host hooks of host_math.hpp / radix_fast.hpp exported by
# nice_abi.cpp, the no-device error paths and the oracle's pthread driver,
# built with ASan + UBSan and with TSan (make ... sanitize) and exercised by
# the CPU test files, each run with the matching clang runtime preloaded into
# the Python process.  Exit status: non-zero on any sanitizer report (the
# runtimes abort on the first one) or test failure.
#   bash scripts/sanitize.sh [pytest args]   -> profiles/r04/sanitize.log
set -e -o pipefail
R="$(cd "$(dirname "$0")/.." && pwd)"
cd "$R"
make -s -C nice_amd -j8 sanitize
make -s -C oracle sanitize
RT=$(ls -d /opt/rocm/lib/llvm/lib/clang/*/lib/linux | head -1)
TESTS="tests/test_cpu_path.py tests/test_abi.py tests/test_oracle_golden.py"
for san in asan tsan; do
    echo "=== $san: $TESTS"
    NICE_LIB_PATH="$R/nice_amd/libnice_hip_$san.so" NICE_ORACLE_LIB_PATH="$R/oracle/liboracle_$san.so" \
    LD_PRELOAD="$RT/libclang_rt.$san-x86_64.so" \
    ASAN_OPTIONS=detect_leaks=0:halt_on_error=1:abort_on_error=1 \
    UBSAN_OPTIONS=halt_on_error=1:print_stacktrace=1 \
    TSAN_OPTIONS=halt_on_error=1:second_deadlock_stack=1 \
        python3 -m pytest $TESTS -q -m "not gpu" -p no:cacheprovider "$@"
done
# Canary: the ASan build must report a deliberate heap overflow (a 32-byte
# histogram buffer where base 40 needs 41 u64 bins), or the runs above prove
# nothing.
echo "=== asan canary (expects a heap-buffer-overflow report)"
if NICE_LIB_PATH="$R/nice_amd/libnice_hip_asan.so" LD_PRELOAD="$RT/libclang_rt.asan-x86_64.so" \
   ASAN_OPTIONS=detect_leaks=0 python3 - 2> /tmp/asan_canary.txt <<'PY'
import ctypes as c
import nice_amd._lib as L
libc = c.CDLL(None)
libc.malloc.restype = c.c_void_p
p = libc.malloc(32)
out, n = (L.nice_number * 16)(), c.c_size_t()
L.lib().nice_cpu_process_range_detailed(1916284264916, 0, 1916284265916, 0, 40, 1,
                                        c.cast(p, c.POINTER(c.c_uint64)), out, 16, n)
PY
then
    echo "canary NOT caught"; exit 1
fi
grep -m1 "ERROR: AddressSanitizer: heap-buffer-overflow" /tmp/asan_canary.txt
