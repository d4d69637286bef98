// probe.hpp -- the probe-build hooks, in one place.
//
// `make -C nice_amd probe` builds libnice_hip_probe.so from the same sources
// with -DNICE_PROBES: environment tuning knobs, the bottleneck probes (kernels
// whose results are wrong by design) and the phase stamps, for scripts/ A/B
// runs.  That library is never shipped.  This header is the only place the
// macro is tested; product sources use the names below, which in the product
// build are compile-time constants or expand to nothing (so no knob string,
// probe kernel or probe export reaches libnice_hip.so: tests/test_abi.py
// test_product_library_has_no_probe_kernels).
//
//   probe_knob(name, dflt)   a tuning knob's environment override (product: dflt)
//   probe_set(name)          whether a probe switch is set (product: false)
//   kProbes                  true in the probe build (`kProbes && cond` guards)
//   NICE_PROBE_ONLY(...)     statements of the probe build only
//   #include NICE_PROBE_INC("x.inc")
//                            a probe-only source fragment (probe-specific
//                            template dispatch, exports); the product build
//                            includes the empty probe_off.inc instead
#pragma once

#include <stdint.h>
#include <stdlib.h>

namespace nice {

#ifdef NICE_PROBES
constexpr bool kProbes = true;
inline uint64_t probe_knob(const char *name, uint64_t dflt) {
    const char *v = getenv(name);
    return v && *v ? strtoull(v, nullptr, 10) : dflt;
}
inline bool probe_set(const char *name) {
    const char *v = getenv(name);
    return v && *v;
}
#define NICE_PROBE_ONLY(...) __VA_ARGS__
#define NICE_PROBE_INC(f) f
#else
constexpr bool kProbes = false;
constexpr uint64_t probe_knob(const char *, uint64_t dflt) { return dflt; }
constexpr bool probe_set(const char *) { return false; }
#define NICE_PROBE_ONLY(...)
#define NICE_PROBE_INC(f) "probe_off.inc"
#endif

}  // namespace nice
