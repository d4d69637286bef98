// fd2_part.hip -- per-base launchers of the FD detailed kernel, one object per
// part (built with -DFD2_PART=k, k < FD2_NPARTS): part k instantiates the
// bases with fd2_part_of(base) == k, so the ~70 kernel instantiations of
// FD2_COMBOS compile in parallel.
#include "fd2_combos.h"
#include "fd2_kernel.hpp"

#ifndef FD2_PART
#error "build with -DFD2_PART=k"
#endif

#define FD2_CAT2(a, b) a##b
#define FD2_CAT(a, b) FD2_CAT2(a, b)

namespace nice {
namespace fd2 {

template <int B_, int ND_, int NE_, int NE2_>
static hipError_t try_combo(const DetailedLaunch &p, int nd, int ne, int ne2, bool wg512, int num_cus,
                            hipStream_t s) {
    if constexpr (fd2_part_of(B_) != FD2_PART) {
        return hipErrorNotFound;
    } else {
        if ((int)p.base != B_ || nd != ND_ || ne != NE_ || ne2 != NE2_) return hipErrorNotFound;
        // the host's occupancy model (big_wg) reads the same layout
        static_assert(Cfg<B_, ND_, NE_, NE2_, 0, 512, valu_limbs(B_)>::LDS_BYTES == lds_bytes(B_, 512) &&
                          Cfg<B_, ND_, NE_, NE2_, 0, big_wg(B_), valu_limbs(B_)>::LDS_BYTES ==
                              lds_bytes(B_, big_wg(B_)),
                      "lds_bytes mirrors Cfg");
#include NICE_PROBE_INC("fd2_part_probe_dispatch.inc")
        // b40 fields >= 1e7: three sibling lanes (Cfg::SIB, fd2_kernel.hpp;
        // launch_sib falls back to the regular kernel below ~1.5 rounds of
        // sibling units): on the first limb layout (the range's first ~29 %,
        // the benchmark fields) pipelined with the lowest C limb above the
        // shared one decoded by VALU, elsewhere per-sibling lookup groups, no
        // VALU decode (profiles/r05/sib_sweep_range.log)
        if constexpr (B_ == 40) {
            if (!wg512) {
                if constexpr (ND_ == 4) return launch_cfg<Cfg<B_, ND_, NE_, NE2_, 0, 512, 4097, 100, 0, 3>>(p, num_cus, s);
                else return launch_cfg<Cfg<B_, ND_, NE_, NE2_, 0, 512, 0, 1, 0, 3>>(p, num_cus, s);
            }
        }
        // b42..45 the same, per-sibling lookup groups: 1e9 at the range start
        // and half-way b42 -11 / -8 %, b43 -12 / -14, b44 -10 / -11, b45 -6 /
        // -3 against their regular kernels (profiles/r05/sib_bases_ab.log)
        if constexpr (B_ >= 42 && B_ <= 45) {
            if (!wg512) return launch_cfg<Cfg<B_, ND_, NE_, NE2_, 0, 512, 0, 1, 0, 3>>(p, num_cus, s);
        }
        // b47..55: two sibling lanes over the short low-digit table (Cfg::LDE,
        // two 512-thread workgroups per CU; with the full 2B table and three
        // lanes they held one and lost +1..+25 %): 1e9 at the range start and
        // half-way -2..-9 %, b50 / b53 half-way -2 / -0.6 %
        // (profiles/r05/sib_short_table_ab.log)
        if constexpr (B_ >= 47 && B_ <= 55 && B_ != 51) {
            if (!wg512) return launch_cfg<Cfg<B_, ND_, NE_, NE2_, 0, 512, 0, 1, 0, 2>>(p, num_cus, s);
        }
        // (the LSDX bases' tables leave room for one workgroup per CU: 1024
        // threads for every field size, 4 waves per SIMD instead of 2)
        // (fields of >= 1e7 take valu_limbs_big: see there)
        constexpr bool small512 = (valu_limbs(B_) & 1024) == 0;
        return wg512 && small512
                   ? launch_cfg<Cfg<B_, ND_, NE_, NE2_, 0, 512, valu_limbs(B_)>>(p, num_cus, s)
                   : launch_cfg<Cfg<B_, ND_, NE_, NE2_, 0, big_wg(B_), valu_limbs_big(B_, ND_, NE_)>>(p, num_cus, s);
    }
}

// hipErrorNotFound: not this part's (base, combo).
hipError_t FD2_CAT(launch_part, FD2_PART)(const DetailedLaunch &p, int nd, int ne, int ne2, bool wg512,
                                          int num_cus, hipStream_t s) {
    hipError_t e;
#define X(B_, ND_, NE_, NE2_)                                                                  \
    if ((e = try_combo<B_, ND_, NE_, NE2_>(p, nd, ne, ne2, wg512, num_cus, s)) != hipErrorNotFound) \
        return e;
    FD2_COMBOS(X)
#undef X
    return hipErrorNotFound;
}

}  // namespace fd2
}  // namespace nice
