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
#ifdef NICE_PROBES
        // VALU-decoded limb sweep (scripts/vd_sweep.py): NICE_FD2_VD = 100 + VD
        switch ((int)probe_knob("NICE_FD2_VD", 0)) {
        case 100: return launch_cfg<Cfg<B_, ND_, NE_, NE2_, 0, big_wg(B_), 0>>(p, num_cus, s);
        case 101: return launch_cfg<Cfg<B_, ND_, NE_, NE2_, 0, big_wg(B_), 1>>(p, num_cus, s);
        case 102: return launch_cfg<Cfg<B_, ND_, NE_, NE2_, 0, big_wg(B_), 2>>(p, num_cus, s);
        case 103: return launch_cfg<Cfg<B_, ND_, NE_, NE2_, 0, big_wg(B_), 3>>(p, num_cus, s);
        case 117: return launch_cfg<Cfg<B_, ND_, NE_, NE2_, 0, big_wg(B_), 17>>(p, num_cus, s);
        case 118: return launch_cfg<Cfg<B_, ND_, NE_, NE2_, 0, big_wg(B_), 18>>(p, num_cus, s);
        case 356: return launch_cfg<Cfg<B_, ND_, NE_, NE2_, 0, big_wg(B_), 256>>(p, num_cus, s);
        case 357: return launch_cfg<Cfg<B_, ND_, NE_, NE2_, 0, big_wg(B_), 257>>(p, num_cus, s);
        case 358: return launch_cfg<Cfg<B_, ND_, NE_, NE2_, 0, big_wg(B_), 258>>(p, num_cus, s);
        default: break;
        }
        // b65..80: VALU-decoded limbs just below the top stepped limb (VD &
        // 2048): NICE_FD2_VD = 100 + VD as above
        if constexpr ((B_ + 31) / 32 == 3) {
            switch ((int)probe_knob("NICE_FD2_VD", 0)) {
            case 2405: return launch_cfg<Cfg<B_, ND_, NE_, NE2_, 0, big_wg(B_), 2305>>(p, num_cus, s);
            case 2406: return launch_cfg<Cfg<B_, ND_, NE_, NE2_, 0, big_wg(B_), 2306>>(p, num_cus, s);
            case 2420: return launch_cfg<Cfg<B_, ND_, NE_, NE2_, 0, big_wg(B_), 2320>>(p, num_cus, s);
            case 2407: return launch_cfg<Cfg<B_, ND_, NE_, NE2_, 0, big_wg(B_), 2307>>(p, num_cus, s);
            case 2421: return launch_cfg<Cfg<B_, ND_, NE_, NE2_, 0, big_wg(B_), 2321>>(p, num_cus, s);
            case 2422: return launch_cfg<Cfg<B_, ND_, NE_, NE2_, 0, big_wg(B_), 2322>>(p, num_cus, s);
            case 2408: return launch_cfg<Cfg<B_, ND_, NE_, NE2_, 0, big_wg(B_), 2308>>(p, num_cus, s);
            case 2423: return launch_cfg<Cfg<B_, ND_, NE_, NE2_, 0, big_wg(B_), 2323>>(p, num_cus, s);
            default: break;
            }
        }
        // Two-word bases: k limbs below the top stepped ones by VALU (VD & 2048,
        // keeping the base's low-digit-table mode): NICE_FD2_VD = 6000 + k
        if constexpr ((B_ + 31) / 32 == 2) {
            constexpr int KEEP = valu_limbs(B_) & 1024;
            switch ((int)probe_knob("NICE_FD2_VD", 0)) {
            case 6001: return launch_cfg<Cfg<B_, ND_, NE_, NE2_, 0, big_wg(B_), KEEP | 2048 | 1>>(p, num_cus, s);
            case 6002: return launch_cfg<Cfg<B_, ND_, NE_, NE2_, 0, big_wg(B_), KEEP | 2048 | 2>>(p, num_cus, s);
            case 6003: return launch_cfg<Cfg<B_, ND_, NE_, NE2_, 0, big_wg(B_), KEEP | 2048 | 3>>(p, num_cus, s);
            case 6017: return launch_cfg<Cfg<B_, ND_, NE_, NE2_, 0, big_wg(B_), KEEP | 2048 | 17>>(p, num_cus, s);
            default: break;
            }
        }
        // Any base with VALU-decoded top limbs: the same count just below the
        // top stepped limbs instead (VD & 2048): NICE_FD2_VD = 5000
        if constexpr ((valu_limbs(B_) & 0xff) != 0 && (valu_limbs(B_) & 2048) == 0) {
            if ((int)probe_knob("NICE_FD2_VD", 0) == 5000)
                return launch_cfg<Cfg<B_, ND_, NE_, NE2_, 0, big_wg(B_), valu_limbs(B_) | 2048>>(p, num_cus, s);
        }
        // Low-digit table with a side table of carries (Cfg::LSDX, b59..64):
        // NICE_FD2_VD = 1100 + VD, VD = the VALU-decoded top limbs
        constexpr int DB_ = B_ - 32;
        if constexpr ((B_ + 31) / 32 == 2 && DB_ > 0 && DB_ + (DB_ > 20 ? 4 : 10) > 30) {
            switch ((int)probe_knob("NICE_FD2_VD", 0)) {
            case 1100: return launch_cfg<Cfg<B_, ND_, NE_, NE2_, 0, big_wg(B_), 1024>>(p, num_cus, s);
            case 1101: return launch_cfg<Cfg<B_, ND_, NE_, NE2_, 0, big_wg(B_), 1025>>(p, num_cus, s);
            case 1102: return launch_cfg<Cfg<B_, ND_, NE_, NE2_, 0, big_wg(B_), 1026>>(p, num_cus, s);
            case 1103: return launch_cfg<Cfg<B_, ND_, NE_, NE2_, 0, big_wg(B_), 1027>>(p, num_cus, s);
            case 1117: return launch_cfg<Cfg<B_, ND_, NE_, NE2_, 0, big_wg(B_), 1041>>(p, num_cus, s);
            case 1118: return launch_cfg<Cfg<B_, ND_, NE_, NE2_, 0, big_wg(B_), 1042>>(p, num_cus, s);
            default: break;
            }
        }
        // Sibling lanes (Cfg::SIB) A/B: NICE_FD2_SIB = 1: the round-4 kernel
        // (no siblings); 31 / 131 / 132 / 141 / 142 / 143 / 144 / 121: M = 3
        // or 2 siblings at the VALU decode / lookup grouping in the cases
        if constexpr (B_ == 40) {
            constexpr int VL = valu_limbs_big(B_, ND_, NE_);
            switch ((int)probe_knob("NICE_FD2_SIB", 0)) {
            case 1: return launch_cfg<Cfg<B_, ND_, NE_, NE2_, 0, big_wg(B_), VL>>(p, num_cus, s);
            case 31: return launch_cfg<Cfg<B_, ND_, NE_, NE2_, 0, 512, VL, 1, 0, 3>>(p, num_cus, s);
            case 131: return launch_cfg<Cfg<B_, ND_, NE_, NE2_, 0, 512, 0, 1, 0, 3>>(p, num_cus, s);
            case 132: return launch_cfg<Cfg<B_, ND_, NE_, NE2_, 0, 512, 0, 100, 0, 3>>(p, num_cus, s);
            case 141: return launch_cfg<Cfg<B_, ND_, NE_, NE2_, 0, 512, 4097, 1, 0, 3>>(p, num_cus, s);
            case 142: return launch_cfg<Cfg<B_, ND_, NE_, NE2_, 0, 512, 4097, 100, 0, 3>>(p, num_cus, s);
            case 143: return launch_cfg<Cfg<B_, ND_, NE_, NE2_, 0, 512, 4098, 1, 0, 3>>(p, num_cus, s);
            case 144: return launch_cfg<Cfg<B_, ND_, NE_, NE2_, 0, 512, 4113, 1, 0, 3>>(p, num_cus, s);
            case 121: return launch_cfg<Cfg<B_, ND_, NE_, NE2_, 0, 512, 4097, 1, 0, 2>>(p, num_cus, s);
            default: break;
            }
        }
        // Persistent grid A/B (NICE_FD2_PERS = 1: on, 2: off; 3 / 4: 1024-thread
        // workgroups with / without it, where the LDS and VGPRs allow one)
        if constexpr (waves_at(B_, 1024) >= 4) {
            switch ((int)probe_knob("NICE_FD2_PERS", 0)) {
            case 3: return launch_cfg<Cfg<B_, ND_, NE_, NE2_, 0, 1024, valu_limbs(B_), -1, 1>>(p, num_cus, s);
            case 4: return launch_cfg<Cfg<B_, ND_, NE_, NE2_, 0, 1024, valu_limbs(B_), -1, 0>>(p, num_cus, s);
            default: break;
            }
        }
        switch ((int)probe_knob("NICE_FD2_PERS", 0)) {
        case 1:
            return wg512 ? launch_cfg<Cfg<B_, ND_, NE_, NE2_, 0, 512, valu_limbs(B_), -1, 1>>(p, num_cus, s)
                         : launch_cfg<Cfg<B_, ND_, NE_, NE2_, 0, big_wg(B_), valu_limbs(B_), -1, 1>>(p, num_cus, s);
        case 2:
            return wg512 ? launch_cfg<Cfg<B_, ND_, NE_, NE2_, 0, 512, valu_limbs(B_), -1, 0>>(p, num_cus, s)
                         : launch_cfg<Cfg<B_, ND_, NE_, NE2_, 0, big_wg(B_), valu_limbs(B_), -1, 0>>(p, num_cus, s);
        default: break;
        }
        // Lookup-group sweep of the three-mask-word bases (NICE_FD2_LG = LG,
        // at the production VALU-decoded limbs of fields >= 1e7)
        if constexpr ((B_ + 31) / 32 == 3) {
            constexpr int VL = valu_limbs_big(B_, ND_, NE_), WGB = big_wg(B_);
            switch ((int)probe_knob("NICE_FD2_LG", 100000)) {
            case 0: return launch_cfg<Cfg<B_, ND_, NE_, NE2_, 0, WGB, VL, 0>>(p, num_cus, s);
            case 5: return launch_cfg<Cfg<B_, ND_, NE_, NE2_, 0, WGB, VL, 5>>(p, num_cus, s);
            case 6: return launch_cfg<Cfg<B_, ND_, NE_, NE2_, 0, WGB, VL, 6>>(p, num_cus, s);
            case 7: return launch_cfg<Cfg<B_, ND_, NE_, NE2_, 0, WGB, VL, 7>>(p, num_cus, s);
            case 8: return launch_cfg<Cfg<B_, ND_, NE_, NE2_, 0, WGB, VL, 8>>(p, num_cus, s);
            case 10: return launch_cfg<Cfg<B_, ND_, NE_, NE2_, 0, WGB, VL, 10>>(p, num_cus, s);
            case 12: return launch_cfg<Cfg<B_, ND_, NE_, NE2_, 0, WGB, VL, 12>>(p, num_cus, s);
            default: break;
            }
        }
#endif
        // b40 fields >= 1e7: three sibling lanes (Cfg::SIB, fd2_kernel.hpp):
        // on the first limb layout (the range's first ~29 %, the benchmark
        // fields) pipelined with the lowest C limb above the shared one
        // decoded by VALU, elsewhere per-sibling lookup groups, no VALU decode
        // (profiles/r05/sib_sweep_range.log)
        if constexpr (B_ == 40) {
            if (!wg512) {
                if constexpr (ND_ == 4) return launch_cfg<Cfg<B_, ND_, NE_, NE2_, 0, 512, 4097, 100, 0, 3>>(p, num_cus, s);
                else return launch_cfg<Cfg<B_, ND_, NE_, NE2_, 0, 512, 0, 1, 0, 3>>(p, num_cus, s);
            }
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
