// Host-only dump of launch_sib's stride model (fd2_kernel.hpp) for the
// sibling-lane configurations: ConflictModel cost of every odd L in [lo, hi]
// at a segment [start, start + count), and pick_lane_stride's choice for a
// few targets.  No GPU call is made.
//   hipcc --offload-arch=gfx950 -O2 -std=c++17 -I nice_amd/csrc scripts/ubench/model_dump.hip -o /tmp/model_dump
//   /tmp/model_dump CFG START COUNT [lo hi]     CFG: 40p (b40 first limb layout, pipelined walk),
//                                                40, 42, 43, 44, 45 (three lanes), 47..55 (two lanes)
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include "../../nice_amd/csrc/fd2_kernel.hpp"
using namespace nice;
using namespace nice::fd2;
std::atomic<uint32_t> nice::fd2::g_force_sib_stride{0};  // (defined by fd2_detailed.hip in the library)

static u128 parse_u128(const char *s) {
    u128 v = 0;
    for (; *s; s++) v = v * 10 + (u128)(*s - '0');
    return v;
}

template <class P>
static int dump(u128 start, u64 count, int lo, int hi) {
    const ConflictModel<P> m((long double)start, (long double)count, P::LO + 1);
    printf("# M=%d TCHUNK=%d LG=%d count=%llu\n", (int)P::SIB, P::TCHUNK, (int)P::LG, (unsigned long long)count);
    for (int L = lo | 1; L <= hi; L += 2) printf("L %d cost %.3f\n", L, m.cost((u64)L));
    for (u64 t : {80ull, 100ull, 140ull, 160ull, 240ull})
        printf("pick_lane_stride target %llu: %llu\n", (unsigned long long)t,
               (unsigned long long)pick_lane_stride<P>(start, count, t * 3 / 4, t * 3 / 2, t, P::LO + 1));
    // the lone-field rounds pick (launch_sib, LG >= 100) at 2 x 512-thread
    // workgroups per CU on 256 CUs
    if constexpr (P::SIB > 1) {
        constexpr u64 D = (u64)P::B * P::B, SB = (u64)P::SIB * D;
        double rounds = 0;
        const u64 L = pick_small_stride<P>(start, count, 105, 210, P::LO + 1, count / SB, 262144, D, rounds);
        printf("rounds pick [105, 210]: %llu (%.3f rounds)\n", (unsigned long long)L, rounds);
    }
    return 0;
}

int main(int argc, char **argv) {
    if (argc < 4) return fprintf(stderr, "usage: model_dump CFG START COUNT [lo hi]\n"), 2;
    const char *cfg = argv[1];
    const u128 start = parse_u128(argv[2]);
    const u64 count = (u64)atof(argv[3]);
    const int lo = argc > 4 ? atoi(argv[4]) : 61, hi = argc > 5 ? atoi(argv[5]) : 255;
    if (!strcmp(cfg, "40p")) return dump<Cfg<40, 4, 8, 5, 0, 512, 4097, 100, 0, 3>>(start, count, lo, hi);
    if (!strcmp(cfg, "40")) return dump<Cfg<40, 5, 8, 5, 0, 512, 0, 1, 0, 3>>(start, count, lo, hi);
    if (!strcmp(cfg, "42")) return dump<Cfg<42, 5, 9, 5, 0, 512, 0, 1, 0, 3>>(start, count, lo, hi);
    if (!strcmp(cfg, "44")) return dump<Cfg<44, 5, 9, 5, 0, 512, 0, 1, 0, 3>>(start, count, lo, hi);
    if (!strcmp(cfg, "50")) return dump<Cfg<50, 5, 10, 6, 0, 512, 0, 1, 0, 2>>(start, count, lo, hi);
    fprintf(stderr, "unknown CFG %s\n", cfg);
    return 2;
}
