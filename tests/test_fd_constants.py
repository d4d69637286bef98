"""Host-side checks of the FD kernel's carry arithmetic (nice_amd/csrc/
fd2_kernel.hpp, Cfg::C1): the carry (0..4) out of a C limb sum t < ES (5B + 4)
is ONE multiply-high by MAGIC = ceil(2^32 / (ES B)), because t is always a
multiple of the table entry size ES.  Checked exhaustively over every
multiple of ES for every base with an FD instantiation (no GPU needed)."""
import pytest

FD_BASES = [40, 42, 43, 44, 45, 47, 48, 49, 50, 52, 53, 54, 55, 57, 58, 59, 60, 62, 63, 64, 65, 67, 68, 80]


def entry_size(base):
    mw = (base + 31) // 32
    return 4 if mw == 1 else (8 if mw == 2 else 16)


@pytest.mark.parametrize("base", FD_BASES)
def test_c_limb_carry_is_one_multiply_high(base):
    es, B = entry_size(base), base * base
    dc = es * B
    magic = ((1 << 32) + dc - 1) // dc
    e = magic * dc - (1 << 32)
    tmax = es * (5 * B + 4)
    # the kernel's compile-time condition (u e < 2^32 with t = ES u) ...
    assert e * (tmax // es) < 1 << 32
    # ... and what it promises, for every t the chain can produce
    for t in range(0, tmax + 1, es):
        assert (t * magic) >> 32 == t // dc, (base, t)
