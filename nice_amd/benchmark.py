"""Offline benchmark fields (common/src/benchmark.rs:10-76)."""
from __future__ import annotations

import enum

from .types import DataToClient


class BenchmarkMode(enum.Enum):
    BASE_TEN = "base-ten"
    DEFAULT = "default"
    LARGE = "large"
    EXTRA_LARGE = "extra-large"
    MASSIVE = "massive"
    HI_BASE = "hi-base"
    MSD_EFFECTIVE = "msd-effective"
    MSD_INEFFECTIVE = "msd-ineffective"


_BASE = {
    BenchmarkMode.BASE_TEN: 10, BenchmarkMode.DEFAULT: 40, BenchmarkMode.LARGE: 40,
    BenchmarkMode.EXTRA_LARGE: 40, BenchmarkMode.MASSIVE: 50, BenchmarkMode.HI_BASE: 80,
    BenchmarkMode.MSD_EFFECTIVE: 50, BenchmarkMode.MSD_INEFFECTIVE: 50,
}
# Sizes as in the code (benchmark.rs:58-66): hi-base is 1e9 there (its doc
# comment and BASELINE.json say 1e6; `hi_base_size` selects), msd-ineffective 1e7.
_SIZE = {
    BenchmarkMode.DEFAULT: 1_000_000, BenchmarkMode.LARGE: 100_000_000,
    BenchmarkMode.EXTRA_LARGE: 1_000_000_000, BenchmarkMode.MASSIVE: 10 ** 13,
    BenchmarkMode.HI_BASE: 1_000_000_000, BenchmarkMode.MSD_EFFECTIVE: 10 ** 12,
    BenchmarkMode.MSD_INEFFECTIVE: 10 ** 7,
}


def get_benchmark_field(mode: BenchmarkMode, hi_base_size: int | None = None) -> DataToClient:
    """get_benchmark_field (benchmark.rs:40-76)."""
    from .api import get_base_range_u128
    base = _BASE[mode]
    br = get_base_range_u128(base)
    if mode is BenchmarkMode.MSD_EFFECTIVE:
        start = 26_507_984_537_059_635
    elif mode is BenchmarkMode.MSD_INEFFECTIVE:
        start = 94_760_515_586_064_977
    else:
        start = br.range_start
    if mode is BenchmarkMode.BASE_TEN:
        size = br.range_size
    elif mode is BenchmarkMode.HI_BASE and hi_base_size is not None:
        size = hi_base_size
    else:
        size = _SIZE[mode]
    return DataToClient(claim_id=0, base=base, range_start=start, range_end=start + size,
                        range_size=size)
