"""Result and range types mirroring the reference's shared types
(common/src/lib.rs).  u128 values are Python ints."""
from __future__ import annotations

import enum
from dataclasses import dataclass, field
from typing import List, Optional


class SearchMode(enum.Enum):
    """SearchMode (common/src/lib.rs:45-52)."""
    DETAILED = "detailed"
    NICEONLY = "niceonly"

    def __str__(self):
        return "Detailed" if self is SearchMode.DETAILED else "Nice-only"


@dataclass(frozen=True)
class FieldSize:
    """Half-open range [range_start, range_end) (common/src/lib.rs:84-153)."""
    range_start: int
    range_end: int

    def __post_init__(self):
        if not self.range_start < self.range_end:
            raise ValueError("Range has invalid bounds, range_start must be < range_end "
                             "(half-open interval)")

    @property
    def range_size(self) -> int:
        return self.range_end - self.range_start

    def first(self) -> int:
        return self.range_start

    def last(self) -> int:
        return self.range_end - 1

    def start(self) -> int:
        return self.range_start

    def end(self) -> int:
        return self.range_end

    def size(self) -> int:
        return self.range_size

    def chunks(self, chunk_size: int) -> List["FieldSize"]:
        out, s = [], self.range_start
        while s < self.range_end:
            e = min(s + chunk_size, self.range_end)
            out.append(FieldSize(s, e))
            s = e
        return out


@dataclass(frozen=True, order=True)
class UniquesDistributionSimple:
    """common/src/lib.rs:166-170."""
    num_uniques: int
    count: int


@dataclass(frozen=True, order=True)
class NiceNumberSimple:
    """common/src/lib.rs:182-186."""
    number: int
    num_uniques: int


@dataclass
class FieldResults:
    """common/src/lib.rs:319-323."""
    distribution: List[UniquesDistributionSimple] = field(default_factory=list)
    nice_numbers: List[NiceNumberSimple] = field(default_factory=list)


@dataclass
class DataToClient:
    """common/src/lib.rs:251-258."""
    claim_id: int
    base: int
    range_start: int
    range_end: int
    range_size: int

    def field(self) -> FieldSize:
        return FieldSize(self.range_start, self.range_end)


@dataclass
class DataToServer:
    """common/src/lib.rs:261-268."""
    claim_id: int
    username: str
    client_version: str
    unique_distribution: Optional[List[UniquesDistributionSimple]]
    nice_numbers: List[NiceNumberSimple]

    def to_json(self) -> dict:
        return {
            "claim_id": self.claim_id,
            "username": self.username,
            "client_version": self.client_version,
            "unique_distribution": None if self.unique_distribution is None else [
                {"num_uniques": d.num_uniques, "count": d.count} for d in self.unique_distribution],
            "nice_numbers": [{"number": n.number, "num_uniques": n.num_uniques}
                             for n in self.nice_numbers],
        }
