"""codemode -- mirror of blobstore/common/codemode/codemode.go (Tactic table and
stripe layout helpers).  Pure host bookkeeping; the same table is compiled into
libcfsec.so (cfsec_codemode_tactic) and tests/test_codemode.py checks both agree.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Optional, Tuple

# codemode.go:26-44
EC15P12 = 1
EC6P6 = 2
EC16P20L2 = 3
EC6P10L2 = 4
EC6P3L3 = 5
EC6P6Align0 = 6
EC6P6Align512 = 7
EC4P4L2 = 8
EC12P4 = 9
EC16P4 = 10
EC3P3 = 11
EC10P4 = 12
EC6P3 = 13
EC12P9 = 14
EC6P6L9 = 200
EC6P8L10 = 201

_ALIGN_0B, _ALIGN_512B, _ALIGN_2KB = 0, 512, 2048


@dataclass(frozen=True)
class Tactic:
    """codemode.Tactic (codemode.go:129-163)."""

    N: int = 0
    M: int = 0
    L: int = 0
    AZCount: int = 0
    PutQuorum: int = 0
    GetQuorum: int = 0
    MinShardSize: int = 0

    def IsValid(self) -> bool:  # codemode.go:267-271
        return (self.N > 0 and self.M > 0 and self.L >= 0 and self.AZCount > 0 and self.PutQuorum > 0
                and self.GetQuorum >= 0 and self.MinShardSize >= 0 and self.N % self.AZCount == 0
                and self.M % self.AZCount == 0 and self.L % self.AZCount == 0)

    def GetECLayoutByAZ(self) -> List[List[int]]:  # codemode.go:274-291
        n, m, l = self.N // self.AZCount, self.M // self.AZCount, self.L // self.AZCount
        out = []
        for idx in range(self.AZCount):
            stripe = [idx * n + i for i in range(n)]
            stripe += [self.N + idx * m + i for i in range(m)]
            stripe += [self.N + self.M + idx * l + i for i in range(l)]
            out.append(stripe)
        return out

    def GlobalStripe(self) -> Tuple[List[int], int, int]:  # codemode.go:294-300
        return list(range(self.N + self.M)), self.N, self.M

    def AllLocalStripe(self) -> Tuple[Optional[List[List[int]]], int, int]:  # codemode.go:303-310
        if self.L == 0:
            return None, 0, 0
        n, m, l = self.N // self.AZCount, self.M // self.AZCount, self.L // self.AZCount
        return self.GetECLayoutByAZ(), n + m, l

    def LocalStripe(self, index: int):  # codemode.go:313-331
        if self.L == 0:
            return None, 0, 0
        n, m, l = self.N // self.AZCount, self.M // self.AZCount, self.L // self.AZCount
        if index < self.N:
            az = index // n
        elif index < self.N + self.M:
            az = (index - self.N) // m
        elif index < self.N + self.M + self.L:
            az = (index - self.N - self.M) // l
        else:
            return None, 0, 0
        return self.LocalStripeInAZ(az)

    def LocalStripeInAZ(self, az_index: int):  # codemode.go:334-345
        if self.L == 0:
            return None, 0, 0
        n, m, l = self.N // self.AZCount, self.M // self.AZCount, self.L // self.AZCount
        stripes = self.GetECLayoutByAZ()
        if az_index < 0 or az_index >= len(stripes):
            return None, 0, 0
        return list(stripes[az_index]), n + m, l


# codemode.go:56-79
_TACTICS = {
    EC15P12: Tactic(15, 12, 0, 3, 24, 0, _ALIGN_2KB),
    EC6P6: Tactic(6, 6, 0, 3, 11, 0, _ALIGN_2KB),
    EC12P9: Tactic(12, 9, 0, 3, 20, 0, _ALIGN_2KB),
    EC16P20L2: Tactic(16, 20, 2, 2, 34, 0, _ALIGN_2KB),
    EC6P10L2: Tactic(6, 10, 2, 2, 14, 0, _ALIGN_2KB),
    EC12P4: Tactic(12, 4, 0, 1, 15, 0, _ALIGN_2KB),
    EC16P4: Tactic(16, 4, 0, 1, 19, 0, _ALIGN_2KB),
    EC3P3: Tactic(3, 3, 0, 1, 5, 0, _ALIGN_2KB),
    EC10P4: Tactic(10, 4, 0, 1, 13, 0, _ALIGN_2KB),
    EC6P3: Tactic(6, 3, 0, 1, 8, 0, _ALIGN_2KB),
    EC6P3L3: Tactic(6, 3, 3, 3, 9, 0, _ALIGN_2KB),
    EC6P6Align0: Tactic(6, 6, 0, 3, 11, 0, _ALIGN_0B),
    EC6P6Align512: Tactic(6, 6, 0, 3, 11, 0, _ALIGN_512B),
    EC4P4L2: Tactic(4, 4, 2, 2, 6, 0, _ALIGN_2KB),
    EC6P6L9: Tactic(6, 6, 9, 3, 11, 0, _ALIGN_2KB),
    EC6P8L10: Tactic(6, 8, 10, 2, 13, 0, _ALIGN_0B),
}

_NAMES = {
    EC15P12: "EC15P12", EC6P6: "EC6P6", EC16P20L2: "EC16P20L2", EC6P10L2: "EC6P10L2",
    EC6P3L3: "EC6P3L3", EC6P6Align0: "EC6P6Align0", EC6P6Align512: "EC6P6Align512",
    EC4P4L2: "EC4P4L2", EC12P4: "EC12P4", EC16P4: "EC16P4", EC3P3: "EC3P3", EC10P4: "EC10P4",
    EC6P3: "EC6P3", EC6P6L9: "EC6P6L9", EC6P8L10: "EC6P8L10", EC12P9: "EC12P9",
}


def GetTactic(mode: int) -> Tactic:
    """CodeMode.Tactic() (codemode.go:208-213); raises ValueError where Go panics."""
    if mode not in _TACTICS:
        raise ValueError(f"Invalid codemode:{mode}")
    return _TACTICS[mode]


def Name(mode: int) -> str:
    if mode not in _NAMES:
        raise ValueError(f"codemode: {mode} is invalid")
    return _NAMES[mode]


def ByName(name: str) -> int:
    for k, v in _NAMES.items():
        if v == name:
            return k
    raise ValueError(f"codemode: {name} is invalid")


def IsValid(mode: int) -> bool:
    return mode in _NAMES


def GetShardNum(mode: int) -> int:
    t = GetTactic(mode)
    return t.N + t.M + t.L


def GetAllCodeModes() -> List[int]:  # codemode.go:348-366
    return [EC15P12, EC6P6, EC16P20L2, EC6P10L2, EC6P3L3, EC6P6Align0, EC6P6Align512, EC4P4L2,
            EC12P4, EC16P4, EC3P3, EC10P4, EC6P3, EC6P6L9, EC6P8L10]
