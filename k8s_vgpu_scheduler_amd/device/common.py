"""Fit-failure reason codes and the "n/N Reason" wire form (pkg/device/common/common.go:25-70)."""

from __future__ import annotations

import re

CARD_TYPE_MISMATCH = "CardTypeMismatch"
CARD_UUID_MISMATCH = "CardUuidMismatch"
CARD_TIME_SLICING_EXHAUSTED = "CardTimeSlicingExhausted"
CARD_COMPUTE_UNITS_EXHAUSTED = "CardComputeUnitsExhausted"
CARD_INSUFFICIENT_MEMORY = "CardInsufficientMemory"
CARD_INSUFFICIENT_CORE = "CardInsufficientCore"
CARD_NOT_HEALTH = "CardNotHealth"
CARD_CORDONED = "CardCordoned"
NUMA_NOT_FIT = "NumaNotFit"
EXCLUSIVE_DEVICE_ALLOCATE_CONFLICT = "ExclusiveDeviceAllocateConflict"
CARD_NOT_FOUND_CUSTOM_FILTER_RULE = "CardNotFoundCustomFilterRule"
CARD_CU_FRAGMENTED = "CardComputeUnitsFragmented"   # AMD: no contiguous CU run of the size
NODE_INSUFFICIENT_DEVICE = "NodeInsufficientDevice"
ALLOCATED_CARDS_INSUFFICIENT_REQUEST = "AllocatedCardsInsufficientRequest"
NODE_UNFIT_POD = "NodeUnfitPod"
NODE_FIT_POD = "NodeFitPod"
RESOURCE_QUOTA_NOT_FIT = "ResourceQuotaNotFit"
MODE_NOT_FIT = "ModeNotFit"


def gen_reason(reasons: dict[str, int], cards: int) -> str:
    return ", ".join(sorted(f"{cnt}/{cards} {r}" for r, cnt in reasons.items()))


_RE = re.compile(r"^\s*(\d+)/(\d+)\s+(\S+)")


def parse_reason(reason: str) -> dict[str, int]:
    out = {}
    for part in reason.split(", "):
        m = _RE.match(part)
        if m:
            out[m.group(3)] = int(m.group(1))
    return out
