"""Per-pod device scoring weights ``hami.io/device-scoring-weights: slot=1,core=1,memory=3``
(pkg/util/device_scoring_weights.go:29-102)."""

from __future__ import annotations

from dataclasses import dataclass

from .types import SCORING_WEIGHTS_ANNOTATION


@dataclass(frozen=True)
class DeviceScoringWeights:
    slot: int = 1
    core: int = 1
    memory: int = 1


DEFAULT_WEIGHTS = DeviceScoringWeights()


def parse_weights(value: str) -> DeviceScoringWeights:
    parts = value.split(",")
    if len(parts) != 3:
        raise ValueError(f"invalid {SCORING_WEIGHTS_ANNOTATION} annotation {value!r}: "
                         "expected slot, core, and memory weights")
    got: dict[str, int] = {}
    for part in parts:
        kv = part.strip().split("=", 1)
        if len(kv) != 2:
            raise ValueError(f"invalid {SCORING_WEIGHTS_ANNOTATION} annotation {value!r}: expected key=value entries")
        key = kv[0].strip()
        if key in got:
            raise ValueError(f"invalid {SCORING_WEIGHTS_ANNOTATION} annotation {value!r}: duplicate {key!r} weight")
        try:
            w = int(kv[1].strip())
        except ValueError as e:
            raise ValueError(f"invalid {SCORING_WEIGHTS_ANNOTATION} annotation {value!r}: "
                             f"{key!r} weight must be an integer") from e
        if w < 0:
            raise ValueError(f"invalid {SCORING_WEIGHTS_ANNOTATION} annotation {value!r}: "
                             f"{key!r} weight must not be negative")
        if key not in ("slot", "core", "memory"):
            raise ValueError(f"invalid {SCORING_WEIGHTS_ANNOTATION} annotation {value!r}: unknown weight {key!r}")
        got[key] = w
    if not any(got.values()):
        raise ValueError(f"invalid {SCORING_WEIGHTS_ANNOTATION} annotation {value!r}: "
                         "at least one weight must be positive")
    return DeviceScoringWeights(got["slot"], got["core"], got["memory"])


def weights_for_pod(pod: dict | None) -> DeviceScoringWeights:
    annos = ((pod or {}).get("metadata") or {}).get("annotations") or {}
    if SCORING_WEIGHTS_ANNOTATION not in annos:
        return DEFAULT_WEIGHTS
    return parse_weights(annos[SCORING_WEIGHTS_ANNOTATION])
