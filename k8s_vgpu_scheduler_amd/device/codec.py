"""Wire codecs for node and pod annotations (byte-compatible with HAMi).

Reference: pkg/device/devices.go:317-556 and docs/develop/protocol.md.
  node registration  JSON ``[DeviceInfo]`` (MarshalNodeDevices :422-443), legacy
                     CSV ``id,count,mem,core,type,numa,health[,index,mode]:``
  pod allocation     ``uuid,type,mem,cores:`` per device, ``;`` per container,
                     init containers first; empty entries are KEPT on decode so
                     annotation index == container index (devices.go:546-551)
  pair scores        JSON ``[{"uuid":..,"score":{peer:int}}]``
New for AMD (no reference equivalent): the CU-range annotation
``uuid=lo-hi,lo-hi:`` per device, ``;`` per container, produced by the
scheduler's CU-bitmap allocator and consumed by the device plugin to build
``HSA_CU_MASK``.
"""

from __future__ import annotations

import json

from .types import ContainerDevice, DeviceInfo

DEV_SEP = ":"   # OneContainerMultiDeviceSplitSymbol
CTR_SEP = ";"   # OnePodMultiContainerSplitSymbol


class CodecError(ValueError):
    pass


def _go_bool(s: str) -> bool:
    if s in ("1", "t", "T", "TRUE", "true", "True"):
        return True
    if s in ("0", "f", "F", "FALSE", "false", "False"):
        return False
    raise CodecError(f"invalid health field: {s!r}")


def _int(s: str, what: str) -> int:
    try:
        v = int(s)
    except ValueError as e:
        raise CodecError(f"invalid {what} field: {s!r}") from e
    if not -(2 ** 31) <= v < 2 ** 31:
        raise CodecError(f"invalid {what} field: {s!r} out of int32 range")
    return v


# ------------------------------------------------------------------ node side
def decode_node_devices(s: str) -> list[DeviceInfo]:
    if DEV_SEP not in s:
        raise CodecError("node annotation missing device separator")
    out = []
    for seg in s.split(DEV_SEP):
        if seg == "":
            continue
        if "," not in seg:
            raise CodecError(f"malformed node annotation segment: {seg!r}")
        items = seg.split(",")
        if len(items) not in (7, 9):
            raise CodecError(f"unexpected field count {len(items)} in node annotation")
        d = DeviceInfo(id=items[0], count=_int(items[1], "count"), devmem=_int(items[2], "memory"),
                       devcore=_int(items[3], "core"), type=items[4], numa=_int(items[5], "numa"),
                       health=_go_bool(items[6]), mode="hami-core", index=0)
        if len(items) == 9:
            idx = _int(items[7], "index")
            if idx < 0:
                raise CodecError(f"index field must not be negative: {idx}")
            d.index, d.mode = idx, items[8]
        out.append(d)
    return out


def encode_node_devices(devs: list[DeviceInfo]) -> str:
    return "".join(
        f"{d.id},{d.count},{d.devmem},{d.devcore},{d.type},{d.numa},{'true' if d.health else 'false'},"
        f"{d.index},{d.mode}{DEV_SEP}" for d in devs)


def marshal_node_devices(devs: list[DeviceInfo]) -> str:
    """JSON registration payload; customInfo deliberately excluded (devices.go:419-443)."""
    return json.dumps([d.to_json() for d in devs], separators=(",", ":"))


def unmarshal_node_devices(s: str) -> list[DeviceInfo]:
    try:
        arr = json.loads(s)
    except json.JSONDecodeError as e:
        raise CodecError(str(e)) from e
    if arr is None:
        return []
    if not isinstance(arr, list):
        raise CodecError("registration annotation is not a JSON array")
    return [DeviceInfo.from_json(x or {}) for x in arr]


def encode_pair_scores(scores: dict[str, dict[str, int]]) -> str:
    return json.dumps([{"uuid": u, "score": dict(sorted(s.items()))} for u, s in sorted(scores.items())],
                      separators=(",", ":"))


def decode_pair_scores(s: str) -> dict[str, dict[str, int]]:
    try:
        arr = json.loads(s)
    except json.JSONDecodeError as e:
        raise CodecError(str(e)) from e
    out = {}
    for e in arr or []:
        out[e.get("uuid", "")] = {k: int(v) for k, v in (e.get("score") or {}).items()}
    return out


# ------------------------------------------------------------------- pod side
def encode_container_devices(cd: list[ContainerDevice]) -> str:
    return "".join(f"{d.uuid},{d.type},{d.usedmem},{d.usedcores}{DEV_SEP}" for d in cd)


def encode_container_device_type(cd: list[ContainerDevice], t: str) -> str:
    return DEV_SEP.join(f"{d.uuid},{d.type},{d.usedmem},{d.usedcores}" for d in cd if d.type == t)


def encode_pod_single_device(pd: list) -> str:
    return "".join(encode_container_devices(c) + CTR_SEP for c in pd)


def encode_pod_devices(checklist: dict, pd: dict) -> dict:
    return {checklist[t]: encode_pod_single_device(single) for t, single in pd.items()}


def decode_container_devices(s: str) -> list[ContainerDevice]:
    if not s:
        return []
    out = []
    for val in s.split(DEV_SEP):
        if "," not in val:
            continue
        f = val.split(",")
        if len(f) < 4:
            raise CodecError("pod annotation format error, missing fields, do not use nodeName in task spec")
        out.append(ContainerDevice(uuid=f[0], type=f[1], usedmem=_int(f[2], "memory"),
                                   usedcores=_int(f[3], "core")))
    return out


def decode_pod_devices(checklist: dict, annos: dict) -> dict:
    if not annos:
        return {}
    pd = {}
    for dev_type, key in checklist.items():
        s = annos.get(key)
        if s is None:
            continue
        # Keep empty entries: index == container index (init first).
        pd[dev_type] = [decode_container_devices(part) for part in s.split(CTR_SEP)]
    return pd


# --------------------------------------------------------------- CU ranges
def format_ranges(ranges) -> str:
    return ",".join(f"{a}-{b}" if b != a else f"{a}" for a, b in ranges)


def parse_ranges(s: str) -> list[tuple[int, int]]:
    out = []
    for part in s.split(","):
        part = part.strip()
        if not part:
            continue
        if "-" in part:
            a, b = part.split("-", 1)
            lo, hi = int(a), int(b)
        else:
            lo = hi = int(part)
        if lo < 0 or hi < lo:
            raise CodecError(f"bad CU range {part!r}")
        out.append((lo, hi))
    return out


def merge_ranges(ranges) -> list[tuple[int, int]]:
    """Union of CU ranges, sorted and coalesced."""
    out: list[list[int]] = []
    for a, b in sorted((int(a), int(b)) for a, b in ranges):
        if out and a <= out[-1][1] + 1:
            out[-1][1] = max(out[-1][1], b)
        else:
            out.append([a, b])
    return [(a, b) for a, b in out]


def ranges_count(ranges) -> int:
    return sum(b - a + 1 for a, b in ranges)


def encode_cu_ranges(pd_single: list) -> str:
    """Per container (``;``), per device (``:``) ``uuid=lo-hi,..``; devices with
    no recorded ranges (whole-device or non-AMD) are omitted."""
    parts = []
    for ctr in pd_single:
        segs = []
        for d in ctr:
            r = (d.custominfo or {}).get("cu_ranges")
            if r:
                segs.append(f"{d.uuid}={format_ranges(r)}")
        parts.append(DEV_SEP.join(segs) + CTR_SEP)
    return "".join(parts)


def decode_cu_ranges(s: str) -> list[dict[str, list]]:
    """-> per container: {uuid: [(lo, hi), ...]} (empty containers kept; a
    pod with no containers encodes to "" and decodes back to [])."""
    if not s:
        return []
    out = []
    for ctr in s.split(CTR_SEP)[:-1] if s.endswith(CTR_SEP) else s.split(CTR_SEP):
        m = {}
        for seg in ctr.split(DEV_SEP):
            if "=" not in seg:
                continue
            u, r = seg.split("=", 1)
            m[u] = parse_ranges(r)
        out.append(m)
    return out


def attach_cu_ranges(pd_single: list, s: str | None):
    """Copy ranges from a decoded CU annotation onto decoded ContainerDevices."""
    if not s:
        return pd_single
    per = decode_cu_ranges(s)
    for i, ctr in enumerate(pd_single):
        if i >= len(per):
            break
        for d in ctr:
            if d.uuid in per[i]:
                d.custominfo = dict(d.custominfo or {})
                d.custominfo["cu_ranges"] = per[i][d.uuid]
    return pd_single
