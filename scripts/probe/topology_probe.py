"""GPU-box probe: the node's GPU topology as both discovery backends see it.

Dumps (JSON, stdout):
  * the KFD topology tree: every node's properties and io_links (type,
    weight, min/max bandwidth, node_to) -- the sysfs backend's source and a
    real 8 x MI355X fixture for the CPU tests (tests/fixtures/);
  * amd-smi per processor: identity (uuid, enumeration, board, asic, kfd) and,
    for every ordered pair, link type / hops / weight / min-max bandwidth /
    p2p status, plus link_metrics.
No GPU work is submitted.
"""

import json
import os
import sys
from pathlib import Path

KFD = Path("/sys/class/kfd/kfd/topology/nodes")


def props(p: Path) -> dict:
    out = {}
    try:
        for line in p.read_text().splitlines():
            k, _, v = line.partition(" ")
            try:
                out[k] = int(v)
            except ValueError:
                out[k] = v
    except OSError as e:
        out["_error"] = str(e)
    return out


def kfd_tree() -> dict:
    nodes = {}
    for n in sorted(KFD.iterdir(), key=lambda p: int(p.name)):
        d = {"properties": props(n / "properties")}
        try:
            d["gpu_id"] = int((n / "gpu_id").read_text().strip() or 0)
        except (OSError, ValueError):
            d["gpu_id"] = None
        try:
            d["name"] = (n / "name").read_text().strip()
        except OSError:
            pass
        links = {}
        for kind in ("io_links", "p2p_links"):
            base = n / kind
            if base.is_dir():
                links[kind] = {l.name: props(l / "properties") for l in sorted(base.iterdir())}
        d.update(links)
        nodes[n.name] = d
    return nodes


def jsonable(v):
    if isinstance(v, dict):
        return {str(k): jsonable(x) for k, x in v.items()}
    if isinstance(v, (list, tuple)):
        return [jsonable(x) for x in v]
    if isinstance(v, (int, float, str, bool)) or v is None:
        return v
    return str(v)


def amdsmi_view() -> dict:
    import amdsmi
    amdsmi.amdsmi_init()
    hs = amdsmi.amdsmi_get_processor_handles()
    out = {"count": len(hs), "link_type_enum": {x.name: int(x) for x in amdsmi.AmdSmiLinkType}, "gpus": []}

    def q(fn, *a):
        try:
            return jsonable(getattr(amdsmi, fn)(*a))
        except Exception as e:  # noqa: BLE001
            return f"ERR {e}"
    for h in hs:
        out["gpus"].append({fn: q(fn, h) for fn in (
            "amdsmi_get_gpu_device_uuid", "amdsmi_get_gpu_enumeration_info", "amdsmi_get_gpu_board_info",
            "amdsmi_get_gpu_asic_info", "amdsmi_get_gpu_kfd_info", "amdsmi_get_gpu_device_bdf",
            "amdsmi_get_gpu_compute_partition", "amdsmi_get_gpu_memory_partition", "amdsmi_get_gpu_xgmi_info",
            "amdsmi_topo_get_numa_node_number")})
    pairs = []
    for i, a in enumerate(hs):
        for j, b in enumerate(hs):
            if i == j:
                continue
            pairs.append({"src": i, "dst": j, "link_type": q("amdsmi_topo_get_link_type", a, b),
                          "weight": q("amdsmi_topo_get_link_weight", a, b),
                          "minmax_bw": q("amdsmi_get_minmax_bandwidth_between_processors", a, b),
                          "p2p": q("amdsmi_topo_get_p2p_status", a, b)})
    out["pairs"] = pairs
    out["link_metrics_0"] = q("amdsmi_get_link_metrics", hs[0]) if hs else None
    return out


def main():
    res = {"kfd": kfd_tree()}
    try:
        res["amdsmi"] = amdsmi_view()
    except Exception as e:  # noqa: BLE001
        res["amdsmi"] = f"ERR {e}"
    res["env"] = {k: os.environ.get(k) for k in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES")}
    json.dump(res, sys.stdout, indent=1)


if __name__ == "__main__":
    main()
