"""A/B of the HBM stream copy under the shim: which part of the shim costs
bandwidth.  Rounds alternate the variants (ABCD DCBA ...), best of each."""
import json
import os
import sys
import tempfile

from k8s_vgpu_scheduler_amd.shim.probe import run_child

tmp = tempfile.mkdtemp(prefix="mivgpu-hs-")
variants = {
    "native": ({}, False),
    "shim": ({"MIVGPU_SHARED_CACHE": os.path.join(tmp, "a.cache")}, True),
    "shim_no_occ": ({"MIVGPU_SHARED_CACHE": os.path.join(tmp, "b.cache"), "MIVGPU_OCCUPANCY": "0"}, True),
    "shim_no_region": ({}, True),
}
names = list(variants)
res = {n: [] for n in names}
for rnd in range(int(sys.argv[1]) if len(sys.argv) > 1 else 3):
    for n in (names if rnd % 2 == 0 else names[::-1]):
        env, shim = variants[n]
        r = run_child("hipstream", env, shim, ["--n", "1024", "--iters", "200"])
        assert r["rc"] == 0, r
        res[n].append(round(r["gbps"], 1))
        print(n, res[n][-1], {k: r.get(k) for k in ("occ_passes", "occ_pass_ms", "occ_pass_max_ms") if k in r},
              flush=True)
print(json.dumps({n: {"runs": v, "best": max(v)} for n, v in res.items()}))
