"""Model test of the shim's HBM hard limit (libmivgpu.so on the mock HIP
runtime, csrc/mockhip): hypothesis generates sequences of hipMalloc,
hipMallocAsync, VMM (hipMemCreate) allocations and free-all, and every
operation must succeed exactly when the container's usage plus the request
fits the limit; ``usage`` and the virtualised ``hipMemGetInfo`` must track the
model after every step.  The reference pins the equivalent C behaviour only
through its Go-side region tests (pkg/monitor/nvidia/v1/spec_test.go)."""

import json
import os
import subprocess

from hypothesis import HealthCheck, given, settings, strategies as st

LIMIT_MIB = 1000

op = st.one_of(st.tuples(st.sampled_from(["alloc", "allocasync", "vmm"]), st.integers(1, 600)),
               st.just(("freeall", None)))


@settings(max_examples=30, deadline=None, suppress_health_check=[HealthCheck.function_scoped_fixture])
@given(st.lists(op, min_size=1, max_size=10))
def test_limit_model(native_build, tmp_path_factory, ops):
    tmp = tmp_path_factory.mktemp("q")
    argv = []
    for name, mib in ops:
        argv += [name] + ([str(mib)] if mib is not None else [])
        argv += ["usage", "meminfo"]
    e = dict(os.environ, MOCKHIP_TOTAL_MIB="65536", MIVGPU_SHARED_CACHE=str(tmp / "c.cache"),
             LD_PRELOAD=str(native_build["shim"]), HIP_DEVICE_MEMORY_LIMIT_0=f"{LIMIT_MIB}m")
    p = subprocess.run([str(native_build["driver"]), *argv], env=e, stdout=subprocess.PIPE,
                       stderr=subprocess.PIPE, text=True, timeout=60)
    assert p.returncode == 0, p.stderr
    out = [json.loads(l) for l in p.stdout.splitlines() if l.startswith("{")]
    used = 0
    i = 0
    for name, mib in ops:
        r = out[i]
        i += 1
        if name != "freeall":
            fits = used + mib <= LIMIT_MIB
            assert (r["rc"] == 0) == fits, (ops, name, mib, used, r)
            if fits:
                used += mib
        else:
            used = 0
        usage, mem = out[i], out[i + 1]
        i += 2
        assert usage["bytes"] == used << 20, (ops, usage, used)
        assert mem["total_mib"] == LIMIT_MIB and mem["free_mib"] == LIMIT_MIB - used, (ops, mem, used)
