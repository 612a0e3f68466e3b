"""Host DRAM bandwidth of the feed path's copy: T threads each memcpy a private slice of a large
pageable source into a pinned destination (the staging copy of the pageable path), optionally
bound to one NUMA node's CPUs.  Prints GB/s of copied bytes (each byte is read once and written
once, so DRAM traffic is >= 2x that, 3x with write-allocate)."""
import ctypes
import json
import os
import sys
import threading
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "neptune-core_amd"))
import neptune_hip as nh  # noqa: E402
import neptune_hip._lib as L  # noqa: E402


def run(threads, nbytes, cpus, reps=3):
    lib = L.load()
    src = np.ones(nbytes // 8, dtype=np.uint64)
    h = ctypes.c_void_p()
    L.check(lib.nhip_host_alloc(nbytes, ctypes.byref(h)), "nhip_host_alloc")
    dst = np.frombuffer((ctypes.c_uint64 * (nbytes // 8)).from_address(h.value), dtype=np.uint64)
    dst[:] = 0
    per = (nbytes // 8) // threads
    best = 0.0
    for _ in range(reps):
        bar = threading.Barrier(threads + 1)

        def work(i):
            if cpus:
                os.sched_setaffinity(0, cpus)
            bar.wait()
            np.copyto(dst[i * per:(i + 1) * per], src[i * per:(i + 1) * per])
            bar.wait()

        ts = [threading.Thread(target=work, args=(i,)) for i in range(threads)]
        for t in ts:
            t.start()
        bar.wait()
        t0 = time.perf_counter()
        bar.wait()
        dt = time.perf_counter() - t0
        for t in ts:
            t.join()
        best = max(best, per * threads * 8 / dt)
    lib.nhip_host_free(h.value)
    return best / 1e9


def main():
    ctx = nh.Context(0)
    topo = ctx.numa()
    ctx.close()
    nbytes = int(os.environ.get("MEMBW_BYTES", str(2 << 30)))
    out = {"gpu_numa_node": topo["node"], "node_cpus": len(topo["cpus"]), "allowed_cpus": len(os.sched_getaffinity(0)),
           "bytes": nbytes, "GBps_copied": {}}
    for t in (1, 2, 4, 8, 16):
        out["GBps_copied"][f"{t}_unbound"] = run(t, nbytes, None)
        if topo["cpus"]:
            out["GBps_copied"][f"{t}_bound"] = run(t, nbytes, topo["cpus"])
    print(json.dumps(out))


if __name__ == "__main__":
    main()
