"""Host DRAM bandwidth of the feed path's staging copy, with page placement controlled.

T threads each copy a private slice of a large pageable source (a Vec's words) into pinned memory
placed on the GPU's NUMA node (nhip_host_alloc_near: the context's staging).  The source pages are
first-touched by threads bound to the GPU's node ("local") or to another node ("remote"); the copy
threads run bound to the GPU's node or unbound.  Each byte copied is one DRAM read plus one DRAM
write (plus a read-for-ownership of the destination for ordinary stores; numpy's copy is memcpy);
the DMA engine then reads the staging once more.  Prints copied GB/s per case and the page nodes
actually obtained (nhip_host_page_node), for the 8-GPU budget of DESIGN.md §6."""
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


def node_cpus(n):
    try:
        with open(f"/sys/devices/system/node/node{n}/cpulist") as f:
            lst = f.read().strip()
    except OSError:
        return []
    out = []
    for part in lst.split(","):
        if "-" in part:
            a, b = part.split("-")
            out += list(range(int(a), int(b) + 1))
        elif part:
            out.append(int(part))
    allowed = os.sched_getaffinity(0)
    return [c for c in out if c in allowed]


def parallel(threads, cpus, fn):
    bar = threading.Barrier(threads + 1)

    def work(i):
        if cpus:
            os.sched_setaffinity(0, cpus)
        bar.wait()
        fn(i)
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
    return dt


def main():
    lib = L.load()
    ctx = nh.Context(0)
    topo = ctx.numa()
    gnode = topo["node"]
    nodes = sorted(int(d[4:]) for d in os.listdir("/sys/devices/system/node") if d.startswith("node") and d[4:].isdigit())
    other = next((n for n in nodes if n != gnode and node_cpus(n)), None)
    nbytes = int(os.environ.get("MEMBW_BYTES", str(2 << 30)))
    words = nbytes // 8
    h = ctypes.c_void_p()
    L.check(lib.nhip_host_alloc_near(ctx.handle, nbytes, ctypes.byref(h)), "nhip_host_alloc_near")
    dst = np.frombuffer((ctypes.c_uint64 * words).from_address(h.value), dtype=np.uint64)
    dst[:] = 0
    out = {"gpu_numa_node": gnode, "numa_nodes": nodes, "gpu_node_cpus": len(topo["cpus"]),
           "allowed_cpus": len(os.sched_getaffinity(0)), "bytes": nbytes,
           "staging_page_node": lib.nhip_host_page_node(ctypes.c_void_p(h.value)), "cases": {}}
    for where, touch_node in (("local", gnode), ("remote", other)):
        if touch_node is None or touch_node < 0:
            continue
        src = np.empty(words, dtype=np.uint64)
        per_t = words // 16
        parallel(16, node_cpus(touch_node), lambda i: src[i * per_t:(i + 1) * per_t].fill(i + 1))
        src_node = lib.nhip_host_page_node(ctypes.c_void_p(src.ctypes.data + nbytes // 2))
        for threads in (4, 8, 16):
            per = words // threads
            binds = [("bound", node_cpus(gnode)), ("unbound", None)]
            if touch_node != gnode:
                binds.append(("on_src_node", node_cpus(touch_node)))
            for bname, cpus in binds:
                best = 0.0
                for _ in range(3):
                    dt = parallel(threads, cpus,
                                  lambda i: np.copyto(dst[i * per:(i + 1) * per], src[i * per:(i + 1) * per]))
                    best = max(best, per * threads * 8 / dt / 1e9)
                out["cases"][f"src_{where}(node {src_node})_{threads}t_{bname}"] = round(best, 1)
        del src
    lib.nhip_host_free(ctypes.c_void_p(h.value))
    ctx.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
