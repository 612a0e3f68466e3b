// Host NUMA topology of a GPU and pinned memory placed on it (host_numa.cpp).
#pragma once
#include <hip/hip_runtime.h>

#include <string>
#include <vector>

namespace nhip {

struct HostTopo {
    int numa_node = -1;     // -1: the platform reports none
    std::vector<int> cpus;  // the node's CPUs this process may run on (empty: unknown)
    std::string bus_id;     // the device's PCI bus id
};

// "0-3,8,10-11" (kernel cpulist syntax, "a-b:stride" included) -> sorted CPU ids
bool parse_cpulist(const char* s, std::vector<int>& out);
// <root>/bus/pci/devices/<bus_id>/numa_node and <root>/devices/system/node/node<N>/cpulist
HostTopo topo_from_sysfs(const char* root, const char* bus_id);
// the topology of HIP device `device` from /sys, limited to this process's allowed CPUs
HostTopo device_topo(int device);
// NHIP_NUMA unset or non-zero
bool numa_enabled();
// the operator's NHIP_HOST_THREADS (0 = unset): host copy threads per upload / ingest, taking
// precedence over the count a group sets per member (nhip_set_host_threads)
unsigned host_threads_env();
// bind the calling thread to `cpus` (no-op when empty or disabled); true if bound
bool bind_thread(const std::vector<int>& cpus);
// pinned host memory (hipHostMalloc `flags`) with its pages on `node` (< 0 or disabled: no placement)
hipError_t host_malloc_on(void** p, size_t bytes, int node, unsigned flags);
// the NUMA node holding the page at p (-1 if unknown)
int page_node(const void* p);

}  // namespace nhip
