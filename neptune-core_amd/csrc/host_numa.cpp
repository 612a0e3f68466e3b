// Host topology of the feed path: which NUMA node a GPU hangs off, which CPUs that node has, and
// pinned memory placed on it.
//
// A node verifying proofs from the network (peer_loop.rs:315-323 block batches, state/mod.rs:
// 2226-2272 bootstrap import, each ending in triton_vm::verify at verifier.rs:60-63) feeds every
// GPU from host DRAM: the proof words are copied into pinned staging (or land in pinned receive
// buffers) and DMA'd over the GPU's PCIe link.  On a two-socket host each GPU's link ends at one
// socket; staging on the other socket sends every DMA read, and every copy thread's writes, over
// the inter-socket fabric.  So each context reads its GPU's NUMA node from sysfs through the
// device's PCI bus id, places its pinned staging on that node (hipHostMallocNumaUser under a
// temporary MPOL_BIND of the allocating thread), and binds its staging copy threads to that node's
// CPUs.  No libnuma: the two policy syscalls are called directly.
//
// NHIP_NUMA=0 turns placement and binding off (A/B runs); sysfs without NUMA information (one
// node, containers) leaves everything as before.
#include <hip/hip_runtime.h>

#include <pthread.h>
#include <sched.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <algorithm>
#include <cctype>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/neptune_hip.h"
#include "host_numa.hpp"

namespace nhip {

namespace {

bool read_small_file(const std::string& path, std::string& out) {
    FILE* f = std::fopen(path.c_str(), "r");
    if (!f) return false;
    char buf[4096];
    const size_t n = std::fread(buf, 1, sizeof(buf) - 1, f);
    std::fclose(f);
    out.assign(buf, n);
    while (!out.empty() && std::isspace((unsigned char)out.back())) out.pop_back();
    return true;
}

constexpr int MPOL_DEFAULT_ = 0, MPOL_PREFERRED_ = 1;
constexpr int MAX_NODES = 1024;

long sys_get_mempolicy(int* mode, unsigned long* mask, unsigned long maxnode, void* addr, unsigned long flags) {
    return syscall(SYS_get_mempolicy, mode, mask, maxnode, addr, flags);
}
long sys_set_mempolicy(int mode, const unsigned long* mask, unsigned long maxnode) {
    return syscall(SYS_set_mempolicy, mode, mask, maxnode);
}

}  // namespace

bool parse_cpulist(const char* s, std::vector<int>& out) {
    out.clear();
    if (!s) return false;
    const char* p = s;
    while (*p) {
        while (*p == ',' || std::isspace((unsigned char)*p)) ++p;
        if (!*p) break;
        if (!std::isdigit((unsigned char)*p)) return false;
        char* e = nullptr;
        const long a = std::strtol(p, &e, 10);
        long b = a;
        p = e;
        if (*p == '-') {
            ++p;
            if (!std::isdigit((unsigned char)*p)) return false;
            b = std::strtol(p, &e, 10);
            p = e;
        }
        if (a < 0 || b < a || b > 1 << 20) return false;
        long stride = 1;
        if (*p == ':') {  // "a-b:stride" (kernel cpulist syntax)
            ++p;
            if (!std::isdigit((unsigned char)*p)) return false;  // strtol would skip whitespace
            stride = std::strtol(p, &e, 10);
            p = e;
            if (stride <= 0) return false;
        }
        for (long c = a; c <= b; c += stride) out.push_back((int)c);
        if (*p && *p != ',' && !std::isspace((unsigned char)*p)) return false;
    }
    std::sort(out.begin(), out.end());
    out.erase(std::unique(out.begin(), out.end()), out.end());
    return true;
}

HostTopo topo_from_sysfs(const char* root, const char* bus_id) {
    HostTopo t;
    if (!root || !bus_id || !*bus_id) return t;
    std::string id(bus_id);
    for (char& c : id) c = (char)std::tolower((unsigned char)c);
    std::string v;
    if (!read_small_file(std::string(root) + "/bus/pci/devices/" + id + "/numa_node", v)) return t;
    char* e = nullptr;
    const long node = std::strtol(v.c_str(), &e, 10);
    if (e == v.c_str() || node < 0 || node >= MAX_NODES) return t;  // -1: the platform reports no node
    t.numa_node = (int)node;
    if (read_small_file(std::string(root) + "/devices/system/node/node" + std::to_string(node) + "/cpulist", v))
        (void)parse_cpulist(v.c_str(), t.cpus);
    return t;
}

unsigned host_threads_env() {
    static const unsigned v = [] {
        const char* e = std::getenv("NHIP_HOST_THREADS");
        return e ? (unsigned)std::strtoul(e, nullptr, 10) : 0u;
    }();
    return v;
}

bool numa_enabled() {
    static const bool on = [] {
        const char* v = std::getenv("NHIP_NUMA");
        return !v || std::strtol(v, nullptr, 10) != 0;
    }();
    return on;
}

HostTopo device_topo(int device) {
    char bus[64] = {0};
    if (hipDeviceGetPCIBusId(bus, (int)sizeof(bus) - 1, device) != hipSuccess) return HostTopo{};
    HostTopo t = topo_from_sysfs("/sys", bus);
    t.bus_id = bus;
    if (!t.cpus.empty()) {  // only CPUs this process may run on (a cpuset-limited container)
        cpu_set_t allowed;
        CPU_ZERO(&allowed);
        if (sched_getaffinity(0, sizeof(allowed), &allowed) == 0) {
            std::vector<int> keep;
            for (int c : t.cpus)
                if (c < CPU_SETSIZE && CPU_ISSET(c, &allowed)) keep.push_back(c);
            t.cpus.swap(keep);
        }
    }
    return t;
}

bool bind_thread(const std::vector<int>& cpus) {
    if (cpus.empty() || !numa_enabled()) return false;
    cpu_set_t set;
    CPU_ZERO(&set);
    for (int c : cpus)
        if (c >= 0 && c < CPU_SETSIZE) CPU_SET(c, &set);
    return pthread_setaffinity_np(pthread_self(), sizeof(set), &set) == 0;
}

hipError_t host_malloc_on(void** p, size_t bytes, int node, unsigned flags) {
    if (node < 0 || node >= MAX_NODES || !numa_enabled()) return hipHostMalloc(p, bytes, flags);
    // this thread's policy, restored after the allocation
    int old_mode = MPOL_DEFAULT_;
    unsigned long old_mask[MAX_NODES / (8 * sizeof(unsigned long))] = {0};
    const bool have_old = sys_get_mempolicy(&old_mode, old_mask, MAX_NODES, nullptr, 0) == 0;
    unsigned long mask[MAX_NODES / (8 * sizeof(unsigned long))] = {0};
    mask[node / (8 * sizeof(unsigned long))] |= 1ul << (node % (8 * sizeof(unsigned long)));
    // preferred, not bound: the pages land on the GPU's node while it has free memory and on another
    // node otherwise (a strict bind of locked pages on a full node would wake the OOM killer instead
    // of failing the allocation)
    if (sys_set_mempolicy(MPOL_PREFERRED_, mask, MAX_NODES) != 0) return hipHostMalloc(p, bytes, flags);
    hipError_t e = hipHostMalloc(p, bytes, flags | hipHostMallocNumaUser);
    if (have_old) (void)sys_set_mempolicy(old_mode, old_mode == MPOL_DEFAULT_ ? nullptr : old_mask, MAX_NODES);
    else (void)sys_set_mempolicy(MPOL_DEFAULT_, nullptr, 0);
    if (e != hipSuccess) e = hipHostMalloc(p, bytes, flags);
    return e;
}

int page_node(const void* p) {
    int node = -1;
    if (!p || sys_get_mempolicy(&node, nullptr, 0, const_cast<void*>(p), 3 /* MPOL_F_NODE | MPOL_F_ADDR */) != 0)
        return -1;
    return node;
}

}  // namespace nhip

extern "C" {

int nhip_numa_from_sysfs(const char* sysfs_root, const char* pci_bus_id, int* numa_node, int* cpus, size_t cpu_cap,
                         size_t* n_cpus) {
    if (!sysfs_root || !pci_bus_id || !numa_node) return NHIP_ERR_ARG;
    const nhip::HostTopo t = nhip::topo_from_sysfs(sysfs_root, pci_bus_id);
    *numa_node = t.numa_node;
    if (n_cpus) *n_cpus = t.cpus.size();
    if (cpus)
        for (size_t i = 0; i < std::min(cpu_cap, t.cpus.size()); ++i) cpus[i] = t.cpus[i];
    return NHIP_OK;
}

int nhip_cpulist_parse(const char* list, int* cpus, size_t cpu_cap, size_t* n_cpus) {
    std::vector<int> v;
    if (!list || !nhip::parse_cpulist(list, v)) return NHIP_ERR_ARG;
    if (n_cpus) *n_cpus = v.size();
    if (cpus)
        for (size_t i = 0; i < std::min(cpu_cap, v.size()); ++i) cpus[i] = v[i];
    return NHIP_OK;
}

int nhip_host_page_node(const void* ptr) { return nhip::page_node(ptr); }

}  // extern "C"
