// The group object (group.cpp), shared with the per-member proof arenas (arena.cpp).
#pragma once
#include <vector>

#include "../../include/neptune_hip.h"

struct nhip_group {
    std::vector<nhip_ctx*> members;
    std::vector<std::vector<int>> cpus;  // per member: its GPU's NUMA-node CPUs (empty: unknown)
};

namespace nhip {
// Host threads a member of g uses for its copies: the operator's NHIP_HOST_THREADS, else the count
// the group set for the member (its share of its NUMA node's CPUs), else min(16, CPUs / members).
unsigned member_copy_threads(const nhip_group* g, size_t member);
}  // namespace nhip
