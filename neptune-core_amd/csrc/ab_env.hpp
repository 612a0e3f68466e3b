// Measurement-only overrides of the library's tuning constants.
//
// The product library reads exactly three environment variables, all operator settings documented
// in include/neptune_hip.h: NHIP_NUMA (host_numa.cpp), NHIP_HOST_THREADS (stark_host.cpp) and
// NHIP_QUEUE_ARENA_MB (queue.cpp).  Every other NHIP_* switch an A/B run used (Fiat-Shamir form,
// wave priorities, OOD program shape, climb thresholds, ...) is read through ab_env(), which returns
// nullptr unless the library was compiled as an A/B build (`make AB=1` -> -DNHIP_AB_BUILD, output
// build/variants/libneptune_hip_ab.so, selected with NHIP_LIB).  So a stray variable on a node
// never changes the shipped verifier's code path; tests that need a non-default form use the
// explicit ABI hooks (nhip_set_fs_form, nhip_set_climb_from_ops, nhip_air_create_ex).
#pragma once
#include <cstdlib>

namespace nhip {

inline const char* ab_env(const char* name) {
#ifdef NHIP_AB_BUILD
    return std::getenv(name);
#else
    (void)name;
    return nullptr;
#endif
}

}  // namespace nhip
