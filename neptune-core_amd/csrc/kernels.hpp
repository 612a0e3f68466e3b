// Internal launch wrappers (C++ linkage) shared between kernel TUs and the C-ABI layer.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace nhip {

hipError_t launch_permutation(uint64_t* d_states, size_t n, hipStream_t st);
hipError_t launch_hash_pair(const uint64_t* d_l, const uint64_t* d_r, uint64_t* d_out, size_t n, hipStream_t st);
hipError_t launch_hash_varlen(const uint64_t* d_data, const uint64_t* d_off, size_t n, uint64_t* d_out,
                              hipStream_t st);
hipError_t launch_mtree_level(const uint64_t* d_children, uint64_t* d_parents, size_t n_parents, hipStream_t st);
hipError_t launch_mtree_verify(const uint64_t* d_roots, int per_path_root, const uint64_t* d_indices,
                               const uint64_t* d_leaves, const uint64_t* d_paths, uint32_t depth, size_t n,
                               uint8_t* d_verdicts, hipStream_t st);

}  // namespace nhip
