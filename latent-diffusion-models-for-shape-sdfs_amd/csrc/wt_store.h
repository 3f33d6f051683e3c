// Vector stores in two flavours: plain, or write-through (WT: `global_store_* ... sc1`, the
// line leaves the XCD's L2 at once instead of staying there dirty).  The persistent training
// step (train_dag.hip) stores everything write-through: an agent-scope release (buffer_wbl2)
// writes back every dirty line of the releasing XCD's L2, so with plain stores each job's
// release paid for the whole XCD's recent output (MI355X guide, inter-workgroup visibility:
// "stores of each flavour", release ~1.7 us clean, ~6.5 us with 16 KB freshly dirtied per
// block; profiles/r05g: the releases took a third of the step).  The launch kernels keep plain
// stores (their launch boundary writes back once).
#pragma once
#include "ldm_internal.h"

namespace ldm {

// base[idx] = v (V: 2-, 4-, 8- or 16-byte value).  The write-through form is a raw buffer store
// with the sc1 cache policy (aux bit 4) on a buffer resource over `base`: the compiler sees the
// store (its waits and scheduling account for it), `base` should be wave-uniform (else the
// compiler makes a waterfall loop of it) and idx * sizeof(T) < 2 GiB.
template <bool WT, typename V, typename T>
__device__ __forceinline__ void vst_at(T* base, int64_t idx, const V& v) {
    if constexpr (!WT) {
        *reinterpret_cast<V*>(base + idx) = v;
    } else {
        constexpr int kSc1 = 16;
        const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(
            (void*)base, (short)0, 0x7ffffff0, 0x00020000);
        const int off = (int)(idx * (int64_t)sizeof(T));
        typedef unsigned u2 __attribute__((ext_vector_type(2)));
        typedef unsigned u4 __attribute__((ext_vector_type(4)));
        if constexpr (sizeof(V) == 16) {
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4, v), r, off, 0, kSc1);
        } else if constexpr (sizeof(V) == 8) {
            __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2, v), r, off, 0, kSc1);
        } else if constexpr (sizeof(V) == 4) {
            __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), r, off, 0,
                                                  kSc1);
        } else {
            static_assert(sizeof(V) == 2, "vst_at: 2-, 4-, 8- or 16-byte values");
            __builtin_amdgcn_raw_buffer_store_b16(__builtin_bit_cast(unsigned short, v), r, off,
                                                  0, kSc1);
        }
    }
}

// v = base[idx], plain or (WT) an sc1 raw buffer load (bypasses this CU's L1: reads what
// another CU stored write-through and drained before its signal -- the MI355X guide's
// inter-workgroup hand-off with sc1 stores and sc1 loads, no release / acquire fences; one
// workgroup per CU).  `base` wave-uniform, idx * sizeof(T) < 2 GiB.
template <bool WT, typename V, typename T>
__device__ __forceinline__ V vld_at(const T* base, int64_t idx) {
    if constexpr (!WT) {
        return *reinterpret_cast<const V*>(base + idx);
    } else {
        constexpr int kSc1 = 16;
        const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(
            (void*)base, (short)0, 0x7ffffff0, 0x00020000);
        const int off = (int)(idx * (int64_t)sizeof(T));
        if constexpr (sizeof(V) == 16) {
            return __builtin_bit_cast(V, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, kSc1));
        } else if constexpr (sizeof(V) == 8) {
            return __builtin_bit_cast(V, __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, kSc1));
        } else {
            static_assert(sizeof(V) == 4, "vld_at: 4-, 8- or 16-byte values");
            return __builtin_bit_cast(V, __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, kSc1));
        }
    }
}

}  // namespace ldm
