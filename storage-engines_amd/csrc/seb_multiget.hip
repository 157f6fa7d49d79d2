// seb_multiget.hip — batched LSM point-lookup filtering over a device-resident filter registry
// (SURVEY.md §8(f) rows 1-2).
//
// The reference's Get walks SSTables one key at a time (lsm/lsm.go:168-198):
//   level 0:    every file, in the level's order (they may overlap)           lsm/lsm.go:173-182
//   level 1..4: the FIRST file whose [MinKey, MaxKey] covers the key, then stop lsm/lsm.go:184-196
// and each visited file first asks its bloom filter (lsm/sstable.go:206).  k_multiget does that
// for a whole key batch in one launch: per key it hashes once, walks the registry's slots in the
// same order, compares the key bytewise against each L1+ file's range (Go string order), tests the
// filter of every file Get would visit and sets bit s of the key's mask when slot s is visited AND
// its filter may contain the key.  The caller reads SSTable blocks only for set bits, in slot order.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "seb_device.h"
#include "seb_kernels.h"

namespace seb {

// Go's string comparison: bytewise, a proper prefix sorts first.  Returns <0, 0, >0.
__device__ __forceinline__ int key_cmp(const uint8_t *a, uint32_t alen, const uint8_t *b, uint32_t blen) {
    const uint32_t n = alen < blen ? alen : blen;
    for (uint32_t i = 0; i < n; ++i) {
        const int d = (int)a[i] - (int)b[i];
        if (d) return d;
    }
    return (int)alen - (int)blen;
}

__global__ __launch_bounds__(256) void k_multiget(KeyBatch kb, const RegSlot *__restrict__ slots, uint32_t nslots,
                                                  const uint8_t *__restrict__ ranges, uint64_t *__restrict__ maybe) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < kb.n; i += stride) {
        const uint8_t *key;
        uint32_t klen;
        if (kb.offsets) {
            key = kb.data + kb.offsets[i];
            klen = (uint32_t)(kb.offsets[i + 1] - kb.offsets[i]);
        } else {
            key = kb.data + i * (uint64_t)kb.stride;
            klen = kb.stride;
        }
        uint64_t h1, h2;
        fnv_range(key, 0, klen, h1, h2);
        uint64_t mask = 0;
        uint32_t done = 0;  // bit L: level L's covering file already found
        for (uint32_t s = 0; s < nslots; ++s) {
            const RegSlot sl = slots[s];
            if (sl.level > 0) {
                if (done & (1u << sl.level)) continue;
                if (key_cmp(key, klen, ranges + sl.min_off, sl.min_len) < 0 ||
                    key_cmp(key, klen, ranges + sl.max_off, sl.max_len) > 0)
                    continue;
                done |= 1u << sl.level;
            }
            uint32_t acc = 1u;
            for_positions<0, false>(h1, h2, sl.md, sl.md.k, [&](uint32_t, uint64_t p) {
                if (acc) acc &= sl.words[p >> 5] >> (uint32_t)(p & 31);
            });
            mask |= (uint64_t)(acc & 1u) << sl.slot;
        }
        maybe[i] = mask;
    }
}

hipError_t launch_multiget(const KeyBatch &kb, const RegSlot *slots, uint32_t nslots, const uint8_t *ranges,
                           uint64_t *maybe, hipStream_t s) {
    if (kb.n == 0) return hipSuccess;
    uint64_t g = (kb.n + 255) / 256;
    if (g > 65536) g = 65536;
    hipLaunchKernelGGL(k_multiget, dim3((unsigned)g), dim3(256), 0, s, kb, slots, nslots, ranges, maybe);
    return hipGetLastError();
}

}  // namespace seb
