// seb_multiget.hip — batched LSM point-lookup filtering over a device-resident filter registry
// (SURVEY.md §8(f) rows 1-2).
//
// The reference's Get walks SSTables one key at a time (lsm/lsm.go:168-198):
//   level 0:    every file, in the level's order (they may overlap)           lsm/lsm.go:173-182
//   level 1..4: the FIRST file whose [MinKey, MaxKey] covers the key, then stop lsm/lsm.go:184-196
// and each visited file first asks its bloom filter (lsm/sstable.go:206).  k_multiget does that
// for a whole key batch in one launch: per key it hashes once, tests every L0 filter, and per
// level 1..4 finds the covering file (bisection over the MinKey-ordered files when the registry
// verified the level is disjoint, else the reference's linear scan), then tests that one filter.
// Bit s of the key's mask = slot s is visited AND its filter may contain the key (registries whose
// slots are all < 64), or, in the list form, the key's row of `cap` u16 slots lists those files in
// the order Get visits them, padded with 0xFFFF (any registry size).  Key ranges are
// compared in Go string order: bytewise, a proper prefix first; the first 16 bytes come from LDS
// as big-endian words, longer ties fall back to the bytes in HBM.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "seb_device.h"
#include "seb_kernels.h"

namespace seb {

constexpr uint32_t kMaxSlots = 64;  // slot tables up to this size are staged in LDS

__device__ __forceinline__ uint64_t be64(const uint8_t *p, uint32_t len) {  // first min(len,8) bytes, big-endian
    uint64_t v = 0;
    for (uint32_t i = 0; i < 8; ++i) v = (v << 8) | (i < len ? p[i] : 0u);
    return v;
}

// The key's first 16 bytes as two big-endian words: one 16-B load for aligned fixed-width 16-B
// keys (the batch layout of the benchmarks), else byte loads.
__device__ __forceinline__ void key_prefix(const KeyBatch &kb, const uint8_t *key, uint32_t klen, uint64_t &k0,
                                           uint64_t &k1) {
    if (!kb.offsets && kb.stride == 16 && ((uintptr_t)kb.data & 15) == 0) {
        const uint4 v = *(const uint4 *)key;
        k0 = __builtin_bswap64((uint64_t)v.x | ((uint64_t)v.y << 32));
        k1 = __builtin_bswap64((uint64_t)v.z | ((uint64_t)v.w << 32));
    } else {
        k0 = be64(key, klen);
        k1 = klen > 8 ? be64(key + 8, klen - 8) : 0ull;
    }
}

// Go bytewise compare of key (k0,k1 = its first 16 bytes big-endian) vs a stored range key.
__device__ __forceinline__ int cmp_key(const uint8_t *key, uint32_t klen, uint64_t k0, uint64_t k1,
                                       const uint64_t be[2], const uint8_t *bytes, uint32_t blen) {
    if (k0 != be[0]) return k0 < be[0] ? -1 : 1;
    if (k1 != be[1]) return k1 < be[1] ? -1 : 1;
    // equal zero-padded 16-byte prefixes: the shorter key is a prefix of the other unless both
    // run past 16 bytes, where the tail bytes (in HBM) decide
    const uint32_t n = klen < blen ? klen : blen;
    for (uint32_t i = 16; i < n; ++i)
        if (key[i] != bytes[i]) return key[i] < bytes[i] ? -1 : 1;
    return (int)klen - (int)blen;
}

// MayContain of one filter, with the reference's early exit (lsm/bloom.go:86-89): a position is
// gathered only while every bit so far is set.  Gathering all k unconditionally cost 42 L2
// requests per key over a MultiGet's 6 filter tests (profiles/r01y_lsm_pmc.csv); the early exit
// leaves ~1.9 per filter that does not hold the key.
template <int KFIX, bool M32>
__device__ __forceinline__ uint32_t test_filter(const RegSlot &sl, uint64_t h1, uint64_t h2) {
    uint32_t acc = 1u;
    for_positions<KFIX, M32>(h1, h2, sl.md, sl.md.k, [&](uint32_t, uint64_t p) {
        if (acc & 1u) acc &= sl.words[p >> 5] >> (uint32_t)(p & 31);
    });
    return acc & 1u;
}

// MODE 0: u64 mask, slot table in LDS.  MODE 1: candidate list, slot table in LDS.  MODE 2:
// candidate list, slot table read from HBM/L2 (more than kMaxSlots files: an LSM past L1 holds
// hundreds, lsm/levels.go:10-14 with ~4 MB files, lsm/compaction.go:253).  (Testing filters 4 at a
// time, and passes of one L2's worth of filters, were measured slower: DESIGN.md 5.7, 8.)
template <typename Src, int KFIX, bool M32, int MODE>
__global__ __launch_bounds__(256) void k_multiget(Src src, KeyBatch kb, const RegSlot *__restrict__ gslots,
                                                  uint32_t nslots, RegLayout lay, const uint8_t *__restrict__ ranges,
                                                  uint64_t *__restrict__ maybe, uint16_t *__restrict__ cand,
                                                  uint32_t cap, const uint32_t *__restrict__ order,
                                                  uint32_t order_keys) {
    constexpr bool kLds = MODE < 2, kList = MODE > 0;
    __shared__ RegSlot lslots[kLds ? kMaxSlots : 1];
    if constexpr (kLds) {
        for (uint32_t s = threadIdx.x; s < nslots; s += blockDim.x) lslots[s] = gslots[s];
        __syncthreads();
    }
    const RegSlot *slots = kLds ? lslots : gslots;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < kb.n; j += stride) {
        // key-range order (multiget_order): answer index oi = order[j]; the keys are read through the
        // order too, or (order_keys == 0) were moved into that order by k_mg_scatter
        const uint64_t oi = order ? (uint64_t)order[j] : j;
        const uint64_t i = order_keys ? oi : j;
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
        src.hash(i, h1, h2);
        uint64_t k0, k1;
        key_prefix(kb, key, klen, k0, k1);
        uint64_t mask = 0;
        uint16_t *row = kList ? cand + oi * (uint64_t)cap : nullptr;
        uint32_t nc = 0;
        auto record = [&](const RegSlot &sl) {  // in Get's visiting order
            if constexpr (kList) {
                if (nc < cap) row[nc++] = (uint16_t)sl.slot;  // the host checks cap >= the walk's length
            } else {
                mask |= 1ull << sl.slot;
            }
        };
        auto take = [&](const RegSlot &sl) {
            if (test_filter<KFIX, M32>(sl, h1, h2)) record(sl);
        };
        for (uint32_t s = lay.lo[0]; s < lay.hi[0]; ++s) take(slots[s]);  // every L0 file
        for (uint32_t L = 1; L < 5; ++L) {
            const uint32_t lo = lay.lo[L], hi = lay.hi[L];
            if (lo == hi) continue;
            int hit = -1;
            if (lay.nonoverlap >> L & 1u) {
                // last file with MinKey <= key; it is the only one that can cover the key
                uint32_t a = lo, b = hi;
                while (a < b) {
                    const uint32_t mid = (a + b) >> 1;
                    const RegSlot &sl = slots[mid];
                    if (cmp_key(key, klen, k0, k1, sl.min_be, ranges + sl.min_off, sl.min_len) >= 0)
                        a = mid + 1;
                    else
                        b = mid;
                }
                if (a > lo) {
                    const RegSlot &sl = slots[a - 1];
                    if (cmp_key(key, klen, k0, k1, sl.max_be, ranges + sl.max_off, sl.max_len) <= 0) hit = (int)a - 1;
                }
            } else {
                for (uint32_t s = lo; s < hi && hit < 0; ++s) {
                    const RegSlot &sl = slots[s];
                    if (cmp_key(key, klen, k0, k1, sl.min_be, ranges + sl.min_off, sl.min_len) >= 0 &&
                        cmp_key(key, klen, k0, k1, sl.max_be, ranges + sl.max_off, sl.max_len) <= 0)
                        hit = (int)s;
                }
            }
            if (hit >= 0) take(slots[hit]);
        }
        if constexpr (kList) {
            for (uint32_t t = nc; t < cap; ++t) row[t] = 0xFFFFu;
        } else {
            maybe[oi] = mask;
        }
    }
}

// ---- key-range order (multiget_order).  A batch probed in key order gathers from a few files of
// each level at a time, so those filters stay in L2: a key-sorted 10M batch took 0.70 ms against
// 1.47 ms in batch order (bench.py --lsm-order sorted).  Three small launches put the batch in
// that order without sorting it: k_mg_bucket finds each key's bucket, the number of files of the
// partition level (the disjoint level with the most files) whose MinKey <= key, which is
// monotone in the key; k_mg_scan turns the bucket counts into cursors; k_mg_scatter writes the
// key indices bucket by bucket (each tile reserves its runs with one atomic per bucket).
// k_multiget then walks `order` and writes every answer at the key's own index, so the results
// are those of the batch order.  Measured (gpurun_out/s3k, 28-file layout): bucket 239 us, scatter
// 48 us, and k_multiget through `order` 1683 us against 1470 in batch order: its key loads and
// answer stores become 64-B sector accesses per key, which costs more than the filter locality
// saves.  Off by default; the next form materialises the keys in bucket order.
constexpr uint32_t kMgTile = 4096;  // keys per k_mg_scatter tile (one cursor atomic per bucket per tile)

__device__ __forceinline__ void key_at(const KeyBatch &kb, uint64_t i, const uint8_t *&key, uint32_t &klen) {
    if (kb.offsets) {
        key = kb.data + kb.offsets[i];
        klen = (uint32_t)(kb.offsets[i + 1] - kb.offsets[i]);
    } else {
        key = kb.data + i * (uint64_t)kb.stride;
        klen = kb.stride;
    }
}

__global__ __launch_bounds__(256) void k_mg_bucket(KeyBatch kb, const RegSlot *__restrict__ slots, uint32_t lo,
                                                   uint32_t hi, const uint8_t *__restrict__ ranges,
                                                   uint16_t *__restrict__ bucket, uint32_t *__restrict__ counts) {
    __shared__ uint32_t h[kMgMaxBuckets];
    __shared__ uint64_t pmin[2 * (kMgMaxBuckets - 1)];  // the level's MinKey prefixes (16 B per file)
    const uint32_t nb = hi - lo + 1;
    for (uint32_t t = threadIdx.x; t < nb; t += blockDim.x) h[t] = 0;
    for (uint32_t t = threadIdx.x; t < nb - 1; t += blockDim.x) {
        pmin[2 * t] = slots[lo + t].min_be[0];
        pmin[2 * t + 1] = slots[lo + t].min_be[1];
    }
    __syncthreads();
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < kb.n; i += stride) {
        const uint8_t *key;
        uint32_t klen;
        key_at(kb, i, key, klen);
        uint64_t k0, k1;
        key_prefix(kb, key, klen, k0, k1);
        uint32_t a = lo, b = hi;
        while (a < b) {
            const uint32_t mid = (a + b) >> 1;
            const uint64_t p0 = pmin[2 * (mid - lo)], p1 = pmin[2 * (mid - lo) + 1];
            int c;
            if (k0 != p0) {
                c = k0 < p0 ? -1 : 1;
            } else if (k1 != p1) {
                c = k1 < p1 ? -1 : 1;
            } else {  // equal 16-byte prefixes: the full compare (tail bytes in HBM)
                const RegSlot &sl = slots[mid];
                c = cmp_key(key, klen, k0, k1, sl.min_be, ranges + sl.min_off, sl.min_len);
            }
            if (c >= 0)
                a = mid + 1;
            else
                b = mid;
        }
        bucket[i] = (uint16_t)(a - lo);
        atomicAdd(&h[a - lo], 1u);
    }
    __syncthreads();
    for (uint32_t t = threadIdx.x; t < nb; t += blockDim.x)
        if (h[t]) atomicAdd(&counts[t], h[t]);
}

__global__ void k_mg_scan(uint32_t *counts, uint32_t nb) {  // exclusive scan in place, one thread (nb <= 1025)
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    uint32_t run = 0;
    for (uint32_t t = 0; t < nb; ++t) {
        const uint32_t c = counts[t];
        counts[t] = run;
        run += c;
    }
}

__global__ __launch_bounds__(256) void k_mg_scatter(uint64_t n, const uint16_t *__restrict__ bucket,
                                                    uint32_t *__restrict__ cursor, uint32_t nb,
                                                    uint32_t *__restrict__ order, const uint4 *__restrict__ keys,
                                                    uint4 *__restrict__ keys_out) {
    __shared__ uint32_t h[kMgMaxBuckets];
    constexpr uint32_t kPer = kMgTile / 256;
    for (uint64_t t0 = (uint64_t)blockIdx.x * kMgTile; t0 < n; t0 += (uint64_t)gridDim.x * kMgTile) {
        for (uint32_t t = threadIdx.x; t < nb; t += blockDim.x) h[t] = 0;
        __syncthreads();
        uint32_t bk[kPer], rk[kPer];
#pragma unroll
        for (uint32_t r = 0; r < kPer; ++r) {
            const uint64_t i = t0 + (uint64_t)r * 256 + threadIdx.x;
            bk[r] = i < n ? bucket[i] : 0u;
            rk[r] = i < n ? atomicAdd(&h[bk[r]], 1u) : 0u;
        }
        __syncthreads();
        for (uint32_t t = threadIdx.x; t < nb; t += blockDim.x)
            if (h[t]) h[t] = atomicAdd(&cursor[t], h[t]);  // this tile's run of bucket t starts here
        __syncthreads();
#pragma unroll
        for (uint32_t r = 0; r < kPer; ++r) {
            const uint64_t i = t0 + (uint64_t)r * 256 + threadIdx.x;
            if (i < n) {
                order[h[bk[r]] + rk[r]] = (uint32_t)i;
                if (keys_out) keys_out[h[bk[r]] + rk[r]] = keys[i];  // 16-B keys move with their index
            }
        }
        __syncthreads();
    }
}

bool multiget_order_moves(const KeyBatch &kb) {
    return !kb.offsets && !kb.hashes && kb.stride == 16 && ((uintptr_t)kb.data & 15) == 0;
}

uint64_t multiget_order_bytes(const KeyBatch &kb) {
    const uint64_t n = kb.n;
    return ((n * 2 + 255) & ~255ull) + ((n * 4 + 255) & ~255ull) + ((4 * kMgMaxBuckets + 255) & ~255ull) +
           (multiget_order_moves(kb) ? n * 16 : 0);
}

hipError_t launch_multiget_order(const KeyBatch &kb, const RegSlot *slots, uint32_t lo, uint32_t hi,
                                 const uint8_t *ranges, void *ws, uint32_t **order_out, const uint8_t **keys_out,
                                 hipStream_t s) {
    *order_out = nullptr;
    *keys_out = nullptr;
    const uint32_t nb = hi - lo + 1;
    if (kb.n == 0 || nb > kMgMaxBuckets || nb < 2 || kb.n > 0xffffffffull) return hipSuccess;
    uint16_t *bucket = (uint16_t *)ws;
    uint32_t *order = (uint32_t *)((uint8_t *)ws + ((kb.n * 2 + 255) & ~255ull));
    uint32_t *counts = (uint32_t *)((uint8_t *)order + ((kb.n * 4 + 255) & ~255ull));
    // aligned fixed 16-B keys are moved into bucket order as well (the MultiGet then streams them)
    const bool move = multiget_order_moves(kb);
    uint4 *sorted = move ? (uint4 *)((uint8_t *)counts + ((4 * kMgMaxBuckets + 255) & ~255ull)) : nullptr;
    hipError_t e = hipMemsetAsync(counts, 0, 4 * nb, s);
    if (e != hipSuccess) return e;
    uint64_t g = (kb.n + 255) / 256;
    if (g > 4096) g = 4096;
    hipLaunchKernelGGL(k_mg_bucket, dim3((unsigned)g), dim3(256), 0, s, kb, slots, lo, hi, ranges, bucket, counts);
    hipLaunchKernelGGL(k_mg_scan, dim3(1), dim3(64), 0, s, counts, nb);
    uint64_t gt = (kb.n + kMgTile - 1) / kMgTile;
    if (gt > 2048) gt = 2048;
    hipLaunchKernelGGL(k_mg_scatter, dim3((unsigned)gt), dim3(256), 0, s, kb.n, bucket, counts, nb, order,
                       (const uint4 *)kb.data, sorted);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    *order_out = order;
    *keys_out = (const uint8_t *)sorted;
    return hipSuccess;
}

hipError_t launch_multiget(const KeyBatch &kb, const RegSlot *slots, uint32_t nslots, const RegLayout &lay,
                           const uint8_t *ranges, uint64_t *maybe, uint16_t *cand, uint32_t cap, hipStream_t s,
                           const uint32_t *order, bool order_keys) {
    if (kb.n == 0) return hipSuccess;
    if (!cand && nslots > kMaxSlots) return hipErrorInvalidValue;  // the mask form stages slots in LDS
    uint64_t g = (kb.n + 255) / 256;
    if (g > 65536) g = 65536;
    const int mode = !cand ? 0 : nslots <= kMaxSlots ? 1 : 2;
    return with_src(kb, [&](auto src) {
        using S = decltype(src);
        auto go = [&](auto kern) {
            hipLaunchKernelGGL(kern, dim3((unsigned)g), dim3(256), 0, s, src, kb, slots, nslots, lay, ranges, maybe, cand,
                               cap, order, (uint32_t)(order && order_keys));
            return hipGetLastError();
        };
        if (lay.all_k7_m32) {
            if (mode == 0) return go(k_multiget<S, 7, true, 0>);
            if (mode == 1) return go(k_multiget<S, 7, true, 1>);
            return go(k_multiget<S, 7, true, 2>);
        }
        if (mode == 0) return go(k_multiget<S, 0, false, 0>);
        if (mode == 1) return go(k_multiget<S, 0, false, 1>);
        return go(k_multiget<S, 0, false, 2>);
    });
}

}  // namespace seb
