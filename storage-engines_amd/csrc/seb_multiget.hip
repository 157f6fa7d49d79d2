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

// A filter word from global memory.  The words pointers come out of RegSlot / RegLayout structs, so
// the compiler cannot tell their address space and would issue flat loads (which also count against
// the LDS wait counter the slot table's reads use); the cast makes them global loads.
__device__ __forceinline__ uint32_t gword(const uint32_t *w, uint64_t i) {
    return ((const __attribute__((address_space(1))) uint32_t *)w)[i];
}

// MayContain of one filter, with the reference's early exit (lsm/bloom.go:86-89): a position is
// gathered only while every bit so far is set.  Gathering all k unconditionally cost 42 L2
// requests per key over a MultiGet's 6 filter tests (profiles/r01y_lsm_pmc.csv); the early exit
// leaves ~1.9 per filter that does not hold the key.
template <int KFIX, bool M32>
__device__ __forceinline__ uint32_t test_filter(const RegSlot &sl, uint64_t h1, uint64_t h2) {
    uint32_t acc = 1u;
    for_positions<KFIX, M32>(h1, h2, sl.md, sl.md.k, [&](uint32_t, uint64_t p) {
        if (acc & 1u) acc &= gword(sl.words, p >> 5) >> (uint32_t)(p & 31);
    });
    return acc & 1u;
}

// The L0 group (RegLayout::l0tab): every member's MayContain at once.  A position's entry holds
// its bit of every member, so the walk gathers one word per position and stops once no member
// is left whose bits so far are all set; each member's answer is the AND of its k bits, as alone.
template <int KFIX, bool M32>
__device__ __forceinline__ uint32_t test_l0_group(const RegLayout &lay, uint64_t h1, uint64_t h2) {
    uint32_t alive = lay.l0g >= 32 ? ~0u : (1u << lay.l0g) - 1u;
    for_positions<KFIX, M32>(h1, h2, lay.l0md, lay.l0md.k, [&](uint32_t, uint64_t p) {
        if (alive) {
            const uint64_t bit = p * lay.l0b;
            alive &= gword(lay.l0tab, bit >> 5) >> (uint32_t)(bit & 31);
        }
    });
    return alive;
}

struct MgSeg;
__device__ __forceinline__ uint64_t mg_seg_key(const MgSeg &sg, uint64_t jw, uint64_t j, uint32_t &sidx);

// MODE 0: u64 mask, slot table in LDS.  MODE 1: candidate list, slot table in LDS.  MODE 2:
// candidate list, slot table read from HBM/L2 (more than kMaxSlots files: an LSM past L1 holds
// hundreds, lsm/levels.go:10-14 with ~4 MB files, lsm/compaction.go:253).  (Testing filters 4 at a
// time, and passes of one L2's worth of filters, were measured slower: DESIGN.md 5.7, 8.)
template <typename Src, int KFIX, bool M32, int MODE>
__global__ __launch_bounds__(256) void k_multiget(Src src, KeyBatch kb, const RegSlot *__restrict__ gslots,
                                                  uint32_t nslots, RegLayout lay, const uint8_t *__restrict__ ranges,
                                                  uint64_t *__restrict__ maybe, uint16_t *__restrict__ cand,
                                                  uint32_t cap, const uint32_t *__restrict__ key_order,
                                                  uint32_t xcd, MgSeg seg, uint32_t narrow) {
    constexpr bool kLds = MODE < 2, kList = MODE > 0;
    __shared__ RegSlot lslots[kLds ? kMaxSlots : 1];
    if constexpr (kLds) {
        for (uint32_t s = threadIdx.x; s < nslots; s += blockDim.x) lslots[s] = gslots[s];
        __syncthreads();
    }
    const RegSlot *slots = kLds ? lslots : gslots;
    // list rows of <= 16 slots are built in registers and stored as the widest aligned words (one
    // u32 store per 2 slots instead of a u16 store per slot: 1.189 -> 1.120 ms on 244 files)
    const uint32_t rowpack = !kList || cap > 16 ? 0u
                             : (cap % 4 == 0 && ((uintptr_t)cand & 7) == 0) ? 8u
                             : (cap % 2 == 0 && ((uintptr_t)cand & 3) == 0) ? 4u : 2u;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    // xcd: the blocks that share an XCD (blockIdx % 8 under round-robin placement, speed only) take
    // one contiguous eighth of the batch, so in key-range order each XCD's L2 holds the filters of
    // its own key stretch instead of every XCD holding the whole chip's window (bijective remap,
    // cdna_hip_programming.md T1)
    uint32_t wg = blockIdx.x;
    if (xcd) {
        const uint32_t q = gridDim.x / 8, r = gridDim.x % 8, x = blockIdx.x % 8;
        wg = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + blockIdx.x / 8;
    }
    // one iteration per wave-uniform row group (its lanes stay together for mg_seg_key's shuffles)
    for (uint64_t jw = (uint64_t)wg * blockDim.x + (threadIdx.x & ~63u); jw < kb.n; jw += stride) {
        // Answer j goes to row j.  In key-range order (multiget_order) that is the sorted position:
        // the keys are read through the segment tables (seg), were moved into that order by
        // k_mg_scatter or are read through key_order, and k_mg_unpermute brings the answers back
        // to batch order as whole lines.
        const uint64_t j = jw + (threadIdx.x & 63u);
        uint32_t sidx = 0;
        const uint64_t segkey = seg.seg ? mg_seg_key(seg, jw, j < kb.n ? j : kb.n - 1, sidx) : 0;
        if (j >= kb.n) continue;
        // segment order: the row's bucket (its segment is b * C + sc) names its partition-level
        // file, so that level needs no bisection, only the MaxKey cover check
        const int pb = seg.seg ? (int)(sidx / seg.C) : -1;
        const uint64_t oi = j;
        const uint64_t i = seg.seg ? segkey : key_order ? (uint64_t)key_order[j] : j;
        const uint8_t *key;
        uint32_t klen;
        if (kb.offsets) {
            key = kb.data + kb.offsets[i];
            klen = (uint32_t)(kb.offsets[i + 1] - kb.offsets[i]);
        } else {
            key = kb.data + i * (uint64_t)kb.stride;
            klen = kb.stride;
        }
        uint64_t h1, h2, k0, k1;
        if constexpr (std::is_same<Src, Keys16>::value) {  // one 16-B load feeds the hash and the compares
            const uint4 v = src.load(i);
            Src::hash_raw(v, h1, h2);
            k0 = __builtin_bswap64((uint64_t)v.x | ((uint64_t)v.y << 32));
            k1 = __builtin_bswap64((uint64_t)v.z | ((uint64_t)v.w << 32));
        } else {
            src.hash(i, h1, h2);
            key_prefix(kb, key, klen, k0, k1);
        }
        uint64_t mask = 0;
        uint16_t *row = kList ? cand + oi * (uint64_t)cap : nullptr;
        uint32_t nc = 0;
        uint64_t rw[4] = {~0ull, ~0ull, ~0ull, ~0ull};  // a row of <= 16 slots in registers (0xFFFF = none)
        auto record = [&](const RegSlot &sl) {  // in Get's visiting order
            if constexpr (kList) {
                if (nc < cap) {  // the host checks cap >= the walk's length
                    if (narrow) {  // u8 slots (0xFF = none), 8 per register word
#pragma unroll
                        for (uint32_t q = 0; q < 2; ++q)
                            if (q == (nc >> 3)) {
                                const uint32_t sh = (nc & 7) * 8;
                                rw[q] = (rw[q] & ~(0xFFull << sh)) | ((uint64_t)sl.slot << sh);
                            }
                    } else if (rowpack) {
#pragma unroll
                        for (uint32_t q = 0; q < 4; ++q)
                            if (q == (nc >> 2)) {
                                const uint32_t sh = (nc & 3) * 16;
                                rw[q] = (rw[q] & ~(0xFFFFull << sh)) | ((uint64_t)sl.slot << sh);
                            }
                    } else {
                        row[nc] = (uint16_t)sl.slot;
                    }
                    ++nc;
                }
            } else {
                mask |= 1ull << sl.slot;
            }
        };
        auto take = [&](const RegSlot &sl) {
            if (test_filter<KFIX, M32>(sl, h1, h2)) record(sl);
        };
        const uint32_t gm = lay.l0g ? test_l0_group<KFIX, M32>(lay, h1, h2) : 0u;
        for (uint32_t s = lay.lo[0]; s < lay.hi[0]; ++s) {  // every L0 file, in order
            const RegSlot &sl = slots[s];
            if (lay.l0g && sl.gbit >= 0) {
                if (gm >> sl.gbit & 1u) record(sl);
            } else {
                take(sl);
            }
        }
        for (uint32_t L = 1; L < 5; ++L) {
            const uint32_t lo = lay.lo[L], hi = lay.hi[L];
            if (lo == hi) continue;
            int hit = -1;
            if (pb >= 0 && lo == seg.part_lo) {  // bucket b >= 1: the last file with MinKey <= key
                if (pb >= 1) {
                    const RegSlot &sl = slots[lo + (uint32_t)pb - 1];
                    if (cmp_key(key, klen, k0, k1, sl.max_be, ranges + sl.max_off, sl.max_len) <= 0)
                        hit = (int)(lo + (uint32_t)pb - 1);
                }
            } else if (lay.nonoverlap >> L & 1u) {
                // last file with MinKey <= key; it is the only one that can cover the key.  In
                // segment order the bucket bounds the key, so the search starts on the few files
                // whose MinKey can fall in the bucket's key range
                uint32_t a = lo, b = hi;
                if (pb >= 0 && seg.brange) {
                    const uint32_t e = seg.brange[4 * (uint32_t)pb + L - 1];
                    a = lo + (e & 0xFFFFu);
                    b = lo + (e >> 16);
                }
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
            if (narrow) {  // sorted rows of cap u8 slots (cap even, <= 16): cap / 2 u16 words
                uint16_t *row8 = (uint16_t *)((uint8_t *)cand + oi * (uint64_t)cap);
#pragma unroll
                for (uint32_t q = 0; q < 8; ++q)
                    if (2 * q < cap) row8[q] = (uint16_t)(rw[q >> 2] >> ((q & 3) * 16));
            } else if (rowpack == 8) {  // the row as whole words: cap % 4 == 0 / cap % 2 == 0, aligned
#pragma unroll
                for (uint32_t q = 0; q < 4; ++q)
                    if (4 * q < cap) ((uint64_t *)row)[q] = rw[q];
            } else if (rowpack == 4) {
#pragma unroll
                for (uint32_t q = 0; q < 8; ++q)
                    if (2 * q < cap) ((uint32_t *)row)[q] = (uint32_t)(rw[q >> 1] >> ((q & 1) * 32));
            } else if (rowpack == 2) {
#pragma unroll
                for (uint32_t q = 0; q < 16; ++q)
                    if (q < cap) row[q] = (uint16_t)(rw[q >> 2] >> ((q & 3) * 16));
            } else {
                for (uint32_t t = nc; t < cap; ++t) row[t] = 0xFFFFu;
            }
        } else if (narrow) {  // sorted rows of a registry whose slots are all < 32: half the bytes
            ((uint32_t *)maybe)[oi] = (uint32_t)mask;
        } else {
            maybe[oi] = mask;
        }
    }
}

// ---- key-range order (multiget_order).  A batch probed in key order gathers from a few files of
// each level at a time, so those filters stay in L2: a key-sorted 10M batch took 0.70 ms against
// 1.47 ms in batch order (bench.py --lsm-order sorted).  The batch is put in that order without
// sorting it, by one counting pass over the buckets of the partition level (the disjoint level
// with the most files; a key's bucket = the number of its files whose MinKey <= key, monotone in
// the key), like one digit of a radix sort:
//   k_mg_bucket     tile t of the batch: each key's bucket, and the tile's bucket counts at
//                   hist[b * T + t] (bucket-major, so one exclusive scan of hist yields every
//                   (bucket, tile) output offset)
//   k_mg_rows       scans each bucket's row of T tile counts in place, and writes the row total
//   k_mg_scatter    tile t: scans the row totals into bucket bases, then per chunk of kMgChunk keys
//                   ranks the keys by bucket (stable, chunk_positions) and writes each bucket's run
//                   of 16-B keys (read through the chunk's lines), or of key indices for batches it
//                   cannot move, contiguously, and where each bucket's run of the chunk starts (runs)
// k_multiget then writes answer j at sorted row j (whole lines, no scattered 8-B stores), and
//   k_mg_unpermute  per chunk: the same stable ranks again, the chunk's runs read in row order into
//                   LDS, every key's answer written back in batch order as whole lines.
// Round 3 wrote answers at each key's own index from k_multiget: one 32-B write per 8-B mask (517 MB
// written per 10M-key call for 80 MB of masks, profiles/r04_lsm_pmc.csv); the order array (40 MB)
// is no longer needed either for moved keys.
constexpr uint32_t kMgChunk = 2048;  // keys ranked in LDS at a time by k_mg_scatter / k_mg_unpermute
// Most tiles (blocks) of the ordering passes: one round on 256 CUs.  2048 and 8192 tiles (one chunk
// each, no serial chunk loop) measured the same within 1% (profiles/r05e_mg_tiles.txt).
constexpr uint32_t kMgTiles = 768;
constexpr uint32_t kMgBucketThreads = 1024;

constexpr uint32_t kMgWaves = 4;                      // 256-thread ordering blocks
constexpr uint32_t kMgSteps = kMgChunk / kMgWaves / 64;  // 64-key steps of one wave's chunk segment
constexpr uint32_t kMgSuper = 2 * kMgChunk;              // the scatter-free order's bucket-sort unit
constexpr uint32_t kMgSuperWaves = 2 * kMgWaves;         // its 512-thread blocks

__device__ __forceinline__ void key_at(const KeyBatch &kb, uint64_t i, const uint8_t *&key, uint32_t &klen) {
    if (kb.offsets) {
        key = kb.data + kb.offsets[i];
        klen = (uint32_t)(kb.offsets[i + 1] - kb.offsets[i]);
    } else {
        key = kb.data + i * (uint64_t)kb.stride;
        klen = kb.stride;
    }
}

// Exclusive scan of a[0..n) in LDS by an NT-thread block (wsum: NT / 64 words); returns the total.
// Every thread must call it; it synchronises before returning.
template <uint32_t NT = 256>
__device__ uint32_t block_scan_lds(uint32_t *a, uint32_t n, uint32_t *wsum) {
    const uint32_t per = (n + NT - 1) / NT;
    const uint32_t b0 = min(threadIdx.x * per, n), b1 = min(b0 + per, n);
    uint32_t own = 0;
    for (uint32_t t = b0; t < b1; ++t) own += a[t];
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint32_t x = own;
#pragma unroll
    for (uint32_t d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(x, d, 64);
        if (lane >= d) x += y;
    }
    if (lane == 63) wsum[w] = x;
    __syncthreads();
    uint32_t run = x - own;
    for (uint32_t v = 0; v < w; ++v) run += wsum[v];
    uint32_t total = 0;
#pragma unroll
    for (uint32_t v = 0; v < NT / 64; ++v) total += wsum[v];
    for (uint32_t t = b0; t < b1; ++t) {
        const uint32_t c = a[t];
        a[t] = run;
        run += c;
    }
    __syncthreads();
    return total;
}

// Tiles are whole chunks (the last one ragged): tile t = keys [t * tl, min(n, (t + 1) * tl)).
__device__ __forceinline__ uint64_t tile_begin(uint64_t n, uint32_t tl, uint32_t t) {
    const uint64_t b = (uint64_t)tl * t;
    return b < n ? b : n;
}

// Chunk key q of this thread's step s: wave w owns the chunk's keys [w * 512, (w + 1) * 512), lane
// l of step s holds key w * 512 + s * 64 + l.
__device__ __forceinline__ uint32_t chunk_key(uint32_t s) {
    return (threadIdx.x >> 6) * (kMgChunk / kMgWaves) + s * 64 + (threadIdx.x & 63);
}

// The chunk's sorted row of each of this thread's keys: bucket-major, keys of one bucket in chunk
// order (stable, so k_mg_scatter and k_mg_unpermute derive the same rows from the bucket array
// alone; no atomic decides a row).  Each wave ranks its segment step by step: equal buckets within
// a step by __ballot peer masks (one ballot per bucket bit), across steps by the wave's running
// count per bucket (cw[w][b]); then the buckets' chunk offsets (loc) and the waves before it.
// bk[s]: bucket of key chunk_key(s) (>= nb for keys past cnt).  loc[0..nb] ends as the exclusive
// scan of the chunk's bucket counts, loc[nb] = cnt.  Every thread calls it; it synchronises.
// WAVES: the block's waves (4: a 2048-key chunk; 8: the 4096-key super-chunk of k_mg_bucket_sort);
// each wave ranks 512 keys.
template <uint32_t WAVES = kMgWaves>
__device__ __forceinline__ void chunk_positions(const uint32_t (&bk)[kMgSteps], uint32_t cnt, uint32_t nb,
                                                uint32_t bits, uint32_t *cw, uint32_t *loc, uint32_t *wsum,
                                                uint32_t (&pos)[kMgSteps]) {
    const uint32_t w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    for (uint32_t u = threadIdx.x; u < WAVES * nb; u += blockDim.x) cw[u] = 0;
    __syncthreads();
    const uint64_t lt = (1ull << lane) - 1ull;
    uint32_t *mine = cw + w * nb;
#pragma unroll
    for (uint32_t s = 0; s < kMgSteps; ++s) {
        const uint32_t b = bk[s];
        uint64_t peers = ~0ull;
        for (uint32_t i = 0; i < bits; ++i) {
            const uint32_t set = (b >> i) & 1u;
            const uint64_t bal = __ballot(set);
            peers &= set ? bal : ~bal;
        }
        // the group's lowest lane alone reads and advances the count, and hands the value it read
        // to its peers: no lane of the group depends on the order of another lane's LDS accesses
        const uint32_t leader = (uint32_t)__ffsll((unsigned long long)peers) - 1u;
        uint32_t got = 0;
        if (b < nb && lane == leader) {
            got = mine[b];
            mine[b] = got + (uint32_t)__popcll(peers);
        }
        const uint32_t before = __shfl(got, (int)leader, 64);
        pos[s] = before + (uint32_t)__popcll(peers & lt);
    }
    __syncthreads();
    for (uint32_t u = threadIdx.x; u < nb; u += blockDim.x) {
        uint32_t t = 0;
        for (uint32_t v = 0; v < WAVES; ++v) {  // cw[v][u] becomes the waves-before offset
            const uint32_t c = cw[v * nb + u];
            cw[v * nb + u] = t;
            t += c;
        }
        loc[u] = t;
    }
    __syncthreads();
    block_scan_lds<64 * WAVES>(loc, nb, wsum);
    if (threadIdx.x == 0) loc[nb] = cnt;
#pragma unroll
    for (uint32_t s = 0; s < kMgSteps; ++s) {
        const uint32_t b = bk[s];
        if (b < nb) pos[s] += loc[b] + mine[b];
    }
    __syncthreads();
}

constexpr uint32_t kMgBucketBatch = 4;

// The partition level's bucket of a key: the number of its files whose MinKey <= key (bisection over
// the 16-B MinKey prefixes in LDS; equal prefixes fall back to the full compare).
__device__ __forceinline__ uint32_t mg_bisect(const uint8_t *key, uint32_t klen, uint64_t k0, uint64_t k1,
                                              const RegSlot *__restrict__ slots, uint32_t lo, uint32_t hi,
                                              const uint8_t *__restrict__ ranges, const uint64_t *pmin) {
    uint32_t a = lo, b = hi;
    while (a < b) {
        const uint32_t mid = (a + b) >> 1;
        const uint64_t p0 = pmin[2 * (mid - lo)], p1 = pmin[2 * (mid - lo) + 1];
        int c;
        if (k0 != p0) {
            c = k0 < p0 ? -1 : 1;
        } else if (k1 != p1) {
            c = k1 < p1 ? -1 : 1;
        } else {
            const RegSlot &sl = slots[mid];
            c = cmp_key(key, klen, k0, k1, sl.min_be, ranges + sl.min_off, sl.min_len);
        }
        if (c >= 0)
            a = mid + 1;
        else
            b = mid;
    }
    return a;
}

// B: the bucket id type, u8 while the partition level has at most 255 files (nb <= 256), else u16.
template <typename B>
__global__ __launch_bounds__(kMgBucketThreads) void k_mg_bucket(KeyBatch kb, const RegSlot *__restrict__ slots, uint32_t lo,
                                                   uint32_t hi, const uint8_t *__restrict__ ranges,
                                                   B *__restrict__ bucket, uint32_t *__restrict__ hist,
                                                   uint32_t tl) {
    __shared__ uint32_t h[kMgMaxBuckets];
    __shared__ uint64_t pmin[2 * (kMgMaxBuckets - 1)];  // the level's MinKey prefixes (16 B per file)
    const uint32_t nb = hi - lo + 1, T = gridDim.x, t = blockIdx.x;
    for (uint32_t u = threadIdx.x; u < nb; u += blockDim.x) h[u] = 0;
    for (uint32_t u = threadIdx.x; u < nb - 1; u += blockDim.x) {
        pmin[2 * u] = slots[lo + u].min_be[0];
        pmin[2 * u + 1] = slots[lo + u].min_be[1];
    }
    __syncthreads();
    const uint64_t end = tile_begin(kb.n, tl, t + 1);
    const uint64_t beg = tile_begin(kb.n, tl, t);
    // aligned 16-B keys: kMgBucketBatch keys per thread loaded at once (clamped indices, no branch
    // to sink a load into), then bisected; other batches one key at a time
    if (!kb.offsets && kb.stride == 16 && ((uintptr_t)kb.data & 15) == 0 && end > beg) {
        const uint4 *kp = (const uint4 *)kb.data;
        for (uint64_t i0 = beg + threadIdx.x; i0 < end; i0 += (uint64_t)kMgBucketBatch * blockDim.x) {
            uint4 v[kMgBucketBatch];
#pragma unroll
            for (uint32_t r = 0; r < kMgBucketBatch; ++r) v[r] = kp[min(i0 + (uint64_t)r * blockDim.x, end - 1)];
#pragma unroll
            for (uint32_t r = 0; r < kMgBucketBatch; ++r) {
                const uint64_t i = i0 + (uint64_t)r * blockDim.x;
                if (i >= end) break;
                const uint64_t k0 = __builtin_bswap64((uint64_t)v[r].x | ((uint64_t)v[r].y << 32));
                const uint64_t k1 = __builtin_bswap64((uint64_t)v[r].z | ((uint64_t)v[r].w << 32));
                const uint32_t a = mg_bisect(kb.data + i * 16, 16, k0, k1, slots, lo, hi, ranges, pmin);
                bucket[i] = (B)(a - lo);
                atomicAdd(&h[a - lo], 1u);
            }
        }
        __syncthreads();
        for (uint32_t u = threadIdx.x; u < nb; u += blockDim.x) hist[(uint64_t)u * T + t] = h[u];
        return;
    }
    for (uint64_t i = beg + threadIdx.x; i < end; i += blockDim.x) {
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
        bucket[i] = (B)(a - lo);
        atomicAdd(&h[a - lo], 1u);
    }
    __syncthreads();
    for (uint32_t u = threadIdx.x; u < nb; u += blockDim.x) hist[(uint64_t)u * T + t] = h[u];
}

// block b: exclusive scan of hist row b (T tile counts) in place; totals[b] = the row's sum
__global__ __launch_bounds__(256) void k_mg_rows(uint32_t *__restrict__ hist, uint32_t T,
                                                 uint32_t *__restrict__ totals) {
    __shared__ uint32_t row[kMgTiles];
    __shared__ uint32_t wsum[4];
    uint32_t *g = hist + (uint64_t)blockIdx.x * T;
    for (uint32_t u = threadIdx.x; u < T; u += blockDim.x) row[u] = g[u];
    __syncthreads();
    const uint32_t total = block_scan_lds(row, T, wsum);
    for (uint32_t u = threadIdx.x; u < T; u += blockDim.x) g[u] = row[u];
    if (threadIdx.x == 0) totals[blockIdx.x] = total;
}

// Bucket bases of tile t: the exclusive scan of the row totals plus the tile's row offsets.
__device__ __forceinline__ void tile_bases(const uint32_t *hist, const uint32_t *totals, uint32_t nb, uint32_t *base,
                                           uint32_t *wsum) {
    const uint32_t T = gridDim.x, t = blockIdx.x;
    for (uint32_t u = threadIdx.x; u < nb; u += blockDim.x) base[u] = totals[u];
    __syncthreads();
    block_scan_lds(base, nb, wsum);
    for (uint32_t u = threadIdx.x; u < nb; u += blockDim.x) base[u] += hist[(uint64_t)u * T + t];
}

// The buckets of chunk [c0, end) into registers (nb, i.e. "no key", past the end).
template <typename B>
__device__ __forceinline__ void load_chunk_buckets(const B *bucket, uint64_t c0, uint64_t end, uint32_t nb,
                                                   uint32_t (&bk)[kMgSteps]) {
    const uint32_t cnt = (uint32_t)min((uint64_t)kMgChunk, end - c0);
#pragma unroll
    for (uint32_t s = 0; s < kMgSteps; ++s) {
        const uint32_t q = chunk_key(s);
        bk[s] = q < cnt ? bucket[c0 + q] : nb;
    }
}

// LDS (dynamic, sized by nb): base[nb] | loc[nb + 1] | cw[kMgWaves * nb] | wsum[4] (u32), then
// sb[kMgChunk] (u16), then the chunk's key indices in sorted order (u32).
static size_t mg_scatter_lds(uint32_t nb) {
    const size_t words = (size_t)nb + (nb + 1) + (size_t)kMgWaves * nb + 4;
    return ((words * 4 + 2 * kMgChunk + 15) & ~(size_t)15) + (size_t)kMgChunk * 4;
}

// MOVE: aligned 16-B keys, read through the chunk's sorted indices (the chunk's 32 KB of lines come
// into L2 on first touch) and stored as contiguous bucket runs.  Staging them instead in LDS, loaded
// in batch order a chunk ahead, measured slower (163 vs 115 us, profiles/r05d_mg_stage.txt).
// Otherwise the key indices are written in that order (key_order) for the MultiGet to read keys
// through.
template <bool MOVE, typename B>
__global__ __launch_bounds__(256) void k_mg_scatter(uint64_t n, const B *__restrict__ bucket,
                                                    const uint32_t *__restrict__ hist,
                                                    const uint32_t *__restrict__ totals, uint32_t nb, uint32_t bits,
                                                    uint32_t *__restrict__ order, const uint4 *__restrict__ keys,
                                                    uint4 *__restrict__ keys_out, uint32_t *__restrict__ runs,
                                                    uint32_t tl) {
    extern __shared__ uint4 mg_lds[];
    uint32_t *base = (uint32_t *)mg_lds;          // next output row of each bucket for this tile
    uint32_t *loc = base + nb;                     // the chunk's bucket offsets
    uint32_t *cw = loc + nb + 1;
    uint32_t *wsum = cw + kMgWaves * nb;
    uint16_t *sb = (uint16_t *)(wsum + 4);
    uint32_t *sidx = (uint32_t *)((uint8_t *)mg_lds +
                                  ((((size_t)nb + (nb + 1) + (size_t)kMgWaves * nb + 4) * 4 + 2 * kMgChunk + 15) & ~(size_t)15));
    tile_bases(hist, totals, nb, base, wsum);
    const uint64_t end = tile_begin(n, tl, blockIdx.x + 1);
    uint32_t bk[kMgSteps], pos[kMgSteps];
    uint64_t c0 = tile_begin(n, tl, blockIdx.x);
    if (c0 < end) load_chunk_buckets(bucket, c0, end, nb, bk);
    for (; c0 < end; c0 += kMgChunk) {
        const uint32_t cnt = (uint32_t)min((uint64_t)kMgChunk, end - c0);
        chunk_positions(bk, cnt, nb, bits, cw, loc, wsum, pos);
#pragma unroll
        for (uint32_t s = 0; s < kMgSteps; ++s)
            if (bk[s] < nb) {
                sidx[pos[s]] = (uint32_t)(c0 + chunk_key(s));
                sb[pos[s]] = (uint16_t)bk[s];
            }
        // where each bucket's run of this chunk starts in the sorted rows: with the stable ranks,
        // which k_mg_unpermute re-derives from the bucket ids, it gives every key's row
        for (uint32_t u = threadIdx.x; u < nb; u += blockDim.x) runs[(c0 / kMgChunk) * nb + u] = base[u];
        __syncthreads();
        if (c0 + kMgChunk < end) load_chunk_buckets(bucket, c0 + kMgChunk, end, nb, bk);  // during the stores
        // each bucket's run of this chunk goes out contiguously: a thread's 8 rows are looked up, then
        // their 8 key loads issued, then the 8 stores (a load-store pair per row waited for every load:
        // one memory round trip per row).  Rows past cnt repeat row cnt - 1 (the same bytes to the same
        // place), so no branch lets the compiler sink a load down to its store.
        uint32_t dst[kMgSteps], src[kMgSteps];
#pragma unroll
        for (uint32_t r = 0; r < kMgSteps; ++r) {
            const uint32_t q = min(r * 256 + threadIdx.x, cnt - 1);
            const uint32_t b = sb[q];
            dst[r] = base[b] + (q - loc[b]);
            src[r] = sidx[q];
        }
        if constexpr (MOVE) {
            uint4 v[kMgSteps];
#pragma unroll
            for (uint32_t r = 0; r < kMgSteps; ++r) v[r] = keys[src[r]];
#pragma unroll
            for (uint32_t r = 0; r < kMgSteps; ++r) keys_out[dst[r]] = v[r];
        } else {
#pragma unroll
            for (uint32_t r = 0; r < kMgSteps; ++r) order[dst[r]] = src[r];
        }
        __syncthreads();
        for (uint32_t u = threadIdx.x; u < nb; u += blockDim.x) base[u] += loc[u + 1] - loc[u];
        __syncthreads();
    }
}

// ---- the scatter-free order (multiget_order 1, aligned 16-B keys; round 6).  The
// sorted rows are those k_mg_scatter produced (bucket-major, batch order within a bucket), but no
// pass moves the keys across the batch:
//   k_mg_bucket_sort  a 4096-key super-chunk (two chunks): each key's bucket, its stable rank in the
//                     super-chunk (chunk_positions over 8 waves) and the keys written back sorted by
//                     bucket inside the super-chunk's own 64 KB (keys_cs); per segment s = b * C2 + sc
//                     (bucket b's run of super-chunk sc) its count cnt[s], where the run starts in
//                     keys_cs, seghi[s] = sc << 12 | offset, and its keys in the first chunk, half[s]
//   k_mg_rows_pieces  scans each bucket's row of C counts in pieces of kMgPiece chunks
//   k_mg_segrows      (bucket bases from the piece totals, per block) seg[s] = first sorted row |
//                     seghi[s] << 32 (rows non-decreasing in s) and the
//                     segment holding row 64 w of every wave w (wstart)
// k_multiget finds each row's segment from its wave's start and a 64-entry window of seg
// (mg_seg_key): three dependent loads (wstart, the window, the key) and no division; every
// segment's keys are contiguous in keys_cs.  k_mg_unpermute reads each chunk's run starts from seg.
__device__ __forceinline__ uint64_t mg_seg_key(const MgSeg &sg, uint64_t jw, uint64_t j, uint32_t &sidx) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t r = (uint32_t)j;
    const uint32_t s0 = sg.wstart[jw >> 6];
    const uint64_t e = s0 + lane < sg.nseg ? sg.seg[s0 + lane] : ~0ull;
    const uint32_t er = (uint32_t)e;
    uint32_t i = 0;  // the last window entry whose row <= r (entry 0's is: it holds row jw <= r)
#pragma unroll
    for (uint32_t step = 32; step; step >>= 1) {
        const uint32_t v = (uint32_t)__shfl((int)er, (int)(i + step), 64);
        if (v <= r) i += step;
    }
    const uint32_t lo = (uint32_t)__shfl((int)er, (int)i, 64);
    const uint32_t hi = (uint32_t)__shfl((int)(uint32_t)(e >> 32), (int)i, 64);
    uint64_t ent = (uint64_t)lo | ((uint64_t)hi << 32);
    sidx = s0 + i;
    if (i == 63) {  // the row may lie past the window (a run of empty segments): bisect the rest
        uint32_t a = s0 + 63, b = sg.nseg;
        while (b - a > 1) {
            const uint32_t mid = (a + b) >> 1;
            if ((uint32_t)sg.seg[mid] <= r)
                a = mid;
            else
                b = mid;
        }
        ent = sg.seg[a];
        sidx = a;
    }
    const uint32_t h = (uint32_t)(ent >> 32);
    return (uint64_t)(h >> 12) * kMgSuper + (h & 4095u) + (r - (uint32_t)ent);
}

// The bucket sort's unit: a super-chunk of two 2048-key chunks, ranked as one by a 512-thread block
// (8 waves of 512 keys), so a bucket's run of it holds twice the keys of a chunk's run: on a
// 161-file level ≈25 keys instead of ≈13, which halves the fragments k_multiget reads its keys in.
// The rows are unchanged: within a bucket, super-chunk order then stable rank = chunk order then
// rank, so k_mg_unpermute keeps its 2048-key chunks and finds chunk 2sc+1's run start past the
// first half's keys of the bucket (half[]).

// LDS (dynamic): stage uint4[kMgSuper] | pmin u64[2 (nb - 1)] | cw u32[8 nb] | loc u32[nb + 1] | wsum u32[8]
static size_t mg_bucket_sort_lds(uint32_t nb) {
    return (size_t)kMgSuper * 16 + (size_t)16 * (nb - 1) + 4 * ((size_t)kMgSuperWaves * nb + nb + 1 + 8);
}

template <typename B>
__global__ __launch_bounds__(512) void k_mg_bucket_sort(uint64_t n, const uint4 *__restrict__ keys,
                                                        const RegSlot *__restrict__ slots, uint32_t lo, uint32_t hi,
                                                        const uint8_t *__restrict__ ranges, uint32_t bits,
                                                        B *__restrict__ bucket, uint32_t *__restrict__ cnt,
                                                        uint32_t *__restrict__ seghi, uint32_t *__restrict__ half,
                                                        uint4 *__restrict__ keys_cs, uint32_t C2) {
    extern __shared__ uint4 mgb_lds[];
    const uint32_t nb = hi - lo + 1;
    uint4 *stage = mgb_lds;
    uint64_t *pmin = (uint64_t *)(stage + kMgSuper);
    uint32_t *cw = (uint32_t *)(pmin + 2 * (nb - 1));
    uint32_t *loc = cw + kMgSuperWaves * nb;
    uint32_t *wsum = loc + nb + 1;
    for (uint32_t u = threadIdx.x; u < nb - 1; u += blockDim.x) {
        pmin[2 * u] = slots[lo + u].min_be[0];
        pmin[2 * u + 1] = slots[lo + u].min_be[1];
    }
    const uint64_t c0 = (uint64_t)blockIdx.x * kMgSuper;
    const uint32_t cn = (uint32_t)min((uint64_t)kMgSuper, n - c0);
    uint4 v[kMgSteps];
#pragma unroll
    for (uint32_t s = 0; s < kMgSteps; ++s) v[s] = keys[c0 + min(chunk_key(s), cn - 1)];  // clamped: no branch
    __syncthreads();
    uint32_t bk[kMgSteps], pos[kMgSteps];
#pragma unroll
    for (uint32_t s = 0; s < kMgSteps; ++s) {
        const uint32_t q = chunk_key(s);
        bk[s] = nb;
        if (q < cn) {
            const uint64_t k0 = __builtin_bswap64((uint64_t)v[s].x | ((uint64_t)v[s].y << 32));
            const uint64_t k1 = __builtin_bswap64((uint64_t)v[s].z | ((uint64_t)v[s].w << 32));
            bk[s] = mg_bisect((const uint8_t *)(keys + c0 + q), 16, k0, k1, slots, lo, hi, ranges, pmin) - lo;
        }
    }
    chunk_positions<kMgSuperWaves>(bk, cn, nb, bits, cw, loc, wsum, pos);
#pragma unroll
    for (uint32_t s = 0; s < kMgSteps; ++s)
        if (bk[s] < nb) {
            stage[pos[s]] = v[s];
            bucket[c0 + chunk_key(s)] = (B)bk[s];
        }
    // per segment s = b * C2 + sc: its count, where its run starts in keys_cs (sc << 12 | offset;
    // an empty run may sit at 4096: masked, never read) and its keys in the first 2048-key chunk
    // (waves 0-3: cw[4][b], the waves-before offset chunk_positions left there)
    for (uint32_t u = threadIdx.x; u < nb; u += blockDim.x) {
        const uint64_t sg = (uint64_t)u * C2 + blockIdx.x;
        cnt[sg] = loc[u + 1] - loc[u];
        seghi[sg] = (blockIdx.x << 12) | (loc[u] & 4095u);
        half[sg] = cw[kMgWaves * nb + u];
    }
    __syncthreads();
    for (uint32_t q = threadIdx.x; q < cn; q += blockDim.x) keys_cs[c0 + q] = stage[q];
}

// block (p, b): exclusive scan of bucket b's counts of chunks [p * kMgPiece, ...) in place;
// ptot[b * P + p] = the piece's total
constexpr uint32_t kMgPiece = 1024;
__global__ __launch_bounds__(256) void k_mg_rows_pieces(uint32_t *__restrict__ cnt, uint32_t C, uint32_t P,
                                                        uint32_t *__restrict__ ptot) {
    __shared__ uint32_t row[kMgPiece];
    __shared__ uint32_t wsum[4];
    const uint32_t b = blockIdx.y, p0 = blockIdx.x * kMgPiece, pl = min(kMgPiece, C - p0);
    uint32_t *g = cnt + (uint64_t)b * C + p0;
    for (uint32_t u = threadIdx.x; u < pl; u += blockDim.x) row[u] = g[u];
    __syncthreads();
    const uint32_t total = block_scan_lds(row, pl, wsum);
    for (uint32_t u = threadIdx.x; u < pl; u += blockDim.x) g[u] = row[u];
    if (threadIdx.x == 0) ptot[(uint64_t)b * P + blockIdx.x] = total;
}

// grid (C / 256, nb): segment s = b * C + c: seg[s] = its first sorted row | seghi[s] << 32, and
// the waves whose first row it holds.  Each block first scans the bucket totals (sums of the piece
// totals ptot) into the bucket bases; a piece's first row adds the pieces before it.
__global__ __launch_bounds__(256) void k_mg_segrows(const uint32_t *__restrict__ cnt, const uint32_t *__restrict__ seghi,
                                                    const uint32_t *__restrict__ ptot, uint32_t nb, uint32_t C,
                                                    uint32_t P, uint32_t n, uint64_t *__restrict__ seg,
                                                    uint32_t *__restrict__ wstart) {
    __shared__ uint32_t base[kMgMaxBuckets];
    __shared__ uint32_t wsum[4];
    for (uint32_t u = threadIdx.x; u < nb; u += blockDim.x) {
        uint32_t t = 0;
        for (uint32_t p = 0; p < P; ++p) t += ptot[(uint64_t)u * P + p];
        base[u] = t;
    }
    __syncthreads();
    block_scan_lds(base, nb, wsum);
    const uint32_t b = blockIdx.y, c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= C) return;
    auto first_row = [&](uint32_t bb, uint32_t cc) {  // of piece cc / kMgPiece of bucket bb
        uint32_t t = base[bb];
        for (uint32_t p = 0; p < cc / kMgPiece; ++p) t += ptot[(uint64_t)bb * P + p];
        return t;
    };
    const uint64_t s = (uint64_t)b * C + c;
    const uint32_t row = first_row(b, c) + cnt[s];
    uint32_t next = n;
    if (c + 1 < C)
        next = first_row(b, c + 1) + cnt[s + 1];
    else if (b + 1 < nb)
        next = base[b + 1] + cnt[s + 1];
    seg[s] = (uint64_t)row | ((uint64_t)seghi[s] << 32);
    for (uint32_t w = (row + 63) / 64; w < (next + 63) / 64; ++w) wstart[w] = (uint32_t)s;
}

// Each key's answer back from its sorted row to batch order, one workgroup per chunk of kMgChunk
// keys: the chunk's stable ranks are derived again from its bucket ids (chunk_positions, as the
// scatter ranked them), so key q of bucket b sits at row runs[chunk][b] + its rank; the chunk's runs
// are read in row order into LDS (contiguous loads, all issued before any is stored) and each key
// stores its answer from its slot there, as whole lines.  G: the unit read and written (uint2 masks,
// uint3 six-slot rows, uint4, or u32 / u16 granules of other row widths, ge per answer, staged
// kMgStage bytes per key per pass).  A per-key gather through a stored row index instead took 44.9 /
// 122.0 us (masks of 28 files / 6-slot rows of 244: short runs cost it a line per key) and its
// index 80 MB of traffic (profiles/r05i_mg_unpermute.txt).
constexpr uint32_t kMgStage = 16;

template <typename G>
static size_t mg_unpermute_lds(uint32_t nb) {
    const size_t head = ((size_t)nb + 1 + (size_t)kMgWaves * nb + 4 + nb) * 4 + 2 * kMgChunk;
    const size_t slice = sizeof(G) >= kMgStage ? 1 : kMgStage / sizeof(G);
    return ((head + 15) & ~(size_t)15) + (size_t)kMgChunk * slice * sizeof(G);
}

// NARROW 1: u32 sorted masks widened to u64 (G = uint2, ge = 1); 2: sorted rows of cap = 2 W u8
// slots widened to the caller's u16 rows, 0xFF -> 0xFFFF (G = the whole row of W u32 words,
// W <= 4, ge = 1; the input row is read as the <= 2 aligned u32 words that cover it).
template <typename G, typename B, int NARROW = 0>
__global__ __launch_bounds__(256) void k_mg_unpermute(uint64_t n, const B *__restrict__ bucket,
                                                      const uint32_t *__restrict__ runs, uint32_t nb, uint32_t bits,
                                                      const G *__restrict__ answers, G *__restrict__ out,
                                                      uint32_t ge, const uint64_t *__restrict__ seg,
                                                      const uint32_t *__restrict__ half, uint32_t C2) {
    extern __shared__ uint4 mgu_lds[];
    constexpr uint32_t kSlice = sizeof(G) >= kMgStage ? 1 : kMgStage / sizeof(G);  // granules per key per pass
    uint32_t *loc = (uint32_t *)mgu_lds;
    uint32_t *cw = loc + nb + 1;
    uint32_t *wsum = cw + kMgWaves * nb;
    uint32_t *rbase = wsum + 4;
    uint16_t *sb = (uint16_t *)(rbase + nb);
    G *stage = (G *)((uint8_t *)mgu_lds +
                     ((((size_t)nb + 1 + (size_t)kMgWaves * nb + 4 + nb) * 4 + 2 * kMgChunk + 15) & ~(size_t)15));
    const uint64_t c0 = (uint64_t)blockIdx.x * kMgChunk;
    const uint32_t cnt = (uint32_t)min((uint64_t)kMgChunk, n - c0);
    // the chunk's run starts: from the scatter's runs table, or the segment table's rows (the
    // scatter-free order; bucket-major, so strided, but a line holds 16 neighbouring chunks)
    for (uint32_t u = threadIdx.x; u < nb; u += blockDim.x) {
        if (seg) {  // super-chunk sc = chunk / 2: its bucket run, past the first chunk's keys for an odd chunk
            const uint64_t sg = (uint64_t)u * C2 + (blockIdx.x >> 1);
            rbase[u] = (uint32_t)seg[sg] + ((blockIdx.x & 1u) ? half[sg] : 0u);
        } else {
            rbase[u] = runs[(uint64_t)blockIdx.x * nb + u];
        }
    }
    uint32_t bk[kMgSteps], pos[kMgSteps];
    load_chunk_buckets(bucket, c0, c0 + cnt, nb, bk);
    chunk_positions(bk, cnt, nb, bits, cw, loc, wsum, pos);  // synchronises (rbase is visible after it)
#pragma unroll
    for (uint32_t s = 0; s < kMgSteps; ++s)
        if (bk[s] < nb) sb[pos[s]] = (uint16_t)bk[s];
    __syncthreads();
    for (uint32_t g0 = 0; g0 < ge; g0 += kSlice) {
        const uint32_t gs = min(kSlice, ge - g0), units = cnt * gs;
        for (uint32_t u0 = threadIdx.x; u0 < units; u0 += 8 * 256) {
            G v[8];
#pragma unroll
            for (uint32_t r = 0; r < 8; ++r) {  // clamped: a unit past the end repeats the last one
                const uint32_t u = min(u0 + r * 256, units - 1), p = u / gs, g = u - p * gs;
                const uint32_t b = min((uint32_t)sb[p], nb - 1);
                uint64_t row = (uint64_t)rbase[b] + (p - loc[b]);
                row = row < n ? row : n - 1;  // always true when the runs are the scatter's; a guard
                if constexpr (NARROW == 1) {
                    v[r] = make_uint2(((const uint32_t *)answers)[row], 0u);
                } else if constexpr (NARROW == 2) {
                    constexpr uint32_t W = sizeof(G) / 4;
                    static_assert(W >= 1 && W <= 4, "narrow list rows of 2..8 slots");
                    const uint64_t off = row * (2 * W);  // even: the row starts 0 or 2 bytes into a word
                    const uint32_t *wp = (const uint32_t *)((const uint8_t *)answers + (off & ~3ull));
                    const uint32_t sh = (uint32_t)(off & 3u) * 8u;
                    const uint32_t a = wp[0], b = (W + 1) / 2 > 1 ? wp[1] : 0u;
                    uint32_t o[W];
#pragma unroll
                    for (uint32_t w = 0; w < W; ++w) {
                        const uint32_t bp = sh + 16 * w;
                        const uint32_t x = ((bp < 32 ? a : b) >> (bp & 31u)) & 0xFFFFu;
                        const uint32_t s0 = x & 0xFFu, s1 = x >> 8;
                        o[w] = (s0 == 0xFFu ? 0xFFFFu : s0) | (s1 == 0xFFu ? 0xFFFFu : s1) << 16;
                    }
                    __builtin_memcpy(&v[r], o, sizeof(G));
                } else {
                    v[r] = answers[row * ge + g0 + g];
                }
            }
#pragma unroll
            for (uint32_t r = 0; r < 8; ++r) {
                const uint32_t u = min(u0 + r * 256, units - 1), p = u / gs, g = u - p * gs;
                stage[p * kSlice + g] = v[r];
            }
        }
        __syncthreads();
#pragma unroll
        for (uint32_t s = 0; s < kMgSteps; ++s)
            if (bk[s] < nb)
                for (uint32_t g = 0; g < gs; ++g)
                    out[(c0 + chunk_key(s)) * ge + g0 + g] = stage[pos[s] * kSlice + g];
        __syncthreads();
    }
}

// L0 group table: one thread per output word (32 / bits entries; every member's bits of those
// positions lie in one of its words).
__global__ __launch_bounds__(256) void k_l0_table(L0Members mem, uint32_t g, uint32_t bits, uint64_t m,
                                                  uint64_t nwords, uint32_t *__restrict__ table) {
    const uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (w >= nwords) return;
    const uint32_t per = 32 / bits;
    const uint64_t p0 = w * per;
    uint32_t out = 0;
    if (p0 < m) {
        const uint32_t sh = (uint32_t)(p0 & 31), lim = m - p0 < per ? (uint32_t)(m - p0) : per;
        for (uint32_t f = 0; f < g; ++f) {
            const uint32_t v = mem.w[f][p0 >> 5] >> sh;
            for (uint32_t e = 0; e < lim; ++e) out |= ((v >> e) & 1u) << (e * bits + f);
        }
    }
    table[w] = out;
}

uint64_t l0_table_words(uint64_t m, uint32_t bits) { return (m * bits + 31) / 32; }

hipError_t launch_l0_table(const L0Members &mem, uint32_t g, uint32_t bits, uint64_t m, uint32_t *table,
                           hipStream_t s) {
    if (g < 2 || g > kL0GroupMax || bits < g || 32 % bits != 0 || m == 0) return hipErrorInvalidValue;
    const uint64_t nw = l0_table_words(m, bits);
    hipLaunchKernelGGL(k_l0_table, dim3((unsigned)((nw + 255) / 256)), dim3(256), 0, s, mem, g, bits, m, nw, table);
    return hipGetLastError();
}

bool multiget_order_moves(const KeyBatch &kb) {
    return !kb.offsets && !kb.hashes && kb.stride == 16 && ((uintptr_t)kb.data & 15) == 0;
}

static uint32_t tile_keys(uint64_t n) {  // keys per tile: whole chunks, at most kMgTiles tiles
    const uint64_t chunks = (n + kMgChunk - 1) / kMgChunk;
    return (uint32_t)((chunks + kMgTiles - 1) / kMgTiles) * kMgChunk;
}

static uint32_t order_tiles(uint64_t n) {
    const uint64_t tl = tile_keys(n);
    return n ? (uint32_t)((n + tl - 1) / tl) : 1u;
}

static uint64_t al256(uint64_t b) { return (b + 255) & ~255ull; }

static uint64_t run_bytes(uint64_t n) { return al256(4ull * kMgMaxBuckets * ((n + kMgChunk - 1) / kMgChunk)); }

static bool order_segments(const KeyBatch &kb) { return multiget_order_moves(kb) && options().multiget_order != 2; }

static uint32_t seg_pieces(uint64_t C) { return (uint32_t)((C + kMgPiece - 1) / kMgPiece); }

// The segment path's tables after the bucket ids, per super-chunk segment: cnt, seghi, half, seg,
// then wstart and the piece totals.
static uint64_t seg_bytes(uint64_t n, uint32_t nb) {
    const uint64_t C2 = (n + kMgSuper - 1) / kMgSuper, ns = C2 * nb;
    return 3 * al256(4 * ns) + al256(8 * ns) + al256(4 * ((n + 63) / 64)) + al256(4ull * nb * seg_pieces(C2));
}

uint64_t multiget_order_bytes(const KeyBatch &kb, uint64_t answer_bytes, uint32_t nb) {
    const uint64_t n = kb.n;
    if (order_segments(kb))  // bucket ids | tables | bucket-sorted keys | answers
        return al256(n * 2) + seg_bytes(n, nb) + al256(n * 16) + al256(n * answer_bytes);
    return al256(n * 2) + al256(4ull * kMgMaxBuckets * order_tiles(n)) + al256(4 * kMgMaxBuckets) +
           al256(multiget_order_moves(kb) ? n * 16 : n * 4) + run_bytes(n) + al256(n * answer_bytes);
}

// multiget_order 1 for aligned fixed 16-B keys: k_mg_bucket_sort, k_mg_rows_pieces, k_mg_segrows,
// over super-chunk segments.
static hipError_t launch_multiget_order_seg(const KeyBatch &kb, const RegSlot *slots, uint32_t lo, uint32_t hi,
                                            const uint8_t *ranges, void *ws, MgOrder *mo, hipStream_t s) {
    const uint32_t nb = hi - lo + 1;
    const uint64_t n = kb.n, C2 = (n + kMgSuper - 1) / kMgSuper, ns = C2 * nb;
    const uint32_t P = seg_pieces(C2);
    uint8_t *p = (uint8_t *)ws;
    void *bucket = p;
    uint32_t *cnt = (uint32_t *)(p += al256(n * 2));
    uint32_t *seghi = (uint32_t *)(p += al256(4 * ns));
    uint32_t *half = (uint32_t *)(p += al256(4 * ns));
    uint64_t *seg = (uint64_t *)(p += al256(4 * ns));
    uint32_t *wstart = (uint32_t *)(p += al256(8 * ns));
    uint32_t *ptot = (uint32_t *)(p += al256(4 * ((n + 63) / 64)));
    uint4 *keys_cs = (uint4 *)(p += al256(4ull * nb * P));
    void *answers = p + al256(n * 16);
    const bool b8 = nb <= 256;
    uint32_t bits = 0;
    while ((1u << bits) <= nb) ++bits;
    const size_t lds = mg_bucket_sort_lds(nb);
    auto sort = [&](auto bt) -> hipError_t {
        using B = decltype(bt);
        hipError_t a = hipFuncSetAttribute((const void *)k_mg_bucket_sort<B>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                           (int)lds);
        if (a != hipSuccess) return a;
        hipLaunchKernelGGL(k_mg_bucket_sort<B>, dim3((unsigned)C2), dim3(512), lds, s, n, (const uint4 *)kb.data, slots,
                           lo, hi, ranges, bits, (B *)bucket, cnt, seghi, half, keys_cs, (uint32_t)C2);
        return hipGetLastError();
    };
    hipError_t e = b8 ? sort(uint8_t{}) : sort(uint16_t{});
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_mg_rows_pieces, dim3(P, nb), dim3(256), 0, s, cnt, (uint32_t)C2, P, ptot);
    hipLaunchKernelGGL(k_mg_segrows, dim3((unsigned)((C2 + 255) / 256), nb), dim3(256), 0, s, cnt, seghi, ptot, nb,
                       (uint32_t)C2, P, (uint32_t)n, seg, wstart);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    mo->active = true;
    mo->n = n;
    mo->nb = nb;
    mo->bits = bits;
    mo->bucket = bucket;
    mo->bucket8 = b8;
    mo->keys = (const uint8_t *)keys_cs;
    mo->answers = answers;
    mo->seg.seg = seg;
    mo->seg.half = half;
    mo->seg.wstart = wstart;
    mo->seg.nseg = (uint32_t)ns;
    mo->seg.C = (uint32_t)C2;
    mo->seg.nb = nb;
    mo->seg.part_lo = lo;
    return hipSuccess;
}

hipError_t launch_multiget_order(const KeyBatch &kb, const RegSlot *slots, uint32_t lo, uint32_t hi,
                                 const uint8_t *ranges, void *ws, MgOrder *mo, hipStream_t s) {
    *mo = MgOrder{};
    const uint32_t nb = hi - lo + 1;
    if (kb.n == 0 || nb > kMgMaxBuckets || nb < 2 || kb.n > 0xffffffffull) return hipSuccess;
    if (order_segments(kb)) return launch_multiget_order_seg(kb, slots, lo, hi, ranges, ws, mo, s);
    const uint32_t T = order_tiles(kb.n), tl = tile_keys(kb.n);
    uint8_t *p = (uint8_t *)ws;
    void *bucket = p;
    const bool b8 = nb <= 256;  // u8 bucket ids: 10 MB less written and 20 MB less read per 10M keys
    uint32_t *hist = (uint32_t *)(p += al256(kb.n * 2));
    uint32_t *totals = (uint32_t *)(p += al256(4ull * kMgMaxBuckets * T));
    uint8_t *moved = p += al256(4 * kMgMaxBuckets);
    const bool moves = multiget_order_moves(kb);
    uint32_t *runs = (uint32_t *)(p + al256(moves ? kb.n * 16 : kb.n * 4));
    void *answers = (uint8_t *)runs + run_bytes(kb.n);
    uint32_t bits = 0;
    while ((1u << bits) <= nb) ++bits;  // bucket ids and the "no key" value nb
    if (b8)
        hipLaunchKernelGGL(k_mg_bucket<uint8_t>, dim3(T), dim3(kMgBucketThreads), 0, s, kb, slots, lo, hi, ranges,
                           (uint8_t *)bucket, hist, tl);
    else
        hipLaunchKernelGGL(k_mg_bucket<uint16_t>, dim3(T), dim3(kMgBucketThreads), 0, s, kb, slots, lo, hi, ranges,
                           (uint16_t *)bucket, hist, tl);
    hipLaunchKernelGGL(k_mg_rows, dim3(nb), dim3(256), 0, s, hist, T, totals);
    // aligned fixed 16-B keys are moved into bucket order (the MultiGet then streams them); other
    // batches get the key indices in that order
    const size_t lds = mg_scatter_lds(nb);
    auto scatter = [&](auto bt) -> hipError_t {
        using B = decltype(bt);
        auto scat = moves ? k_mg_scatter<true, B> : k_mg_scatter<false, B>;
        hipError_t a = hipFuncSetAttribute((const void *)scat, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (a != hipSuccess) return a;
        hipLaunchKernelGGL(scat, dim3(T), dim3(256), lds, s, kb.n, (const B *)bucket, hist, totals, nb, bits,
                           moves ? nullptr : (uint32_t *)moved, (const uint4 *)kb.data, moves ? (uint4 *)moved : nullptr,
                           runs, tl);
        return hipSuccess;
    };
    hipError_t a = b8 ? scatter(uint8_t{}) : scatter(uint16_t{});
    if (a != hipSuccess) return a;
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    mo->active = true;
    mo->n = kb.n;
    mo->nb = nb;
    mo->bits = bits;
    mo->bucket = bucket;
    mo->bucket8 = b8;
    mo->runs = runs;
    mo->key_order = moves ? nullptr : (const uint32_t *)moved;
    mo->keys = moves ? moved : nullptr;
    mo->answers = answers;
    return hipSuccess;
}

hipError_t launch_multiget_unpermute(const MgOrder &mo, void *out, uint64_t answer_bytes, hipStream_t s) {
    if (!mo.active || mo.n == 0) return hipSuccess;
    const uint64_t chunks = (mo.n + kMgChunk - 1) / kMgChunk;
    auto go_b = [&](auto g, auto bt, uint32_t ge, auto nw) -> hipError_t {
        using G = decltype(g);
        using B = decltype(bt);
        constexpr int NW = decltype(nw)::value;
        const size_t lds = mg_unpermute_lds<G>(mo.nb);
        hipError_t a = hipFuncSetAttribute((const void *)k_mg_unpermute<G, B, NW>,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (a != hipSuccess) return a;
        hipLaunchKernelGGL((k_mg_unpermute<G, B, NW>), dim3((unsigned)chunks), dim3(256), lds, s, mo.n,
                           (const B *)mo.bucket, mo.runs, mo.nb, mo.bits, (const G *)mo.answers, (G *)out, ge, mo.seg.seg,
                           mo.seg.half, mo.seg.C);
        return hipGetLastError();
    };
    auto go = [&](auto g, uint32_t ge) {
        using N0 = std::integral_constant<int, 0>;
        return mo.bucket8 ? go_b(g, uint8_t{}, ge, N0{}) : go_b(g, uint16_t{}, ge, N0{});
    };
    if (mo.narrow == 1) {  // u32 sorted masks (launch_multiget narrow) into the caller's u64 masks
        if (answer_bytes != 8 || ((uintptr_t)out & 7) != 0) return hipErrorInvalidValue;
        using N1 = std::integral_constant<int, 1>;
        return mo.bucket8 ? go_b(uint2{}, uint8_t{}, 1u, N1{}) : go_b(uint2{}, uint16_t{}, 1u, N1{});
    }
    if (mo.narrow == 2) {  // u8 sorted list rows (2..8 slots) into the caller's u16 rows, one row per key
        using N2 = std::integral_constant<int, 2>;
        auto go2 = [&](auto g) { return mo.bucket8 ? go_b(g, uint8_t{}, 1u, N2{}) : go_b(g, uint16_t{}, 1u, N2{}); };
        const bool a16 = ((uintptr_t)out & 15) == 0, a8 = ((uintptr_t)out & 7) == 0, a4 = ((uintptr_t)out & 3) == 0;
        if (answer_bytes == 16 && a16) return go2(uint4{});
        if (answer_bytes == 12 && a4) return go2(uint3{});
        if (answer_bytes == 8 && a8) return go2(uint2{});
        if (answer_bytes == 4 && a4) return go2(uint32_t{});
        return hipErrorInvalidValue;
    }
    const bool a16 = ((uintptr_t)out & 15) == 0, a8 = ((uintptr_t)out & 7) == 0, a4 = ((uintptr_t)out & 3) == 0;
    if (answer_bytes == 16 && a16) return go(uint4{}, 1u);
    if (answer_bytes == 12 && a4) return go(uint3{}, 1u);  // 6-slot candidate rows
    if (answer_bytes == 8 && a8) return go(uint2{}, 1u);   // masks
    if (answer_bytes % 4 == 0 && a4) return go(uint32_t{}, (uint32_t)(answer_bytes / 4));
    if (answer_bytes % 2 == 0) return go(uint16_t{}, (uint32_t)(answer_bytes / 2));
    return hipErrorInvalidValue;
}

hipError_t launch_multiget(const KeyBatch &kb, const RegSlot *slots, uint32_t nslots, const RegLayout &lay,
                           const uint8_t *ranges, uint64_t *maybe, uint16_t *cand, uint32_t cap, hipStream_t s,
                           const uint32_t *key_order, const MgSeg &seg, bool narrow) {
    if (kb.n == 0) return hipSuccess;
    if (!cand && nslots > kMaxSlots) return hipErrorInvalidValue;  // the mask form stages slots in LDS
    uint64_t g = (kb.n + 255) / 256;
    if (g > 65536) g = 65536;
    const int mode = !cand ? 0 : nslots <= kMaxSlots ? 1 : 2;
    return with_src(kb, [&](auto src) {
        using S = decltype(src);
        auto go = [&](auto kern) {
            hipLaunchKernelGGL(kern, dim3((unsigned)g), dim3(256), 0, s, src, kb, slots, nslots, lay, ranges, maybe, cand,
                               cap, key_order, (uint32_t)options().multiget_xcd, seg, (uint32_t)narrow);
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
