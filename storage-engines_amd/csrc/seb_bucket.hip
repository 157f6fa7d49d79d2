// seb_bucket.hip — radix-partitioned bloom build: no global atomics on the filter.
//
// The reference ORs k bits per key straight into the bit array (lsm/bloom.go:70-77).  Done
// with device-scope atomics on gfx950 every OR is a memory-side atomic (TCC_EA0_ATOMIC = n*k;
// profiles/r01), which caps the build at ~27 G bit-sets/s.  This path instead partitions the
// n*k bit positions by 64 Ki-bit bucket (one 8 KiB LDS image each) and sets the bits in LDS:
//
//   k_bkt_scatter  one workgroup per super-tile of keys: hash a round of keys, counting-sort its
//                  positions by bucket in LDS, append each bucket's run (u16 in-bucket bit index)
//                  to the fixed-capacity region (bucket, tile); the run lengths go to counts
//   k_bkt_apply    one workgroup per bucket: stream its ntiles regions, ds_or into an 8 KiB LDS
//                  image, then OR the image into the filter words the workgroup owns, or for a
//                  fresh build write them whole (no clear beforehand)
//
// The result is the same bit array bit for bit (OR is order-independent).  Requires m <= 2^28
// (<= 4096 buckets) and n*k < 2^32 per launch; the host splits larger batches.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "seb_device.h"
#include "seb_kernels.h"

namespace seb {

constexpr int kBktShift = 16;                            // 64 Ki bits per bucket
constexpr uint32_t kBktWords = 1u << (kBktShift - 5);   // 2048 u32 words = 8 KiB of LDS
constexpr uint32_t kMaxBuckets = 4096;                   // m <= 2^28 bits
constexpr uint32_t kTilePos = 28672;                     // positions per tile sorted in LDS (112 KiB)
constexpr uint32_t kMaxTiles = 1024;                     // super-tiles (workgroups) per launch
constexpr uint32_t kTargetTiles = 256;                   // workgroups per CU x 256 CUs

// Exclusive scan of one value per thread over a block of kScanThreads / kTileThreads threads.
// wsum: LDS scratch of (threads / 64) words.  Returns the prefix; *total = block sum.
__device__ __forceinline__ uint32_t block_exclusive_scan(uint32_t x, uint32_t *wsum, uint32_t *total) {
    const uint32_t lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
    uint32_t v = x;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        uint32_t y = __shfl_up(v, d, 64);
        if (lane >= (uint32_t)d) v += y;
    }
    if (lane == 63) wsum[wid] = v;
    __syncthreads();
    if (wid == 0) {
        uint32_t s = lane < nw ? wsum[lane] : 0u;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            uint32_t y = __shfl_up(s, d, 64);
            if (lane >= (uint32_t)d) s += y;
        }
        if (lane < nw) wsum[lane] = s;
    }
    __syncthreads();
    const uint32_t pre = (wid ? wsum[wid - 1] : 0u) + v - x;
    *total = wsum[nw - 1];
    __syncthreads();
    return pre;
}

// ---- scatter: one workgroup per super-tile of R rounds x kRoundKeys keys.  Each round
// counting-sorts its positions by bucket in LDS, then appends each bucket run to the
// fixed-capacity region (bucket b, tile t) in HBM.  A run that would overflow its region (never
// for hash-distributed keys: cap = mean + 8 sigma + 32) is OR-ed with device-scope atomics into
// `ovw` instead: the filter itself, which k_bkt_apply's read-modify-write OR preserves, or for a
// fresh build the overflow bitmap that apply folds in.  counts[b][t] is the run's full length, so
// apply can tell an overflowed bucket (count > cap).
// LDS: sorted[THREADS*KPT7*7] u32 | cursor[nb] | fill[nb] | wsum[16] | ovf
template <typename Src, int KFIX, int THREADS, int KPT7>
__global__ __launch_bounds__(THREADS) void k_bkt_scatter(Src src, uint64_t n, ModArg md, uint32_t nb, uint32_t tile_keys,
                                                             uint32_t ntiles, uint32_t cap, uint16_t *__restrict__ regions,
                                                             uint32_t *__restrict__ counts,
                                                             uint32_t *__restrict__ ovw) {
    extern __shared__ uint32_t smem[];
    constexpr uint32_t kPos = (uint32_t)THREADS * KPT7 * 7;  // positions sorted per round
    uint32_t *sorted = smem;
    uint32_t *cursor = smem + kPos;
    uint32_t *fill = cursor + nb;
    uint32_t *wsum = fill + nb;
    uint32_t *ovf = wsum + 16;
    const uint32_t t = blockIdx.x;  // region of bucket b: (b * ntiles + t) * cap
    for (uint32_t b = threadIdx.x; b < nb; b += blockDim.x) {
        cursor[b] = 0u;
        fill[b] = 0u;
    }
    if (threadIdx.x == 0) *ovf = 0u;
    __syncthreads();
    const uint32_t round_keys = KFIX > 0 ? KPT7 * THREADS : kPos / md.k;
    const uint64_t t0 = (uint64_t)t * tile_keys;
    const uint64_t t1 = t0 + tile_keys < n ? t0 + tile_keys : n;
    const uint32_t per = (nb + blockDim.x - 1) / blockDim.x;  // <= 8 buckets per thread in the scan

    constexpr int KP = KFIX > 0 ? KPT7 : 1;
    constexpr int KQ = KFIX > 0 ? KFIX : 1;
    // 16-B sources: the keys of round j+1 are loaded while round j sorts and writes (the whole
    // workgroup passes each barrier together, so a load issued at a round's start would stall
    // every wave of the CU at once).
    constexpr bool kPre = KFIX > 0 && SplitLoad<Src>::value;
    uint4 kv[kPre ? KP : 1];
    auto prefetch = [&](uint64_t r0) {
        if constexpr (kPre) {
            const uint64_t r1 = r0 + round_keys < t1 ? r0 + round_keys : t1;
#pragma unroll
            for (int r = 0; r < KP; ++r) {
                const uint64_t i = r0 + (uint64_t)r * blockDim.x + threadIdx.x;
                if (i < r1) kv[r] = src.load(i);
            }
        }
    };
    prefetch(t0);
    for (uint64_t k0 = t0; k0 < t1; k0 += round_keys) {
        const uint64_t k1 = k0 + round_keys < t1 ? k0 + round_keys : t1;
        uint32_t pos[KP][KQ];
        bool valid[KP];
        if constexpr (KFIX > 0) {  // positions stay in registers between counting and placing
#pragma unroll
            for (int r = 0; r < KP; ++r) {
                const uint64_t i = k0 + (uint64_t)r * blockDim.x + threadIdx.x;
                valid[r] = i < k1;
                if (valid[r]) {
                    if constexpr (IsPacked<Src>::value) {
                        static_assert(KFIX == 7, "packed residues are k == 7");
                        packed_positions((uint64_t)kv[r].x | (uint64_t)kv[r].y << 32, (uint32_t)md.m, (uint32_t)md.c,
                                         pos[r]);
                    } else {
                        uint64_t h1, h2;
                        if constexpr (kPre)
                            Src::hash_raw(kv[r], h1, h2);
                        else
                            src.hash(i, h1, h2);
                        for_positions<KFIX, true>(h1, h2, md, KFIX,
                                                  [&](uint32_t q, uint64_t p) { pos[r][q] = (uint32_t)p; });
                    }
#pragma unroll
                    for (int q = 0; q < KQ; ++q) atomicAdd(&cursor[pos[r][q] >> kBktShift], 1u);
                }
            }
            if (k1 < t1) prefetch(k1);
        } else {
            for (uint64_t i = k0 + threadIdx.x; i < k1; i += blockDim.x) {
                uint64_t h1, h2;
                src.hash(i, h1, h2);
                for_positions<0, true>(h1, h2, md, md.k,
                                       [&](uint32_t, uint64_t p) { atomicAdd(&cursor[(uint32_t)p >> kBktShift], 1u); });
            }
        }
        __syncthreads();
        {  // exclusive scan of this round's bucket counts
            const uint32_t b0 = threadIdx.x * per;
            uint32_t c[8] = {0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u}, s = 0;
            for (uint32_t j = 0; j < per; ++j)
                if (b0 + j < nb) {
                    c[j] = cursor[b0 + j];
                    s += c[j];
                }
            uint32_t tot;
            uint32_t pre = block_exclusive_scan(s, wsum, &tot);
            for (uint32_t j = 0; j < per; ++j)
                if (b0 + j < nb) {
                    cursor[b0 + j] = pre;
                    pre += c[j];
                }
        }
        __syncthreads();
        if constexpr (KFIX > 0) {
            // All slot claims first, then all writes: the atomics are independent and pipeline,
            // where claim-then-write per position serialises on every atomic's return.  (Taking
            // the ranks from the histogram atomics instead, so this pass is an LDS read, measured
            // slower: 193 vs 171 us; returning atomics cost more than the second pass saves.)
            uint32_t slot[KP][KQ];
#pragma unroll
            for (int r = 0; r < KP; ++r)
                if (valid[r]) {
#pragma unroll
                    for (int q = 0; q < KQ; ++q) slot[r][q] = atomicAdd(&cursor[pos[r][q] >> kBktShift], 1u);
                }
#pragma unroll
            for (int r = 0; r < KP; ++r)
                if (valid[r]) {
#pragma unroll
                    for (int q = 0; q < KQ; ++q) sorted[slot[r][q]] = pos[r][q];
                }
        } else {
            for (uint64_t i = k0 + threadIdx.x; i < k1; i += blockDim.x) {
                uint64_t h1, h2;
                src.hash(i, h1, h2);
                for_positions<0, true>(h1, h2, md, md.k, [&](uint32_t, uint64_t p) {
                    sorted[atomicAdd(&cursor[(uint32_t)p >> kBktShift], 1u)] = (uint32_t)p;
                });
            }
        }
        __syncthreads();
        // cursor[b] is now the END of bucket b's run in `sorted` and its start is cursor[b-1].
        // Turn fill[b] into the region element index of sorted[0] (mod 2^32), so that sorted[idx]
        // belongs at regions[fill[b] + idx], and flag a run that would overflow its region.
        for (uint32_t b = threadIdx.x; b < nb; b += blockDim.x) {
            const uint32_t start = b ? cursor[b - 1] : 0u, c = cursor[b] - start;
            const uint32_t reg = b * ntiles + t;
            if (fill[b] + c > cap) *ovf = 1u;
            fill[b] = reg * cap + fill[b] - start;
        }
        __syncthreads();
        const uint32_t cnt = (uint32_t)(k1 - k0) * md.k;
        if (*ovf == 0u) {  // every run fits (hash-distributed keys): one LDS read + store each
#pragma unroll 5
            for (uint32_t idx = threadIdx.x; idx < cnt; idx += blockDim.x) {
                const uint32_t p = sorted[idx];
                regions[fill[p >> kBktShift] + idx] = (uint16_t)p;
            }
        } else {
            for (uint32_t idx = threadIdx.x; idx < cnt; idx += blockDim.x) {
                const uint32_t p = sorted[idx];
                const uint32_t b = p >> kBktShift;
                const uint32_t e = fill[b] + idx;
                if (e - (b * ntiles + t) * cap < cap)
                    regions[e] = (uint16_t)p;
                else
                    __hip_atomic_fetch_or(ovw + (p >> 5), 1u << (p & 31), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        __syncthreads();
        for (uint32_t b = threadIdx.x; b < nb; b += blockDim.x) {
            fill[b] += cursor[b] - (b * ntiles + t) * cap;  // fill + this round's count
            cursor[b] = 0u;
        }
        if (threadIdx.x == 0) *ovf = 0u;
        __syncthreads();
    }
    for (uint32_t b = threadIdx.x; b < nb; b += blockDim.x) counts[(uint64_t)b * ntiles + t] = fill[b];
}

// ---- scatter through fixed bins (k == 7; the default for kBinMinBuckets..kBinMaxBuckets
// buckets, C2/C4's 1463).  The counting sort above costs two LDS atomics per position (histogram,
// then slot claim), a block scan and nine barriers per round, and its hashing cannot overlap its
// LDS work: every wave hashes, then every wave sorts.  Here every bucket owns a fixed bin of S u16
// in LDS (48 for up to 1575 buckets, else 32; a round's mean is ~24.5 positions per bucket), so a
// position is placed with ONE returning LDS atomic (its slot) and a 2-B LDS write, and a thread
// software-pipelines its keys: it hashes key r and issues its 7 claims, then writes key r-1's
// bins, whose claims returned while key r hashed.  The LDS atomics run under the hashing.
// After one barrier each bucket's run goes out as 16-B chunks, its S/8 chunks on adjacent lanes
// of one wave; the run is padded to a multiple of 8 with copies of its last chunk's first index
// (apply ORs that bit again), so every region offset stays 16-B aligned and apply needs no
// per-index bounds.  A claim past the bin (a Poisson tail: ~3e-5 of the bucket-
// rounds with S = 48) is stored straight to its region slot, which the round's start fixes.  The
// lane that advances a bucket's fill sits in the wave whose lanes read it, so a round has two
// barriers.  LDS: bins[nb][S] u16 | cnt[nb] (this round's claims) | fill[nb] (region fill) | a
// scratch word; two arrays, not one of pairs, so the claim atomics spread over all the banks.
constexpr uint32_t kBinMinBuckets = 512;
constexpr uint32_t kBinBig = 48, kBinSmall = 32;  // u16 slots per bin
constexpr uint32_t bin_lds_bytes(uint32_t nb, uint32_t slots) { return nb * (slots * 2 + 8) + 16; }
constexpr uint32_t kBinBigMaxBuckets = (160u * 1024 - 16) / (kBinBig * 2 + 8);      // 1575 (m <= ~103M bits)
constexpr uint32_t kBinMaxBuckets = (160u * 1024 - 16) / (kBinSmall * 2 + 8);       // 2275 (m <= ~149M bits)
constexpr double kBinMeanPos[2] = {20.0, 25.0};  // positions per bucket per round, at most (32 / 48 slots)

__device__ __forceinline__ void bins_overflow_or(uint32_t *ovw, uint32_t b, uint32_t l) {
    const uint32_t p = (b << kBktShift) | l;
    __hip_atomic_fetch_or(ovw + (p >> 5), 1u << (p & 31), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <typename Src, int THREADS, int KPT, uint32_t SB, int G = 1>
__global__ __launch_bounds__(THREADS) void k_bkt_scatter_bins(Src src, uint64_t n, ModArg md, uint32_t nb,
                                                              uint32_t tile_keys, uint32_t round_keys, uint32_t ntiles,
                                                              uint32_t cap, uint16_t *__restrict__ regions,
                                                              uint32_t *__restrict__ counts, uint32_t *__restrict__ ovw) {
    extern __shared__ uint4 smem4[];
    constexpr uint32_t S = SB, PAD = 8;
    static_assert(S % 8 == 0 && S <= 64, "a bucket's chunks must sit in one wave");
    uint16_t *bins = (uint16_t *)smem4;                      // 16-B aligned chunks
    uint32_t *cnt = (uint32_t *)(bins + (size_t)nb * S);
    uint32_t *fill = cnt + nb;
    const uint32_t t = blockIdx.x;
    for (uint32_t b = threadIdx.x; b < nb; b += THREADS) {
        cnt[b] = 0u;
        fill[b] = 0u;
    }
    __syncthreads();
    const uint64_t t0 = (uint64_t)t * tile_keys;
    const uint64_t t1 = t0 + tile_keys < n ? t0 + tile_keys : n;
    constexpr bool kPre = SplitLoad<Src>::value;
    uint4 kv[kPre ? KPT : 1];
    auto prefetch = [&](uint64_t r0) {
        if constexpr (kPre) {
            const uint64_t r1 = r0 + round_keys < t1 ? r0 + round_keys : t1;
#pragma unroll
            for (int r = 0; r < KPT; ++r) {
                const uint64_t i = r0 + (uint64_t)r * THREADS + threadIdx.x;
                if (i < r1) kv[r] = src.load(i);
            }
        }
    };
    prefetch(t0);  // later rounds load key by key, in the pipeline below
    for (uint64_t k0 = t0; k0 < t1; k0 += round_keys) {
        const uint64_t k1 = k0 + round_keys < t1 ? k0 + round_keys : t1;
        // software pipeline over the thread's keys, G at a time: hash keys r..r+G-1 and issue
        // their slot claims, then write the previous G keys' bins (their claims returned while
        // these hashed), so the returning LDS atomics overlap the hashing instead of following it
        constexpr int NSTEP = (KPT + G - 1) / G;
        uint32_t pp[G][7], ps[G][7];
        bool pv[G];
#pragma unroll
        for (int g = 0; g < G; ++g) pv[g] = false;
        auto write_bins = [&](const uint32_t (&pw)[7], const uint32_t (&sw)[7]) {
#pragma unroll
            for (int q = 0; q < 7; ++q) {
                const uint32_t p = pw[q], sl = sw[q], b = p >> kBktShift;
                bins[sl < S ? b * S + sl : nb * S + 4 * nb] = (uint16_t)p;  // past the bin: a scratch word
                if (sl >= S) {  // rare: straight to the region slot (the fill is fixed this round)
                    const uint32_t e = fill[b] + sl;
                    if (e < cap)
                        regions[(uint64_t)(b * ntiles + t) * cap + e] = (uint16_t)p;
                    else
                        bins_overflow_or(ovw, b, p & 0xffffu);
                }
            }
        };
#pragma unroll
        for (int st = 0; st < NSTEP; ++st) {
            uint32_t pos[G][7], sl[G][7];
            bool valid[G];
#pragma unroll
            // Prefetched sources are hashed with no validity branch (kv always holds loadable
            // data; a key past the round is simply not claimed): straight-line hashing of the
            // thread's keys measured 136.5 vs 144.3 us against a branch around each key's hash
            // (tools/diag/scatter_pipeline_single_key.patch)
            for (int g = 0; g < G; ++g) {  // independent chains, hashed side by side
                const int r = st * G + g;
                const uint64_t i = k0 + (uint64_t)r * THREADS + threadIdx.x;
                valid[g] = r < KPT && i < k1;
                if (r < KPT && (kPre || valid[g])) {
                    if constexpr (IsPacked<Src>::value) {
                        packed_positions((uint64_t)kv[r].x | (uint64_t)kv[r].y << 32, (uint32_t)md.m, (uint32_t)md.c,
                                         pos[g]);
                    } else {
                        uint64_t h1, h2;
                        if constexpr (kPre)
                            Src::hash_raw(kv[r], h1, h2);
                        else
                            src.hash(i, h1, h2);
                        for_positions<7, true>(h1, h2, md, 7, [&](uint32_t q, uint64_t p) { pos[g][q] = (uint32_t)p; });
                    }
                }
            }
#pragma unroll
            for (int g = 0; g < G; ++g) {
                const int r = st * G + g;
                if (r >= KPT) continue;
                const uint64_t i = k0 + (uint64_t)r * THREADS + threadIdx.x;
                if constexpr (kPre) {  // this key's register now loads the next round's key r
                    const uint64_t in = i + round_keys;
                    if (valid[g] && k1 < t1 && in < (k1 + round_keys < t1 ? k1 + round_keys : t1)) kv[r] = src.load(in);
                }
                if (valid[g]) {
#pragma unroll
                    for (int q = 0; q < 7; ++q) sl[g][q] = atomicAdd(&cnt[pos[g][q] >> kBktShift], 1u);
                }
            }
#pragma unroll
            for (int g = 0; g < G; ++g) {
                if (pv[g]) write_bins(pp[g], ps[g]);
#pragma unroll
                for (int q = 0; q < 7; ++q) {
                    pp[g][q] = pos[g][q];
                    ps[g][q] = sl[g][q];
                }
                pv[g] = valid[g];
            }
        }
#pragma unroll
        for (int g = 0; g < G; ++g)
            if (pv[g]) write_bins(pp[g], ps[g]);
        __syncthreads();
        // write-out: a bucket's S/8 chunks on S/8 adjacent lanes of one wave (64/(S/8) buckets per
        // wave; with S = 48, lanes 60-63 idle), so the lane that advances the bucket's fill runs in
        // the wave whose other lanes read it
        {
            constexpr uint32_t NCH = S / 8, BPW = 64 / NCH, NW = THREADS / 64;
            const uint32_t lane = threadIdx.x & 63u, g = lane / NCH, j = lane - g * NCH;
            for (uint32_t b0 = (threadIdx.x >> 6) * BPW; b0 < nb; b0 += NW * BPW) {
                const uint32_t b = b0 + g;
                if (g >= BPW || b >= nb) continue;
                const uint32_t c = cnt[b], f = fill[b];  // f: region fill, a multiple of 8
                const uint32_t rb = (b * ntiles + t) * cap;  // region start (< 2^31, host-checked)
                if (j * 8 < c) {
                    const uint4 w = *(const uint4 *)(bins + b * S + j * 8);
                    const uint32_t live = c - j * 8;  // valid indices in this chunk (>= 1)
                    uint32_t ww[4] = {w.x, w.y, w.z, w.w};
                    const uint32_t e0 = w.x & 0xffffu, hi0 = e0 << 16;
#pragma unroll
                    for (uint32_t i = 0; i < 4; ++i)  // pad with the chunk's first index
                        ww[i] = 2 * i + 1 < live ? ww[i] : 2 * i < live ? (ww[i] & 0xffffu) | hi0 : e0 | hi0;
                    const uint32_t e = f + j * 8;  // f and cap are multiples of 8: a chunk fits whole or not at all
                    if (e < cap) {
                        *(uint4 *)(regions + rb + e) = make_uint4(ww[0], ww[1], ww[2], ww[3]);
                    } else {  // the region is full: the run's bits by atomics
#pragma unroll
                        for (uint32_t i = 0; i < 8; ++i) bins_overflow_or(ovw, b, (ww[i >> 1] >> ((i & 1) * 16)) & 0xffffu);
                    }
                }
                if (j == 0) {
                    const uint32_t padded = (c + (PAD - 1)) & ~(PAD - 1);
                    if (c > S) {  // a run past its bin: pad its tail in the region
                        const uint16_t d = bins[b * S];
                        for (uint32_t e = f + c; e < f + padded; ++e)
                            if (e < cap) regions[(uint64_t)rb + e] = d;
                    }
                    cnt[b] = 0u;
                    fill[b] = f + padded;
                }
            }
        }
        __syncthreads();
    }
    for (uint32_t b = threadIdx.x; b < nb; b += THREADS) counts[(uint64_t)b * ntiles + t] = fill[b];
}

// ---- apply: one workgroup per bucket; stream its ntiles regions (16-B loads, 8 positions per
// lane), ds_or into an 8 KiB LDS image, OR the image into the filter words it owns.  FRESH (a new
// filter, its words never cleared): every word of the bucket, padding included, is written
// instead, and a bucket whose runs overflowed folds in (and re-zeroes) its words of the overflow
// bitmap `ovf`, which is all zero between builds.  PADDED: the runs were written by
// k_bkt_scatter_bins, whole 16-B chunks, so a region's count is a multiple of 8 and every index
// below it is valid (a chunk's padding repeats its first index; skipping it by a compare measured
// slower than OR-ing it: apply 43.0 vs 41.7 us, tools/diag/apply_or_padding.patch reversed).
template <int THREADS, bool FRESH, bool PADDED = false>
__global__ __launch_bounds__(THREADS) void k_bkt_apply(const uint16_t *__restrict__ regions,
                                                   const uint32_t *__restrict__ counts, uint32_t ntiles, uint32_t cap,
                                                   uint32_t *__restrict__ words, uint64_t nwords,
                                                   uint32_t *__restrict__ ovf) {
    __shared__ uint32_t img[kBktWords];
    __shared__ uint32_t cnt[kMaxTiles];
    __shared__ uint32_t spilled, longest;
    const uint32_t b = blockIdx.x;
    for (uint32_t j = threadIdx.x; j < kBktWords; j += blockDim.x) img[j] = 0u;
    if (threadIdx.x == 0) {
        spilled = 0u;
        longest = 0u;
    }
    __syncthreads();
    for (uint32_t t = threadIdx.x; t < ntiles; t += blockDim.x) {
        const uint32_t c = counts[(uint64_t)b * ntiles + t];
        if (c > cap) spilled = 1u;
        cnt[t] = min(c, cap);
        atomicMax(&longest, min(c, cap));
    }
    __syncthreads();
    // walk (tile, chunk) pairs only up to this bucket's longest region, not the capacity (which
    // keeps 8 sigma of headroom: ~30% fewer iterations at C2)
    const uint32_t stride = cap / 8;  // cap is a multiple of 8: regions are 16-B aligned
    const uint32_t chunks = (longest + 7) / 8;
    const uint32_t pairs = ntiles * chunks;
    const uint4 *reg = (const uint4 *)(regions + (uint64_t)b * ntiles * cap);
    // U chunk loads in flight per thread: they are issued before any count is consulted (every
    // chunk below the longest region lies inside its region's capacity, so a load past a shorter
    // region's count is in bounds and is simply not used); checking the count first put one load
    // per wave in flight at a time
    constexpr uint32_t U = 4;
    for (uint32_t q0 = threadIdx.x; q0 < pairs; q0 += U * THREADS) {
        uint4 v[U];
#pragma unroll
        for (uint32_t u = 0; u < U; ++u) {
            const uint32_t q = q0 + u * THREADS;
            if (q < pairs) {
                const uint32_t t = q / chunks, c = q - t * chunks;
                v[u] = reg[t * stride + c];
            }
        }
#pragma unroll
        for (uint32_t u = 0; u < U; ++u) {
            const uint32_t q = q0 + u * THREADS;
            if (q >= pairs) break;
            const uint32_t t = q / chunks, c = q - t * chunks;
            const uint32_t valid = cnt[t];
            if (c * 8 < valid) {
                const uint32_t w[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
#pragma unroll
                for (uint32_t e = 0; e < 8; ++e)
                    if (PADDED || c * 8 + e < valid) {  // PADDED: the padding ORs its chunk's first bit again
                        const uint32_t l = (w[e >> 1] >> ((e & 1) * 16)) & 0xffffu;
                        atomicOr(&img[l >> 5], 1u << (l & 31));
                    }
            }
        }
    }
    __syncthreads();
    const uint64_t w0 = (uint64_t)b * kBktWords;
    if constexpr (FRESH) {  // nwords: the allocated words (padding included)
        const bool sp = spilled != 0u;
        for (uint32_t j = threadIdx.x; j < kBktWords; j += blockDim.x)
            if (w0 + j < nwords) {
                uint32_t v = img[j];
                if (sp) {
                    v |= ovf[w0 + j];
                    ovf[w0 + j] = 0u;
                }
                words[w0 + j] = v;
            }
    } else {
        for (uint32_t j = threadIdx.x; j < kBktWords; j += blockDim.x) {
            const uint32_t v = img[j];
            if (v && w0 + j < nwords) words[w0 + j] |= v;
        }
    }
}

// ------------------------------------------------------------------ host side ---------------

struct BktPlan {
    uint32_t nb, tile_keys, ntiles, cap;  // a region of cap u16 per (bucket, tile)
    uint32_t round_keys;
    uint32_t bins;                        // k_bkt_scatter_bins' slots per bin (48 or 32), 0: the counting sort
    uint64_t off_regions, off_counts, bytes;
};

// The fixed-bin scatter takes k == 7 filters of kBinMinBuckets..kBinMaxBuckets buckets.
static uint32_t bin_slots(uint64_t m, uint32_t k) {
    const uint64_t nb = ((m + 31) / 32 + kBktWords - 1) / kBktWords;
    if (k != 7 || nb < kBinMinBuckets || nb > kBinMaxBuckets) return 0;
    return nb <= kBinBigMaxBuckets ? kBinBig : kBinSmall;
}
static uint32_t use_bins(uint64_t m, uint32_t k) { return options().scatter_bins ? bin_slots(m, k) : 0; }

// One 1024-thread scatter workgroup per CU (two of 512 measured slower).
constexpr uint32_t kScatterThreads = 1024;
// 5 keys per thread per round only while its sort buffer and the two per-bucket arrays fit the
// 160 KiB of LDS (nb <= 2551, m <= ~167M bits); 4 otherwise.
static uint32_t scatter_kpt(uint32_t nb) {
    return ((uint64_t)kScatterThreads * 5 * 7 + 2 * nb + 17) * 4 <= 160u * 1024 ? 5u : 4u;
}

static BktPlan plan_bucketed(uint64_t n, uint64_t m, uint32_t k, uint32_t bins) {
    BktPlan p{};
    const uint64_t nwords = (m + 31) / 32;
    p.nb = (uint32_t)((nwords + kBktWords - 1) / kBktWords);
    p.bins = bins;
    const uint32_t thr = kScatterThreads;
    const uint32_t kpt = bins ? 5u : scatter_kpt(p.nb);
    const uint32_t pos = thr * kpt * 7;
    uint32_t round_keys = k == 7 ? kpt * thr : pos / k;
    if (bins) {  // a round's mean run stays well below the bin
        const double mean = kBinMeanPos[bins == kBinBig];
        const uint64_t most = (uint64_t)(mean * (double)m / (double)(1u << kBktShift) / k);
        if (most < round_keys) round_keys = (uint32_t)(most > 64 ? most : 64);
    }
    const uint32_t target = kTargetTiles;
    uint64_t rounds_total = (n + round_keys - 1) / round_keys;
    uint64_t rounds_per_tile = (rounds_total + target - 1) / target;
    if (rounds_per_tile < 1) rounds_per_tile = 1;
    // (shrinking the rounds so C2's tiles are exactly 256 rather than 245 measured the same:
    // scatter 137.4 vs 137.3 us, profiles/r05c_tiles_exact_ab.txt)
    p.round_keys = round_keys;
    p.tile_keys = (uint32_t)(rounds_per_tile * round_keys);
    p.ntiles = (uint32_t)((n + p.tile_keys - 1) / p.tile_keys);
    // positions of one tile landing in one (full) bucket: mean + 8 sigma + 32, 8-aligned
    const double rkeys = (double)p.tile_keys;
    const double mu = rkeys * k * (double)(1u << kBktShift) / (double)m;
    double c = mu + 8.0 * sqrt(mu > 1 ? mu : 1) + 32.0;
    const double most = rkeys * k;  // never more than every position of the tile
    if (c > most) c = most;
    if (bins) c += 7.0 * (double)rounds_per_tile;  // each round's run padded to a multiple of 8
    p.cap = ((uint32_t)c + 7) & ~7u;
    auto al = [](uint64_t x) { return (x + 255) & ~255ull; };
    p.off_regions = 0;
    p.off_counts = al((uint64_t)p.nb * p.ntiles * p.cap * 2);
    p.bytes = al(p.off_counts + (uint64_t)p.nb * p.ntiles * 4);
    return p;
}

bool bucketed_supported(uint64_t m, uint32_t k) {
    const uint64_t nwords = (m + 31) / 32;
    const uint64_t nb = (nwords + kBktWords - 1) / kBktWords;
    return m >= 2 && nb <= kMaxBuckets && k >= 1 && k <= 64;
}

// Keys per launch: bounds the workspace and keeps tiles <= kMaxTiles.
uint64_t bucketed_max_keys(uint32_t k) { return (uint64_t)kMaxTiles * (kTilePos / (k ? k : 1)) * 4; }

uint64_t bucketed_workspace_bytes(uint64_t n, uint64_t m, uint32_t k) {
    if (!bucketed_supported(m, k) || n == 0) return 0;
    const uint64_t cap = bucketed_max_keys(k);
    const uint64_t nn = n < cap ? n : cap;
    // either scatter may run (scatter_bins can change between the query and the build)
    const uint64_t a = plan_bucketed(nn, m, k, 0).bytes;
    const uint32_t sl = bin_slots(m, k);
    const uint64_t b = sl ? plan_bucketed(nn, m, k, sl).bytes : 0;
    return a > b ? a : b;
}

// One launch pair (scatter + apply) per chunk of at most bucketed_max_keys keys; `chunk(k0, n)`
// calls fn with the key source of keys [k0, k0 + n).
// ovf != null: a fresh build (see k_bkt_apply); the first chunk writes the words, later chunks OR.
template <typename Chunk>
static hipError_t run_bucketed(uint64_t n, const ModArg &md, uint32_t *words, void *ws, uint64_t ws_bytes,
                               hipStream_t s, uint32_t *ovf, Chunk &&chunk) {
    const uint64_t maxk = bucketed_max_keys(md.k);
    for (uint64_t k0 = 0; k0 < n; k0 += maxk) {  // OR-accumulative: split large batches
        const bool fresh = ovf && k0 == 0;
        const uint64_t sn = n - k0 < maxk ? n - k0 : maxk;
        const BktPlan p = plan_bucketed(sn, md.m, md.k, use_bins(md.m, md.k));
        if (p.bytes > ws_bytes || p.ntiles > kMaxTiles) return hipErrorInvalidValue;
        if ((uint64_t)p.nb * p.ntiles * p.cap >= (1ull << 31)) return hipErrorInvalidValue;  // u32 region index
        uint8_t *w = (uint8_t *)ws;
        uint16_t *regions = (uint16_t *)(w + p.off_regions);
        uint32_t *counts = (uint32_t *)(w + p.off_counts);
        const uint64_t nwords = (md.m + 31) / 32;
        const uint32_t kpt = scatter_kpt(p.nb);
        const size_t lds = ((size_t)kScatterThreads * kpt * 7 + 2 * p.nb + 17) * sizeof(uint32_t);
        hipError_t e = chunk(k0, sn, [&](auto src) -> hipError_t {
            using S = decltype(src);
            if (p.bins) {
                // (two keys per pipeline step, G = 2: scatter 138.6 vs 137.9 us, not kept)
                auto scat = p.bins == kBinBig ? k_bkt_scatter_bins<S, kScatterThreads, 5, kBinBig>
                                              : k_bkt_scatter_bins<S, kScatterThreads, 5, kBinSmall>;
                const size_t blds = bin_lds_bytes(p.nb, p.bins);
                hipError_t a = hipFuncSetAttribute((const void *)scat, hipFuncAttributeMaxDynamicSharedMemorySize, (int)blds);
                if (a != hipSuccess) return a;
                hipLaunchKernelGGL(scat, dim3(p.ntiles), dim3(kScatterThreads), blds, s, src, sn, md, p.nb, p.tile_keys,
                                   p.round_keys, p.ntiles, p.cap, regions, counts, fresh ? ovf : words);
                if (fresh)
                    hipLaunchKernelGGL((k_bkt_apply<1024, true, true>), dim3(p.nb), dim3(1024), 0, s, regions, counts,
                                       p.ntiles, p.cap, words, (md.m + 127) / 128 * 4, ovf);
                else
                    hipLaunchKernelGGL((k_bkt_apply<1024, false, true>), dim3(p.nb), dim3(1024), 0, s, regions, counts,
                                       p.ntiles, p.cap, words, nwords, nullptr);
                return hipGetLastError();
            }
            constexpr int K0 = IsPacked<S>::value ? 7 : 0;  // packed sources have no generic-k kernel
            auto scat = kpt == 5 ? (md.k == 7 ? k_bkt_scatter<S, 7, kScatterThreads, 5> : k_bkt_scatter<S, K0, kScatterThreads, 5>)
                                 : (md.k == 7 ? k_bkt_scatter<S, 7, kScatterThreads, 4> : k_bkt_scatter<S, K0, kScatterThreads, 4>);
            hipError_t a = hipFuncSetAttribute((const void *)scat, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
            if (a != hipSuccess) return a;
            hipLaunchKernelGGL(scat, dim3(p.ntiles), dim3(kScatterThreads), lds, s, src, sn, md, p.nb, p.tile_keys,
                               p.ntiles, p.cap, regions, counts, fresh ? ovf : words);
            // apply: 1024 threads per bucket (256 and 512 measured slower)
            if (fresh)
                hipLaunchKernelGGL((k_bkt_apply<1024, true>), dim3(p.nb), dim3(1024), 0, s, regions, counts, p.ntiles,
                                   p.cap, words, (md.m + 127) / 128 * 4, ovf);
            else
                hipLaunchKernelGGL((k_bkt_apply<1024, false>), dim3(p.nb), dim3(1024), 0, s, regions, counts, p.ntiles,
                                   p.cap, words, nwords, nullptr);
            return hipGetLastError();
        });
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

hipError_t launch_build_bucketed(const KeyBatch &kb, uint32_t *words, const ModArg &md, void *ws, uint64_t ws_bytes,
                                 hipStream_t s, uint32_t *ovf) {
    if (kb.n == 0 || md.k == 0) return hipSuccess;
    return run_bucketed(kb.n, md, words, ws, ws_bytes, s, ovf, [&](uint64_t k0, uint64_t sn, auto &&fn) {
        KeyBatch sub = kb;
        sub.n = sn;
        if (kb.hashes)
            sub.hashes = kb.hashes + k0;
        else if (kb.offsets)
            sub.offsets = kb.offsets + k0;
        else
            sub.data = kb.data + k0 * (uint64_t)kb.stride;
        return with_src(sub, fn);
    });
}

hipError_t launch_build_bucketed_packed(const uint64_t *packed, uint64_t n, uint32_t *words, const ModArg &md,
                                        void *ws, uint64_t ws_bytes, hipStream_t s, uint32_t *ovf) {
    if (n == 0) return hipSuccess;
    if (md.k != 7 || md.m >= (1ull << kPackBits)) return hipErrorInvalidValue;
    return run_bucketed(n, md, words, ws, ws_bytes, s, ovf,
                        [&](uint64_t k0, uint64_t, auto &&fn) { return fn(KeysPacked{packed + k0}); });
}

}  // namespace seb
