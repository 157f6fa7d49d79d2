// seb_bucket.hip — radix-partitioned bloom build: no global atomics on the filter.
//
// The reference ORs k bits per key straight into the bit array (lsm/bloom.go:70-77).  Done
// with device-scope atomics on gfx950 every OR is a memory-side atomic (TCC_EA0_ATOMIC = n*k;
// profiles/r01), which caps the build at ~27 G bit-sets/s.  This path instead partitions the
// n*k bit positions by 64 Ki-bit bucket (one 8 KiB LDS image each) and sets the bits in LDS:
//
//   A  k_bkt_count    tile of keys per workgroup -> per-(tile, bucket) counts      [ntiles][nb]
//   B  k_bkt_scan_*   exclusive scan in bucket-major order -> global run offsets    [nb][ntiles]
//   C  k_bkt_scatter  re-hash the tile, counting-sort its positions by bucket in LDS, write each
//                     bucket run (u16 in-bucket bit index) contiguously to its global offset
//   D  k_bkt_apply    one workgroup per bucket: stream its contiguous run, ds_or into an 8 KiB
//                     LDS image, OR the image into the filter words (the workgroup owns them)
//
// The result is the same bit array bit for bit (OR is order-independent).  Requires m <= 2^28
// (<= 4096 buckets) and n*k < 2^32 per launch; the host splits larger batches.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "seb_device.h"
#include "seb_kernels.h"

namespace seb {

constexpr int kBktShift = 16;                            // 64 Ki bits per bucket
constexpr uint32_t kBktWords = 1u << (kBktShift - 5);   // 2048 u32 words = 8 KiB of LDS
constexpr uint32_t kMaxBuckets = 4096;                   // m <= 2^28 bits
constexpr uint32_t kTileThreads = 1024;
constexpr uint32_t kTilePos = 28672;                     // positions per tile sorted in LDS (112 KiB)
constexpr uint32_t kScanThreads = 1024;
constexpr uint32_t kScanPer = 8;
constexpr uint32_t kSeg = kScanThreads * kScanPer;       // elements scanned per block in pass B
constexpr uint32_t kKpt7 = 4;                            // keys per thread in pass C when k == 7

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

// ---- A: per-(tile, bucket) counts, tile-major (coalesced row per workgroup)
template <typename Src, int KFIX>
__global__ __launch_bounds__(kTileThreads) void k_bkt_count(Src src, uint64_t n, ModArg md, uint32_t nb,
                                                            uint32_t tile_keys, uint32_t *__restrict__ counts) {
    __shared__ uint32_t hist[kMaxBuckets];
    for (uint32_t b = threadIdx.x; b < nb; b += blockDim.x) hist[b] = 0u;
    __syncthreads();
    const uint64_t k0 = (uint64_t)blockIdx.x * tile_keys;
    const uint64_t k1 = k0 + tile_keys < n ? k0 + tile_keys : n;
    for (uint64_t i = k0 + threadIdx.x; i < k1; i += blockDim.x) {
        uint64_t h1, h2;
        src.hash(i, h1, h2);
        for_positions<KFIX, true>(h1, h2, md, md.k,
                                  [&](uint32_t, uint64_t p) { atomicAdd(&hist[(uint32_t)p >> kBktShift], 1u); });
    }
    __syncthreads();
    uint32_t *row = counts + (uint64_t)blockIdx.x * nb;
    for (uint32_t b = threadIdx.x; b < nb; b += blockDim.x) row[b] = hist[b];
}

// ---- B1: exclusive scan of counts read in bucket-major order v = b*ntiles + t, per segment
__global__ __launch_bounds__(kScanThreads) void k_bkt_scan_seg(const uint32_t *__restrict__ counts, uint32_t nb,
                                                               uint32_t ntiles, uint32_t *__restrict__ offs,
                                                               uint32_t *__restrict__ segsum) {
    __shared__ uint32_t wsum[kScanThreads / 64];
    const uint64_t len = (uint64_t)nb * ntiles;
    const uint64_t base = (uint64_t)blockIdx.x * kSeg;
    uint32_t carry = 0;
    for (uint32_t j = 0; j < kScanPer; ++j) {
        const uint64_t v = base + (uint64_t)j * kScanThreads + threadIdx.x;
        uint32_t x = 0;
        if (v < len) {
            const uint32_t b = (uint32_t)(v / ntiles), t = (uint32_t)(v % ntiles);
            x = counts[(uint64_t)t * nb + b];
        }
        uint32_t tot;
        const uint32_t pre = block_exclusive_scan(x, wsum, &tot);
        if (v < len) offs[v] = carry + pre;
        carry += tot;
    }
    if (threadIdx.x == 0) segsum[blockIdx.x] = carry;
}

// ---- B2: exclusive scan of the segment sums in place (one workgroup)
__global__ __launch_bounds__(kScanThreads) void k_bkt_scan_top(uint32_t *__restrict__ segsum, uint32_t nseg) {
    __shared__ uint32_t wsum[kScanThreads / 64];
    uint32_t carry = 0;
    for (uint32_t c = 0; c < nseg; c += kScanThreads) {
        const uint32_t i = c + threadIdx.x;
        const uint32_t x = i < nseg ? segsum[i] : 0u;
        uint32_t tot;
        const uint32_t pre = block_exclusive_scan(x, wsum, &tot);
        if (i < nseg) segsum[i] = carry + pre;
        carry += tot;
    }
}

__device__ __forceinline__ uint32_t run_offset(const uint32_t *offs, const uint32_t *segsum, uint64_t v) {
    return offs[v] + segsum[v / kSeg];
}

// ---- C: counting-sort one tile's positions by bucket in LDS, write runs to global.
// LDS: sorted[kTilePos] u32 | cursor[nb] | delta[nb] | wsum[16]
template <typename Src, int KFIX>
__global__ __launch_bounds__(kTileThreads) void k_bkt_scatter(Src src, uint64_t n, ModArg md, uint32_t nb,
                                                              uint32_t tile_keys, uint32_t ntiles,
                                                              const uint32_t *__restrict__ offs,
                                                              const uint32_t *__restrict__ segsum,
                                                              uint16_t *__restrict__ local_out) {
    extern __shared__ uint32_t smem[];
    uint32_t *sorted = smem;
    uint32_t *cursor = smem + kTilePos;
    uint32_t *delta = cursor + kMaxBuckets;
    uint32_t *wsum = delta + kMaxBuckets;
    const uint32_t t = blockIdx.x;
    for (uint32_t b = threadIdx.x; b < nb; b += blockDim.x) cursor[b] = 0u;
    __syncthreads();
    const uint64_t k0 = (uint64_t)t * tile_keys;
    const uint64_t k1 = k0 + tile_keys < n ? k0 + tile_keys : n;

    constexpr int KP = KFIX > 0 ? (int)kKpt7 : 1;
    constexpr int KQ = KFIX > 0 ? KFIX : 1;
    uint32_t pos[KP][KQ];
    if constexpr (KFIX > 0) {  // positions stay in registers between counting and placing
#pragma unroll
        for (int r = 0; r < KP; ++r) {
            const uint64_t i = k0 + (uint64_t)r * blockDim.x + threadIdx.x;
            if (i < k1) {
                uint64_t h1, h2;
                src.hash(i, h1, h2);
                for_positions<KFIX, true>(h1, h2, md, KFIX, [&](uint32_t q, uint64_t p) { pos[r][q] = (uint32_t)p; });
#pragma unroll
                for (int q = 0; q < KQ; ++q) atomicAdd(&cursor[pos[r][q] >> kBktShift], 1u);
            }
        }
    } else {
        for (uint64_t i = k0 + threadIdx.x; i < k1; i += blockDim.x) {
            uint64_t h1, h2;
            src.hash(i, h1, h2);
            for_positions<0, true>(h1, h2, md, md.k,
                                   [&](uint32_t, uint64_t p) { atomicAdd(&cursor[(uint32_t)p >> kBktShift], 1u); });
        }
    }
    __syncthreads();
    // exclusive scan of the bucket counts (each thread owns up to 4 consecutive buckets)
    {
        const uint32_t per = (nb + blockDim.x - 1) / blockDim.x;
        const uint32_t b0 = threadIdx.x * per;
        uint32_t c[4] = {0u, 0u, 0u, 0u}, s = 0;
        for (uint32_t j = 0; j < per && j < 4; ++j)
            if (b0 + j < nb) {
                c[j] = cursor[b0 + j];
                s += c[j];
            }
        uint32_t tot;
        uint32_t pre = block_exclusive_scan(s, wsum, &tot);
        for (uint32_t j = 0; j < per && j < 4; ++j)
            if (b0 + j < nb) {
                const uint32_t b = b0 + j;
                cursor[b] = pre;
                delta[b] = run_offset(offs, segsum, (uint64_t)b * ntiles + t) - pre;
                pre += c[j];
            }
    }
    __syncthreads();
    if constexpr (KFIX > 0) {
#pragma unroll
        for (int r = 0; r < KP; ++r) {
            const uint64_t i = k0 + (uint64_t)r * blockDim.x + threadIdx.x;
            if (i < k1) {
#pragma unroll
                for (int q = 0; q < KQ; ++q) sorted[atomicAdd(&cursor[pos[r][q] >> kBktShift], 1u)] = pos[r][q];
            }
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
    const uint32_t cnt = (uint32_t)(k1 > k0 ? (k1 - k0) : 0) * md.k;
    for (uint32_t idx = threadIdx.x; idx < cnt; idx += blockDim.x) {
        const uint32_t p = sorted[idx];
        local_out[delta[p >> kBktShift] + idx] = (uint16_t)p;
    }
}

// ---- D: one workgroup per bucket, LDS image, OR into the filter words
__global__ __launch_bounds__(256) void k_bkt_apply(const uint16_t *__restrict__ local, const uint32_t *__restrict__ offs,
                                                   const uint32_t *__restrict__ segsum, uint32_t nb, uint32_t ntiles,
                                                   uint32_t total, uint32_t *__restrict__ words, uint64_t nwords) {
    __shared__ uint32_t img[kBktWords];
    const uint32_t b = blockIdx.x;
    for (uint32_t j = threadIdx.x; j < kBktWords; j += blockDim.x) img[j] = 0u;
    __syncthreads();
    const uint32_t s = run_offset(offs, segsum, (uint64_t)b * ntiles);
    const uint32_t e = b + 1 < nb ? run_offset(offs, segsum, (uint64_t)(b + 1) * ntiles) : total;
    for (uint32_t i = s + threadIdx.x; i < e; i += blockDim.x) {
        const uint32_t l = local[i];
        atomicOr(&img[l >> 5], 1u << (l & 31));
    }
    __syncthreads();
    const uint64_t w0 = (uint64_t)b * kBktWords;
    for (uint32_t j = threadIdx.x; j < kBktWords; j += blockDim.x) {
        const uint32_t v = img[j];
        if (v && w0 + j < nwords) words[w0 + j] |= v;
    }
}

// ------------------------------------------------------------------ host side ---------------

struct BktPlan {
    uint32_t nb, tile_keys, ntiles, nseg, total;
    uint64_t off_counts, off_offs, off_seg, off_local, bytes;
};

static BktPlan plan_bucketed(uint64_t n, uint64_t m, uint32_t k) {
    BktPlan p{};
    const uint64_t nwords = (m + 31) / 32;
    p.nb = (uint32_t)((nwords + kBktWords - 1) / kBktWords);
    p.tile_keys = k == 7 ? kKpt7 * kTileThreads : kTilePos / k;
    p.ntiles = (uint32_t)((n + p.tile_keys - 1) / p.tile_keys);
    const uint64_t len = (uint64_t)p.nb * p.ntiles;
    p.nseg = (uint32_t)((len + kSeg - 1) / kSeg);
    p.total = (uint32_t)(n * k);
    auto al = [](uint64_t x) { return (x + 255) & ~255ull; };
    p.off_counts = 0;
    p.off_offs = al(p.off_counts + len * 4);
    p.off_seg = al(p.off_offs + len * 4);
    p.off_local = al(p.off_seg + (uint64_t)p.nseg * 4);
    p.bytes = al(p.off_local + (uint64_t)p.total * 2);
    return p;
}

bool bucketed_supported(uint64_t m, uint32_t k) {
    const uint64_t nwords = (m + 31) / 32;
    const uint64_t nb = (nwords + kBktWords - 1) / kBktWords;
    return m >= 2 && nb <= kMaxBuckets && k >= 1 && k <= 64;
}

// Largest key count per launch so that n*k < 2^31 and the scan stays small.
uint64_t bucketed_max_keys(uint32_t k) { return (1ull << 31) / (k ? k : 1) / 2; }

uint64_t bucketed_workspace_bytes(uint64_t n, uint64_t m, uint32_t k) {
    if (!bucketed_supported(m, k) || n == 0) return 0;
    const uint64_t cap = bucketed_max_keys(k);
    return plan_bucketed(n < cap ? n : cap, m, k).bytes;
}

hipError_t launch_build_bucketed(const KeyBatch &kb, uint32_t *words, const ModArg &md, void *ws, uint64_t ws_bytes,
                                 hipStream_t s) {
    if (kb.n == 0 || md.k == 0) return hipSuccess;
    const uint64_t cap = bucketed_max_keys(md.k);
    for (uint64_t k0 = 0; k0 < kb.n; k0 += cap) {  // OR-accumulative: split large batches
        KeyBatch sub = kb;
        sub.n = kb.n - k0 < cap ? kb.n - k0 : cap;
        if (kb.offsets)
            sub.offsets = kb.offsets + k0;
        else
            sub.data = kb.data + k0 * (uint64_t)kb.stride;
        const BktPlan p = plan_bucketed(sub.n, md.m, md.k);
        if (p.bytes > ws_bytes) return hipErrorInvalidValue;
        uint8_t *w = (uint8_t *)ws;
        uint32_t *counts = (uint32_t *)(w + p.off_counts), *offs = (uint32_t *)(w + p.off_offs);
        uint32_t *seg = (uint32_t *)(w + p.off_seg);
        uint16_t *local = (uint16_t *)(w + p.off_local);
        const uint64_t nwords = (md.m + 31) / 32;
        const size_t lds_c = (kTilePos + 2 * kMaxBuckets + 16) * sizeof(uint32_t);
        hipError_t e = with_src(sub, [&](auto src) -> hipError_t {
            using S = decltype(src);
            const bool k7 = md.k == 7;
            if (k7)
                hipLaunchKernelGGL((k_bkt_count<S, 7>), dim3(p.ntiles), dim3(kTileThreads), 0, s, src, sub.n, md, p.nb,
                                   p.tile_keys, counts);
            else
                hipLaunchKernelGGL((k_bkt_count<S, 0>), dim3(p.ntiles), dim3(kTileThreads), 0, s, src, sub.n, md, p.nb,
                                   p.tile_keys, counts);
            hipLaunchKernelGGL(k_bkt_scan_seg, dim3(p.nseg), dim3(kScanThreads), 0, s, counts, p.nb, p.ntiles, offs, seg);
            hipLaunchKernelGGL(k_bkt_scan_top, dim3(1), dim3(kScanThreads), 0, s, seg, p.nseg);
            auto scat = k7 ? k_bkt_scatter<S, 7> : k_bkt_scatter<S, 0>;
            hipError_t a = hipFuncSetAttribute((const void *)scat, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_c);
            if (a != hipSuccess) return a;
            hipLaunchKernelGGL(scat, dim3(p.ntiles), dim3(kTileThreads), lds_c, s, src, sub.n, md, p.nb, p.tile_keys,
                               p.ntiles, offs, seg, local);
            hipLaunchKernelGGL(k_bkt_apply, dim3(p.nb), dim3(256), 0, s, local, offs, seg, p.nb, p.ntiles, p.total,
                               words, nwords);
            return hipGetLastError();
        });
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

}  // namespace seb
