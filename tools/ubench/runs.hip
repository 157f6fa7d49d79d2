// runs.hip — calibrate WRITE_SIZE for the bucketed build's u16 run stores.
//
// k_bkt_scatter writes 70M u16 bit indices (140 MB at C2) as runs of ~24.5 elements (one per
// bucket per 5120-key round) appended to fixed regions [bucket][tile][cap]; rocprof's WRITE_SIZE
// reports ~231-257 MB per launch for it.  Three kernels store the same 140 MB:
//   0 contiguous  one u16 per lane, lane-consecutive addresses (a fully coalesced 2-B stream)
//   1 scatter     the scatter's store pattern without the hashing: per tile (one 1024-thread
//                 workgroup) 8 rounds of 35,840 positions (35 per thread, a cheap integer hash
//                 over 1463 buckets), counting-sorted in LDS, each bucket's run appended to its
//                 region with one u16 store per lane, as k_bkt_scatter's write-out loop does
//   2 whole       the same regions, each written once, contiguously (the ideal layout: what the
//                 runs add up to)
// Mode 1 with --stream also reads a 160 MB key stream (16 B per key, non-temporal, as the real
// scatter does) between rounds, to put the same pressure on L2 between a region's runs.
// Usage: runs MODE [--stream]  -> one JSON line {mode, bytes, us}; run WRITE_SIZE under rocprofv3.
// Build: hipcc --offload-arch=gfx950 -O3 runs.hip -o runs
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstring>

constexpr uint32_t kNb = 1463, kTiles = 245, kCap = 344, kRounds = 8, kThreads = 1024, kKpt = 5, kK = 7;
constexpr uint32_t kPos = kThreads * kKpt * kK;  // 35,840 positions per round
constexpr uint64_t kKeys = (uint64_t)kTiles * kRounds * kThreads * kKpt;

#define CK(x)                                                                                  \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) {                                                                \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                            \
            return 1;                                                                          \
        }                                                                                      \
    } while (0)

__device__ __forceinline__ uint32_t mix(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    x ^= x >> 16;
    return x;
}

__global__ void k_contig(uint16_t *out, uint64_t n) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        out[i] = (uint16_t)i;
}

template <bool STREAM>
__global__ __launch_bounds__(kThreads) void k_scatter_like(uint16_t *regions, uint32_t *counts, const uint4 *keys,
                                                           uint32_t *sink) {
    __shared__ uint32_t sorted[kPos];
    __shared__ uint32_t cursor[kNb];
    __shared__ uint32_t fill[kNb];
    __shared__ uint32_t wsum[16];
    const uint32_t t = blockIdx.x;
    for (uint32_t b = threadIdx.x; b < kNb; b += kThreads) {
        cursor[b] = 0;
        fill[b] = 0;
    }
    __syncthreads();
    uint32_t acc = 0;
    for (uint32_t r = 0; r < kRounds; ++r) {
        uint32_t pos[kKpt * kK];
#pragma unroll
        for (uint32_t q = 0; q < kKpt * kK; ++q) {
            const uint32_t h = mix((t * kRounds + r) * kPos + q * kThreads + threadIdx.x + 0x9e3779b9u);
            pos[q] = (uint32_t)(((uint64_t)h * (kNb * 65536ull)) >> 32);  // a bit index in [0, nb * 2^16)
            atomicAdd(&cursor[pos[q] >> 16], 1u);
        }
        if constexpr (STREAM) {  // the round's 5120 keys, as the scatter streams them
#pragma unroll
            for (uint32_t j = 0; j < kKpt; ++j) {
                const uint64_t i = ((uint64_t)(t * kRounds + r) * kKpt + j) * kThreads + threadIdx.x;
                typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
                const u32x4 v = __builtin_nontemporal_load((const u32x4 *)(keys + i));
                acc += v.x ^ v.w;
            }
        }
        __syncthreads();
        {  // exclusive scan of the bucket counts (per thread <= 2 buckets)
            const uint32_t b0 = threadIdx.x * 2;
            const uint32_t c0 = b0 < kNb ? cursor[b0] : 0u, c1 = b0 + 1 < kNb ? cursor[b0 + 1] : 0u;
            uint32_t v = c0 + c1;
            const uint32_t lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
            uint32_t x = v;
#pragma unroll
            for (int d = 1; d < 64; d <<= 1) {
                const uint32_t y = __shfl_up(x, d, 64);
                if (lane >= (uint32_t)d) x += y;
            }
            if (lane == 63) wsum[wid] = x;
            __syncthreads();
            if (wid == 0) {
                uint32_t s = lane < 16 ? wsum[lane] : 0u;
#pragma unroll
                for (int d = 1; d < 16; d <<= 1) {
                    const uint32_t y = __shfl_up(s, d, 64);
                    if (lane >= (uint32_t)d) s += y;
                }
                if (lane < 16) wsum[lane] = s;
            }
            __syncthreads();
            const uint32_t pre = (wid ? wsum[wid - 1] : 0u) + x - v;
            if (b0 < kNb) cursor[b0] = pre;
            if (b0 + 1 < kNb) cursor[b0 + 1] = pre + c0;
        }
        __syncthreads();
        uint32_t slot[kKpt * kK];
#pragma unroll
        for (uint32_t q = 0; q < kKpt * kK; ++q) slot[q] = atomicAdd(&cursor[pos[q] >> 16], 1u);
#pragma unroll
        for (uint32_t q = 0; q < kKpt * kK; ++q) sorted[slot[q]] = pos[q];
        __syncthreads();
        for (uint32_t b = threadIdx.x; b < kNb; b += kThreads) {
            const uint32_t start = b ? cursor[b - 1] : 0u;
            fill[b] = (b * kTiles + t) * kCap + fill[b] - start;
        }
        __syncthreads();
#pragma unroll 5
        for (uint32_t idx = threadIdx.x; idx < kPos; idx += kThreads) {
            const uint32_t p = sorted[idx];
            regions[fill[p >> 16] + idx] = (uint16_t)p;
        }
        __syncthreads();
        for (uint32_t b = threadIdx.x; b < kNb; b += kThreads) {
            fill[b] += cursor[b] - (b * kTiles + t) * kCap;
            cursor[b] = 0u;
        }
        __syncthreads();
    }
    for (uint32_t b = threadIdx.x; b < kNb; b += kThreads) counts[(uint64_t)b * kTiles + t] = fill[b];
    if (STREAM && acc == 0x12345678u) sink[0] = acc;
}

// Every region written once, contiguously: one wave per region, its count u16 (from mode 1's counts).
__global__ void k_whole(uint16_t *regions, const uint32_t *counts) {
    const uint32_t lane = threadIdx.x & 63;
    for (uint64_t reg = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; reg < (uint64_t)kNb * kTiles;
         reg += ((uint64_t)gridDim.x * blockDim.x) >> 6) {
        const uint32_t c = counts[reg] < kCap ? counts[reg] : kCap;
        for (uint32_t e = lane; e < c; e += 64) regions[reg * kCap + e] = (uint16_t)(reg + e);
    }
}

int main(int argc, char **argv) {
    const int mode = argc > 1 ? atoi(argv[1]) : 0;
    const bool stream = argc > 2 && !strcmp(argv[2], "--stream");
    const uint64_t rbytes = (uint64_t)kNb * kTiles * kCap * 2;
    uint16_t *regions;
    uint32_t *counts, *sink;
    uint4 *keys = nullptr;
    CK(hipMalloc(&regions, rbytes + (1 << 20)));
    CK(hipMalloc(&counts, (uint64_t)kNb * kTiles * 4));
    CK(hipMalloc(&sink, 64));
    CK(hipMemset(regions, 0, rbytes));
    CK(hipMemset(counts, 0, (uint64_t)kNb * kTiles * 4));
    if (stream) {
        CK(hipMalloc(&keys, kKeys * 16));
        CK(hipMemset(keys, 1, kKeys * 16));
    }
    const uint64_t npos = kKeys * kK;  // 70.2M positions = 140 MB of u16
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    // mode 2 needs mode 1's counts: run the scatter once first (not timed)
    if (mode == 2) {
        hipLaunchKernelGGL((k_scatter_like<false>), dim3(kTiles), dim3(kThreads), 0, 0, regions, counts, keys, sink);
        CK(hipGetLastError());
        CK(hipDeviceSynchronize());
    }
    float best = 1e30f;
    for (int rep = 0; rep < 5; ++rep) {
        CK(hipEventRecord(a, 0));
        if (mode == 0)
            hipLaunchKernelGGL(k_contig, dim3(8192), dim3(256), 0, 0, regions, npos);
        else if (mode == 1 && stream)
            hipLaunchKernelGGL((k_scatter_like<true>), dim3(kTiles), dim3(kThreads), 0, 0, regions, counts, keys, sink);
        else if (mode == 1)
            hipLaunchKernelGGL((k_scatter_like<false>), dim3(kTiles), dim3(kThreads), 0, 0, regions, counts, keys, sink);
        else
            hipLaunchKernelGGL(k_whole, dim3(8192), dim3(256), 0, 0, regions, counts);
        CK(hipGetLastError());
        CK(hipEventRecord(b, 0));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        if (ms < best) best = ms;
    }
    printf("{\"mode\": %d, \"stream\": %d, \"u16_stored\": %llu, \"bytes\": %llu, \"us\": %.2f}\n", mode, stream ? 1 : 0,
           (unsigned long long)npos, (unsigned long long)npos * 2, best * 1e3);
    return 0;
}
