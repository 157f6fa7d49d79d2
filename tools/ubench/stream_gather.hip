// stream_gather.hip — does a coalesced key stream compete with random gathers for a CU's vector
// memory path, and does streaming through the scalar data path (s_load into SGPRs, then
// v_writelane into the lanes) leave the gathers their full rate?  Each thread owns one 16-B key;
// modes:
//   0 vector stream only       (16-B nontemporal load per lane, fold, 4-B store)
//   1 gathers only             (7 dependent conditional gathers from a 4 MiB table, as in a probe
//                               phase: the next gather waits for the previous one's result)
//   2 vector stream + gathers  (gather addresses from the streamed key)
//   3 scalar stream + gathers  (the wave's 1 KiB of keys by s_load_dwordx16, v_writelane to lanes)
//   4 scalar stream only
// Build: hipcc --offload-arch=gfx950 -O3 stream_gather.hip -o stream_gather
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <utility>

typedef uint32_t u32x16 __attribute__((ext_vector_type(16)));
typedef __attribute__((address_space(4))) const u32x16 *cu32x16p;

__device__ inline uint32_t mix(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
    return x;
}

// SGPR value -> one lane of a VGPR (the lane an inline constant: one SGPR read per instruction)
template <int LANE>
__device__ inline void wl(uint32_t &v, uint32_t s) {
    asm("v_writelane_b32 %0, %1, %2" : "+v"(v) : "s"(s), "i"(LANE));
}

template <int CH>
__device__ inline void chunk(cu32x16p p, uint32_t &a, uint32_t &b, uint32_t &c, uint32_t &d) {
    const u32x16 s = p[CH];  // 4 keys (64 B) per s_load_dwordx16
    wl<CH * 4 + 0>(a, s[0]); wl<CH * 4 + 0>(b, s[1]); wl<CH * 4 + 0>(c, s[2]); wl<CH * 4 + 0>(d, s[3]);
    wl<CH * 4 + 1>(a, s[4]); wl<CH * 4 + 1>(b, s[5]); wl<CH * 4 + 1>(c, s[6]); wl<CH * 4 + 1>(d, s[7]);
    wl<CH * 4 + 2>(a, s[8]); wl<CH * 4 + 2>(b, s[9]); wl<CH * 4 + 2>(c, s[10]); wl<CH * 4 + 2>(d, s[11]);
    wl<CH * 4 + 3>(a, s[12]); wl<CH * 4 + 3>(b, s[13]); wl<CH * 4 + 3>(c, s[14]); wl<CH * 4 + 3>(d, s[15]);
}
template <int G>
__device__ inline void chunk4(cu32x16p p, uint32_t &a, uint32_t &b, uint32_t &c, uint32_t &d) {
    const u32x16 s0 = p[4 * G], s1 = p[4 * G + 1], s2 = p[4 * G + 2], s3 = p[4 * G + 3];
    const u32x16 ss[4] = {s0, s1, s2, s3};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const u32x16 s = ss[j];
        (void)s;
    }
    wl<G * 16 + 0>(a, s0[0]); wl<G * 16 + 0>(b, s0[1]); wl<G * 16 + 0>(c, s0[2]); wl<G * 16 + 0>(d, s0[3]);
    wl<G * 16 + 1>(a, s0[4]); wl<G * 16 + 1>(b, s0[5]); wl<G * 16 + 1>(c, s0[6]); wl<G * 16 + 1>(d, s0[7]);
    wl<G * 16 + 2>(a, s0[8]); wl<G * 16 + 2>(b, s0[9]); wl<G * 16 + 2>(c, s0[10]); wl<G * 16 + 2>(d, s0[11]);
    wl<G * 16 + 3>(a, s0[12]); wl<G * 16 + 3>(b, s0[13]); wl<G * 16 + 3>(c, s0[14]); wl<G * 16 + 3>(d, s0[15]);
    wl<G * 16 + 4>(a, s1[0]); wl<G * 16 + 4>(b, s1[1]); wl<G * 16 + 4>(c, s1[2]); wl<G * 16 + 4>(d, s1[3]);
    wl<G * 16 + 5>(a, s1[4]); wl<G * 16 + 5>(b, s1[5]); wl<G * 16 + 5>(c, s1[6]); wl<G * 16 + 5>(d, s1[7]);
    wl<G * 16 + 6>(a, s1[8]); wl<G * 16 + 6>(b, s1[9]); wl<G * 16 + 6>(c, s1[10]); wl<G * 16 + 6>(d, s1[11]);
    wl<G * 16 + 7>(a, s1[12]); wl<G * 16 + 7>(b, s1[13]); wl<G * 16 + 7>(c, s1[14]); wl<G * 16 + 7>(d, s1[15]);
    wl<G * 16 + 8>(a, s2[0]); wl<G * 16 + 8>(b, s2[1]); wl<G * 16 + 8>(c, s2[2]); wl<G * 16 + 8>(d, s2[3]);
    wl<G * 16 + 9>(a, s2[4]); wl<G * 16 + 9>(b, s2[5]); wl<G * 16 + 9>(c, s2[6]); wl<G * 16 + 9>(d, s2[7]);
    wl<G * 16 + 10>(a, s2[8]); wl<G * 16 + 10>(b, s2[9]); wl<G * 16 + 10>(c, s2[10]); wl<G * 16 + 10>(d, s2[11]);
    wl<G * 16 + 11>(a, s2[12]); wl<G * 16 + 11>(b, s2[13]); wl<G * 16 + 11>(c, s2[14]); wl<G * 16 + 11>(d, s2[15]);
    wl<G * 16 + 12>(a, s3[0]); wl<G * 16 + 12>(b, s3[1]); wl<G * 16 + 12>(c, s3[2]); wl<G * 16 + 12>(d, s3[3]);
    wl<G * 16 + 13>(a, s3[4]); wl<G * 16 + 13>(b, s3[5]); wl<G * 16 + 13>(c, s3[6]); wl<G * 16 + 13>(d, s3[7]);
    wl<G * 16 + 14>(a, s3[8]); wl<G * 16 + 14>(b, s3[9]); wl<G * 16 + 14>(c, s3[10]); wl<G * 16 + 14>(d, s3[11]);
    wl<G * 16 + 15>(a, s3[12]); wl<G * 16 + 15>(b, s3[13]); wl<G * 16 + 15>(c, s3[14]); wl<G * 16 + 15>(d, s3[15]);
}

template <int... CH>
__device__ inline void chunks(cu32x16p p, uint32_t &a, uint32_t &b, uint32_t &c, uint32_t &d,
                              std::integer_sequence<int, CH...>) {
    (chunk<CH>(p, a, b, c, d), ...);
}

template <int MODE>
__global__ __launch_bounds__(256) void k_sg(const uint4 *__restrict__ keys, uint64_t n,
                                            const uint32_t *__restrict__ tab, uint32_t mask,
                                            uint32_t *__restrict__ out) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t a = 0, b = 0, c = 0, d = 0;
    if constexpr (MODE == 0 || MODE == 2) {
        if (i < n) {
            typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
            const u32x4 v = __builtin_nontemporal_load((const u32x4 *)(keys + i));
            a = v.x; b = v.y; c = v.z; d = v.w;
        }
    } else if constexpr (MODE == 3 || MODE == 4 || MODE == 6 || MODE == 7) {
        // n is a multiple of 256 here (host checks): the wave's 64 keys are in bounds
        const uint64_t wbase = (uint64_t)blockIdx.x * blockDim.x +
                               (uint64_t)__builtin_amdgcn_readfirstlane(threadIdx.x & ~63u);
        const uint64_t addr = (uint64_t)(uintptr_t)(keys + wbase);
        const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)addr);
        const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(addr >> 32));
        cu32x16p p = (cu32x16p)(((uint64_t)hi << 32) | lo);
        if constexpr (MODE == 6 || MODE == 7) {
            chunk4<0>(p, a, b, c, d); chunk4<1>(p, a, b, c, d); chunk4<2>(p, a, b, c, d); chunk4<3>(p, a, b, c, d);
        } else {
            chunks(p, a, b, c, d, std::make_integer_sequence<int, 16>{});
        }
    } else {
        a = (uint32_t)i * 2654435761u; b = a ^ 0x9e3779b9u; c = a + 17; d = a ^ 0x85ebca6bu;
    }
    uint32_t acc = a ^ b ^ c ^ d;
    if constexpr (MODE == 1 || MODE == 2 || MODE == 3 || MODE == 6) {
        uint32_t x = mix(a ^ mix(b)), y = mix(c ^ mix(d)) | 1u;
        uint32_t live = 1u;
#pragma unroll
        for (int q = 0; q < 7; ++q) {
            const uint32_t w = (x >> 5) & mask;
            if (live) live &= tab[w] >> (x & 31);
            x += y;
        }
        acc = acc * 2u + live;
    }
    if (i < n) out[i] = acc;
}

typedef unsigned int u32x4v __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(256) void k_sg_pf(const uint4 *__restrict__ keys, uint64_t n,
                                               const uint32_t *__restrict__ tab, uint32_t mask,
                                               uint32_t *__restrict__ out) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    u32x4v v = __builtin_nontemporal_load((const u32x4v *)(keys + i));
    for (; i < n; i += stride) {
        const uint32_t a = v.x, b = v.y, c = v.z, d = v.w;
        if (i + stride < n) v = __builtin_nontemporal_load((const u32x4v *)(keys + i + stride));
        uint32_t acc = a ^ b ^ c ^ d;
        uint32_t x = mix(a ^ mix(b)), y = mix(c ^ mix(d)) | 1u;
        uint32_t live = 1u;
#pragma unroll
        for (int q = 0; q < 7; ++q) {
            const uint32_t w = (x >> 5) & mask;
            if (live) live &= tab[w] >> (x & 31);
            x += y;
        }
        out[i] = acc * 2u + live;
    }
}

__global__ void k_init(uint4 *k, uint64_t n) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) k[i] = make_uint4(mix((uint32_t)i), mix((uint32_t)i + 1u), mix((uint32_t)i ^ 0xabcdefu), mix((uint32_t)i * 3u));
}

int main() {
    const uint64_t n = 10000000ull - 10000000ull % 256;
    uint4 *keys;
    uint32_t *out, *tab;
    hipMalloc(&keys, n * 16);
    hipMalloc(&out, n * 4);
    const uint64_t tb = 4ull << 20;
    hipMalloc(&tab, tb);
    hipMemset(tab, 0xff, tb);  // every bit set: all 7 gathers run, as for a present key
    hipLaunchKernelGGL(k_init, dim3((n + 255) / 256), dim3(256), 0, 0, keys, n);
    hipDeviceSynchronize();
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    auto run = [&](auto kern, int mode) {
        float best = 1e30f;
        for (int rep = 0; rep < 5; ++rep) {
            hipEventRecord(e0);
            for (int it = 0; it < 10; ++it)
                hipLaunchKernelGGL(kern, dim3(n / 256), dim3(256), 0, 0, keys, n, tab, (uint32_t)(tb / 4 - 1), out);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            best = ms / 10 < best ? ms / 10 : best;
        }
        printf("{\"mode\": %d, \"us\": %.1f, \"stream_TB_s\": %.2f, \"Ggathers_s\": %.1f}\n", mode, best * 1e3,
               (mode == 1 ? 0.0 : 16.0 * n / (best * 1e-3) / 1e12),
               (mode == 0 || mode == 4) ? 0.0 : 7.0 * n / (best * 1e-3) / 1e9);
        fflush(stdout);
    };
    run(k_sg<0>, 0);
    run(k_sg<4>, 4);
    run(k_sg<1>, 1);
    run(k_sg<2>, 2);
    run(k_sg<3>, 3);
    run(k_sg<7>, 4);
    run(k_sg<6>, 3);
    for (uint32_t g : {2048u, 4096u, 8192u, 16384u}) {
        float best = 1e30f;
        for (int rep = 0; rep < 5; ++rep) {
            hipEventRecord(e0);
            for (int it = 0; it < 10; ++it)
                hipLaunchKernelGGL(k_sg_pf, dim3(g), dim3(256), 0, 0, keys, n, tab, (uint32_t)(tb / 4 - 1), out);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            best = ms / 10 < best ? ms / 10 : best;
        }
        printf("{\"mode\": 5, \"grid\": %u, \"us\": %.1f, \"Ggathers_s\": %.1f}\n", g, best * 1e3, 7.0 * n / (best * 1e-3) / 1e9);
    }
    // parity of modes 2 and 3 (same keys, same answers)
    uint32_t *o2 = new uint32_t[n], *o3 = new uint32_t[n];
    hipLaunchKernelGGL(k_sg<2>, dim3(n / 256), dim3(256), 0, 0, keys, n, tab, (uint32_t)(tb / 4 - 1), out);
    hipMemcpy(o2, out, n * 4, hipMemcpyDeviceToHost);
    hipLaunchKernelGGL(k_sg<3>, dim3(n / 256), dim3(256), 0, 0, keys, n, tab, (uint32_t)(tb / 4 - 1), out);
    hipMemcpy(o3, out, n * 4, hipMemcpyDeviceToHost);
    uint64_t diff = 0;
    for (uint64_t j = 0; j < n; ++j) diff += o2[j] != o3[j];
    printf("{\"mode2_vs_mode3_mismatches\": %llu}\n", (unsigned long long)diff);
    return 0;
}
