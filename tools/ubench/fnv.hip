// fnv.hip — cost of the two FNV-64 chains (lsm/bloom.go:44-54) on gfx950, per formulation.
// Each thread hashes one 16-B key (dwordx4 load) and writes (h1, h2); a copy kernel gives the
// memory floor.  Variants:
//   0  plain C: (h ^ b) * P  /  (h * P) ^ b   (compiler: v_mad_u64_u32 + v_mul_lo_u32 + v_add3)
//   1  P = 2^40 + 435, 435 = (3*9)*16 + 3: three v_lshl_add_u64 + one v_lshl_add_u32 per step
//   2  lo/hi split with v_mul_hi_u32 / v_mul_lo_u32 (three 32-bit multiplies per step)
//   3  16-B keys only: the low word runs the chain alone (lo' = low32((lo ^ b) * 435)), and the
//      high word, linear in the per-step terms d_j = carry_j + (x_j << 8), is summed with
//      constant weights 435^(15-j) mod 2^32 off the critical path (one v_mad_u64_u32 each)
// Build: hipcc --offload-arch=gfx950 -O3 fnv.hip -o fnv
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

constexpr uint64_t kOff = 0xcbf29ce484222325ull, kP = 0x100000001b3ull;

template <int S>
__device__ __forceinline__ uint64_t lsa(uint64_t x, uint64_t y) {
    uint64_t r;
    asm volatile("v_lshl_add_u64 %0, %1, %2, %3" : "=v"(r) : "v"(x), "n"(S), "v"(y));
    return r;
}

__device__ __forceinline__ uint64_t mulP_sa(uint64_t h) {
    const uint64_t a = lsa<1>(h, h);   // 3h
    const uint64_t b = lsa<3>(a, a);   // 27h
    const uint64_t c = lsa<4>(b, a);   // 435h
    return c + ((uint64_t)(uint32_t)h << 40);
}

__device__ __forceinline__ uint64_t mulP_split(uint64_t h) {
    const uint32_t lo = (uint32_t)h, hi = (uint32_t)(h >> 32);
    const uint32_t nlo = lo * 435u;
    const uint32_t nhi = __umulhi(lo, 435u) + hi * 435u + (lo << 8);
    return ((uint64_t)nhi << 32) | nlo;
}

template <int V>
__device__ __forceinline__ void step(uint32_t b, uint64_t &h1, uint64_t &h2) {
    if constexpr (V == 0) {
        h1 = (h1 ^ b) * kP;
        h2 = (h2 * kP) ^ b;
    } else if constexpr (V == 1) {
        h1 = mulP_sa(h1 ^ b);
        h2 = mulP_sa(h2) ^ b;
    } else {
        h1 = mulP_split(h1 ^ b);
        h2 = mulP_split(h2) ^ b;
    }
}

// 435^e mod 2^32
__host__ __device__ constexpr uint32_t pw435(int e) {
    uint32_t r = 1;
    for (int i = 0; i < e; ++i) r *= 435u;
    return r;
}

// acc + a * b as one v_mad_u64_u32 (the compiler narrows a mad whose high half is unused into
// v_mul_lo_u32 + v_add3_u32, two instructions)
__device__ __forceinline__ uint64_t mad64(uint32_t a, uint32_t b, uint64_t acc) {
    uint64_t r;
    asm("v_mad_u64_u32 %0, vcc, %1, %2, %3" : "=v"(r) : "v"(a), "s"(b), "v"(acc) : "vcc");
    return r;
}

__device__ __forceinline__ void fnv16_v3(const uint32_t w[4], uint64_t &h1, uint64_t &h2) {
    uint32_t lo1 = (uint32_t)kOff, lo2 = (uint32_t)kOff;
    uint64_t acc1 = (uint64_t)((uint32_t)(kOff >> 32) * pw435(16)), acc2 = acc1;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        const uint32_t b = (w[j >> 2] >> (8 * (j & 3))) & 0xffu;
        const uint32_t cj = pw435(15 - j);
        const uint32_t x = lo1 ^ b;  // FNV-1a: xor, then multiply
        const uint64_t p = (uint64_t)x * 435u;
        lo1 = (uint32_t)p;
        acc1 = mad64((uint32_t)(p >> 32) + (x << 8), cj, acc1);
        const uint64_t q = (uint64_t)lo2 * 435u;  // FNV-1: multiply, then xor
        acc2 = mad64((uint32_t)(q >> 32) + (lo2 << 8), cj, acc2);
        lo2 = (uint32_t)q ^ b;
    }
    h1 = (acc1 << 32) | lo1;
    h2 = (acc2 << 32) | lo2;
}

// R > 1: hash R variants of the key (first word xor r) and xor the results: compute-bound form.
template <int V, int R = 1>
__global__ __launch_bounds__(256) void k_hash(const uint4 *__restrict__ keys, uint64_t n, uint4 *__restrict__ out) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint4 v = keys[i];
    uint64_t a1 = 0, a2 = 0;
    for (int r = 0; r < R; ++r) {
        uint64_t h1 = kOff, h2 = kOff;
        const uint32_t w[4] = {v.x ^ (uint32_t)r, v.y, v.z, v.w};
        if constexpr (V == 3) {
            fnv16_v3(w, h1, h2);
        } else {
#pragma unroll
            for (int j = 0; j < 4; ++j)
#pragma unroll
                for (int s = 0; s < 4; ++s) step<V>((w[j] >> (8 * s)) & 0xffu, h1, h2);
        }
        a1 ^= h1;
        a2 ^= h2;
    }
    out[i] = make_uint4((uint32_t)a1, (uint32_t)(a1 >> 32), (uint32_t)a2, (uint32_t)(a2 >> 32));
}

__global__ __launch_bounds__(256) void k_copy(const uint4 *__restrict__ keys, uint64_t n, uint4 *__restrict__ out) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = keys[i];
}

// Throughput of a single instruction kind: each thread runs a dependent-free mix of 8 chains.
template <int OP>
__global__ __launch_bounds__(256) void k_inst(uint64_t seed, uint64_t *out, int iters) {
    uint64_t x[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) x[c] = seed + threadIdx.x * 8 + c;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int c = 0; c < 8; ++c) {
            if constexpr (OP == 0) {  // v_mad_u64_u32
                uint64_t r;
                asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %3" : "=v"(r) : "v"((uint32_t)x[c]), "v"(435u), "v"(x[c]) : "vcc");
                x[c] = r;
            } else if constexpr (OP == 1) {  // v_mul_lo_u32
                uint32_t r;
                asm volatile("v_mul_lo_u32 %0, %1, %2" : "=v"(r) : "v"((uint32_t)x[c]), "v"((uint32_t)(x[c] >> 32)));
                x[c] = r | (x[c] & 0xffffffff00000000ull);
            } else if constexpr (OP == 2) {  // v_lshl_add_u64
                x[c] = lsa<3>(x[c], x[c]);
            } else if constexpr (OP == 3) {  // v_add_u32 (reference full-rate op)
                uint32_t r;
                asm volatile("v_add_u32 %0, %1, %2" : "=v"(r) : "v"((uint32_t)x[c]), "v"((uint32_t)(x[c] >> 32)));
                x[c] = r | (x[c] & 0xffffffff00000000ull);
            } else if constexpr (OP == 4) {  // v_mul_hi_u32
                uint32_t r;
                asm volatile("v_mul_hi_u32 %0, %1, %2" : "=v"(r) : "v"((uint32_t)x[c]), "v"((uint32_t)(x[c] >> 32)));
                x[c] = r | (x[c] & 0xffffffff00000000ull);
            }
        }
    }
    uint64_t acc = 0;
#pragma unroll
    for (int c = 0; c < 8; ++c) acc ^= x[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

int main() {
    const uint64_t n = 10000000;
    std::vector<uint4> hk(n);
    for (uint64_t i = 0; i < n; ++i) {
        char s[17];
        snprintf(s, sizeof s, "user%010llu", (unsigned long long)i);
        uint8_t b[16];
        for (int j = 0; j < 14; ++j) b[j] = (uint8_t)s[j];
        b[14] = (uint8_t)(i & 0xff);
        b[15] = (uint8_t)((i + 1) & 0xff);
        hk[i] = *(uint4 *)b;
    }
    uint4 *keys, *out;
    hipMalloc(&keys, n * 16);
    hipMalloc(&out, n * 16);
    hipMemcpy(keys, hk.data(), n * 16, hipMemcpyHostToDevice);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    std::vector<uint4> ref(n), got(n);
    auto timeit = [&](auto launch) {
        float best = 1e30f;
        for (int rep = 0; rep < 5; ++rep) {
            hipEventRecord(e0);
            for (int it = 0; it < 10; ++it) launch();
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            best = ms / 10 < best ? ms / 10 : best;
        }
        return best;
    };
    const dim3 g((n + 255) / 256), b(256);
    float tc = timeit([&] { hipLaunchKernelGGL(k_copy, g, b, 0, 0, keys, n, out); });
    printf("{\"kernel\": \"copy\", \"ms\": %.4f}\n", tc);
    float t0 = timeit([&] { hipLaunchKernelGGL(k_hash<0>, g, b, 0, 0, keys, n, out); });
    hipMemcpy(ref.data(), out, n * 16, hipMemcpyDeviceToHost);
    printf("{\"kernel\": \"fnv_v0_plain\", \"ms\": %.4f}\n", t0);
    float t1 = timeit([&] { hipLaunchKernelGGL(k_hash<1>, g, b, 0, 0, keys, n, out); });
    hipMemcpy(got.data(), out, n * 16, hipMemcpyDeviceToHost);
    printf("{\"kernel\": \"fnv_v1_shiftadd\", \"ms\": %.4f, \"equal\": %d}\n", t1,
           (int)(memcmp(ref.data(), got.data(), n * 16) == 0));
    float t2 = timeit([&] { hipLaunchKernelGGL(k_hash<2>, g, b, 0, 0, keys, n, out); });
    hipMemcpy(got.data(), out, n * 16, hipMemcpyDeviceToHost);
    printf("{\"kernel\": \"fnv_v2_split\", \"ms\": %.4f, \"equal\": %d}\n", t2,
           (int)(memcmp(ref.data(), got.data(), n * 16) == 0));
    float t3 = timeit([&] { hipLaunchKernelGGL(k_hash<3>, g, b, 0, 0, keys, n, out); });
    hipMemcpy(got.data(), out, n * 16, hipMemcpyDeviceToHost);
    printf("{\"kernel\": \"fnv_v3_lochain\", \"ms\": %.4f, \"equal\": %d}\n", t3,
           (int)(memcmp(ref.data(), got.data(), n * 16) == 0));
    for (int v = 0; v < 4; ++v) {
        float t = timeit([&] {
            if (v == 0) hipLaunchKernelGGL((k_hash<0, 16>), g, b, 0, 0, keys, n, out);
            if (v == 1) hipLaunchKernelGGL((k_hash<1, 16>), g, b, 0, 0, keys, n, out);
            if (v == 2) hipLaunchKernelGGL((k_hash<2, 16>), g, b, 0, 0, keys, n, out);
            if (v == 3) hipLaunchKernelGGL((k_hash<3, 16>), g, b, 0, 0, keys, n, out);
        });
        hipMemcpy(got.data(), out, n * 16, hipMemcpyDeviceToHost);
        if (v == 0) ref = got;
        printf("{\"kernel\": \"fnv_v%d_x16\", \"ms_per_10M_keys\": %.4f, \"equal\": %d}\n", v, t / 16,
               (int)(memcmp(ref.data(), got.data(), n * 16) == 0));
    }
    uint64_t *o64;
    hipMalloc(&o64, (1 << 20) * 8);
    const int iters = 256;
    const char *names[] = {"v_mad_u64_u32", "v_mul_lo_u32", "v_lshl_add_u64", "v_add_u32", "v_mul_hi_u32"};
    for (int op = 0; op < 5; ++op) {
        auto L = [&] {
            switch (op) {
            case 0: hipLaunchKernelGGL(k_inst<0>, dim3(4096), dim3(256), 0, 0, 1ull, o64, iters); break;
            case 1: hipLaunchKernelGGL(k_inst<1>, dim3(4096), dim3(256), 0, 0, 1ull, o64, iters); break;
            case 2: hipLaunchKernelGGL(k_inst<2>, dim3(4096), dim3(256), 0, 0, 1ull, o64, iters); break;
            case 3: hipLaunchKernelGGL(k_inst<3>, dim3(4096), dim3(256), 0, 0, 1ull, o64, iters); break;
            case 4: hipLaunchKernelGGL(k_inst<4>, dim3(4096), dim3(256), 0, 0, 1ull, o64, iters); break;
            }
        };
        float t = timeit(L);
        const double winst = 4096.0 * 4 * iters * 8;  // wave-instructions
        printf("{\"inst\": \"%s\", \"ms\": %.4f, \"Gwave_inst_s\": %.1f}\n", names[op], t, winst / (t * 1e-3) / 1e9);
    }
    return 0;
}
