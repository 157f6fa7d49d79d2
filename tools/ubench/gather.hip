// gather.hip — ceiling of random 4-byte gathers on MI355X (what the bloom probe's 7 bit tests
// per key are made of).  Each thread does G independent loads at xorshift addresses in a table
// of T bytes; reports gathers/s.  Build: hipcc --offload-arch=gfx950 -O3 gather.hip -o gather
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

template <int G>
__global__ __launch_bounds__(256) void k_gather(const uint32_t *__restrict__ t, uint32_t mask_words, uint64_t n,
                                                uint32_t seed, uint32_t *__restrict__ out) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint32_t x = (uint32_t)i * 2654435761u ^ seed;
    uint32_t acc = 0;
    uint32_t a[G];
#pragma unroll
    for (int g = 0; g < G; ++g) {
        x ^= x << 13; x ^= x >> 17; x ^= x << 5;
        a[g] = x & mask_words;
    }
#pragma unroll
    for (int g = 0; g < G; ++g) acc ^= t[a[g]];
    out[i] = acc;
}

int main(int argc, char **argv) {
    const uint64_t n = 10000000;
    uint32_t *out, *tab;
    hipMalloc(&out, n * 4);
    hipMalloc(&tab, 512ull << 20);
    hipMemset(tab, 1, 512ull << 20);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (uint64_t tb : {1ull << 20, 2ull << 20, 4ull << 20, 8ull << 20, 16ull << 20, 64ull << 20, 256ull << 20, 512ull << 20}) {
        const uint32_t mask = (uint32_t)(tb / 4 - 1);
        for (int rep = 0; rep < 3; ++rep) {
            hipEventRecord(e0);
            for (int it = 0; it < 10; ++it)
                hipLaunchKernelGGL(k_gather<7>, dim3((n + 255) / 256), dim3(256), 0, 0, tab, mask, n, 1234u + it, out);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            if (rep == 2)
                printf("{\"table_bytes\": %llu, \"gathers_per_thread\": 7, \"ms_per_10M_threads\": %.4f, \"Ggathers_s\": %.2f}\n",
                       (unsigned long long)tb, ms / 10, 7.0 * n / (ms / 10 * 1e-3) / 1e9);
        }
    }
    return 0;
}
