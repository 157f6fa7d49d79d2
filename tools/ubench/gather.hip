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

// Partial exec masks: each of the G gathers of a lane is issued with probability 1/DEN (an
// xorshift draw), as in the sliced/phased probes where a gather instruction only has the lanes
// whose position falls in the current range.  Reports issued lane-gathers per second.
template <int G, int DEN>
__global__ __launch_bounds__(256) void k_gather_sparse(const uint32_t *__restrict__ t, uint32_t mask_words, uint64_t n,
                                                       uint32_t seed, uint32_t *__restrict__ out,
                                                       unsigned long long *__restrict__ issued) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint32_t x = (uint32_t)i * 2654435761u ^ seed;
    uint32_t acc = 0, cnt = 0;
#pragma unroll
    for (int g = 0; g < G; ++g) {
        x ^= x << 13; x ^= x >> 17; x ^= x << 5;
        if ((x >> 24) % DEN == 0) {
            acc ^= t[x & mask_words];
            ++cnt;
        }
    }
    out[i] = acc;
    if (i == 0 && issued) *issued = 0;
    (void)cnt;
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
    // partial masks on a 4 MiB table (one XCD's L2), 28 gather slots per thread
    {
        const uint32_t mask = (uint32_t)((4ull << 20) / 4 - 1);
        auto run = [&](auto kern, int den) {
            float best = 1e30f;
            for (int rep = 0; rep < 3; ++rep) {
                hipEventRecord(e0);
                for (int it = 0; it < 10; ++it)
                    hipLaunchKernelGGL(kern, dim3((n + 255) / 256), dim3(256), 0, 0, tab, mask, n, 99u + it, out,
                                       (unsigned long long *)nullptr);
                hipEventRecord(e1);
                hipEventSynchronize(e1);
                float ms;
                hipEventElapsedTime(&ms, e0, e1);
                best = ms / 10 < best ? ms / 10 : best;
            }
            const double lanes = 28.0 * n / den;  // expected issued lane-gathers
            printf("{\"table_bytes\": 4194304, \"slots_per_thread\": 28, \"active_fraction\": %.3f, \"ms\": %.4f, "
                   "\"Glane_gathers_s\": %.2f, \"Gwave_instr_s\": %.3f}\n",
                   1.0 / den, best, lanes / (best * 1e-3) / 1e9, 28.0 * n / 64 / (best * 1e-3) / 1e9);
        };
        run(k_gather_sparse<28, 1>, 1);
        run(k_gather_sparse<28, 2>, 2);
        run(k_gather_sparse<28, 4>, 4);
        run(k_gather_sparse<28, 8>, 8);
    }
    return 0;
}
