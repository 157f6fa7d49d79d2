// cumask.hip — is the L2-resident gather ceiling (~270 G/s, gather.hip) set per CU (vector L1 /
// address path) or per XCD L2?  Runs the 7-gather kernel of gather.hip on streams restricted to a
// subset of the CUs (hipExtStreamCreateWithCUMask), a VALU-bound kernel (an FNV-style u64 chain)
// likewise, and the two together on complementary CU sets.  If gathers keep their rate on half of
// the CUs, a gather-bound phase can share the chip with a VALU-bound kernel.
// Build: hipcc --offload-arch=gfx950 -O3 cumask.hip -o cumask
// Run: cumask TABLE_BYTES CONFIG  — one mask configuration per process (at most two CU-masked
// streams: each takes a hardware queue of its own, and the box has GPU_MAX_HW_QUEUES = 4; in one
// process creating the 4th-6th masked stream stalled until the time limit, round 2).  Driven by
// tools/ubench/run_cumask.py, a parent that never touches the GPU.  Every HIP call is checked.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

constexpr int VSTEPS = 256;

__global__ __launch_bounds__(256) void k_gather7(const uint32_t *__restrict__ t, uint32_t mask_words, uint64_t n,
                                                 uint32_t seed, uint32_t *__restrict__ out) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint32_t x = (uint32_t)i * 2654435761u ^ seed;
    uint32_t acc = 0, a[7];
#pragma unroll
    for (int g = 0; g < 7; ++g) {
        x ^= x << 13; x ^= x >> 17; x ^= x << 5;
        a[g] = x & mask_words;
    }
#pragma unroll
    for (int g = 0; g < 7; ++g) acc ^= t[a[g]];
    out[i] = acc;
}

// VALU-bound: VSTEPS steps of both FNV chains over a lane-private value (no memory beyond one store).
__global__ __launch_bounds__(256) void k_valu(uint64_t n, uint32_t seed, uint64_t *__restrict__ out) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint64_t h1 = 0xcbf29ce484222325ull ^ i, h2 = h1 + seed;
    uint32_t b = (uint32_t)i;
#pragma unroll 4
    for (int s = 0; s < VSTEPS; ++s) {
        h1 = (h1 ^ (b & 0xff)) * 0x100000001b3ull;
        h2 = (h2 * 0x100000001b3ull) ^ ((b >> 8) & 0xff);
        b = b * 1664525u + 1013904223u;
    }
    out[i] = h1 ^ h2;
}

#define CHECK(expr)                                                                          \
    do {                                                                                     \
        hipError_t e_ = (expr);                                                              \
        if (e_ != hipSuccess) {                                                              \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #expr, hipGetErrorString(e_)); \
            exit(3);                                                                         \
        }                                                                                    \
    } while (0)

static hipStream_t make_stream(const std::vector<uint32_t> &mask) {
    hipStream_t s;
    CHECK(hipExtStreamCreateWithCUMask(&s, (uint32_t)mask.size(), mask.data()));
    return s;
}

int main(int argc, char **argv) {
    if (argc != 3) {
        fprintf(stderr, "usage: %s TABLE_BYTES CONFIG(0-4)\n", argv[0]);
        return 2;
    }
    const uint32_t tb = (uint32_t)strtoul(argv[1], 0, 0);
    const int cfg = atoi(argv[2]);
    if (tb < 4096 || tb > (16u << 20) || (tb & (tb - 1)) || cfg < 0 || cfg > 4) {
        fprintf(stderr, "table bytes must be a power of two in [4K, 16M], config 0-4\n");
        return 2;
    }
    int ncu = 0;
    CHECK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
    const uint32_t words = (uint32_t)((ncu + 31) / 32);
    const uint64_t n = 10000000;
    uint32_t *out, *tab;
    uint64_t *vout;
    CHECK(hipMalloc(&out, n * 4));
    CHECK(hipMalloc(&vout, n * 8));
    CHECK(hipMalloc(&tab, 16ull << 20));
    CHECK(hipMemset(tab, 1, 16ull << 20));
    hipEvent_t e0, e1, da, db;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    CHECK(hipEventCreate(&da));
    CHECK(hipEventCreate(&db));

    auto mk = [&](auto pred) {
        std::vector<uint32_t> m(words, 0u);
        for (int c = 0; c < ncu; ++c)
            if (pred(c)) m[c / 32] |= 1u << (c % 32);
        return m;
    };
    struct M { const char *name; std::vector<uint32_t> a, b; };
    // Every mask keeps CUs in every XCD whether CU c sits in XCD c / 32 or c % 8: a mask that
    // leaves an XCD without CUs can stall the round-robin workgroup dispatch.
    std::vector<M> masks = {
        {"all", mk([](int) { return true; }), {}},
        {"even/odd", mk([](int c) { return c % 2 == 0; }), mk([](int c) { return c % 2 == 1; })},
        {"half/half (c%32<16)", mk([](int c) { return c % 32 < 16; }), mk([](int c) { return c % 32 >= 16; })},
        {"quarter/rest (c%32<8)", mk([](int c) { return c % 32 < 8; }), mk([](int c) { return c % 32 >= 8; })},
        {"rest/quarter (c%32>=8)", mk([](int c) { return c % 32 >= 8; }), mk([](int c) { return c % 32 < 8; })},
    };
    const uint64_t gn = n, vn = n;
    auto time_it = [&](hipStream_t sa, hipStream_t sb, bool g, bool v, uint32_t tmask) {
        float best = 1e30f;
        for (int rep = 0; rep < 5; ++rep) {
            CHECK(hipDeviceSynchronize());
            CHECK(hipEventRecord(e0, 0));
            CHECK(hipStreamWaitEvent(sa, e0, 0));
            CHECK(hipStreamWaitEvent(sb, e0, 0));
            for (int it = 0; it < 5; ++it) {
                if (g) hipLaunchKernelGGL(k_gather7, dim3((gn + 255) / 256), dim3(256), 0, sa, tab, tmask, gn, 77u + it, out);
                if (v) hipLaunchKernelGGL(k_valu, dim3((vn + 255) / 256), dim3(256), 0, sb, vn, 5u + it, vout);
                CHECK(hipGetLastError());
            }
            CHECK(hipEventRecord(da, sa));
            CHECK(hipEventRecord(db, sb));
            CHECK(hipStreamWaitEvent(0, da, 0));
            CHECK(hipStreamWaitEvent(0, db, 0));
            CHECK(hipEventRecord(e1, 0));
            CHECK(hipEventSynchronize(e1));
            float ms;
            CHECK(hipEventElapsedTime(&ms, e0, e1));
            if (ms / 5 < best) best = ms / 5;
        }
        return best;
    };
    const uint32_t tmask = tb / 4 - 1;
    const M &mm = masks[cfg];
    hipStream_t sa = make_stream(mm.a);
    hipStream_t sb = mm.b.empty() ? sa : make_stream(mm.b);
    const float g_a = time_it(sa, sa, true, false, tmask);
    const float v_b = time_it(sb, sb, false, true, tmask);
    const float both = time_it(sa, sb, true, true, tmask);
    const float g_b = mm.b.empty() ? g_a : time_it(sb, sb, true, false, tmask);
    printf("{\"table_bytes\": %u, \"masks\": \"%s\", \"gather_on_a_ms\": %.4f, \"Ggathers_s_a\": %.1f, "
           "\"gather_on_b_ms\": %.4f, \"valu_on_b_ms\": %.4f, \"both_concurrent_ms\": %.4f, "
           "\"sum_ms\": %.4f}\n",
           tb, mm.name, g_a, 7.0 * gn / (g_a * 1e-3) / 1e9, g_b, v_b, both, g_a + v_b);
    fflush(stdout);
    CHECK(hipDeviceSynchronize());
    CHECK(hipStreamDestroy(sa));
    if (sb != sa) CHECK(hipStreamDestroy(sb));
    return 0;
}
