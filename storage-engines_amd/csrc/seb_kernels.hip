// seb_kernels.hip — CDNA4 (gfx950) kernels of the bloom build + probe path.
//
// Reference semantics (intellect4all/storage-engines, Go):
//   hash1 = FNV-1a 64, hash2 = FNV-1 64 over the key bytes      lsm/bloom.go:44-54
//   pos_i = (h1 + i*h2) mod 2^64, then mod m, i < k               lsm/bloom.go:58-67
//   Add: bits[pos>>3] |= 1<<(pos&7)                                lsm/bloom.go:70-77
//   MayContain: AND over the k bits                                lsm/bloom.go:82-92
// On the little-endian device byte pos>>3 / bit pos&7 is u32 word pos>>5 / bit pos&31, so the
// filter lives in HBM as u32 words (16-B padded, pad = 0) and its first ceil(m/8) bytes ARE the
// reference's bit array.
//
// Integer-only work; no MFMA.  Per key: two FNV chains over the key bytes (VALU), two exact
// 64-bit Barrett reductions, then k-1 incremental residue steps (u32 when m < 2^31), then k
// random word touches (atomic OR for build, gather for probe).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include <type_traits>

#include "seb_device.h"
#include "seb_kernels.h"

namespace seb {

// ------------------------------------------------------------------ kernels -----------------

// Build: one thread per key (grid-stride), k device-scope atomic ORs into the word array.
template <typename Src, int KFIX, bool M32>
__global__ __launch_bounds__(256) void k_build(Src src, uint64_t n, uint32_t *__restrict__ words, ModArg md) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        uint64_t h1, h2;
        src.hash(i, h1, h2);
        for_positions<KFIX, M32>(h1, h2, md, md.k, [&](uint32_t, uint64_t p) {
            __hip_atomic_fetch_or(words + (p >> 5), 1u << (uint32_t)(p & 31), __ATOMIC_RELAXED,
                                  __HIP_MEMORY_SCOPE_AGENT);
        });
    }
}

// Probe: the answer is the AND of the k bits, as the reference's early-exit loop returns
// (lsm/bloom.go:82-92); 0/1 byte out.  The k == 7 kernel is built for memory-level parallelism:
// each thread owns KPT keys, computes all 7 positions of each, gathers the first SPLIT words of
// every key, and gathers the remaining ones only for keys whose bits so far are all set (a key
// with a clear bit is already "absent": fewer fabric reads, the same answer).
template <typename Src, int KFIX, bool M32, int SPLIT, int KPT>
__global__ __launch_bounds__(256) void k_probe(Src src, uint64_t n, const uint32_t *__restrict__ words, ModArg md,
                                               uint8_t *__restrict__ out) {
    if constexpr (KFIX > 0) {
        using P = typename std::conditional<M32, uint32_t, uint64_t>::type;
        constexpr int S = (SPLIT > 0 && SPLIT < KFIX) ? SPLIT : KFIX;
        const uint64_t span = (uint64_t)blockDim.x * KPT;
        for (uint64_t base = (uint64_t)blockIdx.x * span; base < n; base += (uint64_t)gridDim.x * span) {
            P pos[KPT][KFIX];
            uint32_t acc[KPT];
#pragma unroll
            for (int r = 0; r < KPT; ++r) {
                const uint64_t i = base + (uint64_t)r * blockDim.x + threadIdx.x;
                uint64_t h1 = 0, h2 = 0;
                if (i < n) src.hash(i, h1, h2);
                for_positions<KFIX, M32>(h1, h2, md, KFIX, [&](uint32_t q, uint64_t p) { pos[r][q] = (P)p; });
                acc[r] = i < n ? 1u : 0u;
            }
#pragma unroll
            for (int r = 0; r < KPT; ++r)
#pragma unroll
                for (int q = 0; q < S; ++q)
                    if (acc[r]) acc[r] &= words[pos[r][q] >> 5] >> (uint32_t)(pos[r][q] & 31);
            if constexpr (S < KFIX) {
#pragma unroll
                for (int r = 0; r < KPT; ++r)
                    if (acc[r] & 1u) {
#pragma unroll
                        for (int q = S; q < KFIX; ++q) acc[r] &= words[pos[r][q] >> 5] >> (uint32_t)(pos[r][q] & 31);
                    }
            }
#pragma unroll
            for (int r = 0; r < KPT; ++r) {
                const uint64_t i = base + (uint64_t)r * blockDim.x + threadIdx.x;
                if (i < n) out[src.index(i)] = (uint8_t)(acc[r] & 1u);
            }
        }
    } else {
        const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
        for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
            uint64_t h1, h2;
            src.hash(i, h1, h2);
            uint32_t acc = 1u;
            for_positions<0, M32>(h1, h2, md, md.k, [&](uint32_t, uint64_t p) {
                if (acc & 1u) acc &= words[p >> 5] >> (uint32_t)(p & 31);  // MayContain's early exit
            });
            out[src.index(i)] = (uint8_t)(acc & 1u);
        }
    }
}

// Sliced probe (k == 7, 2^29 <= m < 2^31, filters too large for packed residues): a filter
// larger than one XCD's 4 MiB L2 is probed in phases.  Each thread keeps the 7 positions of its
// KPT keys in registers and, in phase s, gathers only the words of slice s (2^slice_shift words),
// skipping the rest of a key once a clear bit is seen.  Workgroups that progress at the same pace
// on one XCD then share a single slice in that XCD's L2 instead of thrashing the whole filter.
// Which slice a gather belongs to changes only when it is issued, never the answer.  (Variants
// that put more gathers in flight per wave were measured slower)
template <typename Src, int KPT>
__global__ __launch_bounds__(256) void k_probe_sliced(Src src, uint64_t n, const uint32_t *__restrict__ words,
                                                      ModArg md, uint8_t *__restrict__ out, uint32_t slice_shift,
                                                      uint32_t nslices) {
    const uint64_t span = (uint64_t)blockDim.x * KPT;
    for (uint64_t base = (uint64_t)blockIdx.x * span; base < n; base += (uint64_t)gridDim.x * span) {
        uint32_t pos[KPT][7];
        uint32_t acc[KPT];
#pragma unroll
        for (int r = 0; r < KPT; ++r) {
            const uint64_t i = base + (uint64_t)r * blockDim.x + threadIdx.x;
            uint64_t h1 = 0, h2 = 0;
            if (i < n) src.hash(i, h1, h2);
            for_positions<7, true>(h1, h2, md, 7, [&](uint32_t q, uint64_t p) { pos[r][q] = (uint32_t)p; });
            acc[r] = i < n ? 1u : 0u;
        }
        for (uint32_t sl = 0; sl < nslices; ++sl) {
#pragma unroll
            for (int r = 0; r < KPT; ++r)
#pragma unroll
                for (int q = 0; q < 7; ++q) {
                    const uint32_t w = pos[r][q] >> 5;
                    if ((acc[r] & 1u) && (w >> slice_shift) == sl) acc[r] &= words[w] >> (pos[r][q] & 31);
                }
        }
#pragma unroll
        for (int r = 0; r < KPT; ++r) {
            const uint64_t i = base + (uint64_t)r * blockDim.x + threadIdx.x;
            if (i < n) out[src.index(i)] = (uint8_t)(acc[r] & 1u);
        }
    }
}

// ---- packed residues: a probe batch shared by several filters of one size (the filters of one
// SSTable size on different GPUs, compaction outputs) is hashed once into 8 bytes per key and the
// packed words travel instead of the keys (half the bytes of a 16-B key over xGMI).  Layout
// (kPackBits = 29, so m < 2^29): bits 0-28 r0 = h1 mod m, 29-57 b = h2 mod m, 58-63 bit q-1 =
// "the u64 sum h1 + q*h2 wrapped at step q" for q = 1..6.  Positions follow for_positions'
// recurrence, so they are exactly (h1 + q*h2 mod 2^64) mod m of lsm/bloom.go:64.
template <typename Src>
__global__ __launch_bounds__(256) void k_pack_residues(Src src, uint64_t n, ModArg md, uint64_t *__restrict__ out) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        uint64_t h1, h2;
        src.hash(i, h1, h2);
        out[src.index(i)] = pack_residue(h1, h2, md);
    }
}

// The narrow 6-byte form (m < 2^kPack6Bits): 64-key blocks, one u32 and one u16 store per lane,
// each wave writing one block's two rows whole.
template <typename Src>
__global__ __launch_bounds__(256) void k_pack_residues6(Src src, uint64_t n, ModArg md, uint8_t *__restrict__ out) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        uint64_t h1, h2;
        src.hash(i, h1, h2);
        store_packed6(out, i, pack_residue6(h1, h2, md));
    }
}

// Sliced probe from keys that also writes each key's packed residues: the root of a
// multi-GPU probe answers a batch for its own filter and produces the broadcast form in one pass.
template <typename Src, int KPT>
__global__ __launch_bounds__(256) void k_probe_sliced_emit(Src src, uint64_t n, const uint32_t *__restrict__ words,
                                                           ModArg md, uint8_t *__restrict__ out,
                                                           uint64_t *__restrict__ packed, uint32_t slice_shift,
                                                           uint32_t nslices) {
    const uint64_t span = (uint64_t)blockDim.x * KPT;
    for (uint64_t base = (uint64_t)blockIdx.x * span; base < n; base += (uint64_t)gridDim.x * span) {
        uint32_t pos[KPT][7];
        uint32_t acc[KPT];
#pragma unroll
        for (int r = 0; r < KPT; ++r) {
            const uint64_t i = base + (uint64_t)r * blockDim.x + threadIdx.x;
            uint64_t h1 = 0, h2 = 0;
            if (i < n) src.hash(i, h1, h2);
            const uint64_t pw = pack_residue(h1, h2, md);  // each residue and wrap flag once
            packed_positions(pw, (uint32_t)md.m, (uint32_t)md.c, pos[r]);
            acc[r] = i < n ? 1u : 0u;
            if (i < n) __builtin_nontemporal_store(pw, packed + src.index(i));
        }
        for (uint32_t sl = 0; sl < nslices; ++sl) {
#pragma unroll
            for (int r = 0; r < KPT; ++r)
#pragma unroll
                for (int q = 0; q < 7; ++q) {
                    const uint32_t w = pos[r][q] >> 5;
                    if ((acc[r] & 1u) && (w >> slice_shift) == sl) acc[r] &= words[w] >> (pos[r][q] & 31);
                }
        }
#pragma unroll
        for (int r = 0; r < KPT; ++r) {
            const uint64_t i = base + (uint64_t)r * blockDim.x + threadIdx.x;
            if (i < n) out[src.index(i)] = (uint8_t)(acc[r] & 1u);
        }
    }
}

// ---- phased probe (k == 7, m < 2^29; the default).  The sliced probe's cost is its L2 misses: its
// workgroups are only loosely aligned in their sweep over the slices, so each XCD refills its L2
// with the 12 MB filter ~2.3 times per workgroup generation (profiles/r01z).  Here every phase (a
// contiguous word range of the filter, about one L2's worth) is its own launch, so all waves of
// the chip gather from one range at a time and each XCD fetches it into its L2 about once.
// Phase 0 hashes the keys, writes their packed residues (k_pack_residues' layout) and tests the
// positions in range 0; phase p > 0 reads the answer bytes and, for keys still alive,
// regenerates the positions from the packed words and tests those in range p, each gather only
// while the key's bits so far are all set (the sliced probe's early exit; sampling liveness once per phase
// so a key's gathers overlap was measured slower: more gathers).  The answer is the AND of the k
// bits, as MayContain (lsm/bloom.go:82-92) returns.
constexpr unsigned kPhaseBlock = 256;  // 512 measured the same
template <typename Src, int KPT>
__global__ __launch_bounds__(kPhaseBlock) void k_probe_phase0(Src src, uint64_t n, const uint32_t *__restrict__ words,
                                                      ModArg md, uint8_t *__restrict__ out,
                                                      uint64_t *__restrict__ packed, uint32_t hi) {
    const uint64_t span = (uint64_t)blockDim.x * KPT;
    for (uint64_t base = (uint64_t)blockIdx.x * span; base < n; base += (uint64_t)gridDim.x * span) {
        uint32_t pos[KPT][7];
        uint32_t acc[KPT];
#pragma unroll
        for (int r = 0; r < KPT; ++r) {
            const uint64_t i = base + (uint64_t)r * blockDim.x + threadIdx.x;
            uint64_t h1 = 0, h2 = 0;
            if (i < n) src.hash(i, h1, h2);
            const uint64_t pw = pack_residue(h1, h2, md);  // each residue and wrap flag once
            packed_positions(pw, (uint32_t)md.m, (uint32_t)md.c, pos[r]);
            acc[r] = i < n ? 1u : 0u;
            if (i < n) __builtin_nontemporal_store(pw, packed + i);
        }
#pragma unroll
        for (int r = 0; r < KPT; ++r)
#pragma unroll
            for (int q = 0; q < 7; ++q) {
                const uint32_t w = pos[r][q] >> 5;
                if ((acc[r] & 1u) && w < hi) acc[r] &= words[w] >> (pos[r][q] & 31);
            }
#pragma unroll
        for (int r = 0; r < KPT; ++r) {
            const uint64_t i = base + (uint64_t)r * blockDim.x + threadIdx.x;
            if (i < n) out[i] = (uint8_t)(acc[r] & 1u);
        }
    }
}

// Phase p > 0 over words [lo, hi): thread t owns keys 4t..4t+3 (one u32 of answers, two 16-B
// loads of packed words); `out` is 4-byte aligned (the host checks).
__global__ __launch_bounds__(kPhaseBlock) void k_probe_phase(const uint64_t *__restrict__ packed, uint64_t n,
                                                     const uint32_t *__restrict__ words, ModArg md,
                                                     uint8_t *__restrict__ out, uint32_t lo, uint32_t hi,
                                                     uint32_t first) {
    const uint32_t m = (uint32_t)md.m, c = (uint32_t)md.c;
    constexpr uint64_t kMask = (1ull << kPackBits) - 1;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x * 4;
    for (uint64_t i0 = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4; i0 < n; i0 += stride) {
        const bool full = i0 + 4 <= n;
        uint32_t a;
        if (first) {  // a batch probed from packed words alone: every key starts alive
            a = full ? 0x01010101u : 0x01010101u & ((1u << (8 * (uint32_t)(n - i0))) - 1u);
        } else if (full) {
            a = *(const uint32_t *)(out + i0);
        } else {
            a = 0;
            for (uint32_t r = 0; i0 + r < n; ++r) a |= (uint32_t)out[i0 + r] << (8 * r);
        }
        if (a == 0u) continue;
        uint64_t pv[4];
        if (full) {
            typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
            const u32x4 p0 = __builtin_nontemporal_load((const u32x4 *)(packed + i0));
            const u32x4 p1 = __builtin_nontemporal_load((const u32x4 *)(packed + i0 + 2));
            pv[0] = (uint64_t)p0.x | ((uint64_t)p0.y << 32);
            pv[1] = (uint64_t)p0.z | ((uint64_t)p0.w << 32);
            pv[2] = (uint64_t)p1.x | ((uint64_t)p1.y << 32);
            pv[3] = (uint64_t)p1.z | ((uint64_t)p1.w << 32);
        } else {
#pragma unroll
            for (uint32_t r = 0; r < 4; ++r) pv[r] = i0 + r < n ? packed[i0 + r] : 0ull;
        }
        uint32_t na = a;
#pragma unroll
        for (uint32_t r = 0; r < 4; ++r) {
            uint32_t live = (a >> (8 * r)) & 1u;
            uint32_t x = (uint32_t)(pv[r] & kMask);
            const uint32_t b = (uint32_t)((pv[r] >> kPackBits) & kMask), f = (uint32_t)(pv[r] >> (2 * kPackBits));
            const uint32_t nb = m - b, bc = b >= c ? b - c : b + (m - c), nd = m - bc;
#pragma unroll
            for (int q = 0; q < 7; ++q) {
                if (q > 0) {
                    const uint32_t d = (f >> (q - 1)) & 1u ? nd : nb;
                    const uint32_t t = x - d;
                    x = x >= d ? t : t + m;
                }
                const uint32_t w = x >> 5;
                if (live && w >= lo && w < hi) live &= words[w] >> (x & 31);
            }
            na &= ~((((a >> (8 * r)) & 1u) & (live ^ 1u)) << (8 * r));
        }
        if (na != a || first) {
            if (full)
                *(uint32_t *)(out + i0) = na;
            else
                for (uint32_t r = 0; i0 + r < n; ++r) out[i0 + r] = (uint8_t)(na >> (8 * r));
        }
    }
}

// ---- compacted phased probe (keys in, answers out; the default for the phased shape).  The
// phased probe above streams every key's packed word and answer byte through every later phase,
// though after range 0 only about 63% of a half-present batch is still alive.  Here a group of 64
// consecutive keys (one wave) keeps one 16-B record {mask0, live}: mask0 = the keys alive after
// range 0, live = those alive so far.  Phase 0 stores the mask0 keys' packed words compacted at
// the front of the group's 64-slot row; a later phase's lane loads its word at rank
// popcount(mask0 below the lane), only while its key is live, and only the last phase writes
// answer bytes (all 64 of a group in one coalesced store).  Per 10M keys the streams shrink from
// ≈450 MB (every word and answer byte read by every phase) to ≈330 MB.
template <typename Src>
__global__ __launch_bounds__(kPhaseBlock) void k_probe_c0(Src src, uint64_t n, const uint32_t *__restrict__ words,
                                                  ModArg md, uint64_t *__restrict__ rows,
                                                  ulonglong2 *__restrict__ recs, uint32_t hi) {
    const uint32_t lane = threadIdx.x & 63u;
    for (uint64_t base = (uint64_t)blockIdx.x * blockDim.x; base < n; base += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t i = base + threadIdx.x;  // base is a multiple of 64: a wave is one group
        uint32_t pos[7];
        uint64_t pw;
        if constexpr (IsPacked<Src>::value) {  // a batch of packed residues (pre-hashed, or broadcast)
            const uint4 v = i < n ? src.load(i) : make_uint4(0u, 0u, 0u, 0u);
            pw = (uint64_t)v.x | (uint64_t)v.y << 32;
            packed_positions(pw, (uint32_t)md.m, (uint32_t)md.c, pos);
        } else {  // the packed word first, the positions from it: each residue and wrap flag once
            uint64_t h1 = 0, h2 = 0;
            if (i < n) src.hash(i, h1, h2);
            pw = pack_residue(h1, h2, md);
            packed_positions(pw, (uint32_t)md.m, (uint32_t)md.c, pos);
        }
        uint32_t acc = i < n ? 1u : 0u;
#pragma unroll
        for (int q = 0; q < 7; ++q) {
            const uint32_t w = pos[q] >> 5;
            if ((acc & 1u) && w < hi) acc &= words[w] >> (pos[q] & 31);
        }
        const uint64_t alive = __ballot(acc & 1u);
        const uint64_t g = i >> 6;
        if (acc & 1u) __builtin_nontemporal_store(pw, rows + g * 64 + lanes_below(alive));
        if (lane == 0 && i < n) recs[g] = make_ulonglong2(alive, alive);
    }
}

// A wave-uniform u64 as scalar values (readfirstlane returns int: each half is taken unsigned).
__device__ __forceinline__ uint64_t uniform64(uint64_t v) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)v);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
    return (uint64_t)hi << 32 | lo;
}

// Phase p > 0 over words [lo, hi); LAST writes the answers, else updates the records' live masks.
// A wave takes G groups per iteration (lane l = key l of each), so G keys per lane are in flight.
template <int G, bool LAST>
__global__ __launch_bounds__(kPhaseBlock) void k_probe_cp(const uint64_t *__restrict__ rows, ulonglong2 *recs,
                                                  uint64_t n, const uint32_t *__restrict__ words, ModArg md,
                                                  uint8_t *__restrict__ out, uint32_t lo, uint32_t hi) {
    const uint32_t m = (uint32_t)md.m, c = (uint32_t)md.c;
    constexpr uint64_t kMask = (1ull << kPackBits) - 1;
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t below = (1ull << lane) - 1ull;
    const uint64_t ng = (n + 63) >> 6;
    const uint64_t wave = __builtin_amdgcn_readfirstlane((blockIdx.x * blockDim.x + threadIdx.x) >> 6);
    const uint64_t step = (uint64_t)gridDim.x * (blockDim.x >> 6) * G;
    for (uint64_t g0 = wave * G; g0 < ng; g0 += step) {
        uint64_t m0[G], lv[G], pv[G];
        uint32_t live[G];
        // the G records in one wave-uniform load (the record array is padded to a multiple of G)
        struct Recs { ulonglong2 r[G]; };
        const Recs rv = *(const Recs *)(recs + g0);
#pragma unroll
        for (int j = 0; j < G; ++j) {
            const bool in = g0 + j < ng;
            m0[j] = in ? uniform64(rv.r[j].x) : 0ull;
            lv[j] = in ? uniform64(rv.r[j].y) : 0ull;
            live[j] = (uint32_t)(lv[j] >> lane) & 1u;
        }
#pragma unroll
        for (int j = 0; j < G; ++j)
            pv[j] = live[j] ? __builtin_nontemporal_load(rows + (g0 + j) * 64 + __popcll(m0[j] & below)) : 0ull;
#pragma unroll
        for (int j = 0; j < G; ++j) {
            uint32_t x = (uint32_t)(pv[j] & kMask);
            const uint32_t b = (uint32_t)((pv[j] >> kPackBits) & kMask), f = (uint32_t)(pv[j] >> (2 * kPackBits));
            const uint32_t nb = m - b, bc = b >= c ? b - c : b + (m - c), nd = m - bc;
#pragma unroll
            for (int q = 0; q < 7; ++q) {
                if (q > 0) {
                    const uint32_t d = (f >> (q - 1)) & 1u ? nd : nb;
                    const uint32_t t = x - d;
                    x = x >= d ? t : t + m;
                }
                const uint32_t w = x >> 5;
                if (live[j] && w >= lo && w < hi) live[j] &= words[w] >> (x & 31);
            }
        }
#pragma unroll
        for (int j = 0; j < G; ++j) {
            const uint64_t g = g0 + j;
            if constexpr (LAST) {
                const uint64_t i = g * 64 + lane;
                if (g < ng && i < n) out[i] = (uint8_t)live[j];
            } else {
                const uint64_t nl = __ballot(live[j]);
                if (lane == 0 && g < ng && nl != lv[j]) recs[g].y = nl;
            }
        }
    }
}

// Sliced probe over packed residues; k == 7.
template <int KPT>
__global__ __launch_bounds__(256) void k_probe_packed(const uint64_t *__restrict__ packed, uint64_t n,
                                                      const uint32_t *__restrict__ words, ModArg md,
                                                      uint8_t *__restrict__ out, uint32_t slice_shift,
                                                      uint32_t nslices) {
    const uint32_t m = (uint32_t)md.m, c = (uint32_t)md.c;
    constexpr uint64_t kMask = (1ull << kPackBits) - 1;
    const uint64_t span = (uint64_t)blockDim.x * KPT;
    for (uint64_t base = (uint64_t)blockIdx.x * span; base < n; base += (uint64_t)gridDim.x * span) {
        uint32_t pos[KPT][7];
        uint32_t acc[KPT];
#pragma unroll
        for (int r = 0; r < KPT; ++r) {
            const uint64_t i = base + (uint64_t)r * blockDim.x + threadIdx.x;
            const uint64_t v = i < n ? __builtin_nontemporal_load(packed + i) : 0ull;
            uint32_t x = (uint32_t)(v & kMask);
            const uint32_t b = (uint32_t)((v >> kPackBits) & kMask), f = (uint32_t)(v >> (2 * kPackBits));
            const uint32_t nb = m - b, bc = b >= c ? b - c : b + (m - c), nd = m - bc;
            pos[r][0] = x;
#pragma unroll
            for (int q = 1; q < 7; ++q) {
                const uint32_t na = (f >> (q - 1)) & 1u ? nd : nb;
                const uint32_t t = x - na;
                x = x >= na ? t : t + m;
                pos[r][q] = x;
            }
            acc[r] = i < n ? 1u : 0u;
        }
        for (uint32_t sl = 0; sl < nslices; ++sl) {
#pragma unroll
            for (int r = 0; r < KPT; ++r)
#pragma unroll
                for (int q = 0; q < 7; ++q) {
                    const uint32_t w = pos[r][q] >> 5;
                    if ((acc[r] & 1u) && (w >> slice_shift) == sl) acc[r] &= words[w] >> (pos[r][q] & 31);
                }
        }
#pragma unroll
        for (int r = 0; r < KPT; ++r) {
            const uint64_t i = base + (uint64_t)r * blockDim.x + threadIdx.x;
            if (i < n) out[i] = (uint8_t)(acc[r] & 1u);
        }
    }
}

// Multi-filter probe: hash once, test every filter; bit f of the mask = filter f's answer.
// SAME: all filters share (m, k) -> positions computed once per key.
template <typename Src, typename MaskT, bool SAME, int KFIX, bool M32>
__global__ __launch_bounds__(256) void k_probe_multi(Src src, uint64_t n, MultiArg ma, MaskT *__restrict__ mask) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        uint64_t h1, h2;
        src.hash(i, h1, h2);
        MaskT w = 0;
        if constexpr (SAME) {
            uint64_t pos[KFIX > 0 ? KFIX : 1];
            if constexpr (KFIX > 0) {
                for_positions<KFIX, M32>(h1, h2, ma.f[0].md, KFIX, [&](uint32_t q, uint64_t p) { pos[q] = p; });
                for (uint32_t f = 0; f < ma.nf; ++f) {
                    const uint32_t *wd = ma.f[f].words;
                    uint32_t acc = 1u;
#pragma unroll
                    for (int q = 0; q < KFIX; ++q)  // MayContain's early exit (lsm/bloom.go:86-89)
                        if (acc & 1u) acc &= wd[pos[q] >> 5] >> (uint32_t)(pos[q] & 31);
                    w |= (MaskT)(acc & 1u) << f;
                }
            }
        } else {
            for (uint32_t f = 0; f < ma.nf; ++f) {
                const uint32_t *wd = ma.f[f].words;
                uint32_t acc = 1u;
                for_positions<KFIX, M32>(h1, h2, ma.f[f].md, ma.f[f].md.k, [&](uint32_t, uint64_t p) {
                    if (acc & 1u) acc &= wd[p >> 5] >> (uint32_t)(p & 31);
                });
                w |= (MaskT)(acc & 1u) << f;
            }
        }
        mask[src.index(i)] = w;
    }
}

// Interleaved multi-filter table: entry p (one MaskT per bit position p < m) holds bit p of every
// filter, bit f = filter f.  Built per call from the filters' own word arrays (which stay the
// canonical, Encode-able layout); valid when all filters share (m, k), as compaction outputs do.
// One thread per 32 positions: nf coalesced word loads, 32 entries out.
// Bit-transposed table: entry p = bit p of every filter (bit f = filter f).  One thread per entry:
// the 32 lanes of a half-wave read the same word of each filter (one cache line per load
// instruction) and a wave stores 64 consecutive entries, so the table is written with full-line
// stores (a thread per word writing its 32 entries left each store 64 scattered 8-B writes: 49 µs
// for the C5 table of 958,506 u64 entries).
template <typename MaskT>
__global__ __launch_bounds__(256) void k_interleave(MultiArg ma, uint64_t m, MaskT *__restrict__ table) {
    const uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= m) return;
    const uint64_t w = p >> 5;
    const uint32_t j = (uint32_t)(p & 31);
    MaskT e = 0;
    for (uint32_t f0 = 0; f0 < ma.nf; f0 += 16) {  // 16 loads in flight, then combine
        uint32_t v[16];
#pragma unroll
        for (uint32_t r = 0; r < 16; ++r) v[r] = f0 + r < ma.nf ? ma.f[f0 + r].words[w] : 0u;
#pragma unroll
        for (uint32_t r = 0; r < 16; ++r) e |= (MaskT)((v[r] >> j) & 1u) << ((f0 + r) & (8 * sizeof(MaskT) - 1));
    }
    table[p] = e;
}

// Lane r holds row r of a 64 x 64 bit matrix (bit c = column c); returns column `lane` (bit r = row
// r's bit `lane`).  Six butterfly stages: stage j exchanges the off-diagonal j x j blocks of the
// lane pairs (r, r ^ j), one 64-bit shuffle and a masked merge each.
__device__ __forceinline__ uint64_t wave_transpose64(uint64_t x, uint32_t lane) {
    constexpr uint64_t kLow[6] = {0x00000000FFFFFFFFull, 0x0000FFFF0000FFFFull, 0x00FF00FF00FF00FFull,
                                  0x0F0F0F0F0F0F0F0Full, 0x3333333333333333ull, 0x5555555555555555ull};
#pragma unroll
    for (int st = 0; st < 6; ++st) {
        const uint32_t j = 32u >> st;
        const uint64_t lo = kLow[st];  // bit positions c with (c & j) == 0
        const uint32_t ylo = (uint32_t)__shfl_xor((int)(uint32_t)x, (int)j, 64);
        const uint32_t yhi = (uint32_t)__shfl_xor((int)(uint32_t)(x >> 32), (int)j, 64);
        const uint64_t y = (uint64_t)yhi << 32 | ylo;
        x = (lane & j) ? (x & ~lo) | ((y & ~lo) >> j) : (x & lo) | ((y & lo) << j);
    }
    return x;
}

// The same table by a bit transpose per wave: a wave covers 128 bit positions (4 words), lane f
// holds those 4 words of filter f (one 16-B load), and each 64-position half, transposed across
// the wave, leaves lane c holding entry p0 + 64 h + c (bit f = filter f): 64 consecutive entries
// per store.  Round 3 built each entry by a ballot (≈4 VALU per entry to move it into its lane);
// the transpose costs ≈1.5.  Needs 16-B aligned word arrays of seb_words_bytes(m) bytes.
template <typename MaskT>
__global__ __launch_bounds__(256) void k_interleave_xpose(MultiArg ma, uint64_t m, MaskT *__restrict__ table) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t p0 = (((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6) * 128;
    if (p0 >= m) return;  // wave-uniform
    uint4 v = make_uint4(0u, 0u, 0u, 0u);
    if (lane < ma.nf) v = *(const uint4 *)(ma.f[lane].words + (p0 >> 5));
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const uint64_t x = h ? (uint64_t)v.w << 32 | v.z : (uint64_t)v.y << 32 | v.x;
        const uint64_t e = wave_transpose64(x, lane);
        const uint64_t p = p0 + 64 * h + lane;
        if (p < m) table[p] = (MaskT)e;
    }
}

template <typename MaskT>
static void launch_interleave(const MultiArg &ma, uint64_t m, MaskT *table, hipStream_t s) {
    bool aligned = true;
    for (uint32_t f = 0; f < ma.nf; ++f) aligned &= ((uintptr_t)ma.f[f].words & 15) == 0;
    if (aligned)  // (one 4-B load per filter per entry otherwise: 22 vs 17 us for the C5 table)
        hipLaunchKernelGGL((k_interleave_xpose<MaskT>), dim3((unsigned)((m + 511) / 512)), dim3(256), 0, s, ma, m, table);
    else
        hipLaunchKernelGGL((k_interleave<MaskT>), dim3((unsigned)((m + 255) / 256)), dim3(256), 0, s, ma, m, table);
}

// Probe against the interleaved table: 7 gathers of one MaskT per key, AND -> the mask of every
// filter at once (bit f = MayContain of filter f).  Phase-sliced like k_probe_sliced so a table
// larger than one XCD's L2 is walked one slice (2^slice_shift entries) at a time; a key whose
// mask is already 0 stops gathering.
template <typename Src, typename MaskT, int KPT>
__global__ __launch_bounds__(256) void k_probe_interleaved(Src src, uint64_t n, const MaskT *__restrict__ table, ModArg md,
                                                           MaskT *__restrict__ mask, uint32_t slice_shift,
                                                           uint32_t nslices) {
    const uint64_t span = (uint64_t)blockDim.x * KPT;
    for (uint64_t base = (uint64_t)blockIdx.x * span; base < n; base += (uint64_t)gridDim.x * span) {
        uint32_t pos[KPT][7];
        MaskT acc[KPT];
#pragma unroll
        for (int r = 0; r < KPT; ++r) {
            const uint64_t i = base + (uint64_t)r * blockDim.x + threadIdx.x;
            uint64_t h1 = 0, h2 = 0;
            if (i < n) src.hash(i, h1, h2);
            for_positions<7, true>(h1, h2, md, 7, [&](uint32_t q, uint64_t p) { pos[r][q] = (uint32_t)p; });
            acc[r] = i < n ? (MaskT)~(MaskT)0 : (MaskT)0;
        }
        for (uint32_t sl = 0; sl < nslices; ++sl) {
#pragma unroll
            for (int r = 0; r < KPT; ++r)
#pragma unroll
                for (int q = 0; q < 7; ++q)
                    if (acc[r] && (pos[r][q] >> slice_shift) == sl) acc[r] &= table[pos[r][q]];
        }
#pragma unroll
        for (int r = 0; r < KPT; ++r) {
            const uint64_t i = base + (uint64_t)r * blockDim.x + threadIdx.x;
            if (i < n) mask[src.index(i)] = acc[r];
        }
    }
}

// Interleaved multi-filter probe over packed residues: the broadcast form of a batch probed
// against same-size filters on several GPUs (C5 at N > 1).  W = 8: k_pack_residues' 8-byte words
// (29-bit fields); W = 6: the narrow 48-bit form in 64-key blocks (k_pack_residues6, 21-bit fields).
template <typename MaskT, int W>
__global__ __launch_bounds__(256) void k_probe_interleaved_packed(const void *__restrict__ packed, uint64_t n,
                                                                  const MaskT *__restrict__ table, ModArg md,
                                                                  MaskT *__restrict__ mask, uint32_t slice_shift,
                                                                  uint32_t nslices) {
    constexpr int KPT = 2;
    constexpr uint32_t kBits = W == 8 ? kPackBits : kPack6Bits;
    constexpr uint64_t kMask = (1ull << kBits) - 1;
    const uint32_t m = (uint32_t)md.m, c = (uint32_t)md.c;
    const uint64_t span = (uint64_t)blockDim.x * KPT;
    for (uint64_t base = (uint64_t)blockIdx.x * span; base < n; base += (uint64_t)gridDim.x * span) {
        uint32_t pos[KPT][7];
        MaskT acc[KPT];
#pragma unroll
        for (int r = 0; r < KPT; ++r) {
            const uint64_t i = base + (uint64_t)r * blockDim.x + threadIdx.x;
            uint64_t v = 0;
            if (i < n) {
                if constexpr (W == 8)
                    v = __builtin_nontemporal_load((const uint64_t *)packed + i);
                else
                    v = load_packed6((const uint8_t *)packed, i);
            }
            uint32_t x = (uint32_t)(v & kMask);
            const uint32_t b = (uint32_t)((v >> kBits) & kMask), f = (uint32_t)(v >> (2 * kBits));
            const uint32_t nb = m - b, bc = b >= c ? b - c : b + (m - c), nd = m - bc;
            pos[r][0] = x;
#pragma unroll
            for (int q = 1; q < 7; ++q) {
                const uint32_t d = (f >> (q - 1)) & 1u ? nd : nb;
                const uint32_t t = x - d;
                x = x >= d ? t : t + m;
                pos[r][q] = x;
            }
            acc[r] = i < n ? (MaskT)~(MaskT)0 : (MaskT)0;
        }
        for (uint32_t sl = 0; sl < nslices; ++sl) {
#pragma unroll
            for (int r = 0; r < KPT; ++r)
#pragma unroll
                for (int q = 0; q < 7; ++q)
                    if (acc[r] && (pos[r][q] >> slice_shift) == sl) acc[r] &= table[pos[r][q]];
        }
#pragma unroll
        for (int r = 0; r < KPT; ++r) {
            const uint64_t i = base + (uint64_t)r * blockDim.x + threadIdx.x;
            if (i < n) mask[i] = acc[r];
        }
    }
}

// Batched build of independent small filters (compaction outputs, lsm/compaction.go:226-333): each
// filter's keys are split over `splits` workgroups, each holding the whole filter in LDS
// (ds_or_b32, no global atomics while hashing), then OR-merging its image into HBM: a plain
// read-modify-write when one workgroup owns the filter, device-scope atomic ORs of the non-zero
// words when several do.  One workgroup per filter left 32 of the 256 CUs busy for a 32-filter
// launch.  Filters too large for LDS go through k_build.
template <typename Src, int KFIX, bool M32>
__global__ __launch_bounds__(1024) void k_build_many_lds(Src src, ManyArg ma, uint32_t splits) {
    extern __shared__ uint32_t lds[];
    const ManyFilter &F = ma.f[blockIdx.x / splits];
    const uint32_t part = blockIdx.x % splits;
    const uint32_t nw = (uint32_t)F.nwords;
    const uint64_t nk = F.key_end - F.key_begin;
    const uint64_t k0 = F.key_begin + nk * part / splits, k1 = F.key_begin + nk * (part + 1) / splits;
    for (uint32_t j = threadIdx.x; j < nw; j += blockDim.x) lds[j] = 0u;
    __syncthreads();
    for (uint64_t i = k0 + threadIdx.x; i < k1; i += blockDim.x) {
        uint64_t h1, h2;
        src.hash(i, h1, h2);
        for_positions<KFIX, M32>(h1, h2, F.md, F.md.k, [&](uint32_t, uint64_t p) {
            __hip_atomic_fetch_or(lds + (p >> 5), 1u << (uint32_t)(p & 31), __ATOMIC_RELAXED,
                                  __HIP_MEMORY_SCOPE_WORKGROUP);
        });
    }
    __syncthreads();
    if (splits == 1) {
        for (uint32_t j = threadIdx.x; j < nw; j += blockDim.x) {
            const uint32_t v = lds[j];
            if (v) F.words[j] |= v;
        }
    } else {
        for (uint32_t j = threadIdx.x; j < nw; j += blockDim.x) {
            const uint32_t v = lds[j];
            if (v) __hip_atomic_fetch_or(F.words + j, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

// Small-filter build in two launches, no global atomics (build_algo 4; flush- and
// compaction-sized filters whose word array fits one CU's LDS).  k_build_images: workgroup g
// sets the bits of its key range [n*g/G, n*(g+1)/G) in an LDS image of the whole filter with
// ds_or, then stores the image to scratch with 16-B stores.  k_or_images: one thread per 16 B of
// filter ORs the G images (and the old words, unless the filter is fresh) into the filter.  The
// device-scope atomics of k_build go to memory one by one (TCC_EA0_ATOMIC = n*k,
// profiles/r01a_pmc.csv); here the keys are hashed on G CUs and the only global traffic is
// G images written and read once.
template <typename Src, int KFIX, bool M32>
__global__ __launch_bounds__(1024) void k_build_images(Src src, uint64_t n, ModArg md, uint32_t nw4,
                                                       uint4 *__restrict__ images) {
    extern __shared__ uint4 limg[];
    uint32_t *lw = (uint32_t *)limg;
    const uint32_t g = blockIdx.x, G = gridDim.x;
    for (uint32_t j = threadIdx.x; j < nw4; j += blockDim.x) limg[j] = make_uint4(0, 0, 0, 0);
    __syncthreads();
    const uint64_t k0 = n * g / G, k1 = n * (g + 1) / G;
    for (uint64_t i = k0 + threadIdx.x; i < k1; i += blockDim.x) {
        uint64_t h1, h2;
        src.hash(i, h1, h2);
        for_positions<KFIX, M32>(h1, h2, md, md.k, [&](uint32_t, uint64_t p) {
            __hip_atomic_fetch_or(lw + (p >> 5), 1u << (uint32_t)(p & 31), __ATOMIC_RELAXED,
                                  __HIP_MEMORY_SCOPE_WORKGROUP);
        });
    }
    __syncthreads();
    uint4 *out = images + (uint64_t)g * nw4;
    for (uint32_t j = threadIdx.x; j < nw4; j += blockDim.x) out[j] = limg[j];
}

__global__ __launch_bounds__(256) void k_or_images(const uint4 *__restrict__ images, uint32_t G, uint32_t nw4,
                                                   uint4 *__restrict__ words, uint32_t fresh) {
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= nw4) return;
    uint4 a = fresh ? make_uint4(0, 0, 0, 0) : words[j];
    for (uint32_t g0 = 0; g0 < G; g0 += 8) {  // 8 image loads in flight
        uint4 v[8];
#pragma unroll
        for (uint32_t r = 0; r < 8; ++r) v[r] = g0 + r < G ? images[(uint64_t)(g0 + r) * nw4 + j] : make_uint4(0, 0, 0, 0);
#pragma unroll
        for (uint32_t r = 0; r < 8; ++r) {
            a.x |= v[r].x;
            a.y |= v[r].y;
            a.z |= v[r].z;
            a.w |= v[r].w;
        }
    }
    words[j] = a;
}

// ------------------------------------------------------------------ launchers ----------------

static inline unsigned grid_for(uint64_t n, unsigned block, unsigned cap) {
    uint64_t g = (n + block - 1) / block;
    if (g < 1) g = 1;
    return (unsigned)(g > cap ? cap : g);
}



Options &options() {
    static Options o;
    return o;
}

// 1 device-scope atomics, 2 radix-partitioned (bucketed), 3 the whole filter in one CU's LDS
// with the keys split over workgroups (k_build_many_lds), 4 LDS images OR-merged by a second
// kernel (k_build_images).  Auto (tools/small_builds.py, profiles/r03_small_builds.jsonl): the
// image build while the word array fits 160 KiB, bucketed from bucket_min_keys for larger
// filters, device-scope atomics below that.
int choose_build_algo(uint64_t n, uint64_t m, uint32_t k) {
    const Options &o = options();
    const bool lds = (m + 127) / 128 * 16 <= kLdsFilterBytes;
    if (o.build_algo == 1) return 1;
    if (o.build_algo == 2) return bucketed_supported(m, k) ? 2 : 1;
    if (o.build_algo == 3) return lds ? 3 : 1;
    if (o.build_algo == 4) return lds ? 4 : 1;
    if (lds && n >= o.lds_min_keys) return 4;
    return bucketed_supported(m, k) && n >= o.bucket_min_keys ? 2 : 1;
}

// Workgroups of the image build: about 8192 keys each, at most 32 (1024 keys each, up to 128
// workgroups, took 45 us at 100K keys: the merge traffic of 98 images outweighed the hashing).
uint32_t image_groups(uint64_t n) {
    const uint64_t g = (n + 8191) / 8192;
    return (uint32_t)(g < 1 ? 1 : g > 32 ? 32 : g);
}

uint64_t image_workspace_bytes(uint64_t n, uint64_t m) { return image_groups(n) * ((m + 127) / 128) * 16; }

hipError_t launch_build_images(const KeyBatch &kb, uint32_t *words, const ModArg &md, void *ws, uint64_t ws_bytes,
                               bool fresh, hipStream_t s) {
    if (kb.n == 0 || md.k == 0) return hipSuccess;
    const uint32_t nw4 = (uint32_t)((md.m + 127) / 128);
    const uint32_t G = image_groups(kb.n);
    if (nw4 * 16ull > kLdsFilterBytes || ws_bytes < image_workspace_bytes(kb.n, md.m)) return hipErrorInvalidValue;
    // one workgroup: its image goes straight to the filter (fresh) or through the OR kernel
    uint4 *images = G > 1 || !fresh ? (uint4 *)ws : (uint4 *)words;
    const bool m32 = md.m < kM32Limit, k7 = md.k == 7;
    const hipError_t e = with_src(kb, [&](auto src) {
        using S = decltype(src);
        auto go = [&](auto kern) {
            hipError_t a = hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                                               (int)(nw4 * 16));
            if (a != hipSuccess) return a;
            hipLaunchKernelGGL(kern, dim3(G), dim3(1024), nw4 * 16, s, src, kb.n, md, nw4, images);
            return hipGetLastError();
        };
        if (m32) return k7 ? go(k_build_images<S, 7, true>) : go(k_build_images<S, 0, true>);
        return k7 ? go(k_build_images<S, 7, false>) : go(k_build_images<S, 0, false>);
    });
    if (e != hipSuccess || (G == 1 && fresh)) return e;
    hipLaunchKernelGGL(k_or_images, dim3((nw4 + 255) / 256), dim3(256), 0, s, (const uint4 *)images, G, nw4,
                       (uint4 *)words, fresh ? 1u : 0u);
    return hipGetLastError();
}

template <typename Src, int KFIX, bool M32>
static hipError_t launch_build_t(const Src &src, uint64_t n, uint32_t *words, const ModArg &md, hipStream_t s) {
    unsigned g = grid_for(n, 256, options().grid_cap);
    hipLaunchKernelGGL((k_build<Src, KFIX, M32>), dim3(g), dim3(256), 0, s, src, n, words, md);
    return hipGetLastError();
}

template <typename Src, int KFIX, bool M32, int SPLIT, int KPT>
static hipError_t launch_probe_t(const Src &src, uint64_t n, const uint32_t *words, const ModArg &md, uint8_t *out,
                                 hipStream_t s) {
    unsigned g = grid_for((n + KPT - 1) / KPT, 256, options().grid_cap);
    hipLaunchKernelGGL((k_probe<Src, KFIX, M32, SPLIT, KPT>), dim3(g), dim3(256), 0, s, src, n, words, md, out);
    return hipGetLastError();
}

// 2 MiB of filter words per slice of the sliced probes (swept: 2^17-2^20 words).
constexpr uint32_t kSliceShift = 19;

static inline uint32_t slice_count(uint64_t m) {
    const uint64_t nwords = (m + 31) / 32;
    return (uint32_t)((nwords + (1ull << kSliceShift) - 1) >> kSliceShift);
}

// k == 7 probes that are not phased: the sliced probe for m < 2^31 filters spanning more than one
// slice, otherwise all positions of 2 keys per thread, 3 gathers first and the rest only for keys
// still alive.
template <typename Src, bool M32>
static hipError_t launch_probe7(const Src &src, uint64_t n, const uint32_t *words, const ModArg &md, uint8_t *out,
                                hipStream_t s) {
    if constexpr (M32) {
        if (const uint32_t nsl = slice_count(md.m); nsl > 1) {
            const unsigned g = grid_for((n + 1) / 2, 256, options().grid_cap);
            hipLaunchKernelGGL((k_probe_sliced<Src, 2>), dim3(g), dim3(256), 0, s, src, n, words, md, out, kSliceShift,
                               nsl);
            return hipGetLastError();
        }
    }
    return launch_probe_t<Src, 7, M32, 3, 2>(src, n, words, md, out, s);
}

// Filter clear: one 16-B store per lane, 4 per thread (hipMemsetAsync's fill kernel took 7.0 us
// for the 12 MB C2 filter, profiles/r02_kernel_stats.csv).
__global__ __launch_bounds__(256) void k_clear_words(uint4 *__restrict__ w, uint64_t n16) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += stride) w[i] = make_uint4(0, 0, 0, 0);
}

hipError_t launch_clear_words(uint32_t *words, uint64_t bytes, hipStream_t s) {
    const uint64_t n16 = bytes / 16;
    if (n16 == 0) return hipSuccess;
    const unsigned g = grid_for((n16 + 3) / 4, 256, options().grid_cap);
    hipLaunchKernelGGL(k_clear_words, dim3(g), dim3(256), 0, s, (uint4 *)words, n16);
    return hipGetLastError();
}

// Copy `bytes` of device words to host-pinned memory with 16-B stores over PCIe (the small
// builds' bits back to the host): a kernel in the build's stream, where a DMA copy would start
// ~16 us after the build ends (profiles/r03_flush_trace.txt).  dst and src 16-B aligned.
__global__ __launch_bounds__(256) void k_copy_out(const uint4 *__restrict__ src, uint4 *__restrict__ dst, uint64_t n16,
                                                  const uint8_t *__restrict__ tail_src, uint8_t *__restrict__ tail_dst,
                                                  uint32_t tail) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n16) dst[i] = src[i];
    if (i < tail) tail_dst[i] = tail_src[i];
}

hipError_t launch_copy_out(const uint32_t *words, uint8_t *host, uint64_t bytes, hipStream_t s) {
    if (bytes == 0) return hipSuccess;
    const uint64_t n16 = bytes / 16, tail = bytes % 16;
    const uint64_t items = n16 > tail ? n16 : tail;
    hipLaunchKernelGGL(k_copy_out, dim3((unsigned)((items + 255) / 256)), dim3(256), 0, s, (const uint4 *)words,
                       (uint4 *)host, n16, (const uint8_t *)words + n16 * 16, host + n16 * 16, (uint32_t)tail);
    return hipGetLastError();
}

hipError_t launch_build(const KeyBatch &kb, uint32_t *words, const ModArg &md, hipStream_t s) {
    if (kb.n == 0 || md.k == 0) return hipSuccess;
    const bool m32 = md.m < kM32Limit;
    const bool k7 = md.k == 7;
    return with_src(kb, [&](auto src) {
        using S = decltype(src);
        if (m32) return k7 ? launch_build_t<S, 7, true>(src, kb.n, words, md, s) : launch_build_t<S, 0, true>(src, kb.n, words, md, s);
        return k7 ? launch_build_t<S, 7, false>(src, kb.n, words, md, s) : launch_build_t<S, 0, false>(src, kb.n, words, md, s);
    });
}

hipError_t launch_probe(const KeyBatch &kb, const uint32_t *words, const ModArg &md, uint8_t *out, hipStream_t s) {
    if (kb.n == 0) return hipSuccess;
    if (md.k == 0) return hipMemsetAsync(out, 1, kb.n, s);  // zero hashes: MayContain is true
    const bool m32 = md.m < kM32Limit;
    const bool k7 = md.k == 7;
    return with_src(kb, [&](auto src) {
        using S = decltype(src);
        if (m32) return k7 ? launch_probe7<S, true>(src, kb.n, words, md, out, s) : launch_probe_t<S, 0, true, 0, 1>(src, kb.n, words, md, out, s);
        return k7 ? launch_probe7<S, false>(src, kb.n, words, md, out, s) : launch_probe_t<S, 0, false, 0, 1>(src, kb.n, words, md, out, s);
    });
}

template <typename Src, typename MaskT, bool SAME, int KFIX, bool M32>
static hipError_t launch_multi_t(const Src &src, uint64_t n, const MultiArg &ma, void *mask, hipStream_t s) {
    unsigned g = grid_for(n, 256, options().grid_cap);
    hipLaunchKernelGGL((k_probe_multi<Src, MaskT, SAME, KFIX, M32>), dim3(g), dim3(256), 0, s, src, n, ma,
                       (MaskT *)mask);
    return hipGetLastError();
}

// Slice of the interleaved table: 2 MiB of entries.
template <typename MaskT>
constexpr uint32_t table_slice_shift() {
    return 21 - (sizeof(MaskT) == 1 ? 0 : sizeof(MaskT) == 2 ? 1 : sizeof(MaskT) == 4 ? 2 : 3);
}

template <typename MaskT>
static hipError_t interleaved_mask(const KeyBatch &kb, const MultiArg &ma, void *mask, void *ws, hipStream_t s) {
    const ModArg &md = ma.f[0].md;
    MaskT *table = (MaskT *)ws;
    // valid-bit mask: filters beyond nf must read 0, which the zero-initialised entries give
    launch_interleave<MaskT>(ma, md.m, table, s);
    const uint32_t shift = table_slice_shift<MaskT>();
    const uint32_t nsl = (uint32_t)((md.m + (1ull << shift) - 1) >> shift);
    return with_src(kb, [&](auto src) {
        using S = decltype(src);
        unsigned g = grid_for((kb.n + 1) / 2, 256, options().grid_cap);
        hipLaunchKernelGGL((k_probe_interleaved<S, MaskT, 2>), dim3(g), dim3(256), 0, s, src, kb.n, (const MaskT *)table,
                           md, (MaskT *)mask, shift, nsl);
        return hipGetLastError();
    });
}

template <typename MaskT, int W>
static hipError_t interleaved_mask_packed(const void *packed, uint64_t n, const MultiArg &ma, void *mask, void *ws,
                                          hipStream_t s) {
    const ModArg &md = ma.f[0].md;
    MaskT *table = (MaskT *)ws;
    launch_interleave<MaskT>(ma, md.m, table, s);
    const uint32_t shift = table_slice_shift<MaskT>();
    const uint32_t nsl = (uint32_t)((md.m + (1ull << shift) - 1) >> shift);
    const unsigned g = grid_for((n + 1) / 2, 256, options().grid_cap);
    hipLaunchKernelGGL((k_probe_interleaved_packed<MaskT, W>), dim3(g), dim3(256), 0, s, packed, n, (const MaskT *)table, md,
                       (MaskT *)mask, shift, nsl);
    return hipGetLastError();
}

hipError_t launch_probe_interleaved_packed(const uint64_t *packed, uint64_t n, const MultiArg &ma, void *mask,
                                           uint32_t mask_bytes, void *ws, hipStream_t s) {
    if (n == 0) return hipSuccess;
    switch (mask_bytes) {
        case 1: return interleaved_mask_packed<uint8_t, 8>(packed, n, ma, mask, ws, s);
        case 2: return interleaved_mask_packed<uint16_t, 8>(packed, n, ma, mask, ws, s);
        case 4: return interleaved_mask_packed<uint32_t, 8>(packed, n, ma, mask, ws, s);
        default: return interleaved_mask_packed<uint64_t, 8>(packed, n, ma, mask, ws, s);
    }
}

hipError_t launch_probe_interleaved_packed6(const uint8_t *packed6, uint64_t n, const MultiArg &ma, void *mask,
                                            uint32_t mask_bytes, void *ws, hipStream_t s) {
    if (n == 0) return hipSuccess;
    switch (mask_bytes) {
        case 1: return interleaved_mask_packed<uint8_t, 6>(packed6, n, ma, mask, ws, s);
        case 2: return interleaved_mask_packed<uint16_t, 6>(packed6, n, ma, mask, ws, s);
        case 4: return interleaved_mask_packed<uint32_t, 6>(packed6, n, ma, mask, ws, s);
        default: return interleaved_mask_packed<uint64_t, 6>(packed6, n, ma, mask, ws, s);
    }
}

uint64_t interleaved_bytes(const MultiArg &ma, uint32_t mask_bytes) {
    if (ma.nf < 2) return 0;
    for (uint32_t f = 1; f < ma.nf; ++f)
        if (ma.f[f].md.m != ma.f[0].md.m || ma.f[f].md.k != ma.f[0].md.k) return 0;
    if (ma.f[0].md.k != 7 || ma.f[0].md.m >= kM32Limit) return 0;
    return ((ma.f[0].md.m + 31) / 32) * 32 * mask_bytes;
}

hipError_t launch_probe_interleaved(const KeyBatch &kb, const MultiArg &ma, void *mask, uint32_t mask_bytes, void *ws,
                                    hipStream_t s) {
    if (kb.n == 0) return hipSuccess;
    switch (mask_bytes) {
        case 1: return interleaved_mask<uint8_t>(kb, ma, mask, ws, s);
        case 2: return interleaved_mask<uint16_t>(kb, ma, mask, ws, s);
        case 4: return interleaved_mask<uint32_t>(kb, ma, mask, ws, s);
        default: return interleaved_mask<uint64_t>(kb, ma, mask, ws, s);
    }
}

template <typename MaskT>
static hipError_t multi_mask(const KeyBatch &kb, const MultiArg &ma, void *mask, hipStream_t s) {
    bool same = true, m32 = true;
    for (uint32_t f = 0; f < ma.nf; ++f) {
        same &= ma.f[f].md.m == ma.f[0].md.m && ma.f[f].md.k == ma.f[0].md.k;
        m32 &= ma.f[f].md.m < kM32Limit;
    }
    const bool k7same = same && ma.f[0].md.k == 7;
    return with_src(kb, [&](auto src) {
        using S = decltype(src);
        if (k7same) {
            return m32 ? launch_multi_t<S, MaskT, true, 7, true>(src, kb.n, ma, mask, s)
                       : launch_multi_t<S, MaskT, true, 7, false>(src, kb.n, ma, mask, s);
        }
        return m32 ? launch_multi_t<S, MaskT, false, 0, true>(src, kb.n, ma, mask, s)
                   : launch_multi_t<S, MaskT, false, 0, false>(src, kb.n, ma, mask, s);
    });
}

hipError_t launch_probe_multi(const KeyBatch &kb, const MultiArg &ma, void *mask, uint32_t mask_bytes,
                              hipStream_t s) {
    if (kb.n == 0) return hipSuccess;
    switch (mask_bytes) {
        case 1: return multi_mask<uint8_t>(kb, ma, mask, s);
        case 2: return multi_mask<uint16_t>(kb, ma, mask, s);
        case 4: return multi_mask<uint32_t>(kb, ma, mask, s);
        default: return multi_mask<uint64_t>(kb, ma, mask, s);
    }
}

hipError_t launch_build_many_lds(const KeyBatch &kb, const ManyArg &ma, uint32_t lds_bytes, hipStream_t s) {
    if (ma.nf == 0) return hipSuccess;
    bool m32 = true, k7 = true;
    for (uint32_t f = 0; f < ma.nf; ++f) {
        m32 &= ma.f[f].md.m < kM32Limit;
        k7 &= ma.f[f].md.k == 7;
    }
    return with_src(kb, [&](auto src) {
        using S = decltype(src);
        // splits: enough workgroups for one per CU (256), at least 8K keys each
        uint64_t most = 0;
        for (uint32_t f = 0; f < ma.nf; ++f) most = std::max<uint64_t>(most, ma.f[f].key_end - ma.f[f].key_begin);
        uint32_t splits = options().many_splits;
        if (splits == 0) {
            splits = (256 + ma.nf - 1) / ma.nf;
            while (splits > 1 && most / splits < 8192) --splits;
        }
        auto go = [&](auto kern) {
            hipError_t e = hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_bytes);
            if (e != hipSuccess) return e;
            hipLaunchKernelGGL(kern, dim3(ma.nf * splits), dim3(1024), lds_bytes, s, src, ma, splits);
            return hipGetLastError();
        };
        if (m32) return k7 ? go(k_build_many_lds<S, 7, true>) : go(k_build_many_lds<S, 0, true>);
        return k7 ? go(k_build_many_lds<S, 7, false>) : go(k_build_many_lds<S, 0, false>);
    });
}

hipError_t launch_pack_residues(const KeyBatch &kb, const ModArg &md, uint64_t *packed, hipStream_t s) {
    if (kb.n == 0) return hipSuccess;
    return with_src(kb, [&](auto src) {
        using S = decltype(src);
        hipLaunchKernelGGL(k_pack_residues<S>, dim3(grid_for(kb.n, 256, options().grid_cap)), dim3(256), 0, s, src,
                           kb.n, md, packed);
        return hipGetLastError();
    });
}

hipError_t launch_pack_residues6(const KeyBatch &kb, const ModArg &md, uint8_t *packed6, hipStream_t s) {
    if (kb.n == 0) return hipSuccess;
    return with_src(kb, [&](auto src) {
        using S = decltype(src);
        hipLaunchKernelGGL(k_pack_residues6<S>, dim3(grid_for(kb.n, 256, options().grid_cap)), dim3(256), 0, s, src,
                           kb.n, md, packed6);
        return hipGetLastError();
    });
}

hipError_t launch_probe_packed(const uint64_t *packed, uint64_t n, const uint32_t *words, const ModArg &md,
                               uint8_t *out, hipStream_t s) {
    if (n == 0) return hipSuccess;
    const unsigned g = grid_for((n + 1) / 2, 256, options().grid_cap);
    hipLaunchKernelGGL(k_probe_packed<2>, dim3(g), dim3(256), 0, s, packed, n, words, md, out, kSliceShift,
                       slice_count(md.m));
    return hipGetLastError();
}

hipError_t launch_probe_emit(const KeyBatch &kb, const uint32_t *words, const ModArg &md, uint8_t *out,
                             uint64_t *packed, hipStream_t s) {
    if (kb.n == 0) return hipSuccess;
    const unsigned g = grid_for((kb.n + 1) / 2, 256, options().grid_cap);
    return with_src(kb, [&](auto src) {
        using S = decltype(src);
        hipLaunchKernelGGL((k_probe_sliced_emit<S, 2>), dim3(g), dim3(256), 0, s, src, kb.n, words, md, out, packed,
                           kSliceShift, slice_count(md.m));
        return hipGetLastError();
    });
}

// Phased probe.  From keys (kb != nullptr): phase 0 hashes them and writes their packed residues
// to `packed`; from packed words (kb == nullptr): every phase reads them.
hipError_t launch_probe_phased(const KeyBatch *kb, uint64_t n, const uint32_t *words, const ModArg &md, uint8_t *out,
                               uint64_t *packed, hipStream_t s) {
    if (n == 0) return hipSuccess;
    const uint64_t nwords = (md.m + 31) / 32;
    const uint64_t np = probe_phase_count(md.m);
    auto bound = [&](uint64_t p) { return (uint32_t)(nwords * p / np); };
    const unsigned cap = options().grid_cap;
    uint64_t p0 = 0;
    if (kb) {  // phase 0: one key per thread (2 per thread measured 3% slower)
        const hipError_t e = with_src(*kb, [&](auto src) {
            using S = decltype(src);
            hipLaunchKernelGGL((k_probe_phase0<S, 1>), dim3(grid_for(n, kPhaseBlock, cap)), dim3(kPhaseBlock), 0, s, src, n,
                               words, md, out, packed, bound(1));
            return hipGetLastError();
        });
        if (e != hipSuccess) return e;
        p0 = 1;
    }
    const unsigned g = grid_for((n + 3) / 4, kPhaseBlock, cap);
    for (uint64_t p = p0; p < np; ++p) {
        hipLaunchKernelGGL(k_probe_phase, dim3(g), dim3(kPhaseBlock), 0, s, packed, n, words, md, out, bound(p),
                           bound(p + 1), p == 0 ? 1u : 0u);
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

// Compacted phased probe from keys: 64 packed-word slots per group of 64 keys, then the groups'
// 16-B records.
uint64_t probe_compact_bytes(uint64_t n) {
    const uint64_t ng = (n + 63) / 64;
    return ng * 64 * 8 + (ng + 8) * 16;  // records padded for k_probe_cp's G-record loads
}

template <typename Phase0>
static hipError_t run_probe_compact(uint64_t n, const uint32_t *words, const ModArg &md, uint8_t *out, void *ws,
                                    hipStream_t s, Phase0 &&phase0) {
    if (n == 0) return hipSuccess;
    const uint64_t nwords = (md.m + 31) / 32;
    const uint64_t np = probe_phase_count(md.m);
    if (np < 2) return hipErrorInvalidValue;
    auto bound = [&](uint64_t p) { return (uint32_t)(nwords * p / np); };
    const unsigned cap = options().grid_cap;
    const uint64_t ng = (n + 63) / 64;
    uint64_t *rows = (uint64_t *)ws;
    ulonglong2 *recs = (ulonglong2 *)(rows + ng * 64);
    auto launch0 = [&](auto src) {
        using S = decltype(src);
        hipLaunchKernelGGL(k_probe_c0<S>, dim3(grid_for(n, kPhaseBlock, cap)), dim3(kPhaseBlock), 0, s, src, n, words,
                           md, rows, recs, bound(1));
        return hipGetLastError();
    };
    hipError_t e = phase0(launch0, rows, recs, bound(1));
    if (e != hipSuccess) return e;
    // 4 groups per wave iteration (1, 2 and 8 measured slower)
    constexpr int G = 4;
    const unsigned g = grid_for((ng + G - 1) / G * 64, kPhaseBlock, cap);
    for (uint64_t p = 1; p < np; ++p) {
        if (p + 1 < np)
            hipLaunchKernelGGL((k_probe_cp<G, false>), dim3(g), dim3(kPhaseBlock), 0, s, rows, recs, n, words, md, out,
                               bound(p), bound(p + 1));
        else
            hipLaunchKernelGGL((k_probe_cp<G, true>), dim3(g), dim3(kPhaseBlock), 0, s, rows, recs, n, words, md, out,
                               bound(p), bound(p + 1));
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    return hipSuccess;
}

hipError_t launch_probe_compact(const KeyBatch &kb, const uint32_t *words, const ModArg &md, uint8_t *out, void *ws,
                                hipStream_t s) {
    return run_probe_compact(kb.n, words, md, out, ws, s,
                             [&](auto &&launch0, uint64_t *, ulonglong2 *, uint32_t) { return with_src(kb, launch0); });
}

hipError_t launch_probe_compact_packed(const uint64_t *packed, uint64_t n, const uint32_t *words, const ModArg &md,
                                       uint8_t *out, void *ws, hipStream_t s) {
    return run_probe_compact(n, words, md, out, ws, s, [&](auto &&launch0, uint64_t *, ulonglong2 *, uint32_t) {
        return launch0(KeysPacked{packed});
    });
}

hipError_t launch_probe_compact_varlen(const KeyBatch &kb, const uint32_t *words, const ModArg &md, uint8_t *out,
                                       void *ws, hipStream_t s) {
    return run_probe_compact(kb.n, words, md, out, ws, s, [&](auto &&, uint64_t *rows, ulonglong2 *recs, uint32_t hi) {
        return launch_hash_varlen_phase0(kb, md, words, rows, recs, hi, s);
    });
}

// Phases of the phased probe: probe_phases, or one per 4 MiB of filter (one XCD's L2).
uint64_t probe_phase_count(uint64_t m) {
    const int64_t want = options().probe_phases;
    const uint64_t bytes = (m + 7) / 8;
    uint64_t np = want > 0 ? (uint64_t)want : (bytes + (4ull << 20) - 1) / (4ull << 20);
    const uint64_t nwords = (m + 31) / 32;
    if (np > nwords) np = nwords;
    return np < 1 ? 1 : np;
}

// ---- sharded build of one filter: each rank ORs its key shard into a partial
// filter; after an all-to-all every rank holds the G partials of its own word slice, laid out
// slice after slice, and ORs them into its slice of the final filter.  RCCL has no bitwise-OR
// reduction (rccl.h: sum/prod/max/min/avg), so this kernel is the reduction step.  Streaming:
// one 16-B load per slice and one 16-B store per lane when the slice is a multiple of 4 words.
template <bool VEC>
__global__ __launch_bounds__(256) void k_or_slices(const uint32_t *__restrict__ in, uint32_t nslices,
                                                   uint64_t slice_words, uint32_t *__restrict__ out) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    if constexpr (VEC) {
        const uint64_t nv = slice_words / 4;
        const uint4 *v = (const uint4 *)in;
        for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nv; i += stride) {
            uint4 a = v[i];
            for (uint32_t s = 1; s < nslices; ++s) {
                const uint4 b = v[(uint64_t)s * nv + i];
                a.x |= b.x;
                a.y |= b.y;
                a.z |= b.z;
                a.w |= b.w;
            }
            ((uint4 *)out)[i] = a;
        }
    } else {
        for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < slice_words; i += stride) {
            uint32_t a = in[i];
            for (uint32_t s = 1; s < nslices; ++s) a |= in[(uint64_t)s * slice_words + i];
            out[i] = a;
        }
    }
}

hipError_t launch_or_slices(const uint32_t *in, uint32_t nslices, uint64_t slice_words, uint32_t *out, hipStream_t s) {
    if (slice_words == 0 || nslices == 0) return hipSuccess;
    const bool vec = slice_words % 4 == 0 && ((uintptr_t)in & 15) == 0 && ((uintptr_t)out & 15) == 0;
    const uint64_t items = vec ? slice_words / 4 : slice_words;
    const unsigned g = grid_for(items, 256, options().grid_cap);
    if (vec)
        hipLaunchKernelGGL(k_or_slices<true>, dim3(g), dim3(256), 0, s, in, nslices, slice_words, out);
    else
        hipLaunchKernelGGL(k_or_slices<false>, dim3(g), dim3(256), 0, s, in, nslices, slice_words, out);
    return hipGetLastError();
}

}  // namespace seb
