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
// 64-bit Barrett reductions, then k-1 incremental residue steps (u32 when m < 2^32), then k
// random word touches (atomic OR for build, gather for probe).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "seb_kernels.h"

namespace seb {

constexpr uint64_t kFnvOffset = 0xcbf29ce484222325ull;
constexpr uint64_t kFnvPrime = 0x100000001b3ull;

// ------------------------------------------------------------------ hashing ----------------

__device__ __forceinline__ void fnv_byte(uint32_t b, uint64_t &h1, uint64_t &h2) {
    h1 = (h1 ^ (uint64_t)b) * kFnvPrime;  // FNV-1a (hash1)
    h2 = (h2 * kFnvPrime) ^ (uint64_t)b;  // FNV-1  (hash2)
}

__device__ __forceinline__ void fnv_word(uint32_t w, uint64_t &h1, uint64_t &h2) {
    fnv_byte(w & 0xffu, h1, h2);
    fnv_byte((w >> 8) & 0xffu, h1, h2);
    fnv_byte((w >> 16) & 0xffu, h1, h2);
    fnv_byte(w >> 24, h1, h2);
}

// Bytes [lo, hi) of word w (0 <= lo <= hi <= 4), predicated so a wave stays converged.
__device__ __forceinline__ void fnv_word_part(uint32_t w, uint32_t lo, uint32_t hi, uint64_t &h1,
                                              uint64_t &h2) {
#pragma unroll
    for (uint32_t j = 0; j < 4; ++j) {
        uint32_t b = (w >> (8 * j)) & 0xffu;
        uint64_t a1 = (h1 ^ (uint64_t)b) * kFnvPrime;
        uint64_t a2 = (h2 * kFnvPrime) ^ (uint64_t)b;
        bool on = (j >= lo) & (j < hi);
        h1 = on ? a1 : h1;
        h2 = on ? a2 : h2;
    }
}

// Key sources.  Each provides hash(i, h1, h2) for key i.
struct Keys16 {  // fixed 16-B keys, 16-B aligned: one dwordx4 per lane, 1 KiB per wave, coalesced
    const uint4 *p;
    __device__ __forceinline__ void hash(uint64_t i, uint64_t &h1, uint64_t &h2) const {
        uint4 v = p[i];
        h1 = kFnvOffset;
        h2 = kFnvOffset;
        fnv_word(v.x, h1, h2);
        fnv_word(v.y, h1, h2);
        fnv_word(v.z, h1, h2);
        fnv_word(v.w, h1, h2);
    }
};

struct KeysStrideW {  // fixed stride, multiple of 4 bytes, 4-B aligned
    const uint32_t *p;
    uint32_t words;
    __device__ __forceinline__ void hash(uint64_t i, uint64_t &h1, uint64_t &h2) const {
        const uint32_t *k = p + i * words;
        h1 = kFnvOffset;
        h2 = kFnvOffset;
        for (uint32_t j = 0; j < words; ++j) fnv_word(k[j], h1, h2);
    }
};

struct KeysStrideB {  // any fixed stride (including 0)
    const uint8_t *p;
    uint32_t stride;
    __device__ __forceinline__ void hash(uint64_t i, uint64_t &h1, uint64_t &h2) const {
        const uint8_t *k = p + i * stride;
        h1 = kFnvOffset;
        h2 = kFnvOffset;
        for (uint32_t j = 0; j < stride; ++j) fnv_byte(k[j], h1, h2);
    }
};

struct KeysVar {  // variable length: key i = p[off[i], off[i+1])
    const uint8_t *p;
    const uint64_t *off;
    __device__ __forceinline__ void hash(uint64_t i, uint64_t &h1, uint64_t &h2) const {
        uint64_t s = off[i], e = off[i + 1];
        h1 = kFnvOffset;
        h2 = kFnvOffset;
        // Walk the aligned dwords that cover [s, e).  A dword holding at least one byte of
        // the buffer never crosses a page, so the over-read at either end cannot fault.
        uintptr_t a = ((uintptr_t)(p + s)) & ~(uintptr_t)3;
        uintptr_t end = (uintptr_t)(p + e);
        uintptr_t beg = (uintptr_t)(p + s);
        for (; a < end; a += 4) {
            uint32_t w = *(const uint32_t *)a;
            uint32_t lo = beg > a ? (uint32_t)(beg - a) : 0u;
            uint32_t hi = end - a < 4 ? (uint32_t)(end - a) : 4u;
            if (lo == 0 && hi == 4)
                fnv_word(w, h1, h2);
            else
                fnv_word_part(w, lo, hi, h1, h2);
        }
    }
};

// --------------------------------------------------------------- positions -----------------

// Exact x mod m for any m >= 1 with mu = floor((2^64-1)/m): the estimate q is at most 2 low.
__device__ __forceinline__ uint64_t mod64(uint64_t x, uint64_t m, uint64_t mu) {
    uint64_t q = __umul64hi(x, mu);
    uint64_t r = x - q * m;
    r = r >= m ? r - m : r;
    r = r >= m ? r - m : r;
    return r;
}

// Calls f(i, pos_i) for i < k with pos_i = (h1 + i*h2 mod 2^64) mod m, bit-exact with
// lsm/bloom.go:64.  Residues advance incrementally: r_{i+1} = r_i + (h2 mod m), minus
// (2^64 mod m) whenever the u64 sum h1 + (i+1)*h2 wraps.  M32: m < 2^32 -> u32 residues.
template <int KFIX, bool M32, typename F>
__device__ __forceinline__ void for_positions(uint64_t h1, uint64_t h2, const ModArg &md, uint32_t krt, F &&f) {
    const uint32_t k = KFIX > 0 ? (uint32_t)KFIX : krt;
    if (k == 0) return;
    uint64_t x = h1;
    if constexpr (M32) {
        const uint32_t m = (uint32_t)md.m, c = (uint32_t)md.c;
        uint32_t r = (uint32_t)mod64(h1, md.m, md.mu);
        const uint32_t b = (uint32_t)mod64(h2, md.m, md.mu);
        f(0u, (uint64_t)r);
#pragma unroll
        for (uint32_t i = 1; i < k; ++i) {
            uint64_t xn = x + h2;
            bool carry = xn < x;
            x = xn;
            uint32_t s = r + b;
            s = (s < r || s >= m) ? s - m : s;
            uint32_t t = s >= c ? s - c : s + (m - c);
            r = carry ? t : s;
            f(i, (uint64_t)r);
        }
    } else {
        const uint64_t m = md.m, c = md.c;
        uint64_t r = mod64(h1, md.m, md.mu);
        const uint64_t b = mod64(h2, md.m, md.mu);
        f(0u, r);
#pragma unroll
        for (uint32_t i = 1; i < k; ++i) {
            uint64_t xn = x + h2;
            bool carry = xn < x;
            x = xn;
            uint64_t s = r + b;
            s = (s < r || s >= m) ? s - m : s;
            uint64_t t = s >= c ? s - c : s + (m - c);
            r = carry ? t : s;
            f(i, r);
        }
    }
}

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

// Probe: one thread per key, all k word gathers issued before the AND (the answer equals the
// reference's early-exit loop), 0/1 byte out.
template <typename Src, int KFIX, bool M32>
__global__ __launch_bounds__(256) void k_probe(Src src, uint64_t n, const uint32_t *__restrict__ words, ModArg md,
                                               uint8_t *__restrict__ out) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        uint64_t h1, h2;
        src.hash(i, h1, h2);
        uint32_t acc = 1u;
        for_positions<KFIX, M32>(h1, h2, md, md.k,
                                 [&](uint32_t, uint64_t p) { acc &= words[p >> 5] >> (uint32_t)(p & 31); });
        out[i] = (uint8_t)(acc & 1u);
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
                    for (int q = 0; q < KFIX; ++q) acc &= wd[pos[q] >> 5] >> (uint32_t)(pos[q] & 31);
                    w |= (MaskT)(acc & 1u) << f;
                }
            }
        } else {
            for (uint32_t f = 0; f < ma.nf; ++f) {
                const uint32_t *wd = ma.f[f].words;
                uint32_t acc = 1u;
                for_positions<KFIX, M32>(h1, h2, ma.f[f].md, ma.f[f].md.k,
                                         [&](uint32_t, uint64_t p) { acc &= wd[p >> 5] >> (uint32_t)(p & 31); });
                w |= (MaskT)(acc & 1u) << f;
            }
        }
        mask[i] = w;
    }
}

// Batched build of independent small filters: one workgroup per filter, the whole filter held
// in LDS (ds_or_b32 atomics, no global atomics), then OR-merged into HBM with coalesced
// accesses.  Filters too large for LDS go through k_build.
template <typename Src, int KFIX, bool M32>
__global__ __launch_bounds__(1024) void k_build_many_lds(Src src, ManyArg ma) {
    extern __shared__ uint32_t lds[];
    const ManyFilter &F = ma.f[blockIdx.x];
    const uint32_t nw = (uint32_t)F.nwords;
    for (uint32_t j = threadIdx.x; j < nw; j += blockDim.x) lds[j] = 0u;
    __syncthreads();
    for (uint64_t i = F.key_begin + threadIdx.x; i < F.key_end; i += blockDim.x) {
        uint64_t h1, h2;
        src.hash(i, h1, h2);
        for_positions<KFIX, M32>(h1, h2, F.md, F.md.k, [&](uint32_t, uint64_t p) {
            __hip_atomic_fetch_or(lds + (p >> 5), 1u << (uint32_t)(p & 31), __ATOMIC_RELAXED,
                                  __HIP_MEMORY_SCOPE_WORKGROUP);
        });
    }
    __syncthreads();
    for (uint32_t j = threadIdx.x; j < nw; j += blockDim.x) {
        uint32_t v = lds[j];
        if (v) F.words[j] |= v;
    }
}

// ------------------------------------------------------------------ launchers ----------------

static inline unsigned grid_for(uint64_t n, unsigned block, unsigned cap) {
    uint64_t g = (n + block - 1) / block;
    if (g < 1) g = 1;
    return (unsigned)(g > cap ? cap : g);
}

static unsigned g_grid_cap = 1u << 20;  // launch one thread per key by default
void set_grid_cap(unsigned cap) { g_grid_cap = cap ? cap : (1u << 20); }

template <typename Src, int KFIX, bool M32>
static hipError_t launch_build_t(const Src &src, uint64_t n, uint32_t *words, const ModArg &md, hipStream_t s) {
    unsigned g = grid_for(n, 256, g_grid_cap);
    hipLaunchKernelGGL((k_build<Src, KFIX, M32>), dim3(g), dim3(256), 0, s, src, n, words, md);
    return hipGetLastError();
}

template <typename Src, int KFIX, bool M32>
static hipError_t launch_probe_t(const Src &src, uint64_t n, const uint32_t *words, const ModArg &md, uint8_t *out,
                                 hipStream_t s) {
    unsigned g = grid_for(n, 256, g_grid_cap);
    hipLaunchKernelGGL((k_probe<Src, KFIX, M32>), dim3(g), dim3(256), 0, s, src, n, words, md, out);
    return hipGetLastError();
}

template <typename Src, typename MaskT, bool SAME, int KFIX, bool M32>
static hipError_t launch_multi_t(const Src &src, uint64_t n, const MultiArg &ma, void *mask, hipStream_t s) {
    unsigned g = grid_for(n, 256, g_grid_cap);
    hipLaunchKernelGGL((k_probe_multi<Src, MaskT, SAME, KFIX, M32>), dim3(g), dim3(256), 0, s, src, n, ma,
                       (MaskT *)mask);
    return hipGetLastError();
}

// Dispatch on the key source.  Fixed 16-B aligned keys take the vector path.
template <typename Fn>
static hipError_t with_src(const KeyBatch &kb, Fn &&fn) {
    if (kb.offsets) return fn(KeysVar{kb.data, kb.offsets});
    if (kb.stride == 16 && ((uintptr_t)kb.data & 15) == 0) return fn(Keys16{(const uint4 *)kb.data});
    if (kb.stride % 4 == 0 && ((uintptr_t)kb.data & 3) == 0)
        return fn(KeysStrideW{(const uint32_t *)kb.data, kb.stride / 4});
    return fn(KeysStrideB{kb.data, kb.stride});
}

hipError_t launch_build(const KeyBatch &kb, uint32_t *words, const ModArg &md, hipStream_t s) {
    if (kb.n == 0 || md.k == 0) return hipSuccess;
    const bool m32 = md.m <= 0xffffffffull;
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
    const bool m32 = md.m <= 0xffffffffull;
    const bool k7 = md.k == 7;
    return with_src(kb, [&](auto src) {
        using S = decltype(src);
        if (m32) return k7 ? launch_probe_t<S, 7, true>(src, kb.n, words, md, out, s) : launch_probe_t<S, 0, true>(src, kb.n, words, md, out, s);
        return k7 ? launch_probe_t<S, 7, false>(src, kb.n, words, md, out, s) : launch_probe_t<S, 0, false>(src, kb.n, words, md, out, s);
    });
}

template <typename MaskT>
static hipError_t multi_mask(const KeyBatch &kb, const MultiArg &ma, void *mask, hipStream_t s) {
    bool same = true, m32 = true;
    for (uint32_t f = 0; f < ma.nf; ++f) {
        same &= ma.f[f].md.m == ma.f[0].md.m && ma.f[f].md.k == ma.f[0].md.k;
        m32 &= ma.f[f].md.m <= 0xffffffffull;
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
        m32 &= ma.f[f].md.m <= 0xffffffffull;
        k7 &= ma.f[f].md.k == 7;
    }
    return with_src(kb, [&](auto src) {
        using S = decltype(src);
        auto go = [&](auto kern) {
            hipError_t e = hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_bytes);
            if (e != hipSuccess) return e;
            hipLaunchKernelGGL(kern, dim3(ma.nf), dim3(1024), lds_bytes, s, src, ma);
            return hipGetLastError();
        };
        if (m32) return k7 ? go(k_build_many_lds<S, 7, true>) : go(k_build_many_lds<S, 0, true>);
        return k7 ? go(k_build_many_lds<S, 7, false>) : go(k_build_many_lds<S, 0, false>);
    });
}

}  // namespace seb
