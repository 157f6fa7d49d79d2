// seb_device.h — device-side building blocks shared by every gfx950 kernel of the path:
// FNV-1a / FNV-1 over the key bytes (lsm/bloom.go:44-54), the key sources (fixed 16 B,
// fixed stride, variable length) and the exact position generator (lsm/bloom.go:58-67).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

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
// 435^e mod 2^32 (the low part of the FNV prime 2^40 + 435)
__host__ __device__ constexpr uint32_t pow435(int e) {
    uint32_t r = 1;
    for (int i = 0; i < e; ++i) r *= 435u;
    return r;
}

// acc + a * b as one v_mad_u64_u32 (only the low 32 bits of the result are used; the compiler
// narrows such a mad into v_mul_lo_u32 + v_add3_u32, two instructions)
__device__ __forceinline__ uint64_t mad_lo(uint32_t a, uint32_t b, uint64_t acc) {
    uint64_t r;
    asm("v_mad_u64_u32 %0, vcc, %1, %2, %3" : "=v"(r) : "v"(a), "s"(b), "v"(acc) : "vcc");
    return r;
}

// a ^ (byte b of w), as ONE v_xor_b32 whose SDWA source select picks the byte (b is a constant
// once the byte loops are unrolled, and the switch folds away).  Left to itself the compiler
// shifts bytes 1 and 2 down first (v_lshrrev / v_bfe, then a v_bitop3 that masks and xors): one
// extra instruction per byte, ≈22 of the ≈150 that both chains of a 16-B key cost.
__device__ __forceinline__ uint32_t xor_byte(uint32_t a, uint32_t w, int b) {
    uint32_t r;
    switch (b) {
        case 0:
            asm("v_xor_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_0 src1_sel:DWORD"
                : "=v"(r) : "v"(w), "v"(a));
            break;
        case 1:
            asm("v_xor_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_1 src1_sel:DWORD"
                : "=v"(r) : "v"(w), "v"(a));
            break;
        case 2:
            asm("v_xor_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_2 src1_sel:DWORD"
                : "=v"(r) : "v"(w), "v"(a));
            break;
        default:
            asm("v_xor_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_3 src1_sel:DWORD"
                : "=v"(r) : "v"(w), "v"(a));
            break;
    }
    return r;
}

// Both FNV chains over a 16-byte key.  Multiplying by P = 2^40 + 435 leaves the low word
// lo' = low32(lo * 435) independent of the high word, so the low word runs the byte chain alone
// (one v_mad_u64_u32 gives lo' and the carry c) and the high word, which is linear:
//   hi' = 435 * hi + d,  d = c + (lo << 8)
// is summed after the fact as hi_16 = 435^16 hi_0 + sum_j d_j 435^(15-j) with constant weights,
// one mad per byte off the critical path: 18% less VALU time than the plain 64-bit multiply
// chain (tools/ubench/fnv.hip, profiles/r01_ubench_fnv.jsonl), the same bits.
__device__ __forceinline__ void fnv_key16(const uint4 v, uint64_t &h1, uint64_t &h2) {
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
    uint32_t lo1 = (uint32_t)kFnvOffset, lo2 = (uint32_t)kFnvOffset;
    uint64_t acc1 = (uint32_t)(kFnvOffset >> 32) * pow435(16), acc2 = acc1;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        const uint32_t x = xor_byte(lo1, w[j >> 2], j & 3);  // FNV-1a (hash1): xor, then multiply
        const uint64_t p = (uint64_t)x * 435u;
        lo1 = (uint32_t)p;
        acc1 = mad_lo((uint32_t)(p >> 32) + (x << 8), pow435(15 - j), acc1);
        const uint64_t q = (uint64_t)lo2 * 435u;  // FNV-1 (hash2): multiply, then xor
        acc2 = mad_lo((uint32_t)(q >> 32) + (lo2 << 8), pow435(15 - j), acc2);
        lo2 = xor_byte((uint32_t)q, w[j >> 2], j & 3);
    }
    h1 = (acc1 << 32) | lo1;
    h2 = (acc2 << 32) | lo2;
}

// Both chains in the split form of fnv_key16, for walks of unknown length: the high words are
// kept as u64 accumulators whose low 32 bits are the hash's high word, and each 4-byte word
// folds its four d_j into them with constant weights (3 mads), then one mad scales the old value
// by 435^4: 17 VALU instructions per word and hash instead of 20.
struct FnvSplit {
    uint32_t lo1 = (uint32_t)kFnvOffset, lo2 = (uint32_t)kFnvOffset;
    uint64_t a1 = kFnvOffset >> 32, a2 = kFnvOffset >> 32;
    __device__ __forceinline__ void word(uint32_t w) {
        uint32_t d1[4], d2[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t x = xor_byte(lo1, w, j);  // FNV-1a
            const uint64_t p = (uint64_t)x * 435u;
            lo1 = (uint32_t)p;
            d1[j] = (uint32_t)(p >> 32) + (x << 8);
            const uint64_t q = (uint64_t)lo2 * 435u;  // FNV-1
            d2[j] = (uint32_t)(q >> 32) + (lo2 << 8);
            lo2 = xor_byte((uint32_t)q, w, j);
        }
        const uint64_t t1 = mad_lo(d1[0], pow435(3), mad_lo(d1[1], pow435(2), mad_lo(d1[2], 435u, d1[3])));
        const uint64_t t2 = mad_lo(d2[0], pow435(3), mad_lo(d2[1], pow435(2), mad_lo(d2[2], 435u, d2[3])));
        a1 = mad_lo((uint32_t)a1, pow435(4), t1);
        a2 = mad_lo((uint32_t)a2, pow435(4), t2);
    }
    __device__ __forceinline__ void get(uint64_t &h1, uint64_t &h2) const {
        h1 = (a1 << 32) | lo1;
        h2 = (a2 << 32) | lo2;
    }
};

// Sources with kSplit = true also expose load(i) -> uint4 and hash_raw(raw, h1, h2), so a kernel
// can issue the loads of its next batch of keys before it hashes them (software prefetch).
// Fixed 16-B keys, 16-B aligned: one dwordx4 per lane, 1 KiB per wave, coalesced; non-temporal, so
// the streamed batch does not evict filter lines from L2 (+2% over plain loads).
struct Keys16 {
    static constexpr bool kSplit = true;
    const uint4 *p;
    __device__ __forceinline__ uint64_t index(uint64_t i) const { return i; }
    __device__ __forceinline__ uint4 load(uint64_t i) const {
        typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
        const u32x4 v = __builtin_nontemporal_load((const u32x4 *)(p + i));
        return make_uint4(v.x, v.y, v.z, v.w);
    }
    __device__ __forceinline__ static void hash_raw(const uint4 v, uint64_t &h1, uint64_t &h2) { fnv_key16(v, h1, h2); }
    __device__ __forceinline__ void hash(uint64_t i, uint64_t &h1, uint64_t &h2) const { fnv_key16(load(i), h1, h2); }
};

struct KeysStrideW {  // fixed stride, multiple of 4 bytes, 4-B aligned
    const uint32_t *p;
    uint32_t words;
    __device__ __forceinline__ uint64_t index(uint64_t i) const { return i; }
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
    __device__ __forceinline__ uint64_t index(uint64_t i) const { return i; }
    __device__ __forceinline__ void hash(uint64_t i, uint64_t &h1, uint64_t &h2) const {
        const uint8_t *k = p + i * stride;
        h1 = kFnvOffset;
        h2 = kFnvOffset;
        for (uint32_t j = 0; j < stride; ++j) fnv_byte(k[j], h1, h2);
    }
};

// Hash bytes [s, e) of a packed buffer: walk the aligned dwords that cover them.  A dword holding
// at least one byte of the buffer never crosses a page, so the over-read at either end cannot fault.
__device__ __forceinline__ void fnv_range(const uint8_t *p, uint64_t s, uint64_t e, uint64_t &h1, uint64_t &h2) {
    h1 = kFnvOffset;
    h2 = kFnvOffset;
    uintptr_t a = ((uintptr_t)(p + s)) & ~(uintptr_t)3;
    const uintptr_t end = (uintptr_t)(p + e);
    const uintptr_t beg = (uintptr_t)(p + s);
    for (; a < end; a += 4) {
        const uint32_t w = *(const uint32_t *)a;
        const uint32_t lo = beg > a ? (uint32_t)(beg - a) : 0u;
        const uint32_t hi = end - a < 4 ? (uint32_t)(end - a) : 4u;
        if (lo == 0 && hi == 4)
            fnv_word(w, h1, h2);
        else
            fnv_word_part(w, lo, hi, h1, h2);
    }
}

struct KeysVar {  // variable length: key i = p[off[i], off[i+1])
    const uint8_t *p;
    const uint64_t *off;
    __device__ __forceinline__ uint64_t index(uint64_t i) const { return i; }
    __device__ __forceinline__ void hash(uint64_t i, uint64_t &h1, uint64_t &h2) const {
        fnv_range(p, off[i], off[i + 1], h1, h2);
    }
};

struct KeysHashed {  // pre-hashed batch (k_hash_varlen): one coalesced 16-B load per key
    static constexpr bool kSplit = true;
    const uint4 *h;
    __device__ __forceinline__ uint64_t index(uint64_t i) const { return i; }
    __device__ __forceinline__ uint4 load(uint64_t i) const { return h[i]; }
    __device__ __forceinline__ static void hash_raw(const uint4 v, uint64_t &h1, uint64_t &h2) {
        h1 = (uint64_t)v.x | ((uint64_t)v.y << 32);
        h2 = (uint64_t)v.z | ((uint64_t)v.w << 32);
    }
    __device__ __forceinline__ void hash(uint64_t i, uint64_t &h1, uint64_t &h2) const { hash_raw(h[i], h1, h2); }
};

template <typename S, typename = void>
struct SplitLoad { static constexpr bool value = false; };
template <typename S>
struct SplitLoad<S, std::void_t<decltype(S::kSplit)>> { static constexpr bool value = S::kSplit; };

// --------------------------------------------------------------- positions -----------------

// Exact x mod m for any m >= 1 with mu = floor((2^64-1)/m): the estimate q is at most 2 low.
__device__ __forceinline__ uint64_t mod64(uint64_t x, uint64_t m, uint64_t mu) {
    uint64_t q = __umul64hi(x, mu);
    uint64_t r = x - q * m;
    r = r >= m ? r - m : r;
    r = r >= m ? r - m : r;
    return r;
}

// x mod m for m < kM32Limit (2^31).  With mu = floor((2^64-1)/m) the Barrett quotient
// q = floor(x*mu / 2^64) is at most one below floor(x/m) (mu*m > 2^64 - m), so r = x - q*m lies in
// [0, 2m) and fits 32 bits: only q's low word is needed, and r = low32(x) - low32(q)*m exactly.
// q's low word from three 32x32 products (the full 64x64 high product, low word kept), then
// one conditional subtract as min(r, r - m): 9 VALU instructions instead of mod64's ~26.
__device__ __forceinline__ uint32_t mod_m31(uint64_t x, uint32_t m, uint64_t mu) {
    const uint32_t xl = (uint32_t)x, xh = (uint32_t)(x >> 32);
    const uint32_t ul = (uint32_t)mu, uh = (uint32_t)(mu >> 32);
    const uint64_t a = (uint64_t)xh * ul + __umulhi(xl, ul);  // < 2^64
    const uint64_t b = (uint64_t)xl * uh + (uint32_t)a;       // < 2^64
    const uint32_t qlo = xh * uh + (uint32_t)(a >> 32) + (uint32_t)(b >> 32);
    const uint32_t r = xl - qlo * m;
    const uint32_t s = r - m;  // wraps past r exactly when r < m
    return s < r ? s : r;
}

// Calls f(i, pos_i) for i < k with pos_i = (h1 + i*h2 mod 2^64) mod m, bit-exact with
// lsm/bloom.go:64.  Residues advance incrementally: r_{i+1} = r_i + (h2 mod m), minus
// (2^64 mod m) whenever the u64 sum h1 + (i+1)*h2 wraps.  M32: m < kM32Limit -> u32 residues.
template <int KFIX, bool M32, typename F>
__device__ __forceinline__ void for_positions(uint64_t h1, uint64_t h2, const ModArg &md, uint32_t krt, F &&f) {
    const uint32_t k = KFIX > 0 ? (uint32_t)KFIX : krt;
    if (k == 0) return;
    uint64_t x = h1;
    if constexpr (M32) {
        const uint32_t m = (uint32_t)md.m, c = (uint32_t)md.c;
        uint32_t r = mod_m31(h1, m, md.mu);
        const uint32_t b = mod_m31(h2, m, md.mu);
        // Step addend: b, or (b - c) mod m when the u64 sum wraps.  Kept negated (m - a, in
        // [1, m]) so r + a mod m is one subtract, one compare and a conditional add of m, with
        // no u32 overflow for any m < 2^31.
        const uint32_t nb = m - b;
        const uint32_t bc = b >= c ? b - c : b + (m - c);
        const uint32_t nd = m - bc;
        f(0u, (uint64_t)r);
#pragma unroll
        for (uint32_t i = 1; i < k; ++i) {
            uint64_t xn = x + h2;
            const bool carry = xn < x;
            x = xn;
            const uint32_t na = carry ? nd : nb;
            const uint32_t t = r - na;
            r = r >= na ? t : t + m;
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

// Dispatch on the key source.  Fixed 16-B aligned keys take the vector path.
template <typename Fn>
static inline hipError_t with_src(const KeyBatch &kb, Fn &&fn) {
    if (kb.hashes) return fn(KeysHashed{kb.hashes});
    if (kb.offsets) return fn(KeysVar{kb.data, kb.offsets});
    if (kb.stride == 16 && ((uintptr_t)kb.data & 15) == 0) return fn(Keys16{(const uint4 *)kb.data});
    if (kb.stride % 4 == 0 && ((uintptr_t)kb.data & 3) == 0)
        return fn(KeysStrideW{(const uint32_t *)kb.data, kb.stride / 4});
    return fn(KeysStrideB{kb.data, kb.stride});
}

// ---- packed residues (k == 7, m < 2^kPackBits): bits 0-28 r0 = h1 mod m, 29-57 b = h2 mod m,
// 58-63 bit q-1 = "the u64 sum h1 + q*h2 wrapped at step q" for q = 1..6.  The positions follow
// for_positions' recurrence, so they are exactly (h1 + q*h2 mod 2^64) mod m of lsm/bloom.go:64.
__device__ __forceinline__ uint64_t pack_residue(uint64_t h1, uint64_t h2, const ModArg &md) {
    const uint64_t r0 = mod_m31(h1, (uint32_t)md.m, md.mu), b = mod_m31(h2, (uint32_t)md.m, md.mu);
    uint64_t f = 0, x = h1;
#pragma unroll
    for (uint32_t q = 1; q < 7; ++q) {
        const uint64_t xn = x + h2;
        f |= (uint64_t)(xn < x) << (q - 1);
        x = xn;
    }
    return r0 | (b << kPackBits) | (f << (2 * kPackBits));
}

// The 7 positions of packed word v (m, c = 2^64 mod m as u32: m < 2^29).
__device__ __forceinline__ void packed_positions(uint64_t v, uint32_t m, uint32_t c, uint32_t pos[7]) {
    constexpr uint64_t kMask = (1ull << kPackBits) - 1;
    uint32_t x = (uint32_t)(v & kMask);
    const uint32_t b = (uint32_t)((v >> kPackBits) & kMask), f = (uint32_t)(v >> (2 * kPackBits));
    const uint32_t nb = m - b, bc = b >= c ? b - c : b + (m - c), nd = m - bc;
    pos[0] = x;
#pragma unroll
    for (int q = 1; q < 7; ++q) {
        const uint32_t na = (f >> (q - 1)) & 1u ? nd : nb;
        const uint32_t t = x - na;
        x = x >= na ? t : t + m;
        pos[q] = x;
    }
}

// The narrow form (m < 2^kPack6Bits): the same fields at 21 / 21 / 6 bits, 48 bits per key, in
// blocks of 64 keys: low words at u32 index 96 * block + lane, high halves at u16 index
// 192 * block + 128 + lane (seb_kernels.h kPack6Block).
__device__ __forceinline__ uint64_t pack_residue6(uint64_t h1, uint64_t h2, const ModArg &md) {
    const uint64_t r0 = mod_m31(h1, (uint32_t)md.m, md.mu), b = mod_m31(h2, (uint32_t)md.m, md.mu);
    uint64_t f = 0, x = h1;
#pragma unroll
    for (uint32_t q = 1; q < 7; ++q) {
        const uint64_t xn = x + h2;
        f |= (uint64_t)(xn < x) << (q - 1);
        x = xn;
    }
    return r0 | (b << kPack6Bits) | (f << (2 * kPack6Bits));
}
__device__ __forceinline__ void store_packed6(uint8_t *base, uint64_t i, uint64_t v) {
    const uint64_t blk = i >> 6;
    const uint32_t lane = (uint32_t)i & 63u;
    __builtin_nontemporal_store((uint32_t)v, (uint32_t *)(base + blk * kPack6Block) + lane);
    __builtin_nontemporal_store((uint16_t)(v >> 32), (uint16_t *)(base + blk * kPack6Block + 256) + lane);
}
__device__ __forceinline__ uint64_t load_packed6(const uint8_t *base, uint64_t i) {
    const uint64_t blk = i >> 6;
    const uint32_t lane = (uint32_t)i & 63u;
    const uint32_t lo = __builtin_nontemporal_load((const uint32_t *)(base + blk * kPack6Block) + lane);
    const uint16_t hi = __builtin_nontemporal_load((const uint16_t *)(base + blk * kPack6Block + 256) + lane);
    return (uint64_t)lo | ((uint64_t)hi << 32);
}

// A batch given as packed residues (the variable-length pre-hash writes these when the filter
// allows): load(i) carries the 8-byte word in .x/.y; kernels take the positions from it directly.
struct KeysPacked {
    static constexpr bool kSplit = true;
    static constexpr bool kPacked = true;
    const uint64_t *p;
    __device__ __forceinline__ uint64_t index(uint64_t i) const { return i; }
    __device__ __forceinline__ uint4 load(uint64_t i) const {
        const uint64_t v = __builtin_nontemporal_load(p + i);
        return make_uint4((uint32_t)v, (uint32_t)(v >> 32), 0u, 0u);
    }
};

template <typename S, typename = void>
struct IsPacked { static constexpr bool value = false; };
template <typename S>
struct IsPacked<S, std::void_t<decltype(S::kPacked)>> { static constexpr bool value = S::kPacked; };

// Lanes of this wave holding the same `bits`-bit value v as this lane (live lanes only): one ballot
// per bit, so lanes can share one LDS atomic per distinct value instead of one per lane.
__device__ __forceinline__ uint64_t wave_peers(bool live, uint32_t v, uint32_t bits) {
    uint64_t peers = __ballot(live);
    for (uint32_t b = 0; b < bits; ++b) {
        const uint64_t on = __ballot(live && ((v >> b) & 1u));
        peers &= ((v >> b) & 1u) ? on : ~on;
    }
    return peers;
}

// Number of lanes of `mask` below this lane.
__device__ __forceinline__ uint32_t lanes_below(uint64_t mask) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}

}  // namespace seb
