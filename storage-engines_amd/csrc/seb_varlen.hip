// seb_varlen.hip — LDS-staged pre-hash of variable-length keys (BASELINE C4).
//
// The reference hashes each key with a byte-serial FNV chain (lsm/bloom.go:44-54), so a lane's
// work is its key's length.  In a wave of 64 keys drawn from the C4 zipf lengths (8-256 B, mean
// 40 B) almost every wave holds one long key, and the whole wave waits for it.  Batches of >= 64K
// variable-length keys are therefore hashed first, here, with each workgroup sorting its own keys
// by length in LDS; build and probe then read 16 (or 8, packed) bytes per key.  Order never changes
// a result: every key's hashes land at its own index.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "seb_device.h"
#include "seb_kernels.h"

namespace seb {

constexpr uint32_t kLenBuckets = 65;  // ceil(len/4) in [0, 64]; longer keys share bucket 64

// ---- pre-hash: (h1, h2) of every variable-length key, written as one uint4 per key.
// A workgroup owns kHashKeys consecutive keys.  It copies their byte span (16-B aligned chunks,
// coalesced dwordx4 loads) into LDS, counting-sorts its keys by dword length in LDS, and lane t
// then hashes the t-th shortest key from LDS: a wave's lanes walk keys of about one length
// (divergence would otherwise make every wave as slow as its longest key), and each dependent
// read is an LDS access instead of an L2/fabric round trip.  A span larger than the LDS window
// is hashed straight from HBM in input order.  Build and probe then read 16 B per key
// (KeysHashed), exactly like the fixed 16-B path.
// Funnel walk of one key staged in LDS: every 4 key bytes come from two aligned LDS dwords
// (v_alignbyte), so all full words take the same path whatever the key's alignment.  The dword
// after next is read one step ahead, so a step's LDS latency overlaps the previous word's hashing
// (it reads no further than finish() reads: one dword past the key).
struct Funnel {
    uint32_t wi, cur, nxt, sh, len;
    FnvSplit f;
    __device__ __forceinline__ void init(const uint32_t *lds, uint32_t b, uint32_t n) {
        wi = b >> 2;
        sh = b & 3u;
        len = n;
        cur = lds[wi];
        nxt = lds[wi + 1];
    }
    __device__ __forceinline__ void step(const uint32_t *lds) {  // the next 4 bytes
        const uint32_t ahead = lds[wi + 2];
        ++wi;
        f.word(__builtin_amdgcn_alignbyte(nxt, cur, sh));
        cur = nxt;
        nxt = ahead;
    }
    __device__ __forceinline__ void step2(const uint32_t *lds) {  // the next 8 bytes
        const uint32_t a1 = lds[wi + 2], a2 = lds[wi + 3];
        wi += 2;
        f.word(__builtin_amdgcn_alignbyte(nxt, cur, sh));
        f.word(__builtin_amdgcn_alignbyte(a1, nxt, sh));
        cur = a1;
        nxt = a2;
    }
    // every full word of the key, two per iteration (no register rotation, half the loop control)
    __device__ __forceinline__ void walk(const uint32_t *lds) {
        const uint32_t nw = len >> 2;
        for (uint32_t j = 0; j + 2 <= nw; j += 2) step2(lds);
        if (nw & 1u) step(lds);
    }
    // the last len % 4 bytes; returns the key's (h1, h2)
    __device__ __forceinline__ void finish(const uint32_t *, uint64_t &h1, uint64_t &h2) {
        f.get(h1, h2);
        const uint32_t r = len & 3u;
        if (r) fnv_word_part(__builtin_amdgcn_alignbyte(nxt, cur, sh), 0u, r, h1, h2);
    }
};

// One FNV chain in FnvSplit's form, for the tail waves of k_hash_varlen: FNV-1a's recurrence (xor the
// byte, then multiply) from state (lo, acc), the same bits as the matching half of FnvSplit.
struct FnvOne {
    uint32_t lo;
    uint64_t acc;
    __device__ __forceinline__ explicit FnvOne(uint64_t s) : lo((uint32_t)s), acc(s >> 32) {}
    __device__ __forceinline__ void word(uint32_t w) {
        uint32_t d[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t x = xor_byte(lo, w, j);
            const uint64_t p = (uint64_t)x * 435u;
            d[j] = (uint32_t)(p >> 32) + (x << 8);
            lo = (uint32_t)p;
        }
        const uint64_t t = mad_lo(d[0], pow435(3), mad_lo(d[1], pow435(2), mad_lo(d[2], 435u, d[3])));
        acc = mad_lo((uint32_t)acc, pow435(4), t);
    }
    // bytes [0, r) of w (r < 4) with the plain 64-bit step; returns the chain's state
    __device__ __forceinline__ uint64_t finish(uint32_t w, uint32_t r) const {
        uint64_t h = (acc << 32) | lo;
#pragma unroll
        for (uint32_t j = 0; j < 3; ++j) {
            const uint64_t nh = (h ^ ((w >> (8 * j)) & 0xffu)) * kFnvPrime;
            h = j < r ? nh : h;
        }
        return h;
    }
};

// One chain of a key staged in LDS at byte b, n bytes: FNV-1a (fnv1 false) or FNV-1 (true), both
// walked by FNV-1a's recurrence, so the lanes of one wave can run either with the same instructions.
// FNV-1 is s_j = s_{j-1} * P ^ b_{j-1} from s_0 = O; t_j = s_j * P then follows t_j = (t_{j-1} ^
// b_{j-1}) * P from t_0 = O * P, and s_n = t_{n-1} ^ b_{n-1}: FNV-1a's recurrence from O * P over the
// first n - 1 bytes, the last byte xored in after (an empty key keeps O).
__device__ __forceinline__ uint64_t funnel_chain(const uint32_t *lds, uint32_t b, uint32_t n, bool fnv1) {
    const bool shifted = fnv1 && n > 0;
    const uint32_t len = shifted ? n - 1 : n;
    uint32_t wi = b >> 2;
    const uint32_t sh = b & 3u;
    uint32_t cur = lds[wi], nxt = lds[wi + 1];
    FnvOne f(shifted ? kFnvOffset * kFnvPrime : kFnvOffset);
    const uint32_t nw = len >> 2;
    for (uint32_t j = 0; j + 2 <= nw; j += 2) {  // read ahead and two words per step, as Funnel::walk
        const uint32_t a1 = lds[wi + 2], a2 = lds[wi + 3];
        wi += 2;
        f.word(__builtin_amdgcn_alignbyte(nxt, cur, sh));
        f.word(__builtin_amdgcn_alignbyte(a1, nxt, sh));
        cur = a1;
        nxt = a2;
    }
    if (nw & 1u) {
        const uint32_t ahead = lds[wi + 2];
        f.word(__builtin_amdgcn_alignbyte(nxt, cur, sh));
        cur = nxt;
        nxt = ahead;
    }
    uint64_t h = f.finish(__builtin_amdgcn_alignbyte(nxt, cur, sh), len & 3u);
    if (shifted) {
        const uint32_t p = b + n - 1;
        h ^= (lds[p >> 2] >> (8 * (p & 3u))) & 0xffu;
    }
    return h;
}

// A workgroup owns KEYS consecutive keys and an LDS window of WIN bytes per key (C4 keys average
// 40 B).  It copies the keys' byte span into LDS, counting-sorts the keys by dword length so each
// wave walks keys of about one length, and lane t hashes sorted key t with the funnel walk.  The
// work per workgroup is short, so its time is mostly the chain of dependent memory round trips:
// each thread loads its own key's offsets up front (with the span bounds), then the span; the
// sorted slots carry (start, length, key) in LDS so the hash phase touches HBM only to store.
// Output: (h1, h2) as a uint4 per key, or with PACK the key's packed residues for filter md
// (8 B instead of 16; the build and the phased probe take positions straight from them).
template <bool PACK>
__device__ __forceinline__ void put_hash(void *out, uint64_t i, uint64_t h1, uint64_t h2, const ModArg &md) {
    if constexpr (PACK)
        ((uint64_t *)out)[i] = pack_residue(h1, h2, md);
    else
        ((uint4 *)out)[i] = make_uint4((uint32_t)h1, (uint32_t)(h1 >> 32), (uint32_t)h2, (uint32_t)(h2 >> 32));
}

// NS > 0 (KEYS = 512 - 64 * NS, 512 threads): a full workgroup's 64 * NS longest keys (the last
// slots of the length order, which otherwise set the workgroup's lifetime and hold its LDS after
// the other waves are done) are hashed by the last 2 * NS waves, 32 keys per wave, the longest 32
// on the first: lane l < 32 runs key l's FNV-1a chain and lane l + 32 its FNV-1 chain (funnel_chain:
// one instruction stream for both), so each runs half the instructions and a wave lasts as long as
// its own 32 keys' longest (round 4 paired the 64 keys' chains over two waves, each as long as the
// longest of all 64).  Lane l takes lane l + 32's hash by a lane shuffle for the packed output; the
// 16-B output is written in halves.
// P0 (with PACK): the compacted phased probe's phase 0 fused in (k_probe_c0's job for a pre-hashed
// batch): the packed words go to LDS in key order, then each wave takes one group of 64 keys,
// tests the positions in range 0 [0, p0.hi) and stores the live keys' words compacted in the
// group's row and the group's {mask0, live} record, so the dense packed batch never reaches HBM.
struct Phase0Arg {
    const uint32_t *words;
    uint64_t *rows;
    ulonglong2 *recs;
    uint32_t hi;
};

// Every thread of the workgroup arrives here (has: it hashed key k0 + my_j); the packed words go to
// xpk (the staging window), then waves 0 .. KEYS/64 - 1 each take the group of keys
// k0 + 64 * wave + lane (k0 is a multiple of 64).
template <uint32_t KEYS>
__device__ __forceinline__ void varlen_phase0(uint64_t *xpk, bool has, uint32_t my_j, uint64_t my_pw, uint64_t k0,
                                              uint32_t cnt, const ModArg &md, const Phase0Arg &p0) {
    __syncthreads();  // every key is hashed: the staging window is free
    if (has) xpk[my_j] = my_pw;
    __syncthreads();  // every key's packed word is in xpk, in key order
    const uint32_t wid = threadIdx.x >> 6, lane = threadIdx.x & 63u;
    if (wid >= KEYS / 64 || 64 * wid >= cnt) return;  // wave-uniform; no barrier follows
    const uint32_t j = 64 * wid + lane;
    const bool valid = j < cnt;
    const uint64_t pw = valid ? xpk[j] : 0ull;
    uint32_t pos[7];
    packed_positions(pw, (uint32_t)md.m, (uint32_t)md.c, pos);
    uint32_t acc = valid ? 1u : 0u;
#pragma unroll
    for (int q = 0; q < 7; ++q) {
        const uint32_t w = pos[q] >> 5;
        if ((acc & 1u) && w < p0.hi) acc &= p0.words[w] >> (pos[q] & 31);
    }
    const uint64_t alive = __ballot(acc & 1u);
    const uint64_t g = (k0 >> 6) + wid;
    if (acc & 1u) __builtin_nontemporal_store(pw, p0.rows + g * 64 + lanes_below(alive));
    if (lane == 0) p0.recs[g] = make_ulonglong2(alive, alive);
}

template <uint32_t KEYS, uint32_t WIN, bool PACK, uint32_t NS = 0, bool P0 = false>
__global__ __launch_bounds__(KEYS + 64 * NS) void k_hash_varlen(const uint8_t *__restrict__ data,
                                                      const uint64_t *__restrict__ off, uint64_t n,
                                                      void *__restrict__ hashes, ModArg md, Phase0Arg p0) {
    constexpr uint32_t kHashLds = KEYS * WIN;
    static_assert(kHashLds % 16 == 0 && kHashLds + 16 < 65536, "window offsets are 16-bit");
    static_assert(!P0 || (PACK && KEYS % 64 == 0 && KEYS * 8 <= kHashLds), "phase 0: whole groups of 64 keys, words in the window");
    __shared__ uint4 stage[kHashLds / 16 + 1];  // +16 B: the funnel walk reads one dword past a key
    __shared__ uint32_t cur[kLenBuckets];
    __shared__ uint32_t slot_key[KEYS];  // sorted slot -> start byte in the window << 16 | length
    __shared__ uint16_t slot_idx[KEYS];  // sorted slot -> key within the workgroup
    const uint32_t t = threadIdx.x;
    const uint64_t k0 = (uint64_t)blockIdx.x * KEYS;
    const uint64_t k1 = k0 + KEYS < n ? k0 + KEYS : n;
    const uint32_t cnt = (uint32_t)(k1 - k0);
    const bool mine = t < cnt;
    // P0: a thread keeps its key's packed word until every key is hashed, then the words go to the
    // (by then unused) staging window in key order: no LDS of its own, so 5 workgroups still fit a CU
    uint32_t my_j = 0;
    uint64_t my_pw = 0;
    bool has = false;
    auto emit = [&](uint32_t j, uint64_t h1, uint64_t h2) {  // key k0 + j
        if constexpr (P0) {
            my_j = j;
            my_pw = pack_residue(h1, h2, md);
            has = true;
        } else {
            put_hash<PACK>(hashes, k0 + j, h1, h2, md);
        }
    };
    const uint64_t ks = mine ? off[k0 + t] : 0, ke = mine ? off[k0 + t + 1] : 0;
    const uintptr_t s0 = (uintptr_t)(data + off[k0]);
    const uintptr_t s1 = (uintptr_t)(data + off[k1]);
    const uintptr_t base = s0 & ~(uintptr_t)15;
    const uint64_t chunks = (s1 - base + 15) >> 4;
    if (chunks * 16 > kHashLds) {  // block-uniform: a span larger than the window, straight from HBM
        if (mine) {
            uint64_t h1, h2;
            fnv_range(data, ks, ke, h1, h2);
            emit(t, h1, h2);
        }
        if constexpr (P0)
            varlen_phase0<KEYS>((uint64_t *)stage, has, my_j, my_pw, k0, cnt, md, p0);
        return;
    }
    if (t < kLenBuckets) cur[t] = 0u;
    {  // the span, 4 chunks per thread per batch: every load issued before any LDS store (a load-store
       // pair per chunk waited for every load), through a pointer that keeps the kernel argument's
       // global address space (a uintptr_t round trip made these flat loads); clamped chunk indices
       // repeat the last chunk (the same bytes to the same place), so no branch sinks a load
        const uint4 *src = (const uint4 *)(data + (off[k0] - (s0 & 15)));
        const uint32_t nc = (uint32_t)chunks;
        for (uint32_t c0 = t; c0 < nc; c0 += 4 * blockDim.x) {
            uint4 v[4];
#pragma unroll
            for (uint32_t r = 0; r < 4; ++r) v[r] = src[min(c0 + r * blockDim.x, nc - 1)];
#pragma unroll
            for (uint32_t r = 0; r < 4; ++r) stage[min(c0 + r * blockDim.x, nc - 1)] = v[r];
        }
    }
    const uint32_t len = (uint32_t)(ke - ks);
    const uint32_t dw = (len + 3) >> 2;
    const uint32_t bk = dw > 64 ? 64u : dw;
    // a wave whose keys all fall in one length bucket (uniform-length batches) takes its slots with
    // one LDS atomic instead of 64 serialised on one counter; mixed waves (C4's zipf lengths) stay
    // per lane, where full peer grouping (7 ballots) cost more than the contention it saved
    const uint64_t live = __ballot(mine);
    const uint64_t same = __ballot(mine && bk == __builtin_amdgcn_readfirstlane(bk));
    const uint64_t peers = same == live ? live : 1ull << (t & 63);
    const uint32_t below = lanes_below(peers);
    const bool leader = mine && below == 0;
    __syncthreads();
    if (leader) atomicAdd(&cur[bk], (uint32_t)__popcll(peers));
    __syncthreads();
    if (t < 64) {  // exclusive scan of the 65 bucket counts by one wave
        uint32_t c = cur[t] + (t == 63 ? cur[64] : 0u);
        uint32_t v = c;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            uint32_t y = __shfl_up(v, d, 64);
            if (t >= (uint32_t)d) v += y;
        }
        const uint32_t last63 = cur[63];
        cur[t] = v - c;
        if (t == 63) cur[64] = v - c + last63;
    }
    __syncthreads();
    uint32_t q = leader ? atomicAdd(&cur[bk], (uint32_t)__popcll(peers)) : 0u;
    q = __shfl(q, mine ? __ffsll((unsigned long long)peers) - 1 : (int)(t & 63), 64) + below;
    if (mine) {
        slot_key[q] = (uint32_t)((uintptr_t)(data + ks) - base) << 16 | len;
        slot_idx[q] = (uint16_t)t;
    }
    __syncthreads();
    const uint32_t *lds = (const uint32_t *)stage;
    bool tail = false;
    if constexpr (NS > 0) {
        if (cnt == KEYS && t >= KEYS - 64 * NS) {  // the longest keys: 32 per wave, a lane per chain
            tail = true;
            const uint32_t w = (t - (KEYS - 64 * NS)) >> 6, lane = t & 63, half = lane >> 5;
            const uint32_t q = KEYS - 32 * (w + 1) + (lane & 31);  // wave 0: the longest 32 slots
            const uint32_t sk = slot_key[q];
            const uint32_t j = slot_idx[q];
            const uint64_t h = funnel_chain(lds, sk >> 16, sk & 0xffffu, half != 0);
            // lane l < 32 (FNV-1a, hash1) takes lane l + 32's FNV-1 (hash2)
            const uint32_t h2lo = (uint32_t)__shfl((int)(uint32_t)h, (int)(lane | 32u), 64);
            const uint32_t h2hi = (uint32_t)__shfl((int)(uint32_t)(h >> 32), (int)(lane | 32u), 64);
            if constexpr (PACK) {
                if (half == 0) emit(j, h, (uint64_t)h2hi << 32 | h2lo);
            } else {
                ((uint2 *)hashes)[2 * (k0 + j) + half] = make_uint2((uint32_t)h, (uint32_t)(h >> 32));
            }
            if constexpr (!P0) return;
        }
    }
    if (mine && !tail) {  // cnt lanes hash the cnt sorted slots
        const uint32_t sk = slot_key[t];
        Funnel f;
        f.init(lds, sk >> 16, sk & 0xffffu);
        f.walk(lds);
        uint64_t h1, h2;
        f.finish(lds, h1, h2);
        emit(slot_idx[t], h1, h2);
    }
    if constexpr (P0) varlen_phase0<KEYS>((uint64_t *)stage, has, my_j, my_pw, k0, cnt, md, p0);
}

// 512 threads per workgroup, 512 - 64 v keys of which the 64 v longest run on 2 v tail waves
// (varlen_tail v = 1, default: 448 keys; 2: 384; 3: 320), a 64-B window per key; or 448 keys hashed one
// per lane (0: 448 threads).
// 256/384/512/1024-key workgroups, 48-80-B windows, no chain waves and two
// ways of giving the chain waves' lanes more keys measured slower.
constexpr uint32_t kVarKeys = 448, kVarWin = 64;

template <bool PACK, bool P0, uint32_t NS>
static void launch_hash_varlen_ns(const KeyBatch &kb, void *out, const ModArg &md, hipStream_t s, Phase0Arg p0) {
    constexpr uint32_t keys = NS ? 512 - 64 * NS : kVarKeys;
    const uint64_t ntiles = (kb.n + keys - 1) / keys;
    hipLaunchKernelGGL((k_hash_varlen<keys, kVarWin, PACK, NS, P0>), dim3((unsigned)ntiles), dim3(keys + 64 * NS), 0,
                       s, kb.data, kb.offsets, kb.n, out, md, p0);
}

template <bool PACK, bool P0 = false>
static hipError_t launch_hash_varlen_any(const KeyBatch &kb, void *out, const ModArg &md, hipStream_t s,
                                        Phase0Arg p0 = {}) {
    if (!kb.offsets || kb.n == 0) return hipSuccess;
    switch (options().varlen_tail) {
    case 0: launch_hash_varlen_ns<PACK, P0, 0>(kb, out, md, s, p0); break;
    case 2: launch_hash_varlen_ns<PACK, P0, 2>(kb, out, md, s, p0); break;
    case 3: launch_hash_varlen_ns<PACK, P0, 3>(kb, out, md, s, p0); break;
    default: launch_hash_varlen_ns<PACK, P0, 1>(kb, out, md, s, p0); break;
    }
    return hipGetLastError();
}

hipError_t launch_hash_varlen_phase0(const KeyBatch &kb, const ModArg &md, const uint32_t *words, uint64_t *rows,
                                     ulonglong2 *recs, uint32_t hi, hipStream_t s) {
    if (md.k != 7 || md.m >= (1ull << kPackBits)) return hipErrorInvalidValue;
    return launch_hash_varlen_any<true, true>(kb, nullptr, md, s, Phase0Arg{words, rows, recs, hi});
}

hipError_t launch_hash_varlen(const KeyBatch &kb, uint4 *hashes, hipStream_t s) {
    return launch_hash_varlen_any<false>(kb, hashes, ModArg{}, s);
}

hipError_t launch_hash_varlen_packed(const KeyBatch &kb, const ModArg &md, uint64_t *packed, hipStream_t s) {
    if (md.k != 7 || md.m >= (1ull << kPackBits)) return hipErrorInvalidValue;
    return launch_hash_varlen_any<true>(kb, packed, md, s);
}

}  // namespace seb
