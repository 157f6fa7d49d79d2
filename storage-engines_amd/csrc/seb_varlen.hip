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

// One FNV chain (A: FNV-1a = hash1, else FNV-1 = hash2) in FnvSplit's form, for the split tail
// waves of k_hash_varlen: the same bits as the matching half of FnvSplit / fnv_word_part.
template <bool A>
struct FnvOne {
    uint32_t lo = (uint32_t)kFnvOffset;
    uint64_t acc = kFnvOffset >> 32;
    __device__ __forceinline__ void word(uint32_t w) {
        uint32_t d[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t b = (w >> (8 * j)) & 0xffu;
            const uint32_t x = A ? lo ^ b : lo;
            const uint64_t p = (uint64_t)x * 435u;
            d[j] = (uint32_t)(p >> 32) + (x << 8);
            lo = A ? (uint32_t)p : (uint32_t)p ^ b;
        }
        const uint64_t t = mad_lo(d[0], pow435(3), mad_lo(d[1], pow435(2), mad_lo(d[2], 435u, d[3])));
        acc = mad_lo((uint32_t)acc, pow435(4), t);
    }
    // bytes [0, r) of w (r < 4) with the plain 64-bit step; returns the chain's hash
    __device__ __forceinline__ uint64_t finish(uint32_t w, uint32_t r) const {
        uint64_t h = (acc << 32) | lo;
#pragma unroll
        for (uint32_t j = 0; j < 3; ++j) {
            const uint64_t b = (w >> (8 * j)) & 0xffu;
            const uint64_t nh = A ? (h ^ b) * kFnvPrime : (h * kFnvPrime) ^ b;
            h = j < r ? nh : h;
        }
        return h;
    }
};

template <bool A>
__device__ __forceinline__ uint64_t funnel_one(const uint32_t *lds, uint32_t b, uint32_t n) {
    uint32_t wi = b >> 2;
    const uint32_t sh = b & 3u;
    uint32_t cur = lds[wi], nxt = lds[wi + 1];
    FnvOne<A> f;
    const uint32_t nw = n >> 2;
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
    return f.finish(__builtin_amdgcn_alignbyte(nxt, cur, sh), n & 3u);
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

// TAIL > 0 (KEYS = 448, 512 threads): a full workgroup's 64 longest keys (the last slots of the
// length order, which otherwise set the workgroup's lifetime and hold its LDS after the other
// waves are done) are hashed by the last two waves, lane for lane the same key, one wave per FNV
// chain: each runs half the instructions.  The FNV-1 wave hands its hashes to the FNV-1a wave
// through LDS for the packed output; the 16-B output is written in halves.
// TAIL == 2 adds the fill (tail_plan): each of those 64 lanes then hashes up to kTailFill more
// keys, the longest remaining ones that fit the gap between its head and the longest key, so the
// chain waves' lanes run about equally long and the one-key-per-lane waves lose their longest keys.
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

constexpr uint32_t kTailFill = 2;   // fill passes: up to 2 more keys per chain-wave lane
constexpr uint32_t kFillMinDw = 2;  // keys under 2 dwords are not worth a lane's per-key overhead
constexpr uint32_t kNoSlot = 0xffffffffu;

__device__ __forceinline__ uint32_t dw_bucket(uint32_t sk) {  // a sorted slot's dword-length bucket
    const uint32_t dw = ((sk & 0xffffu) + 3) >> 2;
    return dw > 64 ? 64u : dw;
}

// The fill's candidate set: the 384 keys after the 64 longest of a full workgroup, longest first
// (candidate c is sorted slot 447 - 64 - c), as a 384-bit used mask held by every lane.
__device__ __forceinline__ uint32_t used_below(const uint64_t (&used)[6], uint32_t x) {
    uint32_t r = 0;
#pragma unroll
    for (uint32_t w = 0; w < 6; ++w) {
        uint64_t m = used[w];
        if (x <= 64 * w) m = 0;
        else if (x < 64 * w + 64) m &= (1ull << (x - 64 * w)) - 1;
        r += (uint32_t)__popcll(m);
    }
    return r;
}

__device__ __forceinline__ uint32_t select_bit(uint64_t v, uint32_t r) {  // position of set bit r of v
    uint32_t pos = 0;
#pragma unroll
    for (uint32_t sh = 32; sh; sh >>= 1) {
        const uint32_t c = (uint32_t)__popcll(v & ((1ull << sh) - 1));
        if (r >= c) {
            r -= c;
            v >>= sh;
            pos += sh;
        }
    }
    return pos;
}

// The k-th candidate (0-based) not yet taken.
__device__ __forceinline__ uint32_t select_unused(const uint64_t (&used)[6], uint32_t k) {
    uint32_t c = kNoSlot, cum = 0;
#pragma unroll
    for (uint32_t w = 0; w < 6; ++w) {
        const uint64_t fr = ~used[w];
        const uint32_t f = (uint32_t)__popcll(fr);
        if (c == kNoSlot && k < cum + f) c = 64 * w + select_bit(fr, k - cum);
        cum += f;
    }
    return c;
}

__device__ __forceinline__ uint64_t wave_or64(uint64_t v) {
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) v |= __shfl_xor(v, o, 64);
    return v;
}

// The fill plan of a full workgroup's two chain waves (both compute it, identically).  Lane l's
// head is sorted slot 384 + l (lane 0: the shortest of the 64 longest keys, the largest gap to
// the longest, slot 447).  Each pass, the lanes in order take the longest free candidate that fits
// their remaining gap, distinct from the other lanes' (the recurrence c_l = max(c_prev + 1, g_l)
// over the lanes that fit anything, as a prefix maximum); keys[1 + p] is the slot taken in pass p
// or kNoSlot.  Lengths are dword buckets, the units of the work.
__device__ __forceinline__ void tail_plan(const uint32_t *slot_key, uint32_t lane, uint32_t (&keys)[1 + kTailFill],
                                          uint64_t (&used)[6]) {
    constexpr uint32_t kCand = 384;
    auto size = [&](uint32_t c) { return dw_bucket(slot_key[kCand - 1 - c]); };
    const uint32_t longest = dw_bucket(slot_key[447]);
    uint32_t load = dw_bucket(slot_key[kCand + lane]);
    keys[0] = kCand + lane;
    uint32_t nc = 0;  // candidates of at least kFillMinDw dwords: a prefix of the candidate order
    {
        uint32_t lo = 0, hi = kCand;
#pragma unroll
        for (int it = 0; it < 9; ++it)
            if (lo < hi) {
                const uint32_t mid = (lo + hi) >> 1;
                if (size(mid) < kFillMinDw) hi = mid;
                else lo = mid + 1;
            }
        nc = lo;
    }
#pragma unroll
    for (uint32_t w = 0; w < 6; ++w) used[w] = 0;
    uint32_t nused = 0;
#pragma unroll
    for (uint32_t pass = 0; pass < kTailFill; ++pass) {
        const uint32_t gap = longest - load;
        uint32_t lo = 0, hi = nc;  // g: the first candidate that fits the gap
#pragma unroll
        for (int it = 0; it < 9; ++it)
            if (lo < hi) {
                const uint32_t mid = (lo + hi) >> 1;
                if (size(mid) <= gap) hi = mid;
                else lo = mid + 1;
            }
        const bool fit = lo < nc && used_below(used, nc) - used_below(used, lo) < nc - lo;  // a free one fits
        const uint64_t fits = __ballot(fit);
        const int kv = (int)lanes_below(fits);
        int x = fit ? (int)(lo - used_below(used, lo)) - kv : INT_MIN;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int y = __shfl_up(x, o, 64);
            if ((int)lane >= o) x = max(x, y);
        }
        const uint32_t cc = (uint32_t)(kv + x);  // this lane's rank among the free candidates
        const bool ok = fit && cc < nc - nused;
        const uint32_t c = ok ? select_unused(used, cc) : kNoSlot;
        keys[1 + pass] = ok ? kCand - 1 - c : kNoSlot;
        if (ok) load += size(c);
#pragma unroll
        for (uint32_t w = 0; w < 6; ++w) used[w] |= wave_or64(ok && (c >> 6) == w ? 1ull << (c & 63) : 0ull);
        nused += (uint32_t)__popcll(__ballot(ok));
    }
}

// Every thread of the workgroup arrives here; its hashed keys' packed words (n of them, key
// indices j[]) go to xpk (the staging window), then waves 0 .. KEYS/64 - 1 each take the group of
// keys k0 + 64 * wave + lane (k0 is a multiple of 64).
template <uint32_t KEYS, uint32_t NK>
__device__ __forceinline__ void varlen_phase0(uint64_t *xpk, const uint32_t (&my_j)[NK], const uint64_t (&my_pw)[NK],
                                              uint64_t k0, uint32_t cnt, const ModArg &md, const Phase0Arg &p0) {
    __syncthreads();  // every key is hashed: the staging window is free
#pragma unroll
    for (uint32_t s = 0; s < NK; ++s)
        if (my_j[s] != kNoSlot) xpk[my_j[s]] = my_pw[s];
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

template <uint32_t KEYS, uint32_t WIN, bool PACK, uint32_t TAIL = 0, bool P0 = false>
__global__ __launch_bounds__(TAIL ? 512 : KEYS) void k_hash_varlen(const uint8_t *__restrict__ data,
                                                                   const uint64_t *__restrict__ off, uint64_t n,
                                                                   void *__restrict__ hashes, ModArg md, Phase0Arg p0) {
    constexpr uint32_t kHashLds = KEYS * WIN;
    constexpr uint32_t NK = TAIL == 2 ? 1 + kTailFill : 1;  // keys a lane may hash
    static_assert(kHashLds % 16 == 0 && kHashLds + 16 < 65536, "window offsets are 16-bit");
    static_assert(!TAIL || KEYS == 448, "the chain waves: 64 keys, two waves, 512 threads");
    static_assert(!P0 || (PACK && KEYS % 64 == 0 && KEYS * 8 <= kHashLds), "phase 0: whole groups of 64 keys, words in the window");
    __shared__ uint4 stage[kHashLds / 16 + 1];  // +16 B: the funnel walk reads one dword past a key
    // the length sort's bucket counters; after the sort: the fill's used mask (6 words), the
    // handover flags (TAIL == 2)
    __shared__ uint64_t cur64[(kLenBuckets + 1) / 2];
    uint32_t *cur = (uint32_t *)cur64;
    __shared__ uint32_t slot_key[KEYS];  // sorted slot -> start byte in the window << 16 | length
    __shared__ uint16_t slot_idx[KEYS];  // sorted slot -> key within the workgroup
    __shared__ uint64_t xh2[TAIL ? (TAIL == 2 ? 128 : 64) : 1];  // the FNV-1 wave's hashes for the FNV-1a wave
    __shared__ uint32_t xflag[TAIL == 1 ? 1 : 1];
    const uint32_t t = threadIdx.x;
    const uint64_t k0 = (uint64_t)blockIdx.x * KEYS;
    const uint64_t k1 = k0 + KEYS < n ? k0 + KEYS : n;
    const uint32_t cnt = (uint32_t)(k1 - k0);
    const bool mine = t < cnt;
    // P0: a thread keeps its keys' packed words until every key is hashed, then the words go to the
    // (by then unused) staging window in key order: no LDS of its own, so 5 workgroups still fit a CU
    uint32_t my_j[NK];
    uint64_t my_pw[NK];
#pragma unroll
    for (uint32_t s = 0; s < NK; ++s) {
        my_j[s] = kNoSlot;
        my_pw[s] = 0;
    }
    auto emit = [&](uint32_t s, uint32_t j, uint64_t h1, uint64_t h2) {  // key k0 + j, the lane's s-th
        if constexpr (P0) {
            my_j[s] = j;
            my_pw[s] = pack_residue(h1, h2, md);
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
            emit(0, t, h1, h2);
        }
        if constexpr (P0) varlen_phase0<KEYS>((uint64_t *)stage, my_j, my_pw, k0, cnt, md, p0);
        return;
    }
    if (t < kLenBuckets) cur[t] = 0u;
    if (t < 1) xflag[t] = 0u;
    for (uint32_t c = t; c < (uint32_t)chunks; c += blockDim.x) stage[c] = ((const uint4 *)base)[c];
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
    const bool full = TAIL && cnt == KEYS;
    const uint32_t lane = t & 63;
    if constexpr (TAIL == 2) {
        // the chain waves plan the fill; the first writes the used mask for the one-key waves and
        // clears the handover flags (the sort's counters are dead), then everyone proceeds
        uint32_t keys[NK];
        uint64_t used[6];
        uint32_t *flags = (uint32_t *)(cur64 + 6);  // [0..2]: h2 of step s ready; [3]: step 0's slot read
        if (full && t >= 384) {
            tail_plan(slot_key, lane, keys, used);
            if (t < 448 && lane < 6) cur64[lane] = used[lane];
            if (t < 448 && lane < 4) flags[lane] = 0u;
        }
        __syncthreads();
        if (full && t < 384) {  // one key per lane: the t-th longest key not taken by the fill
#pragma unroll
            for (uint32_t w = 0; w < 6; ++w) used[w] = cur64[w];
            const uint32_t nrem = 384 - used_below(used, 384);
            if (t < nrem) {
                const uint32_t sq = 383 - select_unused(used, t);
                const uint32_t sk = slot_key[sq];
                Funnel f;
                f.init(lds, sk >> 16, sk & 0xffffu);
                f.walk(lds);
                uint64_t h1, h2;
                f.finish(lds, h1, h2);
                emit(0, slot_idx[sq], h1, h2);
            }
        } else if (full) {  // the chain waves: a lane's head, then its fill keys, one chain each
            const bool chain_a = t < 448;  // FNV-1a (hash1); the other wave FNV-1 (hash2)
#pragma unroll
            for (uint32_t s = 0; s < NK; ++s) {
                const uint32_t sq = keys[s];
                const bool has = sq != kNoSlot;
                const uint32_t sk = has ? slot_key[sq] : 0u;
                const uint32_t j = has ? slot_idx[sq] : 0u;
                if (chain_a) {
                    const uint64_t h1 = has ? funnel_one<true>(lds, sk >> 16, sk & 0xffffu) : 0ull;
                    if constexpr (PACK) {
                        while (__hip_atomic_load(&flags[s], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) == 0u)
                            __builtin_amdgcn_s_sleep(1);
                        const uint64_t h2 = xh2[64 * (s & 1) + lane];
                        if (s == 0) {
                            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                            __builtin_amdgcn_wave_barrier();
                            if (lane == 0) __hip_atomic_store(&flags[3], 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
                        }
                        if (has) emit(s, j, h1, h2);
                    } else if (has) {
                        ((uint2 *)hashes)[2 * (k0 + j)] = make_uint2((uint32_t)h1, (uint32_t)(h1 >> 32));
                    }
                } else {
                    const uint64_t h2 = has ? funnel_one<false>(lds, sk >> 16, sk & 0xffffu) : 0ull;
                    if constexpr (PACK) {
                        if (s == 2)  // buffer 0 again: the FNV-1a wave has read step 0's hashes
                            while (__hip_atomic_load(&flags[3], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) == 0u)
                                __builtin_amdgcn_s_sleep(1);
                        xh2[64 * (s & 1) + lane] = h2;
                        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                        __builtin_amdgcn_wave_barrier();
                        if (lane == 0) __hip_atomic_store(&flags[s], 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
                    } else if (has) {
                        ((uint2 *)hashes)[2 * (k0 + j) + 1] = make_uint2((uint32_t)h2, (uint32_t)(h2 >> 32));
                    }
                }
            }
        }
        if (!full && mine) {  // a partial workgroup: one key per lane, in length order
            const uint32_t sk = slot_key[t];
            Funnel f;
            f.init(lds, sk >> 16, sk & 0xffffu);
            f.walk(lds);
            uint64_t h1, h2;
            f.finish(lds, h1, h2);
            emit(0, slot_idx[t], h1, h2);
        }
    } else {
        bool tail = false;
        if constexpr (TAIL == 1) {
            if (full && t >= KEYS - 64) {  // the longest keys: a wave pair per 64, one per chain
                tail = true;
                const uint32_t w = (t - (KEYS - 64)) >> 6;
                const uint32_t qq = KEYS - 64 + lane;
                const uint32_t sk = slot_key[qq];
                const uint32_t j = slot_idx[qq];
                if ((w & 1u) == 0u) {  // FNV-1a (hash1)
                    const uint64_t h1 = funnel_one<true>(lds, sk >> 16, sk & 0xffffu);
                    if constexpr (PACK) {
                        while (__hip_atomic_load(&xflag[0], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) == 0u)
                            __builtin_amdgcn_s_sleep(1);
                        emit(0, j, h1, xh2[lane]);
                    } else {
                        ((uint2 *)hashes)[2 * (k0 + j)] = make_uint2((uint32_t)h1, (uint32_t)(h1 >> 32));
                    }
                } else {  // FNV-1 (hash2)
                    const uint64_t h2 = funnel_one<false>(lds, sk >> 16, sk & 0xffffu);
                    if constexpr (PACK) {
                        xh2[lane] = h2;
                        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                        __builtin_amdgcn_wave_barrier();
                        if (lane == 0)
                            __hip_atomic_store(&xflag[0], 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
                    } else {
                        ((uint2 *)hashes)[2 * (k0 + j) + 1] = make_uint2((uint32_t)h2, (uint32_t)(h2 >> 32));
                    }
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
            emit(0, slot_idx[t], h1, h2);
        }
    }
    if constexpr (P0) varlen_phase0<KEYS>((uint64_t *)stage, my_j, my_pw, k0, cnt, md, p0);
}

// 448 keys per 512-thread workgroup, the top 64 split over two chain waves with the fill
// (varlen_tail 2, default) or without it (1), a 64-B window per key (DESIGN.md 5.5 and 8:
// 256/384/512/1024-key workgroups and 48-80-B windows measured slower).
constexpr uint32_t kVarKeys = 448, kVarWin = 64;

template <bool PACK, bool P0 = false>
static hipError_t launch_hash_varlen_any(const KeyBatch &kb, void *out, const ModArg &md, hipStream_t s,
                                        Phase0Arg p0 = {}) {
    if (!kb.offsets || kb.n == 0) return hipSuccess;
    const uint64_t ntiles = (kb.n + kVarKeys - 1) / kVarKeys;
    if (options().varlen_tail == 2)
        hipLaunchKernelGGL((k_hash_varlen<kVarKeys, kVarWin, PACK, 2, P0>), dim3((unsigned)ntiles), dim3(512), 0, s,
                           kb.data, kb.offsets, kb.n, out, md, p0);
    else
        hipLaunchKernelGGL((k_hash_varlen<kVarKeys, kVarWin, PACK, 1, P0>), dim3((unsigned)ntiles), dim3(512), 0, s,
                           kb.data, kb.offsets, kb.n, out, md, p0);
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
