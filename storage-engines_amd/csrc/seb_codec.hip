// seb_codec.hip — the storage engine's other batchable hash/codec steps.
//
//  A  hash-index shard routing.  The reference routes every key through
//       h := fnv.New32a(); h.Write([]byte(key)); shard = h.Sum32() & shardMask
//     (hashindex/shard.go:47-52 getShard, and :104-122 where UpdateBatch distributes a whole batch
//     of updates and deletions over the 256 shards).  k_route hashes a key batch with FNV-1a 32
//     (offset 0x811c9dc5, prime 0x01000193); k_route_tile / k_route_scan_rows / k_route_scatter
//     turn a batch into a stable partition (keys grouped by shard, input order inside a shard).
//  B  WAL record checksums.  A record is [crc32 u32][seq u64][keySize u32][valueSize u32]
//     [deleted u8][key][value], crc = crc32.ChecksumIEEE(record[4:]) (lsm/wal.go:31-62 Append;
//     ReadAll re-checks it at :123-133).  k_wal_crc computes the CRC of many records at once,
//     and optionally seals them (writes the field) or verifies them (framing + stored CRC).
//
// Both are byte-serial per key/record (FNV multiply chain, CRC table chain) and independent across
// keys/records, so the kernels run one lane per key or record and keep everything else HBM-streamed.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "seb_device.h"
#include "seb_kernels.h"

namespace seb {

constexpr uint32_t kFnv32Offset = 0x811c9dc5u;
constexpr uint32_t kFnv32Prime = 0x01000193u;

// ------------------------------------------------------------------ FNV-1a 32 routing -------

__device__ __forceinline__ uint32_t fnv32a_word(uint32_t h, uint32_t w) {
#pragma unroll
    for (int j = 0; j < 4; ++j) h = (h ^ ((w >> (8 * j)) & 0xffu)) * kFnv32Prime;
    return h;
}

// Bytes [lo, hi) of w, predicated (the wave stays converged).
__device__ __forceinline__ uint32_t fnv32a_part(uint32_t h, uint32_t w, uint32_t lo, uint32_t hi) {
#pragma unroll
    for (uint32_t j = 0; j < 4; ++j) {
        const uint32_t a = (h ^ ((w >> (8 * j)) & 0xffu)) * kFnv32Prime;
        h = (j >= lo && j < hi) ? a : h;
    }
    return h;
}

// FNV-1a 32 of bytes [s, e) of p, over the aligned dwords that cover them (a dword holding a byte
// of the buffer never crosses a page, so reading the whole dword cannot fault).
__device__ __forceinline__ uint32_t fnv32a_range(const uint8_t *p, uint64_t s, uint64_t e) {
    uint32_t h = kFnv32Offset;
    const uintptr_t beg = (uintptr_t)(p + s), end = (uintptr_t)(p + e);
    for (uintptr_t a = beg & ~(uintptr_t)3; a < end; a += 4) {
        const uint32_t w = *(const uint32_t *)a;
        const uint32_t lo = beg > a ? (uint32_t)(beg - a) : 0u;
        const uint32_t hi = end - a < 4 ? (uint32_t)(end - a) : 4u;
        h = (lo == 0 && hi == 4) ? fnv32a_word(h, w) : fnv32a_part(h, w, lo, hi);
    }
    return h;
}

__device__ __forceinline__ uint32_t route_hash(const KeyBatch &kb, uint64_t i) {
    if (kb.offsets) return fnv32a_range(kb.data, kb.offsets[i], kb.offsets[i + 1]);
    if (kb.stride == 16 && ((uintptr_t)kb.data & 15) == 0) {
        const uint4 v = ((const uint4 *)kb.data)[i];
        return fnv32a_word(fnv32a_word(fnv32a_word(fnv32a_word(kFnv32Offset, v.x), v.y), v.z), v.w);
    }
    return fnv32a_range(kb.data, i * (uint64_t)kb.stride, (i + 1) * (uint64_t)kb.stride);
}

// shard[i] = FNV-1a32(key i) & mask; hash[i] (optional) = the full 32-bit hash.
__global__ __launch_bounds__(256) void k_route(KeyBatch kb, uint32_t mask, uint16_t *__restrict__ shard,
                                               uint32_t *__restrict__ hash) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < kb.n; i += stride) {
        const uint32_t h = route_hash(kb, i);
        if (shard) shard[i] = (uint16_t)(h & mask);
        if (hash) hash[i] = h;
    }
}

// ---- stable partition by shard (keys grouped by shard, input order inside a shard), three launches:
//   k_route_tile       hash a 4096-key tile, write its shard ids, per-tile histogram (bin-major)
//   k_route_scan_rows  per bin: exclusive prefix of its row of tile counts, row total
//   k_route_scatter    every workgroup scans the bin totals itself (<= 4096 values), then each wave
//                      ranks its own contiguous 1024 keys: pass 1 counts per (wave, bin), pass 2
//                      places keys, equal shards ordered by __ballot peer masks (one ballot per shard
//                      bit).  No atomic decides a position, so the permutation is deterministic.
constexpr uint32_t kRouteThreads = 256;
constexpr uint32_t kRouteWaves = kRouteThreads / 64;
constexpr uint32_t kRoutePerLane = 16;
constexpr uint32_t kRouteTile = kRouteThreads * kRoutePerLane;  // 4096 keys
constexpr uint32_t kRouteMaxBits = 12;

__global__ __launch_bounds__(kRouteThreads) void k_route_tile(KeyBatch kb, uint32_t mask, uint32_t nbins,
                                                              uint32_t ntiles, uint16_t *__restrict__ shard,
                                                              uint32_t *__restrict__ counts) {
    extern __shared__ uint32_t hist[];
    for (uint32_t b = threadIdx.x; b < nbins; b += blockDim.x) hist[b] = 0u;
    __syncthreads();
    const uint64_t t0 = (uint64_t)blockIdx.x * kRouteTile;
    const uint64_t t1 = t0 + kRouteTile < kb.n ? t0 + kRouteTile : kb.n;
    for (uint64_t i = t0 + threadIdx.x; i < t1; i += blockDim.x) {
        const uint32_t sh = route_hash(kb, i) & mask;
        shard[i] = (uint16_t)sh;
        atomicAdd(&hist[sh], 1u);
    }
    __syncthreads();
    for (uint32_t b = threadIdx.x; b < nbins; b += blockDim.x) counts[(uint64_t)b * ntiles + blockIdx.x] = hist[b];
}

// One workgroup per bin: exclusive prefix of the bin's row of tile counts; row total to totals[b].
__global__ __launch_bounds__(1024) void k_route_scan_rows(uint32_t *__restrict__ counts, uint32_t ntiles,
                                                          uint32_t *__restrict__ totals) {
    __shared__ uint32_t wsum[16];
    __shared__ uint32_t carry;
    uint32_t *row = counts + (uint64_t)blockIdx.x * ntiles;
    if (threadIdx.x == 0) carry = 0u;
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    for (uint32_t base = 0; base < ntiles; base += blockDim.x) {
        const uint32_t j = base + threadIdx.x;
        const uint32_t x = j < ntiles ? row[j] : 0u;
        uint32_t v = x;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t y = __shfl_up(v, d, 64);
            if (lane >= (uint32_t)d) v += y;
        }
        if (lane == 63) wsum[wid] = v;
        __syncthreads();
        uint32_t before = carry;
        for (uint32_t w = 0; w < wid; ++w) before += wsum[w];
        if (j < ntiles) row[j] = before + v - x;
        __syncthreads();
        if (threadIdx.x == blockDim.x - 1) carry = before + v;
        __syncthreads();
    }
    if (threadIdx.x == 0) totals[blockIdx.x] = carry;
}

// LDS: wrun[kRouteWaves][nbins] | wsum[kRouteWaves]
__global__ __launch_bounds__(kRouteThreads) void k_route_scatter(const uint16_t *__restrict__ shard, uint64_t n,
                                                                 uint32_t nbins, uint32_t bits, uint32_t ntiles,
                                                                 const uint32_t *__restrict__ counts,
                                                                 const uint32_t *__restrict__ totals,
                                                                 uint64_t *__restrict__ shard_begin,
                                                                 uint32_t *__restrict__ perm) {
    extern __shared__ uint32_t smem[];
    uint32_t *wrun = smem;                         // [wave][bin]
    uint32_t *wsum = smem + kRouteWaves * nbins;   // [wave]
    const uint32_t lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    // 1. bin bases: exclusive scan of the bin totals, thread t owns bins [t*per, (t+1)*per)
    const uint32_t per = (nbins + kRouteThreads - 1) / kRouteThreads;
    const uint32_t b0 = threadIdx.x * per;
    uint32_t sum = 0;
    for (uint32_t j = 0; j < per; ++j)
        if (b0 + j < nbins) sum += totals[b0 + j];
    uint32_t v = sum;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(v, d, 64);
        if (lane >= (uint32_t)d) v += y;
    }
    if (lane == 63) wsum[wid] = v;
    for (uint32_t w = 0; w < kRouteWaves; ++w)
        for (uint32_t j = threadIdx.x; j < nbins; j += kRouteThreads) wrun[w * nbins + j] = 0u;
    __syncthreads();
    uint32_t run = v - sum;
    for (uint32_t w = 0; w < wid; ++w) run += wsum[w];
    // run = first output slot of bin b0; this tile's slots in bin b start at base_b + row prefix
    uint32_t tile_base[16];
    for (uint32_t j = 0; j < per; ++j)
        if (b0 + j < nbins) {
            const uint32_t c = totals[b0 + j];
            if (blockIdx.x == 0 && shard_begin) shard_begin[b0 + j] = run;
            tile_base[j] = run + counts[(uint64_t)(b0 + j) * ntiles + blockIdx.x];
            run += c;
        }
    if (blockIdx.x == 0 && shard_begin && threadIdx.x == kRouteThreads - 1) shard_begin[nbins] = n;
    // 2. pass 1: per-(wave, bin) counts of this wave's 1024 contiguous keys
    const uint64_t w0 = (uint64_t)blockIdx.x * kRouteTile + (uint64_t)wid * 64 * kRoutePerLane;
    uint32_t sv[kRoutePerLane];
    uint64_t pk[kRoutePerLane];  // peer masks, reused by pass 2
    const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
#pragma unroll
    for (uint32_t r = 0; r < kRoutePerLane; ++r) {
        const uint64_t i = w0 + (uint64_t)r * 64 + lane;
        sv[r] = i < n ? shard[i] : 0xffffffffu;
    }
#pragma unroll
    for (uint32_t r = 0; r < kRoutePerLane; ++r) {
        const bool live = sv[r] != 0xffffffffu;
        pk[r] = wave_peers(live, sv[r], bits);
        if (live && (pk[r] & lt) == 0ull) wrun[wid * nbins + sv[r]] += (uint32_t)__popcll(pk[r]);
    }
    __syncthreads();
    // 3. wave bases per bin: tile base + the counts of the waves before
    for (uint32_t j = 0; j < per; ++j)
        if (b0 + j < nbins) {
            uint32_t acc = tile_base[j];
            for (uint32_t w = 0; w < kRouteWaves; ++w) {
                const uint32_t c = wrun[w * nbins + b0 + j];
                wrun[w * nbins + b0 + j] = acc;
                acc += c;
            }
        }
    __syncthreads();
    // 4. pass 2: place; the group leader advances the wave's cursor after every lane has read it
#pragma unroll
    for (uint32_t r = 0; r < kRoutePerLane; ++r) {
        const bool live = sv[r] != 0xffffffffu;
        const uint64_t peers = pk[r];
        uint32_t at = 0;
        if (live) at = wrun[wid * nbins + sv[r]];
        __builtin_amdgcn_wave_barrier();
        if (live) {
            perm[at + (uint32_t)__popcll(peers & lt)] = (uint32_t)(w0 + (uint64_t)r * 64 + lane);
            if ((peers & lt) == 0ull) wrun[wid * nbins + sv[r]] = at + (uint32_t)__popcll(peers);
        }
        __builtin_amdgcn_wave_barrier();
    }
}

uint64_t route_workspace_bytes(uint64_t n, uint32_t bits) {
    const uint64_t ntiles = (n + kRouteTile - 1) / kRouteTile;
    const uint64_t nbins = 1ull << bits;
    auto al = [](uint64_t x) { return (x + 255) & ~255ull; };
    return al(n * 2) + al(nbins * ntiles * 4) + al(nbins * 4);
}

hipError_t launch_route(const KeyBatch &kb, uint32_t bits, uint16_t *shard, uint32_t *hash, hipStream_t s) {
    if (kb.n == 0) return hipSuccess;
    if (bits > 16) return hipErrorInvalidValue;
    const uint32_t mask = bits ? ((1u << bits) - 1u) : 0u;
    uint64_t g = (kb.n + 255) / 256;
    if (g > 65536) g = 65536;
    hipLaunchKernelGGL(k_route, dim3((unsigned)g), dim3(256), 0, s, kb, mask, shard, hash);
    return hipGetLastError();
}

hipError_t launch_route_partition(const KeyBatch &kb, uint32_t bits, uint32_t *perm, uint64_t *shard_begin,
                                  uint16_t *shard_out, void *ws, uint64_t ws_bytes, hipStream_t s) {
    if (bits > kRouteMaxBits || kb.n >= (1ull << 32)) return hipErrorInvalidValue;
    if (ws_bytes < route_workspace_bytes(kb.n, bits)) return hipErrorInvalidValue;
    const uint32_t nbins = 1u << bits;
    if (kb.n == 0) {
        if (shard_begin) return hipMemsetAsync(shard_begin, 0, (nbins + 1) * sizeof(uint64_t), s);
        return hipSuccess;
    }
    const uint32_t ntiles = (uint32_t)((kb.n + kRouteTile - 1) / kRouteTile);
    auto al = [](uint64_t x) { return (x + 255) & ~255ull; };
    uint8_t *w = (uint8_t *)ws;
    uint16_t *shard = (uint16_t *)w;
    uint32_t *counts = (uint32_t *)(w + al(kb.n * 2));
    uint32_t *totals = (uint32_t *)(w + al(kb.n * 2) + al((uint64_t)nbins * ntiles * 4));
    hipLaunchKernelGGL(k_route_tile, dim3(ntiles), dim3(kRouteThreads), nbins * sizeof(uint32_t), s, kb,
                       nbins - 1, nbins, ntiles, shard, counts);
    hipLaunchKernelGGL(k_route_scan_rows, dim3(nbins), dim3(1024), 0, s, counts, ntiles, totals);
    const size_t lds = ((size_t)kRouteWaves * nbins + kRouteWaves) * sizeof(uint32_t);
    hipLaunchKernelGGL(k_route_scatter, dim3(ntiles), dim3(kRouteThreads), lds, s, shard, kb.n, nbins, bits, ntiles,
                       counts, totals, shard_begin, perm);
    if (shard_out) {
        hipError_t e = hipMemcpyAsync(shard_out, shard, kb.n * 2, hipMemcpyDeviceToDevice, s);
        if (e != hipSuccess) return e;
    }
    return hipGetLastError();
}

// ------------------------------------------------------------------ WAL CRC32-IEEE ----------
// crc32.ChecksumIEEE: reflected polynomial 0xEDB88320, init ~0, final ~ (Go hash/crc32).
// Slicing-by-4 tables, generated at compile time, staged in LDS per workgroup.

struct CrcTables {
    uint32_t t[4][256];
};
constexpr CrcTables make_crc_tables() {
    CrcTables c{};
    for (uint32_t i = 0; i < 256; ++i) {
        uint32_t v = i;
        for (int b = 0; b < 8; ++b) v = (v & 1u) ? (v >> 1) ^ 0xEDB88320u : v >> 1;
        c.t[0][i] = v;
    }
    for (uint32_t i = 0; i < 256; ++i)
        for (int k = 1; k < 4; ++k) c.t[k][i] = (c.t[k - 1][i] >> 8) ^ c.t[0][c.t[k - 1][i] & 0xffu];
    return c;
}
__device__ const CrcTables kCrcTab = make_crc_tables();

__device__ __forceinline__ uint32_t crc_word(uint32_t crc, uint32_t w, const uint32_t (*t)[256]) {
    const uint32_t x = crc ^ w;
    return t[3][x & 0xffu] ^ t[2][(x >> 8) & 0xffu] ^ t[1][(x >> 16) & 0xffu] ^ t[0][x >> 24];
}
__device__ __forceinline__ uint32_t crc_byte(uint32_t crc, uint32_t b, const uint32_t (*t)[256]) {
    return (crc >> 8) ^ t[0][(crc ^ b) & 0xffu];
}

// CRC state over bytes [s, e) of p (raw state in/out: caller applies the ~ at both ends).
__device__ __forceinline__ uint32_t crc_range(uint32_t crc, const uint8_t *p, uint64_t s, uint64_t e,
                                              const uint32_t (*t)[256]) {
    uint64_t a = s;
    while (a < e && (((uintptr_t)(p + a)) & 3u)) crc = crc_byte(crc, p[a++], t);  // to a dword boundary
    const uint32_t *w = (const uint32_t *)(p + a);
    uint64_t nw = (e - a) >> 2;
    for (uint64_t j = 0; j < nw; ++j) crc = crc_word(crc, w[j], t);
    for (a += nw << 2; a < e; ++a) crc = crc_byte(crc, p[a], t);
    return crc;
}

__device__ __forceinline__ uint32_t ld_u32_le(const uint8_t *p) {
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

__device__ __forceinline__ void wal_finish(uint8_t *data, uint64_t s, uint64_t len, uint32_t crc, int mode,
                                           uint32_t ks, uint32_t vs, uint32_t stored, uint64_t i,
                                           uint32_t *crc_out, uint8_t *ok) {
    if (crc_out) crc_out[i] = crc;
    if (mode == 1 && len >= 4) {
        data[s] = (uint8_t)crc;
        data[s + 1] = (uint8_t)(crc >> 8);
        data[s + 2] = (uint8_t)(crc >> 16);
        data[s + 3] = (uint8_t)(crc >> 24);
    } else if (mode == 2) {
        ok[i] = (len >= 21 && 21ull + ks + vs == len && stored == crc) ? 1 : 0;
    }
}

// mode 0: crc[i] = ChecksumIEEE(record i [4:]); mode 1: also store it into the record's first 4
// bytes (Append's sealing); mode 2: ok[i] = framing holds (len >= 21, 21 + keySize + valueSize ==
// len) and the stored CRC matches (ReadAll's check).  Records i = data[off[i], off[i+1]).
//
// A workgroup owns kWalRecs consecutive records.  Their byte span is copied into LDS with
// coalesced 16-B loads (one lane per record would otherwise make every wave-wide load touch 64
// different cache lines), and each lane then runs the table CRC over its record from LDS, four
// bytes per step through a funnel shift of two aligned LDS dwords.  A span larger than the LDS
// window is checksummed straight from HBM.
constexpr uint32_t kWalRecs = 256;

template <uint32_t kWalLds>
__global__ __launch_bounds__(kWalRecs) void k_wal_crc(uint8_t *__restrict__ data, const uint64_t *__restrict__ off,
                                                      uint64_t n, int mode, uint32_t *__restrict__ crc_out,
                                                      uint8_t *__restrict__ ok) {
    __shared__ uint32_t tab[4][256];
    __shared__ uint4 stage[kWalLds / 16 + 1];
    for (uint32_t j = threadIdx.x; j < 1024; j += blockDim.x) (&tab[0][0])[j] = (&kCrcTab.t[0][0])[j];
    const uint64_t r0 = (uint64_t)blockIdx.x * kWalRecs;
    const uint64_t r1 = r0 + kWalRecs < n ? r0 + kWalRecs : n;
    const uintptr_t base = ((uintptr_t)(data + off[r0])) & ~(uintptr_t)15;
    const uintptr_t end = (uintptr_t)(data + off[r1]);
    const bool staged = end - base <= kWalLds;
    if (staged) {
        const uint32_t chunks = (uint32_t)((end - base + 15) >> 4);
        const uint4 *src = (const uint4 *)base;
        for (uint32_t c = threadIdx.x; c < chunks; c += blockDim.x) stage[c] = src[c];
    }
    __syncthreads();
    const uint64_t i = r0 + threadIdx.x;
    if (i >= r1) return;
    const uint64_t s = off[i], e = off[i + 1];
    const uint64_t len = e > s ? e - s : 0;
    uint32_t crc = 0u, ks = 0u, vs = 0u, stored = 0u;
    if (staged) {
        const uint8_t *lb = (const uint8_t *)stage;
        const uint32_t b = (uint32_t)((uintptr_t)(data + s) - base);
        if (len >= 4) {
            const uint32_t *lw = (const uint32_t *)stage;
            const uint32_t p = b + 4, L = (uint32_t)len - 4, sh = p & 3u;
            uint32_t wi = p >> 2, cur = lw[wi], c = ~0u;
            for (uint32_t j = 0; j + 4 <= L; j += 4) {
                const uint32_t nxt = lw[++wi];
                c = crc_word(c, __builtin_amdgcn_alignbyte(nxt, cur, sh), tab);
                cur = nxt;
            }
            const uint32_t r = L & 3u;
            if (r) {
                const uint32_t w = __builtin_amdgcn_alignbyte(lw[wi + 1], cur, sh);
                for (uint32_t j = 0; j < r; ++j) c = crc_byte(c, (w >> (8 * j)) & 0xffu, tab);
            }
            crc = ~c;
            stored = (uint32_t)lb[b] | ((uint32_t)lb[b + 1] << 8) | ((uint32_t)lb[b + 2] << 16) |
                     ((uint32_t)lb[b + 3] << 24);
        }
        if (len >= 21) {
            ks = (uint32_t)lb[b + 12] | ((uint32_t)lb[b + 13] << 8) | ((uint32_t)lb[b + 14] << 16) |
                 ((uint32_t)lb[b + 15] << 24);
            vs = (uint32_t)lb[b + 16] | ((uint32_t)lb[b + 17] << 8) | ((uint32_t)lb[b + 18] << 16) |
                 ((uint32_t)lb[b + 19] << 24);
        }
    } else {
        if (len >= 4) {
            crc = ~crc_range(~0u, data, s + 4, e, tab);
            stored = ld_u32_le(data + s);
        }
        if (len >= 21) {
            ks = ld_u32_le(data + s + 12);
            vs = ld_u32_le(data + s + 16);
        }
    }
    wal_finish(data, s, len, crc, mode, ks, vs, stored, i, crc_out, ok);
}

hipError_t launch_wal_crc(uint8_t *data, const uint64_t *off, uint64_t n, int mode, uint32_t *crc, uint8_t *ok,
                          hipStream_t s) {
    if (n == 0) return hipSuccess;
    const uint64_t g = (n + kWalRecs - 1) / kWalRecs;
    if (g >= (1ull << 31)) return hipErrorInvalidValue;
    // 36 KiB of staging: four workgroups per CU (measured 4% faster than 48 KiB)
    hipLaunchKernelGGL(k_wal_crc<36 * 1024>, dim3((unsigned)g), dim3(kWalRecs), 0, s, data, off, n, mode, crc, ok);
    return hipGetLastError();
}

}  // namespace seb
