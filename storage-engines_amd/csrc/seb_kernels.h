// seb_kernels.h — internal interface between the C-ABI host layer and the gfx950 kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace seb {

// Reduction constants for one filter, computed on the host (seb_host.cpp: mod_arg()).
struct ModArg {
    uint64_t m;   // numBits (>= 1)
    uint64_t mu;  // floor((2^64 - 1) / m)
    uint64_t c;   // 2^64 mod m
    uint32_t k;   // numHashes
    uint32_t pad;
};
// Filters with m below this take the u32-residue kernels (template flag M32): the Barrett
// quotient (mod_m31) is at most one low, so x - q*m < 2m fits in 32 bits.
constexpr uint64_t kM32Limit = 1ull << 31;

struct KeyBatch {  // device pointers
    const uint8_t *data;
    const uint64_t *offsets;  // n+1 or nullptr
    uint64_t n;
    uint32_t stride;
    const uint4 *hashes = nullptr;   // pre-hashed batch: (h1 lo, h1 hi, h2 lo, h2 hi) per key
};

constexpr int kMaxMulti = 64;
struct MultiFilter {
    const uint32_t *words;
    ModArg md;
};
struct MultiArg {  // passed by value (kernel arguments), <= 64 filters
    MultiFilter f[kMaxMulti];
    uint32_t nf;
    uint32_t pad;
};

constexpr int kMaxMany = 32;
constexpr uint64_t kLdsFilterBytes = 160 * 1024;  // a filter whose word array fits one CU's LDS
struct ManyFilter {
    uint32_t *words;
    uint64_t nwords;
    uint64_t key_begin, key_end;
    ModArg md;
};
struct ManyArg {
    ManyFilter f[kMaxMany];
    uint32_t nf;
    uint32_t pad;
};

// One registered SSTable filter, in LSM lookup order (k_multiget).
struct RegSlot {
    const uint32_t *words;
    ModArg md;
    uint32_t min_off, min_len, max_off, max_len;  // key range bytes in the registry's range buffer
    int32_t level;
    uint32_t slot;          // bit of the output mask
    int32_t gbit;           // L0 group member: its bit in the group table's entries, else -1
    uint32_t pad;
    uint64_t min_be[2];     // first 16 bytes of MinKey / MaxKey as big-endian words (zero padded)
    uint64_t max_be[2];
};
struct RegLayout {          // slot index ranges per level (lookup order) + shape flags
    uint32_t lo[5], hi[5];
    uint32_t nonoverlap;    // bit L: level L's files are disjoint and in MinKey order (bisection exact)
    uint32_t all_k7_m32;    // every filter has k == 7 and m < kM32Limit (2^31)
    // L0 group: the L0 files sharing one (m, k), every key tests all of them, as one bit-interleaved
    // table (entry p = bit p of each member, l0b bits per entry): one gather per position for the
    // whole group.  l0g == 0: none.
    const uint32_t *l0tab;
    ModArg l0md;
    uint32_t l0g, l0b;
};
constexpr uint32_t kL0GroupMax = 32;
struct L0Members {          // builder argument: the group's word arrays, in bit order
    const uint32_t *w[kL0GroupMax];
};
uint64_t l0_table_words(uint64_t m, uint32_t bits);
hipError_t launch_l0_table(const L0Members &mem, uint32_t g, uint32_t bits, uint64_t m, uint32_t *table,
                           hipStream_t s);
// seb_codec.hip: shard routing (FNV-1a32) and WAL CRC32
hipError_t launch_route(const KeyBatch &kb, uint32_t bits, uint16_t *shard, uint32_t *hash, hipStream_t s);
uint64_t route_workspace_bytes(uint64_t n, uint32_t bits);
hipError_t launch_route_partition(const KeyBatch &kb, uint32_t bits, uint32_t *perm, uint64_t *shard_begin,
                                  uint16_t *shard_out, void *ws, uint64_t ws_bytes, hipStream_t s);
hipError_t launch_wal_crc(uint8_t *data, const uint64_t *off, uint64_t n, int mode, uint32_t *crc, uint8_t *ok,
                          hipStream_t s);
// The scatter-free order's segment tables (multiget_order 1): segment s = b * C + sc is bucket b's
// run of 4096-key super-chunk sc; seg[s] = its first sorted row (low 32 bits, non-decreasing in s)
// | (sc << 12 | the run's offset in the super-chunk's bucket-sorted keys) << 32; half[s] = its keys
// in the super-chunk's first 2048-key chunk; wstart[w] = the segment of row 64 w.
struct MgSeg {
    const uint64_t *seg = nullptr;  // null: rows are read linearly (or through key_order)
    const uint32_t *wstart = nullptr;
    const uint32_t *half = nullptr;
    uint32_t nseg = 0, C = 0, nb = 0, pad = 0;
    uint32_t part_lo = 0;  // the partition level's first lookup-ordered slot: bucket b >= 1's file is part_lo + b - 1
    // per bucket b and level L = 1..4, brange[4 b + L - 1] = A | B << 16: a disjoint level's bisection for a
    // key of bucket b ends in [lo + A, lo + B] (the files whose MinKey can bound the bucket's keys); null: none
    const uint32_t *brange = nullptr;
};
// cand != null: the list form (cap u16 slots per key, any nslots) instead of masks.
constexpr uint32_t kRegMaxFiles = 4096;  // registry capacity (u16 slot ids, 0xFFFF = none)
// Answer j goes to row j of maybe / cand; key_order != null: key j is read as key key_order[j] of kb.
hipError_t launch_multiget(const KeyBatch &kb, const RegSlot *slots, uint32_t nslots, const RegLayout &lay,
                           const uint8_t *ranges, uint64_t *maybe, uint16_t *cand, uint32_t cap, hipStream_t s,
                           const uint32_t *key_order, const MgSeg &seg = MgSeg{}, bool narrow = false);
// Key-range order for MultiGet: buckets = files of slots [lo, hi) (a disjoint, MinKey-ordered
// level) with MinKey <= key.  The MultiGet then answers into mo.answers (sorted rows) and
// launch_multiget_unpermute writes them to the caller's output in batch order.
constexpr uint32_t kMgMaxBuckets = 1025;
struct MgOrder {
    bool active = false;          // false: the level does not apply; answer in batch order directly
    uint64_t n = 0;
    uint32_t nb = 0, bits = 0;            // buckets of the partition level, bits of a bucket id
    const void *bucket = nullptr;         // each key's bucket, in batch order (u8 when bucket8, else u16)
    bool bucket8 = false;
    const uint32_t *runs = nullptr;       // per chunk and bucket: the first sorted row of its run
    const uint32_t *key_order = nullptr;  // batches that are not moved: key index of each sorted row
    const uint8_t *keys = nullptr;        // aligned fixed 16-B batches: the keys moved into that order
    void *answers = nullptr;              // n * answer_bytes: the MultiGet's answers in sorted rows
    MgSeg seg;                            // the scatter-free order: keys read through segments
    int narrow = 0;  // sorted rows held narrow: 1 u32 masks (slots all < 32), 2 u8 list rows (slots all < 255)
};
// Aligned fixed 16-B batches are sorted by bucket inside each chunk and read through the segment
// tables (multiget_order 1) or moved into that order (multiget_order 2; 16 B more per key), others
// get an index.  nb: the partition level's bucket count (its files + 1).
bool multiget_order_moves(const KeyBatch &kb);
uint64_t multiget_order_bytes(const KeyBatch &kb, uint64_t answer_bytes, uint32_t nb);
hipError_t launch_multiget_order(const KeyBatch &kb, const RegSlot *slots, uint32_t lo, uint32_t hi,
                                 const uint8_t *ranges, void *ws, MgOrder *mo, hipStream_t s);
hipError_t launch_multiget_unpermute(const MgOrder &mo, void *out, uint64_t answer_bytes, hipStream_t s);

// Process-wide tuning knobs (seb_set_option): the auto-dispatch thresholds, the build algorithm,
// and the few shape choices tests force to cover both paths.  Variants measured slower were
// removed from the kernels (DESIGN.md 8 keeps their numbers).
struct Options {
    int build_algo = 0;           // 0 auto, 1 device-scope atomics, 2 radix-partitioned (bucketed), 3 LDS-resident
                                  // filter (atomic merge), 4 LDS images + OR kernel
    int multi_interleave = 1;     // multi-filter probe: interleaved table when filters share (m, k)
    int multiget_order = 1;       // MultiGet: probe batches of >= 64K keys in key-range order (1: aligned 16-B keys
                                  // sorted within chunks and read through segment tables; 2: moved across the
                                  // batch by a scatter pass, round 5's form) or in batch order (0)
    int multiget_l0_group = 1;    // MultiGet: L0 files of one (m, k) tested through one interleaved table
    int multiget_xcd = 1;         // MultiGet: the blocks sharing an XCD walk one contiguous eighth of the batch
                                  // (1, default: 575 vs 596 us per 10M-key k_multiget on 28 files), or not (0)
    int probe_compact = 1;        // phased probe from keys: later phases read only the live keys' words
    int scatter_bins = 1;         // bucketed build, k == 7: scatter through fixed LDS bins, pipelined against the
                                  // hashing (1), or the counting sort (0)
    uint64_t varlen_prehash_min_keys = 1u << 16;  // LDS-staged pre-hash from this many var-length keys
    uint64_t bucket_min_keys = 100000;  // auto: bucketed build from this many keys on
    uint64_t lds_min_keys = 75000;      // auto: LDS-resident build (filter <= 160 KiB) from this many keys on
    uint32_t many_splits = 0;     // batched small-filter build: workgroups per filter (0 = auto, one per CU)
    int probe_phases = 0;         // phased probe: number of filter ranges (0 = one per 4 MiB of filter)
    unsigned grid_cap = 1u << 20; // grid-stride kernels: most workgroups per launch
    uint64_t workspace_limit_mib = 0;  // library scratch cap (0 = none); a larger request fails SEB_ERR_NOMEM
    uint64_t multiget_piece_mib = 1024;  // registry MultiGet: a key-range ordered walk's scratch per piece of the batch
    int varlen_tail = 1;          // pre-hash: the 64 * v longest keys of a workgroup of 512 - 64 * v keys on
                                  // 2 * v waves of 32 keys, a lane per chain (v = 1, 2, 3), or one key per
                                  // lane throughout (0, measured slower: DESIGN.md 5.5)
    int cpu_fallback = 1;         // Go API mirror: a build/probe whose device path fails (SEB_ERR_DEVICE/NOMEM)
                                  // is done on the filter's host copy instead (seb_fallback_count)
    int fault_inject = 0;         // test only: the Go API mirror's device path fails with SEB_ERR_DEVICE
};
Options &options();

hipError_t launch_build(const KeyBatch &kb, uint32_t *words, const ModArg &md, hipStream_t s);
// Copy `bytes` of filter words to host-pinned memory (both 16-B aligned) with a kernel.
hipError_t launch_copy_out(const uint32_t *words, uint8_t *host, uint64_t bytes, hipStream_t s);
// Zero `bytes` (a multiple of 16) of filter words.
hipError_t launch_clear_words(uint32_t *words, uint64_t bytes, hipStream_t s);
bool bucketed_supported(uint64_t m, uint32_t k);
uint64_t bucketed_workspace_bytes(uint64_t n, uint64_t m, uint32_t k);
// Build from packed residues (k == 7, m < 2^kPackBits); same workspace as launch_build_bucketed.
// ovf != null: a fresh build: `words` (seb_words_bytes) need no clear and are written whole;
// `ovf` is an all-zero bitmap of the same size, left all zero again.
hipError_t launch_build_bucketed_packed(const uint64_t *packed, uint64_t n, uint32_t *words, const ModArg &md,
                                        void *ws, uint64_t ws_bytes, hipStream_t s, uint32_t *ovf = nullptr);
hipError_t launch_build_bucketed(const KeyBatch &kb, uint32_t *words, const ModArg &md, void *ws, uint64_t ws_bytes,
                                 hipStream_t s, uint32_t *ovf = nullptr);
// 1 = atomic, 2 = bucketed, 3 = LDS-resident (atomic merge), 4 = LDS images + OR kernel, for a
// batch of n keys into an m-bit filter.
int choose_build_algo(uint64_t n, uint64_t m, uint32_t k);
// The image build (algo 4): scratch bytes, and the launch.  fresh: the filter words hold nothing
// yet, so they are written rather than OR-ed (and need no clear beforehand).
uint64_t image_workspace_bytes(uint64_t n, uint64_t m);
hipError_t launch_build_images(const KeyBatch &kb, uint32_t *words, const ModArg &md, void *ws, uint64_t ws_bytes,
                               bool fresh, hipStream_t s);
hipError_t launch_probe(const KeyBatch &kb, const uint32_t *words, const ModArg &md, uint8_t *out, hipStream_t s);
hipError_t launch_probe_multi(const KeyBatch &kb, const MultiArg &ma, void *mask, uint32_t mask_bytes,
                              hipStream_t s);
// Pre-hash a variable-length batch into one uint4 (h1, h2) per key (LDS-staged byte walk).
hipError_t launch_hash_varlen(const KeyBatch &kb, uint4 *hashes, hipStream_t s);
// The same pre-hash writing packed residues for filter md (k == 7, m < 2^kPackBits) instead.
hipError_t launch_hash_varlen_packed(const KeyBatch &kb, const ModArg &md, uint64_t *packed, hipStream_t s);

// Interleaved multi-filter probe (all filters share (m, k), k == 7, m < 2^31): scratch bytes
// needed for the per-call table (0 = not applicable), and the launch (table in `ws`).
uint64_t interleaved_bytes(const MultiArg &ma, uint32_t mask_bytes);
hipError_t launch_probe_interleaved(const KeyBatch &kb, const MultiArg &ma, void *mask, uint32_t mask_bytes, void *ws,
                                    hipStream_t s);
// The same over packed residues (all filters share (m, k), k == 7, m < 2^kPackBits); `ws` holds
// the table (interleaved_table_bytes).
hipError_t launch_probe_interleaved_packed(const uint64_t *packed, uint64_t n, const MultiArg &ma, void *mask,
                                           uint32_t mask_bytes, void *ws, hipStream_t s);
hipError_t launch_build_many_lds(const KeyBatch &kb, const ManyArg &ma, uint32_t lds_bytes, hipStream_t s);

// Packed residues (k == 7, m < 2^kPackBits): 8 bytes per key instead of the key itself.
constexpr uint32_t kPackBits = 29;
hipError_t launch_pack_residues(const KeyBatch &kb, const ModArg &md, uint64_t *packed, hipStream_t s);
// Narrow packed residues (k == 7, m < 2^kPack6Bits, e.g. the 958,506-bit compaction filters): the
// same three fields in 48 bits (21-bit r0, 21-bit b, 6 carries), 6 bytes per key, stored in blocks
// of 64 keys (64 u32 low words, then 64 u16 high words: kPack6Block bytes), so a wave moves a block
// with two coalesced loads and a slice starting at a multiple of 64 keys is one contiguous range.
constexpr uint32_t kPack6Bits = 21;
constexpr uint32_t kPack6Block = 384;
constexpr uint64_t packed6_bytes(uint64_t n) { return ((n + 63) / 64) * kPack6Block; }
hipError_t launch_pack_residues6(const KeyBatch &kb, const ModArg &md, uint8_t *packed6, hipStream_t s);
hipError_t launch_probe_interleaved_packed6(const uint8_t *packed6, uint64_t n, const MultiArg &ma, void *mask,
                                            uint32_t mask_bytes, void *ws, hipStream_t s);
// out[w] = OR over s < nslices of in[s * slice_words + w] (the sharded build's reduction step)
hipError_t launch_or_slices(const uint32_t *in, uint32_t nslices, uint64_t slice_words, uint32_t *out, hipStream_t s);
hipError_t launch_probe_packed(const uint64_t *packed, uint64_t n, const uint32_t *words, const ModArg &md,
                               uint8_t *out, hipStream_t s);
// Phased probe (the default for k == 7, m < 2^kPackBits, 4-byte aligned out): one launch per word
// range of the filter (probe_phase_count of them); `packed` is 8*n bytes of scratch.
uint64_t probe_phase_count(uint64_t m);
// kb == nullptr: probe the packed words themselves (no phase 0 hashing).
hipError_t launch_probe_phased(const KeyBatch *kb, uint64_t n, const uint32_t *words, const ModArg &md, uint8_t *out,
                               uint64_t *packed, hipStream_t s);
// The phased probe from keys with compacted later phases (probe_compact_bytes of 16-B aligned
// scratch in `ws`; needs probe_phase_count(m) >= 2).
uint64_t probe_compact_bytes(uint64_t n);
hipError_t launch_probe_compact(const KeyBatch &kb, const uint32_t *words, const ModArg &md, uint8_t *out, void *ws,
                                hipStream_t s);
// The same from a variable-length batch, phase 0 fused into the LDS-staged pre-hash.
hipError_t launch_probe_compact_varlen(const KeyBatch &kb, const uint32_t *words, const ModArg &md, uint8_t *out,
                                       void *ws, hipStream_t s);
hipError_t launch_hash_varlen_phase0(const KeyBatch &kb, const ModArg &md, const uint32_t *words, uint64_t *rows,
                                     ulonglong2 *recs, uint32_t hi, hipStream_t s);
// The same from a batch of packed residues (the pre-hashed variable-length batch, a broadcast batch).
hipError_t launch_probe_compact_packed(const uint64_t *packed, uint64_t n, const uint32_t *words, const ModArg &md,
                                       uint8_t *out, void *ws, hipStream_t s);
// Probe from keys that also writes the batch's packed residues.
hipError_t launch_probe_emit(const KeyBatch &kb, const uint32_t *words, const ModArg &md, uint8_t *out,
                             uint64_t *packed, hipStream_t s);

}  // namespace seb
