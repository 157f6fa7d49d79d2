/*
 * seb_bloom.h — C ABI of the MI355X-native bloom-filter build + probe path.
 *
 * Drop-in boundary for intellect4all/storage-engines lsm/bloom.go.  The reference is Go; its
 * callers are lsm/sstable_builder.go:30,53,217 (build at flush/compaction) and
 * lsm/sstable.go:129,206 (decode at open, probe on Get).  A cgo shim
 * (storage-engines_amd/go/lsm/bloom.go) binds the "Go API mirror" group
 * below one-for-one, so those callers compile unchanged.  Every entry point takes plain C types
 * (pointers and sizes); no torch or HIP types appear in a signature (streams are `void*`
 * holding a hipStream_t, NULL = the library's own stream / the null stream).
 *
 * Results are bit-exact with the reference: identical bit array (byte h>>3, bit h&7 — on the
 * little-endian device this is u32 word h>>5, bit h&31) and identical MayContain answers.
 *
 * Errors: every int-returning function returns SEB_OK (0) or a negative SEB_ERR_* code, and
 * seb_last_error() gives a thread-local message.  The reference has no error returns (bad input
 * panics or yields nil); the Go shim turns a negative code into the same panic.  The Go API
 * mirror (seb_filter_*) does not fail for want of a device: a build or batched probe whose device
 * path returns SEB_ERR_DEVICE / SEB_ERR_NOMEM is done on the filter's host copy instead (option
 * "cpu_fallback", default on), counted by seb_fallback_count(), the first one per process also
 * logged to stderr.  SEB_ERR_INTERNAL (a failed launch, a kernel fault) is never absorbed.  The
 * fallback needs the filter's host copy to be current: a filter over 64 MiB of bits whose device
 * copy is ahead of it (built on the device with the host mirror off) reports the error instead.
 * Every other entry point (device-resident, host-buffer, registry) reports the error.
 */
#ifndef SEB_BLOOM_H
#define SEB_BLOOM_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SEB_ABI_VERSION 1

enum seb_status {
    SEB_OK = 0,
    SEB_ERR_INVALID = -1, /* bad argument; the reference would panic (e.g. % 0, index out of range) */
    SEB_ERR_DEVICE = -2,  /* no usable gfx950 device: none, no driver, no code object, runtime down */
    SEB_ERR_NOMEM = -3,   /* host or device allocation failed (or over workspace_limit_mib) */
    SEB_ERR_RANGE = -4,   /* sizing outside the reference's defined float->int range */
    SEB_ERR_SHORT = -5,   /* a decoded filter's bits are shorter than ceil(numBits/8) */
    SEB_ERR_INTERNAL = -6, /* any other HIP error: a rejected launch, a kernel fault, a library bug */
};

/* A batch of keys.  Fixed-length keys: offsets == NULL, key i = data[i*stride, (i+1)*stride).
 * Variable-length keys: offsets holds n+1 non-decreasing byte offsets (offsets[0] may be != 0),
 * key i = data[offsets[i], offsets[i+1]).  Host or device memory per the entry point. */
typedef struct seb_keys {
    const uint8_t *data;
    const uint64_t *offsets;
    uint64_t n;
    uint32_t stride;
    uint32_t reserved; /* must be 0 */
} seb_keys;

/* One filter for the multi-filter probe.  `bits` is host bytes (ceil(num_bits/8)) for
 * seb_probe_multi and device u32 words (seb_words_bytes(num_bits) bytes) for
 * seb_dev_probe_multi. */
typedef struct seb_filter_ref {
    const void *bits;
    uint64_t num_bits;
    uint32_t num_hashes;
    uint32_t reserved; /* must be 0 */
} seb_filter_ref;

/* ---------------------------------------------------------------- sizing (host only) ---- */

/* m and k exactly as NewBloomFilter computes them (lsm/bloom.go:19-31): float64 Go math.Log,
 * const-folded Ln2*Ln2, Ceil, k forced to >= 1.  n == 0 gives m = 0, k = 1 (as in Go). */
int seb_params(int64_t expected_keys, double false_positive_rate, uint64_t *num_bits,
               uint32_t *num_hashes);
/* ceil(m/8): the reference's len(bits) (lsm/bloom.go:34). */
uint64_t seb_num_bytes(uint64_t num_bits);
/* Bytes of the device word array for m bits: ceil(m/128)*16 (u32 words, 16-B padded, pad = 0). */
uint64_t seb_words_bytes(uint64_t num_bits);

int seb_abi_version(void);
/* Process-wide tuning knobs (results never change, only speed):
 *   "build_algo"      0 auto, 1 device-scope atomic OR, 2 radix-partitioned LDS build, 3 the whole
 *                     filter in one CU's LDS (word array <= 160 KiB), keys split over workgroups
 *                     (atomic merge), 4 LDS images of the whole filter + an OR kernel (<= 160 KiB)
 *                     Auto: 4 from lds_min_keys keys while the word array fits 160 KiB (3 when
 *                     the words are not 16-B aligned), 2 from bucket_min_keys keys for larger
 *                     filters, 1 below those
 *   "bucket_min_keys" auto build_algo: radix-partitioned from this many keys on
 *   "lds_min_keys"    auto build_algo: LDS-resident filter (<= 160 KiB) from this many keys on
 *   "many_splits"     batched small-filter build: workgroups per filter (0 = auto)
 *   "probe_phases"    k == 7, m < 2^29 probes: filter ranges of the phased probe, one launch each
 *                     (0 = one per 4 MiB of filter; 1 = the single-launch sliced probe)
 *   "probe_compact"   phased probe: later phases read only the live keys' packed words, kept
 *                     compacted per 64-key group (1, default), or every key's (0)
 *   "scatter_bins"    radix-partitioned build, k == 7, 512-2275 buckets (m ~ 33.5M-149M bits):
 *                     positions placed through fixed per-bucket LDS bins, the claims pipelined
 *                     against the hashing (1, default), or by a counting sort (0)
 *   "multi_interleave" multi-filter probes with shared (m, k): bit-transposed table (0/1)
 *   "multiget_order"  registry MultiGet walks batches of >= 64K keys in key-range order (1, default:
 *                     aligned 16-B keys sorted by bucket within 2048-key chunks and read through
 *                     segment tables; 2: moved across the batch by a scatter pass) or batch order (0)
 *   "multiget_piece_mib" registry MultiGet: a batch whose key-range order would need more scratch
 *                     than this (MiB, default 1024) is walked in pieces of whole 2048-key chunks
 *   "multiget_l0_group" registry MultiGet tests the L0 files that share (m, k) through one
 *                     bit-interleaved table, one gather per position for all of them (1, default)
 *   "multiget_xcd"    registry MultiGet: the workgroups that share an XCD walk one contiguous eighth of
 *                     the (key-range ordered) batch, so each XCD's L2 holds its own stretch's filters
 *                     (1, default), or blocks walk the batch in launch order (0)
 *   "varlen_prehash_min_keys"  variable-length batches of this many keys are pre-hashed in LDS
 *   "varlen_tail"     pre-hash: v = 1 (default), 2, 3: workgroups of 512 - 64 v keys whose 64 v longest
 *                     keys run on 2 v waves of 32 keys, one lane per FNV chain; 0: 448 keys, one key per
 *                     lane throughout
 *   "grid_cap"        maximum workgroups of the grid-stride kernels
 *   "workspace_limit_mib"  cap on library scratch and a context's build scratch (0 = none); a
 *                     request above it fails with SEB_ERR_NOMEM (MultiGet's key-range order then
 *                     falls back to batch order; the Go API mirror's build to its CPU fallback)
 *   "cpu_fallback"    Go API mirror: on a device failure build / probe on the host copy (1, default)
 *                     or return the error (0)
 *   "fault_inject"    test only: the Go API mirror's device path fails with SEB_ERR_DEVICE (1) or
 *                     SEB_ERR_INTERNAL (2), or not (0)
 * Environment variables SEB_<NAME> (upper case) set the initial values. */
int seb_set_option(const char *name, int64_t value);
int seb_get_option(const char *name, int64_t *value);
const char *seb_last_error(void);
/* 0 if a gfx950 device is usable, else SEB_ERR_DEVICE (message in seb_last_error). */
int seb_device_check(int device);

/* ------------------------------------------------- device-resident entry points ---------- */
/* All pointers are device memory; work is enqueued on `stream` and NOT synchronised.
 * seb_dev_build ORs the keys into `words` (clear first with seb_dev_clear for a fresh filter),
 * the device form of the reference's Add loop (sstable_builder.go:53 -> bloom.go:70-77). */
int seb_dev_clear(uint32_t *words, uint64_t num_bits, void *stream);
int seb_dev_build(const seb_keys *keys, uint32_t *words, uint64_t num_bits, uint32_t num_hashes,
                  void *stream);
/* A new filter from `keys` (NewBloomFilter + Add per key): `words` (seb_words_bytes) need not be
 * cleared; every word is written.  The radix-partitioned build and the LDS image build write them
 * whole instead of clearing and OR-ing; other build paths clear first.  Device builds take word
 * arrays aligned to 4 B; 16-B aligned ones (any hipMalloc / torch allocation) take the 16-B
 * clear and the image build, others hipMemsetAsync and the LDS-filter build. */
int seb_dev_build_fresh(const seb_keys *keys, uint32_t *words, uint64_t num_bits, uint32_t num_hashes,
                        void *stream);
/* Same, with caller-owned scratch (graph-capture friendly: no allocation inside the call).
 * seb_dev_build_workspace_size gives the bytes needed for n keys (0: this build needs none). */
uint64_t seb_dev_build_workspace_size(uint64_t n, uint64_t num_bits, uint32_t num_hashes);
int seb_dev_build_ws(const seb_keys *keys, uint32_t *words, uint64_t num_bits, uint32_t num_hashes,
                     void *workspace, uint64_t workspace_bytes, void *stream);
/* out[i] = MayContain(key i) as 0/1 bytes (bloom.go:82-92; Go []bool layout). */
int seb_dev_probe(const seb_keys *keys, const uint32_t *words, uint64_t num_bits, uint32_t num_hashes,
                  uint8_t *out, void *stream);
/* Packed residues, for one probe batch shared by several filters of the same (num_bits, num_hashes)
 * (multi-GPU: hash once on the root, broadcast 8 bytes per key instead of the key).  Requires
 * num_hashes == 7 and num_bits < 2^29.  packed[i] = r0 | b << 29 | carries << 58 with
 * r0 = hash1 mod m, b = hash2 mod m and bit q-1 of carries set when hash1 + q*hash2 wraps 2^64 at
 * step q (q = 1..6); seb_dev_probe_packed gives the answers seb_dev_probe gives for the keys
 * (MayContain of lsm/bloom.go:82-92). */
int seb_dev_pack_residues(const seb_keys *keys, uint64_t num_bits, uint32_t num_hashes, uint64_t *packed,
                          void *stream);
int seb_dev_probe_packed(const uint64_t *packed, uint64_t n, const uint32_t *words, uint64_t num_bits,
                         uint32_t num_hashes, uint8_t *out, void *stream);
/* Multi-filter probe of packed residues (seb_dev_probe_multi's mask layout); every filter must
 * have the packed batch's (num_bits, num_hashes). */
int seb_dev_probe_multi_packed(const uint64_t *packed, uint64_t n, const seb_filter_ref *filters, uint32_t num_filters,
                               void *mask, uint32_t mask_bytes, void *stream);
/* Narrow packed residues (6 bytes per key) for num_hashes == 7 and num_bits < 2^21, e.g. the
 * compaction-sized filters of lsm/compaction.go:253,286 (m = 958,506): the same three fields as
 * seb_dev_pack_residues at 21 / 21 / 6 bits, v = r0 | b << 21 | carries << 42, stored in blocks of
 * 64 keys (key i in block i / 64): 64 little-endian u32 low words, then 64 u16 high halves, 384
 * bytes per block; the buffer holds seb_packed6_bytes(n) bytes and must be 4-byte aligned.  A slice
 * of the batch that starts at a multiple of 64 keys is the contiguous byte range from its first
 * block, so a batch split in 64-key multiples travels as plain byte ranges (a quarter fewer bytes
 * over xGMI than the 8-byte form).  seb_dev_probe_multi_packed6 gives the masks
 * seb_dev_probe_multi gives for the keys. */
uint64_t seb_packed6_bytes(uint64_t n);
int seb_dev_pack_residues6(const seb_keys *keys, uint64_t num_bits, uint32_t num_hashes, void *packed6, void *stream);
int seb_dev_probe_multi_packed6(const void *packed6, uint64_t n, const seb_filter_ref *filters, uint32_t num_filters,
                                void *mask, uint32_t mask_bytes, void *stream);
/* seb_dev_probe plus the batch's packed residues in one pass (the broadcast root's probe). */
int seb_dev_probe_emit_packed(const seb_keys *keys, const uint32_t *words, uint64_t num_bits, uint32_t num_hashes,
                              uint8_t *out, uint64_t *packed, void *stream);
/* Multi-filter probe: bit f of mask[i] = MayContain of filters[f] on key i.  mask_bytes is the
 * width of one mask element (1, 2, 4 or 8) and must cover num_filters bits (<= 64). `filters`
 * is a HOST array whose .bits are device word arrays. */
int seb_dev_probe_multi(const seb_keys *keys, const seb_filter_ref *filters, uint32_t num_filters,
                        void *mask, uint32_t mask_bytes, void *stream);
/* Batched build of many independent filters in one launch (compaction output files,
 * lsm/compaction.go:286): keys [key_begin[f], key_begin[f+1]) of `keys` go into filter f.
 * `filters` is a HOST array whose .bits are device word arrays (cleared by the caller);
 * key_begin is a HOST array of num_filters+1 entries. */
int seb_dev_build_many(const seb_keys *keys, const uint64_t *key_begin, const seb_filter_ref *filters,
                       uint32_t num_filters, void *stream);

/* Sharded build of one filter: every rank ORs its key shard into a partial filter,
 * an all-to-all hands rank g the G partials of word slice g (slice after slice), and this call
 * ORs them: out[w] = OR_s slices[s * slice_words + w].  RCCL has no bitwise-OR reduction, so the
 * reduce step of the exchange runs here.  Device pointers; out may not overlap slices. */
int seb_dev_or_slices(const uint32_t *slices, uint32_t num_slices, uint64_t slice_words, uint32_t *out, void *stream);

/* Small device/stream helpers for hosts without their own HIP binding (ctypes, cgo). */
int seb_dev_alloc(void **ptr, uint64_t bytes);
int seb_dev_free(void *ptr);
int seb_host_alloc(void **ptr, uint64_t bytes); /* pinned host memory */
int seb_host_free(void *ptr);
int seb_memcpy_h2d(void *dst, const void *src, uint64_t bytes, void *stream);
int seb_memcpy_d2h(void *dst, const void *src, uint64_t bytes, void *stream);
int seb_stream_sync(void *stream);
/* Timing events created with hipEventDisableSystemFence: a default event's completion fence
 * writes back and invalidates L2 (~15 us between two kernels on gfx950).  elapsed waits for
 * `end`; use only for timing, not to order host reads after device writes. */
int seb_timer_create(void **event);
int seb_timer_record(void *event, void *stream);
int seb_timer_elapsed_ms(void *start, void *end, float *ms);
int seb_timer_destroy(void *event);

/* Library-owned scratch.  Entry points that need scratch and take no workspace argument use
 * grow-only buffers kept per (device, stream); a call holds its stream's buffers until it returns,
 * so calls from several threads on one stream are safe (their launches do not interleave).
 * seb_workspace_bytes: bytes currently held; seb_workspace_release: synchronise the streams that
 * own scratch and free all of it (the next call re-allocates).  A phased probe holds ≈8.3 bytes per
 * key (its compacted packed words and group records); a key-range ordered registry MultiGet
 * 20 bytes per key of aligned 16-B keys (bucket ids, run starts, the moved keys) or 8 for keys it
 * reads through an index, plus its answers in sorted rows (8 bytes per key for masks, 2 per slot for
 * candidate rows); the scratch of a context's (or a registry's) own streams is freed by
 * seb_ctx_destroy (seb_registry_free). */
uint64_t seb_workspace_bytes(void);
int seb_workspace_release(void);

/* ------------------------------------------- host-buffer batched entry points ------------ */
/* Keys and bits in host memory: H2D, kernels and D2H on the context's streams, synchronous.
 * A context owns a device, streams and grow-only scratch buffers; one context per thread
 * (contexts are cheap; calls on one context are serialised by a lock). */
typedef struct seb_ctx seb_ctx;
int seb_ctx_create(int device, seb_ctx **out);
void seb_ctx_destroy(seb_ctx *ctx);

#define SEB_BUILD_FRESH 1u /* `bits` is output only: start from an all-zero filter */
/* bits: ceil(num_bits/8) host bytes, OR-accumulated (or written fresh with SEB_BUILD_FRESH). */
int seb_build(seb_ctx *ctx, const seb_keys *keys, uint8_t *bits, uint64_t num_bits, uint32_t num_hashes,
              uint32_t flags);
int seb_probe(seb_ctx *ctx, const seb_keys *keys, const uint8_t *bits, uint64_t num_bits,
              uint32_t num_hashes, uint8_t *out);
int seb_probe_multi(seb_ctx *ctx, const seb_keys *keys, const seb_filter_ref *filters, uint32_t num_filters,
                    uint64_t *mask);

/* ----------------------------------- Go API mirror (lsm/bloom.go, one call per Go method) ---- */
/* A filter handle.  Its bit array lives in HBM (device-resident filter registry); a host copy is
 * materialised on Encode.  Add() defers: keys are appended to a host arena and built in one
 * batched launch at the next Encode / MayContain / flush (or when the arena passes a size cap).
 * All functions are thread-safe; MayContain may be called concurrently on one filter. */
typedef struct seb_filter seb_filter;

/* NewBloomFilter(expectedKeys, falsePositiveRate)          lsm/bloom.go:19   (NULL + last_error
 * when the sizing leaves the defined range, where Go's behaviour is implementation-defined) */
seb_filter *seb_filter_new(int64_t expected_keys, double false_positive_rate);
void seb_filter_free(seb_filter *f);
/* (*BloomFilter).Add(key)                                    lsm/bloom.go:70 */
int seb_filter_add(seb_filter *f, const uint8_t *key, uint64_t len);
int seb_filter_add_batch(seb_filter *f, const seb_keys *keys);
/* (*BloomFilter).MayContain(key) -> 1 / 0, or < 0 on error  lsm/bloom.go:82 */
int seb_filter_may_contain(seb_filter *f, const uint8_t *key, uint64_t len);
int seb_filter_may_contain_batch(seb_filter *f, const seb_keys *keys, uint8_t *out);
/* (*BloomFilter).Encode() -> 12 + len(bits) bytes           lsm/bloom.go:96 */
uint64_t seb_filter_encoded_size(seb_filter *f);
int seb_filter_encode(seb_filter *f, uint8_t *out, uint64_t cap);
/* DecodeBloomFilter(data) -> NULL when len < 12 (Go: nil)   lsm/bloom.go:105 */
seb_filter *seb_filter_decode(const uint8_t *data, uint64_t len);
/* Accessors and an explicit flush of deferred Adds. */
uint64_t seb_filter_num_bits(const seb_filter *f);
uint32_t seb_filter_num_hashes(const seb_filter *f);
uint64_t seb_filter_pending(seb_filter *f);
int seb_filter_flush(seb_filter *f);
/* How many Go-API-mirror builds / batched probes ran on the host copy because the device path
 * failed (the "cpu_fallback" option); 0 on a healthy GPU. */
uint64_t seb_fallback_count(void);
/* Registry MultiGets (seb_registry_multiget*) that ran in batch order because the key-range
 * order's scratch could not be had (SEB_ERR_NOMEM under "workspace_limit_mib" or the device): the
 * answers are the same, only slower; a benchmark reports it to show which path it measured. */
uint64_t seb_multiget_order_fallbacks(void);

/* ------------------ device-resident filter registry + batched LSM lookup ---- */
/* One registry per LSM instance.  seb_registry_put decodes an SSTable's bloom block (the bytes
 * OpenSSTable reads, lsm/sstable.go:121-129) straight into HBM, with the file's level and
 * [MinKey, MaxKey]; level 0 keeps insertion order, levels 1..4 are ordered by MinKey, as
 * lsm/levels.go:45-63 keeps them.  seb_registry_remove frees it (compaction, lsm/compaction.go).
 * seb_registry_multiget: for each key, bit s of maybe[i] is set when registry slot s is a file
 * LSM.Get would consult for the key (every L0 file; per level 1..4 the first file whose range
 * covers it, lsm/lsm.go:168-198) AND its filter may contain the key; the mask form needs every slot
 * < 64 (a registry that never held more than 64 files).  The list form takes any registry (up to
 * 4096 files, u16 slot ids): row i of cand (cap u16 per key) lists the slots of those files in the
 * order Get visits them (L0 in insertion order, then levels 1..4), padded with 0xFFFF; cap must be
 * >= seb_registry_max_candidates (the L0 file count + the number of non-empty levels 1..4). */
typedef struct seb_registry seb_registry;
seb_registry *seb_registry_new(int device);
void seb_registry_free(seb_registry *reg);
/* returns the slot (>= 0) or < 0 */
int seb_registry_put(seb_registry *reg, uint64_t file_num, int level, const uint8_t *bloom, uint64_t bloom_len,
                     const uint8_t *min_key, uint64_t min_len, const uint8_t *max_key, uint64_t max_len);
int seb_registry_remove(seb_registry *reg, uint64_t file_num);
/* file number and level of every slot (UINT64_MAX / -1 for free slots); returns the file count */
int seb_registry_slots(seb_registry *reg, uint64_t *file_nums, int32_t *levels, uint32_t cap);
int seb_registry_multiget(seb_registry *reg, const seb_keys *keys, uint64_t *maybe);          /* host keys */
int seb_registry_multiget_dev(seb_registry *reg, const seb_keys *keys, uint64_t *maybe, void *stream);
int seb_registry_max_candidates(seb_registry *reg); /* >= 0, or < 0 on error */
int seb_registry_multiget_list(seb_registry *reg, const seb_keys *keys, uint16_t *cand, uint32_t cap); /* host */
int seb_registry_multiget_list_dev(seb_registry *reg, const seb_keys *keys, uint16_t *cand, uint32_t cap,
                                   void *stream);
/* The list form with file numbers instead of slots (host keys): files[i*cap + j] is the file_num of
 * the j-th file Get would read for key i, padded with UINT64_MAX.  Sizing, lookup and slot->file
 * mapping happen under one hold of the registry lock, so a concurrent put/remove (flush,
 * compaction) cannot make rows overflow or a reused slot name the wrong file.  *need (nullable)
 * receives the row width the registry needs now; cap < *need returns SEB_ERR_RANGE (retry). */
int seb_registry_multiget_files(seb_registry *reg, const seb_keys *keys, uint64_t *files, uint32_t cap,
                                uint32_t *need);

/* ---------- hash-index shard routing + WAL record checksums (off the bloom path) ---- */
/* shard[i] = FNV-1a32(key i) & ((1 << shard_bits) - 1), the reference's getShard
 * (hashindex/shard.go:47-52; 256 shards = shard_bits 8).  hash[i] (nullable) = the full FNV-1a32.
 * shard (nullable) is one u16 per key; shard_bits <= 16.  Device pointers. */
int seb_dev_shard_route(const seb_keys *keys, uint32_t shard_bits, uint16_t *shard, uint32_t *hash, void *stream);
/* Stable partition of a key batch by shard: UpdateBatch's distribution step (hashindex/shard.go:104-122).
 * perm = key indices grouped by shard ascending, input order inside a shard; shard s owns
 * perm[shard_begin[s], shard_begin[s+1]) (shard_begin nullable, 2^shard_bits + 1 entries); shard
 * (nullable) as above.  shard_bits <= 12, n < 2^32; workspace of
 * seb_dev_shard_partition_workspace_size bytes.  The reference distributes a Go map, whose order
 * is random: it defines only the set per shard, which this order refines. */
uint64_t seb_dev_shard_partition_workspace_size(uint64_t n, uint32_t shard_bits);
int seb_dev_shard_partition(const seb_keys *keys, uint32_t shard_bits, uint32_t *perm, uint64_t *shard_begin,
                            uint16_t *shard, void *workspace, uint64_t workspace_bytes, void *stream);
/* WAL records (lsm/wal.go:31-62): record i = data[rec_off[i], rec_off[i+1]) =
 * [crc32 u32][seq u64][keySize u32][valueSize u32][deleted u8][key][value], all little-endian,
 * crc = crc32.ChecksumIEEE(record[4:]).  SEB_WAL_CRC: crc[i] only; SEB_WAL_SEAL: also store it in
 * the record (Append, :59-60); SEB_WAL_VERIFY: ok[i] = 1 iff the record is framed (length >= 21
 * and 21 + keySize + valueSize == length) and its stored CRC matches (ReadAll, :98-133).  crc and
 * ok are nullable except ok for VERIFY.  Device pointers. */
enum seb_wal_mode { SEB_WAL_CRC = 0, SEB_WAL_SEAL = 1, SEB_WAL_VERIFY = 2 };
int seb_dev_wal_crc(uint8_t *data, const uint64_t *rec_off, uint64_t n, int mode, uint32_t *crc, uint8_t *ok,
                    void *stream);
/* Host: walk a WAL image's framing as ReadAll does (21-byte header, then keySize + valueSize bytes)
 * into rec_off (cap entries).  *n = complete records; rec_off[0..*n] are their boundaries.
 * SEB_OK if the image ends on a record boundary, SEB_ERR_SHORT if the tail is a truncated header or
 * payload (ReadAll's "failed to read WAL header/data" error), SEB_ERR_INVALID if cap < records + 1. */
int seb_wal_scan(const uint8_t *data, uint64_t bytes, uint64_t *rec_off, uint64_t cap, uint64_t *n);

#ifdef __cplusplus
}
#endif

#endif /* SEB_BLOOM_H */
