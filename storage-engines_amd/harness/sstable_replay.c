/*
 * sstable_replay.c — replays the reference's exact bloom call sequences through the C ABI, the
 * executable stand-in for the cgo shim (storage-engines_amd/go/lsm/bloom.go), since no Go
 * toolchain exists in this pipeline.
 *
 *   flush / compaction build   lsm/sstable_builder.go:30  NewBloomFilter(expectedKeys, 0.01)
 *                              lsm/sstable_builder.go:53  Add(key) once per sorted entry
 *                              lsm/sstable_builder.go:217 Encode() into the bloom block
 *   open + point lookups       lsm/sstable.go:129         DecodeBloomFilter(bloomData)
 *                              lsm/sstable.go:206         MayContain(key) per Get
 *
 * usage: sstable_replay N EXPECTED_KEYS   (N keys key16(0..N-1); probes q < N: even q -> key16(q),
 *        odd q -> key16(N+q)).  Prints one JSON line with sha256(Encode()) and sha256(answers)
 *        for the per-key path and the batched path; exits non-zero if they disagree.
 */
#include <inttypes.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/seb_bloom.h"

#include "harness_common.h"

static void die(const char *what) {
    fprintf(stderr, "%s: %s\n", what, seb_last_error());
    exit(2);
}

int main(int argc, char **argv) {
    if (argc < 3) {
        fprintf(stderr, "usage: %s N EXPECTED_KEYS\n", argv[0]);
        return 2;
    }
    const uint64_t n = strtoull(argv[1], 0, 10);
    const int64_t expected = strtoll(argv[2], 0, 10);
    uint8_t key[16];

    /* SSTableBuilder: New -> Add per sorted entry -> Finish/Encode */
    seb_filter *f = seb_filter_new(expected, 0.01);
    if (!f) die("NewBloomFilter");
    for (uint64_t i = 0; i < n; i++) {
        key16(i, key);
        if (seb_filter_add(f, key, 16) != SEB_OK) die("Add");
    }
    uint64_t esz = seb_filter_encoded_size(f);
    uint8_t *enc = malloc(esz);
    if (seb_filter_encode(f, enc, esz) != SEB_OK) die("Encode");
    char henc[65];
    digest(enc, esz, henc);

    /* OpenSSTable: Decode the bloom block; Get: MayContain per key */
    seb_filter *g = seb_filter_decode(enc, esz);
    if (!g) die("DecodeBloomFilter");
    uint64_t probes = n;
    uint8_t *ans = malloc(probes ? probes : 1), *ans_b = malloc(probes ? probes : 1);
    uint8_t *pk = malloc(16 * (probes ? probes : 1));
    uint64_t positives = 0;
    for (uint64_t q = 0; q < probes; q++) {
        key16(q % 2 == 0 ? q : n + q, pk + 16 * q);
        int r = seb_filter_may_contain(g, pk + 16 * q, 16);
        if (r < 0) die("MayContain");
        ans[q] = (uint8_t)r;
        positives += (uint64_t)r;
        if (q % 2 == 0 && r != 1) {
            fprintf(stderr, "false negative at %" PRIu64 "\n", q);
            return 1;
        }
    }
    seb_keys kb = {pk, NULL, probes, 16, 0};
    if (seb_filter_may_contain_batch(g, &kb, ans_b) != SEB_OK) die("MayContainBatch");
    char hans[65], hans_b[65];
    digest(ans, probes, hans);
    digest(ans_b, probes, hans_b);
    const int same = strcmp(hans, hans_b) == 0;
    printf("{\"n\": %" PRIu64 ", \"expected_keys\": %" PRId64 ", \"num_bits\": %" PRIu64 ", \"num_hashes\": %u, "
           "\"encode_len\": %" PRIu64 ", \"encode_sha256\": \"%s\", \"probe_positives\": %" PRIu64
           ", \"probe_sha256\": \"%s\", \"batch_matches_single\": %s}\n",
           n, expected, seb_filter_num_bits(g), seb_filter_num_hashes(g), esz, henc, positives, hans,
           same ? "true" : "false");
    seb_filter_free(f);
    seb_filter_free(g);
    free(enc), free(ans), free(ans_b), free(pk);
    return same ? 0 : 1;
}
