/*
 * oracle_check.c — drives the CPU restatement (oracle/bloom_oracle.c, oracle/codec_oracle.c) under
 * the host sanitizers (TEST INFRASTRUCTURE: tests/test_sanitize.py builds it with
 * -fsanitize=address,undefined and with -fsanitize=thread).  SURVEY.md §5: the reference's only
 * race/sanitizer story is `go test -race`; here the checker itself is run memory-, UB- and
 * race-checked on the golden cases.
 *
 *   oracle_check OUTDIR THREADS N...   for each N: the filter of key16(0..N-1) sized
 *       NewBloomFilter(N, 0.01) (lsm/bloom.go:19-41) built by Add (single thread) and by the
 *       THREADS-way build, which must agree; writes OUTDIR/enc_N.bin (Encode, lsm/bloom.go:96-102)
 *       and OUTDIR/ans_N.bin (MayContain of the probe rule, lsm/bloom.go:82-92), single and
 *       THREADS-way answers must agree; Decode round trip and Decode of < 12 bytes (nil).
 *   stdout: "fnv x<hex key> <fnv1a> <fnv1>" for each hex key on stdin, then "crc <hex>" of
 *       "123456789" and "ok".
 */
#include <inttypes.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

int oracle_params(int64_t n, double p, uint64_t *m_out, uint32_t *k_out);
uint64_t oracle_fnv1a64(const uint8_t *key, uint64_t len);
uint64_t oracle_fnv1_64(const uint8_t *key, uint64_t len);
void oracle_build(uint8_t *bits, uint64_t m, uint32_t k, const uint8_t *data, const uint64_t *offsets,
                  uint32_t stride, uint64_t n);
void oracle_probe(const uint8_t *bits, uint64_t m, uint32_t k, const uint8_t *data, const uint64_t *offsets,
                  uint32_t stride, uint64_t n, uint8_t *out);
void oracle_encode(const uint8_t *bits, uint64_t nbytes, uint64_t m, uint32_t k, uint8_t *out);
int oracle_decode(const uint8_t *data, uint64_t len, uint64_t *m, uint32_t *k);
int oracle_probe_mt(const uint8_t *bits, uint64_t m, uint32_t k, const uint8_t *data, const uint64_t *offsets,
                    uint32_t stride, uint64_t n, uint8_t *out, int threads);
int oracle_build_mt(uint8_t *bits, uint64_t m, uint32_t k, const uint8_t *data, const uint64_t *offsets,
                    uint32_t stride, uint64_t n, int threads);
uint32_t codec_crc32_ieee(const uint8_t *p, uint64_t len);

static void key16(uint64_t i, uint8_t *out) { /* common/benchmark/keygen.go:89-109 at KeySize 16 */
    char buf[32];
    snprintf(buf, sizeof buf, "user%010" PRIu64, i);
    memcpy(out, buf, 14);
    out[14] = (uint8_t)(i & 0xff);
    out[15] = (uint8_t)((i + 1) & 0xff);
}

static void die(const char *what) {
    fprintf(stderr, "oracle_check: %s\n", what);
    exit(1);
}

static void write_file(const char *dir, const char *name, uint64_t n, const void *p, uint64_t len) {
    char path[4096];
    snprintf(path, sizeof path, "%s/%s_%" PRIu64 ".bin", dir, name, n);
    FILE *f = fopen(path, "wb");
    if (!f || (len && fwrite(p, 1, len, f) != len)) die(path);
    fclose(f);
}

int main(int argc, char **argv) {
    if (argc < 4) die("usage: oracle_check OUTDIR THREADS N...");
    const int threads = atoi(argv[2]);
    char line[4096];
    while (fgets(line, sizeof line, stdin)) {  /* FNV known answers */
        size_t l = strcspn(line, "\r\n");
        line[l] = 0;
        uint8_t key[2048];
        size_t kl = l / 2;
        for (size_t j = 0; j < kl; ++j) {
            unsigned v;
            if (sscanf(line + 2 * j, "%2x", &v) != 1) die("hex");
            key[j] = (uint8_t)v;
        }
        printf("fnv x%s %016" PRIx64 " %016" PRIx64 "\n", line, oracle_fnv1a64(key, kl), oracle_fnv1_64(key, kl));
    }
    for (int a = 3; a < argc; ++a) {
        const uint64_t n = strtoull(argv[a], 0, 10);
        uint64_t m;
        uint32_t k;
        if (oracle_params((int64_t)n, 0.01, &m, &k)) die("params");
        const uint64_t nb = (m + 7) / 8;
        uint8_t *keys = malloc(16 * (n ? n : 1)), *probe = malloc(16 * (n ? n : 1));
        uint8_t *bits = calloc(nb ? nb : 1, 1), *bits_mt = calloc(nb ? nb : 1, 1);
        uint8_t *ans = malloc(n ? n : 1), *ans_mt = malloc(n ? n : 1);
        uint8_t *enc = malloc(12 + nb);
        if (!keys || !probe || !bits || !bits_mt || !ans || !ans_mt || !enc) die("alloc");
        for (uint64_t i = 0; i < n; ++i) {
            key16(i, keys + 16 * i);
            key16(i % 2 == 0 ? i : n + i, probe + 16 * i);  /* even q present, odd q absent */
        }
        oracle_build(bits, m, k, keys, NULL, 16, n);
        if (oracle_build_mt(bits_mt, m, k, keys, NULL, 16, n, threads)) die("build_mt");
        if (memcmp(bits, bits_mt, nb)) die("multi-threaded build differs");
        oracle_encode(bits, nb, m, k, enc);
        uint64_t dm;
        uint32_t dk;
        if (oracle_decode(enc, 12 + nb, &dm, &dk) || dm != m || dk != k) die("decode round trip");
        if (oracle_decode(enc, 11, &dm, &dk) == 0) die("decode of 11 bytes must fail (Go: nil)");
        oracle_probe(bits, m, k, probe, NULL, 16, n, ans);
        if (oracle_probe_mt(bits, m, k, probe, NULL, 16, n, ans_mt, threads)) die("probe_mt");
        if (memcmp(ans, ans_mt, n)) die("multi-threaded probe differs");
        for (uint64_t i = 0; i < n; i += 2)
            if (!ans[i]) die("false negative");
        write_file(argv[1], "enc", n, enc, 12 + nb);
        write_file(argv[1], "ans", n, ans, n);
        free(keys), free(probe), free(bits), free(bits_mt), free(ans), free(ans_mt), free(enc);
    }
    printf("crc %08x\nok\n", codec_crc32_ieee((const uint8_t *)"123456789", 9));
    return 0;
}
