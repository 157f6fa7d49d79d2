/*
 * bloom_oracle.c — CPU restatement of the reference bloom filter (TEST INFRASTRUCTURE ONLY).
 *
 * This file is the parity CHECKER for the MI355X path.  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load it.  The shipped library (storage-engines_amd/)
 * never links, loads or calls it.
 *
 * What it restates (reference = intellect4all/storage-engines, Go, read as text only):
 *   lsm/bloom.go:19-41   NewBloomFilter      sizing in float64, then make([]byte,(m+7)/8)
 *   lsm/bloom.go:44-48   hash1               Go stdlib hash/fnv New64a (FNV-1a 64)
 *   lsm/bloom.go:50-54   hash2               Go stdlib hash/fnv New64  (FNV-1 64)
 *   lsm/bloom.go:58-67   getHashes           (h1 + uint64(i)*h2) % m, wrapping u64
 *   lsm/bloom.go:70-77   Add                 bits[h/8] |= 1 << (h%8)
 *   lsm/bloom.go:82-92   MayContain          false at the first clear bit
 *   lsm/bloom.go:96-102  Encode              [numBits u64 LE][numHashes u32 LE][bits]
 *   lsm/bloom.go:105-120 DecodeBloomFilter   nil if < 12 bytes, copies the rest verbatim
 *
 * The arithmetic lives in the Go standard library (go1.25.5, go.mod:3), which is not under
 * /root/reference: hash/fnv (offset basis 0xcbf29ce484222325, prime 0x100000001b3) and
 * math.Log / math.Ceil / math.Ln2.  math.Log is restated from Go's portable algorithm
 * (src/math/log.go, the FreeBSD e_log.c reduction), evaluated without FMA contraction
 * (compile with -ffp-contract=off).  Ln2*Ln2 is a Go constant expression, folded exactly
 * and rounded once: 0.48045301391820144 (C's M_LN2*M_LN2 is 1 ulp lower).
 *
 * Parity pins (no Go toolchain exists here or on the GPU box, and the reference's own tests
 * pin only "no false negatives"): Go's hash/fnv golden vectors and the FNV reference KATs
 * (tests/golden/fnv_kats.json), and agreement with the independent numpy restatement
 * (oracle/bloom_np.py) on every committed fixture.  See DESIGN.md "Oracle".
 */
#define _POSIX_C_SOURCE 200809L
#define _DEFAULT_SOURCE  /* MADV_HUGEPAGE */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <pthread.h>
#include <sys/mman.h>

#define FNV_OFFSET 0xcbf29ce484222325ULL
#define FNV_PRIME 0x100000001b3ULL

/* Go: math.Log, src/math/log.go (portable version). */
static double go_log(double x) {
    const double Ln2Hi = 6.93147180369123816490e-01;
    const double Ln2Lo = 1.90821492927058770002e-10;
    const double L1 = 6.666666666666735130e-01;
    const double L2 = 3.999999999940941908e-01;
    const double L3 = 2.857142874366239149e-01;
    const double L4 = 2.222219843214978396e-01;
    const double L5 = 1.818357216161805012e-01;
    const double L6 = 1.531383769920937332e-01;
    const double L7 = 1.479819860511658591e-01;
    if (isnan(x) || (isinf(x) && x > 0)) return x;
    if (x < 0) return NAN;
    if (x == 0) return -INFINITY;
    int ki;
    double f1 = frexp(x, &ki);
    if (f1 < 0.70710678118654757) { /* Go: Sqrt2/2, const-folded */
        f1 *= 2;
        ki--;
    }
    double f = f1 - 1;
    double k = (double)ki;
    double s = f / (2 + f);
    double s2 = s * s;
    double s4 = s2 * s2;
    double t1 = s2 * (L1 + s4 * (L3 + s4 * (L5 + s4 * L7)));
    double t2 = s4 * (L2 + s4 * (L4 + s4 * L6));
    double R = t1 + t2;
    double hfsq = 0.5 * f * f;
    return k * Ln2Hi - ((hfsq - (s * (hfsq + R) + k * Ln2Lo)) - f);
}

/* Go float64 -> uint64 / uint32 conversion as compiled for amd64 (CVTTSD2SQ path):
 * values outside the target range are implementation-defined in the Go spec; the oracle
 * only promises the in-range behaviour and reports out-of-range as an error. */
double oracle_go_log(double x) { return go_log(x); }

/* lsm/bloom.go:19-41.  Returns 0 on success, -1 when the reference's arithmetic leaves the
 * defined range (n < 0, p outside (0,1), m overflowing u64). n == 0 gives m = 0, k = 1 as in
 * Go (k = uint32(NaN) = 0, then forced to 1 at bloom.go:29-31). */
int oracle_params(int64_t n, double p, uint64_t *m_out, uint32_t *k_out) {
    const double ln2 = 0.6931471805599453;         /* math.Ln2 rounded to float64 */
    const double ln2sq = 0.48045301391820144;       /* const-folded math.Ln2*math.Ln2 */
    if (n < 0 || !(p > 0.0) || !(p < 1.0)) return -1;
    double mf = ceil(-(double)n * go_log(p) / ln2sq);
    if (!(mf >= 0.0) || mf >= 18446744073709551616.0) return -1;
    uint64_t m = (uint64_t)mf;
    uint32_t k;
    if (n == 0) {
        k = 0; /* uint32(NaN) */
    } else {
        double kf = ceil((double)m / (double)n * ln2);
        if (kf >= 4294967296.0) return -1;
        k = (uint32_t)kf;
    }
    if (k == 0) k = 1;
    *m_out = m;
    *k_out = k;
    return 0;
}

uint64_t oracle_fnv1a64(const uint8_t *key, uint64_t len) {
    uint64_t h = FNV_OFFSET;
    for (uint64_t i = 0; i < len; i++) {
        h ^= key[i];
        h *= FNV_PRIME;
    }
    return h;
}

uint64_t oracle_fnv1_64(const uint8_t *key, uint64_t len) {
    uint64_t h = FNV_OFFSET;
    for (uint64_t i = 0; i < len; i++) {
        h *= FNV_PRIME;
        h ^= key[i];
    }
    return h;
}

/* lsm/bloom.go:58-67 */
void oracle_positions(const uint8_t *key, uint64_t len, uint64_t m, uint32_t k, uint64_t *pos) {
    uint64_t h1 = oracle_fnv1a64(key, len);
    uint64_t h2 = oracle_fnv1_64(key, len);
    for (uint32_t i = 0; i < k; i++) pos[i] = (h1 + (uint64_t)i * h2) % m;
}

static inline const uint8_t *key_at(const uint8_t *data, const uint64_t *offsets, uint32_t stride,
                                    uint64_t i, uint64_t *len) {
    if (offsets) {
        *len = offsets[i + 1] - offsets[i];
        return data + offsets[i];
    }
    *len = stride;
    return data + i * (uint64_t)stride;
}

/* lsm/bloom.go:70-77, one key at a time in order, as sstable_builder.go:53 calls it. */
void oracle_add(uint8_t *bits, uint64_t m, uint32_t k, const uint8_t *key, uint64_t len) {
    uint64_t h1 = oracle_fnv1a64(key, len);
    uint64_t h2 = oracle_fnv1_64(key, len);
    for (uint32_t i = 0; i < k; i++) {
        uint64_t h = (h1 + (uint64_t)i * h2) % m;
        bits[h / 8] |= (uint8_t)(1u << (h % 8));
    }
}

/* lsm/bloom.go:82-92, early exit at the first zero bit. */
int oracle_may_contain(const uint8_t *bits, uint64_t m, uint32_t k, const uint8_t *key, uint64_t len) {
    uint64_t h1 = oracle_fnv1a64(key, len);
    uint64_t h2 = oracle_fnv1_64(key, len);
    for (uint32_t i = 0; i < k; i++) {
        uint64_t h = (h1 + (uint64_t)i * h2) % m;
        if ((bits[h / 8] & (1u << (h % 8))) == 0) return 0;
    }
    return 1;
}

/* Batch wrappers: keys packed at a fixed stride (offsets == NULL) or by n+1 prefix offsets. */
void oracle_build(uint8_t *bits, uint64_t m, uint32_t k, const uint8_t *data, const uint64_t *offsets,
                  uint32_t stride, uint64_t n) {
    for (uint64_t i = 0; i < n; i++) {
        uint64_t len;
        const uint8_t *key = key_at(data, offsets, stride, i, &len);
        oracle_add(bits, m, k, key, len);
    }
}

void oracle_probe(const uint8_t *bits, uint64_t m, uint32_t k, const uint8_t *data, const uint64_t *offsets,
                  uint32_t stride, uint64_t n, uint8_t *out) {
    for (uint64_t i = 0; i < n; i++) {
        uint64_t len;
        const uint8_t *key = key_at(data, offsets, stride, i, &len);
        out[i] = (uint8_t)oracle_may_contain(bits, m, k, key, len);
    }
}

/* Multi-filter probe (C5): bit f of mask[i] = MayContain of filter f (f < 64). */
void oracle_probe_multi(const uint8_t *const *bits, const uint64_t *m, const uint32_t *k, uint32_t nf,
                        const uint8_t *data, const uint64_t *offsets, uint32_t stride, uint64_t n,
                        uint64_t *mask) {
    for (uint64_t i = 0; i < n; i++) {
        uint64_t len;
        const uint8_t *key = key_at(data, offsets, stride, i, &len);
        uint64_t w = 0;
        for (uint32_t f = 0; f < nf; f++)
            if (oracle_may_contain(bits[f], m[f], k[f], key, len)) w |= 1ULL << f;
        mask[i] = w;
    }
}

/* lsm/bloom.go:96-102.  out must hold 12 + nbytes. */
void oracle_encode(const uint8_t *bits, uint64_t nbytes, uint64_t m, uint32_t k, uint8_t *out) {
    for (int b = 0; b < 8; b++) out[b] = (uint8_t)(m >> (8 * b));
    for (int b = 0; b < 4; b++) out[8 + b] = (uint8_t)(k >> (8 * b));
    memcpy(out + 12, bits, nbytes);
}

/* lsm/bloom.go:105-120.  Returns -1 (Go: nil) when len < 12; bits are data+12, len-12 bytes. */
int oracle_decode(const uint8_t *data, uint64_t len, uint64_t *m, uint32_t *k) {
    if (len < 12) return -1;
    uint64_t mm = 0;
    uint32_t kk = 0;
    for (int b = 0; b < 8; b++) mm |= (uint64_t)data[b] << (8 * b);
    for (int b = 0; b < 4; b++) kk |= (uint32_t)data[8 + b] << (8 * b);
    *m = mm;
    *k = kk;
    return 0;
}

/* ---- multi-threaded CPU baseline (same algorithm, key-sharded) ---- */
typedef struct {
    const uint8_t *bits;
    uint8_t *wbits;
    uint64_t m;
    uint32_t k;
    const uint8_t *data;
    const uint64_t *offsets;
    uint32_t stride;
    uint64_t lo, hi;
    uint8_t *out;
} mt_job;

static void *probe_worker(void *arg) {
    mt_job *j = (mt_job *)arg;
    for (uint64_t i = j->lo; i < j->hi; i++) {
        uint64_t len;
        const uint8_t *key = key_at(j->data, j->offsets, j->stride, i, &len);
        j->out[i] = (uint8_t)oracle_may_contain(j->bits, j->m, j->k, key, len);
    }
    return NULL;
}

static void *build_worker(void *arg) {
    mt_job *j = (mt_job *)arg;
    for (uint64_t i = j->lo; i < j->hi; i++) {
        uint64_t len;
        const uint8_t *key = key_at(j->data, j->offsets, j->stride, i, &len);
        uint64_t h1 = oracle_fnv1a64(key, len);
        uint64_t h2 = oracle_fnv1_64(key, len);
        for (uint32_t q = 0; q < j->k; q++) {
            uint64_t h = (h1 + (uint64_t)q * h2) % j->m;
            __atomic_fetch_or(&j->wbits[h / 8], (uint8_t)(1u << (h % 8)), __ATOMIC_RELAXED);
        }
    }
    return NULL;
}

static int run_mt(void *(*fn)(void *), mt_job base, uint64_t n, int threads) {
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    pthread_t tid[256];
    mt_job jobs[256];
    for (int t = 0; t < threads; t++) {
        jobs[t] = base;
        jobs[t].lo = n * (uint64_t)t / (uint64_t)threads;
        jobs[t].hi = n * (uint64_t)(t + 1) / (uint64_t)threads;
        if (pthread_create(&tid[t], NULL, fn, &jobs[t]) != 0) return -1;
    }
    for (int t = 0; t < threads; t++) pthread_join(tid[t], NULL);
    return 0;
}

int oracle_probe_mt(const uint8_t *bits, uint64_t m, uint32_t k, const uint8_t *data, const uint64_t *offsets,
                    uint32_t stride, uint64_t n, uint8_t *out, int threads) {
    mt_job b = {bits, NULL, m, k, data, offsets, stride, 0, 0, out};
    return run_mt(probe_worker, b, n, threads);
}

/* The atomic variant: every thread ORs into the shared bits with relaxed atomic byte ORs.  Kept
 * for comparison; contended cache lines make it scale poorly. */
int oracle_build_mt_atomic(uint8_t *bits, uint64_t m, uint32_t k, const uint8_t *data, const uint64_t *offsets,
                           uint32_t stride, uint64_t n, int threads) {
    mt_job b = {NULL, bits, m, k, data, offsets, stride, 0, 0, NULL};
    return run_mt(build_worker, b, n, threads);
}

/* SURVEY.md 8(d)(ii)'s multi-threaded build: private filters OR-merged, at most kMaxPrivate of
 * them (memory stays <= kMaxPrivate filters at any thread count: never T x 12 MB).  Thread t runs
 * the scalar Add loop (lsm/bloom.go:70-77) over its contiguous key shard into private filter
 * t mod P (P = min(T, kMaxPrivate)); a filter shared by several threads takes relaxed atomic byte
 * ORs, one owned by a single thread plain ones.  After a barrier thread t ORs byte range t of
 * every private filter into `bits` (the merge reads the P filters once, split over the T
 * threads).  OR is commutative, so the result equals the sequential build's. */
enum { kMaxPrivate = 16 };

/* A barrier whose participant count can shrink: when a thread cannot be created the ones already
 * running are released instead of waiting forever (the call then returns -1). */
typedef struct {
    pthread_mutex_t mu;
    pthread_cond_t cv;
    int expected, arrived;
    unsigned phase;
} mt_barrier;

static void bar_wait(mt_barrier *b) {
    pthread_mutex_lock(&b->mu);
    const unsigned ph = b->phase;
    if (++b->arrived >= b->expected) {
        b->arrived = 0;
        b->phase++;
        pthread_cond_broadcast(&b->cv);
    } else {
        while (ph == b->phase) pthread_cond_wait(&b->cv, &b->mu);
    }
    pthread_mutex_unlock(&b->mu);
}

static void bar_shrink(mt_barrier *b, int expected) {
    pthread_mutex_lock(&b->mu);
    b->expected = expected;
    if (b->arrived > 0 && b->arrived >= expected) {
        b->arrived = 0;
        b->phase++;
        pthread_cond_broadcast(&b->cv);
    }
    pthread_mutex_unlock(&b->mu);
}

typedef struct {
    mt_job job;
    uint8_t **priv;
    int t, threads, npriv;
    uint64_t nbytes;
    mt_barrier *bar;
    int err;
} priv_job;

/* The private filters live in a pool kept across calls (slot q of kMaxPrivate, grown when a larger
 * filter comes): a timed build then pays the zeroing of its filters, as NewBloomFilter's make does
 * (lsm/bloom.go:34-37), but not fresh page faults, whose cost depends on the host's other tenants
 * more than on this code.  2 MiB pages where the kernel allows them (madvise; 6 TLB entries for a
 * 12 MB filter instead of ~3000, which the random byte ORs would otherwise miss in).  Zeroed by
 * the thread that uses it first in each call.  Checker code: calls are not concurrent. */
static uint8_t *g_pool[kMaxPrivate];
static size_t g_pool_size[kMaxPrivate];

static uint8_t *private_filter(int q, uint64_t nbytes) {
    const size_t huge = (size_t)2 << 20;
    const size_t size = ((nbytes ? nbytes : 1) + huge - 1) / huge * huge;
    if (g_pool_size[q] < size) {
        free(g_pool[q]);
        g_pool[q] = NULL;
        g_pool_size[q] = 0;
        void *p = NULL;
        if (posix_memalign(&p, huge, size) != 0) return NULL;
#ifdef MADV_HUGEPAGE
        (void)madvise(p, size, MADV_HUGEPAGE);
#endif
        g_pool[q] = (uint8_t *)p;
        g_pool_size[q] = size;
    }
    memset(g_pool[q], 0, nbytes);
    return g_pool[q];
}

static void *build_private_worker(void *arg) {
    priv_job *j = (priv_job *)arg;
    if (j->t < j->npriv) j->priv[j->t] = private_filter(j->t, j->nbytes);
    bar_wait(j->bar);
    uint8_t *mine = j->priv[j->t % j->npriv];
    const int shared = j->threads > j->npriv;  /* more threads than filters: filters are shared */
    if (mine) {
        for (uint64_t i = j->job.lo; i < j->job.hi; i++) {
            uint64_t len;
            const uint8_t *key = key_at(j->job.data, j->job.offsets, j->job.stride, i, &len);
            if (!shared) {
                oracle_add(mine, j->job.m, j->job.k, key, len);
                continue;
            }
            const uint64_t h1 = oracle_fnv1a64(key, len), h2 = oracle_fnv1_64(key, len);
            for (uint32_t q = 0; q < j->job.k; q++) {
                const uint64_t h = (h1 + (uint64_t)q * h2) % j->job.m;
                __atomic_fetch_or(&mine[h / 8], (uint8_t)(1u << (h % 8)), __ATOMIC_RELAXED);
            }
        }
    } else {
        j->err = 1;
    }
    bar_wait(j->bar);
    /* merge: this thread's 8-B aligned slice of the byte array, across every private filter */
    const uint64_t words = (j->nbytes + 7) / 8;
    uint64_t lo = words * (uint64_t)j->t / (uint64_t)j->threads * 8;
    uint64_t hi = words * (uint64_t)(j->t + 1) / (uint64_t)j->threads * 8;
    if (hi > j->nbytes) hi = j->nbytes;
    for (int q = 0; q < j->npriv; q++) {
        const uint8_t *src = j->priv[q];
        if (!src) continue;
        uint64_t b = lo;
        for (; b + 8 <= hi; b += 8) {
            uint64_t x, y;
            memcpy(&x, j->job.wbits + b, 8);
            memcpy(&y, src + b, 8);
            x |= y;
            memcpy(j->job.wbits + b, &x, 8);
        }
        for (; b < hi; b++) j->job.wbits[b] |= src[b];
    }
    bar_wait(j->bar);
    return NULL;
}

int oracle_build_mt(uint8_t *bits, uint64_t m, uint32_t k, const uint8_t *data, const uint64_t *offsets,
                    uint32_t stride, uint64_t n, int threads) {
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    pthread_t tid[256];
    priv_job jobs[256];
    uint8_t *priv[kMaxPrivate];
    mt_barrier bar;
    if (pthread_mutex_init(&bar.mu, NULL) != 0) return -1;
    if (pthread_cond_init(&bar.cv, NULL) != 0) {
        pthread_mutex_destroy(&bar.mu);
        return -1;
    }
    bar.expected = threads;
    bar.arrived = 0;
    bar.phase = 0;
    const uint64_t nbytes = (m + 7) / 8;
    const int nprivate = threads < kMaxPrivate ? threads : kMaxPrivate;
    int started = 0, rc = 0;
    for (int q = 0; q < kMaxPrivate; q++) priv[q] = NULL;
    for (int t = 0; t < threads; t++) {
        mt_job b = {NULL, bits, m, k, data, offsets, stride, n * (uint64_t)t / (uint64_t)threads,
                    n * (uint64_t)(t + 1) / (uint64_t)threads, NULL};
        jobs[t] = (priv_job){b, priv, t, threads, nprivate, nbytes, &bar, 0};
    }
    for (int t = 0; t < threads; t++) {
        if (pthread_create(&tid[t], NULL, build_private_worker, &jobs[t]) != 0) {
            /* release the threads already running (their keys and byte ranges are incomplete:
             * the call fails, never hangs or aborts) */
            rc = -1;
            bar_shrink(&bar, t);
            break;
        }
        started++;
    }
    for (int t = 0; t < started; t++) {
        pthread_join(tid[t], NULL);
        if (jobs[t].err) rc = -1;
    }
    pthread_cond_destroy(&bar.cv);
    pthread_mutex_destroy(&bar.mu);
    return rc;
}
