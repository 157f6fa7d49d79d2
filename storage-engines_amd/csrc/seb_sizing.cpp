// seb_sizing.cpp — NewBloomFilter sizing (lsm/bloom.go:19-31), host float64.
// Compiled with -ffp-contract=off: Go evaluates these expressions without FMA on amd64.
//
//   numBits   = uint64(Ceil(-float64(n) * Log(p) / (Ln2*Ln2)))    bloom.go:22
//   numHashes = uint32(Ceil(float64(numBits) / float64(n) * Ln2))   bloom.go:26
//   if numHashes == 0 { numHashes = 1 }                            bloom.go:29-31
//
// Log is Go's math.Log algorithm (src/math/log.go, FreeBSD e_log.c reduction); Go's amd64
// assembly follows the same operation order.  Ln2*Ln2 is a Go constant expression, folded
// exactly then rounded once (0.48045301391820144).
#include <cmath>
#include <cstdint>

namespace seb {

static double go_math_log(double x) {
    static const double Ln2Hi = 6.93147180369123816490e-01, Ln2Lo = 1.90821492927058770002e-10;
    static const double L1 = 6.666666666666735130e-01, L2 = 3.999999999940941908e-01,
                        L3 = 2.857142874366239149e-01, L4 = 2.222219843214978396e-01,
                        L5 = 1.818357216161805012e-01, L6 = 1.531383769920937332e-01,
                        L7 = 1.479819860511658591e-01;
    if (std::isnan(x) || x == HUGE_VAL) return x;
    if (x < 0) return NAN;
    if (x == 0) return -HUGE_VAL;
    int e = 0;
    double f1 = std::frexp(x, &e);
    if (f1 < 0.70710678118654757) {  // Sqrt2/2
        f1 *= 2;
        --e;
    }
    const double f = f1 - 1, kd = (double)e;
    const double s = f / (2 + f), s2 = s * s, s4 = s2 * s2;
    const double t1 = s2 * (L1 + s4 * (L3 + s4 * (L5 + s4 * L7)));
    const double t2 = s4 * (L2 + s4 * (L4 + s4 * L6));
    const double R = t1 + t2, hfsq = 0.5 * f * f;
    return kd * Ln2Hi - ((hfsq - (s * (hfsq + R) + kd * Ln2Lo)) - f);
}

// Returns 0, or -1 where the reference's float->int conversions leave the range the Go spec
// defines (n < 0, p outside (0,1), m >= 2^64, k >= 2^32).
int params(int64_t n, double p, uint64_t *m_out, uint32_t *k_out) {
    const double kLn2 = 0.6931471805599453;
    const double kLn2Sq = 0.48045301391820144;
    if (n < 0 || !(p > 0.0) || !(p < 1.0)) return -1;
    const double mf = std::ceil(-(double)n * go_math_log(p) / kLn2Sq);
    if (!(mf >= 0.0) || mf >= 18446744073709551616.0) return -1;
    const uint64_t m = (uint64_t)mf;
    uint32_t k = 0;  // n == 0: uint32(NaN) == 0 on Go's amd64 and arm64 lowering
    if (n > 0) {
        const double kf = std::ceil((double)m / (double)n * kLn2);
        if (kf >= 4294967296.0) return -1;
        k = (uint32_t)kf;
    }
    if (k == 0) k = 1;
    *m_out = m;
    *k_out = k;
    return 0;
}

}  // namespace seb
