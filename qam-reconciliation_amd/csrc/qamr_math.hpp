// qamr_math.hpp -- scalar arithmetic of the hot path, shared by the gfx950
// kernels (device) and the host-side table construction (host).
//
// Everything here is written to reproduce the reference's IEEE fp64 operation
// order exactly.  The library is compiled with -ffp-contract=off and without
// fast-math, so no a*b+c is fused and inf/NaN propagate as in the reference.
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#define QR_HD __host__ __device__ __forceinline__

namespace qr {

// ---------------------------------------------------------------- decoder
// decoder.pyx:37-38
QR_HD int sgn(double x) { return (0.0 < x) - (x < 0.0); }

// decoder.pyx:41-45 as Cython 3 emits it:
//   t5 = (|b| < |a|) ? |b| : |a|
//   r  = ((sgn(a)*sgn(b)) * t5 + log(1.0 + exp(-|a+b|))) - log(1.0 + exp(-|a-b|))
// (log(1+x), not log1p; the integer sign product is converted to double.)
QR_HD double box_plus(double a, double b) {
    const int s = sgn(a) * sgn(b);
    const double fb = fabs(b), fa = fabs(a);
    const double m = (fb < fa) ? fb : fa;
    const double t1 = fabs(a + b);
    const double t2 = fabs(a - b);
    return (((double)s * m) + log(1.0 + exp(-t1))) - log(1.0 + exp(-t2));
}

// ---------------------------------------------------------------- erf
// scipy.special.erf as shipped with scipy 1.15.3 (xsf/cephes/ndtr.h, polevl.h):
// the function the reference calls through the Python C-API at
// noisemapper.pyx:66-67.  Horner steps are unfused (ans*x + c).
struct CephesErf {
    static constexpr double P[9] = {2.46196981473530512524E-10, 5.64189564831068821977E-1, 7.46321056442269912687E0,
                                    4.86371970985681366614E1,   1.96520832956077098242E2,  5.26445194995477358631E2,
                                    9.34528527171957607540E2,   1.02755188689515710272E3,  5.57535335369399327526E2};
    static constexpr double Q[8] = {1.32281951154744992508E1, 8.67072140885989742329E1, 3.54937778887819891062E2,
                                    9.75708501743205489753E2, 1.82390916687909736289E3, 2.24633760818710981792E3,
                                    1.65666309194161350182E3, 5.57535340817727675546E2};
    static constexpr double R[6] = {5.64189583547755073984E-1, 1.27536670759978104416E0, 5.01905042251180477414E0,
                                    6.16021097993053585195E0,  7.40974269950448939160E0, 2.97886665372100240670E0};
    static constexpr double S[6] = {2.26052863220117276590E0, 9.39603524938001434673E0, 1.20489539808096656605E1,
                                    1.70814450747565897222E1, 9.60896809063285878198E0, 3.36907645100081516050E0};
    static constexpr double T[5] = {9.60497373987051638749E0, 9.00260197203842689217E1, 2.23200534594684319226E3,
                                    7.00332514112805075473E3, 5.55923013010394962768E4};
    static constexpr double U[5] = {3.35617141647503099647E1, 5.21357949780152679795E2, 4.59432382970980127987E3,
                                    2.26290000613890934246E4, 4.92673942608635921086E4};
    static constexpr double MAXLOG = 7.09782712893383996732E2;
};

// erfc for x >= 1 (the only range erf() reaches: ndtr.h erfc with a = x > 0).
QR_HD double erfc_ge1(double x) {
    double z = -x * x;
    if (z < -CephesErf::MAXLOG) return 0.0;
    z = exp(z);
    double p, q;
    if (x < 8.0) {
        p = CephesErf::P[0];
#pragma unroll
        for (int i = 1; i <= 8; ++i) p = p * x + CephesErf::P[i];
        q = x + CephesErf::Q[0];
#pragma unroll
        for (int i = 1; i < 8; ++i) q = q * x + CephesErf::Q[i];
    } else {
        p = CephesErf::R[0];
#pragma unroll
        for (int i = 1; i <= 5; ++i) p = p * x + CephesErf::R[i];
        q = x + CephesErf::S[0];
#pragma unroll
        for (int i = 1; i < 6; ++i) q = q * x + CephesErf::S[i];
    }
    const double y = (z * p) / q;
    return (y != 0.0) ? y : 0.0;
}

QR_HD double cephes_erf(double x) {
    if (isnan(x)) return __builtin_nan("");
    const bool neg = x < 0.0;
    const double ax = neg ? -x : x;
    double r;
    if (ax > 1.0) {
        r = 1.0 - erfc_ge1(ax);
    } else {
        const double z = ax * ax;
        double p = CephesErf::T[0];
#pragma unroll
        for (int i = 1; i <= 4; ++i) p = p * z + CephesErf::T[i];
        double q = z + CephesErf::U[0];
#pragma unroll
        for (int i = 1; i < 5; ++i) q = q * z + CephesErf::U[i];
        r = ax * p / q;
    }
    return neg ? -r : r;
}

// ---------------------------------------------------------------- demapper
constexpr int kMaxOrder = 256;  // PAM order M = 2^bps, bps <= 8
constexpr int kMaxBps = 8;

// Device-resident NoiseMapper tables (noisemapper.pyx:103-162, alphabet.pyx:62-73).
struct DemapTables {
    int32_t M, bps;
    double den;     // sqrt(2) * sigma   (noisemapper.pyx:24, :67)
    double two_s2;  // 2 * noise_var     (noisemapper.pyx:469)
    double a[kMaxOrder];        // constellation
    double p[kMaxOrder];        // probabilities
    double thr[kMaxOrder + 1];  // decision thresholds
    double Fthr[kMaxOrder + 1]; // F_Y_thresholds
    double dF[kMaxOrder];       // delta_F_Y
    uint8_t sign[kMaxOrder];    // sign_config
};

// noisemapper.pyx:278-286 with __F_Z (:66-67): sum over m in order, m = 0 first.
QR_HD double single_F_Y(const DemapTables& t, double y) {
    double res = (0.5 * (1 + cephes_erf((y - t.a[0]) / t.den))) * t.p[0];
    for (int m = 1; m < t.M; ++m) res += (0.5 * (1 + cephes_erf((y - t.a[m]) / t.den))) * t.p[m];
    return res;
}

// ------------------------------------------------------------------------
// g_inv_search (noisemapper.pyx:310-345, y_accuracy = 1e-9).
//
// The reference brackets the root of F_Y(y) = T by doubling, then bisects to
// |hi - lo| <= 1e-9: 31..40 evaluations of F_Y (M erf each) per call.  Every
// decision is a comparison sign(F_Y(y) - T).  F_Y is strictly increasing, so
// away from the root that sign is sign(y - y*).  The fast path therefore
//   1. locates y* by safeguarded Newton (F_Y and its density, ~4-6 steps), and
//   2. replays the reference's bracket + bisection arithmetic exactly (same
//      lo/hi/mid doubles), deciding each comparison by sign(y - y*) unless y is
//      within a certified window W of y*, where F_Y(y) is evaluated exactly as
//      the reference does.  W bounds the Newton error plus the float error of
//      F_Y (<= (M+2) ulp(1), absolute) divided by the density at y*.
// The returned doubles are bit-identical to the brute-force search with the
// same F_Y (tests/test_demap_replay.py checks this over millions of draws);
// when Newton cannot certify a root (NaN target, T outside (0,1), density
// underflow, W too wide) the brute-force search runs instead.
// ------------------------------------------------------------------------

// Iteration cap on the bracket and bisection loops.  The reference loops are
// unbounded (noisemapper.pyx:323-342); for finite targets they take <= ~1100
// steps, so the cap only turns a reference hang (T > 1 or |y| > ~4e6) into a
// NaN instead of a stuck GPU wave.
constexpr int kSearchCap = 2200;

// Three-way comparison oracle of the search: sign(F_Y(y) - T).
struct SearchCmp {
    const DemapTables *t;
    double T, ystar, W;
    bool have;
    QR_HD int operator()(double y) const {
        if (have) {
            const double d = y - ystar;
            if (d > W) return 1;
            if (d < -W) return -1;
        }
        const double F = single_F_Y(*t, y);
        return (F > T) ? 1 : (F < T) ? -1 : 0;   // NaN -> 0 (neither > nor <)
    }
};

// The reference's bracket + bisection (noisemapper.pyx:314-345) on a comparison oracle.
QR_HD double search_replay(const SearchCmp &cmp) {
    double lo, hi;
    int guard = 0;
    if (cmp.T > .5) {
        hi = 1; lo = 0;
        while (cmp(hi) < 0) {             // while (F_Y(hi) < T)
            if (++guard > kSearchCap) return NAN;
            lo = hi; hi *= 2.;
        }
    } else {
        lo = -1; hi = 0;
        while (cmp(lo) > 0) {             // while (F_Y(lo) > T)
            if (++guard > kSearchCap) return NAN;
            hi = lo; lo *= 2.;
        }
    }
    while ((hi - lo) > 1e-9) {
        if (++guard > kSearchCap) return NAN;
        const double mid = (hi + lo) / 2;
        if (cmp(mid) > 0) hi = mid; else lo = mid;   // if (F_Y(mid) > T) hi = mid else lo = mid
    }
    return (hi + lo) / 2;
}

QR_HD double search_target(const DemapTables &t, double n_hat, int i) {
    if (t.sign[i]) return t.Fthr[i + 1] - n_hat * t.dF[i];
    return n_hat * t.dF[i] + t.Fthr[i];
}

// Brute force: the reference algorithm verbatim.
QR_HD double g_inv_search(const DemapTables &t, double n_hat, int i) {
    SearchCmp cmp{&t, search_target(t, n_hat, i), 0.0, 0.0, false};
    return search_replay(cmp);
}

// F_Y(y) and its density f_Y(y) = sum_m p_m exp(-u_m^2) / (sqrt(pi) den), u_m = (y - a_m)/den.
// Accurate to a few ulp; only steers Newton (never decides a comparison).
QR_HD void F_and_density(const DemapTables &t, double y, double &F, double &f) {
    constexpr double kInvSqrtPi = 0.56418958354775628695;
    double sF = 0.0, sf = 0.0;
    for (int m = 0; m < t.M; ++m) {
        const double u = (y - t.a[m]) / t.den;
        const double au = fabs(u);
        const double e = exp(-au * au);          // shared by the density and cephes' erfc
        double r;
        if (au > 1.0) {
            double p, q;
            if (au < 8.0) {
                p = CephesErf::P[0];
                for (int i = 1; i <= 8; ++i) p = p * au + CephesErf::P[i];
                q = au + CephesErf::Q[0];
                for (int i = 1; i < 8; ++i) q = q * au + CephesErf::Q[i];
            } else {
                p = CephesErf::R[0];
                for (int i = 1; i <= 5; ++i) p = p * au + CephesErf::R[i];
                q = au + CephesErf::S[0];
                for (int i = 1; i < 6; ++i) q = q * au + CephesErf::S[i];
            }
            r = 1.0 - (e * p) / q;
        } else {
            const double z = au * au;
            double p = CephesErf::T[0];
            for (int i = 1; i <= 4; ++i) p = p * z + CephesErf::T[i];
            double q = z + CephesErf::U[0];
            for (int i = 1; i < 5; ++i) q = q * z + CephesErf::U[i];
            r = au * p / q;
        }
        sF += (0.5 * (1 + ((u < 0.0) ? -r : r))) * t.p[m];
        sf += e * t.p[m];
    }
    F = sF;
    f = sf * (kInvSqrtPi / t.den);
}

// Safeguarded Newton for F_Y(y) = T; returns false if no certified root.
QR_HD bool newton_root(const DemapTables &t, double T, double &ystar, double &W) {
    if (!(T > 0.0 && T < 1.0)) return false;
    // bracket from the decision thresholds: F_Y(t_k) = F_Y_thresholds[k]
    int k = 0;
    while (k < t.M && !(t.Fthr[k + 1] >= T)) ++k;
    if (k >= t.M) return false;
    double lo = t.thr[k], hi = t.thr[k + 1];
    double y = (k == 0) ? t.a[0] : (k == t.M - 1) ? t.a[t.M - 1] : 0.5 * (lo + hi);
    if (!(y > lo && y < hi)) y = 0.5 * (lo + hi);
    double F, f, step = hi - lo;
    bool conv = false;
    for (int it = 0; it < 80; ++it) {
        F_and_density(t, y, F, f);
        const double g = F - T;
        if (g > 0) hi = y; else lo = y;
        double yn = y - g / f;
        if (!(yn > lo && yn < hi)) yn = 0.5 * (lo + hi);      // bisection fallback (also f == 0 / NaN)
        step = yn - y;
        y = yn;
        if (fabs(step) <= 1e-13 * (fabs(y) + t.den)) { conv = true; break; }
    }
    if (!conv) return false;
    F_and_density(t, y, F, f);
    if (!(f > 0.0)) return false;
    // window: Newton residual and last step + float error of F_Y (<= (M+2) ulp(1),
    // absolute) over the density, with a x8..x16 margin.  Any finite W is correct
    // (ambiguous comparisons are evaluated exactly); W only sets the cost.
    const double eps = 2.220446049250313e-16;
    const double w = 8.0 * fabs(F - T) / f + 4.0 * fabs(step) + 16.0 * (t.M + 4) * eps / f + 8.0 * eps * fabs(y);
    if (!(w < 1e-3)) return false;
    ystar = y;
    W = w;
    return true;
}

// Fast g_inv_search: bit-identical to g_inv_search (see the block comment).
QR_HD double g_inv_search_fast(const DemapTables &t, double n_hat, int i) {
    SearchCmp cmp{&t, search_target(t, n_hat, i), 0.0, 0.0, false};
    cmp.have = newton_root(t, cmp.T, cmp.ystar, cmp.W);
    return search_replay(cmp);
}

// noisemapper.pyx:450-540 for one symbol; out[k] = LAPPR of Gray bit k (LSB first).
// Note the reference quirk kept on purpose: no /2sigma^2 for k < j (:503-507).
template <bool FAST = true>
QR_HD void demap_symbol(const DemapTables& t, double n, int j, double alpha, double* out) {
    double N[kMaxBps], D[kMaxBps];
#pragma unroll
    for (int k = 0; k < kMaxBps; ++k) { N[k] = 0; D[k] = 0; }
    const double aj = t.a[j];
    for (int i = 0; i < t.M; ++i) {
        const double y = FAST ? g_inv_search_fast(t, n, i) : g_inv_search(t, n, i);
        double s = 0;
        for (int k = 0; k < j; ++k) s += exp((2 * y - t.a[k] - aj) * (t.a[k] - aj)) * t.p[k];
        s += t.p[j];
        for (int k = j + 1; k < t.M; ++k) s += exp((2 * y - t.a[k] - aj) * (t.a[k] - aj) / t.two_s2) * t.p[k];
        const double q = t.dF[i] / s;
        int mi = i;
#pragma unroll
        for (int k = 0; k < kMaxBps; ++k) {
            if (k < t.bps) {
                if ((mi * (mi + 1)) & 3) D[k] += q;
                else                     N[k] += q;
                mi >>= 1;
            }
        }
    }
    // reconciliation.pyx:144-145 (lappr *= alpha) fused into the store.
#pragma unroll
    for (int k = 0; k < kMaxBps; ++k)
        if (k < t.bps) out[k] = (log(N[k]) - log(D[k])) * alpha;
}

// noisemapper.pyx:27-44 (__binsearch over the M+1 thresholds), iterative.
QR_HD int binsearch_thr(const double* dom, int size, double val) {
    int base = 0;
    for (;;) {
        if (size == 1) return base;
        if (val < dom[0]) return base;
        if (val > dom[size - 1]) return base + size - 1;
        const int index = size / 2 - 1;
        if (val < dom[index]) { size = index; continue; }
        if (val >= dom[index + 1]) { base += index + 1; dom += index + 1; size -= index + 1; continue; }
        return base + index;
    }
}

}  // namespace qr
