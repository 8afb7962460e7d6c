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

#include <vector>

#include "exp_table.hpp"
#include "glibc_math.hpp"

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
#ifdef __HIP_DEVICE_COMPILE__
    z = g_exp_full(z, kGlibcConst);  // glibc's exp, bit for bit (glibc_math.hpp)
#else
    z = exp(z);
#endif
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
    double inv_two_s2;  // RN(1 / two_s2): the k > j LLR exponents' division (div_two_s2)
    double a[kMaxOrder];        // constellation
    double p[kMaxOrder];        // probabilities
    double thr[kMaxOrder + 1];  // decision thresholds
    double Fthr[kMaxOrder + 1]; // F_Y_thresholds
    double dF[kMaxOrder];       // delta_F_Y
    double inv_dF[kMaxOrder];   // 1 / delta_F_Y (Newton start only: never decides a comparison)
    uint8_t sign[kMaxOrder];    // sign_config
    double inv_den;             // 1 / den (Newton only)
    double amin, amax;          // constellation extremes (Newton window bound)
    // Piecewise Taylor table of F_Y (Newton only, see build_ftab): interval j covers
    // [lo + j w, lo + (j+1) w]; kFtabDeg+1 coefficients in t = 2 (y - lo)/w - 2j - 1.
    const double *ftab;
    int32_t ftab_n;
    double ftab_lo, ftab_inv_w, ftab_h, ftab_inv_h, ftab_err;
    const double2 *quant;       // [M][kQStride] F_Y^-1 Hermite nodes (Newton start), see build_quantiles
};

// Newton start table, per decision region k: nodes (y, dy/dx) of y = F_Y^-1(F_thr[k] + u dF[k])
// for cubic Hermite interpolation in a table coordinate x (node spacing 1):
//   left zone   u = w < 2^-kZoneOct:        x = (log2 w + kZoneDepth) * kPerOct   (kZone nodes)
//   middle      u in [2^-kZoneOct, 1 - 2^-kZoneOct], uniform, kMid intervals      (kMid + 1 nodes)
//   right zone  u = 1 - w, w < 2^-kZoneOct: as the left zone                     (kZone nodes)
// The log zones straighten the tails of the outer regions and the low-density ends of
// the inner ones; start errors stay ~1e-9 of the region width (one Newton evaluation).
constexpr int kZoneOct = 5;
constexpr int kZoneDepth = 56;
constexpr int kPerOct = 16;
constexpr int kZone = (kZoneDepth - kZoneOct) * kPerOct + 1;
constexpr int kMid = 1024;
constexpr int kQStride = 2 * kZone + kMid + 1;   // nodes per region (double2 each)

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

// Three-way comparison oracle of the search: sign(F_Y(y) - T).  quick() answers from
// the certified window (2 = inside it, or no window: evaluate), exact() evaluates F_Y.
struct SearchCmp {
    const DemapTables *t;
    double T, ystar, W;
    bool have;
    QR_HD int quick(double y) const {             // selects only (no branches)
        const double w = have ? W : __builtin_inf();
        const double d = y - ystar;
        const int c = (d > w) ? 1 : 2;
        return (d < -w) ? -1 : c;
    }
    QR_HD int exact(double y) const {
        const double F = single_F_Y(*t, y);
        return (F > T) ? 1 : (F < T) ? -1 : 0;   // NaN -> 0 (neither > nor <)
    }
};

// The reference's bracket phase (noisemapper.pyx:314-329): up (T > .5) from [0, 1],
// down from [-1, 0], doubling.  Straight-line body; the exact evaluation is the only
// divergent branch.  Returns the guard count (NaN bracket past kSearchCap).
QR_HD int search_bracket(const SearchCmp &cmp, double &lo, double &hi) {
    const bool up = cmp.T > .5;
    lo = up ? 0.0 : -1.0;
    hi = up ? 1.0 : 0.0;
    int guard = 0;
    for (;;) {                                    // while (F_Y(hi) < T) / while (F_Y(lo) > T)
        const double y = up ? hi : lo;
        int c = cmp.quick(y);
        if (c == 2) c = cmp.exact(y);
        if (!(up ? (c < 0) : (c > 0))) break;
        if (++guard > kSearchCap) { lo = hi = NAN; break; }
        lo = up ? hi : 2. * lo;                   // up: lo = hi, hi *= 2; down: hi = lo, lo *= 2
        hi = up ? 2. * hi : y;
    }
    return guard;
}

// The reference's bracket + bisection (noisemapper.pyx:314-345) on a comparison oracle;
// y_accuracy is the cpdef's optional argument (:310, default 1e-9).
QR_HD double search_replay(const SearchCmp &cmp, double y_accuracy = 1e-9) {
    double lo, hi;
    int guard = search_bracket(cmp, lo, hi);
    while ((hi - lo) > y_accuracy) {
        if (++guard > kSearchCap) { lo = hi = NAN; break; }
        const double mid = (hi + lo) / 2;
        int c = cmp.quick(mid);
        if (c == 2) c = cmp.exact(mid);
        if (c > 0) hi = mid; else lo = mid;       // if (F_Y(mid) > T) hi = mid else lo = mid
    }
    return (hi + lo) / 2;
}

// The bisection in closed form, for a certified window W < 2^-31.  The bracket width is
// 2^e >= 1 with dyadic ends, so every mid is exact and the loop ends at width
// g = 2^-30 (the first power of two <= 1e-9) after e + 30 halvings, on the grid
// lo + j g.  Each mid outside the window is decided by sign(mid - ystar); the final
// bracket [L, L + g] is the grid cell holding ystar.  Only its ends can lie within W of
// ystar (every other mid is >= g - W away), and only an end that moved (L != lo,
// H != hi) was a mid: at most one exact evaluation, whose answer shifts the cell by g.
// The closed form split in two, so that a wavefront can evaluate its lanes' exact F_Y
// together (demap.hip k_demap_hyp): search_closed_prepare runs the bracket and locates the
// final cell [L, H]; need = 1 / 2 when the end L / H lies within W of ystar and must be
// decided exactly (at most one per search, see above), 0 when the cell is certain.  Returns
// false when the closed form does not apply (then the general loop, search_replay, runs).
// search_closed_finish applies the exact answer gt = (F_Y(end) > T).
QR_HD bool search_closed_prepare(const SearchCmp &cmp, double &L, double &H, int &need) {
    double lo, hi;
    const int guard = search_bracket(cmp, lo, hi);
    const double width = hi - lo;
    need = 0;
    if (!(width > 1e-9) || !(width <= 0x1p20) || !(cmp.W < 0x1p-31)) return false;
    if (guard + ilogb(width) + 30 > kSearchCap) { L = H = NAN; return true; }
    constexpr double g = 0x1p-30;
    double j = floor((cmp.ystar - lo) * 0x1p30);
    j = fmin(fmax(j, 0.0), width * 0x1p30 - 1.0);
    L = lo + j * g;                               // exact (|L| < 2^22)
    L = (L > cmp.ystar && L > lo) ? L - g : L;    // fix the rounding of j (exact compares)
    L = (L + g <= cmp.ystar && L + g < hi) ? L + g : L;
    H = L + g;
    if (L != lo && cmp.ystar - L <= cmp.W) need = 1;
    else if (H != hi && H - cmp.ystar <= cmp.W) need = 2;
    return true;
}

QR_HD double search_closed_finish(double L, double H, int need, bool gt) {
    constexpr double g = 0x1p-30;
    if (need == 1 && gt) { H = L; L -= g; }       // F_Y(L) > T: hi = L
    if (need == 2 && !gt) { L = H; H += g; }      // else lo = H
    return (H + L) / 2;
}

QR_HD double search_replay_closed(const SearchCmp &cmp) {
    double L, H;
    int need;
    if (!search_closed_prepare(cmp, L, H, need)) return search_replay(cmp);   // general loop
    const bool gt = need ? cmp.exact(need == 1 ? L : H) > 0 : false;
    return search_closed_finish(L, H, need, gt);
}

QR_HD double search_target(const DemapTables &t, double n_hat, int i) {
    if (t.sign[i]) return t.Fthr[i + 1] - n_hat * t.dF[i];
    return n_hat * t.dF[i] + t.Fthr[i];
}

// Brute force: the reference algorithm verbatim.
QR_HD double g_inv_search(const DemapTables &t, double n_hat, int i, double y_accuracy = 1e-9) {
    SearchCmp cmp{&t, search_target(t, n_hat, i), 0.0, 0.0, false};
    return search_replay(cmp, y_accuracy);
}

// noisemapper.pyx:264-275, the public cpdef F_Y: the UNIFORM mixture (sum of the M
// component CDFs accumulated m = 0 first, then divided by the order), not the
// probability-weighted _single_F_Y the search uses.
QR_HD double public_F_Y(const DemapTables &t, double y) {
    double res = 0.5 * (1 + cephes_erf((y - t.a[0]) / t.den));
    for (int m = 1; m < t.M; ++m) res += 0.5 * (1 + cephes_erf((y - t.a[m]) / t.den));
    return res / t.M;
}

// exp(x) with the LDS table of exp_table.hpp (<= ~1 ulp, like ocml/glibc exp): x = k ln2/256 + r,
// exp(x) = 2^(k>>8) 2^((k&255)/256) e^r.  Overflows to inf above ~709.8, underflows to 0;
// NaN propagates.
QR_HD double exp_fast(double x, const MathTables &T) {
    constexpr double kInvL = 0x1.71547652b82fep+8;     // 256 / ln 2
    constexpr double kL2Hi = 0x1.62e42fefa4000p-9;
    constexpr double kL2Lo = -0x1.8432a1b0e2634p-51;
    const double xc = (x > 710.0) ? 710.0 : (x < -746.0) ? -746.0 : x;
    const double kd = __builtin_rint(xc * kInvL);
    double r = __builtin_fma(kd, -kL2Hi, xc);
    r = __builtin_fma(kd, -kL2Lo, r);
    const int k = (int)kd;
    const double s = T.exp2j[k & (kExpN - 1)];
    double p = __builtin_fma(r, 1.0 / 24.0, 1.0 / 6.0);
    p = __builtin_fma(p, r, 0.5);
    p = __builtin_fma(p, r * r, r);
    return __builtin_ldexp(__builtin_fma(s, p, s), k >> kExpBits);
}

QR_HD double exp_neg_fast(double x, const MathTables &T) { return exp_fast(-x, T); }

// True if p holds on any active lane of the wave (host: p).
QR_HD bool wave_any(bool p) {
#ifdef __HIP_DEVICE_COMPILE__
    return __ballot(p) != 0;
#else
    return p;
#endif
}

// F_Y(y), its density f_Y(y) = sum_m p_m exp(-u_m^2) / (sqrt(pi) den), u_m = (y - a_m)/den,
// and A = max_m |u_m| (f'/f = -(2/den) * a density-weighted mean of u_m, so
// |f'/f| <= 2A/den).  Accurate to a few ulp; only steers Newton (never decides a
// comparison).  FMA Horner; the cephes rationals share one division.
QR_HD void F_and_density(const DemapTables &t, const MathTables &mt, double y, double &F, double &f, double &A) {
    constexpr double kInvSqrtPi = 0.56418958354775628695;
    double sF = 0.0, sf = 0.0;
    for (int m = 0; m < t.M; ++m) {
        const double u = (y - t.a[m]) * t.inv_den;
        const double au = fabs(u);
        const double z = au * au;
        const double e = exp_neg_fast(z, mt);
        const bool small = au <= 1.0;
        // Only the rational(s) some lane of the wave needs (wave-uniform branches; the
        // lanes of a wave sit in one decision region, so most components need one).
        double pt = 1.0, qu = 1.0, pp = 1.0, qq = 1.0;
        if (wave_any(small)) {
            pt = CephesErf::T[0];
            for (int i = 1; i <= 4; ++i) pt = __builtin_fma(pt, z, CephesErf::T[i]);
            qu = z + CephesErf::U[0];
            for (int i = 1; i < 5; ++i) qu = __builtin_fma(qu, z, CephesErf::U[i]);
        }
        if (wave_any(!small)) {
            pp = CephesErf::P[0];
            for (int i = 1; i <= 8; ++i) pp = __builtin_fma(pp, au, CephesErf::P[i]);
            qq = au + CephesErf::Q[0];
            for (int i = 1; i < 8; ++i) qq = __builtin_fma(qq, au, CephesErf::Q[i]);
        }
        const double ratio = (small ? au * pt : e * pp) / (small ? qu : qq);   // erf (small) or erfc
        const double er = small ? ratio : 1.0 - ratio;
        sF += (0.5 * (1 + ((u < 0.0) ? -er : er))) * t.p[m];
        sf += e * t.p[m];
    }
    F = sF;
    f = sf * (kInvSqrtPi * t.inv_den);
    A = fmax(fabs(y - t.amin), fabs(y - t.amax)) * t.inv_den;
}

// F_Y and f_Y from the Taylor table (Newton only): ~30 FMA instead of M erf.  Returns
// false outside the table.
constexpr int kFtabDeg = 12;
#ifndef QR_FTAB_HOLD
#define QR_FTAB_HOLD(x) __asm__ volatile("" : "+v"(x))
#endif
constexpr int kFtabStride = 16;   // doubles per interval (128 B)
QR_HD bool F_and_density_tab(const DemapTables &t, double y, double &F, double &f) {
    const double x = (y - t.ftab_lo) * t.ftab_inv_w;
    if (!(x >= 0.0 && x < (double)t.ftab_n)) return false;
    const int j = (int)x;
    // exact: h is a power of two and lo a multiple of 2h, so the centre and y - centre
    // are exact doubles (u may leave [-1, 1] by an ulp at the interval ends)
    const double u = (y - (t.ftab_lo + (2 * j + 1) * t.ftab_h)) * t.ftab_inv_h;
#ifdef __HIP_DEVICE_COMPILE__
    // all kFtabDeg + 1 coefficients (one 128-B row) requested at once, as global (not flat) loads,
    // and held until the last has arrived: one memory round trip per evaluation instead of the
    // compiler's seven (it issued each 16-B piece right before its Horner step, each behind a
    // vmcnt(0) lgkmcnt(0) wait)
    typedef __attribute__((address_space(1))) const double2 gdouble2;
    gdouble2 *C2 = (gdouble2 *)(t.ftab + (size_t)j * kFtabStride);
    double C[kFtabStride];
#pragma unroll
    for (int q = 0; q < (kFtabDeg + 2) / 2; ++q) {
        const double2 v = C2[q];
        C[2 * q] = v.x;
        C[2 * q + 1] = v.y;
    }
#pragma unroll
    for (int q = 0; q <= kFtabDeg; ++q) QR_FTAB_HOLD(C[q]);
#else
    const double *C = t.ftab + (size_t)j * kFtabStride;
#endif
    double F_ = C[kFtabDeg], d = kFtabDeg * C[kFtabDeg];
    for (int k = kFtabDeg - 1; k >= 1; --k) {
        F_ = __builtin_fma(F_, u, C[k]);
        d = __builtin_fma(d, u, k * C[k]);
    }
    F = __builtin_fma(F_, u, C[0]);
    f = d * t.ftab_inv_h;
    return true;
}

// Cubic Hermite on one table interval, x in [0, 1] (node spacing 1 in the table coordinate).
QR_HD double hermite(double2 n0, double2 n1, double x) {
    const double x2 = x * x, x1m = x - 1.0;
    // y0 (1 + 2x)(1-x)^2 + d0 x (1-x)^2 + y1 x^2 (3 - 2x) + d1 x^2 (x - 1)
    return (n0.x * (1.0 + 2.0 * x) + n0.y * x) * (x1m * x1m) + (n1.x * (3.0 - 2.0 * x) + n1.y * x1m) * x2;
}

// Start point for the root of F_Y(y) = T in region k; NaN when out of the table.  (Device: the
// nodes through global, not flat, loads -- a flat load also counts in lgkmcnt, so every LDS wait
// of the wave would wait for it too.)
#ifdef __HIP_DEVICE_COMPILE__
typedef __attribute__((address_space(1))) const double2 qr_gdouble2;
#else
typedef const double2 qr_gdouble2;
#endif
QR_HD double quantile_start(const DemapTables &t, int k, double T) {
    qr_gdouble2 *Qk = (qr_gdouble2 *)(t.quant + (size_t)k * kQStride);
    const double u = (T - t.Fthr[k]) * t.inv_dF[k];
    const double w = (u < 0.5) ? u : 1.0 - u;
    if (w < 1.0 / (1 << kZoneOct)) {
        const double x = (log2(w) + kZoneDepth) * kPerOct;
        if (!(x >= 0.0)) return __builtin_nan("");
        int j = (int)x;
        if (j > kZone - 2) j = kZone - 2;
        qr_gdouble2 *Z = (u < 0.5) ? Qk : Qk + kZone + kMid + 1;
        return hermite(Z[j], Z[j + 1], x - j);
    }
    constexpr double kLo = 1.0 / (1 << kZoneOct), kScale = kMid / (1.0 - 2.0 * kLo);
    const double x = (u - kLo) * kScale;
    int i = (int)x;
    if (i < 0) i = 0;
    if (i > kMid - 1) i = kMid - 1;
    return hermite(Qk[kZone + i], Qk[kZone + i + 1], x - i);
}

// 1/f for the Newton step and window: the device's v_rcp_f64 refined by two Newton-Raphson
// steps (relative error ~2^-52, against the ~10-instruction IEEE division).  It only steers
// the root location; the window keeps a 2^-40 relative margin for it (wf), far below the x2
// and x4 slack of its terms.
QR_HD double newton_recip(double f) {
#ifdef __HIP_DEVICE_COMPILE__
    double r = __builtin_amdgcn_rcp(f);
    r = __builtin_fma(__builtin_fma(-f, r, 1.0), r, r);
    return __builtin_fma(__builtin_fma(-f, r, 1.0), r, r);
#else
    return 1.0 / f;
#endif
}

// Newton from the Hermite start, usually one evaluation; returns false if it cannot
// certify a window (then the brute-force search runs).  Window W bounds |ystar - y*|:
//   Newton:  |y1 - y*| = |f'(xi)| / (2 f(y0)) (y0 - y*)^2 <= (A/den) d^2 (1 + o(1))
//            for |d| (A + 1) <= 1e-3 den (f, A change by < 1% over the step); taken x4;
//   float:   F_Y carries <= (M+4) eps absolute error (erf <= 4 eps, 1+erf and the
//            product/sum roundings <= (M+1) eps), the Newton-side F_Y <= (M+6) eps
//            (components) or ftab_err (Taylor table); their sum over f, taken x2,
//            plus 4 eps |y|.
// Any finite W keeps the result exact (comparisons inside W are evaluated exactly);
// W only sets the cost.
QR_HD bool newton_root(const DemapTables &t, const MathTables &mt, double T, int k, double &ystar, double &W) {
    if (!t.quant || !(T > 0.0 && T < 1.0)) return false;
    double y = quantile_start(t, k, T);
    if (!(fabs(y) < 1e300)) return false;
    constexpr double eps = 2.220446049250313e-16;
    // F_Y error budget: reference F_Y (M+4) eps + this F_Y (table: ftab_err; components:
    // (M+6) eps), taken x2
    const double ef = 2.0 * ((t.M + 4) * eps + (t.ftab ? t.ftab_err : (t.M + 6) * eps));
    for (int it = 0; it < 4; ++it) {
        double F, f;
        if (t.ftab) {
            if (!F_and_density_tab(t, y, F, f)) return false;
        } else {
            double A_;
            F_and_density(t, mt, y, F, f, A_);
        }
        if (!(f > 0.0)) return false;
        const double rf = newton_recip(f);
        const double d = (F - T) * rf;
        y -= d;
        const double A = fmax(fabs(y - t.amin), fabs(y - t.amax)) * t.inv_den;
        const double wn = 4.0 * (A + 1.0) * t.inv_den * d * d;
        const double wf = ef * rf * (1.0 + 0x1p-40) + 4.0 * eps * fabs(y);
        if (fabs(d) * (A + 1.0) <= 1e-3 * t.den && wn <= fmax(wf, 1e-13)) {
            ystar = y;
            W = wn + wf;
            return W < 1e-3;
        }
    }
    return false;
}

// Fast g_inv_search: bit-identical to g_inv_search (see the block comment).
QR_HD double g_inv_search_fast(const DemapTables &t, const MathTables &mt, double n_hat, int i) {
    SearchCmp cmp{&t, search_target(t, n_hat, i), 0.0, 0.0, false};
    cmp.have = newton_root(t, mt, cmp.T, i, cmp.ystar, cmp.W);   // T lies in region i
    return cmp.have ? search_replay_closed(cmp) : search_replay(cmp);
}

// Host: the Taylor table of F_Y (long double): interval half-width h = the power of two
// in (sigma/16, sigma/8] over
// [amin - 38.6 den, amax + 38.6 den] (F_Y is 0 / 1 in double beyond), coefficients
// F^(k)(c) h^k / k! from F^(k) = sum_m p_m (-1)^(k-1) H_(k-1)(v) e^(-v^2) / (sqrt(pi) den^k),
// v = (c - a_m)/den, H the physicists' Hermite polynomials.  The truncation error
// (~1e-6 (h/sigma)^13 / 13! relative) is far below eps; ftab_err is the largest
// |table - F_Y| seen on 32 points per interval (long double reference), plus the
// Horner rounding.  Returns false (no table) when it would exceed max_n intervals.
inline bool build_ftab(const DemapTables &t, std::vector<double> &tab, int32_t &n, double &lo, double &w,
                       double &err, int32_t max_n = 1 << 16) {
    const double sigma = t.den / sqrt(2.0);
    if (!(sigma > 0 && sigma < 1e100)) return false;
    const double h = exp2(floor(log2(sigma / 8)));
    const double ylo = floor((t.amin - 38.6 * t.den) / (2 * h)) * (2 * h);
    const double yhi = t.amax + 38.6 * t.den;
    const double nn = ceil((yhi - ylo) / (2 * h));
    if (!(nn >= 1 && nn <= max_n)) return false;
    n = (int32_t)nn;
    lo = ylo;
    w = 2 * h;
    const long double hw = h;
    tab.assign((size_t)n * kFtabStride, 0.0);
    const long double rsqpi = 0.564189583547756286948079451560772586L;
    auto Fexact = [&](long double y) {
        long double F = 0;
        for (int m = 0; m < t.M; ++m) F += t.p[m] * 0.5L * erfcl(-(y - t.a[m]) / t.den);
        return F;
    };
    for (int j = 0; j < n; ++j) {
        const long double c = (long double)lo + (2 * j + 1) * hw;
        long double coef[kFtabDeg + 1] = {0};
        coef[0] = Fexact(c);
        for (int m = 0; m < t.M; ++m) {
            const long double v = (c - t.a[m]) / t.den;
            const long double g = t.p[m] * expl(-v * v) * rsqpi;
            long double Hm1 = 0, H = 1, scale = 1;               // H_0
            for (int k = 1; k <= kFtabDeg; ++k) {
                scale *= hw / t.den / k;                          // (h/den)^k / k!
                coef[k] += ((k & 1) ? 1 : -1) * H * g * scale;   // (-1)^(k-1) H_(k-1)
                const long double Hn = 2 * v * H - 2 * (k - 1) * Hm1;
                Hm1 = H;
                H = Hn;
            }
        }
        for (int k = 0; k <= kFtabDeg; ++k) tab[(size_t)j * kFtabStride + k] = (double)coef[k];
    }
    // measured error (double Horner, as on the device)
    long double e = 0;
    for (int j = 0; j < n; ++j) {
        const double *C = &tab[(size_t)j * kFtabStride];
        for (int s = 0; s <= 32; ++s) {
            const double u = -1.0 + s / 16.0;
            double F = C[kFtabDeg];
            for (int k = kFtabDeg - 1; k >= 0; --k) F = fma(F, u, C[k]);
            const long double y = (long double)lo + (2 * j + 1) * hw + u * hw;
            e = fmaxl(e, fabsl((long double)F - Fexact(y)));
        }
    }
    err = (double)(2 * e) + 4 * 2.220446049250313e-16;
    return true;
}

// Host: density f_Y with libm exp (table construction only).
inline double host_density(const DemapTables &t, double y) {
    double s = 0.0;
    for (int m = 0; m < t.M; ++m) {
        const double u = (y - t.a[m]) / t.den;
        s += t.p[m] * exp(-u * u);
    }
    return s * 0.56418958354775628695 / t.den;
}

// Host: F_Y^-1(P) in [lo, hi] by safeguarded Newton on the exact F_Y, from y0.
inline double host_inverse(const DemapTables &t, double P, double lo, double hi, double y0) {
    double y = (y0 > lo && y0 < hi) ? y0 : 0.5 * (lo + hi);
    for (int it = 0; it < 400; ++it) {
        const double F = single_F_Y(t, y);
        if (F < P) lo = y; else hi = y;
        double yn = y - (F - P) / host_density(t, y);
        if (!(yn > lo && yn < hi)) yn = 0.5 * (lo + hi);
        const bool done = fabs(yn - y) <= 1e-15 * fabs(y) + 1e-300 || !(hi - lo > 1e-15 * (fabs(lo) + fabs(hi)));
        y = yn;
        if (done) break;
    }
    return y;
}

// Host: the Hermite node table of quantile_start (kQStride nodes per region).
inline void build_quantiles(const DemapTables &t, double2 *quant) {
    constexpr double kLn2 = 0.69314718055994530942;
    constexpr double kLo = 1.0 / (1 << kZoneOct);
    for (int k = 0; k < t.M; ++k) {
        double2 *Qk = quant + (size_t)k * kQStride;
        const double L = t.thr[k], H = t.thr[k + 1];
        auto inv = [&](double u, double lo, double hi) {
            if (u <= 0.0) return L;
            if (u >= 1.0) return H;
            return host_inverse(t, t.Fthr[k] + u * t.dF[k], lo, hi, 0.5 * (lo + hi));
        };
        auto node = [&](double y, double dudx) {
            double2 n;
            n.x = y;
            n.y = t.dF[k] / host_density(t, y) * dudx;   // dy/dx = dy/du du/dx
            return n;
        };
        // middle, ascending u (each solve bracketed by the previous node)
        double prev = L;
        for (int i = 0; i <= kMid; ++i) {
            const double u = kLo + (1.0 - 2.0 * kLo) * i / kMid;
            const double y = inv(u, prev, H);
            prev = y;
            Qk[kZone + i] = node(y, (1.0 - 2.0 * kLo) / kMid);
        }
        // zones, j = 0 deepest (w = 2^-kZoneDepth) to j = kZone-1 (w = 2^-kZoneOct)
        double plo = L, phi = H;
        for (int j = 0; j < kZone; ++j) {
            const double w = exp2((double)j / kPerOct - kZoneDepth);
            const double yl = inv(w, plo, H);
            plo = yl;
            Qk[j] = node(yl, w * kLn2 / kPerOct);
            const double yr = inv(1.0 - w, L, phi);
            phi = yr;
            Qk[kZone + kMid + 1 + j] = node(yr, -w * kLn2 / kPerOct);
        }
    }
}

// x / two_s2 correctly rounded (noisemapper.pyx:512-515 divides) in five operations, with
// y = RN(1/b), b = two_s2:
//   q0 = RN(x y)                  relative error <= 2^-52 (1+2^-53): within 2 ulp of x/b (near a
//                                 power of two a relative 2^-52 is 2 ulp, so q0 need not be
//                                 faithful)
//   q1 = RN(q0 + RN(x - b q0) y)  the residual step: |x/b - q0 - r0 y| <= |x/b - q0| 2^-52
//                                 (+ the residual's own rounding), so q1 lies within
//                                 0.5 + 2^-50 ulp of x/b: faithful
//   q2 = RN(q1 + (x - b q1) y)    Markstein's theorem (y within half an ulp of 1/b, q1 faithful,
//                                 so x - b q1 is exact in one fma): the correctly rounded x/b.
// No overflow or underflow occurs for these arguments (|x| <= ~1e4, b = 2 sigma^2 > 0 normal),
// except that x = -0 gives +0 (harmless: the quotient only feeds exp, exp(+-0) = 1).  Pinned on
// the host against the IEEE division (tests/native/division_check.cpp: random, near-2 quotient
// significands, the configured 2 sigma^2 of 2..16-PAM at 0..40 dB) and on the GPU by the
// bit-exact demap tests.  The device's IEEE division is a ~10-instruction sequence
// (v_div_scale x2, v_rcp, fmas, v_div_fmas, v_div_fixup).
QR_HD double div_two_s2(const DemapTables &t, double x) {
    const double q0 = x * t.inv_two_s2;
    const double q1 = __builtin_fma(__builtin_fma(-q0, t.two_s2, x), t.inv_two_s2, q0);
    const double r1 = __builtin_fma(-q1, t.two_s2, x);
    return __builtin_fma(r1, t.inv_two_s2, q1);
}

// noisemapper.pyx:450-540 for one symbol; out[k] = LAPPR of Gray bit k (LSB first).
// Note the reference quirk kept on purpose: no /2sigma^2 for k < j (:503-507).
// BPS (= t.bps) is a template parameter: exact-size accumulators (fewer VGPRs, higher
// occupancy) and compile-time trip counts for the M = 2^BPS hypothesis / LLR loops.
// The exp of the LLR sums and the final log are glibc's, restated bit for bit
// (glibc_math.hpp, tables `gt` in LDS): the LAPPRs equal the reference's bit for bit.
template <bool FAST, int BPS>
QR_HD void demap_symbol(const DemapTables& t, const MathTables& mt, const GlibcTables& gt, double n, int j, double alpha,
                        double* out) {
    constexpr int M = 1 << BPS;
    double N[BPS], D[BPS];
#pragma unroll
    for (int k = 0; k < BPS; ++k) { N[k] = 0; D[k] = 0; }
    const double aj = t.a[j];
#pragma unroll 1
    for (int i = 0; i < M; ++i) {
#ifdef QR_EXPERIMENT_NO_SEARCH   // cost-breakdown experiments only (scripts/exp_build.sh)
        const double y = quantile_start(t, i, search_target(t, n, i));
#else
        const double y = FAST ? g_inv_search_fast(t, mt, n, i) : g_inv_search(t, n, i);
#endif
        double s = 0;
#ifndef QR_EXPERIMENT_NO_LLR
        // One loop over all M hypotheses in the reference's summation order (k < j,
        // then p[j], then k > j): lanes of a wave hold different j, so the two
        // j-bounded loops of the reference would run max(j) + max(M-1-j) ≈ 2(M-1)
        // exp slots per wave; here it is M. The per-k argument is selected, not
        // recomputed, so each lane's sum is bit-identical to the two-loop form.
#pragma unroll 1
        for (int k = 0; k < M; ++k) {
            const double e = (2 * y - t.a[k] - aj) * (t.a[k] - aj);
            const double arg = k < j ? e : div_two_s2(t, e);   // a division for k > j, as :512-515
            const double term = k == j ? t.p[j] : g_exp_full(arg, gt) * t.p[k];
            s += term;
        }
#else
        s += t.p[j];
        s += y * 1e-300;
#endif
        const double q = t.dF[i] / s;
        int mi = i;
#pragma unroll
        for (int k = 0; k < BPS; ++k) {
            if ((mi * (mi + 1)) & 3) D[k] += q;
            else                     N[k] += q;
            mi >>= 1;
        }
    }
    // reconciliation.pyx:144-145 (lappr *= alpha) fused into the store.
#pragma unroll
    for (int k = 0; k < BPS; ++k) out[k] = (g_log_full(N[k], gt) - g_log_full(D[k], gt)) * alpha;
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
