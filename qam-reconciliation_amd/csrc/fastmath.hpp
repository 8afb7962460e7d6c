// fastmath.hpp -- the transcendental core of the check-node update on gfx950.
//
// The reference box-plus (decoder.pyx:41-45) is
//     bp(a,b) = (sgn(a)sgn(b) * min(|a|,|b|) + h(|a+b|)) - h(|a-b|)
//     h(t)    = log(1.0 + exp(-t))            (glibc exp/log, fp64)
// CDNA has no fp64 transcendental instructions; ROCm's ocml exp/log cost
// ~110 VALU instructions per h (227 per box-plus, measured in the ISA of
// k_check<7>), which made the check sweep VALU-bound.  h() below evaluates the
// same expression in ~22 fp64 + ~8 integer VALU operations, specialised to its
// domain t >= 0:
//
//   * t > 37.5 is clamped to [37.5, 37.5 + 2^-15): there exp(-t) < 2^-54, fl(1 + exp(-t)) == 1
//     and log(1) == 0 exactly, which is what the reference returns for every
//     t >= 36.74 -- so the clamp changes nothing and needs no branch.  NaN
//     survives the clamp and propagates (1 + exp(NaN) -> log(NaN) in the reference).
//   * e = exp(-t): k = rint(-t * 256/ln2), r = -t - k ln2/256 (two-term
//     Cody-Waite with fma), e = 2^(k>>8) * T[k&255] * (1 + expm1(r)),
//     |r| <= ln2/512, expm1 to degree 4 (truncation < 2^-57 relative).
//   * u = fl(1 + e) in (1, 2] (rounded exactly like the reference), then
//     log(u) = logc_i + log1p(q),  q = fma(u, invc_i, -1),  i = the top 9 mantissa
//     bits of u (i = 512 for u = 2): u needs no exponent split because u <= 2.
//     Interval 0 is centred on 1 (invc_0 = 1, logc_0 = 0) so q = u - 1 exactly and
//     h keeps full relative accuracy as u -> 1; |q| <= 2^-9 (i = 0), 2^-10
//     otherwise; log1p to degree 5.
//   * sgn(a)sgn(b)min(|a|,|b|) == copysign(min(|a|,|b|), a*b) up to the sign of
//     an exact zero and to NaN cases, neither of which can change bp's final value
//     (a NaN operand makes h(|a+-b|) NaN; a zero m adds a zero to h >= 0).
//
// Accuracy: max |h - glibc log(1+exp(-t))| <= ulp(1) over t in [0, 37.5]
// (the rounding of 1+e, which both sides share, dominates); tests pin it on
// the host (tests/test_fastmath.py).  The decode parity tests bound the effect
// on 50-iteration outputs: hard decisions, success flags and iteration counts
// exact; LAPPRs within the north-star 1e-6.
//
// Tables (256 + 2x513 doubles, 10 KiB) are computed on the host in 80-bit long
// double and staged into LDS by every workgroup (lane-divergent indices).
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

namespace qr {

constexpr int kExpBits = 8;                 // 2^(j/256)
constexpr int kExpN = 1 << kExpBits;
constexpr int kLogBits = 9;                 // 512 intervals of [1, 2)
constexpr int kLogN = (1 << kLogBits) + 1;  // + the entry for u == 2

struct MathTables {
    double exp2j[kExpN];     // 2^(j/256)
    double2 logt[kLogN + 1]; // {invc_i, logc_i}: c_i = 1 + (i + 0.5)/512 (c_0 = 1, c_512 = 2); +1 pad
};

// Host: tables in 80-bit long double, rounded once to double.
inline void build_math_tables(MathTables *t) {
    for (int j = 0; j < kExpN; ++j) t->exp2j[j] = (double)exp2l((long double)j / (long double)kExpN);
    const int n = 1 << kLogBits;
    for (int i = 0; i <= kLogN; ++i) {
        long double c = 1.0L + ((long double)i + 0.5L) / (long double)n;
        if (i == 0) c = 1.0L;
        if (i >= n) c = 2.0L;
        const double inv = (double)(1.0L / c);
        t->logt[i].x = inv;
        t->logt[i].y = (double)(-logl((long double)inv));
    }
}

// Copy the tables from global memory into LDS (whole workgroup participates).
__device__ __forceinline__ void stage_math_tables(MathTables *lds, const MathTables *__restrict__ g) {
    const double2 *src = reinterpret_cast<const double2 *>(g);
    double2 *dst = reinterpret_cast<double2 *>(lds);
    constexpr int n = sizeof(MathTables) / sizeof(double2);
    for (int i = threadIdx.x; i < n; i += blockDim.x) dst[i] = src[i];
    __syncthreads();
}

// h(t) = log(1 + exp(-t)) for t >= 0 (t = |a +- b|).  Host-callable for tests.
__host__ __device__ __forceinline__ double h_softplus_neg(double t, const MathTables &T) {
    constexpr double kInvL = 0x1.71547652b82fep+8;     // 256 / ln 2
    constexpr double kL2Hi = 0x1.62e42fefa4000p-9;     // ln2/256, 40 significant bits
    constexpr double kL2Lo = -0x1.8432a1b0e2634p-51;   // ln2/256 - kL2Hi
    // clamp t > 37.5 into [37.5, 37.5 + 2^-15) by replacing the high word only (one
    // select instead of two; h == 0 there exactly); NaN fails the compare and passes.
    const uint64_t tb = __builtin_bit_cast(uint64_t, t);
    const uint32_t thi = (t > 37.5) ? 0x4042C000u : (uint32_t)(tb >> 32);
    const double tc = __builtin_bit_cast(double, ((uint64_t)thi << 32) | (uint32_t)tb);
    // k = rint(-t 256/ln2) by the 1.5*2^52 shift: the low word of kb is k (two's
    // complement, |k| <= 13850) and kd = kb - shift is k as a double -- one fma and one
    // add instead of mul + rndne + cvt (a near-tie may pick the neighbouring k; r then
    // exceeds ln2/512 by an ulp, which the polynomial absorbs).  NaN: k = 0, kd = NaN.
    constexpr double kShift = 0x1.8p52;
    const double kb = __builtin_fma(tc, -kInvL, kShift);
    const int k = (int)(uint32_t)__builtin_bit_cast(uint64_t, kb);
    const double kd = kb - kShift;
    double r = __builtin_fma(kd, -kL2Hi, -tc);
    r = __builtin_fma(kd, -kL2Lo, r);
    const double s = T.exp2j[k & (kExpN - 1)];
    double p = __builtin_fma(r, 1.0 / 24.0, 1.0 / 6.0); // expm1(r) = r + r^2 (1/2 + r/6 + r^2/24)
    p = __builtin_fma(p, r, 0.5);
    p = __builtin_fma(p, r * r, r);
    const double e = __builtin_ldexp(__builtin_fma(s, p, s), k >> kExpBits);
    const double u = 1.0 + e;                           // in (1, 2] or NaN
    const uint32_t hi32 = (uint32_t)(__builtin_bit_cast(uint64_t, u) >> 32);
    // i in [0, 512] for u in [1, 2]; a NaN u gives an index past the table, whose LDS
    // read returns whatever (LDS reads do not fault) -- q and h are NaN regardless.
    const uint32_t i = (hi32 >> (20 - kLogBits)) - (0x3ff00000u >> (20 - kLogBits));
#ifdef __HIP_DEVICE_COMPILE__
    const double2 c = T.logt[i];
#else
    const double2 c = T.logt[(i < (uint32_t)kLogN) ? i : (uint32_t)kLogN];  // host: stay in bounds
#endif
    const double q = __builtin_fma(u, c.x, -1.0);
    // log1p(q) = q + q^2 (-1/2 + q/3 - q^2/4 + q^3/5): |q| < 2^-9, the truncation
    // q^6/6 < 2^-56 (absolute; h itself carries the 2^-53 rounding of 1 + e)
    double w = __builtin_fma(q, 1.0 / 5.0, -1.0 / 4.0);
    w = __builtin_fma(w, q, 1.0 / 3.0);
    w = __builtin_fma(w, q, -0.5);
    return c.y + __builtin_fma(w, q * q, q);
}

// ---------------------------------------------------------------------------
// Check-node update in the exp domain ("eps domain").
//
// With eps(x) = exp(-|x|), the reference box-plus has the closed forms
//     |bp(a,b)|      = log(1 + eps_a eps_b) - log(eps_a + eps_b)
//     eps(bp(a,b))   = (eps_a + eps_b) / (1 + eps_a eps_b)
//     sign(bp(a,b))  = sign(a) sign(b)
// (ab > 0: |a+b| = M+m, |a-b| = M-m, and h(M+m) - h(M-m) + m = log((1+eps_a eps_b) /
// (eps_a + eps_b)); ab < 0 is the mirror image).  The F/B recursion of
// decoder.pyx:341-367 therefore runs on eps values only: each of its 3(D-2) box-plus
// costs an add, an fma and a reciprocal instead of two exp and two log.  Only the D
// inputs need an exp and the D outputs a log; the output signs are the syndrome sign
// times the product of the other inputs' signs (one XOR parity per check).
//
// Accuracy: eps carries ~1 ulp relative error, i.e. ~1e-16 ABSOLUTE error in the
// magnitudes (the reference's own box-plus rounds h to ~1e-16 absolute); the final
// LAPPRs stay within the north-star 1e-6 and the hard decisions, success flags and
// iteration counts of the parity tests are unchanged (tests/test_gpu_*.py, both paths).
// Domain: every input finite with |m| <= kEpsMax, so no eps underflows (eps >= e^-700
// is normal and the recursion only grows eps: eps_out >= max(eps_a, eps_b) / 2).
// The decoder narrows it further (knob eps_max, default 40): the error of an output L
// is ~ulp(L) (the final log), while for large magnitudes the exact path reproduces the
// reference's rounding almost always bit for bit (its h terms fall below ulp(L)/2).
// Non-converging frames with LLRs in the hundreds amplify ulp(L) differences over 50
// iterations (measured: 1.8e-6 relative with eps_max = 700, <1e-6 at 100 and below;
// tests/test_gpu_decoder.py::test_exp_domain_and_exact_paths).  At the benchmark's
// operating points practically every check input is below 40 (p99 |post| ~ 24 at
// 3 dB), so the narrower domain costs nothing.  Anything outside (|m| > eps_max,
// inf, NaN: the reference's bp(inf, inf) = NaN) takes the exact path (box_plus_fast).
constexpr double kEpsMax = 700.0;

// exp(-x) for 0 <= x <= kEpsMax (same table/polynomial as h_softplus_neg, no clamp).
__host__ __device__ __forceinline__ double eps_of(double x, const MathTables &T) {
    constexpr double kInvL = 0x1.71547652b82fep+8;     // 256 / ln 2
    constexpr double kL2Hi = 0x1.62e42fefa4000p-9;     // ln2/256, 40 significant bits
    constexpr double kL2Lo = -0x1.8432a1b0e2634p-51;   // ln2/256 - kL2Hi
    constexpr double kShift = 0x1.8p52;
    const double kb = __builtin_fma(x, -kInvL, kShift);
    const int k = (int)(uint32_t)__builtin_bit_cast(uint64_t, kb);
    const double kd = kb - kShift;
    double r = __builtin_fma(kd, -kL2Hi, -x);
    r = __builtin_fma(kd, -kL2Lo, r);
    const double s = T.exp2j[k & (kExpN - 1)];
    double p = __builtin_fma(r, 1.0 / 24.0, 1.0 / 6.0);
    p = __builtin_fma(p, r, 0.5);
    p = __builtin_fma(p, r * r, r);
    return __builtin_ldexp(__builtin_fma(s, p, s), k >> kExpBits);
}

// eps(bp(a, b)) = (ea + eb) / (1 + ea eb); the denominator lies in [1, 2], so the
// reciprocal needs no scaling: hardware estimate + two Newton steps (~1 ulp).
__host__ __device__ __forceinline__ double eps_bp(double ea, double eb) {
    const double num = ea + eb;
    const double den = __builtin_fma(ea, eb, 1.0);
#ifdef __HIP_DEVICE_COMPILE__
    double r = __builtin_amdgcn_rcp(den);
#else
    double r = (double)(1.0f / (float)den);  // a deliberately coarse estimate, like v_rcp_f64
#endif
    double t = __builtin_fma(-den, r, 1.0);
    r = __builtin_fma(t, r, r);
    t = __builtin_fma(-den, r, 1.0);
    r = __builtin_fma(t, r, r);
    return num * r;
}

// -log(e) for e in [e^-701, ~1]: e = 2^k u, u in [1, 2); log u = logc_i + log1p(q) with
// the log table of h (i = the top 9 mantissa bits of u).  The sign of the result is
// meaningless when e rounds a hair above 1 (the caller keeps only the magnitude bits).
__host__ __device__ __forceinline__ double eps_neglog(double e, const MathTables &T) {
    constexpr double kLn2Hi = 0x1.62e42fefa3800p-1;    // ln 2, 43 significant bits: k*hi exact
    constexpr double kLn2Lo = 0x1.ef35793c76730p-45;   // ln 2 - kLn2Hi
    const uint64_t b = __builtin_bit_cast(uint64_t, e);
    const uint32_t hi = (uint32_t)(b >> 32);
    const double kd = (double)((int)(hi >> 20) - 1023);
    const double u = __builtin_bit_cast(double, ((uint64_t)((hi & 0x000FFFFFu) | 0x3FF00000u) << 32) | (uint32_t)b);
    const double2 c = T.logt[(hi >> (20 - kLogBits)) & ((1u << kLogBits) - 1)];
    const double q = __builtin_fma(u, c.x, -1.0);
    double w = __builtin_fma(q, 1.0 / 5.0, -1.0 / 4.0);
    w = __builtin_fma(w, q, 1.0 / 3.0);
    w = __builtin_fma(w, q, -0.5);
    const double lp = __builtin_fma(w, q * q, q);
    return -(__builtin_fma(kd, kLn2Hi, c.y) + __builtin_fma(kd, kLn2Lo, lp));
}

// |L| with the sign bit taken from bit 31 of `s`.
__host__ __device__ __forceinline__ double with_sign(double L, uint32_t s) {
    const uint64_t b = __builtin_bit_cast(uint64_t, L);
    const uint32_t hi = ((uint32_t)(b >> 32) & 0x7FFFFFFFu) | (s & 0x80000000u);
    return __builtin_bit_cast(double, ((uint64_t)hi << 32) | (uint32_t)b);
}

__host__ __device__ __forceinline__ uint32_t hi_word(double x) {
    return (uint32_t)(__builtin_bit_cast(uint64_t, x) >> 32);
}

// True when the eps-domain update may take this input: finite, |m| <= lim (<= kEpsMax).
__host__ __device__ __forceinline__ bool eps_ok(double m, double lim = kEpsMax) { return fabs(m) <= lim; }

// decoder.pyx:322-369 in the eps domain for one check of degree D >= 2 with inputs
// m[0..D-1] (ascending edge order) and syndrome bit sb: emit(i, c2v_i) is called once
// per edge, as soon as that output is known (F forward, outputs during the backward
// pass, like the exact path).  Requires eps_ok(m[i]) for every i.
template <int D, typename Emit>
__host__ __device__ __forceinline__ void check_node_eps(const double (&m)[D], uint32_t sb, const MathTables &T,
                                                       Emit &&emit) {
    uint32_t X = sb ? 0x80000000u : 0u;  // s = -1 for a set syndrome bit
    double e[D];
#pragma unroll
    for (int i = 0; i < D; ++i) {
        X ^= hi_word(m[i]);
        e[i] = eps_of(fabs(m[i]), T);
    }
    double F[D - 1];
    F[0] = e[0];
#pragma unroll
    for (int i = 1; i < D - 1; ++i) F[i] = eps_bp(F[i - 1], e[i]);
    emit(D - 1, with_sign(eps_neglog(F[D - 2], T), X ^ hi_word(m[D - 1])));
    double Bn = e[D - 1];
#pragma unroll
    for (int i = D - 2; i > 0; --i) {
        emit(i, with_sign(eps_neglog(eps_bp(F[i - 1], Bn), T), X ^ hi_word(m[i])));
        Bn = eps_bp(Bn, e[i]);
    }
    emit(0, with_sign(eps_neglog(Bn, T), X ^ hi_word(m[0])));
}

// decoder.pyx:41-45 with h() above; the sum keeps the reference's association:
// (sgn*min + h(|a+b|)) - h(|a-b|).
__host__ __device__ __forceinline__ double box_plus_fast(double a, double b, const MathTables &T) {
    const double m = fmin(fabs(a), fabs(b));
    const double sm = copysign(m, a * b);
#ifdef QR_EXPERIMENT_MINSUM   // roofline experiments only (scripts/exp_build.sh): no transcendentals
    (void)T;
    return sm;
#else
    return (sm + h_softplus_neg(fabs(a + b), T)) - h_softplus_neg(fabs(a - b), T);
#endif
}

}  // namespace qr
