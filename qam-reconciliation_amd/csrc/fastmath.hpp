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
