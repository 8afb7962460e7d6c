// glibc_math.hpp -- bit-exact restatement of the host libm's exp() and log() for the
// strict box-plus (decoder.pyx:41-45 evaluated exactly as the reference evaluates it).
//
// The reference computes h(t) = log(1.0 + exp(-t)) with glibc.  On x86-64 with FMA
// (every host of this project: the EPYC GPU-box hosts and the build container),
// glibc 2.35 resolves exp/log to __exp_fma / __log_fma: sysdeps/ieee754/dbl-64/e_exp.c
// and e_log.c (the ARM optimized-routines algorithms) compiled with -mfma, i.e. with
// GCC's floating-point contraction.  The functions below repeat those routines
// operation for operation -- every fma exactly where the compiled routine has a
// vfmadd/vfnmadd, every other operation as a separately rounded IEEE op -- so that
// on any IEEE fp64 machine (gfx950 VALU included) they return the same bits.  The
// data (128-entry tables and coefficients) is extracted from the library itself at
// build time (gen_glibc_tables.py -> build/glibc_tables.inc).
//
//   exp(x), x in [-512, 512], |x| >= 2^-54 (abstop in range, e_exp.c:90-140):
//     kd = fma(x, InvLn2N, Shift); ki = bits(kd); kd -= Shift
//     r  = fma(kd, NegLn2loN, fma(kd, NegLn2hiN, x))
//     tail, sbits = T[ki % 128] (+ ki << 45)
//     tmp = fma(r^4, fma(r, C5, C4), fma(fma(r, C3, C2), r^2, tail + r))
//     exp = fma(scale, tmp, scale)
//   |x| < 2^-54: 1.0 + x.
//
//   log(x), x positive normal (e_log.c:40-140):
//     x in [1 - 2^-4, 1 + 0x1.09p-4): the near-1 polynomial of degree 12 with the
//       hi/lo split of r = x - 1 (see g_log below for the contraction pattern);
//     otherwise: i, k from the top bits of x - OFF, r = fma(z, invc_i, -1),
//       w = fma(k, Ln2hi, logc_i), hi = r + w, lo = fma(k, Ln2lo, (w - hi) + r),
//       log = fma(r^3, fma(fma(r, A4, A3), r^2, fma(r, A2, A1)), fma(r^2, A0, lo)) + hi.
//
// tests/test_glibc_math.py runs these on the host against libm's exp/log on ~10^7
// inputs (dense on the box-plus domain) and requires identical bits; the GPU tests
// then require decodes bit-identical to the oracle (which calls libm).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "glibc_tables.inc"

namespace qr {

// {tail_i, tab[2i+1]} per exp interval and {invc, logc} per log interval, staged in LDS.
// glibc's sbits = tab[2i+1] + (ki << 45) (e_exp.c): only the high word changes, by
// ki << 13 (mod 2^32; the low 19 bits of ki, i.e. the low word of kd), so the scale's
// high word is ONE v_lshl_add_u32 (ki, 13, hi(tab[2i+1])) -- no separate k = ki >> 7.
//
// lk / lc: the log table path specialised to the box-plus domain u in [1 + 0x1.09p-4, 2]
// (g_log_table).  There the exponent k of e_log.c is a function of the table index i
// (u in [1.0647, 1.375): k = 0, i in [88, 127]; u in [1.375, 2]: k = 1, i in [0, 80]), so
// the k-dependent operations fold into the table, exactly:
//   z * invc            = u * (invc 2^-k)           (scaling by 2^-k is exact)
//   fma(k, Ln2hi, logc) = w_i                       (precomputed, same rounding)
//   fma(k, Ln2lo, lo)   = lo + (k ? Ln2lo : +0.0)   (1*x + lo and 0*x + lo, x > 0)
// lk[j] = {invc_i 2^-k, w_i, k ? Ln2lo : +0.0, 0} stored at j = (i + 48) & 127 =
// (hx >> 13) & 127 (the index needs no subtraction of e_log.c's OFF: OFF's low 17 bits
// are zero and OFF >> 13 = 48 mod 128), 32 B per entry: byte offset (hx >> 8) & 0xFE0.
struct GlibcLogK {
    double invc, w, c, pad;
};
// ex holds the 128 exp entries twice (ex[i + 128] = ex[i]): the strict box-plus indexes it
// by the low BYTE of ki, which gfx9 reads with an SDWA byte select inside the address shift
// (one instruction instead of an and + shift); glibc's own index ki % 128 reads the same data.
struct GlibcTables {
    double2 ex[256];
    GlibcLogK lk[128];
    double2 lg[128];
};
// The box-plus' part of GlibcTables (its leading 8 KiB: ex and lk): what the strict check
// sweep stages in LDS (g_exp_neg, g_log_table, h_packed read nothing else).
struct GlibcTablesBP {
    double2 ex[256];
    GlibcLogK lk[128];
};
static_assert(sizeof(GlibcTablesBP) == 8192, "box-plus tables: 8 KiB");
static_assert(offsetof(GlibcTables, lk) == offsetof(GlibcTablesBP, lk), "GlibcTablesBP is a prefix of GlibcTables");

// The demapper's subset (glibc_math g_exp_full / g_log_full read only ex[ki % 128] and lg):
// 4 KiB of LDS per workgroup instead of 10.
struct GlibcExpLog {
    double2 ex[128];
    double2 lg[128];
};

__host__ __device__ constexpr int glibc_log_k_of_index(int i) { return i <= 80 ? 1 : 0; }

inline void build_glibc_tables(GlibcTables *t) {
    for (int i = 0; i < 128; ++i) {
        t->ex[i].x = t->ex[i + 128].x = __builtin_bit_cast(double, kGxTab[2 * i]);
        t->ex[i].y = t->ex[i + 128].y = __builtin_bit_cast(double, kGxTab[2 * i + 1]);
        t->lg[i].x = kGlTab[2 * i];
        t->lg[i].y = kGlTab[2 * i + 1];
        const int k = glibc_log_k_of_index(i);
        GlibcLogK &e = t->lk[(i + 48) & 127];
        e.invc = k ? kGlTab[2 * i] * 0.5 : kGlTab[2 * i];
        e.w = __builtin_fma((double)k, kGlLn2hi, kGlTab[2 * i + 1]);
        e.c = k ? kGlLn2lo : 0.0;
        e.pad = 0.0;
    }
}

// the exp/log subset from the full tables (ex[0..127] and lg are leading members of both)
__device__ __forceinline__ void stage_glibc_exp_log(GlibcExpLog *lds, const GlibcTables *__restrict__ g) {
    for (int i = threadIdx.x; i < 128; i += blockDim.x) {
        lds->ex[i] = g->ex[i];
        lds->lg[i] = g->lg[i];
    }
    __syncthreads();
}

template <class TT>   // GlibcTables or its prefix GlibcTablesBP
__device__ __forceinline__ void stage_glibc_tables(TT *lds, const GlibcTables *__restrict__ g) {
    const double2 *src = reinterpret_cast<const double2 *>(g);
    double2 *dst = reinterpret_cast<double2 *>(lds);
    constexpr int n = sizeof(TT) / sizeof(double2);
    for (int i = threadIdx.x; i < n; i += blockDim.x) dst[i] = src[i];
    __syncthreads();
}

__host__ __device__ __forceinline__ uint32_t g_hi(double x) { return (uint32_t)(__builtin_bit_cast(uint64_t, x) >> 32); }
__host__ __device__ __forceinline__ uint32_t g_lo(double x) { return (uint32_t)__builtin_bit_cast(uint64_t, x); }
__host__ __device__ __forceinline__ double g_make(uint32_t hi, uint32_t lo) {
    return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}
// high word of glibc's sbits = tab[2i+1] + (ki << 45): hi + (ki << 13) as ONE v_lshl_add_u32
// (left to itself the compiler turns the shift-add into a 64-bit add)
__host__ __device__ __forceinline__ uint32_t g_add_ki(uint32_t hi, uint32_t ki) {
#if defined(__HIP_DEVICE_COMPILE__)
    uint32_t r;
    asm("v_lshl_add_u32 %0, %1, 13, %2" : "=v"(r) : "v"(ki), "v"(hi));
    return r;
#else
    return hi + (ki << 13);
#endif
}

// glibc exp(x) for |x| < 512 (finite; NaN propagates).  The table index and the
// exponent come from the low word of kd (|ki| < 2^17, so ki << 45 only touches the
// high word of sbits).
template <class TT>
__host__ __device__ __forceinline__ double g_exp(double x, const TT &T) {
    double kd = __builtin_fma(x, kGxInvLn2N, kGxShift);
    const uint32_t ki = g_lo(kd);
    kd = kd - kGxShift;
    double r = __builtin_fma(kd, kGxNegLn2hiN, x);
    r = __builtin_fma(kd, kGxNegLn2loN, r);
    const double2 e = T.ex[ki & 127u];
    const double scale = g_make(g_add_ki(g_hi(e.y), ki), g_lo(e.y));  // sbits
    const double r2 = r * r;
    const double p23 = __builtin_fma(r, kGxC3, kGxC2);
    const double tr = e.x + r;
    const double p45 = __builtin_fma(r, kGxC5, kGxC4);
    const double a = __builtin_fma(p23, r2, tr);
    const double r4 = r2 * r2;
    const double tmp = __builtin_fma(r4, p45, a);
    const double res = __builtin_fma(scale, tmp, scale);
    return (__builtin_fabs(x) < 0x1p-54) ? 1.0 + x : res;
}

// glibc log(x) for positive normal finite x (the box-plus only needs x in [1, 2]).
template <class TT>
__host__ __device__ __forceinline__ double g_log(double x, const TT &T) {
    const uint32_t hx = g_hi(x);
    double y;
    if (hx - 0x3FEE0000u < 0x3FF10900u - 0x3FEE0000u) {
        // x in [1 - 2^-4, 1 + 0x1.09p-4): e_log.c "close to 1.0" branch
        const double r = x - 1.0;
        double p2 = __builtin_fma(r, kGlB2, kGlB1);
        double p5 = __builtin_fma(r, kGlB5, kGlB4);
        const double r2 = r * r;
        double p8 = __builtin_fma(r, kGlB8, kGlB7);
        p2 = __builtin_fma(r2, kGlB3, p2);
        p5 = __builtin_fma(r2, kGlB6, p5);
        const double r3 = r * r2;
        p8 = __builtin_fma(r2, kGlB9, p8);
        p8 = __builtin_fma(r3, kGlB10, p8);
        p5 = __builtin_fma(p8, r3, p5);
        const double P = __builtin_fma(p5, r3, p2);
        // rhi = r + w - w, w = r * 2^27 (contracted: both steps are fmas)
        const double t = __builtin_fma(r, 0x1p27, r);
        const double rhi = __builtin_fma(-0x1p27, r, t);
        const double rhi2 = rhi * rhi;
        const double rlo = r - rhi;
        const double hi = __builtin_fma(rhi2, kGlB0, r);    // r + rhi*rhi*B0
        const double d = r - hi;
        const double rr = r + rhi;
        double lo = __builtin_fma(rhi2, kGlB0, d);          // r - hi + w
        const double q = kGlB0 * rlo;
        lo = __builtin_fma(q, rr, lo);                      // lo += B0*rlo*(rhi + r)
        const double yy = __builtin_fma(P, r3, lo);         // y = r3*P; y += lo
        y = hi + yy;                                        // y += hi
        if (__builtin_bit_cast(uint64_t, x) == 0x3FF0000000000000ull) y = 0.0;
    } else {
        // OFF = 0x3fe6000000000000: only the high word takes part in the index arithmetic
        const uint32_t th = hx - 0x3FE60000u;
        const uint32_t i = (th >> 13) & 127u;
        const int k = (int)th >> 20;
        const double z = g_make(hx - (th & 0xFFF00000u), g_lo(x));
        const double2 c = T.lg[i];                          // {invc, logc}
        const double r = __builtin_fma(z, c.x, -1.0);
        const double kd = (double)k;
        const double w = __builtin_fma(kd, kGlLn2hi, c.y);
        const double pA = __builtin_fma(r, kGlA2, kGlA1);
        const double hi = r + w;
        const double r2 = r * r;
        double lo = w - hi;
        lo = lo + r;
        lo = __builtin_fma(kd, kGlLn2lo, lo);
        const double r3 = r * r2;
        double pB = __builtin_fma(r, kGlA4, kGlA3);
        lo = __builtin_fma(r2, kGlA0, lo);
        pB = __builtin_fma(pB, r2, pA);
        y = __builtin_fma(r3, pB, lo) + hi;
    }
    return y;
}

// ---- full-range exp / log (the demapper: noisemapper.pyx:503-515, 534; erfc's exp) --------
//
// __exp_fma for every input: |x| < 2^-54 -> 1.0 + x; |x| >= 1024, inf, NaN -> 0, 1.0 + x
// (inf/NaN) or the overflow/underflow result; 512 <= |x| < 1024 -> the main path with the
// e_exp.c specialcase() rescaling (contraction pattern of the compiled routine: k > 0
// fuses scale + scale*tmp, k < 0 does not, it reuses scale*tmp).
template <class TT>
__host__ __device__ __forceinline__ double g_exp_full(double x, const TT &T) {
    const uint32_t abstop = (g_hi(x) >> 20) & 0x7FFu;
    if (abstop - 0x3C9u >= 0x3Fu) {
        if ((int)(abstop - 0x3C9u) < 0) return 1.0 + x;
        if (abstop >= 0x409u) {
            if (__builtin_bit_cast(uint64_t, x) == 0xFFF0000000000000ull) return 0.0;
            if (abstop >= 0x7FFu) return 1.0 + x;
            return (g_hi(x) >> 31) ? 0.0 : __builtin_inf();
        }
    }
    double kd = __builtin_fma(x, kGxInvLn2N, kGxShift);
    const uint32_t ki = g_lo(kd);
    kd = kd - kGxShift;
    double r = __builtin_fma(kd, kGxNegLn2hiN, x);
    r = __builtin_fma(kd, kGxNegLn2loN, r);
    const double2 e = T.ex[ki & 127u];
    const uint32_t shi = g_add_ki(g_hi(e.y), ki), slo = g_lo(e.y);
    const double r2 = r * r;
    const double p23 = __builtin_fma(r, kGxC3, kGxC2);
    const double tr = e.x + r;
    const double p45 = __builtin_fma(r, kGxC5, kGxC4);
    const double a = __builtin_fma(p23, r2, tr);
    const double r4 = r2 * r2;
    const double tmp = __builtin_fma(r4, p45, a);
    if (abstop < 0x408u) {  // the common case: no rescaling
        const double scale = g_make(shi, slo);
        return __builtin_fma(scale, tmp, scale);
    }
    if (!(ki & 0x80000000u)) {  // k > 0: sbits -= 1009 << 52
        const double scale = g_make(shi - 0x3F100000u, slo);
        return __builtin_fma(scale, tmp, scale) * 0x1p1009;
    }
    const double scale = g_make(shi + 0x3FE00000u, slo);  // k < 0: sbits += 1022 << 52
    const double st = scale * tmp;
    double y = scale + st;
    if (y < 1.0) {
        const double hi = y + 1.0;
        const double lo = (scale - y) + st;
        double t = (1.0 - hi) + y;
        t = t + lo;
        t = t + hi;
        y = t - 1.0;
        if (y == 0.0) y = 0.0;
    }
    return y * 0x1p-1022;
}

// g_exp_full with its special cases kept off the common path: glibc's main path (|x| in
// [2^-54, 512), e_exp.c:90-140 without specialcase) runs branch-free on every lane, and only
// when some lane of the wavefront has an argument outside that range does the wave run
// g_exp_full for those lanes (one wave-uniform branch instead of two per-lane ones and their
// exec-mask bookkeeping).  Same bits as g_exp_full for every input.
template <class TT>
__device__ __forceinline__ double g_exp_wave(double x, const TT &T) {
    // lanes with |x| outside [2^-54, 512) or not finite (e_exp.c's special cases; abstop = the
    // exponent field), as the compare's lane mask itself (llvm.amdgcn.icmp: a ballot of a bool
    // materialised it first)
    const uint64_t special_mask =
        __builtin_amdgcn_uicmp(__builtin_amdgcn_ubfe(g_hi(x), 20, 11) - 0x3C9u, 0x408u - 0x3C9u, 35 /* uge */);
    double kd = __builtin_fma(x, kGxInvLn2N, kGxShift);
    const uint32_t ki = g_lo(kd);
    kd = kd - kGxShift;
    double r = __builtin_fma(kd, kGxNegLn2hiN, x);
    r = __builtin_fma(kd, kGxNegLn2loN, r);
    const double2 e = T.ex[ki & 127u];
    const double scale = g_make(g_add_ki(g_hi(e.y), ki), g_lo(e.y));
    const double r2 = r * r;
    const double p23 = __builtin_fma(r, kGxC3, kGxC2);
    const double tr = e.x + r;
    const double p45 = __builtin_fma(r, kGxC5, kGxC4);
    const double a = __builtin_fma(p23, r2, tr);
    const double r4 = r2 * r2;
    const double tmp = __builtin_fma(r4, p45, a);
    double res = __builtin_fma(scale, tmp, scale);
    // wave-uniform: a wave with a special lane runs the full routine on every lane (for the other
    // lanes it is the same main path, the same bits)
    if (special_mask) res = g_exp_full(x, T);
    return res;
}

// __log_fma for every input: 0 -> -inf, +inf -> +inf, negative or NaN -> NaN, subnormals
// rescaled by 2^52 into the main path (e_log.c special cases).
template <class TT>
__host__ __device__ __forceinline__ double g_log_full(double x, const TT &T) {
    uint32_t hx = g_hi(x), lx = g_lo(x);
    if (hx - 0x3FEE0000u < 0x3FF10900u - 0x3FEE0000u) return g_log(x, T);
    const uint32_t top = hx >> 16;
    if (top - 0x0010u >= 0x7FF0u - 0x0010u) {
        if ((hx << 1) == 0 && lx == 0) return -__builtin_inf();
        if (hx == 0x7FF00000u && lx == 0) return x;
        if ((top & 0x8000u) || (top & 0x7FF0u) == 0x7FF0u) return __builtin_nan("");
        const double xs = x * 0x1p52;  // subnormal: ix = asuint64(x * 2^52) - (52 << 52)
        hx = g_hi(xs) - (52u << 20);
        lx = g_lo(xs);
    }
    const uint32_t th = hx - 0x3FE60000u;
    const int k = (int)th >> 20;
    const double2 c = T.lg[(th >> 13) & 127u];
    const double z = g_make(hx - (th & 0xFFF00000u), lx);
    const double r = __builtin_fma(z, c.x, -1.0);
    const double kd = (double)k;
    const double w = __builtin_fma(kd, kGlLn2hi, c.y);
    const double pA = __builtin_fma(r, kGlA2, kGlA1);
    const double hi = r + w;
    const double r2 = r * r;
    double lo = w - hi;
    lo = lo + r;
    lo = __builtin_fma(kd, kGlLn2lo, lo);
    const double r3 = r * r2;
    double pB = __builtin_fma(r, kGlA4, kGlA3);
    lo = __builtin_fma(r2, kGlA0, lo);
    pB = __builtin_fma(pB, r2, pA);
    return __builtin_fma(r3, pB, lo) + hi;
}

// The tables as device constant data, for call sites that have no LDS copy at hand
// (the rare erfc exp of the demapper's exact F_Y evaluations).
__constant__ static const GlibcTables kGlibcConst = QR_GLIBC_TABLES_INIT;

// ---- the box-plus domain: h(t) = log(1.0 + exp(-t)), t >= 0, inf or NaN ----------------
//
// GlibcK: the addends of the fmas whose two other operands are constants too.  gfx9
// VOP3 reads at most one SGPR, so each such fma costs a v_mov of its constant into a
// VGPR at every use; a kernel that keeps these eight in VGPRs (GlibcK::pinned(), once
// per thread) saves 8 VALU per h.  Host and default construction: plain constants.
#ifndef QR_PIN_K
#define QR_PIN_K 1
#endif
struct GlibcK {
    double shift = kGxShift, c2 = kGxC2, c4 = kGxC4, a1 = kGlA1, a3 = kGlA3, b1 = kGlB1, b4 = kGlB4, b7 = kGlB7;
    double two27 = 0x1p27;  // the near-1 split's multiplier (a VOP3 fma has no literal operand)
    __host__ __device__ static GlibcK pinned() {
        GlibcK k;
#if defined(__HIP_DEVICE_COMPILE__) && QR_PIN_K
        asm volatile("" : "+v"(k.shift), "+v"(k.c2), "+v"(k.c4), "+v"(k.a1));
        asm volatile("" : "+v"(k.a3), "+v"(k.b1), "+v"(k.b4), "+v"(k.b7), "+v"(k.two27));
#endif
        return k;
    }
};
//
// exp(x) for x in [-37.51, 0] or NaN: g_exp without the |x| < 2^-54 case, which the
// main path already rounds to exactly 1.0 + x there (= 1.0; tests/native pin it), and
// with the scale taken by ldexp (exact for these normal results).
template <class TT>
__host__ __device__ __forceinline__ double g_exp_neg(double x, const TT &T, const GlibcK &K = GlibcK()) {
    double kd = __builtin_fma(x, kGxInvLn2N, K.shift);
    const uint32_t ki = g_lo(kd);
    kd = kd - kGxShift;
    double r = __builtin_fma(kd, kGxNegLn2hiN, x);
    r = __builtin_fma(kd, kGxNegLn2loN, r);
#ifdef QR_EXPERIMENT_UNIFORM_EXP_IDX  // timing only (wrong results): a conflict-free broadcast read
    const double2 e = T.ex[__builtin_amdgcn_readfirstlane(ki) & 127u];
#else
    const double2 e = T.ex[ki & 255u];  // = entry ki % 128 (GlibcTables: ex is stored twice)
#endif
    const double r2 = r * r;
    const double p23 = __builtin_fma(r, kGxC3, K.c2);
    const double tr = e.x + r;
    const double p45 = __builtin_fma(r, kGxC5, K.c4);
    const double a = __builtin_fma(p23, r2, tr);
    const double r4 = r2 * r2;
    const double tmp = __builtin_fma(r4, p45, a);
    // sbits = tab[2i+1] + (ki << 45): the normal 2^(i/128) 2^k of glibc
    const double scale = g_make(g_add_ki(g_hi(e.y), ki), g_lo(e.y));
    return __builtin_fma(scale, tmp, scale);
}

// log(u) for u = 1.0 + exp(-t) in [1, 2] or NaN: g_log with the main path's scaled
// mantissa z = u 2^-k taken by ldexp (exact; it also carries a NaN through, which
// the bit arithmetic would not), and without the u == 1 early return (both branches
// return +0 there).  The two branches are written as separate chains:
//   g_log_near1  -- u in [1, 1 + 0x1.09p-4) (e_log.c "close to 1.0");
//   g_log_table  -- the {1/c, log c} table path (any other u).
__host__ __device__ __forceinline__ double g_log_near1(double x, const GlibcK &K) {
    const double r = x - 1.0;
    double p2 = __builtin_fma(r, kGlB2, K.b1);
    double p5 = __builtin_fma(r, kGlB5, K.b4);
    const double r2 = r * r;
    double p8 = __builtin_fma(r, kGlB8, K.b7);
    p2 = __builtin_fma(r2, kGlB3, p2);
    p5 = __builtin_fma(r2, kGlB6, p5);
    const double r3 = r * r2;
    p8 = __builtin_fma(r2, kGlB9, p8);
    p8 = __builtin_fma(r3, kGlB10, p8);
    p5 = __builtin_fma(p8, r3, p5);
    const double P = __builtin_fma(p5, r3, p2);
    const double t = __builtin_fma(r, K.two27, r);
    const double rhi = __builtin_fma(-K.two27, r, t);
    const double rhi2 = rhi * rhi;
    const double rlo = r - rhi;
    const double hi = __builtin_fma(rhi2, kGlB0, r);
    const double d = r - hi;
    const double rr = r + rhi;
    double lo = __builtin_fma(rhi2, kGlB0, d);
    const double q = kGlB0 * rlo;
    lo = __builtin_fma(q, rr, lo);
    return hi + __builtin_fma(P, r3, lo);
}
// (k folded into the lk / lc tables, see GlibcTables: valid for x in [1 + 0x1.09p-4, 2]
// and NaN, the box-plus domain of this path)
template <class TT>
__host__ __device__ __forceinline__ double g_log_table(double x, uint32_t hx, const TT &T,
                                                       const GlibcK &K) {
#ifdef QR_EXPERIMENT_UNIFORM_LOG_IDX  // timing only (wrong results)
    const GlibcLogK &c = T.lk[__builtin_amdgcn_readfirstlane(hx >> 13) & 127u];
#else
    const GlibcLogK &c = T.lk[(hx >> 13) & 127u];          // entry of i = ((hx - OFF) >> 13) & 127
#endif
    const double r = __builtin_fma(x, c.invc, -1.0);       // = fma(x 2^-k, invc, -1)
    const double w = c.w;                                  // = fma(k, Ln2hi, logc)
    const double pA = __builtin_fma(r, kGlA2, K.a1);
    const double hi = r + w;
    const double r2 = r * r;
    double lo = w - hi;
    lo = lo + r;
    lo = lo + c.c;                                         // = fma(k, Ln2lo, lo)
    const double r3 = r * r2;
    double pB = __builtin_fma(r, kGlA4, K.a3);
    lo = __builtin_fma(r2, kGlA0, lo);
    pB = __builtin_fma(pB, r2, pA);
    return __builtin_fma(r3, pB, lo) + hi;
}
template <class TT>
__host__ __device__ __forceinline__ double g_log_u(double x, const TT &T, const GlibcK &K = GlibcK()) {
    const uint32_t hx = g_hi(x);
    if (hx < 0x3FF10900u) return g_log_near1(x, K);  // u in [1, 1 + 0x1.09p-4)
    return g_log_table(x, hx, T, K);
}
// The same bits without divergent control flow: both chains are evaluated and the
// lane's branch is selected.  Within a wavefront the 64 frames' arguments straddle
// the near-1 threshold (t = 2.738) almost always, so the branchy version executes
// both chains anyway -- one after the other, each a serial dependency chain whose
// table path starts with an LDS read.  As one basic block the two chains (and those
// of the other h of the box-plus) interleave and hide each other's latency.
template <class TT>
__host__ __device__ __forceinline__ double g_log_u_sel(double x, const TT &T, const GlibcK &K = GlibcK()) {
    const uint32_t hx = g_hi(x);
    const double yn = g_log_near1(x, K);
    const double yt = g_log_table(x, hx, T, K);
    return (hx < 0x3FF10900u) ? yn : yt;
}

// h(t) exactly as the reference evaluates it.  t > 37.5 is moved into
// [37.5, 37.5 + 2^-15) by replacing its high word (there exp(-t) < 2^-54, so
// 1.0 + exp(-t) == 1.0 and log(1.0) == 0, exactly what the reference returns for
// every t >= 36.74, inf included); NaN fails the compare and propagates.
// The argument may carry a sign: h(|s|) (the box-plus passes a + b and a - b; the abs
// and the negation fold into the source modifiers of exp's first fmas).
template <bool SEL = false, class TT = GlibcTables>
__host__ __device__ __forceinline__ double h_strict(double s, const TT &T, const GlibcK &K = GlibcK()) {
    const double tc = g_make((fabs(s) > 37.5) ? 0x4042C000u : g_hi(s), g_lo(s));
    const double u = 1.0 + g_exp_neg(-fabs(tc), T, K);
    return SEL ? g_log_u_sel(u, T, K) : g_log_u(u, T, K);
}

// decoder.pyx:41-45: (sgn(a)sgn(b) * min + h(|a+b|)) - h(|a-b|), each operation
// rounded separately.  sgn(a)sgn(b)*min == copysign(min, a*b) up to the sign of an
// exact zero and NaN cases, neither of which changes the result (a NaN operand makes
// h(|a+-b|) NaN; a zero min adds a zero to h >= 0).
// QR_STRICT_MAXMIN: the two h are taken at t+ = |a|+|b| and t- = ||a|-|b|| (the same
// two values: |a+b| = t+ and |a-b| = t- when a*b >= 0, swapped otherwise, exactly, also
// for zeros, infinities and NaN) so that each call site sees one population (t+ mostly
// beyond the near-1 threshold t = 2.738 of g_log, t- mostly below) and its waves
// rarely have to run both branches of g_log.
// sgn(a) sgn(b) min(|a|, |b|) with the reference's min, (|b| < |a|) ? |b| : |a|
// (decoder.pyx:41-45), and the sign as the XOR of the operands' sign bits: selects and
// bit operations instead of fmin (whose IEEE-mode NaN canonicalisation costs two more
// fp64 instructions) and a multiply.  Zeros and NaN are discussed above.
__host__ __device__ __forceinline__ uint32_t g_bfi(uint32_t mask, uint32_t a, uint32_t b) {  // (a & mask) | (b & ~mask)
#if defined(__HIP_DEVICE_COMPILE__)
    uint32_t r;
    asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(r) : "s"(mask), "v"(a), "v"(b));  // the compiler's own: and, and, or
    return r;
#else
    return (a & mask) | (b & ~mask);
#endif
}
__host__ __device__ __forceinline__ double signed_min(double a, double b) {
    const bool bl = fabs(b) < fabs(a);
    const uint32_t hm = bl ? g_hi(b) : g_hi(a), lm = bl ? g_lo(b) : g_lo(a);
    // bit-field insert: magnitude bits of the selected operand, sign of a XOR b
    return g_make(g_bfi(0x7FFFFFFFu, hm, g_hi(a) ^ g_hi(b)), lm);
}



// QR_STRICT_SEL: h evaluated branch-free (g_log_u_sel); measured slower on MI355X
// (5.51 vs 5.22 ms per check launch: same fp64 count, +100 selects), so off by default.
#ifndef QR_STRICT_MAXMIN
#define QR_STRICT_MAXMIN 0
#endif
#ifndef QR_STRICT_SEL
#define QR_STRICT_SEL 0
#endif
template <bool SEL, class TT>
__host__ __device__ __forceinline__ double box_plus_strict_t(double a, double b, const TT &T,
                                                            const GlibcK &K = GlibcK()) {
    const double sm = signed_min(a, b);
#if QR_STRICT_MAXMIN
    const double ab = a * b;
#endif
#if QR_STRICT_MAXMIN
    const double hp = h_strict<SEL>(fabs(a) + fabs(b), T, K);
    const double hm = h_strict<SEL>(fabs(fabs(a) - fabs(b)), T, K);
    const bool same = !(ab < 0.0);
    return (sm + (same ? hp : hm)) - (same ? hm : hp);
#else
    return (sm + h_strict<SEL>(a + b, T, K)) - h_strict<SEL>(a - b, T, K);
#endif
}
template <class TT>
__host__ __device__ __forceinline__ double box_plus_strict(double a, double b, const TT &T,
                                                          const GlibcK &K = GlibcK()) {
    return box_plus_strict_t<QR_STRICT_SEL != 0>(a, b, T, K);
}

}  // namespace qr
