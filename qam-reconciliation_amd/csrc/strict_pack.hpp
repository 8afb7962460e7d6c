// strict_pack.hpp -- the strict (bit-exact) check-node update with the two branches of
// glibc log run on full wavefronts.
//
// The reference's check update (decoder.pyx:322-369) is 3(D-2) box-plus per check, each
// two h(t) = log(1.0 + exp(-t)) (decoder.pyx:41-45).  glibc log has two code paths for
// the u = 1 + exp(-t) in [1, 2] of the box-plus: the near-1 polynomial (u < 1 + 0x1.09p-4,
// i.e. t > 2.738) and the table path.  One lane = one frame, so a wavefront's 64 frames
// straddle that threshold in ~98-100 % of all box-plus call sites (scripts/diag/
// branch_stats.py, configs[2] at 3 dB) and the branchy h executes BOTH paths for every
// h: ~40 of its ~54 fp64 instructions are the log, half of them discarded.
//
// Here the box-plus of one check are evaluated in dependency rounds instead of the
// reference's sequential F / B / output loops (same operands for every box-plus, so the
// same bits):
//   F_k = bp(F_{k-1}, m_k)   in round k            (F_0 = m_0)
//   B_j = bp(B_{j+1}, m_j)   in round D-1-j        (B_{D-1} = m_{D-1})
//   O_i = bp(F_{i-1}, B_{i+1}) in round max(i-1, D-2-i) + 1
// which gives D-2 rounds of 2..4 independent box-plus per lane (D = 7: 2, 2, 3, 4, 4).
// Per round every lane computes its exp's (branch-free) and writes its log arguments u
// into a per-wave LDS buffer -- the near-1 ones compacted from the front, the table ones
// from the back (ranks from a wave ballot + mbcnt) -- then the wave runs the near-1 path
// over ceil(nN/64) full slices and the table path over ceil(nT/64), writes the results
// in place, and each lane reads its own back: NJ + 1 log passes for NJ = 2K arguments
// per lane instead of 2 NJ, ~6 VALU of bookkeeping per argument.  Every log is still glibc's __log_fma operation for
// operation on its own argument (glibc_math.hpp); only WHICH lane evaluates it changes.
#pragma once
#include "glibc_math.hpp"

namespace qr {

// LDS pointers by address (32-bit byte addresses in the LDS aperture).
typedef __attribute__((address_space(3))) double lds_f64;

// Log arguments per lane per round: at most 4 box-plus x 2 h.
constexpr int kPackMaxJobs = 8;
// LDS per wavefront: 64 lanes x kPackMaxJobs arguments + one slice of slack (below).
constexpr int kPackWaveDoubles = 64 * kPackMaxJobs + 64;

// round in which the output box-plus O_i (1 <= i <= D-2) becomes computable
__host__ __device__ constexpr int pack_out_round(int D, int i) {
    return ((i - 1) > (D - 2 - i) ? (i - 1) : (D - 2 - i)) + 1;
}

// h(t) = log(1.0 + exp(-|t|)) for nj (<= kPackMaxJobs; compile-time after unrolling)
// arguments per lane.  wb: this wavefront's LDS buffer of kPackWaveDoubles = S slots.
// The near-1 arguments go to slots [0, nN) in job order, the table ones to (S-1-nT, S-1]
// counted from the top; a pass is one full 64-slot slice read at an immediate offset and
// written back in place, unguarded: the surplus lanes of the last near slice write into
// [nN, nN + 64) and those of the last table slice into (S-1-nT-64, S-1-nT], which never
// reach the other kind's slots because nN + nT <= S - 64.
// The argument of exp, -|t|, by clamp mode CL:
//   kClampFull  : t > 37.5 moved into [37.5, 37.5 + 2^-15) by its high word (h_strict; any
//                 input, NaN propagates);
//   kClampFinite: max(-|t|, -700), one v_max_f64 -- for waves whose inputs are all finite,
//                 where no NaN can arise in the box-plus (finite operands give finite t, h);
//   kClampNone  : -|t| as it stands -- every |t| < 700 (the caller has checked its inputs).
// Below 700 glibc exp's main path is valid for -|t| as written (normal result, k >= -1010),
// and for every t > 37.5 exp(-t) < 2^-54, so u = fl(1.0 + exp(-t)) == 1.0 and h == +0 in all
// three modes: the same bits.
enum { kClampNone = 0, kClampFull = 1, kClampFinite = 2 };
template <int CL = kClampFull, class TT = GlibcTables>
__device__ __forceinline__ void h_packed(const double *t, double *h, int nj, double *wb, const TT &T,
                                         const GlibcK &K) {
    constexpr int S = kPackWaveDoubles;
    const uint32_t lane = __lane_id();
    uint32_t addr[kPackMaxJobs];  // byte address of the argument's slot
    uint32_t nN = 0;              // wave-uniform: near-1 arguments written so far
    // element index of slot s: wb0 + s; a table argument's slot is nN + (near lanes below)
    // + (S-1 - lane) - 64 j, i.e. the near formula plus a per-lane, per-job offset
    const uint32_t wb0 = (uint32_t)(uintptr_t)(lds_f64 *)wb / 8u;
#pragma unroll
    for (int j = 0; j < kPackMaxJobs; ++j) {
        if (j >= nj) break;
        double xe;
        if constexpr (CL == kClampFull) xe = -fabs(g_make((fabs(t[j]) > 37.5) ? 0x4042C000u : g_hi(t[j]), g_lo(t[j])));
        else if constexpr (CL == kClampFinite) xe = __builtin_fmax(-fabs(t[j]), -700.0);
        else xe = -fabs(t[j]);
        const double u = 1.0 + g_exp_neg(xe, T, K);  // h_strict: h(|t|)
        const bool near = g_hi(u) < 0x3FF10900u;  // g_log_u's branch (NaN: table path)
        const uint64_t mk = __ballot(near);
        const uint32_t x = near ? wb0 : wb0 + (uint32_t)(S - 1) - lane - 64u * (uint32_t)j;
        const uint32_t a = __builtin_amdgcn_mbcnt_hi((uint32_t)(mk >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mk, x));
        addr[j] = (a + nN) << 3;
        *(lds_f64 *)(uintptr_t)addr[j] = u;
        nN += (uint32_t)__popcll(mk);
    }
    const uint32_t nT = 64u * (uint32_t)nj - nN;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    // slices: near q at wn[64 q], table q at wt[64 (kPackMaxJobs - q)]; the next slice is
    // read before the current one is evaluated (slices past the last one are in bounds)
    double *wn = wb + lane;
    double *wt = wb + (S - 1 - 64 * kPackMaxJobs) - lane;
    double cur = wn[0];
#pragma unroll
    for (int q = 0; q <= kPackMaxJobs; ++q) {
        if (64u * (uint32_t)q >= nN) break;  // wave-uniform
        const double nxt = (q < kPackMaxJobs) ? wn[64 * (q + 1)] : 0.0;
        wn[64 * q] = g_log_near1(cur, K);
        cur = nxt;
    }
    cur = wt[64 * kPackMaxJobs];
#pragma unroll
    for (int q = 0; q <= kPackMaxJobs; ++q) {
        if (64u * (uint32_t)q >= nT) break;  // wave-uniform
        const double nxt = (q < kPackMaxJobs) ? wt[64 * (kPackMaxJobs - q - 1)] : 0.0;
        wt[64 * (kPackMaxJobs - q)] = g_log_table(cur, g_hi(cur), T, K);
        cur = nxt;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
    for (int j = 0; j < kPackMaxJobs; ++j) {
        if (j >= nj) break;
        h[j] = *(const lds_f64 *)(uintptr_t)addr[j];
    }
    // the next round overwrites the buffer: every lane has read its results first
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// sgn(a) sgn(b) min(|a|, |b|) of the box-plus (decoder.pyx:41-45) with the magnitude from
// v_min_f64: every operand here is the result of an fp64 add or subtract, so the compiler
// knows it canonical and emits one v_min_f64 with |.| modifiers instead of the compare + two
// selects.  Equal magnitudes have equal bits (+-0 included), and a NaN operand makes both h
// arguments NaN, so the box-plus is NaN whatever min returns.
__device__ __forceinline__ double signed_min_packed(double a, double b) {
    const double mn = __builtin_fmin(__builtin_fabs(a), __builtin_fabs(b));
    return g_make(g_bfi(0x7FFFFFFFu, g_hi(mn), g_hi(a) ^ g_hi(b)), g_lo(mn));
}

// decoder.pyx:322-369 for one check of degree D (>= 2): out[i] = c2v of edge i before
// the syndrome sign.  The same box-plus (operands and box_plus_strict's operation order)
// as check_exact<kStrict>, evaluated round by round.
template <int D, int CL = kClampFull, class TT = GlibcTables>
__device__ __forceinline__ void check_strict_packed(const double (&m)[D], double (&out)[D], double *wb, const TT &T,
                                                    const GlibcK &K) {
    if constexpr (D == 2) {
        out[0] = m[1];
        out[1] = m[0];
    } else {
        double F[D], Bv[D];
        F[0] = m[0];
        Bv[D - 1] = m[D - 1];
#pragma unroll
        for (int r = 1; r <= D - 2; ++r) {
            // the round's box-plus: kind 0 = F_r, 1 = B_{D-1-r}, 2 = O_i
            int kind[4], idx[4];
            int k = 0;
            kind[k] = 0, idx[k] = r, ++k;
            kind[k] = 1, idx[k] = D - 1 - r, ++k;
#pragma unroll
            for (int i = 1; i <= D - 2; ++i)
                if (pack_out_round(D, i) == r) kind[k] = 2, idx[k] = i, ++k;
            // box_plus_strict_t: (sm + h(|a + b|)) - h(|a - b|)
            double t[8], h[8], sm[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                if (q >= k) break;
                const double a = kind[q] == 0 ? F[r - 1] : kind[q] == 1 ? Bv[D - r] : F[idx[q] - 1];
                const double b = kind[q] == 0 ? m[r] : kind[q] == 1 ? m[D - 1 - r] : Bv[idx[q] + 1];
                sm[q] = signed_min_packed(a, b);
                t[2 * q] = a + b;
                t[2 * q + 1] = a - b;
            }
            h_packed<CL>(t, h, 2 * k, wb, T, K);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                if (q >= k) break;
                const double v = (sm[q] + h[2 * q]) - h[2 * q + 1];
                if (kind[q] == 0) F[idx[q]] = v;
                else if (kind[q] == 1) Bv[idx[q]] = v;
                else out[idx[q]] = v;
            }
        }
        out[0] = Bv[1];
        out[D - 1] = F[D - 2];
    }
}

}  // namespace qr
