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
// per lane instead of 2 NJ.  Every log is still glibc's __log_fma operation for
// operation on its own argument (glibc_math.hpp); only WHICH lane evaluates it changes.
#pragma once
#include "glibc_math.hpp"

namespace qr {

// Log arguments per lane per round: at most 4 box-plus x 2 h.
constexpr int kPackMaxJobs = 8;
// LDS per wavefront: 64 lanes x kPackMaxJobs doubles = 4 KiB.
constexpr int kPackWaveDoubles = 64 * kPackMaxJobs;

// round in which the output box-plus O_i (1 <= i <= D-2) becomes computable
__host__ __device__ constexpr int pack_out_round(int D, int i) {
    return ((i - 1) > (D - 2 - i) ? (i - 1) : (D - 2 - i)) + 1;
}

// h(t) for NJ (<= kPackMaxJobs, compile-time after unrolling) arguments per lane.
// wb: this wavefront's LDS buffer (kPackWaveDoubles).
__device__ __forceinline__ void h_packed(const double *t, double *h, int nj, double *wb, const GlibcTables &T,
                                         const GlibcK &K) {
    const uint32_t lane = __lane_id();
    const uint32_t total = 64u * (uint32_t)nj;
    uint32_t pos[kPackMaxJobs];
    uint32_t nN = 0;  // wave-uniform: near-1 arguments written so far
#pragma unroll
    for (int j = 0; j < kPackMaxJobs; ++j) {
        if (j >= nj) break;
        const double tc = g_make((fabs(t[j]) > 37.5) ? 0x4042C000u : g_hi(t[j]), g_lo(t[j]));
        const double u = 1.0 + g_exp_neg(-fabs(tc), T, K);  // h_strict: h(|t|)
        const bool near = g_hi(u) < 0x3FF10900u;  // g_log_u's branch (NaN: table path)
        const uint64_t mk = __ballot(near);
        const uint32_t below = __builtin_amdgcn_mbcnt_hi((uint32_t)(mk >> 32),
                                                        __builtin_amdgcn_mbcnt_lo((uint32_t)mk, nN));
        // near: rank among the near arguments; table: from the back, rank among the others
        pos[j] = near ? below : (total - 1u) - ((uint32_t)j * 64u + lane - below);
        wb[pos[j]] = u;
        nN += (uint32_t)__popcll(mk);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    // near-1 path over [0, nN), table path over [nN, total); slices are full wavefronts
    // except one of each kind, whose surplus lanes compute on the other kind's argument
    // and do not write.
    for (uint32_t p = 0; p < nN; p += 64u) {
        const uint32_t i = p + lane;
        const double y = g_log_near1(wb[i], K);
        if (i < nN) wb[i] = y;
    }
    for (int p = (int)total - 64; p + 64 > (int)nN; p -= 64) {
        const uint32_t i = (uint32_t)p + lane;
        const double u = wb[i];
        const double y = g_log_table(u, g_hi(u), T, K);
        if (i >= nN) wb[i] = y;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
    for (int j = 0; j < kPackMaxJobs; ++j) {
        if (j >= nj) break;
        h[j] = wb[pos[j]];
    }
    // the next round overwrites the buffer: every lane has read its results first
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// decoder.pyx:322-369 for one check of degree D (>= 2): out[i] = c2v of edge i before
// the syndrome sign.  The same box-plus (operands and box_plus_strict's operation order)
// as check_exact<kStrict>, evaluated round by round.
template <int D>
__device__ __forceinline__ void check_strict_packed(const double (&m)[D], double (&out)[D], double *wb,
                                                    const GlibcTables &T, const GlibcK &K) {
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
            double a[4], b[4];
            int kind[4], idx[4];
            int k = 0;
            a[k] = F[r - 1], b[k] = m[r], kind[k] = 0, idx[k] = r, ++k;
            a[k] = Bv[D - r], b[k] = m[D - 1 - r], kind[k] = 1, idx[k] = D - 1 - r, ++k;
#pragma unroll
            for (int i = 1; i <= D - 2; ++i)
                if (pack_out_round(D, i) == r) a[k] = F[i - 1], b[k] = Bv[i + 1], kind[k] = 2, idx[k] = i, ++k;
            // box_plus_strict_t: (sm + h(|a + b|)) - h(|a - b|)
            double t[8], h[8], sm[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                if (q >= k) break;
                sm[q] = signed_min(a[q], b[q]);
                t[2 * q] = a[q] + b[q];
                t[2 * q + 1] = a[q] - b[q];
            }
            h_packed(t, h, 2 * k, wb, T, K);
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
