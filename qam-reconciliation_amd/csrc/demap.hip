// demap.hip -- PAM/BICM soft demapper (Alice side of the softening scheme) and
// the Bob-side producers of its inputs, for gfx950.
//
// Reference: qamreconciliation/noisemapper.pyx (NoiseMapper), alphabet.pyx,
// bicm.pyx, matrix.pyx, utils.pyx, sims/reconciliation.pyx:93-168.
//
// One lane = one (symbol, frame).  The lane runs the reference's per-symbol
// procedure (noisemapper.pyx:450-540) sequentially: for each hypothesis i a
// bracket + bisection inversion of the mixture CDF F_Y (31..40 F_Y
// evaluations of M scipy-exact erf each), then the Gray-labelled N/D sums in
// i order.  This is fp64-VALU bound (bytes are negligible); lanes of a wave
// hold 64 consecutive frames of the same symbol position so the LAPPR stores
// land directly, coalesced, in the decoder's frame-innermost input layout.
#include <atomic>
#include <vector>

#include "qamr_internal.hpp"
#include "host_build.hpp"

namespace qr {

// 1 = Newton-located root + replayed bisection (bit-identical, ~5x fewer erf), 0 = brute force.
std::atomic<int> g_demap_fast{1};
// Demap kernel on 64-frame tiles (knob demap_hyp): 1 (default) = wave-private (k_demap_wave: one
// wave walks all M hypotheses of its 64-frame tile), 0 = one lane per symbol (k_demap).  Measured
// on MI355X, B = 4096: 16-PAM 13 dB 44.2 vs 47.1 ms, 25 dB 52.2 vs 52.8 ms, 4-PAM 13.7 vs 13.8 ms;
// the round-3 hypothesis-parallel kernel (waves split the hypotheses, two workgroup barriers per
// symbol item) took 46.8 / 54.7 / 20.0 ms and was removed.
std::atomic<int> g_demap_hyp{1};

// Occupancy floor of the per-symbol kernel: 5 waves/SIMD (96 VGPRs, 52-84 B spilled) 53.4 / 58.5 ms
// vs 4 waves 55.9 / 62.5 ms (16-PAM at 13 / 25 dB, 4096 frames), 4-PAM 14.5 ms either way.
constexpr int kDemapWaves = 5;
template <bool FAST, int BPS>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(kDemapWaves, 8))) k_demap(const DemapTables *__restrict__ tab, const MathTables *__restrict__ gmt,
                                               int B, int ld, int64_t S, const double *__restrict__ n,
                                               const int64_t *__restrict__ j, double alpha,
                                               double *__restrict__ lappr) {
    __shared__ MathTables mt;
    __shared__ GlibcTables gt;
    stage_math_tables(&mt, gmt);
    stage_glibc_tables(&gt, &kGlibcConst);
    const int64_t item = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t s = item / ld;
    const int f = (int)(item - s * ld);
    if (s >= S || f >= B) return;
    const DemapTables &t = *tab;
    const double nv = n[s * ld + f];
    const int64_t jv = j[s * ld + f];
    double out[BPS];
    if (jv < 0 || jv >= (1 << BPS)) {
#pragma unroll
        for (int k = 0; k < BPS; ++k) out[k] = __builtin_nan("");
    } else {
        demap_symbol<FAST, BPS>(t, mt, gt, nv, (int)jv, alpha, out);
    }
#pragma unroll
    for (int k = 0; k < BPS; ++k) lappr[(s * BPS + k) * ld + f] = out[k];
}

// ---------------------------------------------------------------------------
// Root search of the 64-frame-tile demapper (k_demap_wave, below).  The certified closed form
// of the search needs at most one exact F_Y per (frame, hypothesis), for ~2 % of the lanes;
// instead of the wave running a divergent M-erf F_Y whenever any of its lanes needs one, the
// lanes' evaluation points are compacted into LDS (ballot + mbcnt) and the wave evaluates
// their M erf terms with one lane per (point, m), 64 / M points per pass, after which each
// owner sums its M terms in m order (noisemapper.pyx:278-286: the same products, the same
// sequence of additions).
constexpr int kDemapWaveMaxBps = 6;
#if QR_EXPERIMENT_CLOCK
// the in-kernel clock of the wave-private demapper's launches (diagnostic twin only): {cycles,
// ticks, workgroups}, read and cleared by qr_debug_clock_demap
__device__ unsigned long long g_clk_demap[3];
#endif
// LLR-sum loop unroll of k_demap_wave (1 / 16: 50.3 / 57.0 ms vs 46.8 at 4, 16-PAM, round 3)
constexpr int kDemapUnroll = 4;

// rank of this lane among the set lanes of mk below it
__device__ __forceinline__ int lane_rank(uint64_t mk) {
    return (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(mk >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mk, 0u));
}

__device__ __forceinline__ void wave_lds_fence() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// g_inv_search_fast (qamr_math.hpp) with the closed form's exact F_Y evaluated by the
// whole wave (see above).  Every lane of the wave must call it (wave-uniform i).
// ey / et: this wave's 64-double LDS buffers (evaluation points, erf terms).
template <int M>
__device__ __forceinline__ double g_inv_search_wave(const DemapTables &t, const MathTables &mt, double n_hat, int i,
                                                    double *ey, double *et, int lane) {
    SearchCmp cmp{&t, search_target(t, n_hat, i), 0.0, 0.0, false};
    cmp.have = newton_root(t, mt, cmp.T, i, cmp.ystar, cmp.W);   // T lies in region i
    double L = 0.0, H = 0.0;
    int need = 0;
    const bool closed = cmp.have && search_closed_prepare(cmp, L, H, need);
    const bool ask = need != 0;
    const uint64_t mk = __ballot(ask);
    bool gt = false;
    if (mk) {  // wave-uniform
        const int cnt = __popcll(mk);
        const int rank = lane_rank(mk);
        if (ask) ey[rank] = (need == 1) ? L : H;
        wave_lds_fence();
        constexpr int P = 64 / M;  // points per pass
        const int sub = lane / M, m = lane % M;
        for (int base = 0; base < cnt; base += P) {   // wave-uniform trip count
            const int item = base + sub;
            if (item < cnt) et[lane] = (0.5 * (1 + cephes_erf((ey[item] - t.a[m]) / t.den))) * t.p[m];
            wave_lds_fence();
            if (ask && rank >= base && rank < base + P) {
                const double *tt = et + (rank - base) * M;
                double F = tt[0];                     // noisemapper.pyx:282-285, m = 0 first
#pragma unroll
                for (int mm = 1; mm < M; ++mm) F += tt[mm];
                gt = F > cmp.T;                       // SearchCmp::exact(y) > 0
            }
            wave_lds_fence();
        }
    }
    if (closed) return search_closed_finish(L, H, need, gt);
    return search_replay(cmp);   // no certified window / outside the closed form (rare): per lane
}

// ---------------------------------------------------------------------------
// Wave-private demapper (knob demap_hyp = 1, the default): ONE wave walks all M hypotheses of its
// own 64-frame tile (lane = frame; the reference's loop over i, noisemapper.pyx:490-530) and
// keeps the Gray-labelled sums N[k] / D[k] of its lanes in a wave-private LDS slice, updated
// in i order (noisemapper.pyx:521-530: per bit the reference's sequence of additions).  No
// workgroup barrier: a wave's search lengths never hold up another wave.  The exact F_Y of the
// closed-form root search is evaluated by the whole wave as in g_inv_search_wave.
// 127 VGPRs, 4 waves/SIMD.  Forced to 5 / 6 waves (96 / 80 VGPRs, 108 / 160 B spilled per lane):
// 16-PAM 44.2-44.3 / 44.6-44.7 ms vs 44.0-44.1, 4-PAM 16.9 / 19.1 ms vs 13.7 (MI355X, B = 4096).
template <int BPS>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4, 8))) k_demap_wave(const DemapTables *__restrict__ tab,
                                                    const MathTables *__restrict__ gmt, int B, int ld, int64_t S,
                                                    const double *__restrict__ n, const int64_t *__restrict__ j,
                                                    double alpha, double *__restrict__ lappr) {
    constexpr int M = 1 << BPS;
#if QR_EXPERIMENT_CLOCK
    ClkScope clk(true, g_clk_demap, nullptr);  // (diagnostic twin only)
#endif
    __shared__ GlibcExpLog gt;
    __shared__ double ey[4][64], et[4][64];
    __shared__ double acc[4][2 * BPS][64];   // per wave: N[k] rows then D[k] rows, lane = frame
    stage_glibc_exp_log(&gt, &kGlibcConst);
    const DemapTables &t = *tab;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    double *accw = &acc[w][0][0];
    const int64_t tiles = ld / 64;
    const int64_t items = S * tiles;
    for (int64_t it = (int64_t)blockIdx.x * 4 + w; it < items; it += (int64_t)gridDim.x * 4) {   // wave-uniform
        const int64_t s = it / tiles;
        const int f = (int)(it - s * tiles) * 64 + lane;
        const bool valid = f < B;
        const double nv = valid ? n[s * ld + f] : 0.5;   // padding lanes: a harmless target
        const int64_t jv = valid ? j[s * ld + f] : 0;
        const bool jok = jv >= 0 && jv < M;
        const int jj = jok ? (int)jv : 0;
        const double aj = t.a[jj], pj = t.p[jj];
#pragma unroll
        for (int k = 0; k < 2 * BPS; ++k) accw[k * 64 + lane] = 0.0;
#pragma unroll 1
        for (int i = 0; i < M; ++i) {
#ifdef QR_EXPERIMENT_NO_SEARCH  // cost-breakdown timing builds only (wrong results): the Hermite start as the root
            const double y = quantile_start(t, i, search_target(t, nv, i));
#else
            const double y = g_inv_search_wave<M>(t, *gmt, nv, i, ey[w], et[w], lane);
#endif
            // noisemapper.pyx:503-515 in the reference's summation order (k < j, p[j], k > j).
            // Straight-line: every lane computes both exponents (e, and e / 2 sigma^2 for k > j;
            // the missing / 2 sigma^2 for k < j is the reference's, noisemapper.pyx:503-507)
            // and selects -- the lanes of a wave hold different j, so a branch around the
            // division ran for nearly every k anyway, plus its exec-mask bookkeeping -- and
            // p[j] is the lane's own, loaded once per tile.
            double sum = 0;
#ifdef QR_EXPERIMENT_NO_LLR  // cost-breakdown timing builds only (wrong results): no LLR sum
            sum = pj + y * 1e-300;
#else
#pragma unroll kDemapUnroll
            for (int k = 0; k < M; ++k) {
                const double ak = t.a[k];
                const double e = (2 * y - ak - aj) * (ak - aj);
                const double ed = div_two_s2(t, e);
                // k == j: the term is p[j] and the exp is not used, but its argument must stay off
                // exp's special cases -- e is 0 there, and one such lane sends the whole wave
                // through the full routine at every k (measured 40.1 -> 46.5 ms)
                const double arg = k < jj ? e : k == jj ? 1.0 : ed;
                const double ex = g_exp_wave(arg, gt);
                const double tk = ex * t.p[k];
                sum += k == jj ? pj : tk;
            }
#endif
            const double q = t.dF[i] / sum;
            int mi = i;
#pragma unroll
            for (int k = 0; k < BPS; ++k) {   // noisemapper.pyx:521-530: Gray bit k of i
                double *a = accw + (((mi * (mi + 1)) & 3) ? BPS + k : k) * 64 + lane;
                *a += q;
                mi >>= 1;
            }
        }
#pragma unroll
        for (int k = 0; k < BPS; ++k) {
            const double out = (g_log_full(accw[k * 64 + lane], gt) - g_log_full(accw[(BPS + k) * 64 + lane], gt)) *
                               alpha;   // :534-538, x alpha
            if (valid) lappr[(s * BPS + k) * ld + f] = jok ? out : __builtin_nan("");
        }
    }
}

static bool launch_demap_wave(int bps, unsigned grid, hipStream_t st, const qr_demap *dm, int B, int ld, int64_t S,
                              const double *n, const int64_t *j, double alpha, double *lappr) {
    switch (bps) {
#define QR_DEMAP_WAVE(b) \
        case b: k_demap_wave<b><<<grid, 256, 0, st>>>(dm->d_tables, dm->d_mtab, B, ld, S, n, j, alpha, lappr); return true;
        QR_DEMAP_WAVE(1) QR_DEMAP_WAVE(2) QR_DEMAP_WAVE(3) QR_DEMAP_WAVE(4) QR_DEMAP_WAVE(5) QR_DEMAP_WAVE(6)
#undef QR_DEMAP_WAVE
        default: return false;
    }
}

// workgroups of the grid-stride demap: enough to fill every CU several times over
static unsigned demap_wave_grid(int device, int64_t items) {
    static std::atomic<int> cus[64];
    int cu = (device >= 0 && device < 64) ? cus[device].load() : 0;
    if (cu <= 0) {
        if (hipDeviceGetAttribute(&cu, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || cu <= 0)
            cu = 256;
        if (device >= 0 && device < 64) cus[device].store(cu);
    }
    const int64_t want = (int64_t)cu * 16;
    return (unsigned)(items < want ? items : want);
}

template <int BPS>
static void launch_demap(bool fast, unsigned grid, hipStream_t st, const qr_demap *dm, int B, int ld, int64_t S,
                         const double *n, const int64_t *j, double alpha, double *lappr) {
    if (fast) k_demap<true, BPS><<<grid, 256, 0, st>>>(dm->d_tables, dm->d_mtab, B, ld, S, n, j, alpha, lappr);
    else k_demap<false, BPS><<<grid, 256, 0, st>>>(dm->d_tables, dm->d_mtab, B, ld, S, n, j, alpha, lappr);
}

static void launch_demap_bps(int bps, bool fast, unsigned grid, hipStream_t st, const qr_demap *dm, int B, int ld,
                             int64_t S, const double *n, const int64_t *j, double alpha, double *lappr) {
    switch (bps) {
        case 1: launch_demap<1>(fast, grid, st, dm, B, ld, S, n, j, alpha, lappr); break;
        case 2: launch_demap<2>(fast, grid, st, dm, B, ld, S, n, j, alpha, lappr); break;
        case 3: launch_demap<3>(fast, grid, st, dm, B, ld, S, n, j, alpha, lappr); break;
        case 4: launch_demap<4>(fast, grid, st, dm, B, ld, S, n, j, alpha, lappr); break;
        case 5: launch_demap<5>(fast, grid, st, dm, B, ld, S, n, j, alpha, lappr); break;
        case 6: launch_demap<6>(fast, grid, st, dm, B, ld, S, n, j, alpha, lappr); break;
        case 7: launch_demap<7>(fast, grid, st, dm, B, ld, S, n, j, alpha, lappr); break;
        default: launch_demap<8>(fast, grid, st, dm, B, ld, S, n, j, alpha, lappr); break;
    }
}

// Bob: hard decision (noisemapper.pyx:349-359), transformed noise g(y, x_hat)
// (:289-292, :373-388) and Gray bits of x_hat (alphabet.pyx:98-107, bicm.pyx:26-41).
__global__ void __launch_bounds__(256) k_bob(const DemapTables *__restrict__ tab, int B, int ld, int64_t S,
                                             const double *__restrict__ y, int64_t *__restrict__ xhat,
                                             double *__restrict__ nhat, uint8_t *__restrict__ word) {
    const int64_t item = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t s = item / ld;
    const int f = (int)(item - s * ld);
    if (s >= S || f >= B) return;
    const DemapTables &t = *tab;
    const double yv = y[s * ld + f];
    int i = binsearch_thr(t.thr, t.M + 1, yv);
    if (i == t.M) i = t.M - 1;
    double g;
    if (t.sign[i]) g = (t.Fthr[i + 1] - single_F_Y(t, yv)) / t.dF[i];
    else           g = (single_F_Y(t, yv) - t.Fthr[i]) / t.dF[i];
    xhat[s * ld + f] = i;
    nhat[s * ld + f] = g;
    const int gray = i ^ (i >> 1);
    for (int k = 0; k < t.bps; ++k) word[(s * t.bps + k) * ld + f] = (uint8_t)((gray >> k) & 1);
}

// Direct reconciliation (sims/reconciliation.pyx:25-51, _y_to_lappr_grey): Bob's
// BICM LAPPRs of his own sample y, Gray-labelled log-sums over the alphabet.
// (y - a_i)**2 is evaluated as a product (the reference's pow(x, 2.0)).
__global__ void __launch_bounds__(256) k_direct_lappr(const DemapTables *__restrict__ tab, double two_var, int B,
                                                      int ld, int64_t S, const double *__restrict__ y,
                                                      double *__restrict__ lappr) {
    const int64_t item = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t s = item / ld;
    const int f = (int)(item - s * ld);
    if (s >= S || f >= B) return;
    const DemapTables &t = *tab;
    const double yv = y[s * ld + f];
    double N[kMaxBps], D[kMaxBps];
#pragma unroll
    for (int k = 0; k < kMaxBps; ++k) { N[k] = 0; D[k] = 0; }
    for (int i = 0; i < t.M; ++i) {
        const double d = yv - t.a[i];
        const double add = g_exp_full(-(d * d) / two_var, kGlibcConst);
        int mi = i;
#pragma unroll
        for (int k = 0; k < kMaxBps; ++k) {
            if (k < t.bps) {
                if ((mi * (mi + 1)) & 3) D[k] += add;
                else                     N[k] += add;
                mi >>= 1;
            }
        }
    }
#pragma unroll
    for (int k = 0; k < kMaxBps; ++k)
        if (k < t.bps) lappr[(s * t.bps + k) * ld + f] = g_log_full(N[k], kGlibcConst) - g_log_full(D[k], kGlibcConst);
}

// Hard reverse reconciliation (noisemapper.pyx:423-432, bare_llr): Alice's LAPPRs
// are the table row of her own symbol, table[M][bps] built on the host (:197-220).
__global__ void __launch_bounds__(256) k_bare_llr(const double *__restrict__ table, int M, int bps, int B, int ld,
                                                  int64_t S, const int64_t *__restrict__ x,
                                                  double *__restrict__ lappr) {
    const int64_t item = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t s = item / ld;
    const int f = (int)(item - s * ld);
    if (s >= S || f >= B) return;
    const int64_t xi = x[s * ld + f];
    const bool ok = xi >= 0 && xi < M;
    for (int k = 0; k < bps; ++k) lappr[(s * bps + k) * ld + f] = ok ? table[xi * bps + k] : __builtin_nan("");
}

// alphabet.pyx:98-107 with the reflected Gray table of bicm.pyx:26-41.
__global__ void __launch_bounds__(256) k_symbols_to_bits(int bps, int B, int ld, int64_t S,
                                                         const int64_t *__restrict__ x, uint8_t *__restrict__ word) {
    const int64_t item = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t s = item / ld;
    const int f = (int)(item - s * ld);
    if (s >= S || f >= ld) return;
    const int64_t xi = (f < B) ? x[s * ld + f] : 0;
    const int64_t g = xi ^ (xi >> 1);
    for (int k = 0; k < bps; ++k) word[(s * bps + k) * ld + f] = (uint8_t)((g >> k) & 1);
}

// noisemapper.pyx:289-292, :373-388 with a caller-given index (x_hat).
__global__ void __launch_bounds__(256) k_map_noise(const DemapTables *__restrict__ tab, int B, int ld, int64_t S,
                                                   const double *__restrict__ y, const int64_t *__restrict__ idx,
                                                   double *__restrict__ nhat) {
    const int64_t item = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t s = item / ld;
    const int f = (int)(item - s * ld);
    if (s >= S || f >= B) return;
    const DemapTables &t = *tab;
    const double yv = y[s * ld + f];
    const int64_t i = idx[s * ld + f];
    double g;
    if (i < 0 || i >= t.M) g = __builtin_nan("");
    else if (t.sign[i]) g = (t.Fthr[i + 1] - single_F_Y(t, yv)) / t.dF[i];
    else g = (single_F_Y(t, yv) - t.Fthr[i]) / t.dF[i];
    nhat[s * ld + f] = g;
}

// noisemapper.pyx:310-345 (cpdef g_inv_search) over arrays, i.e. :407-419 (demap_noise_search):
// y_hat[k] = g_inv_search(n_hat[k], i[k], y_accuracy).  At the default accuracy 1e-9 the fast
// certified search runs (bit-identical to the reference's loops: tests/test_demap_replay.py);
// any other accuracy runs the loops verbatim.  An out-of-range i gives NaN (the reference
// indexes sign_config / F_Y_thresholds out of bounds).
__global__ void __launch_bounds__(256) k_g_inv_search(const DemapTables *__restrict__ tab,
                                                      const MathTables *__restrict__ gmt, int64_t n,
                                                      const double *__restrict__ n_hat, const int64_t *__restrict__ idx,
                                                      double y_accuracy, int fast, double *__restrict__ y_hat) {
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    const DemapTables &t = *tab;
    const int64_t i = idx[k];
    double y;
    if (i < 0 || i >= t.M) y = __builtin_nan("");
    else if (fast && y_accuracy == 1e-9) y = g_inv_search_fast(t, *gmt, n_hat[k], (int)i);
    else y = g_inv_search(t, n_hat[k], (int)i, y_accuracy);
    y_hat[k] = y;
}

// noisemapper.pyx:264-275 (cpdef F_Y, uniform weighting).
__global__ void __launch_bounds__(256) k_public_F_Y(const DemapTables *__restrict__ tab, int64_t n,
                                                    const double *__restrict__ y, double *__restrict__ F) {
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k < n) F[k] = public_F_Y(*tab, y[k]);
}

// matrix.pyx:55-60, frame-innermost; one lane = (check, frame).
__global__ void __launch_bounds__(256) k_syndrome(int64_t C, int ld, int B, const int32_t *__restrict__ chk_ptr,
                                                  const int32_t *__restrict__ chk_var,
                                                  const uint8_t *__restrict__ word, uint8_t *__restrict__ synd) {
    const int f = blockIdx.y * blockDim.x + threadIdx.x;
    const int64_t c = blockIdx.x;
    if (c >= C || f >= ld) return;
    uint8_t x = 0;
    if (f < B)
        for (int k = chk_ptr[c]; k < chk_ptr[c + 1]; ++k) x ^= word[(size_t)chk_var[k] * ld + f];
    synd[(size_t)c * ld + f] = x;
}

// utils.pyx:27-40 (lappr >= 0 decides bit 0) over the first K nodes, then the
// per-frame bookkeeping of reconciliation.pyx:149-157.
__global__ void __launch_bounds__(256) k_count_errors(int B, int ld, int64_t K, int64_t kpb,
                                                      const double *__restrict__ fin,
                                                      const uint8_t *__restrict__ word, int32_t *__restrict__ ferr) {
    const int f = blockIdx.y * blockDim.x + threadIdx.x;
    if (f >= B) return;
    const int64_t v0 = (int64_t)blockIdx.x * kpb;
    const int64_t v1 = (v0 + kpb < K) ? v0 + kpb : K;
    int32_t cnt = 0;
    for (int64_t v = v0; v < v1; ++v) {
        const uint8_t w = word[v * ld + f];
        cnt += (fin[v * ld + f] >= 0) ? w : 1 - w;
    }
    if (cnt) atomicAdd(&ferr[f], cnt);
}

__global__ void k_count_finish(int B, const int32_t *__restrict__ ferr, const uint8_t *__restrict__ success,
                               const int32_t *__restrict__ iters, unsigned long long *counters) {
    const int f = blockIdx.x * blockDim.x + threadIdx.x;
    unsigned long long be = 0, fe = 0, su = 0, it = 0, fr = 0;
    if (f < B) {
        be = (unsigned long long)ferr[f];
        fe = ferr[f] ? 1 : 0;
        su = success[f] ? 1 : 0;
        it = success[f] ? (unsigned long long)iters[f] : 0;
        fr = 1;
    }
    // wave-level sums, then one atomic per wave per counter
    for (int off = 32; off > 0; off >>= 1) {
        be += __shfl_down(be, off);
        fe += __shfl_down(fe, off);
        su += __shfl_down(su, off);
        it += __shfl_down(it, off);
        fr += __shfl_down(fr, off);
    }
    if ((threadIdx.x & 63) == 0) {
        atomicAdd(&counters[0], be);
        atomicAdd(&counters[1], fe);
        atomicAdd(&counters[2], su);
        atomicAdd(&counters[3], it);
        atomicAdd(&counters[4], fr);
    }
}

static int check_shape(int B, int ld, int64_t S) {
    if (B <= 0 || ld < B || ld % kWave) return set_error(QR_EVALUE, "need 0 < B <= ld, ld %% 64 == 0 (B=%d ld=%d)", B, ld);
    if (S <= 0) return set_error(QR_EVALUE, "S must be positive");
    return QR_OK;
}

int demap_batch_device(const qr_demap *dm, int B, int ld, int64_t S, const double *n, const int64_t *j, double alpha,
                       double *lappr, hipStream_t s) {
    int rc = check_shape(B, ld, S);
    if (rc) return rc;
    DeviceGuard g(dm->device);
    ProfScope ps("demap", s);
    const bool fast = g_demap_fast.load() != 0;
    const int hyp = g_demap_hyp.load();
    if (fast && hyp >= 1 && ld % kWave == 0 &&
        dm->h.bps <= kDemapWaveMaxBps) {
        const int64_t items = S * (ld / kWave);
        launch_demap_wave(dm->h.bps, demap_wave_grid(dm->device, (items + 3) / 4), s, dm, B, ld, S, n, j, alpha, lappr);
    } else {
        const int64_t items = S * ld;
        launch_demap_bps(dm->h.bps, fast, (unsigned)((items + 255) / 256), s, dm, B, ld, S, n, j, alpha, lappr);
    }
    QR_LAUNCH_CHECK();
    return QR_OK;
}

}  // namespace qr

// ===================================================================== C-ABI
using namespace qr;

extern "C" {

#if QR_EXPERIMENT_CLOCK
// Diagnostic builds only (not in include/qamr.h): out = {sum cycles, sum ticks, workgroups} of the
// wave-private demapper's stamped launches since the last call.
QR_API int qr_debug_clock_demap(int64_t *out) {
    unsigned long long h[3] = {0, 0, 0};
    if (hipMemcpyFromSymbol(h, HIP_SYMBOL(qr::g_clk_demap), sizeof(h)) != hipSuccess) return QR_EDEVICE;
    const unsigned long long z[3] = {0, 0, 0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(qr::g_clk_demap), z, sizeof(z)) != hipSuccess) return QR_EDEVICE;
    for (int i = 0; i < 3; ++i) out[i] = (int64_t)h[i];
    return QR_OK;
}
#endif

int qr_demap_create(int32_t bps, const double *constellation, const double *probabilities, const double *thresholds,
                    double noise_var, const uint8_t *sign_config, int32_t device, qr_demap **out) {
    if (!out) return set_error(QR_EVALUE, "null output handle");
    *out = nullptr;
    DemapTables t;  // host_build.hpp (noisemapper.pyx:103-236 + the fast search's tables)
    std::vector<double2> quant;
    std::vector<double> ftab;
    std::string err;
    if (int rc = build_demap_host(bps, constellation, probabilities, thresholds, noise_var, sign_config, t, quant, ftab,
                                  err))
        return set_error(rc, "%s", err.c_str());
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0)
        return set_error(QR_EDEVICE, "no HIP device available (libqamr has no CPU fallback)");
    if (device < 0 || device >= ndev) return set_error(QR_EVALUE, "device %d out of range", device);
    qr_demap *dm = new qr_demap();
    dm->h = t;
    std::vector<MathTables> mt(1);
    build_math_tables(&mt[0]);
    dm->device = device;
    dm->scratch.device = device;
    DeviceGuard g(device);
    hipError_t e = hipSuccess;
    if (!quant.empty()) {
        e = hipMalloc((void **)&dm->d_quant, quant.size() * sizeof(double2));
        if (e == hipSuccess)
            e = hipMemcpy(dm->d_quant, quant.data(), quant.size() * sizeof(double2), hipMemcpyHostToDevice);
    }
    if (e == hipSuccess && !ftab.empty()) {
        e = hipMalloc((void **)&dm->d_ftab, ftab.size() * sizeof(double));
        if (e == hipSuccess)
            e = hipMemcpy(dm->d_ftab, ftab.data(), ftab.size() * sizeof(double), hipMemcpyHostToDevice);
    }
    t.quant = dm->d_quant;  // device pointers in the device copy
    t.ftab = dm->d_ftab;
    if (e == hipSuccess) e = hipMalloc((void **)&dm->d_mtab, sizeof(MathTables));
    if (e == hipSuccess) e = hipMemcpy(dm->d_mtab, mt.data(), sizeof(MathTables), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMalloc((void **)&dm->d_tables, sizeof(DemapTables));
    if (e == hipSuccess) e = hipMemcpy(dm->d_tables, &t, sizeof(DemapTables), hipMemcpyHostToDevice);
    t.quant = nullptr;      // the host copy never dereferences them
    t.ftab = nullptr;
    if (e != hipSuccess) {
        (void)hipFree(dm->d_tables);
        (void)hipFree(dm->d_mtab);
        (void)hipFree(dm->d_quant);
        (void)hipFree(dm->d_ftab);
        delete dm;
        return hip_fail(e, "qr_demap_create upload", __FILE__, __LINE__);
    }
    *out = dm;
    return QR_OK;
}

int qr_demap_destroy(qr_demap *dm) {
    if (!dm) return QR_OK;
    {
        DeviceGuard g(dm->device);
        (void)hipFree(dm->d_tables);
        (void)hipFree(dm->d_mtab);
        (void)hipFree(dm->d_quant);
        (void)hipFree(dm->d_ftab);
    }
    delete dm;
    return QR_OK;
}

int qr_demap_tables(const qr_demap *dm, double *Fthr, double *dF) {
    if (!dm) return set_error(QR_EVALUE, "null demapper");
    for (int i = 0; i <= dm->h.M; ++i)
        if (Fthr) Fthr[i] = dm->h.Fthr[i];
    for (int i = 0; i < dm->h.M; ++i)
        if (dF) dF[i] = dm->h.dF[i];
    return QR_OK;
}

int qr_demap_batch_device(const qr_demap *dm, int32_t B, int32_t ld, int64_t S, const double *d_n,
                          const int64_t *d_j, double alpha, double *d_lappr, void *stream) {
    if (!dm) return set_error(QR_EVALUE, "null demapper");
    return demap_batch_device(dm, B, ld, S, d_n, d_j, alpha, d_lappr, (hipStream_t)stream);
}

// One array from host memory: the same kernel with B = ld = 1, i.e. one lane
// per symbol and the interleaved out[s*bps + k] layout of noisemapper.pyx:556.
int qr_demap_host(const qr_demap *dm, int64_t S, const double *n, const int64_t *j, double *lappr) {
    if (!dm) return set_error(QR_EVALUE, "null demapper");
    if (S <= 0) return QR_OK;
    DeviceGuard g(dm->device);
    std::lock_guard<std::mutex> lk(dm->scratch.mu);
    const int bps = dm->h.bps;
    const size_t a = align_up(S * 8, 256), b = align_up(S * 8, 256), c = align_up(S * bps * 8, 256);
    int rc = dm->scratch.reserve(a + b + c);
    if (rc) return rc;
    char *p = (char *)dm->scratch.ptr;
    double *d_n = (double *)p;
    int64_t *d_j = (int64_t *)(p + a);
    double *d_l = (double *)(p + a + b);
    QR_HIP(hipMemcpy(d_n, n, S * 8, hipMemcpyHostToDevice));
    QR_HIP(hipMemcpy(d_j, j, S * 8, hipMemcpyHostToDevice));
    // ld = 1, B = 1: item = s, f = 0; lappr index (s*bps + k) * 1 + 0 = interleaved output.
    {
        ProfScope ps("demap", nullptr);
        launch_demap_bps(dm->h.bps, g_demap_fast.load() != 0, (unsigned)((S + 255) / 256), nullptr, dm, 1, 1, S, d_n,
                         d_j, 1.0, d_l);
        QR_LAUNCH_CHECK();
    }
    QR_HIP(hipMemcpy(lappr, d_l, S * bps * 8, hipMemcpyDeviceToHost));
    return QR_OK;
}

int qr_g_inv_search_host(const qr_demap *dm, int64_t n, const double *n_hat, const int64_t *i, double y_accuracy,
                         double *y_hat) {
    if (!dm) return set_error(QR_EVALUE, "null demapper");
    if (n < 0) return set_error(QR_EVALUE, "negative size");
    if (n == 0) return QR_OK;
    if (!n_hat || !i || !y_hat) return set_error(QR_EVALUE, "null pointer argument");
    DeviceGuard g(dm->device);
    std::lock_guard<std::mutex> lk(dm->scratch.mu);
    const size_t a = align_up((size_t)n * 8, 256);
    int rc = dm->scratch.reserve(3 * a);
    if (rc) return rc;
    char *p = (char *)dm->scratch.ptr;
    double *d_n = (double *)p;
    int64_t *d_i = (int64_t *)(p + a);
    double *d_y = (double *)(p + 2 * a);
    QR_HIP(hipMemcpy(d_n, n_hat, (size_t)n * 8, hipMemcpyHostToDevice));
    QR_HIP(hipMemcpy(d_i, i, (size_t)n * 8, hipMemcpyHostToDevice));
    k_g_inv_search<<<(unsigned)((n + 255) / 256), 256>>>(dm->d_tables, dm->d_mtab, n, d_n, d_i, y_accuracy,
                                                         g_demap_fast.load() != 0, d_y);
    QR_LAUNCH_CHECK();
    QR_HIP(hipMemcpy(y_hat, d_y, (size_t)n * 8, hipMemcpyDeviceToHost));
    return QR_OK;
}

int qr_F_Y_host(const qr_demap *dm, int64_t n, const double *y, double *F) {
    if (!dm) return set_error(QR_EVALUE, "null demapper");
    if (n < 0) return set_error(QR_EVALUE, "negative size");
    if (n == 0) return QR_OK;
    if (!y || !F) return set_error(QR_EVALUE, "null pointer argument");
    DeviceGuard g(dm->device);
    std::lock_guard<std::mutex> lk(dm->scratch.mu);
    const size_t a = align_up((size_t)n * 8, 256);
    int rc = dm->scratch.reserve(2 * a);
    if (rc) return rc;
    char *p = (char *)dm->scratch.ptr;
    double *d_y = (double *)p;
    double *d_F = (double *)(p + a);
    QR_HIP(hipMemcpy(d_y, y, (size_t)n * 8, hipMemcpyHostToDevice));
    k_public_F_Y<<<(unsigned)((n + 255) / 256), 256>>>(dm->d_tables, n, d_y, d_F);
    QR_LAUNCH_CHECK();
    QR_HIP(hipMemcpy(F, d_F, (size_t)n * 8, hipMemcpyDeviceToHost));
    return QR_OK;
}

int qr_bob_map_device(const qr_demap *dm, int32_t B, int32_t ld, int64_t S, const double *d_y, int64_t *d_xhat,
                      double *d_nhat, uint8_t *d_word, void *stream) {
    if (!dm) return set_error(QR_EVALUE, "null demapper");
    int rc = check_shape(B, ld, S);
    if (rc) return rc;
    DeviceGuard g(dm->device);
    hipStream_t s = (hipStream_t)stream;
    ProfScope ps("bob", s);
    const int64_t items = S * ld;
    k_bob<<<(unsigned)((items + 255) / 256), 256, 0, s>>>(dm->d_tables, B, ld, S, d_y, d_xhat, d_nhat, d_word);
    QR_LAUNCH_CHECK();
    return QR_OK;
}

int qr_map_noise_device(const qr_demap *dm, int32_t B, int32_t ld, int64_t S, const double *d_y,
                        const int64_t *d_index, double *d_nhat, void *stream) {
    if (!dm) return set_error(QR_EVALUE, "null demapper");
    int rc = check_shape(B, ld, S);
    if (rc) return rc;
    DeviceGuard g(dm->device);
    hipStream_t s = (hipStream_t)stream;
    const int64_t items = S * ld;
    k_map_noise<<<(unsigned)((items + 255) / 256), 256, 0, s>>>(dm->d_tables, B, ld, S, d_y, d_index, d_nhat);
    QR_LAUNCH_CHECK();
    return QR_OK;
}

int qr_direct_lappr_device(const qr_demap *dm, double two_variance, int32_t B, int32_t ld, int64_t S,
                           const double *d_y, double *d_lappr, void *stream) {
    if (!dm) return set_error(QR_EVALUE, "null demapper");
    int rc = check_shape(B, ld, S);
    if (rc) return rc;
    DeviceGuard g(dm->device);
    hipStream_t s = (hipStream_t)stream;
    ProfScope ps("direct_lappr", s);
    const int64_t items = S * ld;
    k_direct_lappr<<<(unsigned)((items + 255) / 256), 256, 0, s>>>(dm->d_tables, two_variance, B, ld, S, d_y, d_lappr);
    QR_LAUNCH_CHECK();
    return QR_OK;
}

int qr_bare_llr_device(int32_t bps, const double *d_table, int32_t B, int32_t ld, int64_t S, const int64_t *d_x,
                       double *d_lappr, void *stream) {
    if (bps < 1 || bps > kMaxBps) return set_error(QR_EVALUE, "bit_per_symbol out of range");
    int rc = check_shape(B, ld, S);
    if (rc) return rc;
    hipStream_t s = (hipStream_t)stream;
    const int64_t items = S * ld;
    k_bare_llr<<<(unsigned)((items + 255) / 256), 256, 0, s>>>(d_table, 1 << bps, bps, B, ld, S, d_x, d_lappr);
    QR_LAUNCH_CHECK();
    return QR_OK;
}

int qr_symbols_to_bits_device(int32_t bps, int32_t B, int32_t ld, int64_t S, const int64_t *d_x, uint8_t *d_word,
                              void *stream) {
    if (bps < 1 || bps > kMaxBps) return set_error(QR_EVALUE, "bit_per_symbol out of range");
    int rc = check_shape(B, ld, S);
    if (rc) return rc;
    hipStream_t s = (hipStream_t)stream;
    const int64_t items = S * ld;
    k_symbols_to_bits<<<(unsigned)((items + 255) / 256), 256, 0, s>>>(bps, B, ld, S, d_x, d_word);
    QR_LAUNCH_CHECK();
    return QR_OK;
}

int qr_syndrome_device(const qr_code *code, int32_t B, int32_t ld, const uint8_t *d_word, uint8_t *d_synd,
                       void *stream) {
    if (!code) return set_error(QR_EVALUE, "null code");
    int rc = check_shape(B, ld, 1);
    if (rc) return rc;
    DeviceGuard g(code->device);
    hipStream_t s = (hipStream_t)stream;
    ProfScope ps("syndrome", s);
    const int ft = frame_tile(ld);
    dim3 grid((unsigned)code->C, (unsigned)(ld / ft));
    k_syndrome<<<grid, ft, 0, s>>>(code->C, ld, B, code->d_chk_ptr, code->d_chk_var, d_word, d_synd);
    QR_LAUNCH_CHECK();
    return QR_OK;
}

int qr_count_errors_device(int32_t B, int32_t ld, int64_t K, const double *d_final, const uint8_t *d_word,
                           const uint8_t *d_success, const int32_t *d_iters, int32_t *d_frame_errors,
                           int64_t *d_counters, void *stream) {
    int rc = check_shape(B, ld, 1);
    if (rc) return rc;
    if (K < 0) return set_error(QR_EVALUE, "K must be >= 0");
    hipStream_t s = (hipStream_t)stream;
    ProfScope ps("count", s);
    int32_t *ferr = d_frame_errors;
    QR_HIP(hipMemsetAsync(ferr, 0, (size_t)B * 4, s));
    if (K > 0) {
        const int ft = frame_tile(ld);
        const int64_t kpb = 64;
        dim3 grid((unsigned)((K + kpb - 1) / kpb), (unsigned)(ld / ft));
        k_count_errors<<<grid, ft, 0, s>>>(B, ld, K, kpb, d_final, d_word, ferr);
        QR_LAUNCH_CHECK();
    }
    k_count_finish<<<(B + 255) / 256, 256, 0, s>>>(B, ferr, d_success, d_iters, (unsigned long long *)d_counters);
    QR_LAUNCH_CHECK();
    return QR_OK;
}

}  // extern "C"
