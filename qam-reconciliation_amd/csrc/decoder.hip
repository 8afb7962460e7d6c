// decoder.hip -- batched flooding sum-product LDPC syndrome decoder for gfx950.
//
// Reference: qamreconciliation/decoder.pyx (Decoder, _decode :391-436).
//
// Layout (HBM, frame-innermost): every per-edge / per-node quantity of frame f
// lives at row[node] * ld + f.  A wavefront = 64 consecutive frames of ONE
// check (or variable), so every message access is a contiguous 512-B run no
// matter how irregular the Tanner graph is; the graph itself (CSR) is
// wave-uniform and travels through the scalar cache.
//
// Only c2v[E][ld] and post[V][ld] are stored: the reference's v2c is
// post - c2v (decoder.pyx:295-297) and is recomputed in the check kernel,
// bit-identically.  All per-node arithmetic stays sequential in one lane in
// the reference's order (the F/B box-plus recursion is not associative).
//
// Schedule per iteration t (decoder.pyx:424-433):
//   k_check<t==1 ? First : Normal>   c2v(t) from post(t-1); also the parity of
//                                    post(t-1) (the check at the end of
//                                    iteration t-1, fused: it reads post anyway)
//   k_status(t-1)                    frames whose post(t-1) satisfies the
//                                    syndrome stop with (1, t-1)
//   k_var                            post(t) = lappr + sum c2v (ascending edge)
// plus an initial parity check of the input (decoder.pyx:400-405) and a final
// parity check after the last sweep.
#include <atomic>

#include "fastmath.hpp"
#include "qamr_internal.hpp"

namespace qr {

enum CheckMode { kFirst = 0, kNormal = 1, kParityOnly = 2 };

// Edge-message access: NT = non-temporal (streamed once per sweep; keeps the
// re-read posteriors resident in L2/MALL instead of the message stream).
template <bool NT>
__device__ __forceinline__ double ld_msg(const double *p) {
    if constexpr (NT) return __builtin_nontemporal_load(p);
    else return *p;
}
template <bool NT>
__device__ __forceinline__ void st_msg(double *p, double v) {
    if constexpr (NT) __builtin_nontemporal_store(v, p);
    else *p = v;
}

// Block geometry shared by the check and variable sweeps: 256 threads = `ft`
// consecutive frames (ft = 64 << lft, a multiple of the wavefront) x (256/ft)
// node lanes; every wave therefore covers 64 frames of ONE node, which makes
// the node index wave-uniform (readfirstlane -> scalar loads of the CSR).
struct Geom {
    int lft;  // log2(ft)
    int per;  // nodes per thread
};

// One lane = one (check, frame); each thread walks `per` checks of one degree class.
template <int D, int MODE, bool NT>
__global__ void __launch_bounds__(256) k_check(const int32_t *__restrict__ checks, int64_t n_checks, Geom g,
                                               const int32_t *__restrict__ chk_ptr,
                                               const int32_t *__restrict__ chk_edge,
                                               const int32_t *__restrict__ chk_var, const double *__restrict__ post,
                                               double *__restrict__ c2v, const uint8_t *__restrict__ synd,
                                               const uint8_t *__restrict__ active, uint8_t *__restrict__ unsat,
                                               int ld, const MathTables *__restrict__ gtab) {
    __shared__ MathTables tab;
    if (MODE != kParityOnly) stage_math_tables(&tab, gtab);
    const int ft = 1 << g.lft;
    const int nsub = 256 >> g.lft;
    const int f = (blockIdx.y << g.lft) + (threadIdx.x & (ft - 1));
    const int sub = __builtin_amdgcn_readfirstlane(threadIdx.x >> g.lft);
    if (!active[f]) return;
    const int64_t c0 = (int64_t)blockIdx.x * g.per * nsub + sub;
    uint32_t bad = 0;
    for (int j = 0; j < g.per; ++j) {
        const int64_t ci = c0 + (int64_t)j * nsub;
        if (ci >= n_checks) break;
        const int c = checks[ci];
        const int base = chk_ptr[c];
        const uint8_t sb = synd[(size_t)c * ld + f];
        uint32_t par = sb;
        double m[D];
#pragma unroll
        for (int i = 0; i < D; ++i) {
            const double p = post[(size_t)chk_var[base + i] * ld + f];
            if (MODE != kFirst) par ^= (p < 0.0) ? 1u : 0u;   // decoder.pyx:243-246
            if (MODE == kNormal) m[i] = p - ld_msg<NT>(&c2v[(size_t)chk_edge[base + i] * ld + f]);  // :296-297
            else m[i] = p;  // first sweep: c2v == 0 and p - 0.0 == p
        }
        if (MODE != kFirst) bad |= (par == 1u) ? 1u : 0u;  // satisfied iff (parity ^ 1) != 0
        if (MODE == kParityOnly) continue;
        // decoder.pyx:341-367
        double F[D], Bk[D];
        F[0] = m[0];
#pragma unroll
        for (int i = 1; i < D - 1; ++i) F[i] = box_plus_fast(F[i - 1], m[i], tab);
        Bk[D - 1] = m[D - 1];
#pragma unroll
        for (int i = D - 2; i > 0; --i) Bk[i] = box_plus_fast(Bk[i + 1], m[i], tab);
        const double s = sb ? -1.0 : 1.0;
        st_msg<NT>(&c2v[(size_t)chk_edge[base] * ld + f], s * Bk[1]);
#pragma unroll
        for (int i = 1; i < D - 1; ++i)
            st_msg<NT>(&c2v[(size_t)chk_edge[base + i] * ld + f], s * box_plus_fast(F[i - 1], Bk[i + 1], tab));
        st_msg<NT>(&c2v[(size_t)chk_edge[base + D - 1] * ld + f], s * F[D - 2]);
    }
    if (MODE != kFirst && bad) unsat[f] = 1;  // benign race: every writer stores 1
}

// Runtime-degree fallback for check degrees above the templated range (2..16).
constexpr int kMaxGenericDeg = 64;

__device__ __forceinline__ void check_update_generic(int d, const double *m, double *out, double s,
                                                     const MathTables &tab) {
    double F[kMaxGenericDeg], Bk[kMaxGenericDeg];
    F[0] = m[0];
    for (int i = 1; i < d - 1; ++i) F[i] = box_plus_fast(F[i - 1], m[i], tab);
    Bk[d - 1] = m[d - 1];
    for (int i = d - 2; i > 0; --i) Bk[i] = box_plus_fast(Bk[i + 1], m[i], tab);
    out[0] = s * Bk[1];
    for (int i = 1; i < d - 1; ++i) out[i] = s * box_plus_fast(F[i - 1], Bk[i + 1], tab);
    out[d - 1] = s * F[d - 2];
}

template <int MODE>
__global__ void __launch_bounds__(256) k_check_generic(const int32_t *__restrict__ checks, int64_t n_checks, Geom g,
                                                       const int32_t *__restrict__ chk_ptr,
                                                       const int32_t *__restrict__ chk_edge,
                                                       const int32_t *__restrict__ chk_var,
                                                       const double *__restrict__ post, double *__restrict__ c2v,
                                                       const uint8_t *__restrict__ synd,
                                                       const uint8_t *__restrict__ active,
                                                       uint8_t *__restrict__ unsat, int ld,
                                                       const MathTables *__restrict__ gtab) {
    __shared__ MathTables tab;
    if (MODE != kParityOnly) stage_math_tables(&tab, gtab);
    const int ft = 1 << g.lft;
    const int nsub = 256 >> g.lft;
    const int f = (blockIdx.y << g.lft) + (threadIdx.x & (ft - 1));
    const int sub = __builtin_amdgcn_readfirstlane(threadIdx.x >> g.lft);
    if (!active[f]) return;
    const int64_t c0 = (int64_t)blockIdx.x * g.per * nsub + sub;
    uint32_t bad = 0;
    double m[kMaxGenericDeg], out[kMaxGenericDeg];
    for (int j = 0; j < g.per; ++j) {
        const int64_t ci = c0 + (int64_t)j * nsub;
        if (ci >= n_checks) break;
        const int c = checks[ci];
        const int base = chk_ptr[c];
        const int d = chk_ptr[c + 1] - base;
        const uint8_t sb = synd[(size_t)c * ld + f];
        uint32_t par = sb;
        for (int i = 0; i < d; ++i) {
            const double p = post[(size_t)chk_var[base + i] * ld + f];
            if (MODE != kFirst) par ^= (p < 0.0) ? 1u : 0u;
            m[i] = (MODE == kNormal) ? p - c2v[(size_t)chk_edge[base + i] * ld + f] : p;
        }
        if (MODE != kFirst) bad |= (par == 1u) ? 1u : 0u;
        if (MODE == kParityOnly) continue;
        check_update_generic(d, m, out, sb ? -1.0 : 1.0, tab);
        for (int i = 0; i < d; ++i) c2v[(size_t)chk_edge[base + i] * ld + f] = out[i];
    }
    if (MODE != kFirst && bad) unsat[f] = 1;
}

// decoder.pyx:285-298: post[v] = lappr[v] + c2v[e_0] + c2v[e_1] + ... (ascending e).
// INIT: the first sweep with c2v == 0 (decoder.pyx:408,420-421): lappr + 0.0 for
// frames still decoding; frames already successful at iteration 0 get a plain
// copy of their input (decoder.pyx:404).
template <bool INIT, bool NT>
__global__ void __launch_bounds__(256) k_var(int64_t V, Geom g, const int32_t *__restrict__ var_ptr,
                                             const int32_t *__restrict__ var_edge, const double *__restrict__ lappr,
                                             const double *__restrict__ c2v, double *__restrict__ post,
                                             const uint8_t *__restrict__ active, int ld) {
    const int ft = 1 << g.lft;
    const int nsub = 256 >> g.lft;
    const int f = (blockIdx.y << g.lft) + (threadIdx.x & (ft - 1));
    const int sub = __builtin_amdgcn_readfirstlane(threadIdx.x >> g.lft);
    const bool act = active[f] != 0;
    if (!INIT && !act) return;
    const int64_t v0 = (int64_t)blockIdx.x * g.per * nsub + sub;
    for (int j = 0; j < g.per; ++j) {
        const int64_t v = v0 + (int64_t)j * nsub;
        if (v >= V) break;
        const int b = var_ptr[v], e = var_ptr[v + 1];
        double p = ld_msg<NT>(&lappr[(size_t)v * ld + f]);
        if (INIT) {
            if (act && e > b) p = p + 0.0;
        } else {
            for (int k = b; k < e; ++k) p += ld_msg<NT>(&c2v[(size_t)var_edge[k] * ld + f]);
        }
        post[(size_t)v * ld + f] = p;
    }
}

__global__ void k_init_status(int B, int ld, uint8_t *active, uint8_t *success, int32_t *iters) {
    const int f = blockIdx.x * blockDim.x + threadIdx.x;
    if (f >= ld) return;
    active[f] = (f < B) ? 1 : 0;
    if (f < B) {
        success[f] = 0;
        iters[f] = 0;
    }
}

// Frames whose posterior after sweep t satisfies the syndrome stop with
// (success=1, iterations=t) (decoder.pyx:431-433, :402-405 for t = 0).  On the
// final call every still-active frame stops with (0, max_iterations) (:435-436).
__global__ void k_status(int B, int t, int final_call, int32_t final_iters, const uint8_t *__restrict__ unsat_t,
                         uint8_t *active, uint8_t *success, int32_t *iters) {
    const int f = blockIdx.x * blockDim.x + threadIdx.x;
    if (f >= B || !active[f]) return;
    if (!unsat_t[f]) {
        success[f] = 1;
        iters[f] = t;
        active[f] = 0;
    } else if (final_call) {
        success[f] = 0;
        iters[f] = final_iters;
        active[f] = 0;
    }
}

// ------------------------------------------------------------------ launch
struct DecodeWs {
    double *c2v;
    uint8_t *active;
    uint8_t *unsat;  // (max_it + 2) rows of ld flags
};

static size_t ws_bytes(const qr_code *code, int ld, int max_it) {
    const int rows = (max_it > 0 ? max_it : 0) + 2;
    return align_up((size_t)code->E * ld * sizeof(double), 256) + align_up((size_t)ld, 256) +
           align_up((size_t)rows * ld, 256);
}

static DecodeWs carve(const qr_code *code, int ld, void *base) {
    DecodeWs w;
    char *p = (char *)base;
    w.c2v = (double *)p;
    p += align_up((size_t)code->E * ld * sizeof(double), 256);
    w.active = (uint8_t *)p;
    p += align_up((size_t)ld, 256);
    w.unsat = (uint8_t *)p;
    return w;
}

// Runtime tuning knobs (qr_tune_set); defaults picked by scripts/tune.py on MI355X.
struct Tuning {
    std::atomic<int> check_ft{256}, check_per{4}, var_ft{256}, var_per{4}, nt{1};
};
static Tuning g_tune;

static Geom make_geom(int ld, int ft_req, int per) {
    int ft = 256;
    while (ft > 64 && (ft > ft_req || ld % ft)) ft >>= 1;
    int lft = 6;
    while ((1 << lft) < ft) ++lft;
    return Geom{lft, per < 1 ? 1 : per};
}

template <int MODE, bool NT>
static int launch_check_class(const qr_code *code, const DegreeClass &cls, int ld, const double *post, double *c2v,
                              const uint8_t *synd, const uint8_t *active, uint8_t *unsat, hipStream_t s) {
    const Geom g = make_geom(ld, g_tune.check_ft.load(), g_tune.check_per.load());
    const int64_t per_block = (int64_t)g.per * (256 >> g.lft);
    dim3 grid((unsigned)((cls.n + per_block - 1) / per_block), (unsigned)(ld >> g.lft));
    ProfScope ps(profiling_on() ? std::string(MODE == kParityOnly ? "parity_d" : MODE == kFirst ? "check1_d" : "check_d") +
                                      std::to_string(cls.degree)
                                : std::string(),
                 s);
#define QR_CASE(DD)                                                                                          \
    case DD:                                                                                                 \
        k_check<DD, MODE, NT><<<grid, 256, 0, s>>>(cls.d_checks, cls.n, g, code->d_chk_ptr, code->d_chk_edge, \
                                                   code->d_chk_var, post, c2v, synd, active, unsat, ld,        \
                                                   code->d_mtab);                                             \
        break;
    switch (cls.degree) {
        QR_CASE(2) QR_CASE(3) QR_CASE(4) QR_CASE(5) QR_CASE(6) QR_CASE(7) QR_CASE(8) QR_CASE(9) QR_CASE(10)
        QR_CASE(11) QR_CASE(12) QR_CASE(13) QR_CASE(14) QR_CASE(15) QR_CASE(16)
        default:
            k_check_generic<MODE><<<grid, 256, 0, s>>>(cls.d_checks, cls.n, g, code->d_chk_ptr, code->d_chk_edge,
                                                       code->d_chk_var, post, c2v, synd, active, unsat, ld,
                                                       code->d_mtab);
    }
#undef QR_CASE
    QR_LAUNCH_CHECK();
    return QR_OK;
}

template <int MODE>
static int launch_check_all(const qr_code *code, int ld, const double *post, double *c2v, const uint8_t *synd,
                            const uint8_t *active, uint8_t *unsat, hipStream_t s) {
    ProfScope ps(MODE == kParityOnly ? "parity" : MODE == kFirst ? "check1" : "check", s);
    const bool nt = g_tune.nt.load() != 0;
    for (const auto &cls : code->classes) {
        int rc = nt ? launch_check_class<MODE, true>(code, cls, ld, post, c2v, synd, active, unsat, s)
                    : launch_check_class<MODE, false>(code, cls, ld, post, c2v, synd, active, unsat, s);
        if (rc) return rc;
    }
    return QR_OK;
}

template <bool INIT>
static int launch_var(const qr_code *code, int ld, const double *lappr, const double *c2v, double *post,
                      const uint8_t *active, hipStream_t s) {
    ProfScope ps(INIT ? "var_init" : "var", s);
    const Geom g = make_geom(ld, g_tune.var_ft.load(), g_tune.var_per.load());
    const int64_t per_block = (int64_t)g.per * (256 >> g.lft);
    dim3 grid((unsigned)((code->V + per_block - 1) / per_block), (unsigned)(ld >> g.lft));
    if (g_tune.nt.load())
        k_var<INIT, true><<<grid, 256, 0, s>>>(code->V, g, code->d_var_ptr, code->d_var_edge, lappr, c2v, post,
                                               active, ld);
    else
        k_var<INIT, false><<<grid, 256, 0, s>>>(code->V, g, code->d_var_ptr, code->d_var_edge, lappr, c2v, post,
                                                active, ld);
    QR_LAUNCH_CHECK();
    return QR_OK;
}

static int launch_status(int B, int ld, int t, int final_call, int32_t final_iters, const uint8_t *unsat_t,
                         uint8_t *active, uint8_t *success, int32_t *iters, hipStream_t s) {
    ProfScope ps("status", s);
    k_status<<<(B + 255) / 256, 256, 0, s>>>(B, t, final_call, final_iters, unsat_t, active, success, iters);
    QR_LAUNCH_CHECK();
    return QR_OK;
}

int decode_batch_device(const qr_code *code, int B, int ld, const double *lappr, const uint8_t *synd, int max_it,
                        double *final_post, uint8_t *success, int32_t *iters, void *ws_ptr, size_t ws_size,
                        hipStream_t s) {
    if (B <= 0 || ld < B || ld % kWave)
        return set_error(QR_EVALUE, "decode: need 0 < B <= ld and ld %% 64 == 0 (B=%d, ld=%d)", B, ld);
    if (!lappr || !synd || !final_post || !success || !iters || !ws_ptr)
        return set_error(QR_EVALUE, "decode: null pointer argument");
    if (ws_size < ws_bytes(code, ld, max_it))
        return set_error(QR_EVALUE, "decode: workspace too small (%zu < %zu)", ws_size, ws_bytes(code, ld, max_it));
    DeviceGuard dg(code->device);
    DecodeWs w = carve(code, ld, ws_ptr);
    const int rows = (max_it > 0 ? max_it : 0) + 2;
    int rc;
    QR_HIP(hipMemsetAsync(w.unsat, 0, (size_t)rows * ld, s));
    k_init_status<<<(ld + 255) / 256, 256, 0, s>>>(B, ld, w.active, success, iters);
    QR_LAUNCH_CHECK();
    // decoder.pyx:400-405: the input itself may already satisfy the syndrome.
    if ((rc = launch_check_all<kParityOnly>(code, ld, lappr, nullptr, synd, w.active, w.unsat, s))) return rc;
    if ((rc = launch_status(B, ld, 0, 0, 0, w.unsat, w.active, success, iters, s))) return rc;
    // decoder.pyx:408-421: c2v = 0, first variable sweep.
    if ((rc = launch_var<true>(code, ld, lappr, nullptr, final_post, w.active, s))) return rc;
    for (int t = 1; t <= max_it; ++t) {
        uint8_t *unsat_prev = w.unsat + (size_t)(t - 1) * ld;
        if (t == 1) {
            if ((rc = launch_check_all<kFirst>(code, ld, final_post, w.c2v, synd, w.active, unsat_prev, s))) return rc;
        } else {
            if ((rc = launch_check_all<kNormal>(code, ld, final_post, w.c2v, synd, w.active, unsat_prev, s))) return rc;
            if ((rc = launch_status(B, ld, t - 1, 0, 0, unsat_prev, w.active, success, iters, s))) return rc;
        }
        if ((rc = launch_var<false>(code, ld, lappr, w.c2v, final_post, w.active, s))) return rc;
    }
    // Check after the last sweep; then every frame still running stops with (0, max).
    const int tf = max_it > 0 ? max_it : 0;
    uint8_t *unsat_last = w.unsat + (size_t)tf * ld;
    if (max_it > 0) {
        if ((rc = launch_check_all<kParityOnly>(code, ld, final_post, nullptr, synd, w.active, unsat_last, s)))
            return rc;
    } else {
        // decoder.pyx:424 with max_iterations <= 0: no sweep, no check -> (0, max_iterations)
        QR_HIP(hipMemsetAsync(unsat_last, 1, (size_t)ld, s));
    }
    if ((rc = launch_status(B, ld, tf, 1, max_it, unsat_last, w.active, success, iters, s))) return rc;
    return QR_OK;
}

// ------------------------------------------------- unit-test surface kernels
// One frame, frame-major arrays (ld == 1 layout), lane = node.
__global__ void k_check_lappr_nodes(int64_t C, const int32_t *chk_ptr, const int32_t *chk_var, const double *lappr,
                                    const uint8_t *synd, uint8_t *out) {
    const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= C) return;
    uint8_t parity = synd[c];
    for (int k = chk_ptr[c]; k < chk_ptr[c + 1]; ++k)
        if (lappr[chk_var[k]] < 0) parity ^= 1;  // decoder.pyx:241-248
    out[c] = parity ^ 1;
}

__global__ void k_check_word_nodes(int64_t C, const int32_t *chk_ptr, const int32_t *chk_var, const uint8_t *word,
                                   const uint8_t *synd, uint8_t *out) {
    const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= C) return;
    uint8_t parity = synd[c];
    for (int k = chk_ptr[c]; k < chk_ptr[c + 1]; ++k) parity ^= word[chk_var[k]];  // decoder.pyx:182-187
    out[c] = parity ^ 1;
}

__global__ void k_var_nodes(const int64_t *nodes, int64_t n, const int32_t *var_ptr, const int32_t *var_edge,
                            const double *lappr, const double *c2v, double *v2c, double *updated) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int64_t v = nodes[i];
    double p = lappr[v];
    for (int k = var_ptr[v]; k < var_ptr[v + 1]; ++k) p += c2v[var_edge[k]];
    updated[v] = p;
    for (int k = var_ptr[v]; k < var_ptr[v + 1]; ++k) v2c[var_edge[k]] = p - c2v[var_edge[k]];
}

__global__ void k_check_nodes(const int64_t *nodes, int64_t n, const int32_t *chk_ptr, const int32_t *chk_edge,
                              const uint8_t *synd, double *c2v, const double *v2c, const MathTables *gtab) {
    __shared__ MathTables tab;
    stage_math_tables(&tab, gtab);
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int64_t c = nodes[i];
    const int base = chk_ptr[c], d = chk_ptr[c + 1] - base;
    double m[kMaxGenericDeg], out[kMaxGenericDeg];
    for (int k = 0; k < d; ++k) m[k] = v2c[chk_edge[base + k]];
    check_update_generic(d, m, out, synd[c] ? -1.0 : 1.0, tab);
    for (int k = 0; k < d; ++k) c2v[chk_edge[base + k]] = out[k];
}

}  // namespace qr

// ===================================================================== C-ABI
using namespace qr;

static int free_code(qr_code *c) {
    if (!c) return QR_OK;
    DeviceGuard g(c->device);
    for (auto &cls : c->classes) (void)hipFree(cls.d_checks);
    (void)hipFree(c->d_chk_ptr);
    (void)hipFree(c->d_chk_edge);
    (void)hipFree(c->d_chk_var);
    (void)hipFree(c->d_var_ptr);
    (void)hipFree(c->d_var_edge);
    (void)hipFree(c->d_mtab);
    delete c;
    return QR_OK;
}

template <typename T>
static int upload(T **dst, const std::vector<T> &src) {
    QR_HIP(hipMalloc((void **)dst, std::max<size_t>(1, src.size()) * sizeof(T)));
    if (!src.empty()) QR_HIP(hipMemcpy(*dst, src.data(), src.size() * sizeof(T), hipMemcpyHostToDevice));
    return QR_OK;
}

extern "C" {

int qr_code_create(const int64_t *e_to_v, const int64_t *e_to_c, int64_t nv, int64_t nc, int32_t device,
                   qr_code **out) {
    if (!out) return set_error(QR_EVALUE, "null output handle");
    *out = nullptr;
    if (nv != nc) return set_error(QR_EVALUE, "Sizes don't match");  // decoder.pyx:96-97
    const int64_t E = nv;
    if (E <= 0) return set_error(QR_EVALUE, "empty edge list");
    if (E >= (int64_t)1 << 31) return set_error(QR_EUNSUPPORTED, "more than 2^31-1 edges");
    int64_t V = 0, C = 0;
    for (int64_t e = 0; e < E; ++e) {
        if (e_to_v[e] < 0 || e_to_c[e] < 0) return set_error(QR_EVALUE, "negative node id at edge %lld", (long long)e);
        V = std::max(V, e_to_v[e] + 1);
        C = std::max(C, e_to_c[e] + 1);
    }
    if (V >= (int64_t)1 << 31 || C >= (int64_t)1 << 31) return set_error(QR_EUNSUPPORTED, "node ids exceed int32");
    // Stable counting sort by node id == the ascending scan of __build_table (decoder.pyx:69-87).
    std::vector<int32_t> chk_ptr(C + 1, 0), var_ptr(V + 1, 0), chk_edge(E), chk_var(E), var_edge(E);
    for (int64_t e = 0; e < E; ++e) {
        chk_ptr[e_to_c[e] + 1]++;
        var_ptr[e_to_v[e] + 1]++;
    }
    for (int64_t i = 0; i < C; ++i) chk_ptr[i + 1] += chk_ptr[i];
    for (int64_t i = 0; i < V; ++i) var_ptr[i + 1] += var_ptr[i];
    {
        std::vector<int32_t> fc(chk_ptr.begin(), chk_ptr.end() - 1), fv(var_ptr.begin(), var_ptr.end() - 1);
        for (int64_t e = 0; e < E; ++e) {
            const int32_t kc = fc[e_to_c[e]]++;
            chk_edge[kc] = (int32_t)e;
            chk_var[kc] = (int32_t)e_to_v[e];  // c_to_v (decoder.pyx:128-129)
            var_edge[fv[e_to_v[e]]++] = (int32_t)e;
        }
    }
    int32_t max_dc = 0, max_dv = 0;
    std::vector<std::vector<int32_t>> by_deg;
    for (int64_t c = 0; c < C; ++c) {
        const int32_t d = chk_ptr[c + 1] - chk_ptr[c];
        if (d < 2)
            return set_error(QR_EVALUE,
                             "check node %lld has degree %d; degree < 2 is undefined behaviour in the reference "
                             "(decoder.pyx:135-141) and is rejected",
                             (long long)c, d);
        if (d > kMaxGenericDeg)
            return set_error(QR_EUNSUPPORTED, "check degree %d exceeds the supported maximum %d", d, kMaxGenericDeg);
        max_dc = std::max(max_dc, d);
        if ((int)by_deg.size() <= d) by_deg.resize(d + 1);
        by_deg[d].push_back((int32_t)c);
    }
    for (int64_t v = 0; v < V; ++v) max_dv = std::max(max_dv, var_ptr[v + 1] - var_ptr[v]);

    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0)
        return set_error(QR_EDEVICE, "no HIP device available (libqamr has no CPU fallback)");
    if (device < 0 || device >= ndev) return set_error(QR_EVALUE, "device %d out of range (%d devices)", device, ndev);
    DeviceGuard g(device);
    qr_code *code = new qr_code();
    code->E = E;
    code->V = V;
    code->C = C;
    code->max_dc = max_dc;
    code->max_dv = max_dv;
    code->device = device;
    code->scratch.device = device;
    int rc = QR_OK;
    if ((rc = upload(&code->d_chk_ptr, chk_ptr)) || (rc = upload(&code->d_chk_edge, chk_edge)) ||
        (rc = upload(&code->d_chk_var, chk_var)) || (rc = upload(&code->d_var_ptr, var_ptr)) ||
        (rc = upload(&code->d_var_edge, var_edge))) {
        free_code(code);
        return rc;
    }
    {
        std::vector<MathTables> mt(1);
        build_math_tables(&mt[0]);
        if ((rc = upload(&code->d_mtab, mt))) {
            free_code(code);
            return rc;
        }
    }
    for (int d = 0; d < (int)by_deg.size(); ++d) {
        if (by_deg[d].empty()) continue;
        DegreeClass cls{d, (int64_t)by_deg[d].size(), nullptr};
        if ((rc = upload(&cls.d_checks, by_deg[d]))) {
            free_code(code);
            return rc;
        }
        code->classes.push_back(cls);
    }
    *out = code;
    return QR_OK;
}

int qr_code_destroy(qr_code *code) { return free_code(code); }

int qr_tune_set(const char *name, int64_t value) {
    const std::string n = name ? name : "";
    std::atomic<int> *k = n == "check_ft" ? &g_tune.check_ft : n == "check_per" ? &g_tune.check_per
                        : n == "var_ft"   ? &g_tune.var_ft   : n == "var_per"   ? &g_tune.var_per
                        : n == "nt"       ? &g_tune.nt       : nullptr;
    if (!k) return set_error(QR_EVALUE, "unknown tuning knob '%s'", n.c_str());
    if (value < 0 || value > 4096) return set_error(QR_EVALUE, "tuning value out of range");
    k->store((int)value);
    return QR_OK;
}

int qr_tune_get(const char *name, int64_t *value) {
    const std::string n = name ? name : "";
    const std::atomic<int> *k = n == "check_ft" ? &g_tune.check_ft : n == "check_per" ? &g_tune.check_per
                              : n == "var_ft"   ? &g_tune.var_ft   : n == "var_per"   ? &g_tune.var_per
                              : n == "nt"       ? &g_tune.nt       : nullptr;
    if (!k || !value) return set_error(QR_EVALUE, "unknown tuning knob '%s'", n.c_str());
    *value = k->load();
    return QR_OK;
}

int qr_code_info(const qr_code *code, int64_t *vnum, int64_t *cnum, int64_t *ednum, int32_t *max_dc,
                 int32_t *max_dv) {
    if (!code) return set_error(QR_EVALUE, "null code");
    if (vnum) *vnum = code->V;
    if (cnum) *cnum = code->C;
    if (ednum) *ednum = code->E;
    if (max_dc) *max_dc = code->max_dc;
    if (max_dv) *max_dv = code->max_dv;
    return QR_OK;
}

int qr_decode_workspace_size(const qr_code *code, int32_t ld, int32_t max_it, size_t *bytes) {
    if (!code || !bytes) return set_error(QR_EVALUE, "null argument");
    if (ld <= 0 || ld % kWave) return set_error(QR_EVALUE, "ld must be a positive multiple of 64");
    *bytes = ws_bytes(code, ld, max_it);
    return QR_OK;
}

int qr_decode_batch_device(const qr_code *code, int32_t B, int32_t ld, const double *d_lappr, const uint8_t *d_synd,
                           int32_t max_it, double *d_final, uint8_t *d_success, int32_t *d_iters, void *ws,
                           size_t ws_size, void *stream) {
    if (!code) return set_error(QR_EVALUE, "null code");
    return decode_batch_device(code, B, ld, d_lappr, d_synd, max_it, d_final, d_success, d_iters, ws, ws_size,
                               (hipStream_t)stream);
}

int qr_decode_host(const qr_code *code, int32_t B, const double *lappr, const uint8_t *synd, int32_t max_it,
                   double *final_lappr, uint8_t *success, int32_t *iterations) {
    if (!code) return set_error(QR_EVALUE, "null code");
    if (B <= 0) return set_error(QR_EVALUE, "B must be positive");
    const int ld = (int)align_up((size_t)B, kWave);
    const size_t V = code->V, C = code->C;
    const size_t n_fm = align_up(V * B * 8, 256), n_fi = align_up(V * ld * 8, 256);
    const size_t s_fm = align_up(C * B, 256), s_fi = align_up(C * ld, 256);
    const size_t flags = align_up((size_t)B, 256) + align_up((size_t)B * 4, 256);
    const size_t wsb = ws_bytes(code, ld, max_it);
    const size_t total = n_fm + 2 * n_fi + s_fm + s_fi + flags + wsb;
    DeviceGuard g(code->device);
    std::lock_guard<std::mutex> lk(code->scratch.mu);
    int rc = code->scratch.reserve(total);
    if (rc) return rc;
    char *p = (char *)code->scratch.ptr;
    double *d_fm = (double *)p;          p += n_fm;
    double *d_lappr = (double *)p;       p += n_fi;
    double *d_final = (double *)p;       p += n_fi;
    uint8_t *d_sfm = (uint8_t *)p;       p += s_fm;
    uint8_t *d_synd = (uint8_t *)p;      p += s_fi;
    uint8_t *d_succ = (uint8_t *)p;      p += align_up((size_t)B, 256);
    int32_t *d_it = (int32_t *)p;        p += align_up((size_t)B * 4, 256);
    void *d_ws = p;
    hipStream_t s = nullptr;
    QR_HIP(hipMemcpyAsync(d_fm, lappr, V * B * 8, hipMemcpyHostToDevice, s));
    QR_HIP(hipMemcpyAsync(d_sfm, synd, C * B, hipMemcpyHostToDevice, s));
    if ((rc = launch_transpose_to_fi_f64(B, ld, V, d_fm, d_lappr, s))) return rc;
    if ((rc = launch_transpose_to_fi_u8(B, ld, C, d_sfm, d_synd, s))) return rc;
    if ((rc = decode_batch_device(code, B, ld, d_lappr, d_synd, max_it, d_final, d_succ, d_it, d_ws, wsb, s)))
        return rc;
    if ((rc = launch_transpose_to_fm_f64(B, ld, V, d_final, d_fm, s))) return rc;
    QR_HIP(hipMemcpyAsync(final_lappr, d_fm, V * B * 8, hipMemcpyDeviceToHost, s));
    QR_HIP(hipMemcpyAsync(success, d_succ, B, hipMemcpyDeviceToHost, s));
    QR_HIP(hipMemcpyAsync(iterations, d_it, (size_t)B * 4, hipMemcpyDeviceToHost, s));
    QR_HIP(hipStreamSynchronize(s));
    return QR_OK;
}

// ------------------------------------------------------ unit-test surface
static int check_nodes_common(const qr_code *code, const void *vals, size_t val_bytes, const uint8_t *synd,
                              uint8_t *check_ok, uint8_t *all_ok, bool is_word) {
    if (!code) return set_error(QR_EVALUE, "null code");
    DeviceGuard g(code->device);
    std::lock_guard<std::mutex> lk(code->scratch.mu);
    const size_t C = code->C;
    const size_t a = align_up(val_bytes, 256), b = align_up(C, 256);
    int rc = code->scratch.reserve(a + 2 * b);
    if (rc) return rc;
    char *p = (char *)code->scratch.ptr;
    QR_HIP(hipMemcpy(p, vals, val_bytes, hipMemcpyHostToDevice));
    QR_HIP(hipMemcpy(p + a, synd, C, hipMemcpyHostToDevice));
    if (is_word)
        k_check_word_nodes<<<(unsigned)((C + 255) / 256), 256>>>(C, code->d_chk_ptr, code->d_chk_var,
                                                                  (const uint8_t *)p, (const uint8_t *)(p + a),
                                                                  (uint8_t *)(p + a + b));
    else
        k_check_lappr_nodes<<<(unsigned)((C + 255) / 256), 256>>>(C, code->d_chk_ptr, code->d_chk_var,
                                                                   (const double *)p, (const uint8_t *)(p + a),
                                                                   (uint8_t *)(p + a + b));
    QR_LAUNCH_CHECK();
    std::vector<uint8_t> ok(C);
    QR_HIP(hipMemcpy(ok.data(), p + a + b, C, hipMemcpyDeviceToHost));
    uint8_t all = 1;
    for (size_t c = 0; c < C; ++c) {
        if (check_ok) check_ok[c] = ok[c];
        if (!ok[c]) all = 0;  // decoder.pyx:214-217, :254-257
    }
    if (all_ok) *all_ok = all;
    return QR_OK;
}

int qr_check_lappr_host(const qr_code *code, const double *lappr, const uint8_t *synd, uint8_t *check_ok,
                        uint8_t *all_ok) {
    if (!code) return set_error(QR_EVALUE, "null code");
    return check_nodes_common(code, lappr, (size_t)code->V * 8, synd, check_ok, all_ok, false);
}

int qr_check_word_host(const qr_code *code, const uint8_t *word, const uint8_t *synd, uint8_t *check_ok,
                       uint8_t *all_ok) {
    if (!code) return set_error(QR_EVALUE, "null code");
    return check_nodes_common(code, word, (size_t)code->V, synd, check_ok, all_ok, true);
}

int qr_process_var_nodes_host(const qr_code *code, const int64_t *nodes, int64_t n, const double *lappr,
                              const double *c2v, double *v2c, double *updated) {
    if (!code) return set_error(QR_EVALUE, "null code");
    for (int64_t i = 0; i < n; ++i)
        if (nodes[i] < 0 || nodes[i] >= code->V) return set_error(QR_EVALUE, "variable node index out of range");
    if (n <= 0) return QR_OK;
    DeviceGuard g(code->device);
    std::lock_guard<std::mutex> lk(code->scratch.mu);
    const size_t V = code->V, E = code->E;
    const size_t sn = align_up(n * 8, 256), sv = align_up(V * 8, 256), se = align_up(E * 8, 256);
    int rc = code->scratch.reserve(sn + 2 * sv + 2 * se);
    if (rc) return rc;
    char *p = (char *)code->scratch.ptr;
    int64_t *d_nodes = (int64_t *)p;   p += sn;
    double *d_lappr = (double *)p;     p += sv;
    double *d_upd = (double *)p;       p += sv;
    double *d_c2v = (double *)p;       p += se;
    double *d_v2c = (double *)p;
    QR_HIP(hipMemcpy(d_nodes, nodes, n * 8, hipMemcpyHostToDevice));
    QR_HIP(hipMemcpy(d_lappr, lappr, V * 8, hipMemcpyHostToDevice));
    QR_HIP(hipMemcpy(d_upd, updated, V * 8, hipMemcpyHostToDevice));
    QR_HIP(hipMemcpy(d_c2v, c2v, E * 8, hipMemcpyHostToDevice));
    QR_HIP(hipMemcpy(d_v2c, v2c, E * 8, hipMemcpyHostToDevice));
    k_var_nodes<<<(unsigned)((n + 255) / 256), 256>>>(d_nodes, n, code->d_var_ptr, code->d_var_edge, d_lappr, d_c2v,
                                                      d_v2c, d_upd);
    QR_LAUNCH_CHECK();
    QR_HIP(hipMemcpy(v2c, d_v2c, E * 8, hipMemcpyDeviceToHost));
    QR_HIP(hipMemcpy(updated, d_upd, V * 8, hipMemcpyDeviceToHost));
    return QR_OK;
}

int qr_process_check_nodes_host(const qr_code *code, const int64_t *nodes, int64_t n, const uint8_t *synd,
                                double *c2v, const double *v2c) {
    if (!code) return set_error(QR_EVALUE, "null code");
    for (int64_t i = 0; i < n; ++i)
        if (nodes[i] < 0 || nodes[i] >= code->C) return set_error(QR_EVALUE, "check node index out of range");
    if (n <= 0) return QR_OK;
    DeviceGuard g(code->device);
    std::lock_guard<std::mutex> lk(code->scratch.mu);
    const size_t C = code->C, E = code->E;
    const size_t sn = align_up(n * 8, 256), sc = align_up(C, 256), se = align_up(E * 8, 256);
    int rc = code->scratch.reserve(sn + sc + 2 * se);
    if (rc) return rc;
    char *p = (char *)code->scratch.ptr;
    int64_t *d_nodes = (int64_t *)p;   p += sn;
    uint8_t *d_synd = (uint8_t *)p;    p += sc;
    double *d_c2v = (double *)p;       p += se;
    double *d_v2c = (double *)p;
    QR_HIP(hipMemcpy(d_nodes, nodes, n * 8, hipMemcpyHostToDevice));
    QR_HIP(hipMemcpy(d_synd, synd, C, hipMemcpyHostToDevice));
    QR_HIP(hipMemcpy(d_c2v, c2v, E * 8, hipMemcpyHostToDevice));
    QR_HIP(hipMemcpy(d_v2c, v2c, E * 8, hipMemcpyHostToDevice));
    k_check_nodes<<<(unsigned)((n + 255) / 256), 256>>>(d_nodes, n, code->d_chk_ptr, code->d_chk_edge, d_synd, d_c2v,
                                                        d_v2c, code->d_mtab);
    QR_LAUNCH_CHECK();
    QR_HIP(hipMemcpy(c2v, d_c2v, E * 8, hipMemcpyDeviceToHost));
    return QR_OK;
}

}  // extern "C"
