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
// parity check after the last sweep.  Schedules (decode_batch_device): the two
// frame halves pipelined on two streams (run_split2, the DVB-S2 default; the
// running frames of a converging half are listed (k_compact) and, once they are
// few, moved to contiguous columns (column repack)); all frames in lock-step
// (run_flat); small codes with one launch per iteration (run_iter) or one launch
// per decode with a workgroup per frame and its messages in LDS (k_resident).
#include <atomic>
#include <functional>

#include "glibc_math.hpp"
#include "qamr_internal.hpp"
#include "strict_pack.hpp"
#include "host_build.hpp"

namespace qr {

enum CheckMode { kFirst = 0, kNormal = 1, kParityOnly = 2 };
#define QR_STR2(x) #x
#define QR_STR(x) QR_STR2(x)

// Device-side index checks of the debug build (make -C csrc DEBUG=1 -> qamr/libqamr_debug.so,
// QR_DEBUG_ASSERT=1; SURVEY.md 5 -- the reference turns bounds checks off, decoder.pyx:181,240,
// 289,332,399,411): QR_DCHECK(ok, site, a, b) counts every failed check in g_dbg and keeps the
// first failure's site and two values; the first failing lane also prints them.  Non-fatal (no
// trap): the test reads the counts through qr_debug_asserts (tests/test_gpu_debug_build.py).  The
// product library compiles every check away.
#ifndef QR_DEBUG_ASSERT
#define QR_DEBUG_ASSERT 0
#endif
#if QR_DEBUG_ASSERT
__device__ unsigned long long g_dbg[4];  // {failed checks, first site, first a, first b}
__device__ __noinline__ void dcheck_fail(int site, long long a, long long b) {
    if (atomicAdd(&g_dbg[0], 1ull) == 0ull) {
        g_dbg[1] = (unsigned long long)site;
        g_dbg[2] = (unsigned long long)a;
        g_dbg[3] = (unsigned long long)b;
        printf("qamr debug check %d failed: a=%lld b=%lld (block %u thread %u)\n", site, a, b, blockIdx.x, threadIdx.x);
    }
}
#define QR_DCHECK(ok, site, a, b)                                   \
    do {                                                            \
        if (!(ok)) dcheck_fail((site), (long long)(a), (long long)(b)); \
    } while (0)
#else
#define QR_DCHECK(ok, site, a, b) ((void)0)
#endif
// check sites (qr_debug_asserts reports the first failure's site)
enum DebugSite {
    kDbgLaneFrame = 1,     // lane_frame: a listed column outside the sweep's range
    kDbgNarrowFrame = 2,   // narrow sweeps: lane frame outside the repacked range's first 64 columns
    kDbgNarrowNode = 3,    // narrow sweeps: check id / CSR offset out of range
    kDbgRepackList = 4,    // k_repack_rows: list entry not ascending or outside [f0, f0 + w)
    kDbgRepackSlot = 5,    // gather_rows: a slot's byte offset outside its row group
    kDbgRepackFid = 6,     // hand-out / commit / k_repack_output: frame id outside [0, ld)
    kDbgCompact = 7,       // k_compact: list index outside the range
    kDbgResPost = 8,       // k_resident: posterior index outside [0, V)
    kDbgResMsg = 9,        // k_resident: LDS message index outside [0, C D)
};

// Check-node arithmetic: the reference's box-plus bit for bit -- glibc exp/log restated
// (glibc_math.hpp, the box-plus part of its tables, 8 KiB, staged in LDS per workgroup; a few
// constants pinned in VGPRs, GlibcK) -- so every message, posterior and output LAPPR is
// identical to the reference's.  (Rounds 1-4 also carried two approximate arithmetics; they
// missed north_star's 1e-6 LAPPR bar at configs[3] and were removed.)

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

// Read-only graph data (CSR) at a wave-uniform index through the constant address space:
// the load becomes a scalar s_load instead of a vector load + v_readfirstlane (the
// compiler cannot prove the generic pointer is not written by the kernel's own stores).
template <typename T>
__device__ __forceinline__ T sld(const T *p) {
    return *(const __attribute__((address_space(4))) T *)p;
}

// Message / posterior access of the check sweep through a raw buffer resource built from
// the (wave-uniform) row pointer in scalar registers: the lane's byte offset goes in the
// instruction's VGPR offset, so an access costs no VALU (a flat/global access needs a
// 64-bit v_lshl_add per access here, the compiler hoists base + lane offset and adds the
// scalar row offset per access).
typedef unsigned int qr_u32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ __amdgpu_buffer_rsrc_t row_rsrc(const double *rowp, int ld) {
    // word 3 = 0x00020000: DATA_FORMAT 32 (raw dword access), no swizzle; num_records = row bytes
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<double *>(rowp), (short)0, ld * 8, 0x00020000);
}

// Row `row` (wave-uniform) of a frame-innermost array: the row offset is computed in
// scalar registers; lanes add their byte offset f * sizeof(T).
template <typename T>
__device__ __forceinline__ T *row_ptr(T *base, int row, int ld) {
    return base + (size_t)(uint32_t)__builtin_amdgcn_readfirstlane(row) * (size_t)ld;
}
// Element at byte offset `boff` (32-bit, = f * sizeof(T)) of a wave-uniform row.
template <typename T>
__device__ __forceinline__ T *at_byte(T *rowp, uint32_t boff) {
    return (T *)((char *)rowp + boff);
}
// Load / store of the lane's double in a wave-uniform row (row pointer rowp, ld doubles).
template <bool NT>
__device__ __forceinline__ double ld_row(const double *rowp, uint32_t b8, int ld) {
    return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(row_rsrc(rowp, ld), b8, 0, NT ? 2 : 0));
}
template <bool NT>
__device__ __forceinline__ void st_row(double *rowp, uint32_t b8, int ld, double v) {
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(qr_u32x2, v), row_rsrc(rowp, ld), b8, 0, NT ? 2 : 0);
}

// Block geometry shared by the check and variable sweeps: 256 threads = `ft`
// consecutive frames (ft = 64 << k, a multiple of the wavefront) x (256/ft)
// node lanes; every wave therefore covers 64 frames of ONE node, which makes
// the node index wave-uniform (readfirstlane -> scalar loads of the CSR).
struct Geom {
    int lft;  // log2(ft)
    int per;  // nodes per thread
};

// One check sweep over the frame columns [f_off, f_off + ny*ft) of one degree class.
struct CheckArgs {
    const int32_t *checks;  // the class's check ids
    int64_t n_checks;
    const int32_t *chk_ptr, *chk_edge, *chk_var;
    const double *post;
    double *c2v;
    const uint8_t *synd;
    const uint8_t *active;
    uint8_t *unsat;
    int ld, f_off;
    Geom g;
    unsigned nbx;  // blocks along the check axis
    const GlibcTables *gglibc;
    double *fb;          // runtime-degree kernel: F scratch of the class (row fb_base)
    int64_t fb_base;
    const int32_t *alist;   // active-frame list (frame ids at alist[f_off + p]) or null
    const int32_t *acount;  // its length
    const int32_t *finite;  // strict arithmetic: 1 iff the batch's input LAPPRs are all finite (or null)
    // Short-tail grid (knob check_tail; k_check only): a 1-D grid whose first nmain blocks sweep
    // frame tiles 1.. with g.per checks per thread (block b: tile 1 + b / nbx, check block
    // b % nbx) and whose last blocks sweep frame tile 0 with per_t checks per thread -- the
    // workgroups dispatched last are the short ones, so the launch drains in ~a quarter of a
    // workgroup's time.  nmain = 0: the plain 2-D grid (nbx x frame tiles).
    unsigned nmain;
    int per_t;
    // Column repack (run_split2): sel -> the range's RangeSel, or null.  Once the device has
    // repacked the range (sel[kSelOn]) its posteriors live in the work set (post_w) and its
    // messages and syndrome bits in the work set's column set sel[kSelBuf] (c2v / c2v_alt,
    // synd_w[0] / synd_w[1]).
    const int32_t *sel;
    const double *post_w;
    const uint8_t *synd_w[2];
    double *c2v_alt;
    // set by select_range: 1 for the first sweep after a repack (its messages are read from the
    // old column set at the frames' old columns, c2v_rd / the list; everything else is read and
    // written in the new columns, see k_repack_rows)
    int transit;
    const double *c2v_rd;
};

// One variable sweep over the frame columns [f_off, f_off + ny*ft).
struct VarArgs {
    int64_t V;
    const int32_t *var_ptr, *var_edge;
    const double *lappr, *c2v;
    double *post;
    const uint8_t *active;
    int ld, f_off;
    Geom g;
    unsigned nbx;
    const int32_t *alist, *acount;  // as CheckArgs
    unsigned nby;  // frame tiles (grid-stride launches)
    int gs;        // 1: a capped 1-D grid walks the nbx x nby tiles (the paced sweeps of run_split2, knob var_pace)
    int boost;     // gs grid = boost x the paced width; as the live frame tiles drop to nby / k, min(k, boost) widths sweep
    // INIT sweep only: the strict arithmetic's finite flag (see kPackMaxDeg) is cleared when an
    // input LAPPR of a frame < fin_B is not below fin_bound in magnitude (null: not computed)
    int32_t *finite;
    double fin_bound;
    int fin_B;
    const int32_t *sel;  // as CheckArgs: the range's RangeSel or null; work-set LAPPRs / posteriors / messages
    const double *lappr_w[2];
    double *post_w;
    const double *c2v_alt;
    int transit;  // as CheckArgs (set by select_range); in transit c2v is the old column set
};

// The state of one frame range of the two-stream schedule, in device memory (the workspace's
// count block), read by every launch of that range and written only by a repack's commit (k_repack_rows): whether
// the range has moved to the repack work set, its width there (its running frames occupy the
// first columns), how many repacks it went through, and which of the work set's two column sets
// (messages, LAPPRs, syndrome bits) holds it: a repack gathers the running columns of one set
// into the other, so no column is overwritten while another thread may still read it.
// kSelTransit: the range was repacked at its last decision point and the sweeps that follow it
// (its variable sweep, then its check sweeps) have not all run yet: their messages still live in
// the old column set, at the frames' old columns (the active-frame list, which the commit leaves
// as it is until the next status launch rebuilds it).
enum RangeSelField { kSelOn = 0, kSelW = 1, kSelRepacks = 2, kSelArrive = 3, kSelBuf = 4, kSelTransit = 5, kSelInts = 6 };

// Kernel-uniform: the arrays a range's launch reads once the device has repacked the range.
__device__ __forceinline__ void select_range(CheckArgs &a) {
    if (a.sel && sld(a.sel + kSelOn)) {
        const int b = sld(a.sel + kSelBuf);
        a.post = a.post_w;
        a.synd = b ? a.synd_w[1] : a.synd_w[0];  // (selects: a dynamic index would put a in scratch)
        double *const c0 = a.c2v, *const c1 = a.c2v_alt;
        a.c2v = b ? c1 : c0;
        a.transit = sld(a.sel + kSelTransit);
        a.c2v_rd = a.transit ? (b ? c0 : c1) : a.c2v;
    }
}
__device__ __forceinline__ void select_range(VarArgs &a) {
    if (a.sel && sld(a.sel + kSelOn)) {
        const int b = sld(a.sel + kSelBuf);
        a.lappr = b ? a.lappr_w[1] : a.lappr_w[0];
        a.post = a.post_w;
        a.transit = sld(a.sel + kSelTransit);
        if (a.transit ? !b : b) a.c2v = a.c2v_alt;  // transit: the old set
    }
}

// Active-frame compaction (converging operating points, decoder.pyx:431-433: frames stop
// at their own iteration).  Without a list a sweep's lane p of the frame range is frame
// f_off + p and stopped frames in a partly stopped wavefront run along; with one (built
// by k_compact after every status update) lane p is the p-th still-running frame, the
// range's tail blocks exit at once, and lanes past the count (live = false) repeat the
// last frame's reads but store nothing (a store would race with that frame's own lane,
// which may still read the old message).
__device__ __forceinline__ bool frames_block_live(const int32_t *acount, unsigned by, int lft) {
    return !acount || (int)(by << lft) < *acount;
}
__device__ __forceinline__ int lane_frame(const int32_t *alist, const int32_t *acount, int f_off, int p, bool &live) {
    live = true;
    if (!alist) return f_off + p;
    const int cnt = *acount;
    live = p < cnt;
    const int f = alist[f_off + (live ? p : cnt - 1)];
    QR_DCHECK(f >= f_off + (live ? p : cnt - 1), kDbgLaneFrame, f, f_off + p);  // ascending, in the range
    return f;
}


// The inputs of one check update: gathered posteriors, own c2v messages, syndrome bit.
// The gathered posteriors of check j+1 are issued before the arithmetic of check j on the
// unpacked paths (the packed strict update needs those registers: with the prefetch it runs
// at 3 waves/SIMD, 142 VGPRs); the own (streamed, row-contiguous) messages are loaded on use.
template <int D, int MODE, bool NT, bool TRANSIT = false>
struct CheckIn {
    double p[D], c[D];
    int base;
    uint8_t sb;
    __device__ __forceinline__ void load(const CheckArgs &a, int64_t ci, int f) {
        const int ld = a.ld;
        const uint32_t b8 = (uint32_t)f * 8u;
        const int cc = sld(a.checks + ci);
        base = sld(a.chk_ptr + cc);
        sb = *at_byte(row_ptr(a.synd, cc, ld), (uint32_t)f);
#pragma unroll
        for (int i = 0; i < D; ++i) p[i] = ld_row<false>(row_ptr(a.post, sld(a.chk_var + base + i), ld), b8, ld);
    }
    // fc: the frame's column of its messages (in transit its old column, c2v_rd the old set)
    __device__ __forceinline__ void load_c(const CheckArgs &a, int fc) {
        if (MODE != kNormal) return;
        const uint32_t b8 = (uint32_t)fc * 8u;
        const double *c2v = TRANSIT ? a.c2v_rd : a.c2v;
#pragma unroll
        for (int i = 0; i < D; ++i) c[i] = ld_row<NT>(row_ptr(c2v, sld(a.chk_edge + base + i), a.ld), b8, a.ld);
    }
};

// The syndrome sign of a check's outputs (decoder.pyx:360-369: s * message, s = -1 when the
// syndrome bit is set): s * x with s = +-1 only flips x's sign bit (for NaN too, as the compiled
// multiply by the selected constant did), so it is one XOR of the high word with a per-check mask
// instead of the compiler's XOR + select per output.
__device__ __forceinline__ uint32_t sign_mask(uint8_t sb) { return sb ? 0x80000000u : 0u; }
__device__ __forceinline__ double apply_sign(double x, uint32_t smask) { return g_make(g_hi(x) ^ smask, g_lo(x)); }

// Degrees whose round loop the compiler still unrolls fully (above, the packed update's
// register arrays would be indexed dynamically, i.e. live in scratch): the unpacked strict
// update runs there.
constexpr int kPackMaxDeg = 10;
// The strict arithmetic's finite flag: when every input LAPPR of the batch's frames is below
// a bound 2^e (a device flag computed by the decode's first variable sweep), no inf or NaN can
// arise in any sweep: |c2v| <= max |v2c| (a box-plus never exceeds its smaller operand, to
// rounding) and |v2c| <= |L| + (dv - 1) max |c2v|, so X_t = max |post| + max |c2v| after
// sweep t obeys X_{t+1} <= |L| + (dv + 1) X_t and every value (box-plus arguments, twice
// that) stays below 2^e (dv + 1)^(max_it + 2), which e = 1000 - (max_it + 2) log2(dv_max + 1)
// keeps finite.  The check sweeps then run the packed update with the one-instruction clamp
// (strict_pack.hpp kClampFinite) instead of the NaN-preserving two-instruction one.
// LDS of the packed strict update: one buffer per wavefront of a block.
constexpr int kPackLdsDoubles = 4 * kPackWaveDoubles;
template <int D>
constexpr bool kPacked = D <= kPackMaxDeg;

// decoder.pyx:322-369 for one check (strict box-plus).
// Packed strict update (D <= kPackMaxDeg): strict_pack.hpp.  Otherwise
// F[i] = bp(F[i-1], m[i]); the backward values B[i] = bp(B[i+1], m[i]) are consumed as
// they are produced (out_i = bp(F[i-1], B[i+1])): the same operands as
// decoder.pyx:341-367, one live B instead of D.  Lane byte offset b8 = f * 8.
template <int D, bool NT, bool FIN = false>
__device__ __forceinline__ void check_exact(const CheckArgs &a, const double (&m)[D], int base, uint8_t sb, uint32_t b8,
                                            const GlibcTablesBP &tab, const GlibcK &K, double *hb = nullptr,
                                            bool live = true) {
    const int ld = a.ld;
    const double s = sb ? -1.0 : 1.0;
    if constexpr (kPacked<D>) {
        double out[D];
        double *wb = hb + (threadIdx.x >> 6) * kPackWaveDoubles;
        check_strict_packed<D, FIN ? kClampFinite : kClampFull>(m, out, wb, tab, K);
        const uint32_t smask = sign_mask(sb);
#pragma unroll
        for (int i = 0; i < D; ++i)
            if (live) st_row<NT>(row_ptr(a.c2v, sld(a.chk_edge + base + i), ld), b8, ld, apply_sign(out[i], smask));
        return;
    }
    double F[D - 1];
    F[0] = m[0];
#pragma unroll
    for (int i = 1; i < D - 1; ++i) F[i] = box_plus_strict(F[i - 1], m[i], tab, K);
    if (live) st_row<NT>(row_ptr(a.c2v, sld(a.chk_edge + base + D - 1), ld), b8, ld, s * F[D - 2]);
    double Bn = m[D - 1];
#pragma unroll
    for (int i = D - 2; i > 0; --i) {
        const double o = s * box_plus_strict(F[i - 1], Bn, tab, K);
        if (live) st_row<NT>(row_ptr(a.c2v, sld(a.chk_edge + base + i), ld), b8, ld, o);
        Bn = box_plus_strict(Bn, m[i], tab, K);
    }
    if (live) st_row<NT>(row_ptr(a.c2v, sld(a.chk_edge + base), ld), b8, ld, s * Bn);
}

// One lane = one (check, frame); each thread walks `per` checks of one degree class.
// decoder.pyx:322-369 (F/B recursion) with the parity test of decoder.pyx:235-257
// fused on the posteriors it gathers anyway.  Unpacked paths are software-pipelined: the
// posterior gathers of check j+1 are issued before the box-plus arithmetic of check j.
template <int D, int MODE, bool NT, bool FIN = false, bool TRANSIT = false>
__device__ __forceinline__ void check_block(const CheckArgs &a, unsigned bx, unsigned by, int per,
                                            const GlibcTablesBP &tab, double *hb) {
    const int ft = 1 << a.g.lft;
    const int nsub = 256 >> a.g.lft;
    bool live;
    const int lp = (int)(by << a.g.lft) + (threadIdx.x & (ft - 1));
    const int fl = lane_frame(a.alist, a.acount, a.f_off, lp, live);
    // TRANSIT (the first check sweep after a repack): the lane's frame sits in column f_off + lp of
    // the new set; only its old messages are still at its listed (old) column fl
    const int f = TRANSIT ? a.f_off + lp : fl;
    const int sub = __builtin_amdgcn_readfirstlane(threadIdx.x >> a.g.lft);
    // Waves whose 64 frames all stopped leave; in a partly stopped wave the stopped
    // lanes run along (no divergent exit, so the loop state stays scalar): their
    // messages are never read again and their posteriors (the output) are not touched.
    // Lanes past the compacted count (repeating the last listed frame) count as stopped:
    // once fewer than a tile's frames remain, the tile's empty waves leave at once.
    const bool act = live && a.active[f] != 0;
    if (!wave_any(act)) return;
    int64_t ci = (int64_t)bx * per * nsub + sub;
    if (ci >= a.n_checks) return;
    uint32_t bad = 0;
    const auto K = GlibcK::pinned();
    constexpr bool kPrefetch = !kPacked<D>;
    CheckIn<D, MODE, NT, TRANSIT> nx;
    nx.load(a, ci, f);
    for (int j = 0; j < per; ++j) {
        // consume check j's inputs (m, parity) before its registers take check j+1's
        nx.load_c(a, TRANSIT ? fl : f);
        uint32_t par = nx.sb;
        double m[D];
#pragma unroll
        for (int i = 0; i < D; ++i) {
            const double p = nx.p[i];
            if (MODE != kFirst) par ^= (p < 0.0) ? 1u : 0u;   // decoder.pyx:243-246
            if (MODE == kNormal) m[i] = p - nx.c[i];           // :296-297
            else m[i] = p;  // first sweep: c2v == 0 and p - 0.0 == p
        }
        struct { int base; uint8_t sb; } cur = {nx.base, nx.sb};
        const int64_t cn = ci + nsub;
        const bool more = (j + 1 < per) && cn < a.n_checks;   // wave-uniform
        if (kPrefetch && more) nx.load(a, cn, f);
        if (MODE != kFirst) bad |= (par == 1u) ? 1u : 0u;  // satisfied iff (parity ^ 1) != 0
        if (MODE != kParityOnly) {
            const uint32_t b8 = (uint32_t)f * 8u;
            check_exact<D, NT, FIN>(a, m, cur.base, cur.sb, b8, tab, K, hb, live);
        }
        if (!more) break;
        if (!kPrefetch) nx.load(a, cn, f);
        ci = cn;
    }
    if (MODE != kFirst && bad && act && live) a.unsat[f] = 1;  // benign race: every writer stores 1
}

// decoder.pyx:285-298: post[v] = lappr[v] + c2v[e_0] + c2v[e_1] + ... (ascending e).
// INIT: the first sweep with c2v == 0 (decoder.pyx:408,420-421): lappr + 0.0 for
// frames still decoding; frames already successful at iteration 0 get a plain
// copy of their input (decoder.pyx:404).
// TRANSIT (the first variable sweep after a repack): the frame's LAPPRs and posterior are in
// column f_off + lp of the new set, its messages still at its listed (old) column of the old set.
template <bool INIT, bool NT, bool TRANSIT = false>
__device__ __forceinline__ void var_block(const VarArgs &a, unsigned bx, unsigned by) {
    const int ft = 1 << a.g.lft;
    const int nsub = 256 >> a.g.lft;
    const int ld = a.ld;
    bool live;
    const int lp = (int)(by << a.g.lft) + (threadIdx.x & (ft - 1));
    const int fl = lane_frame(a.alist, a.acount, a.f_off, lp, live);
    const int f = TRANSIT ? a.f_off + lp : fl;
    const int fc = TRANSIT ? fl : f;
    const int sub = __builtin_amdgcn_readfirstlane(threadIdx.x >> a.g.lft);
    const bool act = a.active[f] != 0;
    if (!live || (!INIT && !act)) return;
    const int64_t v0 = (int64_t)bx * a.g.per * nsub + sub;
    bool big = false;
    for (int j = 0; j < a.g.per; ++j) {
        const int64_t v = v0 + (int64_t)j * nsub;
        if (v >= a.V) break;
        const int b = sld(a.var_ptr + v), e = sld(a.var_ptr + v + 1);
        double p = ld_msg<NT>(&a.lappr[(size_t)v * ld + f]);
        if (INIT) {
            big |= !(__builtin_fabs(p) < a.fin_bound);
            if (act && e > b) p = p + 0.0;
        } else {
            for (int k = b; k < e; ++k) p += ld_msg<NT>(&a.c2v[(size_t)sld(a.var_edge + k) * ld + fc]);
        }
        a.post[(size_t)v * ld + f] = p;
    }
    if (INIT && a.finite && big && f < a.fin_B) *a.finite = 0;  // every writer stores 0
}

// ---------------------------------------------------------------------------------------
// Narrow sweeps: a repacked range of at most kNarrowW columns (the last running frames of a
// converging half).  The frame-parallel layout gives every check a 64-lane wave of frames, so
// a handful of running frames still pay a whole wave per check, per checks in sequence.  Such
// a range (known only on the device: its RangeSel) switches the SAME launch, kernel-uniformly,
// to lanes = (node, frame): a workgroup task is kNarrowNodes nodes x kNarrowFrames consecutive
// columns (one 128-byte line per row access), one node per lane, tasks walked grid-stride, the
// CSR read per lane.  Every message is the same operation on the same operands as in
// check_block / var_block, so the bits do not depend on the layout.
constexpr int kNarrowFrames = 16;
constexpr int kNarrowNodes = 256 / kNarrowFrames;
constexpr int kNarrowW = 64;

__device__ __forceinline__ bool range_narrow(const int32_t *sel, const int32_t *acount) {
    return sel && acount && sld(sel + kSelOn) && sld(sel + kSelW) <= kNarrowW && !sld(sel + kSelTransit);
}
// Tasks of a narrow sweep over n nodes: (node block, frame group) pairs, frame group fastest, the
// group count (<= 4) rounded up to 2^lg so that a task splits with a shift and a mask (32-bit task
// arithmetic: the variable sweep keeps its register budget)
__device__ __forceinline__ uint32_t narrow_tasks(int64_t n, const int32_t *acount, int &lg) {
    const int ngrp = (sld(acount) + kNarrowFrames - 1) / kNarrowFrames;
    lg = ngrp > 2 ? 2 : ngrp > 1 ? 1 : 0;
    return ngrp > 0 ? (uint32_t)((n + kNarrowNodes - 1) / kNarrowNodes) << lg : 0u;
}

// The NaN-preserving clamp always (the finite flag's one-instruction clamp gives the same bits
// on finite inputs; the narrow body is not worth a second copy).
template <int D>
__device__ __forceinline__ void check_narrow(const CheckArgs &a, uint32_t task, int lg, const GlibcTablesBP &tab,
                                             double *hb, const GlibcK &K) {
    bool live;
    const int grp = (int)(task & ((1u << lg) - 1u));
    const int f = lane_frame(a.alist, a.acount, a.f_off, grp * kNarrowFrames + (int)(threadIdx.x % kNarrowFrames), live);
    const bool act = live && a.active[f] != 0;
    if (!wave_any(act)) return;  // wave-uniform: the packed update exchanges within the wave
    const int64_t ci = (int64_t)(task >> lg) * kNarrowNodes + threadIdx.x / kNarrowFrames;
    const bool valid = ci < a.n_checks;
    const int cc = a.checks[valid ? ci : a.n_checks - 1];
    int base = a.chk_ptr[cc];
    QR_DCHECK(f >= a.f_off && f < a.f_off + kNarrowW, kDbgNarrowFrame, f, a.f_off);
    QR_DCHECK(cc >= 0 && base >= 0 && a.chk_ptr[cc + 1] - base == D, kDbgNarrowNode, cc, base);
    const size_t ld = a.ld;
    const uint8_t sb = a.synd[(size_t)cc * ld + f];
    uint32_t par = sb;
    double m[D];
#pragma unroll
    for (int i = 0; i < D; ++i) {
        const double p = a.post[(size_t)a.chk_var[base + i] * ld + f];
        par ^= (p < 0.0) ? 1u : 0u;                                // decoder.pyx:243-246
        m[i] = p - a.c2v[(size_t)a.chk_edge[base + i] * ld + f];  // :296-297
    }
    double out[D];
    check_strict_packed<D, kClampFull>(m, out, hb + (threadIdx.x >> 6) * kPackWaveDoubles, tab, K);
    // the stores re-read the edge ids: D message addresses held across the update would raise
    // the kernel's register budget (its frame-parallel body runs at 4 waves/SIMD)
    __asm__ volatile("" : "+v"(base));
    const double s = sb ? -1.0 : 1.0;
    if (valid && act) {
#pragma unroll
        for (int i = 0; i < D; ++i) a.c2v[(size_t)a.chk_edge[base + i] * ld + f] = s * out[i];
        if (par == 1u) a.unsat[f] = 1;  // benign race: every writer stores 1
    }
}

template <int D>
__device__ __forceinline__ void check_narrow_sweep(const CheckArgs &a, GlibcTablesBP &tab, double *hb) {
    int lg;
    const uint32_t ntask = narrow_tasks(a.n_checks, a.acount, lg);
    const uint32_t nb = gridDim.x * gridDim.y, b = blockIdx.y * gridDim.x + blockIdx.x;
    if (b >= ntask) return;  // block-uniform
    stage_glibc_tables(&tab, a.gglibc);
    const auto K = GlibcK::pinned();
    for (uint32_t t = b; t < ntask; t += nb) check_narrow<D>(a, t, lg, tab, hb, K);
}

__device__ __forceinline__ void var_narrow_sweep(const VarArgs &a) {
    int lg;
    const uint32_t ntask = narrow_tasks(a.V, a.acount, lg);
    const uint32_t nb = gridDim.x * gridDim.y;
    const size_t ld = a.ld;
    for (uint32_t t = blockIdx.y * gridDim.x + blockIdx.x; t < ntask; t += nb) {
        bool live;
        const int grp = (int)(t & ((1u << lg) - 1u));
        const int f = lane_frame(a.alist, a.acount, a.f_off, grp * kNarrowFrames + (int)(threadIdx.x % kNarrowFrames), live);
        const int64_t v = (int64_t)(t >> lg) * kNarrowNodes + threadIdx.x / kNarrowFrames;
        if (!live || v >= a.V || !a.active[f]) continue;
        QR_DCHECK(f >= a.f_off && f < a.f_off + kNarrowW, kDbgNarrowFrame, f, a.f_off);
        double p = a.lappr[(size_t)v * ld + f];
        const int b = a.var_ptr[v], e = a.var_ptr[v + 1];
        for (int k = b; k < e; ++k) p += a.c2v[(size_t)a.var_edge[k] * ld + f];  // decoder.pyx:292-293
        a.post[(size_t)v * ld + f] = p;
    }
}

// QR_EXPERIMENT_CLOCK (diagnostic builds only, scripts/diag/clock_check.py): every workgroup of
// the degree-7 main-loop check sweep and of the frame-resident decode stamps the shader clock
// (ClkScope, qamr_internal.hpp) around its work and adds its spans to g_clk; the effective clock of
// the unprofiled launch is sum(cycles) / sum(ticks) x 100 MHz (MI355X_MICROARCH.md 'DVFS give-back'
// item 6).  qr_debug_clock reads and clears the sums.
#if QR_EXPERIMENT_CLOCK
__device__ unsigned long long g_clk[3];
// realtime start / end of every workgroup of the last such launch (up to kWgTimes workgroups):
// the launch's occupancy over time, i.e. how much of it is the drain at its end
__device__ unsigned long long g_wgt[2 * kWgTimes];
#endif
template <int D, int MODE, bool NT>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 8))) k_check(CheckArgs a) {
    __shared__ GlibcTablesBP tab;
    __shared__ double hb[kPackLdsDoubles];
    select_range(a);
    if constexpr (MODE == kNormal && kPacked<D>) {
        if (range_narrow(a.sel, a.acount)) {  // kernel-uniform
            check_narrow_sweep<D>(a, tab, hb);
            return;
        }
    }
    unsigned bx = blockIdx.x, by = blockIdx.y;
    int per = a.g.per;
    if (a.nmain) {  // short-tail 1-D grid (block-uniform)
        if (bx < a.nmain) {
            by = 1 + bx / a.nbx;
            bx -= (by - 1) * a.nbx;
        } else {
            bx -= a.nmain;
            by = 0;
            per = a.per_t;
        }
    }
    if (!frames_block_live(a.acount, by, a.g.lft)) return;  // block-uniform
#if QR_EXPERIMENT_CLOCK
    ClkScope clk(D == 7 && MODE == kNormal, g_clk, g_wgt);
#endif
    if (MODE != kParityOnly) stage_glibc_tables(&tab, a.gglibc);
    if constexpr (MODE == kNormal && kPacked<D>) {
        if (a.transit) {  // kernel-uniform: the first sweep after a repack (NaN-preserving clamp)
            check_block<D, MODE, NT, false, true>(a, bx, by, per, tab, hb);
            return;
        }
    }
    if constexpr (MODE != kParityOnly && kPacked<D>) {
        if (a.finite && sld(a.finite)) {  // kernel-uniform: one of the two bodies runs
            check_block<D, MODE, NT, true>(a, bx, by, per, tab, hb);
            return;
        }
    }
    check_block<D, MODE, NT, false>(a, bx, by, per, tab, hb);
}

template <bool INIT, bool NT, bool TRANSIT>
__device__ __forceinline__ void var_sweep_body(const VarArgs &a);

template <bool INIT, bool NT>
__global__ void __launch_bounds__(256) k_var(VarArgs a) {
#ifdef QR_EXPERIMENT_VAR_VGPR  // register-rule probe builds only: allocate this many VGPRs (e.g. 24)
    __asm__ volatile("" ::: "v" QR_STR(QR_EXPERIMENT_VAR_VGPR_LAST));
#endif
    select_range(a);
    if (!INIT && range_narrow(a.sel, a.acount)) {  // kernel-uniform
        var_narrow_sweep(a);
        return;
    }
    if (!INIT && a.transit) var_sweep_body<INIT, NT, true>(a);  // kernel-uniform
    else var_sweep_body<INIT, NT, false>(a);
}

template <bool INIT, bool NT, bool TRANSIT>
__device__ __forceinline__ void var_sweep_body(const VarArgs &a) {
    if (a.gs) {  // capped grid: tile t = (bx fastest, by), the grid's blocks sweep a moving window
        unsigned ny = a.nby, stride = gridDim.x;
        if (a.boost > 1) {
            // The pacing spreads a full sweep over the concurrent check launch; once most frames
            // have stopped, both launches shrink and a paced sweep of the few live tiles would be
            // latency-bound (a few workgroups per CU walking many blocks each): widen it.
            const unsigned w = gridDim.x / (unsigned)a.boost;
            unsigned live = a.nby;
            if (a.acount) live = min(a.nby, (unsigned)((*a.acount + (1 << a.g.lft) - 1) >> a.g.lft));
            const unsigned m = live ? min((unsigned)a.boost, max(1u, a.nby / live)) : 1u;
            stride = w * m;
            ny = live;
            if (blockIdx.x >= stride) return;
        }
        const unsigned n = a.nbx * ny;
        for (unsigned t = blockIdx.x; t < n; t += stride) {
            const unsigned by = t / a.nbx, bx = t - by * a.nbx;
            if (frames_block_live(a.acount, by, a.g.lft)) var_block<INIT, NT, TRANSIT>(a, bx, by);
        }
        return;
    }
    if (!frames_block_live(a.acount, blockIdx.y, a.g.lft)) return;
    var_block<INIT, NT, TRANSIT>(a, blockIdx.x, blockIdx.y);
}


// ---------------------------------------------------------------------------------------
// Small codes (configs[1], reg-(3,6) N=1008): ONE launch per iteration.  A sweep of such a
// code is a few microseconds of chip work, so the three launches of the flat schedule
// (check, status, variable) are dominated by dispatch and drain.  Here the check sweep
// computes the posteriors it needs itself, from the previous iteration's messages:
//   post(t-1)[v] = lappr[v] + c2v(t-1)[e_0] + c2v(t-1)[e_1] + ...   (ascending edge id,
//                  decoder.pyx:292-293 -- the same additions, so the same bits)
// and the check whose edge is v's first edge stores it (the decoder's output), so no
// variable sweep is needed.  The messages are double-buffered by iteration parity (a check
// of iteration t reads c2v(t-1) of edges other checks are rewriting).  Launch P(t):
//   * status of iteration t-2 (t >= 3): frames whose post(t-2) satisfied the syndrome stop
//     with (1, t-2); the check of index 0 of each frame writes it, every lane derives the
//     same running flag act = active && unsat(t-2) (so the write races benignly);
//   * post(t-1) on the fly, its parity (unsat(t-1), t >= 2), c2v(t) (t <= max_it).
// Per frame the order is the reference's: check(t) -> status(t-1) -> var(t) -> check(t+1);
// P(max_it + 1) is the final parity sweep.  Used for single-degree-class codes with D <= 10
// when the split schedules do not pay (knob fused_iter).
struct IterArgs {
    const int32_t *checks;
    int64_t n_checks;
    const int32_t *chk_ptr, *chk_edge, *chk_var, *var_ptr, *var_edge;
    const double *lappr;
    double *post;
    const double *c2v_in;  // c2v(t-1), or null at t = 1 (all messages 0)
    double *c2v_out;       // c2v(t), or null in the final parity sweep
    const uint8_t *synd;
    uint8_t *active, *success;
    int32_t *iters;
    const uint8_t *unsat_s;  // row t-2 (status to apply), or null
    uint8_t *unsat_p;        // row t-1 (parity of post(t-1)), or null at t = 1
    int32_t status_iter;     // t - 2
    int ld, f_off;           // the launch sweeps frames [f_off, f_off + gridDim.y * ft)
    Geom g;
    unsigned nbx;
    const GlibcTables *gglibc;
    const int32_t *finite;
};

// Every access is cached (no non-temporal hint): a small code's messages, posteriors and LAPPRs
// are re-read every iteration from L2 / MALL.
template <int D, bool FIN>
__device__ __forceinline__ void iter_block(const IterArgs &a, unsigned bx, unsigned by, const GlibcTablesBP &tab,
                                           double *hb) {
    const int ft = 1 << a.g.lft;
    const int nsub = 256 >> a.g.lft;
    const int ld = a.ld;
    const int f = a.f_off + (int)(by << a.g.lft) + (threadIdx.x & (ft - 1));
    const int sub = __builtin_amdgcn_readfirstlane(threadIdx.x >> a.g.lft);
    const bool was = a.active[f] != 0;
    const bool act = was && (!a.unsat_s || a.unsat_s[f] != 0);
    int64_t ci = (int64_t)bx * a.g.per * nsub + sub;
    if (ci == 0 && was && !act) {  // decoder.pyx:431-433 for iteration t-2
        a.success[f] = 1;
        a.iters[f] = a.status_iter;
        a.active[f] = 0;
    }
    if (!wave_any(act)) return;
    const auto K = GlibcK::pinned();
    const uint32_t b8 = (uint32_t)f * 8u;
    uint32_t bad = 0;
    for (int j = 0; j < a.g.per; ++j, ci += nsub) {
        if (ci >= a.n_checks) break;
        const int cc = sld(a.checks + ci);
        const int base = sld(a.chk_ptr + cc);
        uint32_t par = *at_byte(row_ptr(a.synd, cc, ld), (uint32_t)f);
        double m[D];
#pragma unroll
        for (int i = 0; i < D; ++i) {
            const int v = sld(a.chk_var + base + i), e = sld(a.chk_edge + base + i);
            const int vb = sld(a.var_ptr + v), ve = sld(a.var_ptr + v + 1);
            double p = ld_row<false>(row_ptr(a.lappr, v, ld), b8, ld);
            double own = 0.0;
            for (int k = vb; k < ve; ++k) {  // decoder.pyx:292-293, ascending edge id
                const int ek = sld(a.var_edge + k);
                const double c = a.c2v_in ? ld_row<false>(row_ptr(a.c2v_in, ek, ld), b8, ld) : 0.0;
                p += c;
                own = (ek == e) ? c : own;
            }
            if (act && sld(a.var_edge + vb) == e) st_row<false>(row_ptr(a.post, v, ld), b8, ld, p);
            par ^= (p < 0.0) ? 1u : 0u;  // decoder.pyx:243-246
            m[i] = p - own;              // :296-297
        }
        bad |= (par == 1u) ? 1u : 0u;
        if (a.c2v_out) {
            const double s = *at_byte(row_ptr(a.synd, cc, ld), (uint32_t)f) ? -1.0 : 1.0;
            double out[D];
            double *wb = hb + (threadIdx.x >> 6) * kPackWaveDoubles;
            check_strict_packed<D, FIN ? kClampFinite : kClampFull>(m, out, wb, tab, K);
#pragma unroll
            for (int i = 0; i < D; ++i)
                if (act) st_row<false>(row_ptr(a.c2v_out, sld(a.chk_edge + base + i), ld), b8, ld, s * out[i]);
        }
    }
    if (a.unsat_p && bad && act) a.unsat_p[f] = 1;  // benign race: every writer stores 1
}

template <int D>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 8))) k_iter(IterArgs a) {
    __shared__ GlibcTablesBP tab;
    __shared__ double hb[4 * kPackWaveDoubles];
    if (a.c2v_out) stage_glibc_tables(&tab, a.gglibc);
    if (a.finite && sld(a.finite)) iter_block<D, true>(a, blockIdx.x, blockIdx.y, tab, hb);
    else iter_block<D, false>(a, blockIdx.x, blockIdx.y, tab, hb);
}

// ---------------------------------------------------------------------------------------
// Small codes, frame-resident (knob resident, default 1): ONE launch per decode, one
// workgroup per frame for all its iterations, the frame's messages and posteriors in LDS
// (configs[1], reg-(3,6) N=1008: 24 KiB of c2v + 8 KiB of posteriors).  Lane = check in the
// check phase (check c's messages at slots D c .. D c + D - 1: single-degree codes only) and
// lane = variable in the variable phase; each message and posterior is the same operation on
// the same operands as in the frame-parallel kernels (only which lane evaluates it changes),
// so the bits are the reference's.  Per frame the order is decoder.pyx:400-436's:
//   post(0) = lappr (+ 0.0 on connected variables), parity -> stop with (1, 0) and the input;
//   t = 1..max_it: check phase c2v(t) from post(t-1) (+ parity of post(t-1) for t >= 2 ->
//   stop with (1, t-1) and post(t-1)); variable phase post(t) = lappr + sum c2v(t) in
//   ascending edge order;  then parity of post(max_it) -> (1 or 0, max_it).
// A frame stops on its own iteration (no lock-step), no per-iteration launch, no HBM
// traffic for the messages.  In LDS message (c, i) lives at i C + c, so the lanes of a check
// phase (consecutive checks) touch consecutive doubles.  Workgroup b takes frame (b % 8) ceil(B / 8) + b / 8, so the frames
// of one XCD are contiguous columns and their LAPPR sectors stay in that XCD's L2.
constexpr int kResThreads = 512;
constexpr int kResMaxIter = 10000;  // one launch runs every iteration: bound its length
constexpr int kResStaticLds = (int)sizeof(GlibcTablesBP) + (kResThreads / 64) * kPackWaveDoubles * 8;

struct ResArgs {
    int C, V, B, ld, max_it;
    const int32_t *chk_var;              // check CSR: check c's variables at D c .. D c + D - 1
    const int32_t *var_ptr, *var_msg;    // per variable, its edges (ascending) as LDS message indices
    const double *lappr;
    const uint8_t *synd;
    double *post;
    uint8_t *success;
    int32_t *iters;
    const GlibcTables *gglibc;
    double fin_bound;  // |lappr| below it for every variable -> the finite clamp (0: never)
    int dv;            // every variable of degree dv <= 3 and E < 2^16 (0: otherwise)
    int32_t *rsel;     // the workspace's RangeSel block: reset to "never repacked" (repack stats)
    int w0, w1;        // its initial widths
};

// parity of the posteriors in LDS (decoder.pyx:235-257): 1 iff some check of this thread fails
template <int D>
__device__ __forceinline__ uint32_t res_parity(const ResArgs &a, int f, const double *post) {
    uint32_t bad = 0;
    for (int c = threadIdx.x; c < a.C; c += kResThreads) {
        uint32_t par = a.synd[(size_t)c * a.ld + f];
#pragma unroll
        for (int i = 0; i < D; ++i) par ^= (post[a.chk_var[c * D + i]] < 0.0) ? 1u : 0u;
        bad |= (par == 1u) ? 1u : 0u;
    }
    return bad;
}

__device__ __forceinline__ void res_finish(const ResArgs &a, int f, const double *post, int ok, int32_t it) {
    for (int v = threadIdx.x; v < a.V; v += kResThreads) a.post[(size_t)v * a.ld + f] = post[v];
    if (threadIdx.x == 0) {
        a.success[f] = (uint8_t)ok;
        a.iters[f] = it;
    }
}

template <int D, bool FIN>
__device__ __forceinline__ void resident_loop(const ResArgs &a, int f, double *msg, double *post,
                                              const GlibcTablesBP &tab, double *wb) {
    const int tid = threadIdx.x;
    const size_t ld = a.ld;
    const auto K = GlibcK::pinned();
    // the first check of this thread (all of them when C <= kResThreads): its syndrome bit stays
    // in a register across the iterations (its variable indices are re-read from L1: pinning
    // them too spilled with the variable phase's registers below, 907 k vs 911 k frames/s)
    const int c_first = min(tid, a.C - 1);
    const uint8_t sb_first = a.synd[(size_t)c_first * ld + f];
    // the LAPPRs of this lane's (at most two) variables stay in registers when V <= 2 x 512
    // (configs[1]: 1 008), instead of an L2 read per variable per iteration
    const bool lreg = a.V <= 2 * kResThreads;  // block-uniform
    const double l0 = lreg && tid < a.V ? a.lappr[(size_t)tid * ld + f] : 0.0;
    const double l1 = lreg && tid + kResThreads < a.V ? a.lappr[(size_t)(tid + kResThreads) * ld + f] : 0.0;
    // regular variable degree dv <= 3 (configs[1]: 3): the LDS message indices of those two
    // variables' edges too, two 16-bit indices per register, instead of index loads per iteration
    const int dv = lreg ? a.dv : 0;  // block-uniform
    uint32_t vm[3] = {0u, 0u, 0u};
#pragma unroll
    for (int q = 0; q < 3; ++q) {
        if (q < dv) {
            const uint32_t i0 = tid < a.V ? (uint32_t)a.var_msg[tid * dv + q] : 0u;
            const uint32_t i1 = tid + kResThreads < a.V ? (uint32_t)a.var_msg[(tid + kResThreads) * dv + q] : 0u;
            vm[q] = i0 | i1 << 16;
        }
    }
    for (int t = 1; t <= a.max_it; ++t) {
        uint32_t bad = 0;
        for (int c0 = 0; c0 < a.C; c0 += kResThreads) {
            if (c0 + (tid & ~63) >= a.C) break;  // wave-uniform: no check left for this wave
            const int c = c0 + tid;
            const bool live = c < a.C;
            const int cc = live ? c : a.C - 1;  // surplus lanes repeat the last check, store nothing
            const uint8_t sb = c0 == 0 ? sb_first : a.synd[(size_t)cc * ld + f];
            uint32_t par = sb;
            double m[D];
#pragma unroll
            for (int i = 0; i < D; ++i) {
                QR_DCHECK(a.chk_var[cc * D + i] >= 0 && a.chk_var[cc * D + i] < a.V, kDbgResPost, cc, a.chk_var[cc * D + i]);
                QR_DCHECK(i * a.C + cc < a.C * D, kDbgResMsg, cc, i);
                const double p = post[a.chk_var[cc * D + i]];
                par ^= (p < 0.0) ? 1u : 0u;     // decoder.pyx:243-246
                m[i] = p - msg[i * a.C + cc];    // :296-297
            }
            if (live) bad |= (par == 1u) ? 1u : 0u;
            double out[D];
            check_strict_packed<D, FIN ? kClampFinite : kClampFull>(m, out, wb, tab, K);
            const uint32_t smask = sign_mask(sb);
            if (live) {
#pragma unroll
                for (int i = 0; i < D; ++i) msg[i * a.C + cc] = apply_sign(out[i], smask);  // only this lane reads them back
            }
        }
        // the parity of post(t-1) (t = 1: post(0), whose parity is the input's, already tested)
        const int any_bad = __syncthreads_or((int)bad);
        if (t >= 2 && !any_bad) {  // decoder.pyx:431-433 at iteration t-1
            res_finish(a, f, post, 1, t - 1);
            return;
        }
        // decoder.pyx:285-298, two variables per lane at a time: their (latency-bound, L1/L2)
        // LAPPR and index loads are issued together; each sum keeps its ascending edge order
        if (dv) {  // block-uniform: LAPPRs and message indices in registers
            double p0 = l0, p1 = l1;
#pragma unroll
            for (int q = 0; q < 3; ++q) {
                if (q < dv) {
                    QR_DCHECK((vm[q] & 0xFFFFu) < (uint32_t)(a.C * D) && (vm[q] >> 16) < (uint32_t)(a.C * D), kDbgResMsg,
                              vm[q] & 0xFFFFu, vm[q] >> 16);
                    const double m0 = msg[vm[q] & 0xFFFFu], m1 = msg[vm[q] >> 16];
                    p0 += m0;
                    p1 += m1;
                }
            }
            if (tid < a.V) post[tid] = p0;
            if (tid + kResThreads < a.V) post[tid + kResThreads] = p1;
        }
        for (int v0 = dv ? a.V : tid; v0 < a.V; v0 += 2 * kResThreads) {
            const int v1 = v0 + kResThreads;
            const bool two = v1 < a.V;
            const int w1 = two ? v1 : v0;
            double p0 = lreg ? l0 : a.lappr[(size_t)v0 * ld + f];
            double p1 = lreg ? l1 : a.lappr[(size_t)w1 * ld + f];
            const int b0 = a.var_ptr[v0], e0 = a.var_ptr[v0 + 1];
            const int b1 = a.var_ptr[w1], e1 = a.var_ptr[w1 + 1];
            const int n = max(e0 - b0, e1 - b1);
            for (int q = 0; q < n; ++q) {
                const bool h0 = b0 + q < e0, h1 = b1 + q < e1;
                QR_DCHECK(a.var_msg[h0 ? b0 + q : 0] < a.C * D && a.var_msg[h1 ? b1 + q : 0] < a.C * D, kDbgResMsg,
                          a.var_msg[h0 ? b0 + q : 0], a.var_msg[h1 ? b1 + q : 0]);
                const double m0 = msg[a.var_msg[h0 ? b0 + q : 0]];  // (edge 0: an in-bounds dummy)
                const double m1 = msg[a.var_msg[h1 ? b1 + q : 0]];
                if (h0) p0 += m0;
                if (h1) p1 += m1;
            }
            post[v0] = p0;
            if (two) post[v1] = p1;
        }
        __syncthreads();
    }
    const int any_bad = __syncthreads_or((int)res_parity<D>(a, f, post));
    res_finish(a, f, post, any_bad ? 0 : 1, a.max_it);  // decoder.pyx:435-436
}

template <int D>
__global__ void __launch_bounds__(kResThreads) __attribute__((amdgpu_waves_per_eu(4, 8))) k_resident(ResArgs a) {
    extern __shared__ double res_dyn[];
    __shared__ GlibcTablesBP tab;
    __shared__ double hb[(kResThreads / 64) * kPackWaveDoubles];
#if QR_EXPERIMENT_CLOCK
    ClkScope clk(true, g_clk, nullptr);  // every exit below is block-uniform
#endif
    const int q = (a.B + 7) / 8;
    const int f = (int)(blockIdx.x & 7u) * q + (int)(blockIdx.x >> 3);
    // qr_decode_repack_stats after a frame-resident decode: 0 repacks, widths ld/2 (no extra launch)
    if (blockIdx.x == 0 && threadIdx.x < 2 * kSelInts)
        a.rsel[threadIdx.x] = (threadIdx.x % kSelInts == kSelW) ? (threadIdx.x < kSelInts ? a.w0 : a.w1) : 0;
    if (f >= a.B) return;  // block-uniform
    stage_glibc_tables(&tab, a.gglibc);
    const int tid = threadIdx.x;
    const size_t ld = a.ld;
    double *msg = res_dyn, *post = res_dyn + (size_t)a.C * D;
    for (int s = tid; s < a.C * D; s += kResThreads) msg[s] = 0.0;
    bool small = true;
    for (int v = tid; v < a.V; v += kResThreads) {  // decoder.pyx:408,420-421
        const double x = a.lappr[(size_t)v * ld + f];
        small &= __builtin_fabs(x) < a.fin_bound;
        post[v] = (a.var_ptr[v + 1] > a.var_ptr[v]) ? x + 0.0 : x;
    }
    const int fin = __syncthreads_and((int)small);
    // decoder.pyx:400-405: post(0) has the input's signs (only -0.0 -> +0.0 differs)
    if (!__syncthreads_or((int)res_parity<D>(a, f, post))) {
        for (int v = tid; v < a.V; v += kResThreads) a.post[(size_t)v * ld + f] = a.lappr[(size_t)v * ld + f];
        if (tid == 0) {
            a.success[f] = 1;
            a.iters[f] = 0;
        }
        return;
    }
    double *wb = hb + (tid >> 6) * kPackWaveDoubles;
    if (fin) resident_loop<D, true>(a, f, msg, post, tab, wb);
    else resident_loop<D, false>(a, f, msg, post, tab, wb);
}

// One launch = the check sweep of one frame half and the variable sweep of the
// other (they never touch the same frame columns).  The check sweep is VALU heavy
// and the variable sweep HBM bound: interleaving their workgroups (evenly spread
// over the 1-D grid, in proportion to their counts) lets the dispatcher co-schedule
// them on every CU, so the message stream of one hides under the arithmetic of the
// other.
// Occupancy floor (amdgpu_waves_per_eu, MI355X, scripts/exp_build.sh): 4 waves/SIMD = 128
// VGPRs, 5.56 ms per launch vs 5.68 at 5 waves (96 VGPRs); issue-bound on fp64 VALU (the F and
// B chains evaluated side by side for more ILP: no gain).
#ifndef QR_FUSED_STRICT_WAVES
#define QR_FUSED_STRICT_WAVES 4
#endif

template <int D, int MODE, bool NT>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(QR_FUSED_STRICT_WAVES, 8)))
k_fused(CheckArgs ca, VarArgs va, unsigned nb_check, unsigned nb_total) {
    __shared__ GlibcTablesBP tab;
    __shared__ double hb[kPackLdsDoubles];
    const unsigned b = blockIdx.x;
    const unsigned c0 = (unsigned)(((uint64_t)b * nb_check) / nb_total);
    const unsigned c1 = (unsigned)(((uint64_t)(b + 1) * nb_check) / nb_total);
    if (c1 > c0) {  // block-uniform branch
        if (!frames_block_live(ca.acount, c0 / ca.nbx, ca.g.lft)) return;
        if (MODE != kParityOnly) stage_glibc_tables(&tab, ca.gglibc);
        check_block<D, MODE, NT>(ca, c0 % ca.nbx, c0 / ca.nbx, ca.g.per, tab, hb);
    } else {
        const unsigned vi = b - c0;
        if (!frames_block_live(va.acount, vi / va.nbx, va.g.lft)) return;
        var_block<false, NT>(va, vi % va.nbx, vi / va.nbx);
    }
}

// Check degrees above the templated range (2..kMaxTemplDeg) take a runtime-degree kernel
// with no per-lane arrays, so any degree works (the reference sizes its F/B buffer per
// check, decoder.pyx:131-141): the forward values F_0..F_{d-3} of the reference's
// recursion are parked in an HBM scratch laid out like c2v (one row of ld doubles per
// (check, i), frame-innermost, coalesced), and the backward pass re-reads each v2c =
// post - c2v(old) before it overwrites that edge's message:
//   forward  F_0 = m_0, F_i = bp(F_{i-1}, m_i)              (rows i-1 <- F_{i-1})
//   backward c2v[e_{d-1}] = s F_{d-2}; B = m_{d-1};
//            for i = d-2..1: c2v[e_i] = s bp(F_{i-1}, B); B = bp(B, m_i)
//            c2v[e_0] = s B
// (decoder.pyx:322-369: the same box-plus operands in the same order per output.)
constexpr int kMaxTemplDeg = 16;

template <int MODE>
__global__ void __launch_bounds__(256) k_check_generic(CheckArgs a) {
    __shared__ GlibcTablesBP tab;
    select_range(a);
    if (MODE != kParityOnly) stage_glibc_tables(&tab, a.gglibc);
    const int ft = 1 << a.g.lft;
    const int nsub = 256 >> a.g.lft;
    const int ld = a.ld;
    if (!frames_block_live(a.acount, blockIdx.y, a.g.lft)) return;
    bool live;
    const int f = lane_frame(a.alist, a.acount, a.f_off, (int)(blockIdx.y << a.g.lft) + (threadIdx.x & (ft - 1)), live);
    const int sub = __builtin_amdgcn_readfirstlane(threadIdx.x >> a.g.lft);
    if (!live || !a.active[f]) return;
    const auto K = GlibcK::pinned();
    const int64_t c0 = (int64_t)blockIdx.x * a.g.per * nsub + sub;
    const uint32_t b8 = (uint32_t)f * 8u;
    uint32_t bad = 0;
    for (int j = 0; j < a.g.per; ++j) {
        const int64_t ci = c0 + (int64_t)j * nsub;
        if (ci >= a.n_checks) break;
        const int c = sld(a.checks + ci);
        const int base = sld(a.chk_ptr + c);
        const int d = sld(a.chk_ptr + c + 1) - base;
        const uint8_t sb = *at_byte(row_ptr(a.synd, c, ld), (uint32_t)f);
        const double s = sb ? -1.0 : 1.0;
        uint32_t par = sb;
        // v2c of edge i (decoder.pyx:296-297; first sweep: c2v == 0), parity of post
        auto msg = [&](int i, bool count) {
            const double p = *at_byte(row_ptr(a.post, sld(a.chk_var + base + i), ld), b8);
            if (count && MODE != kFirst) par ^= (p < 0.0) ? 1u : 0u;
            return (MODE == kNormal) ? p - *at_byte(row_ptr(a.c2v, sld(a.chk_edge + base + i), ld), b8) : p;
        };
        if (MODE == kParityOnly) {
            for (int i = 0; i < d; ++i) (void)msg(i, true);
            bad |= (par == 1u) ? 1u : 0u;
            continue;
        }
        double *fb = a.fb + (size_t)(a.fb_base + ci * (int64_t)(d - 2)) * ld;
        double F = msg(0, true);
        for (int i = 1; i <= d - 2; ++i) {
            *at_byte(fb + (size_t)(i - 1) * ld, b8) = F;  // F_{i-1}
            F = box_plus_strict(F, msg(i, true), tab, K);
        }
        double Bn = msg(d - 1, true);
        if (MODE != kFirst) bad |= (par == 1u) ? 1u : 0u;
        *at_byte(row_ptr(a.c2v, sld(a.chk_edge + base + d - 1), ld), b8) = s * F;  // s F_{d-2}
        for (int i = d - 2; i >= 1; --i) {
            const double m = msg(i, false);  // before its edge's message is replaced
            const double Fi = *at_byte(fb + (size_t)(i - 1) * ld, b8);
            *at_byte(row_ptr(a.c2v, sld(a.chk_edge + base + i), ld), b8) = s * box_plus_strict(Fi, Bn, tab, K);
            Bn = box_plus_strict(Bn, m, tab, K);
        }
        *at_byte(row_ptr(a.c2v, sld(a.chk_edge + base), ld), b8) = s * Bn;
    }
    if (MODE != kFirst && bad) a.unsat[f] = 1;
}

// rsel: the two ranges' RangeSel (widths w0, w1), initialised here for every schedule.
__global__ void k_init_status(int B, int ld, uint8_t *active, uint8_t *success, int32_t *iters, int32_t *finite,
                              int32_t *rsel, int w0, int w1) {
    const int f = blockIdx.x * blockDim.x + threadIdx.x;
    if (f == 0) *finite = 1;
    if (f < 2 * kSelInts) rsel[f] = (f % kSelInts == kSelW) ? (f < kSelInts ? w0 : w1) : 0;
    if (f >= ld) return;
    active[f] = (f < B) ? 1 : 0;
    if (f < B) {
        success[f] = 0;
        iters[f] = 0;
    }
}

// The frame id of column f: f itself, or fid_w[f] once the range (RangeSel sel, or null) lives
// in the repack work set.
__device__ __forceinline__ const int32_t *range_fid(const int32_t *sel, const int32_t *fid_w) {
    return (sel && sld(sel + kSelOn)) ? fid_w : nullptr;
}

// Frames in [f0, f1) whose posterior after sweep t satisfies the syndrome stop with
// (success=1, iterations=t) (decoder.pyx:431-433, :402-405 for t = 0).  On the
// final call every still-active frame stops with (0, max_iterations) (:435-436).
// sel / fid_w: see range_fid.
__global__ void k_status(int f0, int f1, int t, int final_call, int32_t final_iters,
                         const uint8_t *__restrict__ unsat_t, uint8_t *active, uint8_t *success, int32_t *iters,
                         const int32_t *sel, const int32_t *__restrict__ fid_w) {
    const int f = f0 + blockIdx.x * blockDim.x + threadIdx.x;
    if (f >= f1 || !active[f]) return;
    const int32_t *fid = range_fid(sel, fid_w);
    const int id = fid ? fid[f] : f;
    if (!unsat_t[f]) {
        success[id] = 1;
        iters[id] = t;
        active[f] = 0;
    } else if (final_call) {
        success[id] = 0;
        iters[id] = final_iters;
        active[f] = 0;
    }
}

// The still-running frames of [f0, f1) in ascending order -> list[f0 + 0 .. count).
// One workgroup of 1024 threads: per 1024-frame chunk a wave ballot, the waves' counts
// through LDS, one store per running frame.  STATUS: the status update of sweep t
// (k_status, never the final call) is applied first, frame by frame, by the same thread:
// one launch instead of two between the check sweeps of the two-stream schedule.
// sel / fid_w as k_status (a repacked range holds frames only in its first sel[kSelW] columns).
template <bool STATUS>
__global__ void __launch_bounds__(1024) k_compact(int f0, int f1, uint8_t *__restrict__ active,
                                                  int32_t *__restrict__ list, int32_t *__restrict__ count, int t,
                                                  const uint8_t *__restrict__ unsat_t, uint8_t *__restrict__ success,
                                                  int32_t *__restrict__ iters, const int32_t *sel,
                                                  const int32_t *__restrict__ fid_w) {
    __shared__ int wsum[16];
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int32_t *fid = range_fid(sel, fid_w);
    if (fid) f1 = min(f1, f0 + sld(sel + kSelW));
    int base = 0;  // running count (every thread keeps the same value)
    for (int c0 = f0; c0 < f1; c0 += 1024) {
        const int f = c0 + (int)threadIdx.x;
        bool a = f < f1 && active[f];
        if (STATUS && a && !unsat_t[f]) {  // k_status: satisfied -> (1, t), stops
            const int id = fid ? fid[f] : f;
            success[id] = 1;
            iters[id] = t;
            active[f] = 0;
            a = false;
        }
        const uint64_t m = __ballot(a);
        if (lane == 0) wsum[w] = __popcll(m);
        __syncthreads();
        int off = base, tot = 0;
        for (int i = 0; i < 16; ++i) {
            off += i < w ? wsum[i] : 0;
            tot += wsum[i];
        }
        QR_DCHECK(!a || off + __popcll(m & ((1ull << lane) - 1ull)) <= f - f0, kDbgCompact, off, f - f0);
        if (a) list[f0 + off + __popcll(m & ((1ull << lane) - 1ull))] = f;
        base += tot;
        __syncthreads();  // wsum is rewritten by the next chunk
    }
    if (threadIdx.x == 0) {
        *count = base;
        // the status launch after a range's check sweep: the sweeps of a repack's transition have
        // all run (variable sweep, side and main check sweeps), the list is in the new columns
        if (STATUS && sel) const_cast<int32_t *>(sel)[kSelTransit] = 0;
    }
}

// ---------------------------------------------------------------------------------------
// Column repack of a converging frame range (run_split2, knob repack).  With the active-frame
// lists a sweep's lanes map to the still-running frames, but those frames' columns lie
// scattered over the range: once most frames have stopped, every 8-byte message access of a
// lane is a cache line of its own, and a launch over a few hundred frames costs as much as one
// over the whole range (MI355X, 4-PAM 4.0 dB: 3.7 ms for 418 running frames of 2048, 1.6 ms
// for 76).  The repack moves the running frames' columns to the front of the range, so the
// lanes read contiguous columns again.  Each column copy moves the same bits: the decode's
// arithmetic is untouched.
//
// Everything is decided on the device, so the decode stays asynchronous and capturable: at
// each decision point (before a range's variable sweep, on the variable stream) k_repack_rows
// reads the range's running-frame count (written by its last status launch) and its RangeSel;
// when the running frames fill at most pct % of the range's width w, the range moves to
// w' = max(64, count rounded up to 64):
//   * messages, LAPPRs, syndrome bits: gathered from the range's current column set into the
//     other one of the work set's two (set 0: the workspace's c2v rows + lappr_w[0] / synd_w[0],
//     set 1: c2v_alt + lappr_w[1] / synd_w[1]; the first repack reads the caller's LAPPRs and
//     syndrome bits and the workspace's messages, and writes set 1).  Source and destination
//     never alias, so the moves need no ordering between threads: no barrier, any grid, every
//     load of a thread in flight at once -- the row moves run at copy bandwidth (round 5
//     compacted in place, one barrier per row chunk: 2-3 ms per repack, latency-bound);
//   * posteriors are not moved (the variable sweep right after writes every running frame's
//     posterior in its new column, in the work set's post rows); frames stopped since the last
//     repack first hand theirs to the caller's output through fid (again barrier-free:
//     work set -> output);
//   * fid[column] = the frame the column holds (-1: none), the list becomes the identity, the
//     active flags follow the frames.
// The decision points run on the variable stream beside the other range's check launch, whose
// waves hold 4 x 120 of the 512 VGPRs of a SIMD: the repack waves must fit in the 32 left, or
// their workgroups are dispatched only as check workgroups retire (a first 48-VGPR version waited
// ~0.26 ms per decision point at 4-PAM 4.0 dB).  So each thread's slots (source and destination
// element offsets of a group of rows) are computed once and held in registers for all the row
// groups it moves, and loads and stores are raw buffer accesses off a scalar base.
// Register note (MI355X, measured, mechanism not established): the kernels launched beside the
// check waves (120 VGPRs allocated, 4 per SIMD) must allocate 16 or 32 VGPRs, not 24.  With this
// kernel at 24 (22 used) every dense iteration ran slower, although at a dense iteration it only
// reads two words and exits: headline 9 547 vs 9 790 frames/s (same box, alternating runs), 9 798
// with the round's earlier 28-VGPR version; a variable sweep at 24 (18 used) cost the same
// (9 552 vs 9 776).  So k_repack_rows allocates 32 (an empty asm clobbering v31) and k_var stays
// at 16 (32-bit task arithmetic in its narrow sweep); tests/test_vgpr_budget.py checks both in the
// built code object.
constexpr int kRepackThreads = 256;
constexpr int kRepackPer = 4;  // slots per thread per chunk
constexpr int kRepackChunk = kRepackThreads * kRepackPer;
// workgroups of k_repack_rows: knob repack_grid (default 128: the fewer, the less the moves
// disturb the other range's check launch beside them -- 4.0 dB +0.6 % over 512, 32 too few)

struct RepackArgs {
    int f0, h, ld, pct;  // the range's first column and full width; repack threshold (percent)
    int64_t E, V, C;
    const int32_t *count;  // the range's running-frame count
    int32_t *sel;          // its RangeSel
    int32_t *list;         // active-frame list (absolute columns, list[f0 + p])
    uint8_t *active;
    double *c2v[2];              // message rows of column sets 0 (the workspace's) and 1
    double *out_post;            // the caller's posterior output (frame f at column f)
    const double *lappr_in;      // the caller's LAPPRs
    const uint8_t *synd_in;      // the caller's syndrome bits
    double *post_w;              // the work set's posteriors
    double *lappr_w[2];          // its LAPPRs and syndrome bits, column sets 0 and 1
    uint8_t *synd_w[2];
    int32_t *fid_w;
};

// The decision, taken identically by every workgroup of k_repack_rows.
__device__ __forceinline__ bool repack_go(const RepackArgs &r, int &cnt, int &w, int &w_new) {
    cnt = sld(r.count);
    w = sld(r.sel + kSelW);
    if (w <= 64 || cnt <= 0 || (int64_t)cnt * 100 > (int64_t)w * r.pct) return false;
    w_new = max(64, (cnt + 63) / 64 * 64);
    return w_new < w;
}

// make every load of this thread complete, then the workgroup barrier: the loaded values are
// in registers before any thread of the workgroup overwrites what they were loaded from
__device__ __forceinline__ void loads_done_barrier() {
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
}

// Raw buffer access to a run of rows of a frame-innermost array (base in scalar registers, the
// lane's byte offset in a VGPR): an offset past the run reads 0 and drops the store, so empty slots
// need no branch.
template <typename T>
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const T *p, int bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<T *>(p), (short)0, bytes, 0x00020000);
}
__device__ __forceinline__ double rb_load(__amdgpu_buffer_rsrc_t r, uint32_t off, double) {
    return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 0));
}
__device__ __forceinline__ uint8_t rb_load(__amdgpu_buffer_rsrc_t r, uint32_t off, uint8_t) {
    return __builtin_amdgcn_raw_buffer_load_b8(r, off, 0, 0);
}
__device__ __forceinline__ void rb_store(__amdgpu_buffer_rsrc_t r, uint32_t off, double v) {
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(qr_u32x2, v), r, off, 0, 0);
}
__device__ __forceinline__ void rb_store(__amdgpu_buffer_rsrc_t r, uint32_t off, uint8_t v) {
    __builtin_amdgcn_raw_buffer_store_b8(v, r, off, 0, 0);
}

// Gather the columns of this thread's slots from rows [0, n) of src into dst, row groups of rg
// rows walked grid-stride by the workgroups: slot u of a group = (row j < rg of the group, one
// column); src_el / dst_el: its byte offsets inside a group of double rows (8 (j ld + column)),
// kRepackNone for an empty slot (a byte row group shifts them right by 3; an empty slot's offset
// stays past the group either way).  src and dst never alias (two column sets, or work set ->
// output), so there is no ordering to keep.
constexpr uint32_t kRepackNone = 0xFFFFFFF0u;  // past any group: loads 0, stores nothing
template <typename TS, typename TD>
__device__ __forceinline__ void gather_rows(const TS *src, TD *dst, int64_t n, int ld, int dst_ld, int rg,
                                            const uint32_t (&src_el)[kRepackPer],
                                            const uint32_t (&dst_el)[kRepackPer]) {
    constexpr int sh = sizeof(TS) == 8 ? 0 : 3;
    // two row groups per step: the loads of both are in flight together (the moves are bound by
    // the memory round trip of each step, not by bandwidth)
    const int64_t stride = (int64_t)gridDim.x * rg;
    for (int64_t g0 = (int64_t)blockIdx.x * rg; g0 < n; g0 += 2 * stride) {
        const int64_t g1 = g0 + stride;
        const int n0 = (int)min<int64_t>(rg, n - g0);                       // block-uniform
        const int n1 = g1 < n ? (int)min<int64_t>(rg, n - g1) : 0;          // (0: no second group)
        const auto s0 = make_rsrc(src + (size_t)g0 * ld, n0 * ld * (int)sizeof(TS));
        const auto d0 = make_rsrc(dst + (size_t)g0 * dst_ld, n0 * dst_ld * (int)sizeof(TD));
        const auto s1 = make_rsrc(src + (size_t)(n1 ? g1 : g0) * ld, n1 * ld * (int)sizeof(TS));
        const auto d1 = make_rsrc(dst + (size_t)(n1 ? g1 : g0) * dst_ld, n1 * dst_ld * (int)sizeof(TD));
        TS v0[kRepackPer], v1[kRepackPer];
#if QR_DEBUG_ASSERT
        // a slot lies inside a full group of rg rows (slots of rows j >= n0 in the last, short group
        // fall past the buffer's range by design: their loads read 0, their stores are dropped)
        for (int u = 0; u < kRepackPer; ++u) {
            QR_DCHECK(src_el[u] == kRepackNone || (src_el[u] >> sh) < (uint32_t)(rg * ld * (int)sizeof(TS)), kDbgRepackSlot,
                      src_el[u], n0);
            QR_DCHECK(dst_el[u] == kRepackNone || (dst_el[u] >> sh) < (uint32_t)(rg * dst_ld * (int)sizeof(TD)),
                      kDbgRepackSlot, dst_el[u], n0);
        }
#endif
#pragma unroll
        for (int u = 0; u < kRepackPer; ++u) v0[u] = rb_load(s0, src_el[u] >> sh, TS(0));
#pragma unroll
        for (int u = 0; u < kRepackPer; ++u) v1[u] = rb_load(s1, src_el[u] >> sh, TS(0));
#pragma unroll
        for (int u = 0; u < kRepackPer; ++u) rb_store(d0, dst_el[u] >> sh, v0[u]);
#pragma unroll
        for (int u = 0; u < kRepackPer; ++u) rb_store(d1, dst_el[u] >> sh, v1[u]);
    }
}

// The commit of a repack (by the workgroup of k_repack_rows that finishes last): frame ids, active
// flags and the RangeSel (now in column set nb, in transit).  The list keeps the frames' old
// columns: the transition sweeps read the messages there; the next status launch rebuilds it.
__device__ __forceinline__ void repack_commit(const RepackArgs &r, int cnt, int w, int w_new, bool on, int nb) {
    const int f0 = r.f0;
    for (int p0 = 0; p0 < cnt; p0 += kRepackThreads) {
        const int p = p0 + (int)threadIdx.x;
        int id = 0;
        if (p < cnt) {
            const int sc = r.list[f0 + p];
            id = on ? r.fid_w[sc] : sc;  // column = frame in the caller's arrays
            QR_DCHECK(sc >= f0 + p && sc < f0 + w && id >= 0 && id < r.ld, kDbgRepackFid, sc, id);
        }
        loads_done_barrier();  // fid_w is compacted in place: every read of this chunk first
        if (p < cnt) {
            r.fid_w[f0 + p] = id;
            r.active[f0 + p] = 1;
        }
    }
    for (int p = cnt + (int)threadIdx.x; p < w; p += kRepackThreads) {
        r.fid_w[f0 + p] = -1;
        r.active[f0 + p] = 0;
    }
    if (threadIdx.x == 0) {
        r.sel[kSelOn] = 1;
        r.sel[kSelW] = w_new;
        r.sel[kSelRepacks] += 1;
        r.sel[kSelArrive] = 0;
        r.sel[kSelBuf] = nb;
        r.sel[kSelTransit] = 1;
    }
}

// The row moves of a repack.  Posteriors are not moved: the range's variable sweep right after
// rewrites every running frame's posterior in its new column; only the frames stopped since the
// last repack hand theirs (in the work set) to the output first.
__global__ void __launch_bounds__(kRepackThreads) k_repack_rows(RepackArgs r) {
    int cnt, w, w_new;
    // allocate 32 VGPRs (the code needs fewer): see the register note above
    __asm__ volatile("" ::: "v31");
    if (!repack_go(r, cnt, w, w_new)) return;  // kernel-uniform
    const bool on = sld(r.sel + kSelOn) != 0;
    const int b = on ? sld(r.sel + kSelBuf) : 0, nb = on ? 1 - b : 1;  // source / destination column set
    const int ld = r.ld, f0 = r.f0;
    if (on) {
        // frames stopped since the last repack (a column < w with a frame id, no longer active)
        // hand their posteriors to the output: slots (row j of rg, column q < w)
        const int rg = w <= kRepackChunk / 2 ? min(16, kRepackChunk / w) : 1;
        for (int q0 = 0; q0 < w; q0 += kRepackChunk) {
            const int qc = min(w - q0, kRepackChunk);
            uint32_t src_el[kRepackPer], dst_el[kRepackPer];
#pragma unroll
            for (int u = 0; u < kRepackPer; ++u) {
                const int sl = u * kRepackThreads + (int)threadIdx.x;
                const int j = sl / qc, q = q0 + sl - j * qc;
                const int id = j < rg ? r.fid_w[f0 + q] : -1;
                const bool go = id >= 0 && !r.active[f0 + q];
                QR_DCHECK(id < ld, kDbgRepackFid, id, q);
                src_el[u] = go ? (uint32_t)(j * ld + f0 + q) * 8u : kRepackNone;
                dst_el[u] = go ? (uint32_t)(j * ld + id) * 8u : kRepackNone;
            }
            gather_rows<double, double>(r.post_w, r.out_post, r.V, ld, ld, rg, src_el, dst_el);
        }
    }
    // a small count moves several rows per group: rg rows x cnt columns fill the slots
    const int rg = cnt <= kRepackChunk / 2 ? min(16, kRepackChunk / cnt) : 1;
    for (int p0 = 0; p0 < cnt; p0 += kRepackChunk) {
        const int pc = min(cnt - p0, kRepackChunk);  // columns of this chunk (rg = 1 unless one chunk)
        uint32_t src_el[kRepackPer], dst_el[kRepackPer];
#pragma unroll
        for (int u = 0; u < kRepackPer; ++u) {
            const int sl = u * kRepackThreads + (int)threadIdx.x;
            const int j = sl / pc, q = sl - j * pc;
            const bool ok = j < rg;
            QR_DCHECK(!ok || (r.list[f0 + p0 + q] >= f0 + p0 + q && r.list[f0 + p0 + q] < f0 + w), kDbgRepackList,
                      r.list[f0 + p0 + q], f0 + p0 + q);
            src_el[u] = ok ? (uint32_t)(j * ld + r.list[f0 + p0 + q]) * 8u : kRepackNone;
            dst_el[u] = ok ? (uint32_t)(j * ld + f0 + p0 + q) * 8u : kRepackNone;
        }
        // source set b, destination set nb (selects, not dynamic indices into the kernel arguments);
        // the messages are not moved here: the transition sweeps read them at the old columns
        gather_rows<double, double>(!on ? r.lappr_in : b ? r.lappr_w[1] : r.lappr_w[0], nb ? r.lappr_w[1] : r.lappr_w[0],
                                    r.V, ld, ld, rg, src_el, dst_el);
        gather_rows<uint8_t, uint8_t>(!on ? r.synd_in : b ? r.synd_w[1] : r.synd_w[0], nb ? r.synd_w[1] : r.synd_w[0],
                                      r.C, ld, ld, rg, src_el, dst_el);
    }
    // the workgroup that arrives last commits: every other one has read the list, frame ids and
    // active flags it needed (its loads completed before its arrival), so the commit's rewrites of
    // them race with nothing; the next launches see everything (kernel boundary)
    __shared__ int last;
    loads_done_barrier();
    if (threadIdx.x == 0) last = atomicAdd(r.sel + kSelArrive, 1) == (int)gridDim.x - 1;
    __syncthreads();
    if (last) repack_commit(r, cnt, w, w_new, on, nb);
}


// The range's final width is known only here, so the work is (row, 64-column chunk) units, one
// per wave, walked grid-stride by every wave of the grid: a narrow range (the usual end of a
// converging one) still gets the whole grid (one unit per wave, rows in parallel).
__global__ void __launch_bounds__(256) k_repack_output(int64_t rows, int f0, int ld, const int32_t *sel,
                                                       const int32_t *__restrict__ fid_w,
                                                       const double *__restrict__ post_w, double *__restrict__ out_post) {
    if (!sld(sel + kSelOn)) return;  // kernel-uniform: never repacked (the output is the posteriors)
    const int w = sld(sel + kSelW);
    const int nq = (w + 63) >> 6;
    const int lane = (int)(threadIdx.x & 63u);
    const int64_t nwaves = (int64_t)gridDim.x * (blockDim.x >> 6), units = rows * nq;
    for (int64_t u = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); u < units; u += nwaves) {
        const int64_t v = u / nq;
        const int q = (int)(u - v * nq) * 64 + lane;
        const int id = q < w ? fid_w[f0 + q] : -1;
        if (id < 0) continue;
        QR_DCHECK(id < ld, kDbgRepackFid, id, q);
        out_post[(size_t)v * ld + id] = post_w[(size_t)v * ld + f0 + q];
    }
}

// ------------------------------------------------------------------ launch
struct DecodeWs {
    double *c2v;
    double *c2v2;    // the second message buffer of the fused small-code schedule (run_iter), or null
    uint8_t *active;
    uint8_t *unsat;  // (max_it + 2) rows of ld flags
    double *fb;      // F scratch of the runtime-degree classes (fb_rows rows of ld), or null
    int32_t *alist;  // active-frame lists of the frame ranges (ld entries)
    int32_t *acount; // their lengths: [0] range starting at frame 0, [1] the second half;
                     // [2] the finite flag of the input LAPPRs (first variable sweep);
                     // [4, 16) the two ranges' RangeSel (rsel)
    int32_t *rsel;
    // the work set of the column repack (k_repack_rows, run_split2): posteriors and the frame id
    // of each column of the repacked ranges, and two column sets of LAPPRs and syndrome bits (and
    // of messages: set 0 is c2v above, set 1 c2v_alt) that consecutive repacks gather into in
    // turn; present when the caller's workspace has room for it (ws_bytes counts it when knob
    // repack is on)
    struct WorkSet {
        double *post;
        double *lappr[2];
        uint8_t *synd[2];
        double *c2v_alt;
        int32_t *fid;
    } rs;
    bool repack;
};

// Codes the one-launch-per-iteration schedule (k_iter) can run: one check-degree class of a
// packed degree, bounded variable degrees, and messages small enough to double-buffer.
static bool iter_code(const qr_code *code, int ld) {
    return code->classes.size() == 1 && code->classes[0].degree >= 2 && code->classes[0].degree <= kPackMaxDeg &&
           code->max_dv <= 64 && (size_t)code->E * ld * sizeof(double) <= ((size_t)1 << 30);
}

static size_t ws_base_bytes(const qr_code *code, int ld, int max_it) {
    const int64_t rows = (int64_t)(max_it > 0 ? max_it : 0) + 2;  // no int overflow at INT_MAX
    const size_t msg = align_up((size_t)code->E * ld * sizeof(double), 256);
    return msg + (iter_code(code, ld) ? msg : 0) + align_up((size_t)ld, 256) +
           align_up((size_t)rows * ld, 256) + align_up((size_t)code->fb_rows * ld * sizeof(double), 256) +
           align_up((size_t)ld * sizeof(int32_t), 256) + 256;
}
static size_t repack_set_bytes(const qr_code *code, int ld) {
    return 3 * align_up((size_t)code->V * ld * sizeof(double), 256) + 2 * align_up((size_t)code->C * ld, 256) +
           align_up((size_t)code->E * ld * sizeof(double), 256) + align_up((size_t)ld * sizeof(int32_t), 256);
}
static size_t ws_repack_bytes(const qr_code *code, int ld);  // after g_tune
static size_t ws_bytes(const qr_code *code, int ld, int max_it) {
    return ws_base_bytes(code, ld, max_it) + ws_repack_bytes(code, ld);
}

static DecodeWs carve(const qr_code *code, int ld, int max_it, void *base, size_t ws_size) {
    DecodeWs w;
    char *p = (char *)base;
    const int64_t rows = (int64_t)(max_it > 0 ? max_it : 0) + 2;  // no int overflow at INT_MAX
    w.c2v = (double *)p;
    p += align_up((size_t)code->E * ld * sizeof(double), 256);
    w.c2v2 = nullptr;
    if (iter_code(code, ld)) {
        w.c2v2 = (double *)p;
        p += align_up((size_t)code->E * ld * sizeof(double), 256);
    }
    w.active = (uint8_t *)p;
    p += align_up((size_t)ld, 256);
    w.unsat = (uint8_t *)p;
    p += align_up((size_t)rows * ld, 256);
    w.fb = code->fb_rows ? (double *)p : nullptr;
    p += align_up((size_t)code->fb_rows * ld * sizeof(double), 256);
    w.alist = (int32_t *)p;
    p += align_up((size_t)ld * sizeof(int32_t), 256);
    w.acount = (int32_t *)p;
    w.rsel = w.acount + 4;
    p += 256;
    const size_t extra = ws_repack_bytes(code, ld);
    w.repack = extra > 0 && ws_size >= ws_base_bytes(code, ld, max_it) + extra;
    w.rs = DecodeWs::WorkSet{nullptr, {nullptr, nullptr}, {nullptr, nullptr}, nullptr, nullptr};
    if (w.repack) {
        w.rs.post = (double *)p;
        p += align_up((size_t)code->V * ld * sizeof(double), 256);
        for (int k = 0; k < 2; ++k) {
            w.rs.lappr[k] = (double *)p;
            p += align_up((size_t)code->V * ld * sizeof(double), 256);
            w.rs.synd[k] = (uint8_t *)p;
            p += align_up((size_t)code->C * ld, 256);
        }
        w.rs.c2v_alt = (double *)p;
        p += align_up((size_t)code->E * ld * sizeof(double), 256);
        w.rs.fid = (int32_t *)p;
    }
    return w;
}

// Runtime tuning knobs (qr_tune_set); defaults picked by scripts/tune.py on MI355X.
struct Tuning {
    std::atomic<int> check_ft{128}, check_per{16}, var_ft{128}, var_per{8}, nt{1}, split{3},
        lds_pad_kb{0}, compact{1}, side{1}, min_blocks{2048}, split_min_blocks{1024}, var_pace{28},
        check_tail{4}, fused_iter{1}, iter_streams{2}, var_boost{4}, resident{1}, repack{1},
        repack_pct{80}, repack_grid{128};
};
static Tuning g_tune;

// knob repack (default 1): the workspace carries the work set of the repacked ranges when the
// two-stream schedule can run (ld % 512 == 0) and the set takes at most 1/8 of the device's
// memory (N=64800, ld=4096: 4.4 GB of 288 GB)
static size_t ws_repack_bytes(const qr_code *code, int ld) {
    if (!g_tune.repack.load() || ld % 512) return 0;
    const size_t b = repack_set_bytes(code, ld);
    return b <= code->mem_bytes / 8 ? b : 0;
}

// Frame tile ft (a divisor of ncols, <= ft_req) and nodes per thread.  Small problems (few
// nodes x few frame tiles, e.g. the reg-(3,6) N=1008 code of configs[1]) get fewer nodes per
// thread, down to 1, so that a launch still has ~min_blocks workgroups to spread over the
// 256 CUs (knob min_blocks, 0 = off); the DVB-S2 launches keep their per.
static Geom make_geom(int ncols, int ft_req, int per, int64_t nodes = 0) {
    int ft = 256;
    while (ft > 64 && (ft > ft_req || ncols % ft)) ft >>= 1;
    int lft = 6;
    while ((1 << lft) < ft) ++lft;
    per = per < 1 ? 1 : per;
    const int64_t target = g_tune.min_blocks.load();
    if (nodes > 0 && target > 0) {
        const int64_t tiles = ncols >> lft, nsub = 256 >> lft;
        const int64_t fit = nodes * tiles / (target * nsub);   // per that gives ~target blocks
        if (fit < per) per = (int)(fit < 1 ? 1 : fit);
    }
    return Geom{lft, per};
}

// Everything one decode call needs to issue its launches.
struct Plan {
    const qr_code *code;
    int B, ld;
    const double *lappr;
    const uint8_t *synd;
    double *post;
    uint8_t *success;
    int32_t *iters;
    DecodeWs w;
    bool nt;
    hipStream_t s;
    int lds_pad = 0;  // dynamic LDS reserved by each check workgroup (caps their CU residency)
    bool compact = false;  // sweeps of the main loop read the active-frame lists
    int var_pace = 0;      // variable sweeps: workgroups per 128 frames (0 = one per tile)
    // run_split2 with the device-steered column repack: every launch of a range carries the
    // range's RangeSel (steer); parity-only sweeps read the active-frame lists too (list_parity:
    // the final sweep)
    bool steer = false;
    bool list_parity = false;

    const int32_t *count_of(int f0) const { return w.acount + (f0 == 0 ? 0 : 1); }
    const int32_t *sel_of(int f0) const { return steer ? w.rsel + (f0 == 0 ? 0 : kSelInts) : nullptr; }

    CheckArgs check_args(const DegreeClass &cls, const double *post_in, uint8_t *unsat, int f0, int f1) const {
        CheckArgs a;
        a.checks = cls.d_checks;
        a.n_checks = cls.n;
        a.chk_ptr = code->d_chk_ptr;
        a.chk_edge = code->d_chk_edge;
        a.chk_var = code->d_chk_var;
        a.post = post_in;
        a.c2v = w.c2v;
        a.synd = synd;
        a.active = w.active;
        a.unsat = unsat;
        a.ld = ld;
        a.f_off = f0;
        a.g = make_geom(f1 - f0, g_tune.check_ft.load(), g_tune.check_per.load(), cls.n);
        const int64_t per_block = (int64_t)a.g.per * (256 >> a.g.lft);
        a.nbx = (unsigned)((cls.n + per_block - 1) / per_block);
        a.gglibc = code->d_gtab;
        a.fb = w.fb;
        a.fb_base = cls.fb_base;
        a.alist = a.acount = nullptr;
        a.finite = w.acount + 2;
        a.nmain = 0;
        a.per_t = a.g.per;
        a.sel = sel_of(f0);
        a.post_w = w.rs.post;
        a.synd_w[0] = w.rs.synd[0];
        a.synd_w[1] = w.rs.synd[1];
        a.c2v_alt = w.rs.c2v_alt;
        a.transit = 0;
        a.c2v_rd = a.c2v;
        return a;
    }
    VarArgs var_args(int f0, int f1) const {
        VarArgs a;
        a.V = code->V;
        a.var_ptr = code->d_var_ptr;
        a.var_edge = code->d_var_edge;
        a.lappr = lappr;
        a.c2v = w.c2v;
        a.post = post;
        a.active = w.active;
        a.ld = ld;
        a.f_off = f0;
        a.g = make_geom(f1 - f0, g_tune.var_ft.load(), g_tune.var_per.load(), code->V);
        const int64_t per_block = (int64_t)a.g.per * (256 >> a.g.lft);
        a.nbx = (unsigned)((code->V + per_block - 1) / per_block);
        a.alist = a.acount = nullptr;
        a.nby = (unsigned)((f1 - f0) >> a.g.lft);
        a.gs = 0;
        a.boost = 1;
        a.finite = nullptr;
        a.fin_bound = 0.0;
        a.fin_B = 0;
        a.sel = sel_of(f0);
        a.lappr_w[0] = w.rs.lappr[0];
        a.lappr_w[1] = w.rs.lappr[1];
        a.post_w = w.rs.post;
        a.c2v_alt = w.rs.c2v_alt;
        a.transit = 0;
        return a;
    }
};

// Dispatch a templated launch on the check degree (2..16); `handled` is false otherwise.
#define QR_DEG_SWITCH(DEG, CASE, handled)                                                                    \
    switch (DEG) {                                                                                           \
        CASE(2) CASE(3) CASE(4) CASE(5) CASE(6) CASE(7) CASE(8) CASE(9) CASE(10) CASE(11) CASE(12) CASE(13) \
        CASE(14) CASE(15) CASE(16)                                                                           \
        default: handled = false;                                                                            \
    }

template <int MODE, bool NT>
static int launch_check_class(const Plan &P, const DegreeClass &cls, const double *post_in, uint8_t *unsat, int f0,
                              int f1) {
    CheckArgs a = P.check_args(cls, post_in, unsat, f0, f1);
    if (P.compact && (MODE != kParityOnly || P.list_parity)) {
        a.alist = P.w.alist;
        a.acount = P.count_of(f0);
    }
    const dim3 grid2(a.nbx, (unsigned)((f1 - f0) >> a.g.lft));   // the plain 2-D grid
    dim3 grid = grid2;
    // knob check_tail (default 4; 0 = off; MI355X: +1 %): frame tile 0 is swept last with per / check_tail
    // checks per thread (the templated degrees only; the runtime-degree kernel keeps the 2-D grid)
    const int tail = g_tune.check_tail.load();
    const bool templ = cls.degree >= 2 && cls.degree <= kMaxTemplDeg;
    if (tail > 1 && grid.y >= 2 && templ && a.g.per >= tail) {
        const int64_t per_block_t = (int64_t)(a.g.per / tail) * (256 >> a.g.lft);
        const int64_t nbx_t = (cls.n + per_block_t - 1) / per_block_t;
        a.nmain = a.nbx * (grid.y - 1);
        a.per_t = a.g.per / tail;
        grid = dim3((unsigned)(a.nmain + nbx_t), 1);
    }
    ProfScope ps(profiling_on() ? std::string(MODE == kParityOnly ? "parity_d" : MODE == kFirst ? "check1_d" : "check_d") +
                                      std::to_string(cls.degree)
                                : std::string(),
                 P.s);
#define QR_CASE(DD)                                                                                   \
    case DD:                                                                                          \
        k_check<DD, MODE, NT><<<grid, 256, P.lds_pad, P.s>>>(a);                                     \
        break;
    bool handled = true;
    QR_DEG_SWITCH(cls.degree, QR_CASE, handled)
#undef QR_CASE
    if (!handled) {  // the runtime-degree kernel decodes its frame tile from blockIdx.y: 2-D grid only
        a.nmain = 0;
        a.per_t = a.g.per;
        k_check_generic<MODE><<<grid2, 256, 0, P.s>>>(a);
    }
    QR_LAUNCH_CHECK();
    return QR_OK;
}

// Check sweep of frames [f0, f1) over every degree class except `skip` (index or -1).
template <int MODE>
static int launch_checks(const Plan &P, const double *post_in, uint8_t *unsat, int f0, int f1, int skip = -1) {
    for (int k = 0; k < (int)P.code->classes.size(); ++k) {
        if (k == skip) continue;
        const DegreeClass &cls = P.code->classes[k];
        int rc = P.nt ? launch_check_class<MODE, true>(P, cls, post_in, unsat, f0, f1)
                      : launch_check_class<MODE, false>(P, cls, post_in, unsat, f0, f1);
        if (rc) return rc;
    }
    return QR_OK;
}

template <bool INIT>
static int launch_var(const Plan &P, int f0, int f1, int32_t *finite = nullptr, double fin_bound = 0.0) {
    ProfScope ps(INIT ? "var_init" : "var", P.s);
    VarArgs a = P.var_args(f0, f1);
    a.finite = finite;
    a.fin_bound = fin_bound;
    a.fin_B = P.B;
    if (P.compact && !INIT) {
        a.alist = P.w.alist;
        a.acount = P.count_of(f0);
    }
    dim3 grid(a.nbx, a.nby);
    // Paced sweep (the two-stream schedule's variable sweeps, Plan::var_pace): at most var_pace
    // workgroups per 128 frames of the sweep, each walking its tiles grid-stride, so that the sweep streams its
    // bytes over about the length of the concurrent check sweep instead of saturating HBM for
    // the first ~40 % of it.
    const int64_t cap = (int64_t)P.var_pace * (((int64_t)a.nby << a.g.lft) / 128);  // per 128 frames
    if (cap > 0 && (int64_t)a.nbx * a.nby > cap) {
        a.gs = 1;
        // knob var_boost (default 4, 1 = off): the sweep widens as the live tiles drop
        a.boost = std::max(1, std::min(g_tune.var_boost.load(), 16));
        grid = dim3((unsigned)(cap * a.boost), 1);
    }
    if (P.nt) k_var<INIT, true><<<grid, 256, 0, P.s>>>(a);
    else k_var<INIT, false><<<grid, 256, 0, P.s>>>(a);
    QR_LAUNCH_CHECK();
    return QR_OK;
}

template <int MODE, bool NT>
static int launch_fused_nt(const Plan &P, const DegreeClass &cls, uint8_t *unsat, int cf0, int cf1, int vf0, int vf1) {
    CheckArgs ca = P.check_args(cls, P.post, unsat, cf0, cf1);
    VarArgs va = P.var_args(vf0, vf1);
    if (P.compact) {
        ca.alist = va.alist = P.w.alist;
        ca.acount = P.count_of(cf0);
        va.acount = P.count_of(vf0);
    }
    const unsigned nbc = ca.nbx * (unsigned)((cf1 - cf0) >> ca.g.lft);
    const unsigned nbv = va.nbx * (unsigned)((vf1 - vf0) >> va.g.lft);
    bool handled = true;
    {
        ProfScope ps(profiling_on() ? std::string("fused_d") + std::to_string(cls.degree) : std::string(), P.s);
#define QR_CASE(DD)                                                                           \
    case DD:                                                                                  \
        k_fused<DD, MODE, NT><<<nbc + nbv, 256, 0, P.s>>>(ca, va, nbc, nbc + nbv);            \
        break;
        QR_DEG_SWITCH(cls.degree, QR_CASE, handled)
#undef QR_CASE
    }
    if (!handled) {  // runtime degree: the two sweeps as plain launches (disjoint frame columns)
        int rc = launch_check_class<MODE, NT>(P, cls, P.post, unsat, cf0, cf1);
        return rc ? rc : launch_var<false>(P, vf0, vf1);
    }
    QR_LAUNCH_CHECK();
    return QR_OK;
}

template <int MODE>
static int launch_fused(const Plan &P, const DegreeClass &cls, uint8_t *unsat, int cf0, int cf1, int vf0, int vf1) {
    return P.nt ? launch_fused_nt<MODE, true>(P, cls, unsat, cf0, cf1, vf0, vf1)
                : launch_fused_nt<MODE, false>(P, cls, unsat, cf0, cf1, vf0, vf1);
}

static int launch_status(const Plan &P, int f0, int f1, int t, int final_call, int32_t final_iters,
                         const uint8_t *unsat_t) {
    ProfScope ps("status", P.s);
    f1 = std::min(f1, P.B);
    if (f1 <= f0) return QR_OK;
    k_status<<<(f1 - f0 + 255) / 256, 256, 0, P.s>>>(f0, f1, t, final_call, final_iters, unsat_t, P.w.active,
                                                     P.success, P.iters, P.sel_of(f0), P.w.rs.fid);
    QR_LAUNCH_CHECK();
    return QR_OK;
}

// Rebuild the active-frame list of [f0, f1) after a status update (no-op without compaction).
static int launch_compact(const Plan &P, int f0, int f1) {
    if (!P.compact) return QR_OK;
    k_compact<false><<<1, 1024, 0, P.s>>>(f0, f1, P.w.active, P.w.alist, const_cast<int32_t *>(P.count_of(f0)), 0,
                                          nullptr, nullptr, nullptr, P.sel_of(f0), P.w.rs.fid);
    QR_LAUNCH_CHECK();
    return QR_OK;
}

// Status update of sweep t (not the final call) + list rebuild of [f0, f1): one launch with
// compaction, k_status alone without.
static int launch_status_compact(const Plan &P, int f0, int f1, int t, const uint8_t *unsat_t) {
    if (!P.compact) return launch_status(P, f0, f1, t, 0, 0, unsat_t);
    ProfScope ps("status", P.s);
    k_compact<true><<<1, 1024, 0, P.s>>>(f0, f1, P.w.active, P.w.alist, const_cast<int32_t *>(P.count_of(f0)), t,
                                         unsat_t, P.success, P.iters, P.sel_of(f0), P.w.rs.fid);
    QR_LAUNCH_CHECK();
    return QR_OK;
}

// Flooding schedule, all frames in lock-step (decoder.pyx:424-433).
static int run_flat(const Plan &P, int max_it) {
    const int ld = P.ld;
    int rc;
    for (int t = 1; t <= max_it; ++t) {
        uint8_t *unsat_prev = P.w.unsat + (size_t)(t - 1) * ld;
        if (t == 1) {
            if ((rc = launch_checks<kFirst>(P, P.post, unsat_prev, 0, ld))) return rc;
        } else {
            if ((rc = launch_checks<kNormal>(P, P.post, unsat_prev, 0, ld))) return rc;
            if ((rc = launch_status_compact(P, 0, ld, t - 1, unsat_prev))) return rc;
        }
        if ((rc = launch_var<false>(P, 0, ld))) return rc;
    }
    return QR_OK;
}

// The same per-frame schedule with the batch split in two frame halves A | B
// whose sweeps are software-pipelined half an iteration apart:
//   C_A(1); for t: [V_A(t) | C_B(t)], S_B(t-1), [C_A(t+1) | V_B(t)], S_A(t)
// C = check sweep (+ parity of the previous posteriors), S = status update,
// V = variable sweep, [x | y] = one k_fused launch.  Per frame the order
// C(t) -> S(t-1) -> V(t) -> C(t+1) is exactly that of run_flat.
static int run_split(const Plan &P, int max_it) {
    const int ld = P.ld, h = ld / 2;
    const int A0 = 0, A1 = h, B0 = h, B1 = ld;
    int big = 0;
    for (int k = 1; k < (int)P.code->classes.size(); ++k)
        if (P.code->classes[k].n > P.code->classes[big].n) big = k;
    const DegreeClass &cls = P.code->classes[big];
    auto row = [&](int t) { return P.w.unsat + (size_t)t * ld; };
    int rc;
    // C_A(1)
    if ((rc = launch_checks<kFirst>(P, P.post, row(0), A0, A1))) return rc;
    for (int t = 1; t <= max_it; ++t) {
        // [V_A(t) | C_B(t)]   (the other degree classes of C_B(t) as plain launches)
        if (t == 1) {
            if ((rc = launch_checks<kFirst>(P, P.post, row(0), B0, B1, big))) return rc;
            if ((rc = launch_fused<kFirst>(P, cls, row(0), B0, B1, A0, A1))) return rc;
        } else {
            if ((rc = launch_checks<kNormal>(P, P.post, row(t - 1), B0, B1, big))) return rc;
            if ((rc = launch_fused<kNormal>(P, cls, row(t - 1), B0, B1, A0, A1))) return rc;
            if ((rc = launch_status_compact(P, B0, B1, t - 1, row(t - 1)))) return rc;
        }
        if (t < max_it) {
            // [C_A(t+1) | V_B(t)]
            if ((rc = launch_checks<kNormal>(P, P.post, row(t), A0, A1, big))) return rc;
            if ((rc = launch_fused<kNormal>(P, cls, row(t), A0, A1, B0, B1))) return rc;
            if ((rc = launch_status_compact(P, A0, A1, t, row(t)))) return rc;
        } else {
            if ((rc = launch_var<false>(P, B0, B1))) return rc;
        }
    }
    return QR_OK;
}

// run_split's per-frame order with the check and variable sweeps of the two halves
// as separate kernels on two streams (split = 3): the caller's stream s runs the
// check sweeps and status updates, s2 the variable sweeps, events order them:
//   s : C_A(1) | [wait vB] C_B(t) S_B(t-1) | [wait vA] C_A(t+1) S_A(t) | ...
//   s2:        | [wait cA] V_A(t)          | [wait cB] V_B(t)           | ...
// The variable sweep's 12-VGPR waves fill whatever the 128-VGPR check waves leave of
// each SIMD and stream their messages under the check sweep's fp64 arithmetic (in
// the fused launch they take whole check-sized slots instead): 5.15 vs 5.35 ms per
// half-iteration for the strict arithmetic (MI355X, B=4096).  The variable sweeps are paced
// (knob var_pace, workgroups per 128 frames, default 28): unpaced, the sweep saturates HBM for
// the first ~1.7 ms of the 4.3 ms check launch beside it and the check sweep's gathers stall
// (VALU issue 0.72 of the launch); paced to stream over the whole check launch, 4.15 ms and
// 0.85 (MI355X, B=4096: 8.96 k -> 9.70 k frames/s on one box).  Knob lds_pad_kb reserves
// LDS per check workgroup to cap their residency (40/48 KB -> 3 per CU: 5.22-5.26 ms;
// 64 KB -> 2: 5.65 ms; 0 = default).
// The second stream of the two-stream schedules and its events, created on first use (all or
// nothing; the caller holds code->mu).
static int side_stream(const qr_code *code, hipStream_t *out) {
    if (!code->s2) {
        hipStream_t s2 = nullptr;
        hipEvent_t ev[5] = {};
        hipError_t e = hipStreamCreateWithFlags(&s2, hipStreamNonBlocking);
        for (int i = 0; i < 5 && e == hipSuccess; ++i) e = hipEventCreateWithFlags(&ev[i], hipEventDisableTiming);
        if (e != hipSuccess) {
            for (auto x : ev)
                if (x) (void)hipEventDestroy(x);
            if (s2) (void)hipStreamDestroy(s2);
            return set_error(QR_EDEVICE, "decode: second stream: %s", hipGetErrorString(e));
        }
        for (int i = 0; i < 5; ++i) code->ev[i] = ev[i];
        code->s2 = s2;
    }
    *out = code->s2;
    return QR_OK;
}

// A repack decision point of the range starting at column f0 (full width h), on P.s (the variable
// stream): one launch, k_repack_rows, decides and, when it repacks, moves the columns and (its
// last workgroup) updates the range's state.
static int launch_repack(const Plan &P, int f0, int h) {
    const qr_code *code = P.code;
    RepackArgs r;
    r.f0 = f0;
    r.h = h;
    r.ld = P.ld;
    r.pct = std::clamp(g_tune.repack_pct.load(), 1, 90);
    r.E = code->E;
    r.V = code->V;
    r.C = code->C;
    r.count = P.count_of(f0);
    r.sel = P.w.rsel + (f0 == 0 ? 0 : kSelInts);
    r.list = P.w.alist;
    r.active = P.w.active;
    r.c2v[0] = P.w.c2v;
    r.c2v[1] = P.w.rs.c2v_alt;
    r.out_post = P.post;
    r.lappr_in = P.lappr;
    r.synd_in = P.synd;
    r.post_w = P.w.rs.post;
    for (int k = 0; k < 2; ++k) {
        r.lappr_w[k] = P.w.rs.lappr[k];
        r.synd_w[k] = P.w.rs.synd[k];
    }
    r.fid_w = P.w.rs.fid;
    ProfScope ps("repack", P.s);
    // repack_grid workgroups walk the row groups; when the device decides not to repack they all
    // leave at once (a few microseconds on the variable stream)
    k_repack_rows<<<(unsigned)std::clamp(g_tune.repack_grid.load(), 1, 4096), kRepackThreads, 0, P.s>>>(r);
    QR_LAUNCH_CHECK();
    return QR_OK;
}

// *finalized: the final parity check, status and output were issued here (device-steered repack).
static int run_split2(const Plan &P, int max_it, bool *finalized) {
    const qr_code *code = P.code;
    // held while this decode ENQUEUES on the code's second stream and events; nothing here waits
    // for the GPU
    std::lock_guard<std::mutex> lk(code->mu);
    *finalized = false;
    hipStream_t s2 = nullptr;
    if (int rc0 = side_stream(code, &s2)) return rc0;
    hipEvent_t fork = code->ev[0], cA = code->ev[1], cB = code->ev[2], vA = code->ev[3], vB = code->ev[4];
    const int ld = P.ld, h = ld / 2;  // ld % 512 == 0: both ranges are h columns wide
    // Column repack (knob repack, default 1; needs the workspace's work set), decided on the device
    // at every decision point (k_repack_rows before each variable sweep of a
    // range): the host enqueues the same launches whatever the data, never reads anything back
    // and never waits, so the decode is asynchronous and capturable (the host runs far ahead of
    // the GPU anyway: counts it could read without waiting would be an iteration-old at best).
    const bool rp = P.compact && P.w.repack && g_tune.repack.load();
    Plan base = P;
    base.steer = rp;
    Plan Pb = base;  // status launches (P.s)
    Plan V = base;
    V.s = s2;
    V.var_pace = g_tune.var_pace.load();
    Plan C = base;
    C.lds_pad = std::max(0, g_tune.lds_pad_kb.load()) * 1024;
    auto row = [&](int t) { return P.w.unsat + (size_t)t * ld; };
    // Knob side (default 1): the check sweeps of the small degree classes (DVB-S2: the one
    // degree-6 check) run on the variable stream right after the variable sweep they follow,
    // under the other half's big check launch, instead of as a ~30 us launch of their own on
    // the critical check stream.  Per frame the order is unchanged: var(t) -> side checks
    // (t+1) -> [event] big checks(t+1) -> status(t) -> compaction -> [event] var(t+1).
    int big = 0;
    int64_t side_edges = 0;
    for (int k = 1; k < (int)code->classes.size(); ++k)
        if (code->classes[k].n > code->classes[big].n) big = k;
    for (int k = 0; k < (int)code->classes.size(); ++k)
        if (k != big) side_edges += code->classes[k].n * code->classes[k].degree;
    const bool side = g_tune.side.load() && code->classes.size() > 1 && side_edges * 8 <= code->E;
    auto checks_main = [&](int t, int k) {  // check sweep t >= 2 of range k on the check stream
        const int f0 = k * h, f1 = f0 + h;
        if (!side) return launch_checks<kNormal>(C, P.post, row(t - 1), f0, f1);
        const DegreeClass &cls = code->classes[big];
        return P.nt ? launch_check_class<kNormal, true>(C, cls, P.post, row(t - 1), f0, f1)
                    : launch_check_class<kNormal, false>(C, cls, P.post, row(t - 1), f0, f1);
    };
    auto checks_side = [&](int t, int k) {  // the other classes of check sweep t, on V.s
        if (!side) return (int)QR_OK;
        return launch_checks<kNormal>(V, P.post, row(t - 1), k * h, (k + 1) * h, big);
    };
    // range k's variable sweep t, preceded by its repack decision point (the status launch it
    // waits for wrote the count the device decides on); the copies run under the other range's
    // check launch.  No decision before the last variable sweep: a repack's transition ends with
    // the check sweep that follows it (the final parity sweep reads the columns of the list).
    auto var_sweep = [&](int k, int t) {
        const int f0 = k * h;
        if (rp && t < max_it) {
            if (int rc0 = launch_repack(V, f0, h)) return rc0;
        }
        return launch_var<false>(V, f0, f0 + h);
    };
    auto status = [&](int k, int ts) -> int {
        return launch_status_compact(Pb, k * h, (k + 1) * h, ts, row(ts));
    };
    int rc;
    QR_HIP(hipEventRecord(fork, P.s));
    QR_HIP(hipStreamWaitEvent(V.s, fork, 0));
    if ((rc = launch_checks<kFirst>(C, P.post, row(0), 0, h))) return rc;
    QR_HIP(hipEventRecord(cA, P.s));
    for (int t = 1; t <= max_it; ++t) {
        QR_HIP(hipStreamWaitEvent(V.s, cA, 0));
        if ((rc = var_sweep(0, t))) return rc;
        if (t < max_it && (rc = checks_side(t + 1, 0))) return rc;
        QR_HIP(hipEventRecord(vA, V.s));
        if (t == 1) {
            if ((rc = launch_checks<kFirst>(C, P.post, row(0), h, ld))) return rc;
        } else {
            QR_HIP(hipStreamWaitEvent(P.s, vB, 0));
            if ((rc = checks_main(t, 1))) return rc;
            if ((rc = status(1, t - 1))) return rc;
        }
        QR_HIP(hipEventRecord(cB, P.s));
        if (t < max_it) {
            QR_HIP(hipStreamWaitEvent(P.s, vA, 0));
            if ((rc = checks_main(t + 1, 0))) return rc;
            if ((rc = status(0, t))) return rc;
            QR_HIP(hipEventRecord(cA, P.s));
        }
        QR_HIP(hipStreamWaitEvent(V.s, cB, 0));
        if ((rc = var_sweep(1, t))) return rc;
        if (t < max_it && (rc = checks_side(t + 1, 1))) return rc;
        QR_HIP(hipEventRecord(vB, V.s));
    }
    // join: everything after (final parity check, status) follows both sweeps (vB follows cB)
    QR_HIP(hipStreamWaitEvent(P.s, vA, 0));
    QR_HIP(hipStreamWaitEvent(P.s, vB, 0));
    if (!rp) return QR_OK;
    // decoder.pyx:424-436 per range, wherever its frames live: the parity of the last posteriors
    // of its running frames (the lists), the final status, then every frame of a repacked range
    // hands its posteriors to the output
    uint8_t *unsat_last = row(max_it);
    Plan F = base;
    F.list_parity = true;
    for (int k = 0; k < 2; ++k) {
        const int f0 = k * h;
        if ((rc = launch_checks<kParityOnly>(F, P.post, unsat_last, f0, f0 + h))) return rc;
        if ((rc = launch_status(F, f0, f0 + h, max_it, 1, max_it, unsat_last))) return rc;
        ProfScope ps("repack_out", P.s);
        k_repack_output<<<4096, 256, 0, P.s>>>(code->V, f0, ld, F.sel_of(f0), P.w.rs.fid, P.w.rs.post, P.post);
        QR_LAUNCH_CHECK();
    }
    *finalized = true;
    return QR_OK;
}

// The one-launch-per-iteration schedule of small codes (k_iter): P(1) .. P(max_it + 1), the last
// one the final parity sweep.  Knob iter_streams (default 2): the frames are cut into that many
// ranges, each an independent chain of launches on its own stream (frames never depend on other
// frames), so one range's gathers overlap another range's arithmetic instead of every launch
// running a load phase then a compute phase.
static int run_iter(const Plan &P, int max_it) {
    const DegreeClass &cls = P.code->classes[0];
    const int ld = P.ld;
    IterArgs a;
    a.checks = cls.d_checks;
    a.n_checks = cls.n;
    a.chk_ptr = P.code->d_chk_ptr;
    a.chk_edge = P.code->d_chk_edge;
    a.chk_var = P.code->d_chk_var;
    a.var_ptr = P.code->d_var_ptr;
    a.var_edge = P.code->d_var_edge;
    a.lappr = P.lappr;
    a.post = P.post;
    a.synd = P.synd;
    a.active = P.w.active;
    a.success = P.success;
    a.iters = P.iters;
    a.ld = ld;
    // 64-frame tiles (MI355X, configs[1]: 42.3 vs 43.3 us per iteration at 128)
    a.g = make_geom(ld, std::min(64, g_tune.check_ft.load()), g_tune.check_per.load(), cls.n);
    const int64_t per_block = (int64_t)a.g.per * (256 >> a.g.lft);
    a.nbx = (unsigned)((cls.n + per_block - 1) / per_block);
    a.gglibc = P.code->d_gtab;
    a.finite = P.w.acount + 2;
    double *buf[2] = {P.w.c2v, P.w.c2v2};
    const int tiles = ld >> a.g.lft;
    const int nst = std::max(1, std::min({g_tune.iter_streams.load(), 2, tiles}));
    const qr_code *code = P.code;
    std::unique_lock<std::mutex> lk(code->mu, std::defer_lock);
    hipStream_t st[2] = {P.s, P.s};
    if (nst == 2) {
        lk.lock();
        if (int rc0 = side_stream(code, &st[1])) return rc0;
        QR_HIP(hipEventRecord(code->ev[0], P.s));
        QR_HIP(hipStreamWaitEvent(st[1], code->ev[0], 0));
    }
    // enqueue order interleaves the ranges; each stream runs its own chain
    for (int t = 1; t <= max_it + 1; ++t) {
        a.c2v_in = t == 1 ? nullptr : buf[(t - 1) & 1];
        a.c2v_out = t <= max_it ? buf[t & 1] : nullptr;
        a.unsat_s = t >= 3 ? P.w.unsat + (size_t)(t - 2) * ld : nullptr;
        a.unsat_p = t >= 2 ? P.w.unsat + (size_t)(t - 1) * ld : nullptr;
        a.status_iter = t - 2;
        for (int r = 0; r < nst; ++r) {
            const int t0 = tiles * r / nst, t1 = tiles * (r + 1) / nst;
            a.f_off = t0 << a.g.lft;
            const dim3 grid(a.nbx, (unsigned)(t1 - t0));
            ProfScope ps(profiling_on() ? "iter_d" + std::to_string(cls.degree) : std::string(), st[r]);
#define QR_CASE(DD)                                                                     \
    case DD:                                                                            \
        k_iter<DD><<<grid, 256, 0, st[r]>>>(a);                                         \
        break;
            switch (cls.degree) {
                QR_CASE(2) QR_CASE(3) QR_CASE(4) QR_CASE(5) QR_CASE(6) QR_CASE(7) QR_CASE(8) QR_CASE(9) QR_CASE(10)
                default: return set_error(QR_EVALUE, "decode: no fused-iteration kernel for degree %d", cls.degree);
            }
#undef QR_CASE
            QR_LAUNCH_CHECK();
        }
    }
    if (nst == 2) {  // join: the final status follows both chains
        QR_HIP(hipEventRecord(code->ev[4], st[1]));
        QR_HIP(hipStreamWaitEvent(P.s, code->ev[4], 0));
    }
    return QR_OK;
}

// The frame-resident decode (k_resident) runs a code whose messages and posteriors fit two
// workgroups' LDS per CU (so 16 waves of <= 128 VGPRs per CU) under the strict arithmetic.
static size_t resident_lds(const qr_code *code) { return (size_t)(code->E + code->V) * sizeof(double); }
static bool resident_code(const qr_code *code) {
    // 80 KiB keeps two workgroups per gfx950 CU (160 KiB); never more than the device lets a
    // workgroup take (otherwise the fused-iteration or flat schedule runs the code)
    const size_t lds_cap = std::min<size_t>(80 * 1024, code->lds_per_block);
    return g_tune.resident.load() && code->classes.size() == 1 &&
           code->classes[0].degree >= 2 && code->classes[0].degree <= kPackMaxDeg &&
           code->classes[0].n == code->C && code->C <= INT32_MAX / kPackMaxDeg && code->V < INT32_MAX &&
           resident_lds(code) + kResStaticLds <= lds_cap;
}

static int run_resident(const qr_code *code, int B, int ld, const double *lappr, const uint8_t *synd, int max_it,
                        double *final_post, uint8_t *success, int32_t *iters, int32_t *rsel, hipStream_t s) {
    ResArgs a;
    a.rsel = rsel;
    a.w0 = ld / 2;
    a.w1 = ld - ld / 2;
    a.C = (int)code->C;
    a.V = (int)code->V;
    a.B = B;
    a.ld = ld;
    a.max_it = max_it;
    a.chk_var = code->d_chk_var;
    a.var_ptr = code->d_var_ptr;
    a.var_msg = code->d_var_msg;
    a.lappr = lappr;
    a.synd = synd;
    a.post = final_post;
    a.success = success;
    a.iters = iters;
    a.gglibc = code->d_gtab;
    // the finite clamp's bound, as decode_batch_device's: 2^e, e = 1000 - (max_it + 2) log2(dv_max + 1)
    const double fin_x = ((double)max_it + 2.0) * std::log2((double)code->max_dv + 1.0);
    const int fin_e = fin_x > 999.0 ? 0 : 1000 - (int)std::ceil(fin_x);
    a.fin_bound = fin_e >= 1 ? std::ldexp(1.0, fin_e) : 0.0;
    a.dv = code->reg_dv >= 1 && code->reg_dv <= 3 && code->E < 65536 ? code->reg_dv : 0;
    const unsigned grid = (unsigned)(8 * ((B + 7) / 8));
    const size_t lds = resident_lds(code);
    ProfScope ps(profiling_on() ? "resident_d" + std::to_string(code->classes[0].degree) : std::string(), s);
#define QR_CASE(DD)                                          \
    case DD:                                                 \
        k_resident<DD><<<grid, kResThreads, lds, s>>>(a);    \
        break;
    switch (code->classes[0].degree) {
        QR_CASE(2) QR_CASE(3) QR_CASE(4) QR_CASE(5) QR_CASE(6) QR_CASE(7) QR_CASE(8) QR_CASE(9) QR_CASE(10)
        default: return set_error(QR_EVALUE, "decode: no frame-resident kernel for degree %d", code->classes[0].degree);
    }
#undef QR_CASE
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
    if (ws_size < ws_base_bytes(code, ld, max_it))
        return set_error(QR_EVALUE, "decode: workspace too small (%zu < %zu)", ws_size,
                         ws_base_bytes(code, ld, max_it));
    DeviceGuard dg(code->device);
    if (max_it > 0 && max_it <= kResMaxIter && resident_code(code))
        return run_resident(code, B, ld, lappr, synd, max_it, final_post, success, iters,
                            carve(code, ld, max_it, ws_ptr, ws_size).rsel, s);
    Plan P{code, B, ld, lappr, synd, final_post, success, iters, carve(code, ld, max_it, ws_ptr, ws_size), g_tune.nt.load() != 0, s};
    const int64_t rows = (int64_t)(max_it > 0 ? max_it : 0) + 2;  // no int overflow at INT_MAX
    int rc;
    QR_HIP(hipMemsetAsync(P.w.unsat, 0, (size_t)rows * ld, s));
    k_init_status<<<(ld + 255) / 256, 256, 0, s>>>(B, ld, P.w.active, success, iters, P.w.acount + 2, P.w.rsel, ld / 2,
                                                   ld - ld / 2);
    QR_LAUNCH_CHECK();
    // the strict arithmetic's finite flag: bound 2^e with e = 1000 - (max_it + 2) log2(dv_max + 1)
    // (in double, clamped before the cast: max_it may be as large as INT_MAX)
    const double fin_x = ((double)std::max(max_it, 0) + 2.0) * std::log2((double)code->max_dv + 1.0);
    const int fin_e = fin_x > 999.0 ? 0 : 1000 - (int)std::ceil(fin_x);
    if (fin_e < 1) QR_HIP(hipMemsetAsync(P.w.acount + 2, 0, sizeof(int32_t), s));
    // the flag itself is computed by the first variable sweep, which reads every LAPPR anyway
    int32_t *fin_flag = fin_e >= 1 ? P.w.acount + 2 : nullptr;
    // decoder.pyx:400-405: the input itself may already satisfy the syndrome.
    if ((rc = launch_checks<kParityOnly>(P, lappr, P.w.unsat, 0, ld))) return rc;
    if ((rc = launch_status(P, 0, ld, 0, 0, 0, P.w.unsat))) return rc;
    // decoder.pyx:408-421: c2v = 0, first variable sweep.
    if ((rc = launch_var<true>(P, 0, ld, fin_flag, fin_flag ? std::ldexp(1.0, fin_e) : 0.0))) return rc;
    int max_deg = 0;
    int64_t max_n = 0;
    for (const auto &c : code->classes) max_deg = std::max(max_deg, c.degree), max_n = std::max(max_n, c.n);
    const int sp = g_tune.split.load();
    // The split schedules overlap one half's check sweep with the other half's variable sweep;
    // that pays only when a half's check launch fills the chip on its own (DVB-S2 N=64800:
    // 1013 check blocks x 16 frame tiles at B = 4096).  A small code (configs[1]: reg-(3,6)
    // N=1008, B = 1024: 64 blocks) runs all frames in lock-step instead -- 4.9x the frames/s
    // of the split schedule on MI355X.  Knob split_min_blocks (0 = always split).
    const Geom gh = make_geom(ld / 2, g_tune.check_ft.load(), g_tune.check_per.load());
    const int64_t half_blocks = (max_n + (int64_t)gh.per * (256 >> gh.lft) - 1) / ((int64_t)gh.per * (256 >> gh.lft)) *
                                ((ld / 2) >> gh.lft);
    const bool split = sp >= 2 && ld % 512 == 0 && max_deg <= 16 && half_blocks >= g_tune.split_min_blocks.load();
    const bool iter = !split && max_it > 0 && g_tune.fused_iter.load() && P.w.c2v2;
    if (iter) {
        if ((rc = run_iter(P, max_it))) return rc;
        // P(max_it + 1) was the parity sweep of the last posteriors; every frame still running stops
        return launch_status(P, 0, ld, max_it, 1, max_it, P.w.unsat + (size_t)max_it * ld);
    }
    // active-frame lists of the ranges the schedule sweeps (after the iteration-0 status)
    P.compact = g_tune.compact.load() != 0;
    if (split) {
        if ((rc = launch_compact(P, 0, ld / 2)) || (rc = launch_compact(P, ld / 2, ld))) return rc;
    } else if ((rc = launch_compact(P, 0, ld))) {
        return rc;
    }
    bool finalized = false;
    if ((rc = !split ? run_flat(P, max_it) : sp == 3 ? run_split2(P, max_it, &finalized) : run_split(P, max_it)))
        return rc;
    if (finalized) return QR_OK;
    // Check after the last sweep; then every frame still running stops with (0, max).
    const int tf = max_it > 0 ? max_it : 0;
    uint8_t *unsat_last = P.w.unsat + (size_t)tf * ld;
    if (max_it > 0) {
        if ((rc = launch_checks<kParityOnly>(P, final_post, unsat_last, 0, ld))) return rc;
    } else {
        // decoder.pyx:424 with max_iterations <= 0: no sweep, no check -> (0, max_iterations)
        QR_HIP(hipMemsetAsync(unsat_last, 1, (size_t)ld, s));
    }
    if ((rc = launch_status(P, 0, ld, tf, 1, max_it, unsat_last))) return rc;
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

// The node-level surface (process_check_node, decoder.pyx:322-369) for any degree: v2c is
// a separate input here, so the forward values can be parked in the output slots
// c2v[e_i] <- F_{i-1} and replaced in the backward pass.
__global__ void k_check_nodes(const int64_t *nodes, int64_t n, const int32_t *chk_ptr, const int32_t *chk_edge,
                              const uint8_t *synd, double *c2v, const double *v2c, const GlibcTables *gtab) {
    __shared__ GlibcTables tab;
    stage_glibc_tables(&tab, gtab);
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int64_t c = nodes[i];
    const int base = chk_ptr[c], d = chk_ptr[c + 1] - base;
    const double s = synd[c] ? -1.0 : 1.0;
    const int32_t *e = chk_edge + base;
    double F = v2c[e[0]];
    for (int k = 1; k <= d - 2; ++k) {
        c2v[e[k]] = F;  // F_{k-1}
        F = box_plus_strict(F, v2c[e[k]], tab);
    }
    double Bn = v2c[e[d - 1]];
    c2v[e[d - 1]] = s * F;
    for (int k = d - 2; k >= 1; --k) {
        const double Fk = c2v[e[k]];
        c2v[e[k]] = s * box_plus_strict(Fk, Bn, tab);
        Bn = box_plus_strict(Bn, v2c[e[k]], tab);
    }
    c2v[e[0]] = s * Bn;
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
    (void)hipFree(c->d_var_msg);
    (void)hipFree(c->d_gtab);
    for (auto &e : c->ev)
        if (e) (void)hipEventDestroy(e);
    if (c->s2) (void)hipStreamDestroy(c->s2);
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
    TannerCsr T;  // host_build.hpp (decoder.pyx:60-146)
    std::string err;
    if (int rc = build_tanner_csr(e_to_v, e_to_c, nv, nc, T, err)) return set_error(rc, "%s", err.c_str());
    const int64_t E = T.E, V = T.V, C = T.C;
    const int32_t max_dc = T.max_dc, max_dv = T.max_dv;
    std::vector<int32_t> &chk_ptr = T.chk_ptr, &chk_edge = T.chk_edge, &chk_var = T.chk_var, &var_ptr = T.var_ptr,
                         &var_edge = T.var_edge;
    std::vector<std::vector<int32_t>> &by_deg = T.by_deg;

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
    code->reg_dv = max_dv;  // the common variable degree, or 0
    for (int64_t v = 0; v < V; ++v)
        if (var_ptr[(size_t)v + 1] - var_ptr[(size_t)v] != max_dv) code->reg_dv = 0;
    code->device = device;
    code->scratch.device = device;
    {
        size_t mem = 0;
        int lds = 0;
        if (hipDeviceTotalMem(&mem, device) != hipSuccess) mem = 0;
        if (hipDeviceGetAttribute(&lds, hipDeviceAttributeMaxSharedMemoryPerBlock, device) != hipSuccess) lds = 0;
        code->mem_bytes = mem;
        code->lds_per_block = (size_t)(lds > 0 ? lds : 0);
    }
    int rc = QR_OK;
    if ((rc = upload(&code->d_chk_ptr, chk_ptr)) || (rc = upload(&code->d_chk_edge, chk_edge)) ||
        (rc = upload(&code->d_chk_var, chk_var)) || (rc = upload(&code->d_var_ptr, var_ptr)) ||
        (rc = upload(&code->d_var_edge, var_edge))) {
        free_code(code);
        return rc;
    }
    {
        // the frame-resident decode's LDS message index of every edge, in the variable CSR's
        // order: edge i of check c (check-CSR slot chk_ptr[c] + i) lives at i * C + c
        std::vector<int32_t> msg_of_edge((size_t)E), var_msg((size_t)E);
        for (int64_t c = 0; c < C; ++c)
            for (int32_t s = chk_ptr[(size_t)c]; s < chk_ptr[(size_t)c + 1]; ++s)
                msg_of_edge[(size_t)chk_edge[(size_t)s]] = (int32_t)((s - chk_ptr[(size_t)c]) * C + c);
        for (int64_t k = 0; k < E; ++k) var_msg[(size_t)k] = msg_of_edge[(size_t)var_edge[(size_t)k]];
        if ((rc = upload(&code->d_var_msg, var_msg))) {
            free_code(code);
            return rc;
        }
    }
    {
        std::vector<GlibcTables> gt(1);
        build_glibc_tables(&gt[0]);
        if ((rc = upload(&code->d_gtab, gt))) {
            free_code(code);
            return rc;
        }
    }
    for (int d = 0; d < (int)by_deg.size(); ++d) {
        if (by_deg[d].empty()) continue;
        DegreeClass cls{d, (int64_t)by_deg[d].size(), nullptr};
        if (d > kMaxTemplDeg) {
            cls.fb_base = code->fb_rows;
            code->fb_rows += cls.n * (d - 2);
        }
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

#if QR_DEBUG_ASSERT
// Debug build only (libqamr_debug.so; not in include/qamr.h): out = {failed device checks, first
// failing site (DebugSite), its two values}; reads and clears them.
QR_API int qr_debug_asserts(int64_t *out) {
    unsigned long long h[4] = {0, 0, 0, 0};
    if (hipDeviceSynchronize() != hipSuccess) return QR_EDEVICE;
    if (hipMemcpyFromSymbol(h, HIP_SYMBOL(qr::g_dbg), sizeof(h)) != hipSuccess) return QR_EDEVICE;
    const unsigned long long z[4] = {0, 0, 0, 0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(qr::g_dbg), z, sizeof(z)) != hipSuccess) return QR_EDEVICE;
    for (int i = 0; i < 4; ++i) out[i] = (int64_t)h[i];
    return QR_OK;
}
#endif

#if QR_EXPERIMENT_CLOCK
// Diagnostic builds only (not in include/qamr.h): out = {sum cycles, sum ticks, workgroups}.
QR_API int qr_debug_clock(int64_t *out) {
    unsigned long long h[3] = {0, 0, 0};
    if (hipMemcpyFromSymbol(h, HIP_SYMBOL(qr::g_clk), sizeof(h)) != hipSuccess) return QR_EDEVICE;
    const unsigned long long z[3] = {0, 0, 0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(qr::g_clk), z, sizeof(z)) != hipSuccess) return QR_EDEVICE;
    for (int i = 0; i < 3; ++i) out[i] = (int64_t)h[i];
    return QR_OK;
}
// out[2 n]: realtime {start, end} of workgroups 0..n-1 of the last stamped launch
QR_API int qr_debug_wg_times(int64_t *out, int32_t n) {
    if (n < 0 || n > qr::kWgTimes) return QR_EVALUE;
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(qr::g_wgt), (size_t)n * 16) != hipSuccess) return QR_EDEVICE;
    return QR_OK;
}
#endif

// name -> knob (nullptr if unknown)
static std::atomic<int> *tune_knob(const char *name) {
    static const std::pair<const char *, std::atomic<int> *> knobs[] = {
        {"check_ft", &g_tune.check_ft},     {"check_per", &g_tune.check_per},
        {"var_ft", &g_tune.var_ft},         {"var_per", &g_tune.var_per},
        {"nt", &g_tune.nt},                 {"split", &g_tune.split},
        {"lds_pad_kb", &g_tune.lds_pad_kb}, {"compact", &g_tune.compact},
        {"side", &g_tune.side},             {"demap_fast", &g_demap_fast},
        {"demap_hyp", &g_demap_hyp},        {"min_blocks", &g_tune.min_blocks},
        {"split_min_blocks", &g_tune.split_min_blocks},
        {"var_pace", &g_tune.var_pace},     {"check_tail", &g_tune.check_tail}, {"var_boost", &g_tune.var_boost},
        {"fused_iter", &g_tune.fused_iter}, {"iter_streams", &g_tune.iter_streams},
        {"resident", &g_tune.resident},   {"repack", &g_tune.repack},
        {"repack_pct", &g_tune.repack_pct}, {"repack_grid", &g_tune.repack_grid},
    };
    const std::string n = name ? name : "";
    for (const auto &k : knobs)
        if (n == k.first) return k.second;
    return nullptr;
}

int qr_tune_set(const char *name, int64_t value) {
    std::atomic<int> *k = tune_knob(name);
    if (!k) return set_error(QR_EVALUE, "unknown tuning knob '%s'", name ? name : "");
    if (value < 0 || value > 4096 || (k == &g_tune.split && value > 3))
        return set_error(QR_EVALUE, "tuning value out of range");
    k->store((int)value);
    return QR_OK;
}

int qr_tune_get(const char *name, int64_t *value) {
    const std::atomic<int> *k = tune_knob(name);
    if (!k || !value) return set_error(QR_EVALUE, "unknown tuning knob '%s'", name ? name : "");
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

int qr_decode_repack_stats(const qr_code *code, int32_t ld, int32_t max_it, const void *ws, size_t ws_size,
                           int32_t *out) {
    if (!code || !ws || !out) return set_error(QR_EVALUE, "null argument");
    if (ld <= 0 || ld % kWave) return set_error(QR_EVALUE, "ld must be a positive multiple of 64");
    if (ws_size < ws_base_bytes(code, ld, max_it)) return set_error(QR_EVALUE, "workspace too small");
    const DecodeWs w = carve(code, ld, max_it, const_cast<void *>(ws), ws_size);
    int32_t sel[2 * kSelInts];
    DeviceGuard dg(code->device);
    QR_HIP(hipMemcpy(sel, w.rsel, sizeof(sel), hipMemcpyDeviceToHost));
    for (int k = 0; k < 2; ++k) {
        out[k] = sel[k * kSelInts + kSelRepacks];
        out[2 + k] = sel[k * kSelInts + kSelW];
    }
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
                                                        d_v2c, code->d_gtab);
    QR_LAUNCH_CHECK();
    QR_HIP(hipMemcpy(c2v, d_c2v, E * 8, hipMemcpyDeviceToHost));
    return QR_OK;
}

}  // extern "C"
