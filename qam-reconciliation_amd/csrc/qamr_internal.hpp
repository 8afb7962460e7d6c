// qamr_internal.hpp -- shared host-side definitions of libqamr.so.
#pragma once
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "qamr.h"
#include "qamr_math.hpp"
#include "exp_table.hpp"
#include "glibc_math.hpp"

namespace qr {

// ------------------------------------------------------------------ errors
int set_error(int code, const char *fmt, ...);
int hip_fail(hipError_t e, const char *what, const char *file, int line);

#define QR_HIP(call)                                                            \
    do {                                                                        \
        hipError_t _qr_e = (call);                                              \
        if (_qr_e != hipSuccess) return ::qr::hip_fail(_qr_e, #call, __FILE__, __LINE__); \
    } while (0)

#define QR_LAUNCH_CHECK() QR_HIP(hipGetLastError())

// --------------------------------------------------------------- profiling
// hipEvent pair recorded on the launch stream around one kernel launch.
struct ProfScope {
    ProfScope(std::string name, hipStream_t s);
    ~ProfScope();
    std::string name_;
    hipStream_t s_;
    hipEvent_t a_ = nullptr, b_ = nullptr;
    bool capture_ = false;  // recorded into a graph being captured (external event-record nodes)
    void record(hipEvent_t e);
};
bool profiling_on();

// ------------------------------------------------------------------ layout
constexpr int kWave = 64;
inline int frame_tile(int ld) { return (ld % 256 == 0) ? 256 : (ld % 128 == 0) ? 128 : 64; }
inline size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

// Device scratch owned by a handle, grown on demand (host-API calls only).
struct Scratch {
    std::mutex mu;
    void *ptr = nullptr;
    size_t bytes = 0;
    int device = 0;
    int reserve(size_t want);  // caller holds mu
    ~Scratch();
};

// Kernel launchers shared between translation units.
int launch_transpose_to_fi_f64(int B, int ld, int64_t n, const double *src, double *dst, hipStream_t s);
int launch_transpose_to_fm_f64(int B, int ld, int64_t n, const double *src, double *dst, hipStream_t s);
int launch_transpose_to_fi_u8(int B, int ld, int64_t n, const uint8_t *src, uint8_t *dst, hipStream_t s);
int launch_transpose_to_fi_i64(int B, int ld, int64_t n, const int64_t *src, int64_t *dst, hipStream_t s);

extern std::atomic<int> g_demap_fast;  // demap.hip (tuning knob "demap_fast")
extern std::atomic<int> g_demap_hyp;   // demap.hip (tuning knob "demap_hyp")

struct DeviceGuard {
    explicit DeviceGuard(int dev) {
        (void)hipGetDevice(&prev_);
        if (prev_ != dev) (void)hipSetDevice(dev);
        dev_ = dev;
    }
    ~DeviceGuard() {
        if (prev_ != dev_) (void)hipSetDevice(prev_);
    }
    int prev_ = 0, dev_ = 0;
};

// Diagnostic twin only (libqamr_clock.so, QR_EXPERIMENT_CLOCK=1; the product library carries no
// stamp): a workgroup's shader-clock (s_memtime) and 100 MHz realtime (s_memrealtime) spans added
// to acc[0..2] = {cycles, ticks, workgroups} by thread 0 (vector atomics) when the scope ends, and
// its realtime start / end stored in wgt (first kWgTimes workgroups) if given.  Every thread of
// the workgroup must reach the end of the scope (it ends with a barrier).
#ifndef QR_EXPERIMENT_CLOCK
#define QR_EXPERIMENT_CLOCK 0
#endif
constexpr int kWgTimes = 1 << 16;
#if QR_EXPERIMENT_CLOCK
struct ClkScope {
    bool on;
    unsigned long long *acc, *wgt;
    uint64_t c0, r0;
    __device__ ClkScope(bool on_, unsigned long long *acc_, unsigned long long *wgt_) : on(on_), acc(acc_), wgt(wgt_) {
        c0 = __builtin_amdgcn_s_memtime();
        r0 = __builtin_amdgcn_s_memrealtime();
    }
    __device__ ~ClkScope() {
        __syncthreads();
        if (on && threadIdx.x == 0) {
            const uint64_t c1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
            atomicAdd(&acc[0], (unsigned long long)(c1 - c0));
            atomicAdd(&acc[1], (unsigned long long)(r1 - r0));
            atomicAdd(&acc[2], 1ull);
            const unsigned b = blockIdx.y * gridDim.x + blockIdx.x;
            if (wgt && b < (unsigned)kWgTimes) {
                wgt[2 * b] = r0;
                wgt[2 * b + 1] = r1;
            }
        }
    }
};
#endif

}  // namespace qr

// --------------------------------------------------------------- handles
struct DegreeClass {
    int32_t degree;
    int64_t n;
    int32_t *d_checks;  // check ids of this degree, ascending
    // degree > kMaxTemplDeg (runtime-degree kernel): first row of this class's forward
    // values in the decode workspace's F scratch (n * (degree - 2) rows of ld doubles)
    int64_t fb_base = 0;
};

struct qr_code {
    int64_t E = 0, V = 0, C = 0;
    int32_t max_dc = 0, max_dv = 0;
    int32_t reg_dv = 0;  // every variable node's degree when they are all equal, else 0
    int device = 0;
    size_t mem_bytes = 0;       // the device's memory (bounds the optional repack work set)
    size_t lds_per_block = 0;   // LDS a workgroup may take (the frame-resident decode needs it)
    // CSR, int32 (E < 2^31): per check, edge ids ascending and their variables;
    // per variable, edge ids ascending.
    int32_t *d_chk_ptr = nullptr, *d_chk_edge = nullptr, *d_chk_var = nullptr;
    int32_t *d_var_ptr = nullptr, *d_var_edge = nullptr;
    // per variable, edges ascending as above, each given by the frame-resident small-code
    // decoder's LDS message index i * C + c (edge i of check c)
    int32_t *d_var_msg = nullptr;
    std::vector<DegreeClass> classes;
    int64_t fb_rows = 0;  // rows of the F scratch (sum over runtime-degree classes)
    qr::GlibcTables *d_gtab = nullptr; // strict box-plus: glibc exp/log data (glibc_math.hpp)
    uint32_t *d_cu_arrivals = nullptr; // per-CU arrival counters of the frame-resident decode (knob res_stagger)
    mutable qr::Scratch scratch;
    // two-stream schedule (decoder.hip run_split2): a second stream for the variable
    // sweeps and the events that order the two; created on first use, guarded by mu
    // while a decode enqueues (concurrent decodes on one code enqueue one at a time).
    mutable std::mutex mu;
    mutable hipStream_t s2 = nullptr;
    mutable hipEvent_t ev[5] = {nullptr, nullptr, nullptr, nullptr, nullptr};
};

struct qr_demap {
    int device = 0;
    qr::DemapTables h;                      // host copy
    qr::DemapTables *d_tables = nullptr;    // device copy
    qr::MathTables *d_mtab = nullptr;       // exp table for the Newton root search
    double2 *d_quant = nullptr;             // F_Y^-1 Hermite nodes (Newton start), may be null
    double *d_ftab = nullptr;               // Taylor table of F_Y (Newton), may be null
    mutable qr::Scratch scratch;
};
