// runtime.hip -- error reporting, per-kernel event timing, device scratch and
// the frame-major <-> frame-innermost transposes of libqamr.so.
#include <stdarg.h>
#include <stdio.h>

#include <atomic>
#include <map>
#include <set>

#include "qamr_internal.hpp"

namespace qr {

static thread_local std::string g_err;

int set_error(int code, const char *fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

int hip_fail(hipError_t e, const char *what, const char *file, int line) {
    if (e == hipErrorOutOfMemory)
        return set_error(QR_EMEMORY, "out of device memory in %s (%s:%d)", what, file, line);
    return set_error(QR_EDEVICE, "HIP error %d (%s) in %s (%s:%d)", (int)e, hipGetErrorString(e), what, file, line);
}

// ------------------------------------------------------------------ profiling
namespace {
struct Pending {
    std::string name;
    hipEvent_t a, b;
};
struct Stat {
    double ms = 0;
    int64_t n = 0;
};
std::atomic<bool> g_prof{false};
// External event-record nodes accepted in stream captures: probed once, outside any capture of
// the caller's, when profiling is switched on (-1 = not probed yet).  A failed external record
// inside a live capture would invalidate that capture, so it is never attempted there.
std::atomic<int> g_prof_external{-1};

// A private relaxed-mode capture on a private stream holding one external event record.
bool probe_external_records() {
    hipStream_t s = nullptr;
    hipEvent_t e = nullptr;
    bool ok = hipStreamCreateWithFlags(&s, hipStreamNonBlocking) == hipSuccess && hipEventCreate(&e) == hipSuccess;
    if (ok && hipStreamBeginCapture(s, hipStreamCaptureModeRelaxed) == hipSuccess) {
        ok = hipEventRecordWithFlags(e, s, hipEventRecordExternal) == hipSuccess;
        hipGraph_t g = nullptr;
        if (hipStreamEndCapture(s, &g) != hipSuccess) ok = false;
        if (g) (void)hipGraphDestroy(g);
    } else {
        ok = false;
    }
    if (e) (void)hipEventDestroy(e);
    if (s) (void)hipStreamDestroy(s);
    (void)hipGetLastError();
    return ok;
}
std::mutex g_prof_mu;
std::vector<Pending> g_pending;
std::map<std::string, Stat> g_stats;
std::set<std::string> g_prof_select;  // empty: every launch is timed

void drain_pending_locked() {
    for (auto &p : g_pending) {
        float ms = 0.f;
        if (hipEventSynchronize(p.b) == hipSuccess && hipEventElapsedTime(&ms, p.a, p.b) == hipSuccess) {
            auto &s = g_stats[p.name];
            s.ms += ms;
            s.n += 1;
        }
        (void)hipEventDestroy(p.a);
        (void)hipEventDestroy(p.b);
    }
    g_pending.clear();
}
}  // namespace

bool profiling_on() { return g_prof.load(std::memory_order_relaxed); }

ProfScope::ProfScope(std::string name, hipStream_t s) : name_(std::move(name)), s_(s) {
    if (!profiling_on()) return;
    {
        std::lock_guard<std::mutex> lk(g_prof_mu);
        if (!g_prof_select.empty() && !g_prof_select.count(name_)) return;
    }
    if (hipEventCreate(&a_) != hipSuccess || hipEventCreate(&b_) != hipSuccess) {
        a_ = b_ = nullptr;
        return;
    }
    // Inside a stream capture a plain record only marks a dependency; an external record
    // becomes an event-record node of the graph, re-recorded at every replay (the pair then
    // times the launch of the latest replay when qr_profile_query drains it).
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    capture_ = s_ && hipStreamIsCapturing(s_, &cs) == hipSuccess && cs == hipStreamCaptureStatusActive;
    if (capture_ && g_prof_external.load() != 1) {  // no event-record nodes: captured launches go untimed
        (void)hipEventDestroy(a_);
        (void)hipEventDestroy(b_);
        a_ = b_ = nullptr;
        return;
    }
    record(a_);
}

void ProfScope::record(hipEvent_t e) {
    if (capture_) (void)hipEventRecordWithFlags(e, s_, hipEventRecordExternal);
    else (void)hipEventRecord(e, s_);
}

ProfScope::~ProfScope() {
    if (!a_) return;
    record(b_);
    std::lock_guard<std::mutex> lk(g_prof_mu);
    g_pending.push_back({name_, a_, b_});
    if (g_pending.size() > 4096) drain_pending_locked();
}

// ------------------------------------------------------------------ scratch
int Scratch::reserve(size_t want) {
    if (want <= bytes) return QR_OK;
    if (ptr) {
        (void)hipFree(ptr);
        ptr = nullptr;
        bytes = 0;
    }
    QR_HIP(hipMalloc(&ptr, want));
    bytes = want;
    return QR_OK;
}

Scratch::~Scratch() {
    if (ptr) {
        DeviceGuard g(device);
        (void)hipFree(ptr);
    }
}

// ---------------------------------------------------------------- transposes
// Frame-major src[f * n + i] (f < B)  ->  frame-innermost dst[i * ld + f].
// 64x64 tiles staged through LDS (padded by one element against bank
// conflicts); 256 threads = 4 waves, each lane moves 16 elements.
template <typename T>
__global__ void __launch_bounds__(256) k_to_fi(int B, int ld, int64_t n, const T *__restrict__ src, T *__restrict__ dst) {
    __shared__ T tile[64][65];
    const int64_t i0 = (int64_t)blockIdx.x * 64;
    const int f0 = blockIdx.y * 64;
    const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int f = f0 + ty * 16 + r;
        const int64_t i = i0 + tx;
        tile[ty * 16 + r][tx] = (f < B && i < n) ? src[(int64_t)f * n + i] : T(0);
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int64_t i = i0 + ty * 16 + r;
        const int f = f0 + tx;
        if (i < n && f < ld) dst[i * ld + f] = tile[tx][ty * 16 + r];
    }
}

// Frame-innermost src[i * ld + f] -> frame-major dst[f * n + i] (f < B).
template <typename T>
__global__ void __launch_bounds__(256) k_to_fm(int B, int ld, int64_t n, const T *__restrict__ src, T *__restrict__ dst) {
    __shared__ T tile[64][65];
    const int64_t i0 = (int64_t)blockIdx.x * 64;
    const int f0 = blockIdx.y * 64;
    const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int64_t i = i0 + ty * 16 + r;
        const int f = f0 + tx;
        tile[ty * 16 + r][tx] = (i < n && f < B) ? src[i * ld + f] : T(0);
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int f = f0 + ty * 16 + r;
        const int64_t i = i0 + tx;
        if (f < B && i < n) dst[(int64_t)f * n + i] = tile[tx][ty * 16 + r];
    }
}

template <typename T>
static int launch_to_fi(int B, int ld, int64_t n, const T *src, T *dst, hipStream_t s) {
    if (B <= 0 || ld < B || ld % kWave || n <= 0) return set_error(QR_EVALUE, "bad transpose shape B=%d ld=%d n=%lld", B, ld, (long long)n);
    dim3 grid((unsigned)((n + 63) / 64), (unsigned)((ld + 63) / 64));
    k_to_fi<T><<<grid, 256, 0, s>>>(B, ld, n, src, dst);
    QR_LAUNCH_CHECK();
    return QR_OK;
}
template <typename T>
static int launch_to_fm(int B, int ld, int64_t n, const T *src, T *dst, hipStream_t s) {
    if (B <= 0 || ld < B || ld % kWave || n <= 0) return set_error(QR_EVALUE, "bad transpose shape B=%d ld=%d n=%lld", B, ld, (long long)n);
    dim3 grid((unsigned)((n + 63) / 64), (unsigned)((B + 63) / 64));
    k_to_fm<T><<<grid, 256, 0, s>>>(B, ld, n, src, dst);
    QR_LAUNCH_CHECK();
    return QR_OK;
}

int launch_transpose_to_fi_f64(int B, int ld, int64_t n, const double *src, double *dst, hipStream_t s) {
    return launch_to_fi<double>(B, ld, n, src, dst, s);
}
int launch_transpose_to_fm_f64(int B, int ld, int64_t n, const double *src, double *dst, hipStream_t s) {
    return launch_to_fm<double>(B, ld, n, src, dst, s);
}
int launch_transpose_to_fi_u8(int B, int ld, int64_t n, const uint8_t *src, uint8_t *dst, hipStream_t s) {
    return launch_to_fi<uint8_t>(B, ld, n, src, dst, s);
}
int launch_transpose_to_fi_i64(int B, int ld, int64_t n, const int64_t *src, int64_t *dst, hipStream_t s) {
    return launch_to_fi<int64_t>(B, ld, n, src, dst, s);
}

}  // namespace qr

// ===================================================================== C-ABI
namespace qr {
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
// Streaming copy, one 16-B non-temporal load and store per lane per step, grid-stride over 1024
// workgroups (scripts/native/copybw.hip on MI355X, 4 GiB: 5.32 TB/s; 4-deep per lane 4.60 at
// 8 workgroups per CU, 5.29 at 65 536 workgroups).
__global__ void __launch_bounds__(256) k_stream_copy(const u32x4 *__restrict__ src, u32x4 *__restrict__ dst, int64_t n) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
        __builtin_nontemporal_store(__builtin_nontemporal_load(&src[i]), &dst[i]);
}
// One wave per workgroup; lane 0 alone times the spin (scalar counters), then stores with
// an ordinary vector store.
__global__ void __launch_bounds__(64) k_clock_probe(int64_t *__restrict__ out, int64_t ticks) {
    if (threadIdx.x != 0) return;
    const int64_t r0 = (int64_t)__builtin_amdgcn_s_memrealtime();
    const int64_t t0 = (int64_t)__builtin_amdgcn_s_memtime();
    int64_t r1 = r0;
    while (r1 - r0 < ticks) {
        __builtin_amdgcn_s_sleep(4);
        r1 = (int64_t)__builtin_amdgcn_s_memrealtime();
    }
    const int64_t t1 = (int64_t)__builtin_amdgcn_s_memtime();
    out[2 * blockIdx.x] = t1 - t0;
    out[2 * blockIdx.x + 1] = r1 - r0;
}
}  // namespace qr

extern "C" {

const char *qr_last_error(void) { return qr::g_err.c_str(); }

int qr_version(int32_t *major, int32_t *minor) {
    if (major) *major = 0;
    if (minor) *minor = 1;
    return QR_OK;
}

int qr_device_count(int32_t *count) {
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess) n = 0;
    *count = n;
    return QR_OK;
}

int qr_profile_enable(int32_t on) {
    if (on && qr::g_prof_external.load() < 0) qr::g_prof_external.store(qr::probe_external_records() ? 1 : 0);
    qr::g_prof.store(on != 0);
    return QR_OK;
}

int qr_profile_select(const char *names) {
    std::lock_guard<std::mutex> lk(qr::g_prof_mu);
    qr::g_prof_select.clear();
    std::string n = names ? names : "";
    size_t p = 0;
    while (p <= n.size()) {
        const size_t q = std::min(n.find(',', p), n.size());
        if (q > p) qr::g_prof_select.insert(n.substr(p, q - p));
        p = q + 1;
    }
    return QR_OK;
}

int qr_profile_reset(void) {
    std::lock_guard<std::mutex> lk(qr::g_prof_mu);
    qr::drain_pending_locked();
    qr::g_stats.clear();
    return QR_OK;
}

int qr_profile_query(const char *name, double *total_ms, int64_t *launches) {
    std::lock_guard<std::mutex> lk(qr::g_prof_mu);
    qr::drain_pending_locked();
    auto it = qr::g_stats.find(name ? name : "");
    *total_ms = (it == qr::g_stats.end()) ? 0.0 : it->second.ms;
    *launches = (it == qr::g_stats.end()) ? 0 : it->second.n;
    return QR_OK;
}

int qr_to_frame_innermost_f64(int32_t B, int32_t ld, int64_t n, const double *s, double *d, void *st) {
    return qr::launch_transpose_to_fi_f64(B, ld, n, s, d, (hipStream_t)st);
}
int qr_to_frame_major_f64(int32_t B, int32_t ld, int64_t n, const double *s, double *d, void *st) {
    return qr::launch_transpose_to_fm_f64(B, ld, n, s, d, (hipStream_t)st);
}
int qr_to_frame_innermost_u8(int32_t B, int32_t ld, int64_t n, const uint8_t *s, uint8_t *d, void *st) {
    return qr::launch_transpose_to_fi_u8(B, ld, n, s, d, (hipStream_t)st);
}
int qr_to_frame_innermost_i64(int32_t B, int32_t ld, int64_t n, const int64_t *s, int64_t *d, void *st) {
    return qr::launch_transpose_to_fi_i64(B, ld, n, s, d, (hipStream_t)st);
}

int qr_stream_copy(const void *src, void *dst, int64_t bytes, void *st) {
    if (!src || !dst || bytes < 0 || (bytes & 15) || (((uintptr_t)src | (uintptr_t)dst) & 15))
        return qr::set_error(QR_EVALUE, "qr_stream_copy: 16-B aligned pointers and a multiple of 16 bytes required");
    if (bytes == 0) return QR_OK;
    const int64_t n = bytes / 16;
    const unsigned grid = (unsigned)std::min<int64_t>((n + 255) / 256, 1024);   // 4 workgroups per CU
    qr::k_stream_copy<<<grid, 256, 0, (hipStream_t)st>>>((const qr::u32x4 *)src, (qr::u32x4 *)dst, n);
    QR_LAUNCH_CHECK();
    return QR_OK;
}

int qr_clock_probe(int64_t *d_out, int32_t n, int64_t realtime_ticks, void *st) {
    if (!d_out || n <= 0 || n > 4096 || realtime_ticks <= 0 || realtime_ticks > 100000000)
        return qr::set_error(QR_EVALUE, "qr_clock_probe: need d_out, 0 < n <= 4096, 0 < ticks <= 1e8");
    qr::k_clock_probe<<<(unsigned)n, 64, 0, (hipStream_t)st>>>(d_out, realtime_ticks);
    QR_LAUNCH_CHECK();
    return QR_OK;
}

}  // extern "C"
