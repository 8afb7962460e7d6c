// Streaming-copy bandwidth probe (variants of the copy used as bench.py's ceiling).
#include <hip/hip_runtime.h>
#include <cstdio>
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
template <bool NT, int U>
__global__ void __launch_bounds__(256) cp(const u32x4 *__restrict__ s, u32x4 *__restrict__ d, long n) {
    const long stride = (long)gridDim.x * blockDim.x;
    long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    for (; i + (U - 1) * stride < n; i += U * stride) {
        u32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = NT ? __builtin_nontemporal_load(&s[i + u * stride]) : s[i + u * stride];
#pragma unroll
        for (int u = 0; u < U; ++u) { if (NT) __builtin_nontemporal_store(v[u], &d[i + u * stride]); else d[i + u * stride] = v[u]; }
    }
    for (; i < n; i += stride) d[i] = s[i];
}
template <bool NT, int U>
float run(const u32x4 *a, u32x4 *b, long n, int grid) {
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    cp<NT, U><<<grid, 256>>>(a, b, n);
    hipEventRecord(e0);
    for (int r = 0; r < 10; ++r) cp<NT, U><<<grid, 256>>>(a, b, n);
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    return 2.0f * n * 16 * 10 / (ms / 1e3f) / 1e9f;
}
int main() {
    const long bytes = 4L << 30, n = bytes / 16;
    u32x4 *a, *b; hipMalloc(&a, bytes); hipMalloc(&b, bytes); hipMemset(a, 1, bytes);
    for (int grid : {1024, 4096, 16384, 65536}) {
        printf("grid %6d: plain U1 %7.1f  U4 %7.1f | nt U1 %7.1f  U4 %7.1f GB/s\n", grid, run<false, 1>(a, b, n, grid),
               run<false, 4>(a, b, n, grid), run<true, 1>(a, b, n, grid), run<true, 4>(a, b, n, grid));
    }
    return 0;
}
