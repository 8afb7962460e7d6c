// Issue cost of fp64 vs 32-bit VALU instructions on gfx950 (MI355X): every SIMD runs W
// waves of 8 independent chains of one instruction kind; cycles from s_memtime.
//   hipcc --offload-arch=gfx950 -O3 -o valu_rate valu_rate.hip && ./valu_rate
#include <hip/hip_runtime.h>
#include <cstdio>

#define R8(X) X X X X X X X X
template <int KIND>
__global__ void __launch_bounds__(1024) k(long long *cyc, double *out, int iters) {
    double d0 = threadIdx.x, d1 = d0 + 1, d2 = d0 + 2, d3 = d0 + 3, d4 = d0 + 4, d5 = d0 + 5, d6 = d0 + 6, d7 = d0 + 7;
    unsigned x0 = threadIdx.x, x1 = x0 ^ 1, x2 = x0 ^ 2, x3 = x0 ^ 3, x4 = x0 ^ 4, x5 = x0 ^ 5, x6 = x0 ^ 6, x7 = x0 ^ 7;
    const double b = 1.0000001, c = 1e-9;
    const unsigned y = 3;
    long long t0 = clock64();
    for (int i = 0; i < iters; ++i) {
        if (KIND == 0) {
            R8(asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(d0) : "v"(b), "v"(c));
               asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(d1) : "v"(b), "v"(c));
               asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(d2) : "v"(b), "v"(c));
               asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(d3) : "v"(b), "v"(c));
               asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(d4) : "v"(b), "v"(c));
               asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(d5) : "v"(b), "v"(c));
               asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(d6) : "v"(b), "v"(c));
               asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(d7) : "v"(b), "v"(c));)
        } else if (KIND == 1) {
            R8(asm volatile("v_add_u32 %0, %0, %1" : "+v"(x0) : "v"(y));
               asm volatile("v_add_u32 %0, %0, %1" : "+v"(x1) : "v"(y));
               asm volatile("v_add_u32 %0, %0, %1" : "+v"(x2) : "v"(y));
               asm volatile("v_add_u32 %0, %0, %1" : "+v"(x3) : "v"(y));
               asm volatile("v_add_u32 %0, %0, %1" : "+v"(x4) : "v"(y));
               asm volatile("v_add_u32 %0, %0, %1" : "+v"(x5) : "v"(y));
               asm volatile("v_add_u32 %0, %0, %1" : "+v"(x6) : "v"(y));
               asm volatile("v_add_u32 %0, %0, %1" : "+v"(x7) : "v"(y));)
        } else if (KIND == 2) {
            R8(asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(x0) : "v"(y));
               asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(x1) : "v"(y));
               asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(x2) : "v"(y));
               asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(x3) : "v"(y));
               asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(x4) : "v"(y));
               asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(x5) : "v"(y));
               asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(x6) : "v"(y));
               asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(x7) : "v"(y));)
        } else if (KIND == 3) {  // alternating fp64 fma / 32-bit add
            R8(asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(d0) : "v"(b), "v"(c));
               asm volatile("v_add_u32 %0, %0, %1" : "+v"(x0) : "v"(y));
               asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(d1) : "v"(b), "v"(c));
               asm volatile("v_add_u32 %0, %0, %1" : "+v"(x1) : "v"(y));
               asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(d2) : "v"(b), "v"(c));
               asm volatile("v_add_u32 %0, %0, %1" : "+v"(x2) : "v"(y));
               asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(d3) : "v"(b), "v"(c));
               asm volatile("v_add_u32 %0, %0, %1" : "+v"(x3) : "v"(y));)
        } else if (KIND == 4) {
            R8(asm volatile("v_ldexp_f64 %0, %0, %1" : "+v"(d0) : "v"(y));
               asm volatile("v_ldexp_f64 %0, %0, %1" : "+v"(d1) : "v"(y));
               asm volatile("v_ldexp_f64 %0, %0, %1" : "+v"(d2) : "v"(y));
               asm volatile("v_ldexp_f64 %0, %0, %1" : "+v"(d3) : "v"(y));
               asm volatile("v_ldexp_f64 %0, %0, %1" : "+v"(d4) : "v"(y));
               asm volatile("v_ldexp_f64 %0, %0, %1" : "+v"(d5) : "v"(y));
               asm volatile("v_ldexp_f64 %0, %0, %1" : "+v"(d6) : "v"(y));
               asm volatile("v_ldexp_f64 %0, %0, %1" : "+v"(d7) : "v"(y));)
        } else {  // one dependent fp64 chain (latency)
            R8(asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(d0) : "v"(b), "v"(c));)
        }
    }
    long long t1 = clock64();
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
    out[blockIdx.x * blockDim.x + threadIdx.x] = d0 + d1 + d2 + d3 + d4 + d5 + d6 + d7 + x0 + x1 + x2 + x3 + x4 + x5 + x6 + x7;
}

int main() {
    const int iters = 2000, blocks = 256;
    long long *cyc;
    double *out;
    hipMalloc(&cyc, blocks * sizeof(long long));
    hipMalloc(&out, blocks * 1024 * sizeof(double));
    const char *names[] = {"v_fma_f64", "v_add_u32", "v_cndmask_b32", "fma_f64+add_u32 alt", "v_ldexp_f64", "fma_f64 dep chain"};
    const double insts[] = {64, 64, 64, 64, 64, 8};  // per iteration per wave
    for (int waves = 1; waves <= 16; waves *= 2) {  // waves per block = per CU (4 SIMDs)
        for (int kind = 0; kind < 6; ++kind) {
            auto fn = kind == 0 ? k<0> : kind == 1 ? k<1> : kind == 2 ? k<2> : kind == 3 ? k<3> : kind == 4 ? k<4> : k<5>;
            hipLaunchKernelGGL(fn, dim3(blocks), dim3(64 * waves), 0, 0, cyc, out, iters);
            hipEvent_t e0, e1;
            hipEventCreate(&e0);
            hipEventCreate(&e1);
            hipEventRecord(e0);
            hipLaunchKernelGGL(fn, dim3(blocks), dim3(64 * waves), 0, 0, cyc, out, iters);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            long long c[blocks];
            hipMemcpy(c, cyc, sizeof(c), hipMemcpyDeviceToHost);
            double avg = 0;
            for (int i = 0; i < blocks; ++i) avg += c[i];
            avg /= blocks;
            // waves per SIMD = waves/4 (>= 1); cycles per instruction per SIMD
            const double wps = waves < 4 ? 1.0 : waves / 4.0;
            printf("waves/CU %2d  %-22s  %7.2f cyc per wave-instr per SIMD (clock64), %.3f ms, clk %.2f GHz\n", waves,
                   names[kind], avg / (iters * insts[kind] * wps), ms, avg / (ms * 1e6));
        }
    }
    return 0;
}
