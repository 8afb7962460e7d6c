// exp_table.hpp -- the 2^(j/256) table of the demapper's steering exp (qamr_math.hpp::exp_fast).
//
// The root search of g_inv_search (noisemapper.pyx:310-345, qamr_math.hpp) steers Newton with the
// density of F_Y, which needs exp(-u^2) per mixture component; that exp never decides a comparison
// (the certified window carries its error), so a table exp of ~1 ulp is enough there:
// x = k ln2/256 + r, exp(x) = 2^(k>>8) 2^((k&255)/256) e^r.  Every exp whose result reaches an
// output is glibc's, restated bit for bit (glibc_math.hpp).
//
// The table (256 doubles, 2 KiB) is computed on the host in 80-bit long double and staged into
// LDS by every workgroup that uses it.
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

namespace qr {

constexpr int kExpBits = 8;  // 2^(j/256)
constexpr int kExpN = 1 << kExpBits;

struct MathTables {
    double exp2j[kExpN];  // 2^(j/256)
};

// Host: the table in 80-bit long double, rounded once to double.
inline void build_math_tables(MathTables *t) {
    for (int j = 0; j < kExpN; ++j) t->exp2j[j] = (double)exp2l((long double)j / (long double)kExpN);
}

// Copy the table from global memory into LDS (the whole workgroup participates).
__device__ __forceinline__ void stage_math_tables(MathTables *lds, const MathTables *__restrict__ g) {
    const double2 *src = reinterpret_cast<const double2 *>(g);
    double2 *dst = reinterpret_cast<double2 *>(lds);
    constexpr int n = sizeof(MathTables) / sizeof(double2);
    for (int i = threadIdx.x; i < n; i += blockDim.x) dst[i] = src[i];
    __syncthreads();
}

}  // namespace qr
