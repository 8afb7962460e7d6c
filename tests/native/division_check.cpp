// Host check of qamr_math.hpp::div_two_s2 (the demapper's x / (2 sigma^2), noisemapper.pyx:512-515):
// reciprocal product + two FMA residual corrections must equal the IEEE division bit for bit over
// the demapper's argument range and beyond, incl. quotients whose significand is just below 2
// (where RN(x RN(1/b)) can be 2 ulp off) and the 2 sigma^2 the simulations configure.  Compiled by tests/test_demap_replay.py.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "qamr_math.hpp"

int main(int argc, char **argv) {
    const long n = argc > 1 ? atol(argv[1]) : 20000000;
    std::mt19937_64 g(99);
    std::uniform_real_distribution<double> U(0.0, 1.0);
    qr::DemapTables t;
    memset(&t, 0, sizeof t);
    long bad = 0, total = 0;
    auto one = [&](double x, double b) {
        t.two_s2 = b;
        t.inv_two_s2 = 1.0 / b;
        const double r = x / b, q = qr::div_two_s2(t, x);
        uint64_t u, v;
        memcpy(&u, &r, 8);
        memcpy(&v, &q, 8);
        ++total;
        // the one difference: -0 / b comes out +0 (q0 = -0, r = +0, +0 + -0 = +0); the
        // demapper only feeds the quotient to exp, and exp(+-0) = 1
        if (x == 0.0 && q == 0.0) return;
        if (u != v) {
            if (bad < 5) printf("mismatch x=%a b=%a ref=%a got=%a\n", x, b, r, q);
            ++bad;
        }
    };
    for (long i = 0; i < n; ++i) {
        // b = 2 sigma^2 over 1e-6 .. 1e4 (SNR -40 .. 60 dB for the PAM orders used); x over
        // the LLR exponents' range |x| <= 1e4 (log-uniform magnitudes) and random bit patterns
        // of the significand
        const double b = std::exp2(-20.0 + 33.0 * U(g));
        const double x = (g() & 1 ? -1.0 : 1.0) * std::exp2(-60.0 + 74.0 * U(g));
        one(x, b);
        uint64_t bits = (g() & 0x000FFFFFFFFFFFFFull) | (uint64_t)(1023 + (int)(g() % 24) - 12) << 52;
        double y;
        memcpy(&y, &bits, 8);
        one(y, b);
        one((double)(int64_t)(g() % 20001 - 10000), b);  // integer-valued products
    }
    // quotients with significands just below 2 (and just above 1) for random and configured b
    std::vector<double> bs;
    for (double Es : {1.0, 5.0, 21.0, 85.0})           // 2-, 4-, 8-, 16-PAM variance (step 2)
        for (int d = 0; d <= 80; ++d) bs.push_back(Es * std::pow(10.0, -0.5 * d / 10.0));  // 0..40 dB
    for (long i = 0; i < n / 20; ++i) bs.push_back(std::exp2(-20.0 + 33.0 * U(g)));
    long near2 = 0;
    for (double b : bs)
        for (int k = 1; k <= 24; ++k) {
            const int e = (int)(g() % 40) - 20;
            const double q_hi = std::ldexp(2.0 - k * 0x1p-52, e), q_lo = std::ldexp(1.0 + k * 0x1p-52, e);
            for (double q : {q_hi, q_lo}) {
                const double x = q * b;                // x/b lands within an ulp or two of q
                one(x, b);
                one(std::nextafter(x, 0.0), b);
                one(std::nextafter(x, 1e300), b);
                one(-x, b);
                near2 += 4;
            }
        }
    printf("near power-of-two quotients: %ld\n", near2);
    for (double b : {1.0, 2.0, 0.5, 3.0, 0x1.fffffffffffffp+0, 0x1.0000000000001p+0, 1e-6, 1e4})
        for (double x : {0.0, -0.0, 1.0, -1.0, 0x1.fffffffffffffp+0, 1e4, -1e4, 3.0, 7.0})
            one(x, b);
    printf("division: %ld inputs, mismatches=%ld\n", total, bad);
    return bad ? 1 : 0;
}
