// Host check of qamr_math.hpp::div_two_s2 (the demapper's x / (2 sigma^2), noisemapper.pyx:512-515):
// Markstein's reciprocal + one FMA correction must equal the IEEE division bit for bit over
// the demapper's argument range and beyond.  Compiled by tests/test_demap_replay.py.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>

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
    for (double b : {1.0, 2.0, 0.5, 3.0, 0x1.fffffffffffffp+0, 0x1.0000000000001p+0, 1e-6, 1e4})
        for (double x : {0.0, -0.0, 1.0, -1.0, 0x1.fffffffffffffp+0, 1e4, -1e4, 3.0, 7.0})
            one(x, b);
    printf("division: %ld inputs, mismatches=%ld\n", total, bad);
    return bad ? 1 : 0;
}
