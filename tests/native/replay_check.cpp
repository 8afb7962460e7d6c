// Host harness: the fast g_inv_search (Newton + replayed bisection) must return
// bit-identical doubles to the brute-force reference search over random
// (n_hat, hypothesis, PAM order, SNR, sign configuration) draws.  Compiled by
// tests/test_demap_replay.py with hipcc as host code (glibc exp inside erf).
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <cmath>
#include <random>
#include "qamr_math.hpp"

int main(int argc, char** argv) {
    const long draws = argc > 1 ? atol(argv[1]) : 200000;
    std::mt19937_64 g(12345);
    std::uniform_real_distribution<double> U(0.0, 1.0);
    long mism = 0, fallback = 0, total = 0;
    long evals_fast = 0;
    for (int bps = 1; bps <= 4; ++bps) {
        const int M = 1 << bps;
        for (double snr : {-2.0, 3.0, 9.5, 13.0, 25.0, 40.0}) {
            qr::DemapTables t;
            memset(&t, 0, sizeof t);
            t.M = M; t.bps = bps;
            double Es = 0;
            for (int i = 0; i < M; ++i) {
                t.a[i] = ((double)i - (double)(M - 1) / 2.0) * 2.0;
                t.p[i] = 1.0 / M;
                Es += t.p[i] * (t.a[i] * t.a[i]);
                t.sign[i] = (uint8_t)(g() & 1);
            }
            for (int i = 1; i < M; ++i) t.thr[i] = t.a[i] - 1.0;
            t.thr[0] = t.a[0] * 100; t.thr[M] = t.a[M - 1] * 100;
            const double nv = Es * pow(10.0, -snr / 10) / 2;
            t.den = sqrt(2.0) * sqrt(nv); t.two_s2 = 2 * nv;
            t.Fthr[0] = 0; t.Fthr[M] = 1;
            for (int i = 1; i < M; ++i) t.Fthr[i] = qr::single_F_Y(t, t.thr[i]);
            for (int i = 0; i < M; ++i) t.dF[i] = t.Fthr[i + 1] - t.Fthr[i];
            for (long d = 0; d < draws / 24; ++d) {
                double n = U(g);
                if (d % 97 == 0) n = (d % 2) ? 0.0 : 1.0;
                if (d % 101 == 0) n = U(g) * 1e-12;
                const int i = (int)(g() % M);
                const double a = qr::g_inv_search(t, n, i);
                qr::SearchCmp cmp{&t, qr::search_target(t, n, i), 0.0, 0.0, false};
                cmp.have = qr::newton_root(t, cmp.T, cmp.ystar, cmp.W);
                if (!cmp.have) ++fallback;
                const double b = qr::g_inv_search_fast(t, n, i);
                ++total;
                if (memcmp(&a, &b, 8) != 0 && !(std::isnan(a) && std::isnan(b))) {
                    if (mism < 10) printf("MISMATCH bps=%d snr=%g n=%.17g i=%d ref=%.17g fast=%.17g W=%g\n",
                                          bps, snr, n, i, a, b, cmp.W);
                    ++mism;
                }
            }
        }
    }
    (void)evals_fast;
    printf("draws=%ld mismatches=%ld fallbacks=%ld\n", total, mism, fallback);
    return mism ? 1 : 0;
}
