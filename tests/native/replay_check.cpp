// Host harness: the fast g_inv_search (Newton + replayed bisection) must return
// bit-identical doubles to the brute-force reference search over random
// (n_hat, hypothesis, PAM order, SNR, sign configuration) draws.  Compiled by
// tests/test_demap_replay.py with hipcc as host code (glibc exp inside erf).
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <cmath>
#include <random>
#include <vector>
#include "qamr_math.hpp"

int main(int argc, char** argv) {
    const long draws = argc > 1 ? atol(argv[1]) : 200000;
    std::mt19937_64 g(12345);
    std::uniform_real_distribution<double> U(0.0, 1.0);
    long mism = 0, fallback = 0, total = 0, near_grid = 0;
    long evals_fast = 0;
    qr::MathTables mt;
    qr::build_math_tables(&mt);
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
            for (int i = 0; i < M; ++i) t.inv_dF[i] = 1.0 / t.dF[i];
            t.inv_den = 1.0 / t.den; t.amin = t.a[0]; t.amax = t.a[M - 1];
            std::vector<double2> quant((size_t)M * qr::kQStride);
            qr::build_quantiles(t, quant.data());
            t.quant = quant.data();
            std::vector<double> ftab; double fw = 0;
            if (qr::build_ftab(t, ftab, t.ftab_n, t.ftab_lo, fw, t.ftab_err)) { t.ftab = ftab.data(); t.ftab_inv_w = 1 / fw; t.ftab_h = fw / 2; t.ftab_inv_h = 2 / fw; }
            for (long d = 0; d < draws / 24; ++d) {
                double n = U(g);
                int i = (int)(g() % M);
                if (d % 97 == 0) n = (d % 2) ? 0.0 : 1.0;
                if (d % 101 == 0) n = U(g) * 1e-12;
                if (d % 3 == 1) {
                    // adversarial: the root sits within ~1e-12 of a bisection grid point
                    // (lo + j 2^-30), where the window decisions need exact F_Y
                    const double y0 = fmax(t.thr[i], t.a[i] - 3.0) + U(g) * (fmin(t.thr[i + 1], t.a[i] + 3.0) - fmax(t.thr[i], t.a[i] - 3.0));
                    const double off[] = {0.0, 1e-15, -1e-15, 1e-13, -1e-13, 3e-12, -3e-12, 1e-11};
                    const double yg = ldexp(floor(ldexp(y0, 30)), -30) + off[g() % 8];
                    const double T = qr::single_F_Y(t, yg);
                    n = t.sign[i] ? (t.Fthr[i + 1] - T) / t.dF[i] : (T - t.Fthr[i]) / t.dF[i];
                    if (!(n >= 0.0 && n <= 1.0)) n = U(g);
                }
                const double a = qr::g_inv_search(t, n, i);
                qr::SearchCmp cmp{&t, qr::search_target(t, n, i), 0.0, 0.0, false};
                cmp.have = qr::newton_root(t, mt, cmp.T, i, cmp.ystar, cmp.W);
                if (!cmp.have) ++fallback;
                else {
                    const double c = ldexp(floor(ldexp(cmp.ystar, 30) + 0.5), -30);
                    if (fabs(c - cmp.ystar) <= cmp.W) ++near_grid;
                }
                const double b = qr::g_inv_search_fast(t, mt, n, i);
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
    printf("draws=%ld mismatches=%ld fallbacks=%ld window-on-grid=%ld\n", total, mism, fallback, near_grid);
    return mism ? 1 : 0;
}
