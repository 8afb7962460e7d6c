// Host harness for fastmath.hpp: h(t) = log(1 + exp(-t)) and the box-plus built on it
// against the reference expressions with glibc exp/log (decoder.pyx:41-45).
// Compiled by tests/test_fastmath.py with hipcc as host code.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include "qamr_math.hpp"

static double h_ref(double t) { return log(1.0 + exp(-t)); }

int main(int argc, char **argv) {
    const long n = argc > 1 ? atol(argv[1]) : 2000000;
    qr::MathTables T;
    qr::build_math_tables(&T);
    std::mt19937_64 g(7);
    std::uniform_real_distribution<double> U(0.0, 40.0);
    double herr = 0, bperr = 0;
    long heq = 0, bad = 0;
    for (long i = 0; i < n; ++i) {
        double t = (i % 4 == 0) ? U(g) * 1e-3 : (i % 4 == 1) ? U(g) * 0.05 : U(g);
        if (i < 4096) t = i / 4096.0 * 40.0;
        const double a = h_ref(t), b = qr::h_softplus_neg(t, T);
        herr = fmax(herr, fabs(a - b));
        heq += (a == b);
        // box-plus on random operands of both signs and mixed magnitudes
        const double x = (U(g) - 20.0) * ((i & 8) ? 1.0 : 0.01), y = (U(g) - 20.0) * ((i & 16) ? 1.0 : 0.05);
        const double r = qr::box_plus(x, y), q = qr::box_plus_fast(x, y, T);
        bperr = fmax(bperr, fabs(r - q) / fmax(1.0, fabs(r)));
    }
    // special values: NaN propagates, inf gives 0 (exp(-inf) = 0), 0 gives log 2
    const double nan = std::nan("");
    if (!std::isnan(qr::h_softplus_neg(nan, T))) { puts("FAIL h(NaN) not NaN"); ++bad; }
    if (qr::h_softplus_neg(INFINITY, T) != 0.0) { puts("FAIL h(inf) != 0"); ++bad; }
    if (fabs(qr::h_softplus_neg(0.0, T) - log(2.0)) > 2.3e-16) { puts("FAIL h(0)"); ++bad; }
    if (!std::isnan(qr::box_plus_fast(nan, 1.0, T)) || !std::isnan(qr::box_plus_fast(1.0, nan, T))) { puts("FAIL bp NaN"); ++bad; }
    if (!std::isnan(qr::box_plus_fast(INFINITY, -INFINITY, T))) { puts("FAIL bp(inf,-inf)"); ++bad; }
    if (qr::box_plus_fast(INFINITY, 2.5, T) != qr::box_plus(INFINITY, 2.5)) { puts("FAIL bp(inf,2.5)"); ++bad; }
    printf("h: max|err|=%.3g (%.2f ulp(1)) bit-equal=%.1f%%  box_plus: max rel err=%.3g\n", herr,
           herr / 2.220446049250313e-16, 100.0 * heq / n, bperr);
    if (!(herr <= 2.220446049250313e-16)) { puts("FAIL h error > ulp(1)"); ++bad; }
    if (!(bperr <= 8.9e-16)) { puts("FAIL box_plus error > 4 ulp(1)"); ++bad; }
    return bad ? 1 : 0;
}
