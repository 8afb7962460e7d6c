// Host harness for fastmath.hpp: h(t) = log(1 + exp(-t)) and the box-plus built on it
// against the reference expressions with glibc exp/log (decoder.pyx:41-45).
// Compiled by tests/test_fastmath.py with hipcc as host code.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include "qamr_math.hpp"

static double h_ref(double t) { return log(1.0 + exp(-t)); }

// decoder.pyx:322-369 verbatim (glibc box-plus) for one degree-D check.
template <int D>
static void check_ref(const double (&m)[D], bool sb, double (&out)[D]) {
    double F[D], B[D];
    F[0] = m[0];
    for (int i = 1; i < D - 1; ++i) F[i] = qr::box_plus(F[i - 1], m[i]);
    B[D - 1] = m[D - 1];
    for (int i = D - 2; i > 0; --i) B[i] = qr::box_plus(B[i + 1], m[i]);
    const double s = sb ? -1.0 : 1.0;
    out[0] = s * B[1];
    for (int i = 1; i < D - 1; ++i) out[i] = s * qr::box_plus(F[i - 1], B[i + 1]);
    out[D - 1] = s * F[D - 2];
}

// The exp-domain check update (fastmath.hpp::check_node_eps) against the reference
// F/B recursion: every output within 4e-15 absolute + 4 ulp relative, the sign exact
// whenever the reference output is not within that bound of zero.
template <int D>
static long eps_case(const double (&m)[D], bool sb, const qr::MathTables &T, double &maxabs, double &maxrel) {
    double ref[D], got[D];
    check_ref<D>(m, sb, ref);
    qr::check_node_eps<D>(m, sb, T, [&](int i, double v) { got[i] = v; });
    long bad = 0;
    for (int i = 0; i < D; ++i) {
        const double d = fabs(got[i] - ref[i]);
        const double tol = 4e-15 + 8.9e-16 * fabs(ref[i]);
        maxabs = fmax(maxabs, d);
        if (fabs(ref[i]) > 1e-3) maxrel = fmax(maxrel, d / fabs(ref[i]));
        if (!(d <= tol) || (fabs(ref[i]) > tol && (got[i] < 0) != (ref[i] < 0))) {
            if (bad < 3) {
                printf("eps mismatch D=%d i=%d ref=%.17g got=%.17g m=", D, i, ref[i], got[i]);
                for (int k = 0; k < D; ++k) printf("%.17g ", m[k]);
                printf("\n");
            }
            ++bad;
        }
    }
    return bad;
}

static long check_eps_domain(long n, const qr::MathTables &T, std::mt19937_64 &g) {
    std::uniform_real_distribution<double> U(0.0, 1.0);
    double maxabs = 0, maxrel = 0;
    long bad = 0;
    const double scales[] = {1e-12, 1e-3, 0.1, 1.0, 5.0, 20.0, 60.0, 300.0, 699.0};
    for (long it = 0; it < n; ++it) {
        double m7[7], m2[2], m3[3];
        const double sc = scales[it % 9];
        for (double &x : m7) {
            x = (U(g) * 2 - 1) * sc * ((g() & 3) ? 1.0 : U(g));
            if ((g() & 31) == 0) x = 0.0;
            if ((g() & 63) == 0) x = -0.0;
        }
        if ((it & 7) == 3) m7[2] = m7[5];                      // equal operands
        if ((it & 7) == 5) m7[1] = -m7[4];
        if (sc > 600) for (double &x : m7) x = copysign(fmin(fabs(x), 700.0), x);
        for (int k = 0; k < 2; ++k) m2[k] = m7[k];
        for (int k = 0; k < 3; ++k) m3[k] = m7[k + 2];
        const bool sb = g() & 1;
        bad += eps_case<7>(m7, sb, T, maxabs, maxrel);
        bad += eps_case<2>(m2, sb, T, maxabs, maxrel);
        bad += eps_case<3>(m3, sb, T, maxabs, maxrel);
    }
    printf("eps-domain check update: %ld checks x {7,2,3}, max|err|=%.3g, max rel err (|ref|>1e-3)=%.3g, bad=%ld\n",
           n, maxabs, maxrel, bad);
    if (bad) puts("FAIL eps-domain check update");
    return bad ? 1 : 0;
}

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
    bad += check_eps_domain(n / 8, T, g);
    return bad ? 1 : 0;
}
