// Host harness for glibc_math.hpp: the restated exp/log/h/box-plus must return the
// same bits as the host libm (the reference's arithmetic, decoder.pyx:41-45) on every
// input.  Compiled by tests/test_glibc_math.py with hipcc as host code.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>

#include "glibc_math.hpp"
#include "qamr_math.hpp"

static uint64_t bits(double x) {
    uint64_t u;
    memcpy(&u, &x, 8);
    return u;
}
static bool same(double a, double b) { return bits(a) == bits(b) || (std::isnan(a) && std::isnan(b)); }

struct Count {
    const char *what;
    long n = 0, bad = 0;
    void check(double ref, double got, double arg, double arg2 = 0) {
        ++n;
        if (!same(ref, got)) {
            if (bad < 5) printf("  %s mismatch: arg=%a %a ref=%a got=%a\n", what, arg, arg2, ref, got);
            ++bad;
        }
    }
    long report() const {
        printf("%-10s %10ld inputs, %ld mismatches\n", what, n, bad);
        return bad;
    }
};

int main(int argc, char **argv) {
    const long n = argc > 1 ? atol(argv[1]) : 4000000;
    qr::GlibcTables T;
    qr::build_glibc_tables(&T);
    {  // the generated constant initializer (device __constant__ copy) == the host builder
        static const qr::GlibcTables init = QR_GLIBC_TABLES_INIT;
        if (memcmp(&init, &T, sizeof(T)) != 0) {
            puts("FAIL QR_GLIBC_TABLES_INIT differs from build_glibc_tables");
            return 1;
        }
    }
    std::mt19937_64 g(11);
    std::uniform_real_distribution<double> U(0.0, 1.0);
    Count ce{"exp"}, cl{"log"}, ch{"h"}, cb{"box_plus"};

    // exp: the box-plus domain x = -t, t in [0, 40] (dense), |x| in [2^-60, 512) log-uniform, both signs
    for (long i = 0; i < n; ++i) {
        const double x = -40.0 * U(g);
        ce.check(exp(x), qr::g_exp(x, T), x);
        const double y = (g() & 1 ? -1.0 : 1.0) * exp2(-60.0 + 69.0 * U(g));
        ce.check(exp(y), qr::g_exp(y, T), y);
    }
    for (int k = -128 * 40; k <= 0; ++k) {  // interval boundaries k ln2 / 128
        const double x = k * 0x1.62e42fefa39efp-1 / 128.0;
        ce.check(exp(x), qr::g_exp(x, T), x);
        ce.check(exp(nextafter(x, 0.0)), qr::g_exp(nextafter(x, 0.0), T), x);
    }
    for (double x : {0.0, -0.0, 0x1p-54, -0x1p-54, 0x1p-55, -0x1p-1074, -40.0})
        ce.check(exp(x), qr::g_exp(x, T), x);
    // the box-plus specialisation (no tiny-argument branch): [-37.51, 0] incl. tiny and zero
    Count cn{"exp_neg"};
    for (long i = 0; i < n; ++i) {
        const double x = (i & 1) ? -37.51 * U(g) : -exp2(-1074.0 + 1080.0 * U(g));
        cn.check(exp(x), qr::g_exp_neg(x, T), x);
    }
    for (double x : {0.0, -0.0, -0x1p-54, -0x1p-55, -0x1p-1074, -37.5, -0x1.2c00000000000p+5})
        cn.check(exp(x), qr::g_exp_neg(x, T), x);
    if (cn.report()) return 1;

    // log: u = 1 + exp(-t) (the box-plus domain), [1, 2] uniform, near-1 window, random normals
    for (long i = 0; i < n; ++i) {
        const double t = (i & 1) ? 40.0 * U(g) : 4.0 * U(g);
        const double u = 1.0 + exp(-t);
        cl.check(log(u), qr::g_log(u, T), u);
        const double v = 1.0 + U(g);
        cl.check(log(v), qr::g_log(v, T), v);
        const double w = 0.9375 + 0.127 * U(g);
        cl.check(log(w), qr::g_log(w, T), w);
        uint64_t b = (g() & 0x000FFFFFFFFFFFFFull) | ((uint64_t)(1 + g() % 2046) << 52);
        double z;
        memcpy(&z, &b, 8);
        cl.check(log(z), qr::g_log(z, T), z);
        cl.check(log(u), qr::g_log_u(u, T), u);
        cl.check(log(v), qr::g_log_u(v, T), v);
        cl.check(log(u), qr::g_log_u_sel(u, T), u);
        cl.check(log(v), qr::g_log_u_sel(v, T), v);
    }
    for (double x : {1.0, 2.0, nextafter(1.0, 2.0), nextafter(2.0, 1.0), 1.0 + 0x1.09p-4, nextafter(1.0 + 0x1.09p-4, 1.0)})
    {
        cl.check(log(x), qr::g_log_u(x, T), x);
        cl.check(log(x), qr::g_log_u_sel(x, T), x);
    }
    if (!std::isnan(qr::g_log_u(std::nan(""), T)) || !std::isnan(qr::g_log_u(-std::nan(""), T)) ||
        !std::isnan(qr::g_log_u_sel(std::nan(""), T)) || !std::isnan(qr::g_log_u_sel(-std::nan(""), T))) {
        puts("FAIL g_log_u(NaN) not NaN");
        return 1;
    }
    for (double x : {1.0, 2.0, nextafter(1.0, 2.0), nextafter(2.0, 1.0), 1.0 + 0x1.09p-4, nextafter(1.0 + 0x1.09p-4, 1.0),
                     1.0 - 0x1p-4, 0x1p-1022, 0x1.fffffffffffffp1023})
        cl.check(log(x), qr::g_log(x, T), x);

    // h(t) = log(1.0 + exp(-t)) incl. 0, inf, NaN and the clamp region
    for (long i = 0; i < n; ++i) {
        const double t = (i % 3 == 0) ? 45.0 * U(g) : (i % 3 == 1) ? 3.0 * U(g) : exp2(-60.0 + 66.0 * U(g));
        ch.check(log(1.0 + exp(-t)), qr::h_strict(t, T), t);
        ch.check(log(1.0 + exp(-t)), qr::h_strict<true>(t, T), t);
        ch.check(log(1.0 + exp(-t)), qr::h_strict(-t, T), -t);  // h(|s|)
    }
    for (double t : {0.0, 36.0, 36.7, 36.75, 37.0, 40.0, 41.0, 700.0, 1e300, (double)INFINITY, std::nan("")})
    {
        ch.check(log(1.0 + exp(-t)), qr::h_strict(t, T), t);
        ch.check(log(1.0 + exp(-t)), qr::h_strict<true>(t, T), t);
    }

    // box-plus: random operands of both signs, mixed magnitudes, zeros, equal magnitudes, inf/NaN
    const double sc[] = {1e-9, 1e-3, 0.3, 2.0, 8.0, 30.0, 200.0, 1e6};
    for (long i = 0; i < n; ++i) {
        double a = (2 * U(g) - 1) * sc[g() % 8], b = (2 * U(g) - 1) * sc[g() % 8];
        if ((i & 63) == 1) b = -a;
        if ((i & 63) == 2) b = a;
        if ((i & 127) == 3) a = 0.0;
        if ((i & 127) == 4) b = -0.0;
        cb.check(qr::box_plus(a, b), qr::box_plus_strict_t<false>(a, b, T), a, b);
        cb.check(qr::box_plus(a, b), qr::box_plus_strict_t<true>(a, b, T), a, b);
    }
    const double sp[] = {0.0, -0.0, 1.5, -2.25, 40.0, (double)INFINITY, -(double)INFINITY, std::nan("")};
    for (double a : sp)
        for (double b : sp) {
            cb.check(qr::box_plus(a, b), qr::box_plus_strict_t<false>(a, b, T), a, b);
            cb.check(qr::box_plus(a, b), qr::box_plus_strict_t<true>(a, b, T), a, b);
        }

    // full-range exp/log (demapper): random bit patterns over every exponent, specials, subnormals
    Count cef{"exp_full"}, clf{"log_full"};
    for (long i = 0; i < n; ++i) {
        uint64_t b = g();
        double x;
        memcpy(&x, &b, 8);
        cef.check(exp(x), qr::g_exp_full(x, T), x);
        clf.check(log(x), qr::g_log_full(x, T), x);
        const double y = (2 * U(g) - 1) * 760.0;  // over/underflow, subnormal results
        cef.check(exp(y), qr::g_exp_full(y, T), y);
        const double z = (2 * U(g) - 1) * 40.0;
        cef.check(exp(z), qr::g_exp_full(z, T), z);
        const double w = exp2(-1074.0 + 2100.0 * U(g));  // positive, subnormal..huge
        clf.check(log(w), qr::g_log_full(w, T), w);
        const double v = 0.9 + 0.2 * U(g);
        clf.check(log(v), qr::g_log_full(v, T), v);
    }
    for (double x : {0.0, -0.0, (double)INFINITY, -(double)INFINITY, std::nan(""), 709.78, 709.79, -708.4, -745.1,
                     -745.2, -1e5, 1e5, 512.0, -512.0, 1023.9, -1023.9, 1024.0, -1024.0, 0x1p-1074, -0x1p-1074, 1.0,
                     0x1p-1022, 0x1.fffffffffffffp1023, -1.0})
        for (double v : {x, nextafter(x, 0.0), nextafter(x, INFINITY)}) {
            cef.check(exp(v), qr::g_exp_full(v, T), v);
            clf.check(log(v), qr::g_log_full(v, T), v);
        }

    long bad = ce.report() + cl.report() + ch.report() + cb.report() + cef.report() + clf.report();
    if (bad) puts("FAIL glibc_math restatement differs from libm");
    return bad ? 1 : 0;
}
