// Host-side code of libqamr under AddressSanitizer + UndefinedBehaviorSanitizer
// (tests/test_sanitizers.py builds it with -Xarch_host -fsanitize=address,undefined and
// -fno-sanitize-recover: any report aborts with a non-zero status).
//
//   * build_tanner_csr (host_build.hpp; decoder.pyx:60-146) on random codes with parallel
//     edges, irregular and high degrees, plus the rejected inputs (size mismatch, negative
//     ids, degree < 2, empty);
//   * the table builders: build_glibc_tables, build_math_tables, build_demap_host
//     (noisemapper.pyx:103-236, Newton-start and Taylor tables) for 1..5 bits per symbol;
//   * the per-symbol demapper (qamr_math.hpp demap_symbol, noisemapper.pyx:450-540) on the
//     host over random inputs, fast root search against the brute one: identical bits.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "host_build.hpp"

using namespace qr;

static int fails = 0;
#define EXPECT(c, ...)                  \
    do {                                \
        if (!(c)) {                     \
            printf("FAIL: " __VA_ARGS__); \
            printf("\n");               \
            ++fails;                    \
        }                               \
    } while (0)

static void check_csr(std::mt19937_64 &g) {
    for (int rep = 0; rep < 40; ++rep) {
        const int C = 1 + (int)(g() % 300), V = 2 + (int)(g() % 500);
        std::vector<int64_t> vid, cid;
        for (int c = 0; c < C; ++c) {
            const int d = 2 + (int)(g() % (rep % 5 == 0 ? 120 : 9));
            for (int k = 0; k < d; ++k) {
                cid.push_back(c);
                vid.push_back((int64_t)(g() % V));  // parallel edges happen
            }
        }
        // shuffle the edge order (the builder must sort stably by node id)
        for (size_t i = vid.size(); i > 1; --i) {
            const size_t j = g() % i;
            std::swap(vid[i - 1], vid[j]);
            std::swap(cid[i - 1], cid[j]);
        }
        TannerCsr t;
        std::string err;
        const int rc = build_tanner_csr(vid.data(), cid.data(), (int64_t)vid.size(), (int64_t)cid.size(), t, err);
        EXPECT(rc == QR_OK, "csr rc %d (%s)", rc, err.c_str());
        if (rc) continue;
        // every check's edges ascending, chk_var consistent, var lists ascending
        for (int64_t c = 0; c < t.C; ++c)
            for (int k = t.chk_ptr[c]; k < t.chk_ptr[c + 1]; ++k) {
                EXPECT(cid[t.chk_edge[k]] == c, "edge in wrong check");
                EXPECT(vid[t.chk_edge[k]] == t.chk_var[k], "c_to_v mismatch");
                if (k > t.chk_ptr[c]) EXPECT(t.chk_edge[k] > t.chk_edge[k - 1], "check edges not ascending");
            }
        for (int64_t v = 0; v < t.V; ++v)
            for (int k = t.var_ptr[v] + 1; k < t.var_ptr[v + 1]; ++k)
                EXPECT(t.var_edge[k] > t.var_edge[k - 1], "variable edges not ascending");
    }
    TannerCsr t;
    std::string err;
    const int64_t v2[] = {0, 1, 2}, c2[] = {0, 0, 1};
    EXPECT(build_tanner_csr(v2, c2, 3, 2, t, err) == QR_EVALUE && err == "Sizes don't match", "size mismatch");
    EXPECT(build_tanner_csr(v2, c2, 3, 3, t, err) == QR_EVALUE, "degree-1 check accepted");
    const int64_t vn[] = {0, -1}, cn[] = {0, 0};
    EXPECT(build_tanner_csr(vn, cn, 2, 2, t, err) == QR_EVALUE, "negative id accepted");
    EXPECT(build_tanner_csr(v2, c2, 0, 0, t, err) == QR_EVALUE, "empty accepted");
}

template <int BPS>
static void check_demap_bps(std::mt19937_64 &g, const DemapTables &t, const MathTables &mt, const GlibcTables &gt,
                            int draws) {
    constexpr int M = 1 << BPS;
    std::uniform_real_distribution<double> U(0.0, 1.0);
    for (int i = 0; i < draws; ++i) {
        const double n = U(g);
        const int j = (int)(g() % M);
        double a[BPS], b[BPS];
        demap_symbol<true, BPS>(t, mt, gt, n, j, 1.0, a);
        demap_symbol<false, BPS>(t, mt, gt, n, j, 1.0, b);
        for (int k = 0; k < BPS; ++k) {
            uint64_t x, y;
            memcpy(&x, &a[k], 8);
            memcpy(&y, &b[k], 8);
            EXPECT(x == y || (std::isnan(a[k]) && std::isnan(b[k])), "demap fast != brute (bps %d, n %a, j %d)", BPS,
                   n, j);
        }
    }
}

static void check_demap(std::mt19937_64 &g) {
    MathTables mt;
    build_math_tables(&mt);
    static GlibcTables gt;
    build_glibc_tables(&gt);
    for (int bps = 1; bps <= 5; ++bps) {
        const int M = 1 << bps;
        std::vector<double> a(M), thr(M + 1);
        double Es = 0;
        for (int i = 0; i < M; ++i) {
            a[i] = ((double)i - (M - 1) / 2.0) * 2.0;  // alphabet.pyx:62
            Es += a[i] * a[i] / M;
        }
        for (int i = 1; i < M; ++i) thr[i] = a[i] - 1.0;  // alphabet.pyx:69-73
        thr[0] = 100 * a[0];
        thr[M] = 100 * a[M - 1];
        std::vector<uint8_t> sign(M);
        for (int i = 0; i < M; ++i) sign[i] = i & 1;
        for (double snr : {0.0, 3.0, 13.0, 25.0}) {
            const double nv = Es * pow(10.0, -snr / 10) / 2;
            DemapTables t;
            std::vector<double2> quant;
            std::vector<double> ftab;
            std::string err;
            const int rc = build_demap_host(bps, a.data(), nullptr, thr.data(), nv, sign.data(), t, quant, ftab, err);
            EXPECT(rc == QR_OK, "demap tables rc %d (%s)", rc, err.c_str());
            if (rc) continue;
            t.quant = quant.empty() ? nullptr : quant.data();  // host evaluation reads the host copies
            t.ftab = ftab.empty() ? nullptr : ftab.data();
            const int draws = bps <= 2 ? 300 : bps == 3 ? 120 : 40;
            switch (bps) {
                case 1: check_demap_bps<1>(g, t, mt, gt, draws); break;
                case 2: check_demap_bps<2>(g, t, mt, gt, draws); break;
                case 3: check_demap_bps<3>(g, t, mt, gt, draws); break;
                case 4: check_demap_bps<4>(g, t, mt, gt, draws); break;
                default: check_demap_bps<5>(g, t, mt, gt, draws); break;
            }
        }
    }
    DemapTables t;
    std::vector<double2> q;
    std::vector<double> f;
    std::string err;
    const double a2[] = {-1, 1}, th[] = {-100, 0, 100};
    EXPECT(build_demap_host(0, a2, nullptr, th, 1.0, nullptr, t, q, f, err) == QR_EVALUE, "bps 0 accepted");
    EXPECT(build_demap_host(1, a2, nullptr, th, 0.0, nullptr, t, q, f, err) == QR_EVALUE, "noise_var 0 accepted");
}

int main() {
    std::mt19937_64 g(2024);
    check_csr(g);
    check_demap(g);
    printf("host_asan_check: %d failures\n", fails);
    return fails ? 1 : 0;
}
