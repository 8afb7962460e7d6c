// host_build.hpp -- the host-side construction steps of libqamr, free of HIP runtime
// calls so that they also build and run in a sanitizer harness
// (tests/native/host_asan_check.cpp, tests/test_sanitizers.py):
//
//   build_tanner_csr   Decoder.__cinit__ / __build_table (decoder.pyx:60-146): O(E) stable
//                      counting sort of the edge list into int32 CSR per check and per
//                      variable (ascending edge id), checks grouped by degree;
//   build_demap_host   NoiseMapper.__cinit__ tables (noisemapper.pyx:103-236) plus the
//                      Newton-start and Taylor tables of the fast root search.
#pragma once
#include <math.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <cstdio>
#include <string>
#include <vector>

#include "qamr.h"
#include "qamr_math.hpp"

namespace qr {

struct TannerCsr {
    int64_t E = 0, V = 0, C = 0;
    int32_t max_dc = 0, max_dv = 0;
    std::vector<int32_t> chk_ptr, chk_edge, chk_var, var_ptr, var_edge;
    std::vector<std::vector<int32_t>> by_deg;  // check ids per degree, ascending
};

// Returns QR_OK or an error code with `err` set (the messages of the reference where it
// has one: decoder.pyx:96-97 "Sizes don't match").
inline int build_tanner_csr(const int64_t *e_to_v, const int64_t *e_to_c, int64_t nv, int64_t nc, TannerCsr &t,
                            std::string &err) {
    auto fail = [&](int code, const char *fmt, long long a = 0, long long b = 0) {
        char buf[256];
        snprintf(buf, sizeof buf, fmt, a, b);
        err = buf;
        return code;
    };
    if (nv != nc) return fail(QR_EVALUE, "Sizes don't match");
    const int64_t E = nv;
    if (E <= 0) return fail(QR_EVALUE, "empty edge list");
    if (!e_to_v || !e_to_c) return fail(QR_EVALUE, "null edge list");
    if (E >= (int64_t)1 << 31) return fail(QR_EUNSUPPORTED, "more than 2^31-1 edges");
    int64_t V = 0, C = 0;
    for (int64_t e = 0; e < E; ++e) {
        if (e_to_v[e] < 0 || e_to_c[e] < 0) return fail(QR_EVALUE, "negative node id at edge %lld", e);
        if (e_to_v[e] >= ((int64_t)1 << 31) - 1 || e_to_c[e] >= ((int64_t)1 << 31) - 1)
            return fail(QR_EUNSUPPORTED, "node ids exceed int32 (edge %lld)", e);
        V = std::max(V, e_to_v[e] + 1);
        C = std::max(C, e_to_c[e] + 1);
    }
    t.E = E;
    t.V = V;
    t.C = C;
    // Stable counting sort by node id == the ascending scan of __build_table (decoder.pyx:69-87).
    t.chk_ptr.assign(C + 1, 0);
    t.var_ptr.assign(V + 1, 0);
    t.chk_edge.resize(E);
    t.chk_var.resize(E);
    t.var_edge.resize(E);
    for (int64_t e = 0; e < E; ++e) {
        t.chk_ptr[e_to_c[e] + 1]++;
        t.var_ptr[e_to_v[e] + 1]++;
    }
    for (int64_t i = 0; i < C; ++i) t.chk_ptr[i + 1] += t.chk_ptr[i];
    for (int64_t i = 0; i < V; ++i) t.var_ptr[i + 1] += t.var_ptr[i];
    {
        std::vector<int32_t> fc(t.chk_ptr.begin(), t.chk_ptr.end() - 1), fv(t.var_ptr.begin(), t.var_ptr.end() - 1);
        for (int64_t e = 0; e < E; ++e) {
            const int32_t kc = fc[e_to_c[e]]++;
            t.chk_edge[kc] = (int32_t)e;
            t.chk_var[kc] = (int32_t)e_to_v[e];  // c_to_v (decoder.pyx:128-129)
            t.var_edge[fv[e_to_v[e]]++] = (int32_t)e;
        }
    }
    t.max_dc = t.max_dv = 0;
    t.by_deg.clear();
    for (int64_t c = 0; c < C; ++c) {
        const int32_t d = t.chk_ptr[c + 1] - t.chk_ptr[c];
        if (d < 2)
            return fail(QR_EVALUE,
                        "check node %lld has degree %lld; degree < 2 is undefined behaviour in the reference "
                        "(decoder.pyx:135-141) and is rejected",
                        c, d);
        t.max_dc = std::max(t.max_dc, d);
        if ((int)t.by_deg.size() <= d) t.by_deg.resize(d + 1);
        t.by_deg[d].push_back((int32_t)c);
    }
    for (int64_t v = 0; v < V; ++v) t.max_dv = std::max(t.max_dv, t.var_ptr[v + 1] - t.var_ptr[v]);
    return QR_OK;
}

// NoiseMapper tables on the host (noisemapper.pyx:103-236) and the fast root search's
// Newton-start (quant) and Taylor (ftab) tables; quant/ftab stay empty where the brute
// search is used.  t.quant / t.ftab are left null (device pointers are set on upload).
inline int build_demap_host(int32_t bps, const double *constellation, const double *probabilities,
                            const double *thresholds, double noise_var, const uint8_t *sign_config, DemapTables &t,
                            std::vector<double2> &quant, std::vector<double> &ftab, std::string &err) {
    if (bps < 1 || bps > kMaxBps) {
        err = "bit_per_symbol must be in [1, " + std::to_string(kMaxBps) + "], got " + std::to_string(bps);
        return QR_EVALUE;
    }
    if (!(noise_var > 0)) {  // noisemapper.pyx:111-112
        err = "noise variance must be strictly positive";
        return QR_EVALUE;
    }
    if (!constellation || !thresholds) {
        err = "null constellation/thresholds";
        return QR_EVALUE;
    }
    memset(&t, 0, sizeof t);
    const int M = 1 << bps;
    t.M = M;
    t.bps = bps;
    for (int i = 0; i < M; ++i) {
        t.a[i] = constellation[i];
        t.p[i] = probabilities ? probabilities[i] : 1.0 / M;  // alphabet.pyx:46-47
        t.sign[i] = sign_config ? sign_config[i] : 0;       // noisemapper.pyx:115-116
    }
    for (int i = 0; i <= M; ++i) t.thr[i] = thresholds[i];
    const double sigma = sqrt(noise_var);                     // noisemapper.pyx:132
    t.den = sqrt(2.0) * sigma;                                // __sqrt2 * sigma (:24, :67)
    t.two_s2 = 2 * noise_var;                                 // :469
    t.inv_two_s2 = 1.0 / t.two_s2;                            // div_two_s2
    t.Fthr[0] = 0;                                            // :149-153
    t.Fthr[M] = 1;
    for (int i = 1; i < M; ++i) t.Fthr[i] = single_F_Y(t, t.thr[i]);
    for (int i = 0; i < M; ++i) t.dF[i] = t.Fthr[i + 1] - t.Fthr[i];  // :159-162
    t.inv_den = 1.0 / t.den;
    for (int i = 0; i < M; ++i) t.inv_dF[i] = 1.0 / t.dF[i];          // Newton start only
    t.amin = t.amax = t.a[0];
    for (int i = 1; i < M; ++i) {
        t.amin = fmin(t.amin, t.a[i]);
        t.amax = fmax(t.amax, t.a[i]);
    }
    // Newton start table (qamr_math.hpp, build_quantiles): M * kQStride * M exact F_Y
    // bisections; beyond 32-PAM its cost grows as M^2 and the brute search is used.
    quant.clear();
    ftab.clear();
    if (M <= 32) {
        quant.resize((size_t)M * kQStride);
        build_quantiles(t, quant.data());
    }
    // Taylor table of F_Y for the Newton evaluation (qamr_math.hpp, build_ftab)
    double ftab_w = 0;
    if (!quant.empty() && build_ftab(t, ftab, t.ftab_n, t.ftab_lo, ftab_w, t.ftab_err)) {
        t.ftab_inv_w = 1.0 / ftab_w;
        t.ftab_h = ftab_w / 2;
        t.ftab_inv_h = 2.0 / ftab_w;
    } else {
        ftab.clear();
    }
    t.quant = nullptr;
    t.ftab = nullptr;
    return QR_OK;
}

}  // namespace qr
