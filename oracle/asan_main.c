/* oracle/asan_main.c -- TEST INFRASTRUCTURE: drives the C restatement (qamr_oracle.c)
 * under AddressSanitizer + UndefinedBehaviorSanitizer (`make -C oracle asan`, run by
 * tests/test_sanitizers.py): Tanner-graph build with parallel edges and high degrees,
 * node rules, batched decode incl. inf/NaN/-0.0 LAPPRs, syndrome, error count, the
 * NoiseMapper tables, demap, hard decision, noise mapping and Gray bits for 1..4 bits
 * per symbol.  Any sanitizer report aborts (-fno-sanitize-recover=all). */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

typedef struct orc_code orc_code;
typedef struct orc_nm orc_nm;
int orc_code_create(const int64_t *e_to_v, const int64_t *e_to_c, int64_t E, orc_code **out);
void orc_code_destroy(orc_code *g);
void orc_code_info(const orc_code *g, int64_t *V, int64_t *C, int64_t *E, int64_t *max_dc);
void orc_process_check_node(const orc_code *g, int64_t c, const uint8_t *synd, double *c2v, const double *v2c,
                            double *buf);
void orc_process_var_node(const orc_code *g, int64_t v, const double *lappr, const double *c2v, double *v2c,
                          double *post);
int orc_decode_batch(const orc_code *g, int64_t B, const double *lappr, const uint8_t *synd, int max_it,
                     double *final, uint8_t *success, int32_t *iters, int nthreads);
void orc_eval_syndrome(const orc_code *g, const uint8_t *word, uint8_t *synd);
int64_t orc_count_errors_from_lappr(const double *lappr, const uint8_t *word, int64_t n);
int orc_nm_create(int bps, double step, const double *probabilities, double noise_var, const uint8_t *sign_config,
                  orc_nm **out);
void orc_nm_destroy(orc_nm *nm);
int64_t orc_demap_lappr_array(const orc_nm *nm, const double *n, const int64_t *j, int64_t S, double *lappr,
                              int nthreads);
void orc_hard_decide_index(const orc_nm *nm, const double *y, int64_t S, int64_t *xhat);
void orc_map_noise(const orc_nm *nm, const double *y, const int64_t *xhat, int64_t S, double *n);
void orc_symbols_to_bits(int bps, const int64_t *x, int64_t S, uint8_t *bits);

static uint64_t rs = 88172645463325252ull;
static uint64_t rnd(void) {
    rs ^= rs << 13;
    rs ^= rs >> 7;
    rs ^= rs << 17;
    return rs;
}
static double unif(void) { return (double)(rnd() >> 11) * 0x1p-53; }
static double gauss(void) { return sqrt(-2 * log(unif() + 1e-300)) * cos(6.283185307179586 * unif()); }

int main(void) {
    int fails = 0;
    for (int rep = 0; rep < 6; ++rep) {
        const int C = 40 + (int)(rnd() % 60), V = 120;
        int64_t *vid = malloc(sizeof(int64_t) * 20000), *cid = malloc(sizeof(int64_t) * 20000);
        int64_t E = 0;
        for (int c = 0; c < C; ++c) {
            const int d = 2 + (int)(rnd() % (rep == 5 ? 90 : 8));
            for (int k = 0; k < d; ++k) {
                vid[E] = (int64_t)(rnd() % V);
                cid[E++] = c;
            }
        }
        for (int v = 0; v < V; ++v) vid[v % E] = v; /* every variable used */
        orc_code *g = NULL;
        if (orc_code_create(vid, cid, E, &g)) {
            printf("FAIL code_create\n");
            return 1;
        }
        int64_t VV, CC, EE, maxdc;
        orc_code_info(g, &VV, &CC, &EE, &maxdc);
        const int B = 5;
        double *llr = malloc(sizeof(double) * B * VV), *fin = malloc(sizeof(double) * B * VV);
        uint8_t *word = malloc(B * VV), *synd = malloc(B * CC), *succ = malloc(B);
        int32_t *its = malloc(sizeof(int32_t) * B);
        for (int f = 0; f < B; ++f) {
            for (int64_t v = 0; v < VV; ++v) {
                word[f * VV + v] = rnd() & 1;
                llr[f * VV + v] = 4.0 * ((1 - 2.0 * word[f * VV + v]) + 0.8 * gauss());
            }
            orc_eval_syndrome(g, word + f * VV, synd + f * CC);
        }
        llr[0] = INFINITY;
        llr[1] = -INFINITY;
        llr[2] = NAN;
        llr[3] = -0.0;
        orc_decode_batch(g, B, llr, synd, 20, fin, succ, its, 1);
        fails += orc_count_errors_from_lappr(fin, word, VV) < 0;
        double *c2v = malloc(sizeof(double) * EE), *v2c = malloc(sizeof(double) * EE), *post = malloc(sizeof(double) * VV);
        double *buf = malloc(sizeof(double) * (2 * maxdc + 2));
        for (int64_t e = 0; e < EE; ++e) {
            c2v[e] = gauss();
            v2c[e] = 3 * gauss();
        }
        for (int64_t c = 0; c < CC; ++c) orc_process_check_node(g, c, synd, c2v, v2c, buf);
        for (int64_t v = 0; v < VV; ++v) orc_process_var_node(g, v, llr, c2v, v2c, post);
        free(c2v); free(v2c); free(post); free(buf);
        free(llr); free(fin); free(word); free(synd); free(succ); free(its);
        free(vid); free(cid);
        orc_code_destroy(g);
    }
    for (int bps = 1; bps <= 4; ++bps) {
        const int M = 1 << bps;
        uint8_t sign[16];
        for (int i = 0; i < M; ++i) sign[i] = i & 1;
        double Es = 0;
        for (int i = 0; i < M; ++i) {
            const double a = (i - (M - 1) / 2.0) * 2.0;
            Es += a * a / M;
        }
        for (int s = 0; s < 3; ++s) {
            const double snr = s == 0 ? 0.0 : s == 1 ? 13.0 : 25.0;
            orc_nm *nm = NULL;
            if (orc_nm_create(bps, 2.0, NULL, Es * pow(10, -snr / 10) / 2, sign, &nm)) {
                printf("FAIL nm_create\n");
                return 1;
            }
            const int64_t S = 64;
            double y[64], n[64], out[64 * 4];
            int64_t x[64], xh[64];
            uint8_t bits[64 * 4];
            for (int64_t k = 0; k < S; ++k) {
                x[k] = (int64_t)(rnd() % M);
                y[k] = (x[k] - (M - 1) / 2.0) * 2.0 + sqrt(Es * pow(10, -snr / 10) / 2) * gauss();
            }
            orc_hard_decide_index(nm, y, S, xh);
            orc_map_noise(nm, y, xh, S, n);
            orc_demap_lappr_array(nm, n, x, S, out, 1);
            orc_symbols_to_bits(bps, xh, S, bits);
            orc_nm_destroy(nm);
        }
    }
    printf("oracle_asan: %d failures\n", fails);
    return fails ? 1 : 0;
}
