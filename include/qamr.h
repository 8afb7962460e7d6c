/*
 * qamr.h -- C-ABI of libqamr.so, the MI355X (gfx950) LDPC syndrome decoder and
 * PAM/BICM soft demapper that replaces the hot path of
 * moriglia/qam-reconciliation.
 *
 * The reference exposes this path only as Cython extension types (no C-ABI):
 *   qamreconciliation.Decoder(e_to_v, e_to_c)            decoder.pyx:92-146
 *   Decoder.decode(lappr, synd, max_iterations)           decoder.pyx:441-455
 *   Decoder._decode(...)  (cdef, called by the sims)      decoder.pyx:391-436
 *   NoiseMapper(pa, noise_var, sign_config)               noisemapper.pyx:103-236
 *   NoiseMapper.demap_lappr_array(n, j)                   noisemapper.pyx:544-559
 * Every entry point below names the reference interface it replaces.  The
 * Python facade (qam-reconciliation_amd/qamr) binds these with ctypes; see
 * INTEGRATION.md for the binding a maintainer would add on the reference side.
 *
 * Conventions
 *  - Every function returns an int status (QR_OK = 0).  On error
 *    qr_last_error() returns a thread-local message.  Status -> Python:
 *    QR_EVALUE -> ValueError, QR_EMEMORY -> MemoryError, others -> RuntimeError.
 *  - "_host" functions take host (CPU) buffers, frame-major ([B][V] etc.), and
 *    run synchronously on the device the handle was created on.
 *  - "_device" functions take device (HBM) pointers in the FRAME-INNERMOST
 *    layout: element (node n, frame f) lives at ptr[n * ld + f], with
 *    B <= ld and ld a multiple of 64 (one wavefront = 64 frames).  They are
 *    asynchronous on `stream` (a hipStream_t; NULL = the null stream), make no
 *    allocation and no host synchronisation (graph-capturable).
 *  - All arithmetic is IEEE fp64, unfused, in the reference's operation order.
 */
#ifndef QAMR_H
#define QAMR_H
#include <stddef.h>
#include <stdint.h>

#if defined(__GNUC__)
#define QR_API __attribute__((visibility("default")))
#else
#define QR_API
#endif

#ifdef __cplusplus
extern "C" {
#endif

#define QR_OK 0
#define QR_EVALUE 1      /* -> ValueError  */
#define QR_EMEMORY 2     /* -> MemoryError */
#define QR_EDEVICE 3     /* HIP runtime error -> RuntimeError */
#define QR_EUNSUPPORTED 4

typedef struct qr_code qr_code;   /* Tanner graph resident in HBM   */
typedef struct qr_demap qr_demap; /* NoiseMapper tables in HBM      */

/* ------------------------------------------------------------------ misc */
QR_API const char *qr_last_error(void);
QR_API int qr_version(int32_t *major, int32_t *minor);
QR_API int qr_device_count(int32_t *count);

/* Per-kernel timing with hipEvents on the launch stream (bench.py uses it to
 * price the dominant kernel).  Off by default; zero cost when off. */
QR_API int qr_profile_enable(int32_t on);
QR_API int qr_profile_reset(void);
/* Restrict the timing to the launches whose profile name is in the comma-separated list
 * `names` (NULL or "" = every launch): the events of the other launches are not recorded
 * at all, so timing only the kernel being priced perturbs the stream less. */
QR_API int qr_profile_select(const char *names);
/* name: "check" (one check sweep, all degree classes), "check_d<D>" (the launch
 * for check degree D), "check1" (first sweep), "var", "var_init", "status",
 * "parity", "demap", "bob", "syndrome", "count".  Synchronises pending events. */
QR_API int qr_profile_query(const char *name, double *total_ms, int64_t *launches);

/* Kernel-geometry knobs (process-wide; performance only, results unchanged):
 * "check_ft"/"var_ft" frames per workgroup (64/128/256), "check_per"/"var_per"
 * nodes per thread, "nt" non-temporal edge-message stream (0/1), "split"
 * (1 = all frames in lock-step, 2 = two frame halves software-pipelined half an
 * iteration apart so each launch overlaps one half's check sweep with the
 * other half's variable sweep), "demap_fast" (1 = Newton-located root +
 * replayed bisection, bit-identical to 0 = the reference's brute-force search). */
QR_API int qr_tune_set(const char *name, int64_t value);
QR_API int qr_tune_get(const char *name, int64_t *value);

/* ------------------------------------------------------------ Tanner graph */
/* Replaces Decoder.__cinit__ (decoder.pyx:93-146).  e_to_v / e_to_c: host int64
 * edge lists (edge e joins variable e_to_v[e] and check e_to_c[e]).  V = max+1,
 * C = max+1 (decoder.pyx:101-103).  Per-check and per-variable edge lists keep
 * ascending edge id (decoder.pyx:73-75).  QR_EVALUE on size mismatch
 * (decoder.pyx:96-97), negative ids, or a check of degree < 2 (undefined
 * behaviour in the reference, decoder.pyx:135-141; rejected here). */
QR_API int qr_code_create(const int64_t *e_to_v, const int64_t *e_to_c, int64_t n_edges_v, int64_t n_edges_c,
                   int32_t device, qr_code **out);
QR_API int qr_code_destroy(qr_code *code);
/* Decoder.vnum / cnum / ednum properties (decoder.pyx:157-172). */
QR_API int qr_code_info(const qr_code *code, int64_t *vnum, int64_t *cnum, int64_t *ednum, int32_t *max_check_degree,
                 int32_t *max_var_degree);

/* ------------------------------------------------------------------ decode */
/* Device workspace (bytes) for qr_decode_batch_device at leading dim ld and
 * max_iterations (edge messages E*ld fp64 + per-frame flags; with tuning knob "repack" on
 * (default) and ld % 512 == 0, plus the column-repack work set: posteriors, frame ids and two
 * column sets of messages, LAPPRs and syndrome bits used in turn by consecutive repacks (the
 * repack gathers LAPPRs and syndrome bits, the check sweep after it writes the messages),
 * (8E + 24V + 2C + 4)*ld bytes -- a workspace without it runs the same decode without the
 * repack). */
QR_API int qr_decode_workspace_size(const qr_code *code, int32_t ld, int32_t max_iterations, size_t *bytes);

/* Batched Decoder._decode (decoder.pyx:391-436) of B independent frames.
 *   d_lappr [V][ld] fp64   input LAPPRs          (not modified)
 *   d_synd  [C][ld] uint8  target syndromes      (0/1)
 *   d_final [V][ld] fp64   final LAPPRs = posterior after the last variable sweep,
 *                          or a copy of d_lappr when the input already satisfies
 *                          the syndrome (decoder.pyx:400-405)
 *   d_success[B] uint8, d_iters[B] int32: the (success, iterations) pair of
 *                          _decode for every frame (decoder.pyx:433,436).
 * Per-frame early termination; results per frame are identical to decoding
 * that frame alone.
 * Asynchronous: every launch is enqueued on `stream` (the two-stream schedule also on a
 * library-owned second stream, forked from and joined back into `stream` by events) and the
 * call returns without waiting for the GPU; every schedule decision that depends on the data
 * (early termination, active-frame lists, column repack) is taken on the device, so the call
 * is capturable into a HIP graph and the replay computes the same results. */
QR_API int qr_decode_batch_device(const qr_code *code, int32_t B, int32_t ld, const double *d_lappr, const uint8_t *d_synd,
                           int32_t max_iterations, double *d_final, uint8_t *d_success, int32_t *d_iters,
                           void *d_workspace, size_t workspace_bytes, void *stream);

/* Diagnostics of the column repack of the last qr_decode_batch_device that used this workspace
 * (the same code, ld, max_iterations and workspace): out[0], out[1] = how many times the device
 * repacked frame range 0 / 1 of the two-stream schedule, out[2], out[3] = the width each range
 * ended at (0 repacks and width ld / 2 for a range never repacked, and for every decode that did
 * not take the two-stream schedule).
 * Synchronous device-to-host copy: call after the decode has completed. */
QR_API int qr_decode_repack_stats(const qr_code *code, int32_t ld, int32_t max_iterations, const void *d_workspace,
                                  size_t workspace_bytes, int32_t *out);

/* Decoder.decode (decoder.pyx:441-455) for B frames from host memory,
 * frame-major: lappr[B][V], synd[B][C], final[B][V]. */
QR_API int qr_decode_host(const qr_code *code, int32_t B, const double *lappr, const uint8_t *synd, int32_t max_iterations,
                   double *final_lappr, uint8_t *success, int32_t *iterations);

/* --------------------------------------------- Decoder unit-test surface */
/* Decoder.check_lappr (decoder.pyx:235-281): per-check satisfied flags
 * (check_ok[C]) and the whole-word flag, for one frame, computed on the GPU. */
QR_API int qr_check_lappr_host(const qr_code *code, const double *lappr, const uint8_t *synd, uint8_t *check_ok,
                        uint8_t *all_ok);
/* Decoder.check_synd_node / check_word (decoder.pyx:177-232) on a hard word. */
QR_API int qr_check_word_host(const qr_code *code, const uint8_t *word, const uint8_t *synd, uint8_t *check_ok,
                       uint8_t *all_ok);
/* Decoder.process_var_node (decoder.pyx:285-319) for a list of variable nodes:
 * updated[v] = lappr[v] + sum c2v[e]; v2c[e] = updated[v] - c2v[e]. */
QR_API int qr_process_var_nodes_host(const qr_code *code, const int64_t *nodes, int64_t n_nodes, const double *lappr,
                              const double *c2v, double *v2c, double *updated);
/* Decoder.process_check_node (decoder.pyx:322-388) for a list of check nodes. */
QR_API int qr_process_check_nodes_host(const qr_code *code, const int64_t *nodes, int64_t n_nodes, const uint8_t *synd,
                                double *c2v, const double *v2c);

/* ------------------------------------------------------------ soft demap */
/* Replaces the hot-path part of NoiseMapper.__cinit__ (noisemapper.pyx:103-162)
 * for a PAMAlphabet (alphabet.pyx:35-76): constellation[M], probabilities[M]
 * (NULL = uniform), thresholds[M+1], noise_var > 0, sign_config[M] (NULL = zeros).
 * Computes F_Y_thresholds / delta_F_Y with the scipy-exact erf and uploads the
 * tables to `device`. */
QR_API int qr_demap_create(int32_t bit_per_symbol, const double *constellation, const double *probabilities,
                    const double *thresholds, double noise_var, const uint8_t *sign_config, int32_t device,
                    qr_demap **out);
QR_API int qr_demap_destroy(qr_demap *dm);
/* F_Y_thresholds[M+1], delta_F_Y[M] as the reference exposes them (noisemapper.pxd). */
QR_API int qr_demap_tables(const qr_demap *dm, double *F_Y_thresholds, double *delta_F_Y);

/* Batched NoiseMapper.demap_lappr_array (noisemapper.pyx:544-559) fused with the
 * LLR scaling of the softening pipeline (reconciliation.pyx:143-145):
 *   d_n [S][ld] fp64, d_j [S][ld] int64 (transmitted symbol index 0..M-1)
 *   d_lappr [S*bps][ld] fp64: d_lappr[(s*bps + k)*ld + f] = alpha * LAPPR of Gray bit k
 * i.e. directly the decoder's input layout (variable node v = s*bps + k).
 * Out-of-range symbol indices yield NaN LAPPRs. */
QR_API int qr_demap_batch_device(const qr_demap *dm, int32_t B, int32_t ld, int64_t S, const double *d_n,
                          const int64_t *d_j, double alpha, double *d_lappr, void *stream);
/* NoiseMapper.demap_lappr_array for one array from host memory: lappr[S*bps]. */
QR_API int qr_demap_host(const qr_demap *dm, int64_t S, const double *n, const int64_t *j, double *lappr);

/* NoiseMapper.g_inv_search (noisemapper.pyx:310-345) over arrays, i.e.
 * NoiseMapper.demap_noise_search (noisemapper.pyx:407-419): y_hat[k] = the root of
 * F_Y(y) = target(n_hat[k], i[k]) by the reference's doubling bracket + bisection to
 * hi - lo <= y_accuracy (default 1e-9 in the reference).  Bit-identical to the
 * reference.  i[k] outside [0, M) gives NaN (out-of-bounds reads in the reference);
 * the bracket + bisection loops are capped at 2200 steps (NaN), where the reference
 * loops forever (targets outside [0, 1], y_accuracy below the spacing of the doubles
 * near the root).  Host arrays of n elements; synchronous. */
QR_API int qr_g_inv_search_host(const qr_demap *dm, int64_t n, const double *n_hat, const int64_t *i,
                                double y_accuracy, double *y_hat);
/* NoiseMapper.F_Y (noisemapper.pyx:264-275): F[k] = (sum_m F_Z(y[k], a_m, sigma)) / M, the
 * uniformly weighted mixture CDF (the cpdef ignores the alphabet's probabilities).  Host
 * arrays of n elements; synchronous. */
QR_API int qr_F_Y_host(const qr_demap *dm, int64_t n, const double *y, double *F);

/* ---------------------------------------------- softening pipeline (Bob) */
/* NoiseMapper.hard_decide_index + map_noise (noisemapper.pyx:349-388) and
 * PAMAlphabet.demap_symbols_to_bits (alphabet.pyx:98-107), fused, frame-innermost:
 *   d_y[S][ld] -> d_xhat[S][ld] int64, d_nhat[S][ld] fp64, d_word[S*bps][ld] uint8 */
QR_API int qr_bob_map_device(const qr_demap *dm, int32_t B, int32_t ld, int64_t S, const double *d_y, int64_t *d_xhat,
                      double *d_nhat, uint8_t *d_word, void *stream);
/* NoiseMapper.map_noise (noisemapper.pyx:373-388) with caller-given indices:
 * d_nhat[s][f] = g(d_y[s][f], d_index[s][f]) (noisemapper.pyx:289-292). */
QR_API int qr_map_noise_device(const qr_demap *dm, int32_t B, int32_t ld, int64_t S, const double *d_y,
                               const int64_t *d_index, double *d_nhat, void *stream);
/* PAMAlphabet.demap_symbols_to_bits (alphabet.pyx:98-107): d_x[S][ld] -> d_word[S*bps][ld]
 * (padding frames f in [B, ld) get the bits of symbol 0). */
QR_API int qr_symbols_to_bits_device(int32_t bit_per_symbol, int32_t B, int32_t ld, int64_t S, const int64_t *d_x,
                                     uint8_t *d_word, void *stream);
/* Direct reconciliation LAPPRs (sims/reconciliation.pyx:25-51, _y_to_lappr_grey):
 * d_y[S][ld] -> d_lappr[S*bps][ld], two_variance = 2 * noise variance. */
QR_API int qr_direct_lappr_device(const qr_demap *dm, double two_variance, int32_t B, int32_t ld, int64_t S,
                                  const double *d_y, double *d_lappr, void *stream);
/* Hard reverse reconciliation LAPPRs (noisemapper.pyx:423-432, bare_llr):
 * d_lappr[(s*bps+k)][f] = d_table[x * bps + k] with the device table[M][bps]. */
QR_API int qr_bare_llr_device(int32_t bit_per_symbol, const double *d_table, int32_t B, int32_t ld, int64_t S,
                              const int64_t *d_x, double *d_lappr, void *stream);
/* Matrix.eval_syndrome (matrix.pyx:55-60): d_word[V][ld] -> d_synd[C][ld]. */
QR_API int qr_syndrome_device(const qr_code *code, int32_t B, int32_t ld, const uint8_t *d_word, uint8_t *d_synd,
                       void *stream);
/* count_errors_from_lappr (utils.pyx:27-40) over the first K variable nodes of
 * every frame plus the frame bookkeeping of simulate_softening_snr_dB
 * (reconciliation.pyx:149-157), accumulated into d_counters (int64[5], not
 * cleared): {bit_errors, frame_errors, successes, iteration_sum_of_successes, frames}.
 * d_frame_errors[B] (int32) receives the per-frame bit-error counts. */
QR_API int qr_count_errors_device(int32_t B, int32_t ld, int64_t K, const double *d_final, const uint8_t *d_word,
                           const uint8_t *d_success, const int32_t *d_iters, int32_t *d_frame_errors,
                           int64_t *d_counters, void *stream);

/* --------------------------------------------------------- layout helpers */
/* Frame-major [B][n] <-> frame-innermost [n][ld] transposes on the device. */
QR_API int qr_to_frame_innermost_f64(int32_t B, int32_t ld, int64_t n, const double *d_src, double *d_dst, void *stream);
QR_API int qr_to_frame_major_f64(int32_t B, int32_t ld, int64_t n, const double *d_src, double *d_dst, void *stream);
QR_API int qr_to_frame_innermost_u8(int32_t B, int32_t ld, int64_t n, const uint8_t *d_src, uint8_t *d_dst, void *stream);
QR_API int qr_to_frame_innermost_i64(int32_t B, int32_t ld, int64_t n, const int64_t *d_src, int64_t *d_dst, void *stream);

/* ------------------------------------------------------------ measurement */
/* Streaming device copy (4 x 16 B per lane in flight, grid-stride): the practical HBM ceiling
 * the decoder's roofline is related to in bench.py. bytes % 16 == 0,
 * 16-B aligned pointers.  Not a reference interface. */
QR_API int qr_stream_copy(const void *d_src, void *d_dst, int64_t bytes, void *stream);

/* Shader-clock probe: n one-wave workgroups, each spinning (scalar only, s_sleep) for
 * `realtime_ticks` of the 100 MHz constant clock and writing {shader cycles, realtime
 * ticks} to d_out[2i], d_out[2i+1].  Launched on a side stream while the decode runs, it
 * reads the clock the chip holds under that load without a profiler attached
 * (MI355X_MICROARCH.md "DVFS give-back" item 6).  Not a reference interface. */
QR_API int qr_clock_probe(int64_t *d_out, int32_t n, int64_t realtime_ticks, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* QAMR_H */
