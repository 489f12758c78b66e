/*
 * qkd_ldpc.h — C ABI of the MI355X-native QKD LDPC sum-product decoder.
 *
 * Drop-in boundary for the hot path of ColdCloudd/QKD_LDPC (snapshot
 * 2024-12-23). Every entry point below names the reference interface it
 * replaces (file:line under the reference tree). Plain C types only: no HIP,
 * no torch. Device pointers are raw addresses on the code's device; `stream`
 * is a hipStream_t passed as void* (NULL = the null stream).
 *
 * Bit-exactness contract: for the same inputs, every per-frame output here
 * (decoded bits, iteration count, syndrome match, key match, exact QBER) is
 * identical to the reference's fp64 CPU path (glibc tanh/atanh, flooding
 * schedule, reference accumulation order).
 *
 * Threading: a qkd_code is immutable after creation and may be shared by any
 * number of host threads. Calls that need device scratch take a
 * qkd_workspace*; pass NULL to use the code's internal workspace, which is
 * guarded by a mutex and therefore serialises such calls at the host (calls
 * on different streams then must not overlap on the device: they are
 * ordered by an internal event). For concurrent streams create one
 * workspace per stream.
 *
 * Errors: no exception crosses this boundary. Every call returns a
 * qkd_status; qkd_last_error() returns a thread-local message for the most
 * recent failure on the calling thread. The reference signals the same
 * conditions by throwing std::runtime_error (e.g.
 * array_and_matrix_operations.cpp:116,159,223; simulation.cpp:174).
 */
#ifndef QKD_LDPC_H
#define QKD_LDPC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define QKD_LDPC_ABI_VERSION 1

#if defined(__GNUC__)
#define QKD_API __attribute__((visibility("default")))
#else
#define QKD_API
#endif

typedef enum qkd_status {
    QKD_OK = 0,
    QKD_ERR_INVALID_ARG = 1,     /* null pointer, zero size, bad flag        */
    QKD_ERR_BAD_CODE = 2,        /* adjacency out of range / inconsistent    */
    QKD_ERR_UNSORTED = 3,        /* an adjacency row is not ascending: the
                                    reference would silently route messages
                                    to the wrong edges (A1 invariant)        */
    QKD_ERR_QBER_TOO_SMALL = 4,  /* floor(N*q) == 0 (simulation.cpp:170-175) */
    QKD_ERR_DEVICE = 5,          /* HIP runtime failure                      */
    QKD_ERR_OUT_OF_MEMORY = 6,
    QKD_ERR_IO = 7,              /* matrix file unreadable / malformed       */
    QKD_ERR_UNSUPPORTED = 8      /* code shape outside what the kernels take */
} qkd_status;

/* Decoder flags (bitwise OR). */
#define QKD_FLAG_THRESHOLD 0x1u  /* CFG.ENABLE_SUM_PRODUCT_MSG_LLR_THRESHOLD
                                    (qkd_ldpc_algorithm.cpp:246,313)         */

/* Check-node rule (flag bits 4-5). QKD_VARIANT_SP_F64 is the reference's
 * decoder (qkd_ldpc_algorithm.cpp:175-345), bit-exact. The other two are
 * build-defined variants with binary32 messages and totals (SURVEY.md §8(d),
 * config 5): same flooding schedule, stopping rule, clamp and outputs; their
 * frame error rates are compared with the reference's, not their frames. */
#define QKD_VARIANT_MASK   0x30u
#define QKD_VARIANT_SP_F64 0x00u  /* sum-product, binary64 (the reference)    */
#define QKD_VARIANT_SP_F32 0x10u  /* sum-product, binary32, Gallager form:
                                     c2b = sign * phi(sum of the other
                                     phi(|b2c|)), phi(x) = -ln tanh(x/2),
                                     hardware exp2/log2                      */
#define QKD_VARIANT_MINSUM 0x20u  /* normalised min-sum, binary32:
                                     c2b = scale * sign * min |b2c| over the
                                     check's other edges                     */
/* Min-sum scale in flag bits 8-15 as round(scale * 256); 0 selects
 * QKD_MINSUM_DEFAULT_SCALE. */
#define QKD_MINSUM_SCALE_SHIFT 8
#define QKD_MINSUM_SCALE(x) ((((uint32_t)((x) * 256.0 + 0.5)) & 0xffu) << QKD_MINSUM_SCALE_SHIFT)
#define QKD_MINSUM_DEFAULT_SCALE 0.8125  /* best FER of {0.625..0.875} on config 3 */
/* Min-sum offset in flag bits 16-23 as round(offset * 64): the message magnitude
 * is max(scale * min |b2c| - offset, 0) (offset min-sum); 0 = no offset. */
#define QKD_MINSUM_OFFSET_SHIFT 16
#define QKD_MINSUM_OFFSET(x) ((((uint32_t)((x) * 64.0 + 0.5)) & 0xffu) << QKD_MINSUM_OFFSET_SHIFT)
/* Self-corrected min-sum (QKD_VARIANT_MINSUM only; needs the LDS-state
 * min-sum kernel): a bit-to-check message whose sign flipped since the last
 * iteration (both nonzero) is erased to 0 before the check rule. */
#define QKD_MINSUM_SELF_CORRECT 0x1000000u

typedef struct qkd_code qkd_code;
typedef struct qkd_workspace qkd_workspace;

typedef struct qkd_code_info {
    int32_t n_bits;              /* H_matrix::num_bit_nodes                  */
    int32_t n_checks;            /* H_matrix::num_check_nodes                */
    int32_t n_edges;
    int32_t max_bit_degree;      /* H_matrix::max_bit_nodes_weight           */
    int32_t max_check_degree;    /* H_matrix::max_check_nodes_weight         */
    int32_t is_regular;          /* H_matrix::is_regular                     */
    int32_t device;
} qkd_code_info;

/* Per-QBER-point reduction of a trial batch (simulation.cpp:252-312): only
 * frames whose syndrome matched contribute to the iteration statistics, and
 * ldpc_ok counts key matches among them. */
typedef struct qkd_counters {
    uint64_t frames;
    uint64_t sp_ok;              /* trials_successful_sp                     */
    uint64_t ldpc_ok;            /* trials_successful_ldpc                   */
    uint64_t sum_iters;          /* sum of iterations over sp_ok frames      */
    uint64_t sum_iters_sq;       /* sum of squares, same frames              */
    uint32_t min_iters;          /* over sp_ok frames (UINT32_MAX if none)   */
    uint32_t max_iters;          /* over sp_ok frames (0 if none)            */
} qkd_counters;

/* ---- library ----------------------------------------------------------- */
QKD_API int qkd_abi_version(void);
QKD_API const char *qkd_last_error(void);
QKD_API const char *qkd_status_string(qkd_status s);
/* Number of visible HIP devices (0 when none; never fails). */
QKD_API int qkd_device_count(void);

/* ---- code object: replaces H_matrix + its readers -----------------------
 * H_matrix (array_and_matrix_operations.hpp:16-27), read_sparse_alist_matrix
 * (array_and_matrix_operations.cpp:109-292), read_dense_matrix (:295-421),
 * free_matrix_H (:88-94).
 * check_ptr[m+1] / check_idx[E]: 0-based CSR of check_nodes (bits of each
 * check, each row ascending). The bit-side lists (bit_nodes) are derived.
 * Validation: indices in range, no duplicate edge, rows ascending
 * (QKD_ERR_UNSORTED otherwise). Device data is uploaded once. */
QKD_API qkd_code *qkd_code_create(int32_t n_bits, int32_t n_checks, const int32_t *check_ptr,
                          const int32_t *check_idx, int device, qkd_status *status);
/* Reads an alist file with the reference reader's rules (weights line,
 * non-zero counts per line, 1-based entries, the first `weight` entries
 * of each line). */
QKD_API qkd_code *qkd_code_from_alist(const char *path, int device, qkd_status *status);
/* Reader options (reader hardening). QKD_READ_SORT_ROWS: sort
 * every bit and check line before validation, so a file whose rows are not
 * ascending is read as the matrix it describes (default: QKD_ERR_UNSORTED,
 * where the reference would silently mis-route messages, §8(a) A1). */
#define QKD_READ_SORT_ROWS 0x1u
QKD_API qkd_code *qkd_code_from_alist_ex(const char *path, int device, uint32_t read_flags,
                                         qkd_status *status);
/* Reads a dense 0/1 matrix file (one row per line). */
QKD_API qkd_code *qkd_code_from_dense(const char *path, int device, qkd_status *status);
QKD_API void qkd_code_destroy(qkd_code *code);
QKD_API qkd_status qkd_code_get_info(const qkd_code *code, qkd_code_info *info);
/* Host copies of the adjacency (any pointer may be NULL). bit_ptr[n+1],
 * bit_idx[E] are the reference's bit_nodes rows (ascending checks). */
QKD_API qkd_status qkd_code_get_adjacency(const qkd_code *code, int32_t *check_ptr, int32_t *check_idx,
                                  int32_t *bit_ptr, int32_t *bit_idx);

/* ---- workspace ------------------------------------------------------------ */
QKD_API qkd_workspace *qkd_workspace_create(const qkd_code *code, qkd_status *status);
QKD_API void qkd_workspace_destroy(qkd_workspace *ws);

/* ---- batched device entry points (all arrays device-resident) ------------ */

/* calculate_syndrome_irregular / _regular (array_and_matrix_operations.cpp:463-486)
 * bits[F*N] (0/1 bytes) -> syndrome[F*M] (0/1 bytes). */
QKD_API qkd_status qkd_syndrome_batch(const qkd_code *code, const uint8_t *bits, size_t n_frames,
                              uint8_t *syndrome, void *stream);

/* sum_product_decoding_irregular / _regular (qkd_ldpc_algorithm.cpp:3-345):
 * llr[F*N] fp64 channel LLRs, syndrome[F*M] 0/1 bytes -> bits_out[F*N] (last
 * hard decision), iterations[F] (SP_result::iterations_num) and
 * syndromes_match[F] (SP_result::syndromes_match). msg_threshold is
 * CFG.SUM_PRODUCT_MSG_LLR_THRESHOLD, applied when QKD_FLAG_THRESHOLD is set.
 * bits_out may be NULL. */
QKD_API qkd_status qkd_decode_batch(const qkd_code *code, qkd_workspace *ws, const double *llr,
                            const uint8_t *syndrome, size_t n_frames, uint32_t max_iterations,
                            double msg_threshold, uint32_t flags, uint8_t *bits_out,
                            uint32_t *iterations, uint8_t *syndromes_match, void *stream);

/* QKD_LDPC_irregular / _regular (qkd_ldpc_algorithm.cpp:347-447), batched:
 * LLR_i = bob_i ? -log((1-q)/q) : +log((1-q)/q), Alice's syndrome, decode,
 * keys_match = (decoded == alice). alice/bob [F*N] 0/1 bytes; one QBER for
 * the batch. bits_out may be NULL. */
QKD_API qkd_status qkd_qkd_ldpc_batch(const qkd_code *code, qkd_workspace *ws, const uint8_t *alice,
                              const uint8_t *bob, size_t n_frames, double qber,
                              uint32_t max_iterations, double msg_threshold, uint32_t flags,
                              uint8_t *bits_out, uint32_t *iterations, uint8_t *syndromes_match,
                              uint8_t *keys_match, void *stream);

/* generate_random_bit_array + introduce_errors (array_and_matrix_operations.cpp:424-460)
 * for frame k seeded with seeds[k] + seed_offset (simulation.cpp:163,247),
 * on the device. alice/bob [F*N] 0/1 bytes; exact_qber[F] may be NULL.
 * Returns QKD_ERR_QBER_TOO_SMALL when floor(N*q_nominal) == 0. */
QKD_API qkd_status qkd_keygen_batch(const qkd_code *code, qkd_workspace *ws, const uint64_t *seeds,
                            uint64_t seed_offset, size_t n_frames, double q_nominal,
                            uint8_t *alice, uint8_t *bob, double *exact_qber, void *stream);

/* run_trial (simulation.cpp:161-189) for F frames, fused on the device:
 * keygen -> LLR -> Alice syndrome -> decode -> key compare. Per-frame outputs
 * (any may be NULL) and, if counters != NULL (device memory, one
 * qkd_counters), the batch reduction of simulation.cpp:252-312. */
QKD_API qkd_status qkd_trials_batch(const qkd_code *code, qkd_workspace *ws, const uint64_t *seeds,
                            uint64_t seed_offset, size_t n_frames, double q_nominal,
                            uint32_t max_iterations, double msg_threshold, uint32_t flags,
                            uint32_t *iterations, uint8_t *syndromes_match, uint8_t *keys_match,
                            double *exact_qber, qkd_counters *counters, void *stream);

/* QKD_LDPC_interactive_simulation (simulation.cpp:73-137) over n_points
 * nominal QBERs (host array): ONE xoshiro256++(simulation_seed) stream feeds
 * every point's key pair in turn (:95, :102-103), then each point runs
 * QKD_LDPC_* at its exact QBER (:122-129). Outputs are HOST arrays of
 * n_points: iterations, syndromes_match, keys_match (the reference prints
 * SUCCESSFUL when both hold, :131), exact_qber ("Actual QBER"), errors
 * ("Number of errors in a key"). *points_done = points run. Like the
 * reference, a point with floor(N*q) == 0 stops the run there and returns
 * QKD_ERR_QBER_TOO_SMALL with the earlier points' results filled in.
 * Synchronous (device-synchronising); ws may be NULL. */
QKD_API qkd_status qkd_interactive_batch(const qkd_code *code, qkd_workspace *ws, uint64_t simulation_seed,
                                         size_t n_points, const double *q_nominal, uint32_t max_iterations,
                                         double msg_threshold, uint32_t flags, uint32_t *iterations,
                                         uint8_t *syndromes_match, uint8_t *keys_match, double *exact_qber,
                                         uint32_t *errors, size_t *points_done);

/* Reduction alone: per-frame results -> counters (device memory). */
QKD_API qkd_status qkd_counters_batch(const uint32_t *iterations, const uint8_t *syndromes_match,
                              const uint8_t *keys_match, size_t n_frames, qkd_counters *counters,
                              int device, void *stream);

/* Combination of n_records counter records (device memory, e.g. one per rank
 * after an all-gather) into *out (device memory; may alias a record): the
 * reduction the reference's single process performs over every trial of a
 * point (simulation.cpp:252-312) -- sums add, min_iters / max_iters take the
 * minimum / maximum. One launch on `stream`. */
QKD_API qkd_status qkd_counters_merge(const qkd_counters *records, size_t n_records, qkd_counters *out,
                                      int device, void *stream);

/* ---- diagnostics ------------------------------------------------------------
 * Debug and A/B options. The library reads NO environment variable: every
 * option defaults to the product behaviour and changes only through this
 * call. ws != NULL sets the option for that workspace; ws == NULL sets the
 * process-wide value every workspace uses unless it has its own. value NULL
 * restores the default. Options (test infrastructure; outputs are bit-exact
 * under every value unless a variant says otherwise):
 *   QKD_SPEC_CAP <k>           interval iterations per frame before the exact
 *                              ones (0: off; default 8)
 *   QKD_SPEC_CKPT 0|1          force the checkpointed speculation off / on
 *   QKD_CKPT_UNSAT <k>         its trigger (unsatisfied checks; default 128)
 *   QKD_SPEC_POLICY always     the in-launch replay policy never turns off
 *   QKD_FOLD_TABLE 0           the folded first iteration per bit, not tabled
 *   QKD_DECODE_KERNEL classic  the classic message-store decoder
 *   QKD_MINSUM_STORE lds|global  the LDS-state / global-store min-sum kernels
 *   QKD_DECODE_GRID <k>        cap the decoder's resident workgroups
 *   QKD_SPLIT_BUDGET <bytes>   lower the split decoder's LDS budget
 *   QKD_C2B_PAD <slots>        a fixed pad of the split decoder's regions
 *   QKD_ILV 0|1, QKD_ILV_GRID <k>  the interleaved long-code decoder off / on,
 *                              its workgroup cap
 *   QKD_KEYGEN serial|replay|lanes|matrix  the other key generators
 *   QKD_SYN_SLICED 0, QKD_SYN_BYTES 0  the gather frame-syndrome kernel / the
 *                              separate key packing
 *   QKD_BIT_ORDER identity|runs  (ws == NULL, read when a code is created)
 *                              the split decoder's internal bit order
 *   QKD_PHASE_TIMING 1         per-phase shader clocks (qkd_debug_phase_cycles)
 * An unknown name fails with QKD_ERR_INVALID_ARG. Thread-safe. No reference
 * counterpart (the reference's CFG fields are the decode parameters). */
QKD_API qkd_status qkd_debug_set_option(qkd_workspace *ws, const char *name, const char *value);
/* With QKD_PHASE_TIMING set (qkd_debug_set_option), decode launches on `ws`
 * accumulate shader-clock cycles per phase, summed over workgroups (thread 0
 * between barriers): [0] per-frame prologue, [1] check phase, [2] bit phase,
 * [3] syndrome test, [4] frame fetch + outputs, [5] / [6] the table-driven
 * first / second check phases of the QKD path. Synchronises the device. No
 * reference counterpart (the reference prints TRACE_* arrays instead,
 * qkd_ldpc_algorithm.cpp:42-155). */
QKD_API qkd_status qkd_debug_phase_cycles(qkd_workspace *ws, uint64_t *cycles7);
/* Decoder-kernel timing (the measurement's live roofline figure): start != 0
 * turns it on for `ws` (zeroed): every later decoder launch on ws is bracketed
 * by two HIP events on its stream, so only the decode kernel is timed (not the
 * packing, frame-syndrome or key-compare kernels around it). start == 0
 * synchronises those events, returns the summed kernel milliseconds and the
 * number of launches, and turns timing off. No reference counterpart. */
QKD_API qkd_status qkd_debug_decoder_timing(qkd_workspace *ws, int start, double *ms_total, uint64_t *launches);
/* Frames of the QKD path (qkd_qkd_ldpc_batch / qkd_trials_batch, binary64
 * rule, clamp on) whose speculative interval iterations could not certify a
 * hard decision (or reached the cap) and were decoded again with the exact
 * iterations, accumulated over the launches on `ws` since the last reset;
 * reset != 0 zeroes the count. The QKD_SPEC_CAP option (qkd_debug_set_option)
 * sets how many interval iterations a frame may run first (0: off; default 8).
 * Outputs never depend on it. No reference counterpart. */
QKD_API qkd_status qkd_debug_spec_replays(qkd_workspace *ws, uint64_t *replays, int reset);
/* Trace of one frame, the reference's TRACE_SUM_PRODUCT / TRACE_SUM_PRODUCT_LLR
 * (qkd_ldpc_algorithm.cpp:212-330): decodes llr[N] / syndrome[M] (host arrays)
 * with the reference rule (QKD_VARIANT_SP_F64 only) and records, for every
 * executed iteration t < *iterations, the messages the reference prints:
 *   c2b_trace[t*E + e]   "E:" check-to-bit messages after the clamp, in the
 *                        reference's check_to_bit_msg order (bit by bit, each
 *                        bit's checks ascending; bit_ptr of get_adjacency)
 *   total_trace[t*N + i] "L:" bit totals
 * (host arrays of max_iterations*E / *N, either may be NULL). "z:", "s:",
 * "M:" and MAX_LLR follow from these exactly (qkd_ldpc_amd.trace_decode). */
QKD_API qkd_status qkd_trace_decode(const qkd_code *code, const double *llr, const uint8_t *syndrome,
                                    uint32_t max_iterations, double msg_threshold, uint32_t flags,
                                    double *c2b_trace, double *total_trace, uint32_t *iterations,
                                    uint8_t *syndrome_match);
/* The decoder's tanh (which = 0) / atanh (which = 1) restatement applied to
 * x[n] -> y[n] (device arrays): the bit-exactness check of the device build
 * against glibc (reference qkd_ldpc_algorithm.cpp:224, :241). which = 2 / 3:
 * the binary32 variant's two transcendental steps (QKD_VARIANT_SP_F32): the
 * published sign(x) * phi(|x|) / ln 2 and phi(S ln 2) of a psi-unit sum S, x
 * rounded to binary32, result widened. which = 4 / 5: certified bounds of
 * phi(x) = -ln tanh(x/2) over [x[2k], x[2k+1]] (the speculative iterations'
 * input / output forms, qkd_spec.h) -> y[2k] = lower, y[2k+1] = upper; n even;
 * which = 5 takes its interval in log2-domain units (x = S / ln 2).
 * which = 8 / 9: quadruples (a, b, s_lo, s_hi) -> raw binary32 (in lo, in hi,
 * out lo, out hi) of the packed phi_pair (8) and of the scalar phi_bounds +
 * phi_bounds_out it must equal bit for bit (9); n a multiple of 4.
 * which = 10 / 11: pairs of exact b2c -> the raw bits of their psi bounds
 * (two binary32 per output double) from the packed psi_of_exact2 (10) and
 * the scalar psi_of_exact (11); n even.
 * which = 12 / 13: pairs (x, S) -> (|sign(x) phi(|x|) / ln 2|, phi(S ln 2))
 * of the binary32 variant, from its packed evaluation (12) and from the
 * scalar forms of which = 2 / 3 (13), which must agree bit for bit; n even.
 * which = 14 / 15: quadruples (a lo, a hi, b lo, b hi) -> the input-form phi
 * bounds of both intervals from the packed phi_bounds2 (14, the interleaved
 * decoder's) and two scalar phi_bounds (15); which = 16 / 17 the same for the
 * output form, phi_bounds_out2 (16) and phi_bounds_out (17); n % 4 == 0. */
QKD_API qkd_status qkd_debug_math(int which, const double *x, double *y, size_t n, void *stream);
/* Exhaustive check of the speculative iterations' phi bounds (qkd_spec.h) at
 * EVERY binary32 a with bit pattern in [first_bits, last_bits] (positive
 * finite): which = 4 the input form phi_bounds (a in nep units, psi result),
 * which = 5 the output form phi_bounds_out (a in log2-domain units, S = a ln 2),
 * both at the degenerate interval [a, a], against a binary64 phi on the
 * device. result[8] (host): [0] points, [1] upper bound below phi(a),
 * [2] lower bound above phi(a), [3] slope bound (with half its 2^-20 margin)
 * below |phi'(a)|, [4] max |eval/phi - 1| / 2^-20 (binary32 bits), [5] max
 * |phi'| / slope bound (binary32 bits), [6] / [7] bit patterns where [4] / [5]
 * peak (either of the tied points); [4]-[7] over normal a with a finite
 * evaluation only (a subnormal argument overflows the reciprocal: infinite
 * upper bound, zero lower bound; the kernel never feeds such an argument to
 * the output form, whose sums are at least phi(80) / ln 2). Synchronous. Test infrastructure: no
 * reference counterpart (the reference has no speculative iterations). */
QKD_API qkd_status qkd_debug_phi_sweep(int which, uint32_t first_bits, uint32_t last_bits, uint64_t *result);

/* The split decoder's internal bit order of a code given as a check-side CSR
 * (as qkd_code_create), computed on the host without a device: perm_out[q]
 * (n_bits entries) = the original bit at internal position q; plan_out
 * (optional, 64 * n_tasks entries, n_tasks from *n_tasks_out when plan_out is
 * null) = the check-phase wave plan's first words (bit | row << 24, idle lanes
 * bit = n_bits); mode: NULL for the shipped order, "runs" without its LDS bank
 * pass, "identity". Test infrastructure (tests/test_bit_order.py, CPU); no
 * reference counterpart. */
QKD_API qkd_status qkd_debug_bit_order(int32_t n_bits, int32_t n_checks, const int32_t *check_ptr,
                                       const int32_t *check_idx, const char *mode, int32_t *perm_out,
                                       uint32_t *plan_out, int32_t *n_tasks_out);

/* ---- host helpers --------------------------------------------------------- */
/* seeds[k] = k-th raw xoshiro256++(simulation_seed) output (simulation.cpp:222-228). */
QKD_API qkd_status qkd_make_seeds(uint64_t simulation_seed, size_t count, uint64_t *seeds_host);
/* get_rate_based_QBER_range (simulation.cpp:48-70) for one table row:
 * writes min(capacity, steps) values, returns the step count in *count. */
QKD_API qkd_status qkd_qber_range(double begin, double end, double step, double *values_host,
                          size_t capacity, size_t *count);

#ifdef __cplusplus
}
#endif

#endif /* QKD_LDPC_H */
