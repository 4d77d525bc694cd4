/*
 * ldpc_abi.h — C ABI of the MI355X-native LDPC belief-propagation decoder (libldpc_hip.so).
 *
 * Plain C: pointers, sizes and ints only; no torch / HIP types in any signature (hip streams are passed
 * as void*).  Every entry point returns 0 (LDPC_OK) or a negative LDPC_E* code and leaves a message in
 * ldpc_last_error() (thread-local).  The reference (realjwin/ldpc-sims) has no C surface at all: its
 * decode boundary is Python.  Each function below names the reference interface it replaces.
 */
#ifndef LDPC_ABI_H
#define LDPC_ABI_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ABI revision of this header.  2: ldpc_decode gained iters_used (before the stream argument) in round 5 —
 * a caller built against revision 1 would pass its stream where iters_used is read.  Loaders compare
 * ldpc_abi_version() with the revision they were written for and refuse a mismatch (ldpc_amd/_abi.py does). */
#define LDPC_ABI_VERSION 2

typedef struct ldpc_graph ldpc_graph;

enum {
    LDPC_OK = 0,
    LDPC_EINVAL = -1,      /* bad argument (shape, range, null pointer)                */
    LDPC_EHIP = -2,        /* HIP runtime error (message names the call)                */
    LDPC_ENOMEM = -3,      /* device allocation failed / workspace too small            */
    LDPC_EUNSUPPORTED = -4 /* combination of algo/flags not implemented for this graph  */
};

enum {
    LDPC_ALGO_TANH_SP = 0, /* the reference's algorithm: bp/bp.py, bp_vc.py, bp_cv.py     */
    LDPC_ALGO_MIN_SUM = 1, /* normalized/offset min-sum (new; see oracle/ldpc_oracle.c) */
    LDPC_ALGO_QMIN_SUM = 2 /* integer (quantized-LLR) offset min-sum (new)              */
};

enum {
    LDPC_F_EARLY_STOP = 1,    /* stop a codeword once its syndrome is zero                   */
    LDPC_F_DEVICE_PTRS = 2,   /* llr/bits/soft/iters_used are device pointers (else host)     */
    LDPC_F_F64 = 4,           /* tanh-SP in float64: llr/soft are double* (reference .double()) */
    LDPC_F_SOFT_Z = 8,        /* soft_out = z = 0.5*(L + sum c2v) (half posterior LLR, P0/P1)  */
    LDPC_F_FORCE_GENERIC = 16 /* never use a structure-specialised (QC) kernel                 */
};

typedef struct {
    int32_t iters;   /* iterations (maximum when LDPC_F_EARLY_STOP)                         */
    int32_t algo;    /* LDPC_ALGO_*                                                          */
    int32_t flags;   /* LDPC_F_*                                                             */
    float clamp;     /* c2v clamp, the reference's clamp_value (bp/bp.py:47)                 */
    float alpha;     /* min-sum normalisation (1 = plain min-sum; QMIN_SUM requires 1)       */
    float beta;      /* min-sum offset (float algo) / integer offset >= 0 (QMIN_SUM; a
                        non-integer beta is LDPC_EINVAL there)                               */
    int32_t qmax;    /* QMIN_SUM: message/LLR saturation (15 = 5-bit signed)                 */
    int32_t app_max; /* QMIN_SUM: posterior saturation                                       */
    float qstep;     /* QMIN_SUM: LLR quantizer step; q = sat(rint(llr * (1.0f / qstep)), qmax)
                        in fp32 (reciprocal multiply, not division: the two can round
                        differently at .5 boundaries)                                         */
} ldpc_params;

/* Build a Tanner graph from H in CSR form (rows = checks, ascending columns).  Replaces
 * generate_masks(H) (pytorch/bp/masking.py:12-147) and BeliefPropagation.__init__ (bp/bp.py:20-39):
 * the graph is built once and reused, instead of dense E x E masks rebuilt per decode_bits call
 * (ofdm/ofdm_functions.py:143/145).  If H is the lifting of a base matrix for which a specialised
 * kernel is compiled in (802.11n codes), the handle carries it. */
int ldpc_graph_create(int32_t m, int32_t n, int32_t nnz, const int32_t* row_ptr, const int32_t* col_idx,
                      int32_t device, ldpc_graph** out);

/* Same, from a QC base matrix: shifts[mb*nb] row-major, -1 = null block, lifting size z. */
int ldpc_graph_create_qc(int32_t mb, int32_t nb, int32_t z, const int32_t* shifts, int32_t device,
                         ldpc_graph** out);

int ldpc_graph_destroy(ldpc_graph* g);

/* m, n, nnz (=E, the reference's layer_size(), bp/bp.py:61-62), and the QC lifting size of the
 * specialised kernel in use (0 = generic CSR kernels). */
int ldpc_graph_info(const ldpc_graph* g, int32_t* m, int32_t* n, int32_t* nnz, int32_t* qc_z);

/* The kernel family a decode with these params runs on this graph: "qc-z<Z>" (register-resident
 * quasi-cyclic kernels, 802.11n), "ira-z360" (DVB-S2-structured IRA codes, min-sum, fixed count or early
 * stop) or
 * "generic-csr" (any H).  Introspection only (benchmarks label their records with it); NULL on bad
 * arguments.  The string is thread-local and valid until the next call on this thread.  No reference
 * counterpart: the reference has one code path (dense masks, bp/masking.py). */
const char* ldpc_kernel_path(const ldpc_graph* g, const ldpc_params* p);

/* Device bytes ldpc_decode_ex needs as caller-provided workspace for a batch of B codewords. */
int ldpc_workspace_size(const ldpc_graph* g, int64_t B, const ldpc_params* p, size_t* bytes);

/* Decode B codewords.  Replaces BeliefPropagation.forward(x=0, llr, clamp) -> p1 (bp/bp.py:43-51) and
 * the batch loop of decode_bits (ofdm/ofdm_functions.py:152-161).
 *   llr[B][n]     log P(bit=1)/P(bit=0), the reference's convention (ofdm_functions.py:72);
 *                 float* (double* with LDPC_F_F64).
 *   bits_out[B][n] 0/1 hard decisions, np.round(p1) semantics (ties -> 0).  May be NULL.
 *   soft_out[B][n] p1 = 1 - sigmoid(z) (or z with LDPC_F_SOFT_Z); float* (double* with F64).  May be NULL.
 *   iters_used[B] iterations run per codeword (== iters unless early stop).  May be NULL.
 *   workspace     device buffer of >= ldpc_workspace_size bytes, or NULL to use a per-graph internal
 *                 one (then the call is synchronous and serialised per graph).
 *   stream        hipStream_t as void* (NULL = default stream).  With LDPC_F_DEVICE_PTRS and a caller
 *                 workspace the call is asynchronous on the stream and graph-capturable; with host
 *                 pointers it copies in/out and returns after the stream synchronises. */
int ldpc_decode_ex(const ldpc_graph* g, const void* llr, int64_t B, const ldpc_params* p, uint8_t* bits_out,
                   void* soft_out, int32_t* iters_used, void* workspace, size_t workspace_bytes, void* stream);

/* Convenience form (float llr, internal workspace, alpha 1 / beta 0 / qmax 15 / app_max 127 / qstep 1) —
 * the signature SURVEY.md §8(b) sketches: iters_used[B] (may be NULL) as in ldpc_decode_ex.  Replaces the
 * same reference interface (bp/bp.py:43-51, ofdm/ofdm_functions.py:152-161); LDPC_F_F64 is ignored. */
int ldpc_decode(const ldpc_graph* g, const float* llr, int64_t B, int32_t iters, float clamp, int32_t algo,
                int32_t flags, uint8_t* bits_out, float* soft_out, int32_t* iters_used, void* stream);

/* Weighted BP — the reference module with trained (non-unit) VC weights: layers[i][0].input_weight
 * (E x E, masked by mask_v) and llr_weight (1 x n) per iteration, final_layer[0].input_weight (n x E) and
 * llr_weight (pytorch/bp/bp_vc.py:16-27, bp/bp.py:27-39).  Compact layout (element type = the decode
 * precision, DEVICE pointers, any may be NULL = all ones):
 *   vn      [iters][W]  vn[it*W + wofs[v] + t*d_v + u] = weight of var-slot u's c2v into var-slot t's v2c
 *                       (slot = position among v's edges in ascending check order; u == t unused);
 *                       W = sum_v d_v^2, wofs[v] = sum_{v' < v} d_v'^2
 *   llr     [iters][n]  per-variable LLR weight of each iteration
 *   fin     [E]         final layer: fin[var_ptr[v] + u] = weight of var-slot u into z_v
 *   fin_llr [n]
 * v2c = tanh(0.5 * (llr_w * L + sum_{u != t} w_tu * c2v_u)); z = 0.5 * (fin_llr * L + sum_u fin_u c2v_u).
 * tanh sum-product only, no early stop; always runs the generic CSR kernels (query the workspace with
 * LDPC_F_FORCE_GENERIC set). */
typedef struct ldpc_bp_weights {
    const void* vn;
    const void* llr;
    const void* fin;
    const void* fin_llr;
} ldpc_bp_weights;

int ldpc_weights_layout(const ldpc_graph* g, int64_t* vn_per_iter, int64_t* fin_len);
int ldpc_decode_weighted(const ldpc_graph* g, const void* llr, int64_t B, const ldpc_params* p,
                         const ldpc_bp_weights* w, uint8_t* bits_out, void* soft_out, int32_t* iters_used,
                         void* workspace, size_t workspace_bytes, void* stream);

/* BeliefPropagation.forward(x, llr, clamp) with NON-ZERO initial messages x (pytorch/bp/bp.py:43-47: the
 * first layer consumes x exactly as later layers consume the previous c2v).  x0: DEVICE [B][E] in the
 * reference's check-order edge numbering (masking.py:84-88), element type = the decode precision; NULL =
 * zeros.  w: optional weights as ldpc_decode_weighted (NULL = plain BP).  Requires LDPC_F_DEVICE_PTRS when
 * x0 is given; tanh sum-product without early stop; generic CSR kernels (workspace as LDPC_F_FORCE_GENERIC). */
int ldpc_decode_x0(const ldpc_graph* g, const void* llr, int64_t B, const ldpc_params* p, const ldpc_bp_weights* w,
                   const void* x0, uint8_t* bits_out, void* soft_out, int32_t* iters_used, void* workspace,
                   size_t workspace_bytes, void* stream);

/* The drop-in decode_bits (pytorch/ofdm/ofdm_functions.py:131-163) end to end from HOST memory: rows
 * codewords of float64 llr[rows][n] (log P1/P0) -> out[rows][n] float64 0.0/1.0 (np.round(p1) semantics).
 * The caller passes rows = (N // batch_size) * batch_size and leaves the remainder rows zero, as the
 * reference does (:133-135); every batch is independent, so the batches are decoded in chunks of `chunk`
 * codewords (0 = ~16 MB of float32 LLRs) through a two-slot pinned staging ring: the host converts chunk
 * c+1 to float32 (the reference's torch.tensor(..., dtype=torch.float), :156) while the GPU copies in,
 * decodes and copies out chunk c on its own stream, and the host expands chunk c-1's uint8 bits to float64.
 * `threads` host threads for the staging copies (0 = min(16, hardware threads)).  p: float32 arithmetic on
 * host buffers (LDPC_F_F64 / LDPC_F_DEVICE_PTRS / LDPC_F_SOFT_Z are EINVAL); synchronous. */
int ldpc_decode_bits_host(const ldpc_graph* g, const double* llr, int64_t rows, const ldpc_params* p, double* out,
                          int64_t chunk, int32_t threads);

/* Error counting on device, the metrics of evaluate_quantized.py:139-141 for one SNR point:
 *   counts[0] += bit errors over the first info_bits positions of each codeword (coded BER numerator)
 *   counts[1] += codewords with any error over all n positions              (coded BLER numerator)
 *   counts[2] += B
 * bits, ref: device uint8 [B][n]; counts: device int64[3] (accumulated, not cleared). */
int ldpc_count_errors(const uint8_t* bits, const uint8_t* ref, int64_t B, int32_t n, int32_t info_bits,
                      int64_t* counts, void* stream);

/* BPSK/AWGN channel on device: llr[b][v] = -2 y / sigma^2 with y = (1 - 2 c[b][v]) + sigma * N(0,1),
 * N from a counter-based generator keyed by (seed, b0 + b, v).  codeword may be NULL (all-zero).
 * Distributionally equal to the reference's QPSK-OFDM path for rate-1/2 at SNR = Eb/N0
 * (ofdm_functions.py:17-35,63-78). */
int ldpc_awgn_llr(const uint8_t* codeword, float* llr, int64_t B, int32_t n, float sigma, uint64_t seed,
                  int64_t b0, void* stream);

/* Uniform random information bits on device: out[b][i] = bit of Philox(key = seed, counter = (b0+b)*k + i),
 * so the bits of global codeword b0+b do not depend on how a sweep is sharded.  out: device uint8 [B][k]. */
int ldpc_random_bits(uint8_t* out, int64_t B, int32_t k, uint64_t seed, int64_t b0, void* stream);

/* OFDM transmitter, the reference's modulate_bits + transmit_symbols (ofdm/ofdm_functions.py:17-35):
 * bits[nsym * bits_per_symbol] (uint8, device) -> symbols (QPSK bits_per_symbol = 2, the reference's
 * mapping; 16-QAM = 4, Gray per dimension, new) -> blocks of ofdm_size -> unitary IDFT -> + complex AWGN
 * of per-dimension variance 1/(2 snr).  rx_out / tx_out: interleaved complex float [nsym][2] (tx_out may
 * be NULL).  Noise of stream sample sym0 + i is keyed by (seed, sym0 + i). nsym % ofdm_size == 0. */
int ldpc_ofdm_tx(const uint8_t* bits, int64_t nsym, int32_t ofdm_size, int32_t bits_per_symbol, float snr,
                 uint64_t seed, int64_t sym0, float* rx_out, float* tx_out, void* stream);

/* OFDM receiver, the reference's demodulate_signal (ofdm_functions.py:63-78): unitary DFT per block,
 * LLR = log P(1)/P(0) per bit with noise_power 0.5/snr (QPSK: the reference's closed form; 16-QAM:
 * exact log-sum-exp).  llr_out: float [nsym * bits_per_symbol]; sym_out (may be NULL): [nsym][2]. */
int ldpc_ofdm_demod(const float* rx, int64_t nsym, int32_t ofdm_size, int32_t bits_per_symbol, float snr,
                    float* llr_out, float* sym_out, void* stream);

/* ADC quantizer — replaces quantizer (pytorch/ofdm/ofdm_functions.py:37-51) and the AGC of gen_qdata
 * (:118-128).  rx / q_out: complex64 interleaved DEVICE buffers [nsym].  Exactly one of clip_ratio (AGC:
 * clip = std(rx) * clip_ratio computed on device over these nsym samples, as np.std of the complex
 * signal) or clip_value (fixed clip) must be > 0.  Arithmetic in fp64 as the reference:
 * step = 2 clip / (2^b - 1), q = clip(step * floor(x/step + .5), -(2^b/2) step + 1, (2^b/2) step - 1).
 * clip_out (optional, device double) receives the clip used in AGC mode.  Asynchronous on stream. */
int ldpc_adc_quantize(const float* rx, int64_t nsym, int32_t num_bits, double clip_ratio, double clip_value,
                      float* q_out, double* clip_out, void* stream);

const char* ldpc_last_error(void);
int ldpc_device_count(void);
const char* ldpc_version(void);
/* LDPC_ABI_VERSION of the header the library was built from (compare before binding any other symbol). */
int ldpc_abi_version(void);

#ifdef __cplusplus
}
#endif
#endif /* LDPC_ABI_H */
