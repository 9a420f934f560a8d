/*
 * fpldpc.h -- C ABI of the MI355X-native fixed-point LDPC decoder (libfpldpc.so).
 *
 * Drop-in boundary for the reference's decode path (tyc85/FixedPointLDPC).  The reference has
 * no FFI of its own: its "operator API" is the FP_Decoder class (ArrayLDPCMacro.h:121-158) and
 * the PerfTest.h free functions.  Every entry point below names the reference interface it
 * replaces.  The C++ class-level compatibility layer (FP_Decoder / PerfTest names) is in
 * fpldpc_compat.hpp and is built on this ABI.
 *
 * Conventions
 *   - Every function returns int status: FPLDPC_OK (0) or a negative FPLDPC_ERR_* code; the
 *     message of the last error on the calling thread is fpldpc_last_error().
 *   - "dev" pointers are HIP device pointers, "host" pointers are host memory.  Streams are
 *     hipStream_t passed as void* (NULL = the null stream).
 *   - Decoder objects are independent (no function-static state, unlike the reference's
 *     decode_general_fp, ArrayLDPC_Decoder.cpp:21-37); one object may be used from one thread at
 *     a time, different objects concurrently.
 *   - A decoder is single-stream: its decode calls share one device work counter and fallback
 *     list, so two calls on the same decoder must not overlap on the device (issue them on one
 *     stream, or synchronise between streams).  Use one decoder per stream for concurrency.
 */
#ifndef FPLDPC_H
#define FPLDPC_H
#include <stddef.h>
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

#define FPLDPC_OK 0
#define FPLDPC_ERR_ARG (-1)         /* invalid argument */
#define FPLDPC_ERR_IO (-2)          /* file open/read failed (reference: ignored, ReadH :646) */
#define FPLDPC_ERR_FORMAT (-3)      /* malformed / inconsistent alist */
#define FPLDPC_ERR_UNSUPPORTED (-4) /* code shape outside the kernels' envelope */
#define FPLDPC_ERR_HIP (-5)         /* HIP runtime error or no GPU / kernel image */
#define FPLDPC_ERR_NOMEM (-6)

#define FPLDPC_LLR_I32 0 /* const int32_t LLR[batch][n] (the reference's const int *LLR) */
#define FPLDPC_LLR_I16 1 /* const int16_t LLR[batch][n] (compact: |LLR_fp| <= 644 measured) */
#define FPLDPC_LLR_F64 2 /* double LLR[batch][n], unquantised (channel output for fpldpc_decode_float) */

typedef struct fpldpc_code *fpldpc_code_t;
typedef struct fpldpc_decoder *fpldpc_decoder_t;

/* Decoder parameters.  The reference fixes these at compile time (ArrayLDPCMacro.h:17-39). */
typedef struct {
    int32_t max_iter;   /* MAX_ITER, ArrayLDPCMacro.h:17 (default 30) */
    int32_t frac_bits;  /* FRAC_WIDTH, ArrayLDPCMacro.h:36; Constant = int(5/8 * 2^frac) (default 4) */
    int32_t width_mask; /* WIDTH_MASK, ArrayLDPCMacro.h:29, applied inside sxor (default 0xff) */
    int32_t early_term; /* 1 = stop at the first passing syndrome, ArrayLDPC_Decoder.cpp:164-167 (default 1) */
    int32_t precheck;   /* 1 = decode_fixpoint's channel-syndrome pre-check, ArrayLDPC_Decoder.cpp:443-450
                           (iterations 0, hard = channel decision, posteriors left untouched) (default 0) */
    int32_t device;     /* HIP device ordinal; -1 = the calling thread's current device (default -1) */
} fpldpc_params;

const char *fpldpc_last_error(void);
const char *fpldpc_version(void);
/* Content hash (16 hex digits) of the device sources and compile flags this library was built
 * from (no reference counterpart): committed profiler counters are bound to it, so that counters
 * measured on one kernel build are never reported for another. */
const char *fpldpc_kernel_build_id(void);

/* ---------------------------------------------------------------- parity-check codes */
/* Replaces FP_Decoder::ReadH() (ArrayLDPC_Decoder.cpp:642-674), which hard-codes
 * "H_802.11_IndZero.txt" and ignores errors.  Alist format: N M / dv_max dc_max / vdeg[N] /
 * cdeg[M] / N vlist rows / M clist rows, 0-based.  Validated: rows ascending (the reference's
 * addr_count bank selection relies on it, :137), vlist/clist consistent, 2 <= cdeg. */
int fpldpc_code_load_alist(const char *path, fpldpc_code_t *out);
int fpldpc_code_parse_alist(const char *text, size_t len, fpldpc_code_t *out);
/* Array code, p prime, r block rows: check (i,j) <-> var k*p + (j + i*k) mod p ("forward",
 * ROM::CirShift ArrayLDPCMacro.h:57 and codes/alist_from_arraycode.m) or (j - i*k) mod p. */
int fpldpc_code_array(int32_t p, int32_t r, int32_t forward, fpldpc_code_t *out);
/* IEEE 802.11n rate-1/2 n=1944 (Z=81) code, the reference's H_802.11_IndZero.txt. */
int fpldpc_code_wifi_1944_r12(fpldpc_code_t *out);
/* dims[0..7] = n, m, dv_max, dc_max, edges, qc_z (0 if not quasi-cyclic), gf2_rank, regular_checks */
int fpldpc_code_dims(fpldpc_code_t code, int32_t dims[8]);
/* ROM::getRate (ArrayLDPCMacro.h:60) for array codes, 1 - rank/n otherwise. */
int fpldpc_code_rate(fpldpc_code_t code, double *rate);
/* Copy out degree and adjacency lists (row-padded to dv_max / dc_max with -1).  Any may be NULL. */
int fpldpc_code_lists(fpldpc_code_t code, int32_t *vdeg, int32_t *cdeg, int32_t *vlist, int32_t *clist);
/* Serialise to alist text; *len receives the size needed (excluding NUL). */
int fpldpc_code_write_alist(fpldpc_code_t code, char *buf, size_t cap, size_t *len);
/* Syndrome of hard bits (uint8 per var) on the host: returns 0 pass, 1 fail, <0 error. */
int fpldpc_code_syndrome_host(fpldpc_code_t code, const uint8_t *bits);
void fpldpc_code_free(fpldpc_code_t code);

/* ---------------------------------------------------------------- decoder */
void fpldpc_params_default(fpldpc_params *p);
/* Replaces constructing FP_Decoder (ArrayLDPCMacro.h:121-176) + ReadH.  Uploads the code's
 * edge tables to the device and picks the kernel variant for the code shape. */
int fpldpc_decoder_create(fpldpc_code_t code, const fpldpc_params *params, fpldpc_decoder_t *out);
int fpldpc_decoder_destroy(fpldpc_decoder_t dec);
/* Kernel variant chosen (e.g. "flood_reg<47,1,regular>") and its resident workgroups. */
int fpldpc_decoder_describe(fpldpc_decoder_t dec, char *buf, size_t cap);
/* Words per frame of the packed hard-decision output: ceil(n / 32). */
int fpldpc_decoder_hard_words(fpldpc_decoder_t dec);
/* Diagnostics (no reference counterpart): frames the most recent fpldpc_decode call on this
 * decoder re-decoded in its exact fallback chain -- counts[0] by the first fallback kernel (frames
 * that left the packed kernel's int16 range, plus a partner sharing their posterior words),
 * counts[1] by the second.  Both 0 for variants without a chain.  Blocking: waits for the last
 * decode call's kernels on whatever stream they were launched (a decode captured into a graph is
 * not tracked: synchronise its replay first). */
int fpldpc_decoder_fallback_counts(fpldpc_decoder_t dec, int32_t counts[2]);

/* Reference information bits for on-device BER accounting.  Replaces setInfoIndex
 * (ArrayLDPC_Decoder.cpp:698-705) + setInfoBit (:178-197): errors are counted as
 * DecodedCodeword[info_index[i]] != info_bits[i] over i < k (calculateBER, :707-722).
 * Host pointers; copied.  k = 0 clears. */
int fpldpc_set_reference(fpldpc_decoder_t dec, const int32_t *info_index, const uint8_t *info_bits, int32_t k);

/* Batched flooding decode of `batch` frames, asynchronous on `stream` (all pointers device).
 * Replaces per-frame FP_Decoder::decode_general_fp (ArrayLDPC_Decoder.cpp:18-171), or
 * decode_fixpoint (:422-639) when params.precheck = 1, and the result getters.
 *   llr        [batch][n] FPLDPC_LLR_I32 or _I16                              (required)
 *   hard       [batch][hard_words] uint32, bit (v % 32) of word v/32 = DecodedCodeword[v]
 *   iters      [batch] returned iteration count (1..max_iter; 0 on a pre-check pass)
 *   syndrome_ok[batch] 1 if the output hard decision satisfies H
 *   post       [batch][n] int32 Posteriori_fp (getPost_fp, ArrayLDPCMacro.h:138)
 *   bit_errors [batch] calculateBER per frame (needs fpldpc_set_reference)
 *   totals     [4] int64, ADDED to: {bit_errors, frame_errors, frames, iteration_sum}
 * Any output may be NULL.  Bit-exact with the reference decoder for every frame. */
int fpldpc_decode(fpldpc_decoder_t dec, const void *llr, int32_t llr_type, int32_t batch,
                  uint32_t *hard, int32_t *iters, uint8_t *syndrome_ok, int32_t *post,
                  int32_t *bit_errors, int64_t *totals, void *stream);
/* Same on host buffers (synchronous; stages through device memory owned by the decoder). */
int fpldpc_decode_host(fpldpc_decoder_t dec, const void *llr, int32_t llr_type, int32_t batch,
                       uint32_t *hard, int32_t *iters, uint8_t *syndrome_ok, int32_t *post,
                       int32_t *bit_errors, int64_t *totals);

/* Stateful single-frame decode: FP_Decoder::decode_general_fp / decode_fixpoint with the decoder's
 * edge RAM kept across calls, as the reference's FSM uses it (ArrayLDPC_Decoder.cpp:443-488,
 * :621-630).  edge_ram is FP_Decoder's EdgeRAM (ArrayLDPCMacro.h:162), owned by the caller:
 * int32 edge_ram[k * m + c] = the v2c message on slot k (clist order) of check c as the last
 * variable-node phase left it (accum - c2v, :152 and :615); fpldpc_edge_ram_words gives dc_max * m.
 *   keep_edges = 0: edge init from the channel values first (:45-61, decode_fixpoint in state PCV
 *                   :462-485) -- decode_general_fp, or decode_fixpoint after setState(PCV);
 *   keep_edges = 1: no edge init: iterate from edge_ram with these LLRs in the variable-node phase
 *                   -- decode_fixpoint in state C2V without setState(PCV) (:488-618).
 * With params.precheck the channel syndrome is tested first (:443-450): on a pass the frame returns
 * 0 iterations with the channel decision and edge_ram / post left as they were.  Otherwise edge_ram
 * is overwritten with the final edge messages; iterations, hard decisions, syndrome flag and
 * posteriors as fpldpc_decode for one frame.  One workgroup of the int32 kernel (flood_edges):
 * the per-frame drop-in path; batches belong to fpldpc_decode.  Device pointers, async on stream.
 * The decoder holds one c2v scratch for this path: calls on one decoder must be serialised (one
 * stream, or wait for the previous call), even with distinct edge_ram buffers -- independent
 * per-channel states need one decoder each. */
int fpldpc_edge_ram_words(fpldpc_decoder_t dec, int64_t *words);
int fpldpc_decode_frame(fpldpc_decoder_t dec, const void *llr, int32_t llr_type, int32_t keep_edges,
                        int32_t *edge_ram, uint32_t *hard, int32_t *iters, uint8_t *syndrome_ok,
                        int32_t *post, void *stream);
/* Same on host buffers (synchronous); llr int32[n]; post (nullable) in/out like fpldpc_decode_host. */
int fpldpc_decode_frame_host(fpldpc_decoder_t dec, const int32_t *llr, int32_t keep_edges, int32_t *edge_ram,
                             uint32_t *hard, int32_t *iters, uint8_t *syndrome_ok, int32_t *post);

/* Floating-point BP decode (exact-Jacobian box-plus in double), replacing FP_Decoder::decode_general
 * (ArrayLDPC_Decoder.cpp:735-933, sxor(double,double) :724-732, checkPost :335-372) batched, async
 * on `stream`, device pointers.  llr [batch][n] double (unquantised, e.g. fpldpc_channel_llr with
 * FPLDPC_LLR_F64); post [batch][n] double (getPost, ArrayLDPCMacro.h:149); the other outputs as
 * fpldpc_decode.  Uses params.max_iter and early_term; frac_bits, width_mask and precheck do not
 * apply.  Same flooding schedule and fold order as the reference, but by default each check's exact
 * box-plus is folded in the tanh domain (E = exp(-|x|), E_r = (E_x + E_y) / (1 + E_x E_y), one exp
 * in and one log out per edge); the reference's log-domain operation order is used only for a check
 * holding a message >= 690 in magnitude, or in a build with -DFPLDPC_FLOAT_TANH=0.  Different
 * rounding, same decisions: tests/test_gpu_float.py requires 0 frames differing in iterations / hard
 * decisions from the reference's fixtures and the oracle, and posteriors within 1e-8 relative
 * (measured worst 3.4e-9).  Supports n <= 16384, degrees <= 255. */
int fpldpc_decode_float(fpldpc_decoder_t dec, const double *llr, int32_t batch, uint32_t *hard,
                        int32_t *iters, uint8_t *syndrome_ok, double *post, int32_t *bit_errors,
                        int64_t *totals, void *stream);
/* Same on host buffers (synchronous). */
int fpldpc_decode_float_host(fpldpc_decoder_t dec, const double *llr, int32_t batch, uint32_t *hard,
                             int32_t *iters, uint8_t *syndrome_ok, double *post, int32_t *bit_errors,
                             int64_t *totals);

/* ---------------------------------------------------------------- channel model */
/* Lehmer state after `draws` calls of Random() from `seed` (rngs.cpp:52-69, a = 48271,
 * m = 2^31 - 1): seed * a^draws mod m. */
int64_t fpldpc_rng_skip(int64_t seed, uint64_t draws);
/* Quantised BPSK/AWGN LLRs exactly as the reference harness (PerfTest.cpp:108-120, 287-297):
 *   LLR_fp[f][i] = (int)(2*snr*(1 - 2*cw[i] + Normal(0, sigma)) * 2^frac_bits)
 * Normal = Odeh-Evans inverse CDF on one Random() draw (rvgs.cpp:152-181); frame f uses draws
 * [f*n, (f+1)*n) of the stream started at `seed` (the reference never re-seeds, rngs.cpp:47).
 * cw (uint8[n]) NULL = all-zero codeword.  out is [frames][n] of out_type; FPLDPC_LLR_F64 stores
 * the unquantised double 2*snr*(...) (PerfTest.cpp:108-110, the float decoder's input).
 * nthreads <= 0: all.
 * Returns FPLDPC_ERR_ARG if a value does not fit int16 for FPLDPC_LLR_I16. */
int fpldpc_channel_llr_host(int64_t seed, int64_t first_frame, int32_t frames, int32_t n,
                            double snr, double sigma, int32_t frac_bits, const uint8_t *cw,
                            void *out, int32_t out_type, int32_t nthreads);
/* The same channel on the device, asynchronous on `stream` (hipStream_t, NULL = default): every
 * pointer is device memory.  cw NULL = all-zero codeword; else cw is uint8[n] shared by all frames
 * (cw_per_frame = 0) or uint8[frames][n] (cw_per_frame = 1, e.g. fpldpc_encoder_encode output).
 * The Lehmer states are the host's exactly; the normals use the device's double log/sqrt, so an
 * LLR can in principle differ from the host's by one quantum where the product lands within an
 * ulp of an integer (never observed: tests/test_gpu_gen.py compares the full KAT-W stream).
 * For FPLDPC_LLR_I16, the number of values outside int16 is added to *overflow (device int32, may
 * be NULL; the caller zeroes it); such values are stored truncated to 16 bits. */
int fpldpc_channel_llr(int64_t seed, int64_t first_frame, int32_t frames, int32_t n, double snr,
                       double sigma, int32_t frac_bits, const uint8_t *cw, int32_t cw_per_frame,
                       void *out, int32_t out_type, int32_t *overflow, void *stream);

/* ---------------------------------------------------------------- systematic encoder */
/* Replaces FP_Encoder (ArrayLDPC_Encoder.cpp:22-225, decl ArrayLDPCMacro.h:179-214). */
typedef struct fpldpc_encoder *fpldpc_encoder_t;
/* FP_Encoder(char *Filename, int) (:34-157): the reference's G file ("N M_G / x cmax /
 * ColumnFlag[N] / ChkDeg[M_G] / rows").  Unlike the reference, errors are returned, not exit(0). */
int fpldpc_encoder_load_g(const char *path, fpldpc_encoder_t *out);
/* The same encoder derived natively from H (what codes/simplfy_generator_alist.m made offline):
 * parity positions = pivot columns of a column-order GF(2) row reduction, info = the rest in
 * ascending order; identical to the reference's G files for its codes (tests/test_encoder.py). */
int fpldpc_encoder_from_code(fpldpc_code_t code, fpldpc_encoder_t *out);
/* dims = n, k, max parity-row weight */
int fpldpc_encoder_dims(fpldpc_encoder_t enc, int32_t dims[3]);
/* getInfoIndex (ArrayLDPCMacro.h:186): info_index[k], parity_index[n-k]; either may be NULL. */
int fpldpc_encoder_info_index(fpldpc_encoder_t enc, int32_t *info_index, int32_t *parity_index);
/* setInfoBit / encode bit unpacking of a char stream (ArrayLDPC_Decoder.cpp:178-197). */
int fpldpc_unpack_info_bytes(const char *in, int32_t in_len, int32_t k, uint8_t *bits);
/* encode (:160-225) of `batch` frames: info [batch][k] bits -> cw [batch][n] bits (host). */
int fpldpc_encoder_encode_host(fpldpc_encoder_t enc, const uint8_t *info, int32_t batch, uint8_t *cw, int32_t nthreads);
/* The same on the device, asynchronous on `stream`: info [batch][k] and cw [batch][n] are device
 * uint8 arrays (bit in the LSB).  The encoder binds to the current device on first use and keeps
 * a packed-info scratch sized to the largest batch seen: like a decoder, one encoder object is
 * used from one thread / stream at a time. */
int fpldpc_encoder_encode(fpldpc_encoder_t enc, const uint8_t *info, int32_t batch, uint8_t *cw, void *stream);
void fpldpc_encoder_free(fpldpc_encoder_t enc);

/* ---------------------------------------------------------------- BER/FER simulation */
/* The frame loop the reference's harness runs around one decoder (ArrayLDPC_Debug_Wifi
 * PerfTest.cpp:97-135, ArrayLDPC_Debug :275-311, ArrayLDPC_Debug_Shorten :385-426,
 * ArrayLDPC_PerfTest :485-511, ArrayLDPC_TimeTrial :574-600), batched: frames are generated on the
 * host (channel model above, skip-ahead, all threads) while the GPU decodes the previous chunk, and
 * errors are accounted IN FRAME ORDER so that "stop at the frame with the Nth frame error" is
 * reproduced exactly.  Two chunks are in flight: the call creates a twin of `dec` (same code,
 * parameters and kernel choice, no diagnostics; its own stream and a second set of decoder device
 * buffers, about the decoder's own footprint) for the duration of the call, and submits the next
 * chunk before waiting for the current one, so that its launch fills the CUs a chunk's last frames
 * leave idle (environment FPLDPC_SIM_OVERLAP=0: one chunk at a time on `dec` alone).  Counters are
 * the same either way; a chunk decoded past the stop frame is waited for and not counted. */
#define FPLDPC_COUNT_BITS 0  /* blkerror = calculateBER() (ArrayLDPC_Decoder.cpp:707-722) */
#define FPLDPC_COUNT_ITERS 1 /* blkerror = decode_fixpoint()'s return value: the reference's
                                ArrayLDPC_PerfTest/TimeTrial count iterations as bit errors
                                (PerfTest.cpp:507-510, 596-600); kept for output parity */
typedef struct {
    int64_t seed;                 /* Lehmer state of draw 0 (rngs.cpp:45 DEFAULT = 123456789) */
    int64_t first_frame;          /* frame f uses draws [f*n, (f+1)*n) */
    double snr, sigma;            /* LLR = 2*snr*(1 - 2c + Normal(0, sigma)), PerfTest.cpp:108-120 */
    int32_t frac_bits;            /* LLR_fp = (int)(LLR * 2^frac_bits) */
    const uint8_t *codeword;      /* [n] transmitted codeword, NULL = all-zero */
    const int32_t *info_index;    /* [k] setInfoIndex (host) */
    const uint8_t *info_bits;     /* [k] setInfoBit (host) */
    int32_t k;
    const int32_t *forced_index;  /* shortening: LLR_fp[forced_index[i]] = forced_llr after the */
    int32_t n_forced;             /* channel (PerfTest.cpp:410-414); NULL/0 = none */
    int32_t forced_llr;
    int64_t max_frame_errors;     /* stop at the frame that reaches this many frame errors (0 = none) */
    int64_t max_frames;           /* stop after this many frames (0 = none); one limit is required */
    int32_t count_mode;           /* FPLDPC_COUNT_* */
    int32_t chunk;                /* frames per launch (0 = auto) */
    int32_t host_threads;         /* channel threads (<= 0 = all) */
    /* optional, called in frame order for every counted frame (e.g. ArrayLDPC_Debug_Shorten
     * prints each decode_fixpoint return value, PerfTest.cpp:419) */
    void (*on_frame)(void *ctx, int64_t frame, int32_t iterations, int64_t blkerror);
    void *on_frame_ctx;
    int32_t device_channel;       /* 1 = generate the LLRs on the device (fpldpc_channel_llr) in the
                                     decoding stream instead of on host threads (default 0) */
} fpldpc_sim_params;

typedef struct {
    int64_t bit_errors, frame_errors, frames, iter_sum; /* over frames [first_frame, first_frame + frames) */
    int64_t frames_decoded;       /* incl. the tail of the last waited chunk past the stop frame */
    double seconds;               /* wall time of the whole simulation */
} fpldpc_sim_result;

void fpldpc_sim_params_default(fpldpc_sim_params *p);
int fpldpc_ber_sim(fpldpc_decoder_t dec, const fpldpc_sim_params *sp, fpldpc_sim_result *out);

/* The same simulation over `ndev` decoders (one per device; SURVEY §8e: codeword batches shard
 * across the GPUs of a node), one host thread per decoder.  Frames go out in rounds: in round r
 * decoder i takes frames [first_frame + (r*ndev + i)*chunk, +chunk), so frame f keeps draws
 * [f*n, (f+1)*n) of the one channel stream; after each round the decoders exchange their chunk sums
 * (an all-gather), the one holding the stop frame locates it, and an all-reduce adds the counts.
 * The result equals fpldpc_ber_sim's (same frames, same counters) for any ndev and chunk.
 * Replaces the reference's single-threaded frame loop (PerfTest.cpp:97-135) on a multi-GPU node.
 *   collective: FPLDPC_COLL_RCCL  = RCCL communicators over the decoders' devices (ncclCommInitAll in
 *                                   this process; collectives on each decoder's stream, xGMI on MI355X);
 *                                   the devices must be distinct
 *               FPLDPC_COLL_HOST  = exchange through host memory (decoders may share a device)
 *               FPLDPC_COLL_AUTO  = RCCL when ndev > 1 and the devices are distinct, else host
 *   collective_used (nullable) receives the one that ran (HOST after an AUTO fallback, whose RCCL
 *   error goes to stderr).  Every decoder must be a different object
 *   (each is single-stream) on the same code; on_frame is called in frame order from one thread. */
#define FPLDPC_COLL_AUTO 0
#define FPLDPC_COLL_RCCL 1
#define FPLDPC_COLL_HOST 2
int fpldpc_ber_sim_multi(const fpldpc_decoder_t *decs, int32_t ndev, const fpldpc_sim_params *sp,
                         int32_t collective, fpldpc_sim_result *out, int32_t *collective_used);

#ifdef __cplusplus
}
#endif
#endif /* FPLDPC_H */
