/*
 * polar_mi355x.h -- C ABI of the MI355X (gfx950) SC / SC-list polar decoder library.
 *
 * This is the drop-in boundary for the hot path named in BASELINE.json: the Python decoder
 * modules (polar_amd.SC_Dec / SCL_Dec, mirroring the reference constructors and forward())
 * call these entry points through ctypes.  All pointers are device pointers unless a comment
 * says otherwise; the caller (PyTorch) owns every buffer; launches are asynchronous and
 * ordered on the given hipStream_t (passed as void*; NULL = legacy default stream).
 * No exceptions cross this boundary: 0 = success, negative = error, details from
 * pl_last_error_string() (thread-local).
 *
 * Plans are device-bound: pl_plan_create allocates the plan's tables and loads its kernel module
 * on the device current at that call (hipSetDevice).  Decode/encode calls must pass a stream of
 * that device (or NULL with that device current); any other device gives PL_EINVAL.  Create one
 * plan per GPU to decode on several GPUs.
 *
 * Reference interfaces replaced (jaco267/polar-code-pytorch-sionna):
 *   pl_plan_create   SC_Dec.__init__   x_run_sn_polar/polar/polar_sc.py:10-32
 *                    SCL_Dec.__init__  x_run_sn_polar/polar/polar_scl.py:13-42
 *                    (my_sn/fec/polar/dec.py:18-31 and :183-242 for the exact-f variants)
 *   pl_sc_decode     SC_Dec.forward    x_run_sn_polar/polar/polar_sc.py:113-133
 *                    (f_mode=PL_F_EXACT: my_sn/fec/polar/dec.py:130-157)
 *   pl_plan_info / pl_plan_device: the plan's n, k, list size (polar_sc.py:14-17) and device
 *   pl_scl_decode    SCL_Dec.forward   x_run_sn_polar/polar/polar_scl.py:210-234
 *                    (+ final sorted msg_pm of _decode_np_batch :178-209)
 *   pl_polar_encode  PolarEncoder.forward x_run_sn_polar/polar/enc.py:30-43
 *                    (butterfly form of my_sn/fec/polar/enc.py:85-96)
 *   pl_crc_attach    CRCEncoder.forward my_sn/fec/crc.py:85-104 (G-matrix CRC, 5G polynomials :38-52)
 *   pl_crc_check     CRCDecoder.forward my_sn/fec/crc.py:119-138 (re-encode, valid iff parity == 0)
 *   pl_gather_rows   Polar5GEncoder.forward rate matching c[:, ind_rate_matching]
 *                    my_sn/fec/polar/enc.py:378-392
 *   pl_rate_recover  Polar5GDecoder.forward rate recovery my_sn/fec/polar/dec.py:621-654
 *   pl_plan_kernel / pl_sc_specialize: no reference counterpart (kernel specialisation per
 *                    frozen set, the tree walk of polar_sc.py:54-98 resolved at compile time)
 */
#ifndef POLAR_MI355X_H
#define POLAR_MI355X_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PL_OK 0
#define PL_EINVAL -1  /* bad argument / shape */
#define PL_EHIP -2    /* HIP runtime error */
#define PL_ENOTSUP -3 /* configuration not supported by this build */

#define PL_F_MINSUM 0 /* f = sign*sign*min(|x|,|y|) on clipped inputs (polar_sc.py:46) */
#define PL_F_EXACT 1  /* f = log(1+e^(x+y)) - log(e^x+e^y) (my_sn dec.py:39-43) */
#define PL_F_WIDE_RANGE 0x100 /* pl_sc_source / pl_sc_specialize: or-ed into PL_F_EXACT, the code object
                                 of plans whose llr_max exceeds 43 (full-range exp/log); without it,
                                 the code object of plans with llr_max <= 43 */

#define PL_PLAN_GENERIC 1u    /* pl_plan_create flag: never specialise the SC kernel */
#define PL_PLAN_CACHE_ONLY 2u /* pl_plan_create flag: use a cached specialised kernel, never compile */
#define PL_PLAN_FAST_SCL 4u   /* pl_plan_create flag (SCL): fast-SCL rate-0 / repetition pruning of
                                 my_sn/fec/polar/dec.py:367-376 (use with f_mode PL_F_EXACT for
                                 my_sn SCL_Dec semantics) */
#define PL_PLAN_JIT 8u        /* pl_plan_create flag (SC): compile a specialised kernel missing from
                                 the caches in this process (hiprtc, seconds); without it a cache
                                 miss runs the generic kernel */

#define PL_KERNEL_GENERIC 0     /* pl_plan_kernel kinds */
#define PL_KERNEL_SPECIALIZED 1
#define PL_KERNEL_SCL_SUBTREE 2 /* SCL plans: lane-per-path register-subtree kernel (default for
                                   2 <= L <= 32, 32 <= n <= 1024, no fast-SCL pruning) */

#define PL_OUT_F32 0  /* output 0.0f/1.0f floats, [bs, k] (reference output dtype) */
#define PL_OUT_U8 1   /* output 0/1 bytes, [bs, k] */

typedef struct pl_plan pl_plan;

/* Build an immutable decoding plan for a length-n polar code.
 * frozen_mask: HOST pointer to n bytes, nonzero = frozen position (frozen_pos of the reference).
 * list_size:   1 for SC plans; a power of two <= 32 for SCL plans.
 * f_mode:      PL_F_MINSUM or PL_F_EXACT.  llr_max: clipping bound (reference: 30; at most 700
 *              for list_size > 1, where log(1 + exp(llr_max)) must stay finite).
 * flags:       0, or PL_PLAN_GENERIC / PL_PLAN_CACHE_ONLY / PL_PLAN_JIT (/ PL_PLAN_FAST_SCL).
 *              An SC plan (list_size 1) runs a kernel specialised to its frozen set when a code
 *              object for it is cached ($PL_KERNEL_CACHE, <library dir>/kcache,
 *              ~/.cache/polar_mi355x; pl_sc_source + hipcc --genco, or pl_sc_specialize, put it
 *              there), otherwise the generic kernel (also exact).  PL_PLAN_JIT compiles a missing
 *              one in-process with hiprtc at plan creation (seconds; not in a process whose HIP
 *              runtime came with another ROCm's amd_comgr, e.g. torch's).  PL_SC_SPECIALIZE=0 in
 *              the environment selects the generic kernel.
 * n must be a power of two, 2 <= n <= 2048.  List plans: list_size <= 32 for n <= 1024,
 * list_size <= 16 at n = 2048 (the list state of one codeword must fit one CU's LDS); larger ones
 * are rejected here with PL_ENOTSUP. */
int pl_plan_create(pl_plan** out, int32_t n, const uint8_t* frozen_mask, int32_t list_size,
                   int32_t f_mode, float llr_max, uint32_t flags);
int pl_plan_destroy(pl_plan* plan);
/* n, k (information bits) and list size of a plan (any pointer may be NULL). */
int pl_plan_info(const pl_plan* plan, int32_t* n, int32_t* k, int32_t* list_size);
/* The HIP device the plan was created on (its tables and kernel module live there). */
int pl_plan_device(const pl_plan* plan, int32_t* device);

/* SC decode.  llr_logits: [bs, n] fp32 logits log(P(b=1)/P(b=0)) (NOT negated; the decoder
 * negates, polar_sc.py:122).  out_bits: [bs, k] decided information bits at info_pos ascending,
 * dtype per out_kind (PL_OUT_F32 / PL_OUT_U8). */
int pl_sc_decode(const pl_plan* plan, const float* llr_logits, int64_t bs, void* out_bits,
                 int32_t out_kind, void* hip_stream);

/* SCL decode.  out_pm (nullable): [bs, 2L] fp64, the reference's final sorted msg_pm.
 * workspace: device scratch of pl_scl_workspace_size(plan, bs) bytes -- the exact-f list kernels
 * keep path-independent caches of the upper tree there (22 KB per codeword at n = 1024, for at
 * most 16384 codewords: larger batches are decoded in chunks over it).  NULL with ws_bytes 0 runs
 * without them (same results, slower); a non-NULL workspace smaller than the size is PL_EINVAL. */
size_t pl_scl_workspace_size(const pl_plan* plan, int64_t bs);
int pl_scl_decode(const pl_plan* plan, const float* llr_logits, int64_t bs, void* out_bits,
                  int32_t out_kind, double* out_pm, void* workspace, size_t ws_bytes,
                  void* hip_stream);

/* Polar encoding with the plan's frozen set: u_bits [bs, k] fp32 0/1 -> codewords [bs, n] fp32. */
int pl_polar_encode(const pl_plan* plan, const float* u_bits, int64_t bs, float* codewords,
                    void* hip_stream);

/* CRC-aided SCL (my_sn/fec/polar/dec.py:507-518): after decoding, every path whose k decoded
 * bits fail the CRC (generator x^degree + sum of the bits of poly_mask, MSB-first shift register,
 * my_sn/fec/crc.py) gets +llr_max*k on its metric (the plan's llr_max; 30 in the reference,
 * dec.py:517) before the first argmin.  degree 0 turns it off.
 * Call before the plan's first decode.  Replaces SCL_Dec(crc_degree=...) (dec.py:210-218). */
int pl_plan_set_crc(pl_plan* plan, int32_t degree, uint32_t poly_mask);

/* Which kernel a plan launches: *kind = PL_KERNEL_GENERIC / PL_KERNEL_SPECIALIZED (SC plans) or
 * PL_KERNEL_GENERIC / PL_KERNEL_SCL_SUBTREE (SCL plans; PL_PLAN_GENERIC or PL_SCL_TREE=0 in the
 * environment select the generic SCL kernel); path
 * (nullable) receives the code object file of a specialised kernel. */
int pl_plan_kernel(const pl_plan* plan, int32_t* kind, char* path, size_t path_len);

/* Compile (or find) the specialised SC kernel of a code into cache_dir (NULL = default cache)
 * without touching a GPU; path (nullable) receives the code object file.  Used to pre-build the
 * kernels of known codes.  f_mode: PL_F_MINSUM, PL_F_EXACT or PL_F_EXACT | PL_F_WIDE_RANGE (an
 * exact-f plan picks one of the two by its llr_max). */
int pl_sc_specialize(int32_t n, const uint8_t* frozen_mask, int32_t f_mode, const char* cache_dir,
                     char* path, size_t path_len);
/* The HIP source of the specialised SC kernel of a code and its cache file name (what
 * pl_sc_specialize would compile and look up), for compiling it out of process (hipcc --genco;
 * polar_amd/build.py).  *src_size = bytes needed including the NUL; src may be NULL. */
int pl_sc_source(int32_t n, const uint8_t* frozen_mask, int32_t f_mode, char* src, size_t src_len,
                 size_t* src_size, char* name, size_t name_len);

/* 5G NR data path (polar_amd/polar5g.py builds the tables on the host, 3GPP TS 38.212 5.4.1).
 * All pointers are device pointers; rows are contiguous fp32.
 * pl_crc_attach:   out[b] = [u[b], parity(u[b])], parity bit c = XOR of g_rows[m] bit c over the
 *                  1 bits m of u[b] (g_rows: k generator rows, bit c = parity column c; degree <= 32).
 * pl_crc_check:    valid[b] = 1 iff the parity of the whole received word[b] (len bits, g_rows: len
 *                  generator rows) is all zero, i.e. its last degree bits are the CRC of the first
 *                  len - degree bits; else 0.
 * pl_gather_rows:  out[b, j] = in[b, idx[j]], j < n_out <= 4096 (rate matching).
 * pl_rate_recover: out[b, j] = src_a[j] < 0 ? fill[j] : in[b, src_a[j]] (+ in[b, src_b[j]] if
 *                  src_b (nullable) has src_b[j] >= 0), j < n <= 2048 (de-interleaving, puncturing
 *                  = fill 0, shortening = fill -llr_max, repetition = the sum, sub-block
 *                  de-interleaving folded into one table). */
int pl_crc_attach(const float* u, int64_t bs, int32_t k, const uint32_t* g_rows, int32_t degree, float* out,
                  void* hip_stream);
int pl_crc_check(const float* word, int64_t bs, int32_t len, const uint32_t* g_rows, int32_t degree,
                 uint8_t* valid, void* hip_stream);
int pl_gather_rows(const float* in, int64_t bs, int32_t n_in, const int32_t* idx, int32_t n_out, float* out,
                   void* hip_stream);
int pl_rate_recover(const float* llr, int64_t bs, int32_t e, const int32_t* src_a, const int32_t* src_b,
                    const float* fill, int32_t n, float* out, void* hip_stream);

/* Monte-Carlo caller side, fused (polar_amd.channel.FusedAWGN, polar_amd.sim):
 * pl_awgn_qpsk_llr: System_AWGN_model.forward up to the decoder call (x_run_sn_polar/z_sys_model/
 *                  awgn_model.py:33-41) for rows row0 .. row0+bs-1 of a random stream: information bits
 *                  (BinarySource, my_sn/trans/binary_source.py:18-19; Philox4x32-10 keyed by seed,
 *                  counter (row, iteration)), codeword x = u G_n with the plan's frozen set
 *                  (x_run enc.py:30-43), Gray QPSK (mapping.py:136-149), AWGN of variance no
 *                  (awgn.py:19-29), logits log P(b=1)/P(b=0) (mapping.py:225-241).
 *                  u_out (nullable): [bs, k] fp32 0/1; llr_out: [bs, n] fp32.  no > 0.
 *                  Stream keys: row0 + row is the 64-bit counter row (words 0-1); iteration is
 *                  one 32-bit counter word, so 0 <= iteration < 2^32 (PL_EINVAL otherwise).
 *                  polar_amd.channel.FusedAWGN keys a draw by (SNR point, iteration) with the
 *                  point in the row's high word: row0 + (point << 32), iteration.
 * pl_count_errors: count_errors + count_block_errors (my_sn/sim.py:7-18) of two [rows, k] fp32 0/1
 *                  tensors: counts[0] += differing elements, counts[1] += rows with a difference
 *                  (int64 device counters, accumulated).
 * pl_awgn_qpsk_llr_bits: pl_awgn_qpsk_llr with the information bits packed instead of fp32:
 *                  ubits_out (nullable) [bs, ceil(k/32)] uint32, bit m % 32 of word m / 32 = bit m
 *                  (bits past k zero).  Same stream, same logits.
 * pl_sc_decode_count: SC decode (as pl_sc_decode) fused with the harness's error count: instead of
 *                  writing the decided bits, compares them with ref_bits (packed as above) and
 *                  accumulates counts[0] += bit errors, counts[1] += block errors (int64 device
 *                  counters) -- pl_sc_decode + pl_count_errors in one pass (sim.py:84-100).
 *                  workspace: pl_sc_count_workspace_size(plan, bs) bytes of device scratch.
 *                  PL_ENOTSUP for plans on the generic SC kernel (pl_plan_kernel: 0).
 * pl_sc_sim_count: one whole Monte-Carlo iteration of the harness (System_AWGN_model.forward,
 *                  awgn_model.py:33-44, then sim.py:84-100's counters) in the SC kernel itself:
 *                  information bits, polar encoding, QPSK, AWGN and logits are generated in the
 *                  decoder's lane layout (Philox4x32-10 keyed by seed, counter (row0 + row,
 *                  iteration, stream word); streams distinct from pl_awgn_qpsk_llr's), decoded, and
 *                  compared in registers: counts[0] += bit errors, counts[1] += block errors.  No
 *                  LLR or bit row is written unless llr_dump ([bs, n] fp32 logits) / u_dump ([bs, k]
 *                  fp32 information bits) are given (nullable; for tests).  workspace as
 *                  pl_sc_decode_count.  PL_ENOTSUP unless the plan's specialised kernel has 64
 *                  channel slots per lane (min-sum n = 64 ... 1024; pl_plan_kernel: 1).
 *                  0 <= iteration < 2^32, as pl_awgn_qpsk_llr. */
int pl_awgn_qpsk_llr(const pl_plan* plan, uint64_t seed, uint64_t iteration, int64_t row0, int64_t bs, float no,
                     float* u_out, float* llr_out, void* hip_stream);
int pl_awgn_qpsk_llr_bits(const pl_plan* plan, uint64_t seed, uint64_t iteration, int64_t row0, int64_t bs,
                          float no, uint32_t* ubits_out, float* llr_out, void* hip_stream);
int pl_count_errors(const float* a, const float* b, int64_t rows, int32_t k, int64_t* counts, void* hip_stream);
size_t pl_sc_count_workspace_size(const pl_plan* plan, int64_t bs);
int pl_sc_decode_count(const pl_plan* plan, const float* llr_logits, int64_t bs, const uint32_t* ref_bits,
                       int64_t* counts, void* workspace, size_t ws_bytes, void* hip_stream);
int pl_sc_sim_count(const pl_plan* plan, uint64_t seed, uint64_t iteration, int64_t row0, int64_t bs, float no,
                    int64_t* counts, void* workspace, size_t ws_bytes, float* llr_dump, float* u_dump,
                    void* hip_stream);

/* pl_clock_probe: diagnostics, not on the reference's path.  One wave runs iters dependent VALU adds
 * and writes ticks[0] = s_memtime cycles (shader clock), ticks[1] = s_memrealtime ticks (100 MHz)
 * and ticks[2] (the chain's result) to the DEVICE buffer ticks[3]; clock GHz = 0.1 * ticks[0] /
 * ticks[1].  bench.py reads the clock around its timed region with it (DVFS moves the MI355X clock
 * with load and from box to box). */
int pl_clock_probe(uint64_t* ticks, int32_t iters, void* hip_stream);

const char* pl_last_error_string(void);
/* "polar_mi355x <version> (gfx950) src <16 hex digits>": the FNV-1a hash of the sources the library was
 * built from (polar_amd/build.py source_hash()). */
const char* pl_version(void);

#ifdef __cplusplus
}
#endif
#endif /* POLAR_MI355X_H */
