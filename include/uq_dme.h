/* uq_dme.h — C-ABI of the MI355X-native unbiased L1-ball type quantizer.
 *
 * The reference (Ritesh622/Unbiased-Quantization-Distributed-Mean-Estimation) is pure
 * Python/PyTorch and has no FFI; every entry point below replaces one group of torch
 * ops inside `Type_unbiased_quantize` (NMSE_Results/Codes/All_Schemes.py:609-641) or
 * the DME client-mean around it (NMSE_Results/Codes/Normal_dist.py:137-138).  The
 * Python binding that calls these through ctypes is the drop-in; INTEGRATION.md shows
 * the binding a maintainer of the reference would add.
 *
 * Conventions
 *   - All buffers are DEVICE pointers, caller-allocated, row-major [n][d] f32 for
 *     client vectors.  `stream` is a hipStream_t passed as void* (NULL = default stream).
 *   - The library never allocates, never synchronises, and is stream-ordered.
 *   - Return 0 on success, a negative UQ_E* code on error; uq_last_error() gives a
 *     thread-local message.  Launch errors are reported; kernel-side protocol
 *     timeouts are reported by uq_check_status() after the stream is synchronised.
 *   - No hidden RNG: the per-client uniform X of AS:634 is an input.
 *   - m (lattice sum, AS:622-623) is passed explicitly; uq_rate_to_m() reproduces the
 *     reference's rate table for callers that want it.
 *   - torch_threads selects the f32 summation order of torch CPU `sum` (AS:624) for a
 *     given intra-op thread count, so results are bit-identical to the CPU reference
 *     run with that many threads.
 */
#ifndef UQ_DME_H
#define UQ_DME_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define UQ_OK 0
#define UQ_E_INVALID (-1)   /* bad argument */
#define UQ_E_HIP (-2)       /* HIP runtime error */
#define UQ_E_WORKSPACE (-3) /* workspace too small */
#define UQ_E_TIMEOUT (-4)   /* inter-workgroup protocol timed out (see uq_check_status) */

/* Library ABI version (major*100 + minor). */
int uq_version(void);
/* SHA-256 (hex) of the sources and flags the library was built from (build_ext.build_id()). */
const char* uq_build_id(void);
/* Test hook, process-wide: on != 0 makes every later torch-tie replay (biased quantizer,
 * UQ_TIES_TORCH) take its failure path, so the defined fallback (lowest-index order plus the
 * internal-error status) can be tested.  Returns the previous setting.  Never set by the
 * library; production callers leave it at 0. */
int uq_test_force_replay_failure(int on);
/* Test hooks of the QUIC-FL kernels, process-wide (never set by the library): bit 0 makes the
 * runs of the few-message team kernels (sender KQ1t, receiver KQ2t) skip their waits and report
 * UQ_QFL_TIMEOUT, so the callers' timeout handling can be tested (the sender then takes KQ1t);
 * bit 1 sends every call to the one-wave-per-message kernels (KQ1 / KQ2); bit 2 sends the
 * sender's few-message calls to the team kernel KQ1t instead of the jump path (KQ0j + KQ1j), so
 * the forms can be compared on the same message.  Returns the previous flags. */
int uq_test_set_quicfl_hooks(int flags);
/* Host-only, for tests and tools: the MT19937 state (ATen's 624-word array, block-aligned) that
 * `blocks` twists ahead of state624, computed the way the QUIC-FL sender's jump path does it
 * (t^(624 (blocks - 1)) mod phi, phi from Berlekamp-Massey; the correlation with the stream's
 * first 19937 + 623 words; one twist) -- see uq_mt_poly.cpp.  Replaces nothing in the
 * reference: its generators (All_Schemes.py:457, 465, 484, 489) are walked word by word. */
int uq_mt_jump_host(const uint32_t* state624, int64_t blocks, uint32_t* out624);

/* Host-only: the NMSE drivers' input vectors, bit-identical to numpy's legacy RandomState and
 * multi-threaded (uq_legacy_rng.cpp).  Replaces the per-vector draws of
 * NMSE_Results/Codes/Normal_dist.py:88-91 (np.random.normal(0, 1, size=d)), Laplace_dist.py:89,
 * Gamma_dist.py:86, Bernoulli_dist.py:90 (choice(arange(2), p)) and Lognormal_dist.py:90:
 * n successive size-d calls on the state (key624, pos, has_gauss, gauss) -- numpy's
 * get_state() tuple, advanced in place -- into out [n][d] as f32 (the drivers' cast to a f32
 * tensor), and norm2[i] = np.linalg.norm(v_i) ** 2 summed in f64 in a fixed order.
 * dist / (a, b): 0 normal (loc, scale), 1 laplace (loc, scale), 2 gamma (shape > 1, scale),
 * 3 choice of {0, 1} (the normalised cdf), 4 lognormal (mean, sigma), 5 uniform (low,
 * high - low).  threads: host threads (1 = sequential).  Returns 0, -1 bad arguments, -2 jump
 * unavailable, -3 internal inconsistency.  Does not set uq_last_error. */
int uq_legacy_draw_f32(uint32_t* key624, int32_t* pos, int32_t* has_gauss, double* gauss, int32_t dist,
                       double a, double b, int64_t n, int64_t d, float* out, double* norm2, int32_t threads);
/* Test hook: set the parallel draw's chunking (words per chunk, words of overlap; 0 keeps) and
 * read-and-reset its counters (waves run, chunk meetings missed). */
int uq_legacy_test_params(int64_t min_chunk, int64_t overlap, int64_t* waves, int64_t* misses);

/* Thread-local description of the last error returned on this thread. */
const char* uq_last_error(void);

/* AS:614-623: m = int(table[bits] * d).  Unknown `bits` -> UQ_E_INVALID (the
 * reference raises KeyError). */
int uq_rate_to_m(double bits_per_dimension, int64_t d, int64_t* m_out);

/* Bytes of device workspace needed by the calls below for a batch of n vectors of
 * length d summed in torch order for `torch_threads`.  The workspace also holds the
 * status word read by uq_check_status().  A workspace must be zero-filled once before
 * its first use (later calls re-initialise what they need themselves). */
int uq_workspace_bytes(int64_t n, int64_t d, int32_t torch_threads, size_t* bytes_out);

/* AS:624 — l1_out[j] = sum_i |x[j][i]| in torch CPU cascade order (f32 accumulate). */
int uq_l1_torch_order_f32(const float* x, int64_t n, int64_t d, int32_t torch_threads,
                          float* l1_out, void* ws, size_t ws_bytes, void* stream);

/* AS:609-641 for a batch — out[j] = Type_unbiased_quantize(x[j], ·) with uniform X[j].
 *   m       lattice sum (AS:623)
 *   X       [n] device f32, the AS:634 draw per client
 *   l1      [n] device f32 L1 norms, or NULL to compute them here (torch order)
 *   l1_out  [n] device f32 or NULL: receives the L1 norms used */
int uq_type_unbiased_f32(const float* x, float* out, int64_t n, int64_t d, int64_t m,
                         const float* X, const float* l1, float* l1_out,
                         int32_t torch_threads, void* ws, size_t ws_bytes, void* stream);

/* AS:609-641 for ONE vector per call, the form the reference's callers use (Normal_dist.py:137,
 * Type_unbiased.py:160): out = Type_unbiased_quantize(x, ·) with the AS:634 draw X passed by
 * value (no device copy of it), L1 computed here (torch order).  Same bits as
 * uq_type_unbiased_f32 with n = 1. */
int uq_type_unbiased_vec_f32(const float* x, float* out, int64_t d, int64_t m, float X, int32_t torch_threads,
                             void* ws, size_t ws_bytes, void* stream);

/* Normal_dist.py:137-138 — est[i] (+)= q[j][i] / n_div for j = 0..n-1 in client order
 * (f32 IEEE division, f32 add).  Row j starts at q + j*ld (ld >= d, so a column block
 * of a wider batch can be folded in).  accumulate=0 starts from zeros; accumulate=1
 * continues from `est`, which makes the sum over a sequence of calls bit-identical
 * to one call over all rows in the same order. */
int uq_client_mean_f32(const float* q, int64_t n, int64_t d, int64_t ld, float n_div,
                       int32_t accumulate, float* est, void* stream);

/* Quantize a batch and fold it into the client mean in one call:
 *   q = Type_unbiased_quantize(x[j]) for all j (into `out`, which must be non-NULL),
 *   then est (+)= q[j] / n_div in client order.  Bit-identical to the two calls above. */
int uq_type_unbiased_mean_f32(const float* x, float* out, int64_t n, int64_t d, int64_t m,
                              const float* X, const float* l1, int32_t torch_threads,
                              float n_div, int32_t accumulate, float* est,
                              void* ws, size_t ws_bytes, void* stream);

/* Type codes (wire format; see unbiased-quantization-distributed-mean-estimation_amd/codes.py).
 * Per coordinate one int8: k = fl + r (the lattice count, 0..127) for sign(v) >= 0 and
 * -k-1 for sign(v) < 0.  With the client's L1 and m, q is rebuilt bit-for-bit:
 * q = +-RN(RN(L1*k)/f32(m)).  kmax[j] = the client's largest count; 128 means some count
 * exceeded 127 and saturated (overflow: send that client as floats).
 *
 * uq_type_unbiased_codes_f32: as uq_type_unbiased_f32, writing q (out, may be NULL)
 * and/or codes [n][d] int8 (may be NULL; then kmax may be NULL too).  kmax [n] int32 is
 * zeroed by the call. */
int uq_type_unbiased_codes_f32(const float* x, float* out, int8_t* codes, int32_t* kmax,
                               int64_t n, int64_t d, int64_t m, const float* X, const float* l1,
                               float* l1_out, int32_t torch_threads, void* ws, size_t ws_bytes,
                               void* stream);

/* As uq_type_unbiased_codes_f32 with row pitches: q row j at out + j*ldq (floats, ldq >= d),
 * codes row j at codes + j*ldc (bytes, ldc >= d), e.g. rows of wider caller buffers.  Same
 * bits as the dense call; nothing is written between rows. */
int uq_type_unbiased_codes_ld_f32(const float* x, float* out, int64_t ldq, int8_t* codes, int64_t ldc,
                                  int32_t* kmax, int64_t n, int64_t d, int64_t m, const float* X,
                                  const float* l1, float* l1_out, int32_t torch_threads, void* ws,
                                  size_t ws_bytes, void* stream);

/* 4-bit type codes (the bench pipeline "codes4"): as uq_type_unbiased_codes_ld_f32 writing q
 * (required) and the codes as 4-bit fields, two per byte (element 2i in the low nibble of byte
 * i of row j at nib + j*ldn, ldn >= d/2 bytes): the low nibble of the int8 code, i.e. k for
 * sign >= 0 and 15-k for -k-1, exact while k <= 7.  kmax as for the int8 codes (the largest
 * count, 128 above 127); a client with kmax > 7 is read from q by uq_nibbles_q_mean_ld_f32.
 * Stream form only: n >= 256, d % 4096 == 0, d <= 2^29, 16-byte aligned rows (UQ_E_INVALID
 * otherwise).  Internal format between K2 and the mean; no wire format (the UQR1 codec takes
 * the int8 codes). */
int uq_type_unbiased_nibbles_ld_f32(const float* x, float* out, int64_t ldq, uint8_t* nib, int64_t ldn,
                                    int32_t* kmax, int64_t n, int64_t d, int64_t m, const float* X,
                                    const float* l1, float* l1_out, int32_t torch_threads, void* ws,
                                    size_t ws_bytes, void* stream);

/* est[i] (+)= q[j][i] / n_div, clients in order, from the 4-bit codes above: bit-identical to
 * uq_client_mean_f32(q); clients with kmax[j] > 7 add q[j][i] / n_div (q required).
 * d % 4096 == 0, ldq >= d, ldn >= d/2, 16-byte aligned est and q. */
int uq_nibbles_q_mean_ld_f32(const uint8_t* nib, int64_t ldn, const float* q, int64_t ldq, const float* l1,
                             const int32_t* kmax, int64_t n, int64_t d, int64_t m, float n_div,
                             int32_t accumulate, float* est, void* stream);

/* q[j][i] = decode(codes[j][i]; l1[j], m). */
int uq_codes_decode_f32(const int8_t* codes, const float* l1, int64_t n, int64_t d, int64_t m,
                        float* out, void* stream);

/* Normal_dist.py:137-138 from codes: est[i] (+)= q[j][i] / n_div, clients in order,
 * bit-identical to uq_client_mean_f32 on the decoded batch (reads d bytes per client).
 * kmax [n] as produced by the encoder (sizes the per-client decode tables). */
int uq_codes_mean_f32(const int8_t* codes, const float* l1, const int32_t* kmax, int64_t n, int64_t d,
                      int64_t m, float n_div, int32_t accumulate, float* est, void* stream);

/* As uq_codes_mean_f32, with the dequantized batch q (row j at q + j*ldq, ldq >= d) beside
 * the codes: a client whose counts overflowed its codes (kmax[j] > 127, saturated) adds
 * q[j][i] / n_div instead, so est is always bit-identical to uq_client_mean_f32(q).
 * q == NULL is uq_codes_mean_f32 (overflowed clients then add their saturated codes).
 * Clients without overflow read only their codes. */
int uq_codes_q_mean_f32(const int8_t* codes, const float* q, int64_t ldq, const float* l1, const int32_t* kmax,
                        int64_t n, int64_t d, int64_t m, float n_div, int32_t accumulate, float* est,
                        void* stream);

/* As uq_codes_q_mean_f32 with the codes' row pitch: codes row j at codes + j*ldc (ldc >= d). */
int uq_codes_q_mean_ld_f32(const int8_t* codes, int64_t ldc, const float* q, int64_t ldq, const float* l1,
                           const int32_t* kmax, int64_t n, int64_t d, int64_t m, float n_div,
                           int32_t accumulate, float* est, void* stream);

/* ---- type messages "UQR1": entropy-coded type codes ---------------
 * The reference has no wire format (parity unpinned); its client output is AS:640's
 * dequantized vector, fully described by (L1, m, signed counts k) = the int8 codes above.
 * One message per client: rANS over symbols s = 2k + neg with a per-client static model
 * (frequencies quantized to 2^12), 32-bit states, 16-bit words, W = min(64, ceil(d/1024))
 * interleaved states per chunk of W*1024 symbols, so ~R bits per coordinate at rate R.
 * flags bit 0 (UQ_TC_EXACT_ZERO_SIGNS): keep the sign of zero counts (neg for k = 0), so
 * the decoded q is bit-identical to AS:640 (-0.0 included); without it the sign of a zero
 * count is dropped and q is value-identical (+0.0 where the reference has -0.0), at ~R bits.
 * Byte layout: oracle/uq_codec.c (the CPU restatement the tests compare against).
 *
 * uq_tc_bound: the largest message of a client of length d (bytes).
 * uq_tc_encode: codes [n][d] int8, l1 [n] f32 (device) -> messages packed back to back in
 *   msgs (device, msgs_bytes >= n * bound), offsets [n+1] u64 (device): client j's message is
 *   msgs[offsets[j] .. offsets[j+1]).  Workspace: uq_tc_workspace_bytes (no zero-fill needed).
 * uq_tc_decode: messages (device buffer of msgs_bytes, offsets [n+1]) -> codes [n][d], l1 [n],
 *   kmax [n]; status [n] int32 (device) is 0 for a well-formed message, else bit 0 bad header,
 *   d mismatch or offsets outside [0, msgs_bytes] / not increasing / unaligned (nothing is read
 *   outside the buffer), bit 1 bad frequency table, bit 2 word stream overrun or underrun,
 *   bit 3 wrong final state, bit 4 the header's m differs from `m` (m < 0: any m). */
#define UQ_TC_EXACT_ZERO_SIGNS 1
int uq_tc_bound(int64_t d, size_t* bytes_out);
int uq_tc_workspace_bytes(int64_t n, int64_t d, size_t* bytes_out);
int uq_tc_encode(const int8_t* codes, const float* l1, int64_t n, int64_t d, int64_t m, int32_t flags,
                 uint8_t* msgs, size_t msgs_bytes, uint64_t* offsets, void* ws, size_t ws_bytes, void* stream);
int uq_tc_decode(const uint8_t* msgs, size_t msgs_bytes, const uint64_t* offsets, int64_t n, int64_t d, int64_t m,
                 int8_t* codes, float* l1, int32_t* kmax, int32_t* status, void* stream);

/* ---- biased type quantizer (Reznik rounding) ------------------------------------------
 * NMSE_Results/Codes/All_Schemes.py:669-687 Type_biased_quantize and :644-666 Reznik for
 * a batch: out[j] = Type_biased_quantize(x[j], ·) with m = the lattice sum (AS:684).
 *   k' = floor(m p + 0.5), m' = sum k' (torch CPU order for torch_threads), Delta = int(m' - m);
 *   the |Delta| coordinates with the largest delta' = k' - m p (Delta > 0: k' -= 1) or the
 *   smallest (Delta < 0: k' += 1) are adjusted; out = (L1 * sign(x)) * (k' / m).
 * tie_policy decides which of several coordinates with the same delta' at the selection
 * threshold are taken (torch.topk compares values only):
 *   UQ_TIES_TORCH         the coordinates torch CPU's topk returns (libstdc++
 *                         nth_element / partial_sort replayed on the GPU): bit-identical
 *                         to the reference on every input
 *   UQ_TIES_LOWEST_INDEX  the lowest indices (cheaper; identical whenever no tie straddles
 *                         the threshold, i.e. info flag 1 is clear)
 * l1_out [n] f32 or NULL.  info [n][2] int32 or NULL: {Delta, flags}; flags bit0 = a tie
 * straddled the threshold, bit1 = m' not finite (the reference raises; output is NaN-laden),
 * bit2 = |Delta| > d (the reference's topk raises), bit3 = torch tie choice replayed,
 * bit4 = threshold digits 2-3 found on the compacted first-digit bucket (informational).
 * Workspace: uq_biased_workspace_bytes; zero-filled once before first use (it holds the
 * status word of uq_check_status, which reports an inconsistent tie replay).  The tests
 * exercise the replay's index-order fallback through uq_test_force_replay_failure, not
 * through the workspace: no workspace content changes which path a replay takes. */
#define UQ_TIES_TORCH 0
#define UQ_TIES_LOWEST_INDEX 1
/* OR'd into UQ_TIES_TORCH: the call synchronises `stream` once, to read the number of clients
 * whose tie choice needs the replay, and skips the replay's kernels when it is zero -- for
 * synchronous few-client callers (the per-vector drop-in); results are the same bits either
 * way. */
#define UQ_TIES_HOST_CHECK 4
int uq_biased_workspace_bytes(int64_t n, int64_t d, int32_t torch_threads, size_t* bytes_out);
int uq_type_biased_f32(const float* x, float* out, int64_t n, int64_t d, int64_t m,
                       int32_t torch_threads, int32_t tie_policy, float* l1_out, int32_t* info,
                       void* ws, size_t ws_bytes, void* stream);

/* ---- EDEN with the randomized Hadamard transform (baseline) -------
 * NMSE_Results/Codes/All_Schemes.py:95-153 (RHT), :324-413 (EdenSender / EdenReceiver),
 * :792-811 (EDEN_quantize_Hadamard).  D = dim rounded up to a power of two.
 *
 * uq_rht_signs: the RHT diagonal of AS:117-120 for each seed: signs[r][i] = +-1 (int8) as
 *   2 * torch.bernoulli(1/2, generator seeded with seeds[r]) - 1 on torch's CPU generator
 *   (MT19937).  Callers cache rows per (seed, D); seeds is a device int32 [rows].
 * uq_eden_compress_f32: bins [n][D] u8 and scale [n] f32 of EdenSender.compress for integer
 *   nbits (1 or 2, the tables the reference defines); client j uses diagonal row
 *   sign_row[j] (device int32 [n]).  Rotation, norm (torch CPU order) and bins are
 *   bit-identical to the reference; scale's dot product is accumulated in fp64 (the
 *   reference's MKL sdot order is CPU-dependent): scale within 1e-6 relative.
 * uq_eden_decompress_f32: out [n][dim] = scale * RHT^-1(centroids[bins])[:dim].
 * uq_eden_f32: both (EDEN_quantize_Hadamard for a batch); scale_out [n] or NULL.
 * Workspace: uq_eden_workspace_bytes. */
int uq_rht_signs(const int32_t* seeds, int64_t rows, int64_t D, int8_t* signs, void* stream);
/* The randomized Hadamard transform itself, for a batch (workspace: uq_eden_workspace_bytes):
 *   inverse = 0: out [n][D] = H(pad(x[j], D) * diag) (HadamardSender.randomized_hadamard_transform,
 *                AS:123-141); x rows have length dim
 *   inverse = 1: out [n][D] = H(x[j]) * diag (HadamardReceiver, AS:146-153); dim must be D
 * bit-identical to the reference (f32 butterflies a + b, (a + b) - 2b; / f32(sqrt(D))).
 * (It uses only the vector part of that workspace, not the norm's tables, so a smaller
 * buffer passes the size check; uq_eden_workspace_bytes is always enough.) */
int uq_rht_f32(const float* x, float* out, int64_t n, int64_t dim, int32_t inverse, const int8_t* signs,
               const int32_t* sign_row, void* ws, size_t ws_bytes, void* stream);
/* uq_quicfl_prepare_f32: QuicFLReceiver.decompress (AS:526-532) up to its inverse RHT, for a
 * batch: out [n][D] = (exact ? exact_vals : recv_table[X * h_len + h]) / scale[j], with
 * h = torch.randint(0, h_len, (D,)) of a CPU generator seeded with prng_seeds[j] (MT19937
 * word % h_len).  X [n][D] int32 in [0, table_rows); recv_table [table_rows][h_len] f32
 * (<= 1024 entries: the reference tables <b>_X_<s>_h_256_q_recv_table.pt); exact_mask u8 [n][D] and
 * exact_vals f32 [n][D] (dense) or both NULL; scale [n] f32.  The inverse RHT is uq_rht_f32
 * (inverse = 1). */
int uq_quicfl_prepare_f32(const int32_t* X, int64_t n, int64_t D, const float* recv_table, int32_t table_rows,
                          int32_t h_len, const int32_t* prng_seeds, const uint8_t* exact_mask, const float* exact_vals,
                          const float* scale, float* out, void* stream);
/* uq_quicfl_receive_f32: the same for messages as they come (uq_quicfl_compress_f32's or the
 * reference's dict): X [n][D] int64 (x_kind 0), uint8 (1) or int32 (2), read in place; the
 * index X * h_len + h is taken like torch.take (AS:530): -numel <= index < numel, negatives
 * wrap, any other index sets UQ_QFL_BAD_INDEX in info[j] (that coordinate's output is 0; the
 * reference raises IndexError).  exact_mask u8/bool [n][D] or NULL; exact_vals f32 [n][D]
 * dense (exact_layout 0: the value at its coordinate) or compact (exact_layout 1: row j's
 * exact values in index order in its first entries, as uq_quicfl_compress_f32 writes them;
 * exact_vals rows are still D entries long).  exact_count [n] or NULL (compact only): a row
 * whose mask does not hold exactly exact_count[j] coordinates gets UQ_QFL_BAD_EXACT (the
 * reference's `vec[exact_indeces] = exact_values` raises).  info [n] int32 or NULL.
 * D <= 2^28.  uq_quicfl_prepare_f32 = x_kind 2, dense, no info. */
#define UQ_QFL_BAD_EXACT 32
int uq_quicfl_receive_f32(const void* X, int32_t x_kind, int64_t n, int64_t D, const float* recv_table,
                          int32_t table_rows, int32_t h_len, const int32_t* prng_seeds, const uint8_t* exact_mask,
                          const float* exact_vals, int32_t exact_layout, const int32_t* exact_count, const float* scale,
                          float* out, int32_t* info, void* stream);
/* uq_quicfl_receive_ws_f32: uq_quicfl_receive_f32 with a device workspace of
 * uq_quicfl_receive_workspace_bytes(n, D) bytes (0 means none is used; NULL is accepted then):
 * with it, few-message calls start every run of the h stream at once from jumped generator
 * blocks (MT19937 jump-ahead, uq_mt_poly.cpp) instead of walking the stream; same results. */
int uq_quicfl_receive_workspace_bytes(int64_t n, int64_t D, size_t* bytes_out);
int uq_quicfl_receive_ws_f32(const void* X, int32_t x_kind, int64_t n, int64_t D, const float* recv_table,
                             int32_t table_rows, int32_t h_len, const int32_t* prng_seeds, const uint8_t* exact_mask,
                             const float* exact_vals, int32_t exact_layout, const int32_t* exact_count,
                             const float* scale, float* out, int32_t* info, void* ws, size_t ws_bytes, void* stream);

/* ---- QUIC-FL sender (baseline) --------------------------------------
 * QuicFLSender.compress (NMSE_Results/Codes/All_Schemes.py:455-503) for a batch of n messages,
 * bit-identical to the reference's CPU run (tests/golden/quicfl_sender_vectors.*):
 *   rotation: the sender RHT of uq_rht_f32 (diagonal row sign_row[j] of signs [rows][D]);
 *   scale[j] = f32(1 / torch.norm(rot)) * f32(sqrt(D))       (AS:466/470, Tensor.__rtruediv__)
 *   v = rot * scale; exact = |v| > f32(norm.ppf(1 - 2^-9));   (AS:472-478)
 *   q = v / delta (0 where exact); p = q - floor(q);           (AS:480-483)
 *   h = randint(0, h_len, (D,)) and bernoulli(p) from MT19937 seeded with prng_seeds[j]
 *       (= xxh64(str(seed)) % 2^16, uq_xxh64), the D randint words first;
 *   idx = ((floor(q) + b) * h_len + h) + half_table in f32, truncated (torch.take wraps
 *       negatives), half_table = ((table_numel / h_len) - 1) * h_len / 2   (AS:443, AS:486);
 *   X = table[idx].X + bernoulli(table[idx].p) from a second generator, truncated (AS:489-490).
 * table_xp: device f32 [table_numel][2] = (sender_table_X, sender_table_p) pairs; table_packed
 *   (or NULL): the same table as u32 (X << 25) | ceil(p * 2^24), valid when every X is an integer
 *   in 0..127 and every p in [0, 1] (the caller checks): one 4-byte gather per coordinate instead
 *   of 8 -- bernoulli(p) draws low24(w) * 2^-24 < p, i.e. low24(w) < ceil(p * 2^24), the same bits.
 * The second generator (the reference's global torch generator): px_state [n][626] u32 =
 *   (left, next, state[624]) of ATen's mt19937 per message (next = 625 - left unless left = 1),
 *   or px_state = NULL and px_seeds [n] (fresh generators, manual_seed(px_seeds[j]));
 *   px_state_out [n][626] (or NULL) receives the state after the message's D draws.
 * Outputs: X [n][D] int64 (x_kind 0, the reference's X.long()) or uint8 (x_kind 1; values
 *   outside 0..255 flag UQ_QFL_X_RANGE); exact_mask [n][D] u8; exact_vals [n][D] f32 with
 *   message j's exact values compacted in index order in its first exact_count[j] entries;
 *   scale [n] f32; info [n] int32 flags: UQ_QFL_BAD_P (some p outside [0, 1]: the reference's
 *   bernoulli raises RuntimeError, e.g. an all-zero vector), UQ_QFL_BAD_INDEX (an index outside
 *   [-numel, numel): torch.take raises IndexError), UQ_QFL_BAD_PX (a table p outside [0, 1]),
 *   UQ_QFL_X_RANGE.  h_len must be 1..256; workspace: uq_quicfl_workspace_bytes. */
#define UQ_QFL_BAD_P 1
#define UQ_QFL_BAD_INDEX 2
#define UQ_QFL_BAD_PX 4
#define UQ_QFL_X_RANGE 8
#define UQ_QFL_TIMEOUT 16   /* internal: a wait of the few-message kernel ran out (never expected) */
#define UQ_QFL_STATE_WORDS 626
int uq_quicfl_workspace_bytes(int64_t n, int64_t dim, size_t* bytes_out);
int uq_quicfl_compress_f32(const float* x, int64_t n, int64_t dim, const int8_t* signs, const int32_t* sign_row,
                           const float* table_xp, const uint32_t* table_packed, int64_t table_numel, int32_t h_len,
                           float delta,
                           const int32_t* prng_seeds, const uint32_t* px_state, const int32_t* px_seeds,
                           uint32_t* px_state_out, void* X, int32_t x_kind, uint8_t* exact_mask, float* exact_vals,
                           int32_t* exact_count, float* scale, int32_t* info, void* ws, size_t ws_bytes, void* stream);
/* uq_quicfl_quantize_f32: QUICFL_quantize (All_Schemes.py:814-832) for a batch: the sender of
 * uq_quicfl_compress_f32 (same arguments, same generators, px_state_out likewise) with the
 * receiver QuicFLReceiver.decompress (AS:526-535) on each message fused into it: out[j][:dim]
 * = inverse RHT of (exact ? v : recv_table[X * h_len + h]) / scale, where h is the sender's
 * own randint stream (the receiver regenerates the same words from the same prng seed).  No
 * message is written.  recv_table: device f32 [recv_numel] (<= 1024; torch.take's flat index
 * range, negatives wrap, others flag UQ_QFL_RECV_INDEX: the reference's receiver raises
 * IndexError after its sender returned).  scale [n] (or NULL) = the messages' scales.  info as
 * uq_quicfl_compress_f32 plus UQ_QFL_RECV_INDEX.  Workspace: uq_quicfl_workspace_bytes. */
#define UQ_QFL_RECV_INDEX 64
int uq_quicfl_quantize_f32(const float* x, int64_t n, int64_t dim, const int8_t* signs, const int32_t* sign_row,
                           const float* table_xp, const uint32_t* table_packed, int64_t table_numel, int32_t h_len,
                           float delta, const float* recv_table, int32_t recv_numel, const int32_t* prng_seeds,
                           const uint32_t* px_state, const int32_t* px_seeds, uint32_t* px_state_out, float* out,
                           float* scale, int32_t* info, void* ws, size_t ws_bytes, void* stream);
/* xxHash64 of `len` bytes (AS:457 hashes str(seed) with seed 0); host-only, no GPU. */
uint64_t uq_xxh64(const void* data, size_t len, uint64_t seed);
int uq_eden_workspace_bytes(int64_t n, int64_t dim, size_t* bytes_out);
int uq_eden_compress_f32(const float* x, int64_t n, int64_t dim, int32_t nbits, const int8_t* signs,
                         const int32_t* sign_row, uint8_t* bins, float* scale, void* ws, size_t ws_bytes,
                         void* stream);
int uq_eden_decompress_f32(const uint8_t* bins, const float* scale, int64_t n, int64_t dim, int32_t nbits,
                           const int8_t* signs, const int32_t* sign_row, float* out, void* ws, size_t ws_bytes,
                           void* stream);
int uq_eden_f32(const float* x, float* out, int64_t n, int64_t dim, int32_t nbits, const int8_t* signs,
                const int32_t* sign_row, float* scale_out, void* ws, size_t ws_bytes, void* stream);
/* The same three with the diagonal rows also as bits: sign_bits [rows][ceil(D / 32)] u32, bit
 * i % 32 of word i / 32 set where signs[row][i] is -1 (uq_rht_sign_bits makes them from the
 * int8 rows); the passes that apply the diagonal (the sender's first, the receiver's last) read
 * 1/8 byte per coordinate instead of 1.  sign_bits NULL: the int8 rows, as above.  Same results. */
int uq_rht_sign_bits(const int8_t* signs, int64_t rows, int64_t D, uint32_t* bits, void* stream);
int uq_eden_compress_f32_sb(const float* x, int64_t n, int64_t dim, int32_t nbits, const int8_t* signs,
                            const int32_t* sign_row, const uint32_t* sign_bits, uint8_t* bins, float* scale, void* ws,
                            size_t ws_bytes, void* stream);
int uq_eden_decompress_f32_sb(const uint8_t* bins, const float* scale, int64_t n, int64_t dim, int32_t nbits,
                              const int8_t* signs, const int32_t* sign_row, const uint32_t* sign_bits, float* out,
                              void* ws, size_t ws_bytes, void* stream);
int uq_eden_f32_sb(const float* x, float* out, int64_t n, int64_t dim, int32_t nbits, const int8_t* signs,
                   const int32_t* sign_row, const uint32_t* sign_bits, float* scale_out, void* ws, size_t ws_bytes,
                   void* stream);
/* torch.norm(v[j], 2) of each row of v [n][D] f32 in torch's CPU order (AS:329: 8 lanes of
 * fma chains, lanes added in order, sqrt), the norm the EDEN entry points use:
 *   mode 1: the sequential chains (one chain per torch lane; what batches above 256 rows use)
 *   mode 2: the segmented chains (1 <= n <= 256, D a power of two >= 16384; workspace
 *           uq_eden_norm_workspace_bytes): the same bits, the chains cut into segments that
 *           are resolved in parallel (include/../DESIGN.md §4, EDEN)
 *   mode 0: mode 2 where it applies, else mode 1 (the choice the EDEN entry points make).
 * nrm [n] f32. */
int uq_eden_norm_workspace_bytes(int64_t n, int64_t D, size_t* bytes_out);
int uq_eden_norm_f32(const float* v, int64_t n, int64_t D, int32_t mode, float* nrm, void* ws, size_t ws_bytes,
                     void* stream);

/* After the stream has been synchronised: UQ_OK, or UQ_E_TIMEOUT if any
 * inter-workgroup wait in a previous call on this workspace gave up. Clears it. */
int uq_check_status(void* ws, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* UQ_DME_H */
