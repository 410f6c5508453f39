/* encx.h -- C ABI of libencx.so, the MI355X (gfx950) hot path of EnCodec training.
 *
 * Drop-in boundary. The reference (Madhudorai/encodec-pytorch) has no FFI: its hot path sits
 * behind PyTorch nn.Module.forward methods and ATen kernels. Each entry point
 * below replaces the device work of one such reference interface, cited as file:line.
 *
 * Conventions:
 *  - plain device pointers (fp32 unless noted), int64 sizes, contiguous row-major tensors;
 *  - the CALLER owns all memory (PyTorch's caching allocator); workspaces are caller-provided
 *    after a *_workspace query; the library never allocates or frees;
 *  - every call is stream-ordered on the given hipStream_t (pass torch's current stream) and
 *    never synchronises, so a caller may capture it into a hipGraph;
 *  - return 0 on success, a hipError_t value, or ENCX_EINVAL for a shape/argument error;
 *    encx_strerror() turns a code into text. No exceptions cross the ABI;
 *  - deterministic: no floating-point atomics; split reductions are summed in a fixed order.
 */
#ifndef ENCX_H
#define ENCX_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ihipStream_t* encx_stream_t; /* == hipStream_t */

#define ENCX_OK 0
#define ENCX_EINVAL 9001

#define ENCX_PAD_ZERO 0
#define ENCX_PAD_REFLECT 1
#define ENCX_ACT_NONE 0
#define ENCX_ACT_ELU 1

/* ---------------------------------------------------------------- library */
int encx_version(void);
/* Hash of the sources this library was built from (encodec-pytorch_amd/buildid.py); the
 * Python binding refuses a library whose hash differs from the sources beside it. */
const char* encx_build_id(void);
const char* encx_strerror(int code);
/* Kernel-selection options (A/B switches and variants of the hot kernels). Each starts from its
 * environment variable ENCX_<name> or its default, and every launch reads the current value, so
 * tests flip them in-process. Process-wide. Set them before querying workspaces: a workspace size
 * and the launch using it must see the same options. Names with or without the ENCX_ prefix. */
int encx_option_count(void);
const char* encx_option_name(int i);  /* NULL past the last */
int encx_get_option(const char* name, int64_t* value);
int encx_set_option(const char* name, int64_t value, int64_t* previous /* may be NULL */);
/* Select the device; cheap, idempotent. */
int encx_init(int device);
/* Kernel timing for bench.py's roofline: while enabled, every launch of the named kernel
 * family is bracketed by hipEvents on its own stream together with its algorithmic FLOPs and
 * bytes. family: 0 = all conv/GEMM MFMA kernels. */
int encx_prof_enable(int on);
/* 1 while profiling is on (the HIP-graph trainer steps eagerly then: events are not captured) */
int encx_prof_enabled(void);
int encx_prof_read(double* total_ms, double* total_flops, double* total_bytes, int64_t* launches);
/* One recorded launch group: event time, algorithmic FLOPs / bytes and its label
 * ("<op> <shape>"), for per-layer tables (tools/layer_table.py). */
int encx_prof_slot(int64_t i, double* ms, double* flops, double* bytes, const char** tag);

/* ---------------------------------------------------------------- weight norm
 * torch.nn.utils.weight_norm(dim=0) installed by modules/conv.py:25-34 (apply_parametrization_norm):
 * w = v * (g / ||v||_row). v is [A0][A1][K] (Conv1d: [Cout][Cin][K]; ConvTranspose1d: [Cin][Cout][K]).
 * Writes the GEMM operand layouts the conv kernels read:
 *   wf [A1][K][A0]            (conv forward / conv-transpose backward-data)
 *   wp [A0][J][A1*s + r] = w[a0][a1][r + s*j], J = ceil(K/s)   (polyphase transposed kernels)
 * Either output may be NULL. `g` may be NULL for an un-normalised weight (w = v). */
int encx_weightnorm_fwd(const float* v, const float* g, float* wf, float* wp, int64_t A0,
                        int64_t A1, int64_t K, int64_t stride, encx_stream_t stream);
/* Backward of w = v*(g/||v||): dg = (dw.v)/||v||, dv = (g/||v||)(dw - (dw.v/||v||^2) v).
 * rows = A0, cols = A1*K. accumulate: 0 overwrite, 1 add into dv/dg. */
int encx_weightnorm_bwd(const float* v, const float* g, const float* dw, float* dv, float* dg,
                        int64_t rows, int64_t cols, int accumulate, encx_stream_t stream);
/* Batched forms: every weight-normed layer of a model in ONE launch (one workgroup per row
 * over all layers; same arithmetic per row as the single-layer calls, so bit-identical). The
 * descriptor arrays live in device memory (caller-owned, built once per model: the pointers
 * are the persistent parameter / operand buffers); row0 = first row of the layer in the
 * concatenation (ascending), rows_total = sum of the layers' rows. */
typedef struct {
    const float* v; const float* g; float* wf; float* wp;
    int64_t A0, A1, K, stride, row0;
} encx_wn_fwd_desc;
typedef struct {
    const float* v; const float* g; const float* dw; float* dv; float* dg;
    int64_t rows, cols, row0, accumulate;
} encx_wn_bwd_desc;
int encx_weightnorm_fwd_batch(const encx_wn_fwd_desc* layers, int64_t n_layers, int64_t rows_total,
                              encx_stream_t stream);
int encx_weightnorm_bwd_batch(const encx_wn_bwd_desc* layers, int64_t n_layers, int64_t rows_total,
                              encx_stream_t stream);

/* ---------------------------------------------------------------- Conv1d
 * SConv1d.forward (modules/conv.py:195-210): pad1d (:79-96, reflect or zero, `short_ext` =
 * the zero extension of a too-short reflect input, :86-91), then Conv1d (NormConv1d :119-122).
 * y[b,co,t] = bias[co] + sum_{ci,k} W[co,ci,k] act(xpad[b,ci,t*s+k*d]) (+ residual[b,co,t]).
 * pre_act = ENCX_ACT_ELU fuses the nn.ELU that precedes the conv in the SEANet stacks
 * (modules/seanet.py:49,124,136,204,223). residual may alias y (SEANetResnetBlock sum, :63).
 * ws: encx_conv1d_fwd_workspace bytes (split-K partials of low-rate layers; may be 0). */
size_t encx_conv1d_fwd_workspace(int64_t B, int64_t Cin, int64_t Cout, int64_t Tout, int64_t K,
                                 int64_t stride, int64_t dilation);
int encx_conv1d_fwd(const float* x, const float* wf, const float* bias, const float* residual,
                    float* y, float* ws, int64_t B, int64_t Cin, int64_t Tin, int64_t Cout,
                    int64_t Tout, int64_t K, int64_t stride, int64_t dilation, int64_t pad_left,
                    int64_t short_ext, int pad_mode, int pre_act, encx_stream_t stream);
/* d loss / d x of the above (with the pad folded back and the act' applied):
 * dx = [accumulate ? dx : 0] + act'(x) * fold(W^T * dy). `x` is the pre-activation input
 * (read only when pre_act != NONE). ws: encx_conv1d_bwd_data_workspace bytes. */
size_t encx_conv1d_bwd_data_workspace(int64_t B, int64_t Cin, int64_t Tin, int64_t Cout,
                                      int64_t Tout, int64_t K, int64_t stride, int64_t pad_left,
                                      int64_t pad_right);
int encx_conv1d_bwd_data(const float* dy, const float* wp, const float* x, float* dx, float* ws,
                         int64_t B, int64_t Cin, int64_t Tin, int64_t Cout, int64_t Tout,
                         int64_t K, int64_t stride, int64_t pad_left, int64_t pad_right,
                         int64_t short_ext, int pad_mode, int pre_act, int accumulate,
                         encx_stream_t stream);
/* Backward-data of a DILATED Conv1d (nn.Conv1d with dilation > 1 inside SConv1d,
 * modules/conv.py:195-210; SEANetResnetBlock dilates its k3 conv when n_residual_layers > 1,
 * modules/seanet.py:114-117): as encx_conv1d_bwd_data, but from the FORWARD weight layout wf
 * [Cin][K][Cout] (encx_weightnorm_fwd's wf) with any stride and dilation. ws: B*Cin*(pad_left +
 * pad_right) floats when pad_mode is reflect (the pad positions' grads before the fold), else
 * may be NULL. */
int encx_conv1d_bwd_data_dilated(const float* dy, const float* wf, const float* x, float* dx, float* ws,
                                 int64_t B, int64_t Cin, int64_t Tin, int64_t Cout, int64_t Tout,
                                 int64_t K, int64_t stride, int64_t dilation, int64_t pad_left,
                                 int64_t pad_right, int64_t short_ext, int pad_mode, int pre_act,
                                 int accumulate, encx_stream_t stream);
/* dW[co,ci,k] = sum_{b,t} dy[b,co,t] act(xpad[b,ci,t*s+k*d]); db[co] = sum dy (db may be NULL).
 * dw is [Cout][Cin][K]; accumulate as above. ws: encx_conv1d_bwd_weight_workspace bytes. */
int encx_conv1d_bwd_weight(const float* dy, const float* x, float* dw, float* db, float* ws,
                           int64_t B, int64_t Cin, int64_t Tin, int64_t Cout, int64_t Tout,
                           int64_t K, int64_t stride, int64_t dilation, int64_t pad_left,
                           int64_t short_ext, int pad_mode, int pre_act, int accumulate,
                           encx_stream_t stream);
/* encx_conv1d_bwd_weight with separate accumulate flags for dw and db; the bias grad (sum of dy
 * over b, t) is the GEMM's ones column, summed from the staged dy tile in the same kernel (no
 * separate channel-sum pass; falls back to one for the tiny VALU shapes). */
int encx_conv1d_bwd_weight_bias(const float* dy, const float* x, float* dw, float* db, float* ws, int64_t B,
                                int64_t Cin, int64_t Tin, int64_t Cout, int64_t Tout, int64_t K, int64_t stride,
                                int64_t dilation, int64_t pad_left, int64_t short_ext, int pad_mode, int pre_act,
                                int acc_w, int acc_b, encx_stream_t stream);
size_t encx_conv1d_bwd_weight_workspace(int64_t B, int64_t Cin, int64_t Cout, int64_t Tout,
                                        int64_t K);

/* ---------------------------------------------------------------- ConvTranspose1d
 * SConvTranspose1d.forward (modules/conv.py:230-252): ConvTranspose1d then unpad1d (:99-105).
 * y[b,co,j] = bias[co] + sum_{ci,t,k: t*s+k = j+trim_left} Wt[ci,co,k] act(x[b,ci,t]),
 * j in [0,Tout). Polyphase: for each output phase r = (j+trim_left) mod s only the taps
 * k = r + s*q contribute, so the work is a dense GEMM over (co,r) x (b,u) x (ci,q).
 * ws: encx_convtr1d_fwd_workspace bytes. */
size_t encx_convtr1d_fwd_workspace(int64_t B, int64_t Cin, int64_t Cout, int64_t Tout, int64_t K,
                                   int64_t stride, int64_t trim_left);
int encx_convtr1d_fwd(const float* x, const float* wp, const float* bias, float* y, float* ws,
                      int64_t B, int64_t Cin, int64_t Tin, int64_t Cout, int64_t Tout, int64_t K,
                      int64_t stride, int64_t trim_left, int pre_act, encx_stream_t stream);
/* dx = [accumulate ? dx : 0] + act'(x) * sum_{co,k} Wt[ci,co,k] dy[co, t*s+k-trim_left]. */
size_t encx_convtr1d_bwd_data_workspace(int64_t B, int64_t Cin, int64_t Tin, int64_t Cout,
                                        int64_t K, int64_t stride);
int encx_convtr1d_bwd_data(const float* dy, const float* wf, const float* x, float* dx, float* ws,
                           int64_t B, int64_t Cin, int64_t Tin, int64_t Cout, int64_t Tout,
                           int64_t K, int64_t stride, int64_t trim_left, int pre_act,
                           int accumulate, encx_stream_t stream);
/* dWt[ci,co,k] = sum_{b,t} act(x[b,ci,t]) dy[b,co,t*s+k-trim_left]; db[co] = sum dy. */
int encx_convtr1d_bwd_weight(const float* x, const float* dy, float* dw, float* db, float* ws,
                             int64_t B, int64_t Cin, int64_t Tin, int64_t Cout, int64_t Tout,
                             int64_t K, int64_t stride, int64_t trim_left, int pre_act,
                             int accumulate, encx_stream_t stream);
size_t encx_convtr1d_bwd_weight_workspace(int64_t B, int64_t Cin, int64_t Cout, int64_t Tin,
                                          int64_t K);

/* ---------------------------------------------------------------- fused residual block
 * SEANetResnetBlock.forward (modules/seanet.py:21-63) with the EnCodec defaults (kernel_sizes
 * [3, 1], dilations [1, 1], compress 2, true_skip False -> 1x1 shortcut; causal SConv1d with
 * reflect padding, conv.py:195-210) as ONE kernel per direction for the high-rate stages:
 *   h = b1 + W1 * ELU(pad_reflect(x, 2, 0))   (k3, C -> C/2),   y = bs + Ws x + b2 + W2 ELU(h).
 * C in {32, 64}; T >= 3. Weights in the forward layout of encx_weightnorm_fwd (wf [Cin][K][Cout]):
 * w1 [C][3][C/2], w2 [C/2][C], ws [C][C]. h [B][C/2][T] (pre-ELU) is written for the backward; NULL skips it (inference). */
int encx_resblock_fwd(const float* x, const float* w1, const float* b1, const float* w2, const float* b2,
                      const float* ws, const float* bs, float* h, float* y, int64_t B, int64_t C, int64_t T,
                      encx_stream_t stream);
/* Backward of the above: dx = Ws^T dy + ELU'(x) * fold(W1^T * (ELU'(h) * W2^T dy)) (written, not
 * accumulated) and the weight grads in the natural layouts dw1 [C/2][C][3], dw2 [C][C/2][1],
 * dws [C][C][1] (+= when acc_w), db1 [C/2], db2 = dbs = sum dy (+= when acc_b); any grad pointer
 * may be NULL. ws: encx_resblock_bwd_workspace bytes (per-workgroup partials, summed in a
 * fixed order). */
size_t encx_resblock_bwd_workspace(int64_t B, int64_t C, int64_t T);
int encx_resblock_bwd(const float* dy, const float* x, const float* h, const float* w1, const float* w2,
                      const float* ws, float* dx, float* dw1, float* db1, float* dw2, float* db2, float* dws,
                      float* dbs, int acc_w, int acc_b, float* wsp, int64_t B, int64_t C, int64_t T,
                      encx_stream_t stream);

/* ---------------------------------------------------------------- elementwise / reductions */
/* db[c] = [acc ? db : 0] + sum_{b,t} dy[b,c,t] (the bias grads of every conv); ws: workspace
 * of encx_channel_sum_workspace(C) bytes. */
size_t encx_channel_sum_workspace(int64_t C);
int encx_channel_sum(const float* dy, float* db, float* ws, int64_t B, int64_t C, int64_t T,
                     int accumulate, encx_stream_t stream);
/* EncodecModel._encode_frame normalisation (model.py:152-157): scale[b] = 1e-8 +
 * sqrt(mean_t (mean_c x)^2); xn = x / scale. */
int encx_normalize_fwd(const float* x, float* xn, float* scale, int64_t B, int64_t C, int64_t T,
                       encx_stream_t stream);
/* y[b,c,t] = x[b,c,t] * scale[b] (model.py:191-192 out * scale; also its backward) */
int encx_scale_rows(const float* x, const float* scale, float* y, int64_t B, int64_t CT,
                    encx_stream_t stream);
/* y = alpha * x (+ beta * y); alpha read from device scalar alpha_dev when non-NULL */
int encx_axpby(const float* x, float* y, int64_t n, float alpha, const float* alpha_dev,
               float beta, encx_stream_t stream);
/* l_t = mean |x - y| (losses.py:37) into loss[0]; grad = sign(y - x)/n (may be NULL). ws:
 * >= 1024 floats. */
int encx_l1_loss(const float* x, const float* y, float* loss, float* grad, float* ws, int64_t n,
                 encx_stream_t stream);

/* ---------------------------------------------------------------- RVQ (quantization/core_vq.py)
 * res is the encoder-layout residual [B][D][Tf] (the reference rearranges 'b d n -> b n d',
 * core_vq.py:303; the kernels index it in place). N = B*Tf frames.
 * Nearest code, EuclideanCodebook.quantize (core_vq.py:181-189): idx[n] = argmax_k
 * -((|x_n|^2 - 2 x_n.e_k) + |e_k|^2), first index on ties. direct != 0 selects kmeans' form
 * -sum_d (x_n,d - e_k,d)^2 (core_vq.py:86-89). keys: workspace of N uint64. */
int encx_rvq_argmin(const float* res, const float* embed, int64_t* idx, uint64_t* keys,
                    int64_t B, int64_t D, int64_t Tf, int64_t Kc, int direct,
                    encx_stream_t stream);
/* One VectorQuantization layer after its argmin (core_vq.py:301-324, :346-349), x = layer input:
 * q = embed[idx]; q_ste = ste ? x + (q - x) : q; res_out = x - q_ste (may alias x);
 * out (+)= q_ste; commit_dir (+)= x - q_ste; commit_part[blk] = partial sums of (q_ste - x)^2
 * (reduce with encx_reduce_sum). first != 0 initialises out / commit_dir; out, commit_dir and
 * commit_part may be NULL (eval-mode encode, core_vq.py:357-367, uses ste = 0). */
int encx_rvq_apply(const float* x, float* res_out, const float* embed, const int64_t* idx,
                   float* out, float* commit_dir, float* commit_part, int64_t B, int64_t D,
                   int64_t Tf, int first, int ste, encx_stream_t stream);
/* ResidualVectorQuantization.decode (core_vq.py:369-375) one layer: out (+)= embed[idx]. */
int encx_rvq_gather(const float* embed, const int64_t* idx, float* out, int64_t B, int64_t D,
                    int64_t Tf, int accumulate, encx_stream_t stream);
int64_t encx_rvq_apply_parts(int64_t B, int64_t D, int64_t Tf);
/* EMA codebook update (core_vq.py:227-235): counts/sums of the frames assigned to each code,
 * cluster_size = d*cs + (1-d)*count; embed_avg = d*ea + (1-d)*sum; embed = embed_avg /
 * laplace(cluster_size)*sum(cluster_size). x = the layer input (pre-update residual),
 * layout [B][D][Tf]. Deterministic (fixed summation order per code). */
/* The per-code sums are x^T @ onehot (core_vq.py:228) as an MFMA GEMM with the one-hot operand
 * generated on the fly; ws: encx_rvq_bucket_workspace(N = B*Tf, D, Kc) bytes. */
size_t encx_rvq_bucket_workspace(int64_t N, int64_t D, int64_t Kc);
int encx_rvq_ema(const float* x, const int64_t* idx, float* cluster_size, float* embed_avg,
                 float* embed, float* ws, int64_t B, int64_t D, int64_t Tf, int64_t Kc,
                 float decay, float eps, encx_stream_t stream);
/* encx_rvq_ema in two halves, for the opt-in cross-rank codebook sync: the
 * per-code sums of core_vq.py:227-228 (embed_onehot.sum(0), x.t() @ embed_onehot) land in
 * sums [Kc][D+1] (column D = the count), so a caller can all-reduce them across data-parallel
 * ranks before the EMA; encx_rvq_ema_from_sums then applies :227-235 from them. sums may alias
 * nothing else; ws as for encx_rvq_ema. Same fixed summation order as encx_rvq_ema, so the two
 * halves back to back give bit-identical buffers. */
int encx_rvq_code_sums(const float* x, const int64_t* idx, float* sums, float* ws, int64_t B,
                       int64_t D, int64_t Tf, int64_t Kc, encx_stream_t stream);
int encx_rvq_ema_from_sums(const float* sums, float* cluster_size, float* embed_avg, float* embed,
                           int64_t D, int64_t Kc, float decay, float eps, encx_stream_t stream);
/* One kmeans iteration (core_vq.py:85-100): means <- bucket means where bins > 0.
 * samples [N][D] row-major; means [Kc][D] in/out; bins int64 [Kc] out; ws as above. */
int encx_kmeans_step(const float* samples, float* means, int64_t* bins, int64_t* idx,
                     uint64_t* keys, float* ws, int64_t N, int64_t D, int64_t Kc,
                     encx_stream_t stream);
/* sample_vectors (core_vq.py:69-77) for kmeans' init: rows of a uniform random permutation
 * (num <= N) or uniform draws with replacement, from a counter-based hash of `seed`. */
int encx_sample_rows(const float* samples, float* out, int64_t N, int64_t D, int64_t num,
                     uint64_t seed, encx_stream_t stream);
/* out_rows[n][d] = res[b][d][t] (n = b*Tf + t): the 'b d n -> (b n) d' rearrange */
int encx_bdt_to_nd(const float* res, float* out, int64_t B, int64_t D, int64_t Tf,
                   encx_stream_t stream);
/* out[0] = scale * sum(parts[0..n)) in a fixed order (+ out[0] if accumulate) */
int encx_reduce_sum(const float* parts, int64_t n, float scale, float* out, int accumulate,
                    encx_stream_t stream);

/* ---------------------------------------------------------------- multi-scale mel loss
 * Audio2Mel (audio_to_mel.py:34-55) + the l_f term of total_loss (losses.py:40-42):
 * logmel = log10(clamp(mel_basis @ |STFT(reflect_pad(wav))|^2, 1e-5)), n_fft = win = n,
 * hop = n/4, hann window. encx_mel_spec writes logmel [B*F][64] and (optionally) the raw
 * spectrum (re, im) [B*F][2*nb] for the backward. tables: encx_mel_tables layout. */
size_t encx_mel_tables_floats(int64_t n_fft, int64_t n_mels);
/* window*cos / window*sin DFT tables + mel basis, built on the device from the mel basis
 * uploaded by the caller (host restatement of librosa.filters.mel). */
/* Rewrite the DFT part of a table buffer for window [n_fft] (any window; the mel part is kept). */
int encx_spec_tables_window(float* tables, const float* window, int64_t n_fft, encx_stream_t stream);
int encx_mel_tables_init(float* tables, const float* mel_basis, int64_t n_fft, int64_t n_mels,
                         encx_stream_t stream);
size_t encx_mel_workspace_floats(int64_t B, int64_t T, int64_t n_fft, int64_t n_mels);
/* Forward of one scale for the pair (x = target, y = output): loss_part[0] += (L1 + MSE)
 * between logmel(x) and logmel(y); if grad != NULL, grad (+)= d(L1+MSE)/dy (always added:
 * zero it before the first scale). */
int encx_mel_loss(const float* x, const float* y, const float* tables, float* ws, float* loss,
                  float* grad, int64_t B, int64_t T, int64_t n_fft, int64_t n_mels,
                  encx_stream_t stream);

/* Every scale of the l_f term (losses.py:40-42, n_fft = 2^5..2^11) in one call (round 6): per scale
 * ONE fused launch -- the real FFT of the frames of x and y in LDS, the power spectrum through the
 * mel filters (sparse; the supports are built by encx_mel_tables_init), log10, the L1 + MSE partial
 * sums, and (grad != NULL) d/d|Y|^2 back through the filters and the inverse real FFT to frame
 * gradients -- then one overlap-add of all scales' frame gradients (grad (+)=) and one finish,
 * loss[0] (+)= the scales' L1 + MSE in order (the reference's accumulation, losses.py:41-42).
 * tables: host array of nscales device table pointers (encx_mel_tables_init, 64 mels); n_ffts:
 * host array of the transform sizes (powers of 2, 32..2048). ws:
 * encx_mel_loss_multi_workspace_floats floats. Replaces nscales calls of encx_mel_loss. */
size_t encx_mel_loss_multi_workspace_floats(int64_t B, int64_t T, const int64_t* n_ffts, int64_t nscales);
int encx_mel_loss_multi(const float* x, const float* y, const float* const* tables, const int64_t* n_ffts,
                        int64_t nscales, float* ws, float* loss, float* grad, int64_t B, int64_t T,
                        encx_stream_t stream);
/* Audio2Mel.forward (audio_to_mel.py:34-55) alone: out [B][n_mels][F] log-mel spectrogram
 * (the reference's [B*C, 64, F] before its final reshape). ws: encx_mel_workspace_floats. */
int encx_mel_logmel(const float* x, const float* tables, float* ws, float* out, int64_t B,
                    int64_t T, int64_t n_fft, int64_t n_mels, encx_stream_t stream);
/* frame count of one scale: (T + 2p - n)/h + 1 with h = n/4, p = (n-h)/2 */
int64_t encx_mel_frames(int64_t T, int64_t n_fft);
/* Audio2Mel.forward with any hop and win_length <= n_fft (audio_to_mel.py:34-55): the reflect pad
 * p = (n - hop)/2, the spectrogram of encx_disc_spec_fwd_scaled over `win_tables` (the hann(win)
 * window centred in n zeros, encx_spec_tables_window; scale 1), then out[b][m][f] =
 * log10(max(sum_k mel_basis[m][k] (re^2 + im^2), 1e-5)); mel_basis [n_mels][n/2 + 1] as the
 * caller builds it (librosa.filters.mel, :24). Frames (T + 2p - n)/hop + 1 (T + 2p >= n, p < T).
 * ws: encx_mel_logmel_framed_workspace_floats floats. */
size_t encx_mel_logmel_framed_workspace_floats(int64_t B, int64_t T, int64_t n_fft, int64_t hop);
int encx_mel_logmel_framed(const float* x, const float* win_tables, const float* mel_basis, float* ws, float* out,
                           int64_t B, int64_t T, int64_t n_fft, int64_t hop, int64_t n_mels, encx_stream_t stream);

/* ---------------------------------------------------------------- step-level (train.hip) */
/* out = a*x + (bdev ? bdev[0]*bscale : bscale) * z  -- the RVQ backward (core_vq.py:309,319):
 * d emb = n_q * d quantized + d penalty * 2/(n_q*numel) * sum_i (x_i - q_ste_i). */
int encx_lincomb(const float* x, const float* z, float* out, int64_t n, float a, const float* bdev,
                 float bscale, encx_stream_t stream);
/* Balancer (balancer.py:83-118) on the device. item_norm_mean: out[0] = mean_b ||g_b||_2
 * (grad.norm(dim=1..).mean(), :88-90); ws: encx_item_norm_workspace(B) bytes. */
size_t encx_item_norm_workspace(int64_t B);
int encx_item_norm_mean(const float* g, float* out, float* ws, int64_t B, int64_t L,
                        encx_stream_t stream);
/* Most losses one balancer combines (update / scales); combine takes four grads per call, more
 * are chained (g0 = the previous out, its scale 1). */
#define ENCX_BALANCER_MAX_LOSSES 64
/* averager EMA (:10-28) in fp64: total = total*beta + norm; fix = fix*beta + 1; avg = total/fix;
 * red = [avg*count .., count] for the average_metrics all-reduce (distrib.py:112-124). */
int encx_balancer_update(const float* norms, double* total, double* fix, double* avg, float* red,
                         int nl, double beta, float count, encx_stream_t stream);
/* scales[k] = ratio[k]*total_norm/(eps + avg_k); avg_k from `avg`, or red[k]/red[nl] when
 * from_red (after the all-reduce). */
int encx_balancer_scales(const double* avg, const float* red, const double* ratio, float* scales,
                         int nl, double total_norm, double eps, int from_red,
                         encx_stream_t stream);
/* out = g0*s0 + g1*s1 + g2*s2 + g3*s3 (g1..g3 may be NULL), the balanced output grad (:110-118),
 * summed left to right; out may alias g0, so five or more losses chain calls with g0 = out and
 * s0 = 1 (the reference's `out_grad += grad` order, exactly) */
int encx_balancer_combine(const float* g0, const float* g1, const float* g2, const float* g3,
                          const float* scales, float* out, int64_t n, encx_stream_t stream);
/* torch.optim.Adam step (amsgrad off, no weight decay) over flat fp32 buffers; step >= 1 is the
 * step count after increment (train_multi_gpu.py:295-296 betas (0.5, 0.9)). */
int encx_adam_step(float* p, const float* g, float* m, float* v, int64_t n, double lr, double beta1,
                   double beta2, double eps, int64_t step, encx_stream_t stream);
/* The same step split for HIP-graph replay: encx_adam_hyper writes the step's scalars
 * {1-beta1, beta2, 1-beta2, lr/bc1, sqrt(bc2), eps} (6 floats) into device memory `hp` as a
 * launch argument (eager, before the replay); encx_adam_step_dev (the captured launch) reads them.
 * Bit-identical to encx_adam_step for the same arguments. */
int encx_adam_hyper(float* hp, double lr, double beta1, double beta2, double eps, int64_t step,
                    encx_stream_t stream);
int encx_adam_step_dev(float* p, const float* g, float* m, float* v, int64_t n, const float* hp,
                       encx_stream_t stream);

/* ---- SLSTM (modules/lstm.py:12-28 -> torch.nn.LSTM(dim, dim, num_layers) + skip) ----
 * All L layers run as one diagonal wavefront (launch k advances layer l to frame k - l):
 * T + L - 1 dependent launches forward and 2(T + L) - 1 backward. B <= 64, H % 16 == 0,
 * H <= 1024; gate order i, f, g, o; sequence tensors are [L][B][T][.].
 * Pack layer `layer` for the step kernels: wcat[layer] = [W_ih | W_hh] ([4H][2H]), wcatT[layer]
 * its transpose ([2H][4H]) and bsum[layer] = b_ih + b_hh ([4H]); the buffers hold L layers. */
int encx_lstm_pack(const float* w_ih, const float* w_hh, const float* b_ih, const float* b_hh, float* wcat,
                   float* wcatT, float* bsum, int64_t H, int64_t layer, encx_stream_t stream);
/* Forward (lstm.py:22-28): x, out [B][H][T] (conv layout), out = h_{L-1} (+ x when skip). Saves
 * for the backward xt [B][T][H] (x transposed), Y = h and Cst = c [L][B][T][H], and the gate
 * activations Gs [L][B][T][4H]. */
int encx_lstm_fwd(const float* x, const float* wcat, const float* bsum, float* xt, float* Y, float* Cst,
                  float* Gs, float* out, int skip, int64_t B, int64_t T, int64_t H, int64_t L,
                  encx_stream_t stream);
size_t encx_lstm_bwd_workspace(int64_t B, int64_t T, int64_t H, int64_t L);
/* Backward through time of all layers from dout [B][H][T] (the grad of the LSTM output, before
 * the skip): the gate pre-activation grads DA [L][B][T][4H] and the input grad dx [B][H][T]
 * (added when acc_x; NULL to skip). ws: encx_lstm_bwd_workspace bytes. */
int encx_lstm_bwd(const float* dout, const float* wcatT, const float* Cst, const float* Gs, float* DA, float* dx,
                  int acc_x, float* ws, int64_t B, int64_t T, int64_t H, int64_t L, encx_stream_t stream);
size_t encx_lstm_bwd_weight_workspace(int64_t B, int64_t T, int64_t H);
/* The persistent forward / backward (option LSTM_PERSIST) run the recurrence in ONE launch whose
 * workgroups hand frames to each other through counters with bounded spins (option LSTM_SPIN:
 * log2 of the bound, default about 1 s). They are used only when every workgroup of the grid can
 * be resident at once (the kernel's occupancy times the CU count). The counters are one set per
 * device: persistent launches must be serialised, i.e. every encx_lstm_fwd / encx_lstm_bwd of a
 * process on one stream (or otherwise ordered). A spin that times out, or a counter that ends a
 * launch off its expected count, is counted in a per-device error word: nonzero means a launch's
 * results are garbage. encx_lstm_sync_errors returns (in *count) and clears it; synchronises the
 * device. */
int encx_lstm_sync_errors(int64_t* count);
/* The same without a synchronisation: a one-thread kernel on `stream` adds the error word to
 * *count (a device int32 the caller zeroed once) and clears the word. Capturable; the caller reads
 * *count whenever convenient (e.g. an async copy to pinned memory checked a step later). */
int encx_lstm_sync_read(int32_t* count, encx_stream_t stream);
/* Development: the persistent kernels' per-frame clock stamps (steady clock, 100 MHz) as
 * [kernel 0 fwd / 1 bwd][workgroup < 256][frame < 128][8 points] int64, first n of them; EINVAL
 * unless the library was built with -DENCX_LSTM_TRACE (tools/lstm_trace.py). Synchronises. */
int encx_lstm_trace(int64_t* out, int64_t n);
/* Weight grads of layer `layer` from DA: dw_ih, dw_hh [4H][H] and the bias grad (to both db_ih
 * and db_hh; either may be NULL), written (acc = 0) or added (acc = 1). */
int encx_lstm_bwd_weight(const float* DA, const float* xt, const float* Y, float* dw_ih, float* dw_hh,
                         float* db_ih, float* db_hh, int acc, float* ws, int64_t B, int64_t T, int64_t H,
                         int64_t L, int64_t layer, encx_stream_t stream);

/* ---- MS-STFT discriminator (msstftd.py:28-149) ----
 * NormConv2d (modules/conv.py:125-139) as used by DiscriminatorSTFT: input [B][Ci][T2][Fi]
 * (frames x bins), kernel (KT, KF), stride (1, sf), dilation (dt, 1), zero padding (pt, pf)
 * with T2 preserved, Fo = (Fi + 2 pf - KF)/sf + 1. Weights in the wf layout written by
 * encx_weightnorm_fwd(v, g, wf, NULL, Co, Ci*KT, KF, 1, .) (g may be NULL: plain weight).
 * act = 1 fuses LeakyReLU(0.2) (msstftd.py:101-102) into the output. */
int encx_conv2d_fwd(const float* x, const float* wf, const float* bias, float* y, int64_t B, int64_t Ci,
                    int64_t T2, int64_t Fi, int64_t Co, int64_t Fo, int64_t KT, int64_t KF, int64_t sf,
                    int64_t dt, int64_t pt, int64_t pf, int act, encx_stream_t stream);
/* polyphase weight layout for the backward-data: wp[(co,kt)][ceil(KF/sf)][ci*sf + r] */
int encx_conv2d_wpoly(const float* wf, float* wp, int64_t Co, int64_t Ci, int64_t KT, int64_t KF, int64_t sf,
                      encx_stream_t stream);
/* dx (+)= d/dx, from dy masked by LeakyReLU'(yact) (yact NULL: no output activation, or dy
 * already carries the mask) and multiplied by LeakyReLU'(xact) (xact NULL: the input had no
 * activation, or the caller wants the grad of the post-activation input map). With xact the
 * result is the grad of the input's PRE-activation, which the producing layer then passes as its
 * dy with yact NULL (its bwd-data and bwd-weight skip reading its output map). */
int encx_conv2d_bwd_data(const float* dy, const float* yact, const float* wp, const float* xact, float* dx,
                         int accumulate, int64_t B, int64_t Ci, int64_t T2, int64_t Fi, int64_t Co, int64_t Fo,
                         int64_t KT, int64_t KF, int64_t sf, int64_t dt, int64_t pt, int64_t pf,
                         encx_stream_t stream);
/* encx_conv2d_bwd_data + the feature-matching loss's grad of this layer's input map added in the
 * epilogue (FeatFn's d l_feat / d ff, losses.py:53, fused instead of a grad tensor and an add):
 * dx += c * sign(feat_fake - feat_real), c = feat_g[0] * feat_scale / feat_denom[0] (feat_g NULL:
 * 1); feat_fake is this layer's input map, feat_real its real-audio counterpart. The feature
 * term is added before the xact mask: dx (+)= (d/dx + feature term) * LeakyReLU'(xact). With a
 * feature term, xact must be NULL or feat_fake itself (the layer's input map is both the map whose
 * LeakyReLU' masks the grad and the fake side of the feature pair; the kernels read it once):
 * any other xact is refused (ENCX_EINVAL). */
int encx_conv2d_bwd_data_feat(const float* dy, const float* yact, const float* wp, const float* xact, float* dx,
                              int accumulate, const float* feat_real, const float* feat_fake,
                              const float* feat_denom, const float* feat_g, double feat_scale,
                              const uint8_t* feat_code /* may be NULL */, int64_t B, int64_t Ci, int64_t T2,
                              int64_t Fi, int64_t Co, int64_t Fo, int64_t KT, int64_t KF, int64_t sf, int64_t dt,
                              int64_t pt, int64_t pf, encx_stream_t stream);
size_t encx_conv2d_bwd_weight_workspace(int64_t B, int64_t Ci, int64_t T2, int64_t Fi, int64_t Co, int64_t Fo,
                                        int64_t KT, int64_t KF, int64_t sf, int64_t dt, int64_t pt, int64_t pf);
/* dw [Co][Ci][KT][KF] and db [Co] (either may be NULL), written or added (acc_w / acc_b). */
int encx_conv2d_bwd_weight(const float* dy, const float* yact, const float* x, float* dw, float* db,
                           int acc_w, int acc_b, float* ws, int64_t B, int64_t Ci, int64_t T2, int64_t Fi, int64_t Co,
                           int64_t Fo, int64_t KT, int64_t KF, int64_t sf, int64_t dt, int64_t pt, int64_t pf,
                           encx_stream_t stream);
/* Kernel family of the Conv2d layers: 0 = chosen per layer by the cost model (default), 1 =
 * register-window kernels wherever their shape limits allow, 2 = tiled kernels only. Process-wide;
 * returns the previous setting (any other value only queries). The results of the families agree
 * to fp32 rounding (different summation orders), so tests exercise each at every size. */
int encx_conv2d_select(int mode);
/* Spectrogram(n_fft, hop, win=n_fft, hann, normalized=True, center=False, power=None) of
 * x [B][C][T], written as cat([re, im], 1) in 'b c t w' layout: z [B][2C][Fr][n/2+1]
 * (msstftd.py:97-99). tables: the mel-table buffer of this n_fft (encx_mel_tables_init). */
int encx_disc_spec_fwd(const float* x, const float* tables, float* z, int64_t B, int64_t C, int64_t T,
                       int64_t n_fft, int64_t hop, encx_stream_t stream);
size_t encx_disc_spec_bwd_workspace(int64_t B, int64_t C, int64_t T, int64_t n_fft, int64_t hop);
int encx_disc_spec_bwd(const float* dz, const float* tables, float* dx, float* ws, int accumulate, int64_t B,
                       int64_t C, int64_t T, int64_t n_fft, int64_t hop, encx_stream_t stream);
/* The same with the window and the scale of the caller: tables built by encx_mel_tables_init then
 * encx_spec_tables_window (the window centred in n_fft zeros, as torch.stft does for win_length <
 * n_fft), scale = 1/sqrt(sum w^2) for normalized=True or 1 (msstftd.py:62-64). */
int encx_disc_spec_fwd_scaled(const float* x, const float* tables, float* z, int64_t B, int64_t C, int64_t T,
                              int64_t n_fft, int64_t hop, double scale, encx_stream_t stream);
int encx_disc_spec_bwd_scaled(const float* dz, const float* tables, float* dx, float* ws, int accumulate,
                              int64_t B, int64_t C, int64_t T, int64_t n_fft, int64_t hop, double scale,
                              encx_stream_t stream);
/* Hinge / relative feature-matching losses (losses.py:44-56, 65-80). ws: workspace bytes. */
size_t encx_disc_loss_workspace(void);
/* out[0] (+)= scale * mean(relu(1 + s*x)) */
int encx_hinge_loss(const float* x, int64_t n, double s, double scale, float* out, int accumulate, float* ws,
                    encx_stream_t stream);
int encx_hinge_loss_bwd(const float* x, int64_t n, double s, double scale, const float* g0, float* dx,
                        encx_stream_t stream);
/* out[0] (+)= scale * mean|fr - ff| / mean|fr|; denom[0] = sum|fr| for the backward */
int encx_feat_loss(const float* fr, const float* ff, int64_t n, double scale, float* out, float* denom,
                   int accumulate, float* ws, encx_stream_t stream);
/* encx_feat_loss that also writes the pair's per-element code (1 byte each: bit 0 ff > fr, bit 1
 * ff < fr, bit 2 ff > 0; `code` 4-byte aligned). encx_conv2d_bwd_data_feat given the code
 * (feat_code) reads it in place of feat_real / feat_fake where its kernel supports it. */
int encx_feat_loss_code(const float* fr, const float* ff, int64_t n, double scale, float* out, float* denom,
                        int accumulate, float* ws, uint8_t* code, encx_stream_t stream);
int encx_feat_loss_bwd(const float* fr, const float* ff, int64_t n, double scale, const float* denom,
                       const float* g0, float* dff, encx_stream_t stream);

/* ---- 48 kHz model (config 5) ----
 * GroupNorm(1, C) of norm='time_group_norm' (modules/conv.py:45-49, applied after the conv at
 * :121/:155): y = (x - mean_b) * rstd_b * gamma[c] + beta[c] with the statistics over all of
 * x [B][C][T]; only the window [trim_left, trim_left + Ty) is written, y [B][C][Ty] (the
 * ConvTranspose1d normalises BEFORE SConvTranspose1d trims, conv.py:153-156 then :248-252;
 * Conv1d passes trim_left 0, Ty = T). stats [2B] (mean, rstd) is written for the backward;
 * ws: encx_groupnorm_workspace bytes (fp64 rows). */
size_t encx_groupnorm_workspace(int64_t B, int64_t C);
int encx_groupnorm_fwd(const float* x, const float* gamma, const float* beta, float* y, float* stats, void* ws,
                       int64_t B, int64_t C, int64_t T, int64_t trim_left, int64_t Ty, double eps,
                       encx_stream_t stream);
/* dy [B][C][Ty] (zero outside the window) -> dx [B][C][T] (+)= (acc_x), dgamma / dbeta (+)=
 * (acc_params; either may be NULL); coef: [2B] scratch */
int encx_groupnorm_bwd(const float* dy, const float* x, const float* gamma, const float* stats, float* dx,
                       float* dgamma, float* dbeta, int acc_x, int acc_params, void* ws, float* coef, int64_t B,
                       int64_t C, int64_t T, int64_t trim_left, int64_t Ty, encx_stream_t stream);
/* _linear_overlap_add (utils.py:22-61) of nf <= 32 decoded segments [BC][len_k] (host arrays of
 * device pointers / lengths; all but the last of equal length) at `stride` -> out [BC][total]. */
int encx_overlap_add(const float* const* frames, const int64_t* lengths, int nf, int64_t stride, int64_t BC,
                     float* out, encx_stream_t stream);
/* d frame_k = w * dout[k*stride + j] / sum_w (L0 = the first segment's length) */
int encx_overlap_add_bwd(const float* dout, int nf, int64_t stride, int64_t L0, int64_t BC, int64_t total, int k,
                         int64_t len, float* dframe, encx_stream_t stream);

/* ------------------------------------------------------- .ecdc payload (binary.py, compress.py)
 * The codes of one encoded frame [K][T] are pushed t-major, then codebook (compress.py:88-98),
 * each as `bits` bits of a little-endian bit stream (BitPacker, binary.py:55-88); flush emits the
 * last partial byte, so a frame of n = K*T codes is encx_bitpack_bytes(n, bits) = ceil(n*bits/8)
 * bytes (-1 for bits outside 1..32). Codes are int64 addressed as codes[item*s_item + k*s_k +
 * t*s_t] (any strides, e.g. the transposed view EncodecModel.encode returns); `items` frames of
 * equal (K, T) go in one launch, frame i at out + i*out_stride. *err (device int, caller
 * zeroed) gets 1 if a code is >= 2^bits, which the reference would silently mis-pack. */
int64_t encx_bitpack_bytes(int64_t n_values, int bits);
int encx_bitpack(const int64_t* codes, int64_t s_item, int64_t s_k, int64_t s_t, int64_t items,
                 int64_t K, int64_t T, int bits, uint8_t* out, int64_t out_stride, int* err,
                 encx_stream_t stream);
/* BitUnpacker.pull (binary.py:105-123) for n = K*T codes of each of `items` frames, frame i's
 * bytes at in + i*in_stride (in_stride >= ceil(n*bits/8)). */
int encx_bitunpack(const uint8_t* in, int64_t in_stride, int64_t items, int64_t K, int64_t T,
                   int bits, int64_t* codes, int64_t s_item, int64_t s_k, int64_t s_t,
                   encx_stream_t stream);

/* ------------------------------------------------------ batch assembly (customAudioDataset.py)
 * Clip i of the pool is [src_channels[i]][lengths[i]] fp32 at pool + offsets[i] (device arrays,
 * int64). out [B][C][Tmax]: out[b][c][t] = clip_b[src_channels[b] == 1 ? 0 : c][starts[b] + t]
 * for t < out_len[b], else 0 -- the random tensor_cut crop (customAudioDataset.py:64-69), the
 * mono expand (:51-54) and the zero-pad collate (pad_sequence, :72-91) in one launch. The
 * caller guarantees starts[b] + out_len[b] <= lengths[b] and src_channels[b] in {1, C}; B*C <= 65535. */
int encx_crop_collate(const float* pool, const int64_t* offsets, const int64_t* lengths,
                      const int64_t* src_channels, const int64_t* starts, const int64_t* out_len,
                      float* out, int64_t B, int64_t C, int64_t Tmax, encx_stream_t stream);

/* ------------------------------------------------------ LM entropy coding (use_lm=True)
 * LMModel (model.py:27-65) over StreamingTransformerEncoder (modules/transformer.py:62-119),
 * inference only, and the arithmetic coder of quantization/ac.py. Activations are [B][T][D]
 * fp32 (row n = b*T + t). Every kernel computes a row from that row's inputs alone in a fixed
 * reduction order, so a row's bits do not depend on how many rows share a launch: the encoder
 * runs a frame's T steps as one pass, the decoder one step at a time, and both see identical
 * cdfs (the precondition of arithmetic decoding, ac.py:220-224).
 *
 * encx_lm_input: the LM input (model.py:59-60: sum_k emb[k][idx], k in order), norm_in
 * LayerNorm and the sin position embedding of step offset + t (transformer.py:16-27, 104-113).
 * emb is the K stacked nn.Embedding tables [n_q][card1 = card + 1][D]; idx(b,k,t) =
 * idx[b*s_b + k*s_k + t*s_t], or with `shifted` (offset 0 only) the teacher-forced input of a
 * known code sequence, 0 at t = 0 and codes[b][k][t-1] + 1 after (compress.py:74-79). */
int encx_lm_input(const int64_t* idx, int64_t s_b, int64_t s_k, int64_t s_t, int64_t B, int64_t K,
                  int64_t T, int shifted, const float* emb, int64_t card1, int64_t D, const float* ln_w,
                  const float* ln_b, int64_t offset, const int64_t* dev_step, float max_period, float* x,
                  encx_stream_t stream);
/* One StreamingTransformerEncoderLayer (transformer.py:30-59; nn.TransformerEncoderLayer with
 * norm_first=False, GELU, dropout 0): x [B][T][D] -> y. kv [B][L][2D] is the layer's key |
 * value cache, position s = seq0 + t for row t (seq0 = offset + 1); position 0, the zero state
 * every layer starts with (transformer.py:106), is read from the in_proj bias. Row t attends
 * positions [max(0, s - past_context), s] (transformer.py:52-58, 117-118). Weights in
 * nn.MultiheadAttention / nn.Linear layout; work: encx_lm_layer_workspace(B*T, D, F) bytes. */
int64_t encx_lm_layer_workspace(int64_t N, int64_t D, int64_t F);
int encx_lm_layer(const float* x, float* y, int64_t B, int64_t T, float* kv, int64_t L, int64_t seq0,
                  const int64_t* dev_step, int64_t past_context, int64_t D, int64_t heads, int64_t F, const float* in_w,
                  const float* in_b, const float* out_w, const float* out_b, const float* l1_w,
                  const float* l1_b, const float* l2_w, const float* l2_b, const float* n1_w,
                  const float* n1_b, const float* n2_w, const float* n2_b, float* work,
                  encx_stream_t stream);
/* The first K per-codebook heads (model.py:62-64: linears[k], softmax over the codebook) with
 * the quantized cdf of every (row, k) fused (ac.py:18-53 as compress.py:84-85 calls it,
 * check=False). w [>=K][card][D] stacked, bias [>=K][card]; work: encx_lm_heads_workspace.
 * probas [B][T][K][card] and cdf int32 [B][T][K][card] are each optional (one is required).
 * With sym (codes, sym[b*s_b + k*s_k + t*s_t]) lohi [B][T][K][2] receives each symbol's coding
 * interval (cdf[s-1] or 0, cdf[s] - 1) for encx_ac_encode. *err (device, caller-zeroed) |= 1
 * when a cdf total exceeds 2^total_range_bits (check=True would reject it, ac.py:50; the coder
 * asserts, ac.py:116), |= 2 for a symbol outside [0, card). */
int64_t encx_lm_heads_workspace(int64_t N, int64_t K, int64_t card);
int encx_lm_heads(const float* x, int64_t B, int64_t T, int64_t D, const float* w, const float* bias,
                  int64_t K, int64_t card, float* work, float* probas, int32_t* cdf, int total_range_bits,
                  float roundoff, int min_range, const int64_t* sym, int64_t s_b, int64_t s_k, int64_t s_t,
                  int32_t* lohi, int* err, encx_stream_t stream);
/* build_stable_quantized_cdf (ac.py:18-53) of `rows` pdfs (row r at pdf + r*ld) -> cdf int32
 * [rows][card] (values < 2^31 since total_range_bits <= 30). ENCX_EINVAL where the reference
 * asserts alpha <= 1 or min_range >= 2; *err |= 1 where its check=True would fail. */
int encx_ac_cdf(const float* pdf, int64_t rows, int64_t card, int64_t ld, int total_range_bits, float roundoff,
                int min_range, int32_t* cdf, int* err, encx_stream_t stream);
/* coding interval of sym[r] in cdf row r (ac.py:144-145) -> lohi [rows][2]; *err |= 2 for a
 * symbol outside [0, card). */
int encx_ac_lohi(const int32_t* cdf, int64_t ld, const int64_t* sym, int64_t rows, int64_t card, int32_t* lohi,
                 int* err, encx_stream_t stream);
/* ArithmeticCoder: push every (lo, hi) of a stream in order, then flush (ac.py:130-167); stream
 * s reads lohi + s*n*2 and writes out + s*cap. nbytes[s] = bytes of the stream (the BitPacker's
 * final partial byte included); err[s] = 0, 1 (cdf total above 2^bits: the reference asserts,
 * ac.py:116), 2 (cap too small; nbytes holds the size needed) or 3 (max_bit > 61, ac.py:157).
 * encx_ac_encode_capacity(n, bits) bytes always suffice. */
int64_t encx_ac_encode_capacity(int64_t n_symbols, int total_range_bits);
int encx_ac_encode(const int32_t* lohi, int64_t streams, int64_t n, int total_range_bits, uint8_t* out,
                   int64_t cap, int64_t* nbytes, int* err, encx_stream_t stream);
/* ArithmeticDecoder.pull (ac.py:217-260) of K symbols per stream, symbol k against cdf row
 * cdf[s][k][:card]. Stream s reads data + s*stride (nbytes[s] bytes); state [streams][ENCX_AC_STATE]
 * int64 = (low, high, current as 128-bit values, low word first; max_bit; bits consumed), zero
 * with max_bit (word ENCX_AC_MAXBIT) = -1 for a new stream. The
 * symbol goes to codes[s*c_s + k*c_k + t*c_t] (codes nullable) and sym + 1 to next_idx[s][k]
 * (nullable: the LM input of the next step, compress.py:154-155). err[s]: 1 = the stream ran out
 * (pull returns None), 2 = no interval contains the value (ac.py:238), 3 = max_bit past 96 (a
 * stream the reference's encoder cannot have written, ac.py:157); a failed stream is left
 * untouched by later calls. Bytes consumed = ceil(bits consumed / 8). */
#define ENCX_AC_STATE 8
#define ENCX_AC_MAXBIT 6
#define ENCX_AC_POS 7
int encx_ac_decode(const uint8_t* data, int64_t stride, const int64_t* nbytes, int64_t streams, int64_t* state,
                   const int32_t* cdf, int64_t K, int64_t card, int total_range_bits, int64_t* codes, int64_t c_s,
                   int64_t c_k, int64_t c_t, int64_t t, const int64_t* dev_step, int64_t* next_idx, int* err,
                   encx_stream_t stream);
/* *dev_step += by on the stream. encx_lm_input / encx_lm_layer / encx_ac_decode add *dev_step
 * (nullable) to their offset / seq0 / t, so one captured decode step (a hipGraph) replays for
 * every step; the caller guarantees seq0 + *dev_step + T <= L. */
int encx_lm_step_advance(int64_t* dev_step, int64_t by, encx_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* ENCX_H */
