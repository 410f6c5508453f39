// encx -- the entropy-coding language model (model.py:27-65 LMModel over
// modules/transformer.py:62-119 StreamingTransformerEncoder), inference only.
//
// One code path serves both directions of the LM entropy coder (compress.py:74-89 /
// 129-155): the encoder knows every code up front and runs all T steps of a frame as ONE pass
// (rows = B*T), the decoder runs one row per stream per step. The arithmetic decoder only
// works if both sides see bit-identical probabilities, so every kernel here computes an output
// row from that row's inputs alone with a fixed reduction order: the GEMMs never split K (the
// per-element MFMA accumulation order is the same for every tile shape), the attention /
// LayerNorm / softmax reductions are fixed wave / block trees. A row's bits therefore do not
// depend on how many rows share the launch, and the one-pass encoder and the step-by-step
// decoder agree exactly.
//
// Streaming state (transformer.py:105-118) is kept as a key/value cache per layer,
// kv[b][s][2D] = (k | v) of sequence position s, where s = 0 is the zero vector each layer's
// state starts as (transformer.py:106: a real key with k = in_proj bias, v = its bias) and
// s = offset + t + 1 is step t. Query s attends positions [max(0, s - P), s], P = past_context:
// exactly the keys the reference's truncated state + mask leave (transformer.py:52-58, 117-118).
#include "common.h"
#include "gemm.h"

namespace {

// ---- GEMM operands: activations [N][D] row-major times W^T, W [Nout][D] row-major (nn.Linear)
struct LdRows {
    static constexpr bool A_K_FAST = true, B_N_FAST = false;
    const float* x;
    const float* w;
    int ldx, ldw;
    ENCX_DEV float a(int m, int k) const { return x[(int64_t)m * ldx + k]; }
    ENCX_DEV float b(int k, int n) const { return w[(int64_t)n * ldw + k]; }
};

// in_proj: columns [0, D) -> q rows, [D, 3D) -> the (k | v) cache row of the token's position
struct EpQKV {
    const float* bias;
    float* q;
    float* kv;
    int D, T;
    int64_t L, seq0;
    FastDiv fT;
    ENCX_DEV void operator()(int m, int n, float v) const {
        const float r = v + bias[n];
        if (n < D) {
            q[(int64_t)m * D + n] = r;
        } else {
            const int b = (int)fdiv((uint32_t)m, fT), t = m - b * T;
            kv[((int64_t)b * L + seq0 + t) * (2 * D) + (n - D)] = r;
        }
    }
};

// out = acc + bias (+ residual) (GELU'd when GELU)
template <bool GELU>
struct EpBias {
    const float* bias;
    const float* res;  // nullable
    float* out;
    int ldo;
    ENCX_DEV void operator()(int m, int n, float v) const {
        float r = v + bias[n];
        if (GELU) r = 0.5f * r * (1.f + erff(r * 0.70710678118654752f));  // F.gelu (erf form)
        if (res) r += res[(int64_t)m * ldo + n];
        out[(int64_t)m * ldo + n] = r;
    }
};

constexpr int LN_MAXV = 8;  // D <= 64 * 8

// LayerNorm over one row held by one wave (lane i owns d = i, i + 64, ...), eps 1e-5, biased
// variance (nn.LayerNorm). Deterministic: per-lane sums in d order, then the xor-butterfly.
ENCX_DEV void ln_row(float (&v)[LN_MAXV], int D, const float* w, const float* b, int lane) {
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < LN_MAXV; ++i)
        if (lane + 64 * i < D) s += v[i];
    const float mean = wave_sum(s) / (float)D;
    float q = 0.f;
#pragma unroll
    for (int i = 0; i < LN_MAXV; ++i)
        if (lane + 64 * i < D) {
            const float c = v[i] - mean;
            q += c * c;
        }
    const float rstd = 1.f / sqrtf(wave_sum(q) / (float)D + 1e-5f);
#pragma unroll
    for (int i = 0; i < LN_MAXV; ++i) {
        const int d = lane + 64 * i;
        if (d < D) v[i] = (v[i] - mean) * rstd * w[d] + b[d];
    }
}

// model.py:59-60 + transformer.py:108-113: x = LayerNorm(sum_k emb_k[idx]) + sin embedding.
// One wave per row (b, t). shifted: idx(b,k,t) = t + offset == 0 ? 0 : codes[b][k][t-1] + 1
// (the encoder's teacher-forced inputs, compress.py:74-79), else idx = codes[b][k][t].
__global__ __launch_bounds__(64) void lm_input_kernel(const int64_t* __restrict__ idx, int64_t s_b,
                                                      int64_t s_k, int64_t s_t, int K, int T,
                                                      int shifted, const float* __restrict__ emb,
                                                      int64_t card1, int D, const float* ln_w,
                                                      const float* ln_b, int64_t offset,
                                                      float max_period, float* __restrict__ x) {
    const int row = blockIdx.x, lane = threadIdx.x;
    const int b = row / T, t = row - b * T;
    float v[LN_MAXV];
#pragma unroll
    for (int i = 0; i < LN_MAXV; ++i) v[i] = 0.f;
    for (int k = 0; k < K; ++k) {
        int64_t id;
        if (shifted) id = (t == 0) ? 0 : idx[b * s_b + k * s_k + (int64_t)(t - 1) * s_t] + 1;
        else id = idx[b * s_b + k * s_k + (int64_t)t * s_t];
        const float* e = emb + ((int64_t)k * card1 + id) * D;
#pragma unroll
        for (int i = 0; i < LN_MAXV; ++i)
            if (lane + 64 * i < D) v[i] += e[lane + 64 * i];
    }
    ln_row(v, D, ln_w, ln_b, lane);
    // create_sin_embedding (transformer.py:16-27): phase = pos / max_period^(i / (half - 1))
    const int half = D / 2;
    const float pos = (float)(offset + t);
    float* out = x + (int64_t)row * D;
#pragma unroll
    for (int i = 0; i < LN_MAXV; ++i) {
        const int d = lane + 64 * i;
        if (d < D) {
            const int a = d < half ? d : d - half;
            const float ph = pos / powf(max_period, (float)a / (float)(half - 1));
            out[d] = v[i] + (d < half ? cosf(ph) : sinf(ph));
        }
    }
}

// row-wise LayerNorm (norm1 / norm2, transformer.py:38-39), one wave per row
__global__ __launch_bounds__(64) void lm_ln_kernel(const float* __restrict__ h, int D, const float* w,
                                                   const float* b, float* __restrict__ y) {
    const int row = blockIdx.x, lane = threadIdx.x;
    const float* in = h + (int64_t)row * D;
    float v[LN_MAXV];
#pragma unroll
    for (int i = 0; i < LN_MAXV; ++i) v[i] = (lane + 64 * i < D) ? in[lane + 64 * i] : 0.f;
    ln_row(v, D, w, b, lane);
    float* out = y + (int64_t)row * D;
#pragma unroll
    for (int i = 0; i < LN_MAXV; ++i)
        if (lane + 64 * i < D) out[lane + 64 * i] = v[i];
}

// position 0 of every stream's cache: the zero state's key / value = the in_proj biases
__global__ void lm_phantom_kernel(float* kv, int64_t L, int D, const float* in_b, int B) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= B * 2 * D) return;
    const int b = i / (2 * D), c = i - b * 2 * D;
    kv[(int64_t)b * L * 2 * D + c] = in_b[D + c];
}

// Windowed multi-head attention, one wave per (row, head): scores of the row's query against
// keys s0..s (lane j owns keys s0 + j, s0 + j + 64, ...), softmax (max, exp, fixed-order sum,
// normalise, as torch.softmax), then lane d < hd sums p_j v_j[d] over j in ascending order.
// Dynamic LDS: the window's probabilities (P + 1 floats) + the query (hd floats).
__global__ __launch_bounds__(64) void lm_attn_kernel(const float* __restrict__ q, const float* __restrict__ kv,
                                                     float* __restrict__ ctx, int T, int D, int H, int64_t L,
                                                     int64_t seq0, int64_t P) {
    extern __shared__ float sh[];
    const int wid = blockIdx.x, lane = threadIdx.x;
    const int row = wid / H, h = wid - row * H;
    const int b = row / T, t = row - b * T;
    const int hd = D / H;
    const int64_t s = seq0 + t;
    const int64_t s0 = s - P > 0 ? s - P : 0;
    const int nk = (int)(s - s0 + 1);
    float* qs = sh;
    float* ps = sh + hd;
    const float scale = 1.f / sqrtf((float)hd);
    if (lane < hd) qs[lane] = q[(int64_t)row * D + h * hd + lane];
    __syncthreads();
    const float* kb = kv + ((int64_t)b * L + s0) * (2 * D) + h * hd;
    float mx = -INFINITY;
    for (int j = lane; j < nk; j += 64) {
        const float* kr = kb + (int64_t)j * 2 * D;
        float acc = 0.f;
        for (int d = 0; d < hd; ++d) acc += qs[d] * kr[d];
        acc *= scale;
        ps[j] = acc;
        mx = fmaxf(mx, acc);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 64));
    float sum = 0.f;
    for (int j = lane; j < nk; j += 64) {
        const float e = expf(ps[j] - mx);
        ps[j] = e;
        sum += e;
    }
    sum = wave_sum(sum);
    for (int j = lane; j < nk; j += 64) ps[j] = ps[j] / sum;
    __syncthreads();
    if (lane < hd) {
        const float* vb = kb + D + lane;
        float acc = 0.f;
        for (int j0 = 0; j0 < nk; j0 += 8) {
            float vv[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int j = j0 + u < nk ? j0 + u : nk - 1;
                vv[u] = vb[(int64_t)j * 2 * D];
            }
#pragma unroll
            for (int u = 0; u < 8; ++u)
                if (j0 + u < nk) acc += ps[j0 + u] * vv[u];
        }
        ctx[(int64_t)row * D + h * hd + lane] = acc;
    }
}

}  // namespace

// ---- softmax over the codebook + quantized CDF (ac.hip), shared with the coder entry points
int encx_lm_softmax_cdf_launch(const float* logits, int64_t rows, int card, int64_t ld_in,
                               int from_logits, float* probas, int32_t* cdf, int total_range_bits,
                               float roundoff, int min_range, const int64_t* sym, int64_t s_b,
                               int64_t s_k, int64_t s_t, int K, int T, int32_t* lohi, int* err,
                               hipStream_t st);

extern "C" {

int64_t encx_lm_layer_workspace(int64_t N, int64_t D, int64_t F) {
    if (N < 0 || D <= 0 || F <= 0) return -1;
    return (N * (5 * D + F)) * (int64_t)sizeof(float);
}

int encx_lm_input(const int64_t* idx, int64_t s_b, int64_t s_k, int64_t s_t, int64_t B, int64_t K,
                  int64_t T, int shifted, const float* emb, int64_t card1, int64_t D, const float* ln_w,
                  const float* ln_b, int64_t offset, float max_period, float* x, encx_stream_t stream) {
    ENCX_REQUIRE(B >= 0 && K >= 1 && T >= 0 && D >= 4 && D % 2 == 0 && D <= 64 * LN_MAXV && card1 >= 1);
    ENCX_REQUIRE(!shifted || offset == 0);
    const int64_t rows = B * T;
    if (rows == 0) return 0;
    ENCX_REQUIRE(idx && emb && ln_w && ln_b && x && rows <= INT32_MAX);
    hipLaunchKernelGGL(lm_input_kernel, dim3((unsigned)rows), dim3(64), 0, (hipStream_t)stream, idx, s_b,
                       s_k, s_t, (int)K, (int)T, shifted, emb, card1, (int)D, ln_w, ln_b, offset,
                       max_period, x);
    ENCX_CHECK_LAUNCH();
    return 0;
}

int encx_lm_layer(const float* x, float* y, int64_t B, int64_t T, float* kv, int64_t L, int64_t seq0,
                  int64_t past_context, int64_t D, int64_t heads, int64_t F, const float* in_w,
                  const float* in_b, const float* out_w, const float* out_b, const float* l1_w,
                  const float* l1_b, const float* l2_w, const float* l2_b, const float* n1_w,
                  const float* n1_b, const float* n2_w, const float* n2_b, float* work,
                  encx_stream_t stream) {
    ENCX_REQUIRE(B >= 1 && T >= 0 && D >= 1 && heads >= 1 && D % heads == 0 && D <= 64 * LN_MAXV);
    ENCX_REQUIRE(D / heads <= 64 && F >= 1 && past_context >= 0 && seq0 >= 1 && seq0 + T <= L);
    const int64_t N = B * T;
    if (N == 0) return 0;
    ENCX_REQUIRE(x && y && kv && in_w && in_b && out_w && out_b && l1_w && l1_b && l2_w && l2_b);
    ENCX_REQUIRE(n1_w && n1_b && n2_w && n2_b && work && N <= INT32_MAX && 3 * D <= INT32_MAX);
    hipStream_t st = (hipStream_t)stream;
    const int n = (int)N, d = (int)D, f = (int)F;
    float* q = work;
    float* ctx = q + N * D;
    float* h1 = ctx + N * D;
    float* x1 = h1 + N * D;
    float* ff = x1 + N * D;
    float* h2 = ff + N * F;
    if (seq0 == 1) {
        hipLaunchKernelGGL(lm_phantom_kernel, dim3((unsigned)cdiv(B * 2 * D, 256)), dim3(256), 0, st, kv, L,
                           d, in_b, (int)B);
        ENCX_CHECK_LAUNCH();
    }
    // in_proj (MultiheadAttention), q to the work buffer, k | v into the cache
    int rc = gemm_launch(LdRows{x, in_w, d, d}, EpQKV{in_b, q, kv, d, (int)T, L, seq0, make_fastdiv((uint32_t)T)},
                         n, 3 * d, d, st);
    if (rc) return rc;
    const int64_t P = past_context;
    const int64_t win = (P + 1 < seq0 + T) ? P + 1 : seq0 + T;
    const size_t lds = (size_t)(win + D / heads) * sizeof(float);
    ENCX_REQUIRE(lds <= 64 * 1024);
    hipLaunchKernelGGL(lm_attn_kernel, dim3((unsigned)(N * heads)), dim3(64), lds, st, q, kv, ctx, (int)T, d,
                       (int)heads, L, seq0, P);
    ENCX_CHECK_LAUNCH();
    // out_proj + residual, norm1 (post-norm layer, transformer.py:38)
    rc = gemm_launch(LdRows{ctx, out_w, d, d}, EpBias<false>{out_b, x, h1, d}, n, d, d, st);
    if (rc) return rc;
    hipLaunchKernelGGL(lm_ln_kernel, dim3((unsigned)N), dim3(64), 0, st, h1, d, n1_w, n1_b, x1);
    ENCX_CHECK_LAUNCH();
    // feed-forward: linear1 + GELU, linear2 + residual, norm2 (transformer.py:39)
    rc = gemm_launch(LdRows{x1, l1_w, d, d}, EpBias<true>{l1_b, nullptr, ff, f}, n, f, d, st);
    if (rc) return rc;
    rc = gemm_launch(LdRows{ff, l2_w, f, f}, EpBias<false>{l2_b, x1, h2, d}, n, d, f, st);
    if (rc) return rc;
    hipLaunchKernelGGL(lm_ln_kernel, dim3((unsigned)N), dim3(64), 0, st, h2, d, n2_w, n2_b, y);
    ENCX_CHECK_LAUNCH();
    return 0;
}

int64_t encx_lm_heads_workspace(int64_t N, int64_t K, int64_t card) {
    if (N < 0 || K < 1 || card < 1) return -1;
    return N * K * card * (int64_t)sizeof(float);
}

int encx_lm_heads(const float* x, int64_t B, int64_t T, int64_t D, const float* w, const float* bias,
                  int64_t K, int64_t card, float* work, float* probas, int32_t* cdf, int total_range_bits,
                  float roundoff, int min_range, const int64_t* sym, int64_t s_b, int64_t s_k, int64_t s_t,
                  int32_t* lohi, int* err, encx_stream_t stream) {
    ENCX_REQUIRE(B >= 0 && T >= 0 && D >= 1 && K >= 1 && card >= 1 && card <= 65536);
    const int64_t N = B * T;
    if (N == 0) return 0;
    ENCX_REQUIRE(x && w && bias && work && (probas || cdf) && N <= INT32_MAX && K * card <= INT32_MAX);
    ENCX_REQUIRE(!sym || (cdf && lohi));
    hipStream_t st = (hipStream_t)stream;
    // the K per-codebook projections (model.py:62-63) as one GEMM: W stacked [K*card][D]
    int rc = gemm_launch(LdRows{x, w, (int)D, (int)D}, EpBias<false>{bias, nullptr, work, (int)(K * card)},
                         (int)N, (int)(K * card), (int)D, st);
    if (rc) return rc;
    return encx_lm_softmax_cdf_launch(work, N * K, (int)card, card, 1, probas, cdf, total_range_bits,
                                      roundoff, min_range, sym, s_b, s_k, s_t, (int)K, (int)T, lohi, err, st);
}

}  // extern "C"
