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
// kv[b][s][2D] = (k | v) of sequence position s = offset + t + 1 for step t. Position 0 is the
// zero vector each layer's state starts as (transformer.py:106): a real key, with k = the
// in_proj bias and v = its bias, which the attention reads from the bias (never stored). Query s attends positions [max(0, s - P), s], P = past_context:
// exactly the keys the reference's truncated state + mask leave (transformer.py:52-58, 117-118).
#include "common.h"
#include "gemm.h"

// No mul+add contraction anywhere in this file: the same quantity computed by two kernels (e.g.
// a score scaled, stored, then offset by the max, against the same expression inline) must round
// identically, and __fmul_rn alone does not stop clang fusing it into a following add.
#pragma clang fp contract(off)

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
    const int64_t* dstep;  // nullable: device-side step added to seq0 (graph-captured decode)
    FastDiv fT;
    ENCX_DEV void operator()(int m, int n, float v) const {
        const float r = v + bias[n];
        if (n < D) {
            q[(int64_t)m * D + n] = r;
        } else {
            const int b = (int)fdiv((uint32_t)m, fT), t = m - b * T;
            const int64_t s = seq0 + (dstep ? *dstep : 0) + t;
            kv[((int64_t)b * L + s) * (2 * D) + (n - D)] = r;
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
                                                      const int64_t* dstep, float max_period,
                                                      float* __restrict__ x) {
    const int row = blockIdx.x, lane = threadIdx.x;
    if (dstep) offset += *dstep;
    const int b = row / T, t = row - b * T;
    // lane k < K fetches index k (all in flight together), the table rows follow; the sum
    // stays in k order (model.py:59: sum over k = 0.. of emb[k](indices[:, k]))
    int64_t my = 0;
    if (lane < K) {
        if (shifted) my = (t == 0) ? 0 : idx[b * s_b + lane * s_k + (int64_t)(t - 1) * s_t] + 1;
        else my = idx[b * s_b + lane * s_k + (int64_t)t * s_t];
    }
    float v[LN_MAXV];
#pragma unroll
    for (int i = 0; i < LN_MAXV; ++i) v[i] = 0.f;
    for (int k0 = 0; k0 < K; k0 += 4) {
        float e[4][LN_MAXV];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int k = k0 + u < K ? k0 + u : K - 1;
            const int64_t id = __shfl(my, k, 64);
            const float* er = emb + ((int64_t)k * card1 + id) * D;
#pragma unroll
            for (int i = 0; i < LN_MAXV; ++i) e[u][i] = (lane + 64 * i < D) ? er[lane + 64 * i] : 0.f;
        }
#pragma unroll
        for (int u = 0; u < 4; ++u)
            if (k0 + u < K) {
#pragma unroll
                for (int i = 0; i < LN_MAXV; ++i) v[i] += e[u][i];
            }
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

// Windowed multi-head attention. The arithmetic of one (query, head) is fixed as
//   s_j = (fmaf chain over d of q_d k_jd, from 0) * scale,  m = max_j s_j,
//   S = sum_j expf(s_j - m) in ascending j,  o_d = fmaf chain over ascending j of
//   (expf(s_j - m) / S) v_jd, from 0
// (softmax then p.V as torch computes it), over the window j = s0..s, s0 = max(0, s - P).
// Two kernels evaluate exactly that sequence -- a workgroup per (row, head) for a few rows (the
// decoder's step), a wave per 64 queries with the keys staged in LDS for many (the encoder's
// one pass) -- so a row's bits never depend on which kernel or launch produced them.
// Sequence position 0, the zero state every layer starts with (transformer.py:106), is not
// stored: its key and value are the in_proj biases, read from `in_b`.
// head-slice element d of a row, clamped so the load is unconditional (a bounds test around
// each load compiles to one branch and one memory round trip per element)
ENCX_DEV int dcl(int d, int hd) { return d < hd ? d : hd - 1; }
ENCX_DEV float sel(bool c, float v) { return c ? v : 0.f; }
ENCX_DEV const float* kv_row(const float* kv, const float* in_b, int64_t base, int64_t pos, int D, int hoff, int v) {
    return pos == 0 ? in_b + D + v * D + hoff : kv + (base + pos) * (2 * D) + v * D + hoff;
}

// a few rows: one 256-thread workgroup per (row, head); dynamic LDS = scores / weights [P + 1]
// + the window's values [P + 1][hd]
template <int HD>
__global__ __launch_bounds__(256) void lm_attn_row_kernel(const float* __restrict__ q, const float* __restrict__ kv,
                                                          const float* __restrict__ in_b, float* __restrict__ ctx,
                                                          int T, int D, int H, int64_t L, int64_t seq0,
                                                          const int64_t* dstep, int64_t P) {
    extern __shared__ float sh[];
    __shared__ float red[8];
    __shared__ float Ssh;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int row = blockIdx.x / H, h = blockIdx.x - row * H;
    const int b = row / T, t = row - b * T;
    const int hd = D / H, hoff = h * hd;
    const int64_t s = seq0 + (dstep ? *dstep : 0) + t;
    const int64_t s0 = s - P > 0 ? s - P : 0;
    const int nk = (int)(s - s0 + 1);
    const int64_t base = (int64_t)b * L;
    float* es = sh;            // [nk]
    float* vs = sh + nk;       // [nk][hd]
    const float scale = 1.f / sqrtf((float)hd);
    float qv[HD];
    const float* qr = q + (int64_t)row * D + hoff;
#pragma unroll
    for (int d = 0; d < HD; ++d) qv[d] = sel(d < hd, qr[dcl(d, hd)]);
    // values of the window into LDS (coalesced along d), scores of this thread's keys
    for (int i = tid; i < nk * hd; i += 256) {
        const int j = i / hd, d = i - j * hd;
        vs[i] = kv_row(kv, in_b, base, s0 + j, D, hoff, 1)[d];
    }
    float mx = -INFINITY;
    for (int j = tid; j < nk; j += 256) {
        const float* kr = kv_row(kv, in_b, base, s0 + j, D, hoff, 0);
        float kk[HD];
#pragma unroll
        for (int d = 0; d < HD; ++d) kk[d] = kr[dcl(d, hd)];
        float acc = 0.f;
#pragma unroll
        for (int d = 0; d < HD; ++d) acc = fmaf(qv[d], kk[d], acc);   // qv = 0 past hd: adds a zero
        acc = __fmul_rn(acc, scale);  // never contracted into the next subtraction
        es[j] = acc;
        mx = fmaxf(mx, acc);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 64));
    if (lane == 0) red[w] = mx;
    __syncthreads();
    mx = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
    for (int j = tid; j < nk; j += 256) es[j] = expf(es[j] - mx);
    __syncthreads();
    if (tid == 0) {
        float S = 0.f;
        for (int j = 0; j < nk; ++j) S += es[j];
        Ssh = S;
    }
    __syncthreads();
    const float S = Ssh;
    for (int j = tid; j < nk; j += 256) es[j] = es[j] / S;
    __syncthreads();
    if (tid < hd) {
        float o = 0.f;
        for (int j = 0; j < nk; ++j) o = fmaf(es[j], vs[j * hd + tid], o);
        ctx[(int64_t)row * D + hoff + tid] = o;
    }
}

// many rows: one wave per (stream, head, 64 consecutive queries), lane = query. The wave walks
// the union of the 64 windows key by key, so every key / value row address is wave-uniform
// (scalar loads, no LDS, high occupancy); each lane takes the keys inside its own window, in
// ascending order. The scores are recomputed in each of the three passes (max, sum, p.V).
template <int HD>
__global__ __launch_bounds__(256) void lm_attn_block_kernel(const float* __restrict__ q, const float* __restrict__ kv,
                                                            const float* __restrict__ in_b, float* __restrict__ ctx,
                                                            int T, int D, int H, int64_t L, int64_t seq0, int64_t P,
                                                            int tblocks, int nwaves) {
    const int lane = threadIdx.x & 63;
    int id = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (id >= nwaves) return;
    const int tb = id % tblocks;
    id /= tblocks;
    const int h = id % H, b = id / H;
    const int hd = D / H, hoff = h * hd;
    const int t0 = tb * 64;
    const int t = t0 + lane;
    const bool live = t < T;
    const int64_t sfirst = seq0 + t0;
    const int64_t slast = seq0 + min(T, t0 + 64) - 1;
    const int64_t u0 = sfirst - P > 0 ? sfirst - P : 0;
    const int64_t base = (int64_t)b * L;
    const int64_t s = seq0 + (live ? t : t0);
    const int64_t s0 = s - P > 0 ? s - P : 0;
    const float scale = 1.f / sqrtf((float)hd);
    float qv[HD];
    const int64_t row = (int64_t)b * T + (live ? t : t0);
    const float* qr = q + row * D + hoff;
#pragma unroll
    for (int d = 0; d < HD; ++d) qv[d] = sel(d < hd, qr[dcl(d, hd)]);
    auto score = [&](int64_t pos) {
        const float* kr = kv_row(kv, in_b, base, pos, D, hoff, 0);
        float kk[HD];
#pragma unroll
        for (int d = 0; d < HD; ++d) kk[d] = kr[dcl(d, hd)];
        float acc = 0.f;
#pragma unroll
        for (int d = 0; d < HD; ++d) acc = fmaf(qv[d], kk[d], acc);   // qv = 0 past hd: adds a zero
        return __fmul_rn(acc, scale);
    };
    float mx = -INFINITY;
    for (int64_t pos = u0; pos <= slast; ++pos) {
        const float sc = score(pos);
        if (pos >= s0 && pos <= s) mx = fmaxf(mx, sc);
    }
    float S = 0.f;
    for (int64_t pos = u0; pos <= slast; ++pos) {
        const float e = expf(score(pos) - mx);
        if (pos >= s0 && pos <= s) S += e;
    }
    float o[HD];
#pragma unroll
    for (int d = 0; d < HD; ++d) o[d] = 0.f;
    for (int64_t pos = u0; pos <= slast; ++pos) {
        const float p = expf(score(pos) - mx) / S;
        const float* vr = kv_row(kv, in_b, base, pos, D, hoff, 1);
        float vv[HD];
#pragma unroll
        for (int d = 0; d < HD; ++d) vv[d] = vr[dcl(d, hd)];
        if (pos >= s0 && pos <= s) {
#pragma unroll
            for (int d = 0; d < HD; ++d) o[d] = fmaf(p, vv[d], o[d]);
        }
    }
    if (live) {
        float* out = ctx + row * D + hoff;
#pragma unroll
        for (int d = 0; d < HD; ++d)
            if (d < hd) out[d] = o[d];
    }
}

// ---- few-row GEMM (the decode step: one row per stream) on the VALU ----------------------
// out(m, n) = sum_k x[m][k] w[n][k] as an fmaf chain in ascending k from 0: bitwise what
// gemm_kernel's v_mfma_f32_32x32x2_f32 chain gives (MI355X_MICROARCH.md: exact f32, fmaf-chain
// identical), so a row comes out the same from either kernel. One output per thread; a
// workgroup covers 32 columns x 8 rows, staging x and w 128 k at a time through LDS
// (coalesced float4 loads, the next chunk's loads in flight while this one is summed).
constexpr int GV_NB = 32, GV_MB = 8, GV_KC = 128, GV_MMAX = 64;
template <class EP>
__global__ __launch_bounds__(256) void lm_gemv_kernel(const float* __restrict__ x, int ldx,
                                                      const float* __restrict__ w, int ldw, int M, int N,
                                                      int K, EP ep) {
    __shared__ float xs[GV_MB][GV_KC + 1];
    __shared__ float ws[GV_NB][GV_KC + 1];
    const int tid = threadIdx.x;
    const int nl = tid % GV_NB, r = tid / GV_NB;
    const int n0 = blockIdx.x * GV_NB, m0 = blockIdx.y * GV_MB;
    // staging roles: x -> thread tid loads 4 consecutive k of row tid / 32; w -> 4 float4 of
    // rows (tid / 32) + 8 i, i < 4, at k offset 4 * (tid % 32)
    const int sr = tid / 32, sk = 4 * (tid % 32);
    const int xm = min(m0 + sr, M - 1);
    float4 xr, wr[4];
    auto fetch = [&](int k0) {
        const int k = k0 + sk;
        const bool full = k + 4 <= K;
        const float* xp = x + (int64_t)xm * ldx;
        if (full) {
            xr = make_float4(xp[k], xp[k + 1], xp[k + 2], xp[k + 3]);
        } else {
            xr.x = k < K ? xp[k] : 0.f;
            xr.y = k + 1 < K ? xp[k + 1] : 0.f;
            xr.z = k + 2 < K ? xp[k + 2] : 0.f;
            xr.w = k + 3 < K ? xp[k + 3] : 0.f;
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int n = min(n0 + sr + 8 * i, N - 1);
            const float* wp = w + (int64_t)n * ldw;
            if (full) {
                wr[i] = *reinterpret_cast<const float4*>(wp + k);
            } else {
                wr[i].x = k < K ? wp[k] : 0.f;
                wr[i].y = k + 1 < K ? wp[k + 1] : 0.f;
                wr[i].z = k + 2 < K ? wp[k + 2] : 0.f;
                wr[i].w = k + 3 < K ? wp[k + 3] : 0.f;
            }
        }
    };
    float acc = 0.f;
    fetch(0);
    for (int k0 = 0; k0 < K; k0 += GV_KC) {
        __syncthreads();
        xs[sr][sk] = xr.x;
        xs[sr][sk + 1] = xr.y;
        xs[sr][sk + 2] = xr.z;
        xs[sr][sk + 3] = xr.w;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            ws[sr + 8 * i][sk] = wr[i].x;
            ws[sr + 8 * i][sk + 1] = wr[i].y;
            ws[sr + 8 * i][sk + 2] = wr[i].z;
            ws[sr + 8 * i][sk + 3] = wr[i].w;
        }
        __syncthreads();
        if (k0 + GV_KC < K) fetch(k0 + GV_KC);
        const int kc = min(GV_KC, K - k0);
#pragma unroll 8
        for (int k = 0; k < kc; ++k) acc = fmaf(xs[r][k], ws[nl][k], acc);
    }
    const int m = m0 + r, n = n0 + nl;
    if (m < M && n < N) ep(m, n, acc);
}

// out(M x N) = x W^T through the epilogue; M <= 64 rows on the VALU kernel, more on the MFMA
// GEMM (never split over k: the reduction order is the same in both)
template <class EP>
int lm_linear(const float* x, int ldx, const float* w, int ldw, int M, int N, int K, const EP& ep, hipStream_t st) {
    const bool vec4 = (ldw % 4) == 0 && ((uintptr_t)w % 16) == 0;
    if (M <= GV_MMAX && vec4) {
        hipLaunchKernelGGL(lm_gemv_kernel<EP>, dim3((unsigned)cdiv(N, GV_NB), (unsigned)cdiv(M, GV_MB)), dim3(256),
                           0, st, x, ldx, w, ldw, M, N, K, ep);
        ENCX_CHECK_LAUNCH();
        return 0;
    }
    return gemm_launch(LdRows{x, w, ldx, ldw}, ep, M, N, K, st);
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
                  const float* ln_b, int64_t offset, const int64_t* dev_step, float max_period, float* x,
                  encx_stream_t stream) {
    ENCX_REQUIRE(B >= 0 && K >= 1 && K <= 64 && T >= 0 && D >= 4 && D % 2 == 0 && D <= 64 * LN_MAXV && card1 >= 1);
    ENCX_REQUIRE(!shifted || (offset == 0 && !dev_step));
    const int64_t rows = B * T;
    if (rows == 0) return 0;
    ENCX_REQUIRE(idx && emb && ln_w && ln_b && x && rows <= INT32_MAX);
    hipLaunchKernelGGL(lm_input_kernel, dim3((unsigned)rows), dim3(64), 0, (hipStream_t)stream, idx, s_b,
                       s_k, s_t, (int)K, (int)T, shifted, emb, card1, (int)D, ln_w, ln_b, offset,
                       dev_step, max_period, x);
    ENCX_CHECK_LAUNCH();
    return 0;
}

int encx_lm_layer(const float* x, float* y, int64_t B, int64_t T, float* kv, int64_t L, int64_t seq0,
                  const int64_t* dev_step, int64_t past_context, int64_t D, int64_t heads, int64_t F, const float* in_w,
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
    // in_proj (MultiheadAttention), q to the work buffer, k | v into the cache
    int rc = lm_linear(x, d, in_w, d, n, 3 * d, d,
                       EpQKV{in_b, q, kv, d, (int)T, L, seq0, dev_step, make_fastdiv((uint32_t)T)}, st);
    if (rc) return rc;
    const int64_t P = past_context;
    // with a device-side step the window is unknown here: size for the full P + 1
    const int64_t win = (P + 1 < seq0 + T || dev_step) ? P + 1 : seq0 + T;
    const int hd = (int)(D / heads);
    ENCX_REQUIRE(N * heads <= INT32_MAX);
    if (N * heads <= 4096 || dev_step) {
        const size_t lds = (size_t)win * (hd + 1) * sizeof(float);
        ENCX_REQUIRE(lds <= 150 * 1024);
        if (hd <= 32)
            hipLaunchKernelGGL(lm_attn_row_kernel<32>, dim3((unsigned)(N * heads)), dim3(256), lds, st, q, kv, in_b,
                               ctx, (int)T, d, (int)heads, L, seq0, dev_step, P);
        else
            hipLaunchKernelGGL(lm_attn_row_kernel<64>, dim3((unsigned)(N * heads)), dim3(256), lds, st, q, kv, in_b,
                               ctx, (int)T, d, (int)heads, L, seq0, dev_step, P);
    } else {
        const int tblocks = (int)cdiv(T, 64);
        const int64_t nw = B * heads * tblocks;
        ENCX_REQUIRE(nw <= INT32_MAX);
        if (hd <= 32)
            hipLaunchKernelGGL(lm_attn_block_kernel<32>, dim3((unsigned)cdiv(nw, 4)), dim3(256), 0, st, q, kv, in_b,
                               ctx, (int)T, d, (int)heads, L, seq0, P, tblocks, (int)nw);
        else
            hipLaunchKernelGGL(lm_attn_block_kernel<64>, dim3((unsigned)cdiv(nw, 4)), dim3(256), 0, st, q, kv, in_b,
                               ctx, (int)T, d, (int)heads, L, seq0, P, tblocks, (int)nw);
    }
    ENCX_CHECK_LAUNCH();
    // out_proj + residual, norm1 (post-norm layer, transformer.py:38)
    rc = lm_linear(ctx, d, out_w, d, n, d, d, EpBias<false>{out_b, x, h1, d}, st);
    if (rc) return rc;
    hipLaunchKernelGGL(lm_ln_kernel, dim3((unsigned)N), dim3(64), 0, st, h1, d, n1_w, n1_b, x1);
    ENCX_CHECK_LAUNCH();
    // feed-forward: linear1 + GELU, linear2 + residual, norm2 (transformer.py:39)
    rc = lm_linear(x1, d, l1_w, d, n, f, d, EpBias<true>{l1_b, nullptr, ff, f}, st);
    if (rc) return rc;
    rc = lm_linear(ff, f, l2_w, f, n, d, f, EpBias<false>{l2_b, x1, h2, d}, st);
    if (rc) return rc;
    hipLaunchKernelGGL(lm_ln_kernel, dim3((unsigned)N), dim3(64), 0, st, h2, d, n2_w, n2_b, y);
    ENCX_CHECK_LAUNCH();
    return 0;
}

namespace {
__global__ void lm_step_advance_kernel(int64_t* step, int64_t by) {
    if (threadIdx.x == 0) *step += by;
}
}  // namespace

int encx_lm_step_advance(int64_t* dev_step, int64_t by, encx_stream_t stream) {
    ENCX_REQUIRE(dev_step);
    hipLaunchKernelGGL(lm_step_advance_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, dev_step, by);
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
    int rc = lm_linear(x, (int)D, w, (int)D, (int)N, (int)(K * card), (int)D,
                       EpBias<false>{bias, nullptr, work, (int)(K * card)}, st);
    if (rc) return rc;
    return encx_lm_softmax_cdf_launch(work, N * K, (int)card, card, 1, probas, cdf, total_range_bits,
                                      roundoff, min_range, sym, s_b, s_k, s_t, (int)K, (int)T, lohi, err, st);
}

}  // extern "C"
