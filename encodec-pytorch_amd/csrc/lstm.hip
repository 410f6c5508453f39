// SLSTM (modules/lstm.py:12-28): nn.LSTM(H, H, num_layers) over the 75 latent frames + skip.
//
// Per layer the work splits into
//   * the input projection Gx = X W_ih^T + b_ih + b_hh for ALL frames at once: one MFMA GEMM
//     [B*T x H] x [H x 4H] on the generic skeleton (gemm.h);
//   * the recurrence, one fused launch per frame: h_{t-1} W_hh^T on v_mfma_f32_16x16x4_f32
//     (4 waves split the reduction, summed in LDS in wave order) + the gate nonlinearities +
//     the cell update, writing h_t, c_t and the gate activations the backward needs;
//   * backward: per frame an elementwise kernel (gate grads, cell-grad carry) and a small
//     MFMA GEMM for the recurrent grad da_t W_hh; then three big GEMMs for dW_hh, dW_ih
//     (+ the bias column) and dX over all frames.
// Sequence tensors are [B][T][.] (row m = b*T + t). Gate order i, f, g, o (torch).
#include "common.h"
#include "gemm.h"

typedef float f32x4v __attribute__((ext_vector_type(4)));

namespace {

ENCX_DEV f32x4v mfma16(float a, float b, f32x4v c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}
ENCX_DEV float sigm(float x) { return 1.f / (1.f + expf(-x)); }

constexpr int UNITS = 4;  // hidden units per forward workgroup (16 gate columns)

// Operand fragments for v_mfma_f32_16x16x4_f32 over a 16-deep k group: lane (col = l&15,
// kk = l>>4) supplies k = 16*grp + 4*kk + s for s = 0..3 in four consecutive MFMAs, so both
// operands come in as one aligned float4 per lane and group (the summation order over k is
// a permutation of the natural one; fp32 accumulate).
ENCX_DEV float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }
ENCX_DEV float at4(const float4& v, int s) { return s == 0 ? v.x : s == 1 ? v.y : s == 2 ? v.z : v.w; }

// ------------------------------------------------------------------------- forward step
// Workgroup: UNITS hidden units = 16 gate columns; 4 waves interleave the H/16 k-groups.
// G = k-groups per wave, RT = 16-row batch tiles.
template <int G, int RT>
__global__ __launch_bounds__(256) void lstm_fwd_step(const float* Gx, const float* Whh, float* Y,
                                                     float* C, float* Gs, int B, int T, int H, int t) {
    __shared__ float red[4][64][17];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int u0 = blockIdx.x * UNITS;
    const int col = lane & 15, kk = lane >> 4;
    const int NG = H >> 4;
    const int j = (col >> 2) * H + u0 + (col & 3);  // gate column of this lane
    // the gate phase's own operands (B*UNITS <= 256 threads), fetched before the MFMA chain
    const int pb = tid / UNITS, pu = u0 + (tid - pb * UNITS);
    const bool pact = tid < B * UNITS && pu < H;
    const int64_t po = ((int64_t)pb * T + t) * H + pu;
    float gxv[4] = {0.f, 0.f, 0.f, 0.f}, cpv = 0.f;
    if (pact) {
        const float* gx = Gx + ((int64_t)pb * T + t) * 4 * H;
#pragma unroll
        for (int g = 0; g < 4; ++g) gxv[g] = gx[g * H + pu];
        if (t > 0) cpv = C[po - H];
    }
    float4 wv[G], hv[RT][G];
#pragma unroll
    for (int g = 0; g < G; ++g) {
        const int gi = wave + 4 * g;
        wv[g] = gi < NG ? ld4(Whh + (int64_t)j * H + gi * 16 + 4 * kk) : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
        for (int r = 0; r < RT; ++r) {
            const int row = r * 16 + col;
            hv[r][g] = (t > 0 && row < B && gi < NG)
                           ? ld4(Y + ((int64_t)row * T + (t - 1)) * H + gi * 16 + 4 * kk)
                           : make_float4(0.f, 0.f, 0.f, 0.f);
        }
    }
    f32x4v acc[RT];
#pragma unroll
    for (int r = 0; r < RT; ++r) acc[r] = (f32x4v){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int g = 0; g < G; ++g)
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
            for (int r = 0; r < RT; ++r) acc[r] = mfma16(at4(hv[r][g], s), at4(wv[g], s), acc[r]);
#pragma unroll
    for (int r = 0; r < RT; ++r)
#pragma unroll
        for (int q = 0; q < 4; ++q) red[wave][r * 16 + kk * 4 + q][col] = acc[r][q];
    __syncthreads();
    if (pact) {
        const int uu = pu - u0;
        float pre[4];
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const int cc = g * 4 + uu;
            pre[g] = gxv[g] + (((red[0][pb][cc] + red[1][pb][cc]) + red[2][pb][cc]) + red[3][pb][cc]);
        }
        const float ig = sigm(pre[0]), fg = sigm(pre[1]), gg = tanhf(pre[2]), og = sigm(pre[3]);
        const float c = fg * cpv + ig * gg;
        C[po] = c;
        Y[po] = og * tanhf(c);
        float* gs = Gs + ((int64_t)pb * T + t) * 4 * H;
        gs[pu] = ig;
        gs[H + pu] = fg;
        gs[2 * H + pu] = gg;
        gs[3 * H + pu] = og;
    }
}

// ------------------------------------------------------------------------- backward step
// Per frame t (descending) two launches:
//   E(t): dh = dY[t] + sum_s P[s] (the recurrent grad from frame t+1, split partials summed in
//         a fixed order); dc = dh o (1 - tanh^2 c) + dcn; da_{i,f,g,o} -> DA[b][t]; dcn <- dc f
//   G(t): P[s][b][u] = sum_{j in split s} DA[b][t][j] W_hh[j][u]  (MFMA 16x16x4; the 4H
//         reduction split over blockIdx.y so the grid covers ~256 CUs instead of H/16)
__global__ void lstm_bwd_elem(const float* dY, const float* P, int ns, float* dcn, const float* C,
                              const float* Gs, float* DA, int B, int T, int H, int t) {
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= B * H) return;
    const int b = p / H, u = p - b * H;
    const bool rec = t < T - 1;
    float dhr = 0.f;
    if (rec)
        for (int s = 0; s < ns; ++s) dhr += P[(int64_t)s * B * H + p];
    const int64_t o = ((int64_t)b * T + t) * H + u;
    const float dh = dY[o] + dhr;
    const float* gs = Gs + ((int64_t)b * T + t) * 4 * H;
    const float ig = gs[u], fg = gs[H + u], gg = gs[2 * H + u], og = gs[3 * H + u];
    const float c = C[o], cp = t > 0 ? C[o - H] : 0.f, tc = tanhf(c);
    const float dc = dh * og * (1.f - tc * tc) + (rec ? dcn[p] : 0.f);
    float* da = DA + ((int64_t)b * T + t) * 4 * H;
    da[u] = dc * gg * ig * (1.f - ig);
    da[H + u] = dc * cp * fg * (1.f - fg);
    da[2 * H + u] = dc * ig * (1.f - gg * gg);
    da[3 * H + u] = dh * tc * og * (1.f - og);
    dcn[p] = dc * fg;
}

template <int G, int RT>
__global__ __launch_bounds__(256) void lstm_bwd_gemm(const float* DA, const float* WhhT, float* P, int B,
                                                     int T, int H, int t, int gper) {
    __shared__ float red[4][64][17];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int c0 = blockIdx.x * 16, s = blockIdx.y, col = lane & 15, kk = lane >> 4;
    const int K = 4 * H, g0 = s * gper;
    float4 wv[G], av[RT][G];
#pragma unroll
    for (int g = 0; g < G; ++g) {
        const int gl = wave + 4 * g, gi = g0 + gl;
        const bool ok = gl < gper;
        wv[g] = ok ? ld4(WhhT + (int64_t)(c0 + col) * K + gi * 16 + 4 * kk) : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
        for (int r = 0; r < RT; ++r) {
            const int row = r * 16 + col;
            av[r][g] = (ok && row < B) ? ld4(DA + ((int64_t)row * T + t) * K + gi * 16 + 4 * kk)
                                       : make_float4(0.f, 0.f, 0.f, 0.f);
        }
    }
    f32x4v acc[RT];
#pragma unroll
    for (int r = 0; r < RT; ++r) acc[r] = (f32x4v){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int g = 0; g < G; ++g)
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
            for (int r = 0; r < RT; ++r) acc[r] = mfma16(at4(av[r][g], q), at4(wv[g], q), acc[r]);
#pragma unroll
    for (int r = 0; r < RT; ++r)
#pragma unroll
        for (int q = 0; q < 4; ++q) red[wave][r * 16 + kk * 4 + q][col] = acc[r][q];
    __syncthreads();
    for (int p = tid; p < B * 16; p += 256) {
        const int b = p >> 4, cc = p & 15;
        P[((int64_t)s * B + b) * H + c0 + cc] = ((red[0][b][cc] + red[1][b][cc]) + red[2][b][cc]) + red[3][b][cc];
    }
}

__global__ void transpose_kernel(const float* in, float* out, int R, int Cc) {  // out[c][r] = in[r][c]
    __shared__ float tile[32][33];
    const int r0 = blockIdx.y * 32, c0 = blockIdx.x * 32;
    for (int i = threadIdx.y; i < 32; i += 8) {
        const int r = r0 + i, c = c0 + threadIdx.x;
        if (r < R && c < Cc) tile[i][threadIdx.x] = in[(int64_t)r * Cc + c];
    }
    __syncthreads();
    for (int i = threadIdx.y; i < 32; i += 8) {
        const int c = c0 + i, r = r0 + threadIdx.x;
        if (r < R && c < Cc) out[(int64_t)c * R + r] = tile[threadIdx.x][i];
    }
}

template <int G>
static void fwd_step_rt(int RT, dim3 grid, hipStream_t st, const float* Gx, const float* Whh, float* Y,
                        float* C, float* Gs, int B, int T, int H, int t) {
    switch (RT) {
        case 1: hipLaunchKernelGGL((lstm_fwd_step<G, 1>), grid, dim3(256), 0, st, Gx, Whh, Y, C, Gs, B, T, H, t); break;
        case 2: hipLaunchKernelGGL((lstm_fwd_step<G, 2>), grid, dim3(256), 0, st, Gx, Whh, Y, C, Gs, B, T, H, t); break;
        case 3: hipLaunchKernelGGL((lstm_fwd_step<G, 3>), grid, dim3(256), 0, st, Gx, Whh, Y, C, Gs, B, T, H, t); break;
        default: hipLaunchKernelGGL((lstm_fwd_step<G, 4>), grid, dim3(256), 0, st, Gx, Whh, Y, C, Gs, B, T, H, t); break;
    }
}
static void fwd_step(int G, int RT, dim3 grid, hipStream_t st, const float* Gx, const float* Whh, float* Y,
                     float* C, float* Gs, int B, int T, int H, int t) {
    if (G <= 1) fwd_step_rt<1>(RT, grid, st, Gx, Whh, Y, C, Gs, B, T, H, t);
    else if (G <= 2) fwd_step_rt<2>(RT, grid, st, Gx, Whh, Y, C, Gs, B, T, H, t);
    else if (G <= 4) fwd_step_rt<4>(RT, grid, st, Gx, Whh, Y, C, Gs, B, T, H, t);
    else if (G <= 8) fwd_step_rt<8>(RT, grid, st, Gx, Whh, Y, C, Gs, B, T, H, t);
    else fwd_step_rt<16>(RT, grid, st, Gx, Whh, Y, C, Gs, B, T, H, t);
}
template <int G>
static void bwd_gemm_rt(int RT, dim3 grid, hipStream_t st, const float* DA, const float* WhhT, float* P, int B,
                        int T, int H, int t, int gper) {
    switch (RT) {
        case 1: hipLaunchKernelGGL((lstm_bwd_gemm<G, 1>), grid, dim3(256), 0, st, DA, WhhT, P, B, T, H, t, gper); break;
        case 2: hipLaunchKernelGGL((lstm_bwd_gemm<G, 2>), grid, dim3(256), 0, st, DA, WhhT, P, B, T, H, t, gper); break;
        case 3: hipLaunchKernelGGL((lstm_bwd_gemm<G, 3>), grid, dim3(256), 0, st, DA, WhhT, P, B, T, H, t, gper); break;
        default: hipLaunchKernelGGL((lstm_bwd_gemm<G, 4>), grid, dim3(256), 0, st, DA, WhhT, P, B, T, H, t, gper); break;
    }
}
static void bwd_gemm(int G, int RT, dim3 grid, hipStream_t st, const float* DA, const float* WhhT, float* P, int B,
                     int T, int H, int t, int gper) {
    if (G <= 1) bwd_gemm_rt<1>(RT, grid, st, DA, WhhT, P, B, T, H, t, gper);
    else if (G <= 2) bwd_gemm_rt<2>(RT, grid, st, DA, WhhT, P, B, T, H, t, gper);
    else if (G <= 4) bwd_gemm_rt<4>(RT, grid, st, DA, WhhT, P, B, T, H, t, gper);
    else bwd_gemm_rt<8>(RT, grid, st, DA, WhhT, P, B, T, H, t, gper);
}
// k-splits of the recurrent backward GEMM: <= 8, dividing the H/4 k-groups, >= 4 groups each
static int bwd_splits(int64_t H) {
    const int groups = (int)(H / 4);
    int ns = groups / 4 < 8 ? groups / 4 : 8;
    if (ns < 1) ns = 1;
    while (groups % ns) --ns;
    return ns;
}

// ------------------------------------------------------------------------- GEMM operands
// X operand of a layer: layer 0 reads the conv layout [B][C][T]; deeper layers [B][T][H]
struct XRows {
    const float* p;
    int bct, C, T;
    ENCX_DEV float at(int m, int c) const {
        if (bct) {
            const int b = m / T, t = m - b * T;
            return p[((int64_t)b * C + c) * T + t];
        }
        return p[(int64_t)m * C + c];
    }
};
struct LdProj {  // Gx[m][j] = sum_c X(m, c) W_ih[j][c]
    static constexpr bool A_K_FAST = false, B_N_FAST = false;
    XRows x;
    const float* w;
    int C;
    ENCX_DEV float a(int m, int k) const { return x.at(m, k); }
    ENCX_DEV float b(int k, int n) const { return w[(int64_t)n * C + k]; }
};
struct EpProj {
    float* out;
    const float* bih;
    const float* bhh;
    int N;
    ENCX_DEV void operator()(int m, int n, float v) const {
        out[(int64_t)m * N + n] = v + (bih[n] + bhh[n]);
    }
};
// dW_hh[j][u] (u < H) and db[j] (u == H): sum_m DA[m][j] * h_{t-1}(m, u)
struct LdWhh {
    static constexpr bool A_K_FAST = false, B_N_FAST = true;
    const float* DA;
    const float* Y;
    int H, T;
    ENCX_DEV float a(int j, int m) const { return DA[(int64_t)m * 4 * H + j]; }
    ENCX_DEV float b(int m, int u) const {
        if (u == H) return 1.f;
        const int t = m % T;
        return t > 0 ? Y[(int64_t)(m - 1) * H + u] : 0.f;
    }
};
struct LdWih {  // dW_ih[j][c] = sum_m DA[m][j] X(m, c)
    static constexpr bool A_K_FAST = false, B_N_FAST = false;
    const float* DA;
    XRows x;
    int H;
    ENCX_DEV float a(int j, int m) const { return DA[(int64_t)m * 4 * H + j]; }
    ENCX_DEV float b(int m, int c) const { return x.at(m, c); }
};
struct EpSlabs {  // split-K partial slabs [z][M][N]
    float* ws;
    int M, N;
    ENCX_DEV void operator()(int m, int n, float v) const {
        ws[((int64_t)blockIdx.z * M + m) * N + n] = v;
    }
};
struct LdDX {  // dX(m, c) = sum_j DA[m][j] W_ih[j][c]
    static constexpr bool A_K_FAST = true, B_N_FAST = true;
    const float* DA;
    const float* w;
    int H, C;
    ENCX_DEV float a(int m, int j) const { return DA[(int64_t)m * 4 * H + j]; }
    ENCX_DEV float b(int j, int c) const { return w[(int64_t)j * C + c]; }
};
struct EpDX {  // to [B][C][T] (+ accumulate) or [B][T][C]
    float* out;
    int bct, C, T, acc;
    ENCX_DEV void operator()(int m, int c, float v) const {
        int64_t o;
        if (bct) {
            const int b = m / T, t = m - b * T;
            o = ((int64_t)b * C + c) * T + t;
        } else {
            o = (int64_t)m * C + c;
        }
        out[o] = acc ? out[o] + v : v;
    }
};

// sum split slabs [S][M][N] into dw[M][Nw] (+= when acc); a column n == Nw (the ones column
// of the dW_hh GEMM) is the bias grad, written to both bias vectors
__global__ void slab_reduce(const float* ws, int S, int M, int N, int Nw, float* dw, float* db1,
                            float* db2, int acc) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (int64_t)M * N) return;
    float s = 0.f;
    for (int z = 0; z < S; ++z) s += ws[(int64_t)z * M * N + i];
    const int m = (int)(i / N), n = (int)(i - (int64_t)m * N);
    if (n < Nw) {
        float* p = dw + (int64_t)m * Nw + n;
        *p = acc ? *p + s : s;
    } else {
        if (db1) db1[m] = acc ? db1[m] + s : s;
        if (db2) db2[m] = acc ? db2[m] + s : s;
    }
}

// final layer: out[b][u][t] = Y[b][t][u] + x[b][u][t] (lstm.py:24-27 skip, back to [B][C][T])
__global__ void lstm_out_skip(const float* Y, const float* x, float* out, int B, int T, int H) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (int64_t)B * H * T) return;
    const int t = (int)(i % T);
    const int64_t bu = i / T;
    const int b = (int)(bu / H), u = (int)(bu - (int64_t)b * H);
    out[i] = Y[((int64_t)b * T + t) * H + u] + x[i];
}
// dY_last[b][t][u] = dout[b][u][t]
__global__ void lstm_dout_t(const float* dout, float* dY, int B, int T, int H) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (int64_t)B * H * T) return;
    const int t = (int)(i % T);
    const int64_t bu = i / T;
    const int b = (int)(bu / H), u = (int)(bu - (int64_t)b * H);
    dY[((int64_t)b * T + t) * H + u] = dout[i];
}

}  // namespace

extern "C" {

/* One layer forward. x: layer input ([B][C][T] if x_bct else [B][T][C]); W_ih [4H][C],
 * W_hh [4H][H]; outputs Y, Cst [B][T][H] and gate activations Gs [B][T][4H]; Gx: [B*T][4H]
 * scratch. */
int encx_lstm_layer_fwd(const float* x, int x_bct, const float* w_ih, const float* w_hh,
                        const float* b_ih, const float* b_hh, float* Gx, float* Y, float* Cst,
                        float* Gs, int64_t B, int64_t T, int64_t C, int64_t H, encx_stream_t stream) {
    ENCX_REQUIRE(x && w_ih && w_hh && b_ih && b_hh && Gx && Y && Cst && Gs);
    ENCX_REQUIRE(B > 0 && B <= 64 && T > 0 && H > 0 && (H % 16) == 0 && H <= 1024 && C > 0);
    hipStream_t st = (hipStream_t)stream;
    const int M = (int)(B * T), N = (int)(4 * H);
    int rc = gemm_launch(LdProj{XRows{x, x_bct, (int)C, (int)T}, w_ih, (int)C},
                         EpProj{Gx, b_ih, b_hh, N}, M, N, (int)C, st);
    if (rc) return rc;
    const int RT = (int)cdiv(B, 16), G = (int)cdiv(H / 16, 4);
    for (int t = 0; t < T; ++t)
        fwd_step(G, RT, dim3((unsigned)cdiv(H, UNITS)), st, Gx, w_hh, Y, Cst, Gs, (int)B, (int)T, (int)H, t);
    ENCX_CHECK_LAUNCH();
    return 0;
}

size_t encx_lstm_bwd_workspace(int64_t B, int64_t T, int64_t C, int64_t H) {
    const int M = (int)(B * T), N4 = (int)(4 * H);
    const int s1 = gemm_slabs(M, gemm_splits(N4, (int)H + 1, M));
    const int s2 = gemm_slabs(M, gemm_splits(N4, (int)C, M));
    size_t a = (size_t)s1 * N4 * (H + 1), b = (size_t)s2 * N4 * C;
    return ((a > b ? a : b) + B * H + 4 * H * H + (size_t)bwd_splits(H) * B * H) * sizeof(float);
}

/* One layer backward. dY [B][T][H] (the grad of this layer's output sequence), states from
 * the forward; writes DA [B][T][4H] scratch, dW_ih, dW_hh, db (added to BOTH b_ih and b_hh
 * grads) with `acc_w` (1: accumulate into existing grads), dx ([B][C][T] if x_bct, then
 * accumulated when acc_x, else [B][T][C]). ws: encx_lstm_bwd_workspace bytes. */
int encx_lstm_layer_bwd(const float* x, int x_bct, const float* w_ih, const float* w_hh,
                        const float* Y, const float* Cst, const float* Gs, const float* dY,
                        float* DA, float* dx, int acc_x, float* dw_ih, float* dw_hh,
                        float* db_ih, float* db_hh, int acc_w, float* ws, int64_t B, int64_t T,
                        int64_t C, int64_t H, encx_stream_t stream) {
    ENCX_REQUIRE(x && w_ih && w_hh && Y && Cst && Gs && dY && DA && ws);
    ENCX_REQUIRE(B > 0 && B <= 64 && T > 0 && H > 0 && (H % 16) == 0 && H <= 512);
    hipStream_t st = (hipStream_t)stream;
    const int M = (int)(B * T), N4 = (int)(4 * H);
    float* dcn = ws;
    float* whhT = ws + B * H;
    float* P = whhT + 4 * H * H;
    const int ns = bwd_splits(H);
    float* slabs = P + (int64_t)ns * B * H;
    hipLaunchKernelGGL(transpose_kernel, dim3((unsigned)cdiv(H, 32), (unsigned)cdiv(4 * H, 32)), dim3(32, 8), 0, st,
                       w_hh, whhT, (int)(4 * H), (int)H);
    const int RT = (int)cdiv(B, 16), gper = (int)(H / 4) / ns, G = (int)cdiv(gper, 4);
    const int BH = (int)(B * H);
    for (int t = (int)T - 1; t >= 0; --t) {
        hipLaunchKernelGGL(lstm_bwd_elem, dim3((unsigned)cdiv(BH, 256)), dim3(256), 0, st, dY, P, ns, dcn, Cst, Gs,
                           DA, (int)B, (int)T, (int)H, t);
        if (t > 0)
            bwd_gemm(G, RT, dim3((unsigned)(H / 16), (unsigned)ns), st, DA, whhT, P, (int)B, (int)T, (int)H, t, gper);
    }
    ENCX_CHECK_LAUNCH();
    int rc;
    if (dw_hh) {
        const int sp = gemm_splits(N4, (int)H + 1, M);
        const int S = gemm_slabs(M, sp);
        rc = gemm_launch(LdWhh{DA, Y, (int)H, (int)T}, EpSlabs{slabs, N4, (int)H + 1}, N4, (int)H + 1, M,
                         st, sp);
        if (rc) return rc;
        hipLaunchKernelGGL(slab_reduce, dim3(cdiv((int64_t)N4 * (H + 1), 256)), dim3(256), 0, st, slabs,
                           S, N4, (int)H + 1, (int)H, dw_hh, db_ih, db_hh, acc_w);
        ENCX_CHECK_LAUNCH();
    }
    if (dw_ih) {
        const int sp = gemm_splits(N4, (int)C, M);
        const int S = gemm_slabs(M, sp);
        rc = gemm_launch(LdWih{DA, XRows{x, x_bct, (int)C, (int)T}, (int)H}, EpSlabs{slabs, N4, (int)C},
                         N4, (int)C, M, st, sp);
        if (rc) return rc;
        hipLaunchKernelGGL(slab_reduce, dim3(cdiv((int64_t)N4 * C, 256)), dim3(256), 0, st, slabs, S, N4,
                           (int)C, (int)C, dw_ih, (float*)nullptr, (float*)nullptr, acc_w);
        ENCX_CHECK_LAUNCH();
    }
    if (dx) {
        rc = gemm_launch(LdDX{DA, w_ih, (int)H, (int)C}, EpDX{dx, x_bct, (int)C, (int)T, acc_x}, M, (int)C,
                         N4, st);
        if (rc) return rc;
    }
    return 0;
}

int encx_lstm_out_skip(const float* Y, const float* x, float* out, int64_t B, int64_t T, int64_t H,
                       encx_stream_t stream) {
    ENCX_REQUIRE(Y && x && out);
    const int64_t n = B * H * T;
    hipLaunchKernelGGL(lstm_out_skip, dim3(cdiv(n, 256)), dim3(256), 0, (hipStream_t)stream, Y, x, out,
                       (int)B, (int)T, (int)H);
    ENCX_CHECK_LAUNCH();
    return 0;
}

int encx_lstm_dout_t(const float* dout, float* dY, int64_t B, int64_t T, int64_t H,
                     encx_stream_t stream) {
    ENCX_REQUIRE(dout && dY);
    const int64_t n = B * H * T;
    hipLaunchKernelGGL(lstm_dout_t, dim3(cdiv(n, 256)), dim3(256), 0, (hipStream_t)stream, dout, dY,
                       (int)B, (int)T, (int)H);
    ENCX_CHECK_LAUNCH();
    return 0;
}

}  // extern "C"
