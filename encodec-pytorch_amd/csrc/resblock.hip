// Fused SEANet residual block for the high-rate stages (modules/seanet.py:21-63 with the EnCodec
// defaults: kernel_sizes [3, 1], dilations [1, 1], compress 2, true_skip False, causal reflect
// padding, weight_norm):
//     y = Ws x + bs  +  W2 ELU(h) + b2,    h = W1 * ELU(xpad) + b1  (k3, causal, reflect pad 2)
// At T = 24000 / 12000 (C = 32 / 64) the three convs are HBM-bound one by one: the unfused
// forward reads x twice and writes / re-reads the shortcut and the hidden tensor, the backward
// moves dy, x, h and their grads through HBM six times. Three kernels, each over 64-position
// tiles held in LDS (persistent grids):
//   rb_fwd   : x tile (+2 left halo) -> h (k3 GEMM) -> y ([ELU(h) | x] x [W2 | Ws] GEMM);
//              reads x once, writes y and h (the backward's saved tensor);
//   rb_dgrad : dy tile (+2 right halo) -> dh = (W2^T dy) ELU'(h) -> dx = Ws^T dy + ELU'(x) (W1^T * dh)
//              (the reflect pad folded back at t = 1, 2); writes dx and dh;
//   rb_wgrad : dy, dh, x, h tiles -> dWs = dy x^T, dW2 = dy ELU(h)^T, dW1[k] = dh ELU(x)_{+k}^T and
//              the bias sums, accumulated in registers over the workgroup's tiles, stored once per
//              workgroup as a slab and summed in a fixed order by rb_wgrad_reduce.
// The data-grad and weight-grad halves are separate kernels because their GEMMs read the tiles
// along different axes: position-major (16x16x4, 16 positions x 4 channels per wave read) wants
// LDS rows 16 banks apart, channel-major (32x32x2, 32 channels x 1 position) wants an odd row
// stride; one kernel holding every tile in both layouts would not fit two workgroups per CU.
// Weights live in VGPRs as MFMA B fragments (loaded once per workgroup), so the only LDS reads in
// the inner loops are conflict-free A / B tile reads. Each workgroup loads its next tile into
// registers (buffer loads) while the current one computes (config-3 step: 778 vs 766 audio-s/s
// over staging each tile just in time, profiles/r05/bench_ab_variants.txt).
// MFMA: v_mfma_f32_16x16x4_f32 (lane l: A[l&15][k=l>>4], B[k=l>>4][l&15], D[row 4(l>>4)+i][col l&15])
// and v_mfma_f32_32x32x2_f32 (common.h), exact fp32 products.
#include "common.h"
#include "prof.h"

namespace {

typedef float f32x4v __attribute__((ext_vector_type(4)));
ENCX_DEV f32x4v mfma16(float a, float b, f32x4v c) { return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0); }

constexpr int TT = 64;        // positions per tile
constexpr int XF = 80;        // position-major row stride (== 16 mod 32: lanes lk = 0 / 1 on disjoint banks)
constexpr int XW = 67;        // channel-major row stride (odd: 32 rows on 32 distinct banks)

template <int C>
struct Rb {
    static constexpr int HD = C / 2;
    static constexpr int CG = C == 64 ? 2 : 1;  // column groups: waves per 16-position strip
    static constexpr int NT = 256 * CG;         // threads of rb_fwd / rb_dgrad
    static constexpr int SLAB = C * C + C * HD + HD * 3 * C + C + HD;
};

struct RbArgs {
    const float* x;   // [B][C][T]
    const float* w1;  // [C][3][HD]   k3 conv, wf layout (encx weight prep: [Cin][K][Cout])
    const float* b1;  // [HD]
    const float* w2;  // [HD][C]      1x1 conv HD -> C, wf layout
    const float* b2;  // [C]
    const float* ws;  // [C][C]       shortcut 1x1, wf layout
    const float* bs;  // [C]
    float* h;         // [B][HD][T]   forward: written (pre-ELU); backward: read
    float* y;         // [B][C][T]    forward output
    const float* dy;  // [B][C][T]    backward input
    float* dx;        // [B][C][T]    backward output
    float* dh;        // [B][HD][T]   rb_dgrad: written; rb_wgrad: read
    float* slab;      // [grid][Rb::SLAB] weight-grad partials
    int B, T, NT;     // NT = tiles per batch item
};

// store 4 consecutive positions t .. t+3 of row `row` (bounded by T)
ENCX_DEV void st4(float* row, int t, int T, f32x4v v) {
    if (t + 4 <= T) {
        *(f32x4u*)(row + t) = (f32x4u){v[0], v[1], v[2], v[3]};
    } else {
#pragma unroll
        for (int i = 0; i < 4; ++i)
            if (t + i < T) row[t + i] = v[i];
    }
}
// load 4 consecutive positions (0 past T)
ENCX_DEV f32x4v ld4(const float* row, int t, int T) {
    if (t + 4 <= T) return ld4u(row + t);
    f32x4v v;
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = t + i < T ? row[t + i] : 0.f;
    return v;
}
ENCX_DEV int reflect_clamp(int t, int T) { return t < 0 ? -t : (t < T ? t : T - 1); }
// Tile staging loads as buffer loads: one 32-bit per-lane byte offset and a uniform (SGPR) row
// offset per load, instead of a 64-bit address per load held across the loop.
typedef __amdgpu_buffer_rsrc_t rsrc_t;
ENCX_DEV rsrc_t rsrc(const float* base, int64_t n) {
    return __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, (int)(n * sizeof(float)), 0x00020000);
}
ENCX_DEV float bload(rsrc_t r, int voff, int soff) {
    return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, voff, soff, 0));
}

// ------------------------------------------------------------------------------------ forward
// Wave (strip s = wv & 3, group g = wv >> 2): positions 16 s .. 16 s + 15 of the tile, h columns
// g * HD / CG .., y columns g * C / CG ..
template <int C>
__global__ __launch_bounds__(Rb<C>::NT) void rb_fwd_kernel(RbArgs a) {
    constexpr int HD = C / 2, CG = Rb<C>::CG, NT = Rb<C>::NT, N1 = HD / 16 / CG, N2 = C / 16 / CG;
    extern __shared__ float sm[];
    float* xs = sm;           // [C][XF]: x at t0 - 2 + p
    float* es = xs + C * XF;  // ELU(xs)
    float* hs = es + C * XF;  // [HD][XF]: ELU(h) at t0 + p
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, lc = lane & 15, lk = lane >> 4;
    const int m0 = 16 * (wv & 3), g = wv >> 2;
    float bw1[3][C / 4][N1], bw2[HD / 4][N2], bws[C / 4][N2], b1v[N1], bov[N2];
#pragma unroll
    for (int n = 0; n < N1; ++n) {
        const int j = (g * N1 + n) * 16 + lc;
        b1v[n] = a.b1[j];
#pragma unroll
        for (int k = 0; k < 3; ++k)
#pragma unroll
            for (int c4 = 0; c4 < C / 4; ++c4) bw1[k][c4][n] = a.w1[((4 * c4 + lk) * 3 + k) * HD + j];
    }
#pragma unroll
    for (int n = 0; n < N2; ++n) {
        const int o = (g * N2 + n) * 16 + lc;
        bov[n] = a.b2[o] + a.bs[o];
#pragma unroll
        for (int j4 = 0; j4 < HD / 4; ++j4) bw2[j4][n] = a.w2[(4 * j4 + lk) * C + o];
#pragma unroll
        for (int c4 = 0; c4 < C / 4; ++c4) bws[c4][n] = a.ws[(4 * c4 + lk) * C + o];
    }
    const int T = a.T, ntiles = a.B * a.NT;
    // the next tile's x in registers, loaded while the current tile computes: rows wv + NW u at
    // positions lane (p < TT), and the last two halo columns p = TT, TT + 1 (threads < 2 C)
    constexpr int NW = NT / 64, PR = C / NW;
    float pf[PR], pfh = 0.f;
    const int hc = tid >> 1, hp = TT + (tid & 1);
    auto fetch = [&](int tile) {
        const int b = tile / a.NT, t0 = (tile - b * a.NT) * TT;
        const rsrc_t rx = rsrc(a.x + (int64_t)b * C * T, (int64_t)C * T);
        const int vo = (wv * T + reflect_clamp(t0 - 2 + lane, T)) * 4;  // past T: unused
#pragma unroll
        for (int u = 0; u < PR; ++u) pf[u] = bload(rx, vo, u * NW * T * 4);
        if (tid < 2 * C) pfh = bload(rx, (hc * T + reflect_clamp(t0 - 2 + hp, T)) * 4, 0);
    };
    if ((int)blockIdx.x < ntiles) fetch(blockIdx.x);
    for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        const int b = tile / a.NT, t0 = (tile - b * a.NT) * TT;
        __syncthreads();  // the previous tile's LDS reads are done
#pragma unroll
        for (int u = 0; u < PR; ++u) {
            xs[(wv + NW * u) * XF + lane] = pf[u];
            es[(wv + NW * u) * XF + lane] = elu(pf[u]);
        }
        if (tid < 2 * C) {
            xs[hc * XF + hp] = pfh;
            es[hc * XF + hp] = elu(pfh);
        }
        __syncthreads();
        if (tile + (int)gridDim.x < ntiles) fetch(tile + gridDim.x);
        // h^T[m][j] = b1[j] + sum_{c,k} ELU(x)[c][t - 2 + k] W1[c][k][j]   (rows = positions)
        f32x4v acc1[N1];
#pragma unroll
        for (int n = 0; n < N1; ++n) acc1[n] = (f32x4v){0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int k = 0; k < 3; ++k)
#pragma unroll
            for (int c4 = 0; c4 < C / 4; ++c4) {
                const float av = es[(4 * c4 + lk) * XF + m0 + lc + k];
#pragma unroll
                for (int n = 0; n < N1; ++n) acc1[n] = mfma16(av, bw1[k][c4][n], acc1[n]);
            }
        const int tq = t0 + m0 + 4 * lk;  // this lane's 4 positions
#pragma unroll
        for (int n = 0; n < N1; ++n) {
            const int j = (g * N1 + n) * 16 + lc;
            f32x4v hv, ev;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                hv[i] = acc1[n][i] + b1v[n];
                ev[i] = elu(hv[i]);
            }
            *(f32x4v*)(hs + j * XF + m0 + 4 * lk) = ev;
            if (a.h) st4(a.h + ((int64_t)b * HD + j) * T, tq, T, hv);
        }
        __syncthreads();  // the other column group's h rows
        // y^T[m][o] = (b2 + bs)[o] + sum_j ELU(h)[j][m] W2[j][o] + sum_c x[c][m] Ws[c][o]
        f32x4v acc2[N2];
#pragma unroll
        for (int n = 0; n < N2; ++n) acc2[n] = (f32x4v){0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int j4 = 0; j4 < HD / 4; ++j4) {
            const float av = hs[(4 * j4 + lk) * XF + m0 + lc];
#pragma unroll
            for (int n = 0; n < N2; ++n) acc2[n] = mfma16(av, bw2[j4][n], acc2[n]);
        }
#pragma unroll
        for (int c4 = 0; c4 < C / 4; ++c4) {
            const float av = xs[(4 * c4 + lk) * XF + m0 + lc + 2];
#pragma unroll
            for (int n = 0; n < N2; ++n) acc2[n] = mfma16(av, bws[c4][n], acc2[n]);
        }
#pragma unroll
        for (int n = 0; n < N2; ++n) {
            const int o = (g * N2 + n) * 16 + lc;
            st4(a.y + ((int64_t)b * C + o) * T, tq, T, acc2[n] + bov[n]);
        }
    }
}

// ---------------------------------------------------------------------------- backward: data
// Wave (strip, group) as in the forward: dh columns g * HD / CG .., dx columns g * C / CG ..
// The right-halo dh (positions TT, TT + 1, read by the k3 transpose of the last positions) on
// the vector ALU: TPO threads per (j, p), C / TPO terms each, summed by lane shuffles.
template <int C>
__global__ __launch_bounds__(Rb<C>::NT) void rb_dgrad_kernel(RbArgs a) {
    constexpr int HD = C / 2, CG = Rb<C>::CG, NT = Rb<C>::NT, NH = HD / 16 / CG, NX = C / 16 / CG;
    constexpr int TPO = NT / (2 * HD), U = C / TPO;
    static_assert(TPO == 8, "halo reduction assumes 8 lanes per output");
    extern __shared__ float sm[];
    float* dys = sm;            // [C][XF]: dy at t0 + p, p < TT + 2 (0 past T)
    float* dhs = dys + C * XF;  // [HD][XF]: dh at t0 + p (0 past T)
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, lc = lane & 15, lk = lane >> 4;
    const int m0 = 16 * (wv & 3), g = wv >> 2;
    float bh[C / 4][NH], bs[C / 4][NX], b3[3][HD / 4][NX];
#pragma unroll
    for (int n = 0; n < NH; ++n) {  // B[k = o][n = j] = W2[j][o]
        const int j = (g * NH + n) * 16 + lc;
#pragma unroll
        for (int o4 = 0; o4 < C / 4; ++o4) bh[o4][n] = a.w2[j * C + 4 * o4 + lk];
    }
#pragma unroll
    for (int n = 0; n < NX; ++n) {  // B[k = o][n = c] = Ws[c][o];  B[k = j][n = c] = W1[c][k][j]
        const int c = (g * NX + n) * 16 + lc;
#pragma unroll
        for (int o4 = 0; o4 < C / 4; ++o4) bs[o4][n] = a.ws[c * C + 4 * o4 + lk];
#pragma unroll
        for (int k = 0; k < 3; ++k)
#pragma unroll
            for (int j4 = 0; j4 < HD / 4; ++j4) b3[k][j4][n] = a.w1[(c * 3 + k) * HD + 4 * j4 + lk];
    }
    const int hq = tid / TPO, hr = tid - hq * TPO, hj = hq >> 1, hp = TT + (hq & 1);
    float hw[U];
#pragma unroll
    for (int u = 0; u < U; ++u) hw[u] = a.w2[hj * C + hr * U + u];
    const int T = a.T, ntiles = a.B * a.NT;
    // the next tile's dy (rows wv + NW u at positions lane, halo columns TT, TT + 1 by threads
    // < 2 C; 0 past T) and the h / x values of the epilogues, in registers, loaded while the
    // current tile computes
    constexpr int NW = NT / 64, PR = C / NW;
    float pf[PR], pfh = 0.f, hh = 0.f;
    const int hc = tid >> 1, hpp = TT + (tid & 1);
    f32x4v hv[NH], xv[NX];
    auto fetch = [&](int tile) {
        const int b = tile / a.NT, t0 = (tile - b * a.NT) * TT, t = t0 + lane;
        const rsrc_t rdy = rsrc(a.dy + (int64_t)b * C * T, (int64_t)C * T);
        const int vo = (wv * T + (t < T ? t : T - 1)) * 4;
#pragma unroll
        for (int u = 0; u < PR; ++u) {
            const float v = bload(rdy, vo, u * NW * T * 4);
            pf[u] = t < T ? v : 0.f;
        }
        if (tid < 2 * C) {
            const int th = t0 + hpp;
            const float v = bload(rdy, (hc * T + (th < T ? th : T - 1)) * 4, 0);
            pfh = th < T ? v : 0.f;
        }
        const int tq = t0 + m0 + 4 * lk;
#pragma unroll
        for (int n = 0; n < NH; ++n) hv[n] = ld4(a.h + ((int64_t)b * HD + (g * NH + n) * 16 + lc) * T, tq, T);
#pragma unroll
        for (int n = 0; n < NX; ++n) xv[n] = ld4(a.x + ((int64_t)b * C + (g * NX + n) * 16 + lc) * T, tq, T);
        const int th = t0 + hp;
        hh = a.h[((int64_t)b * HD + hj) * T + (th < T ? th : T - 1)];
    };
    if ((int)blockIdx.x < ntiles) fetch(blockIdx.x);
    for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        const int b = tile / a.NT, t0 = (tile - b * a.NT) * TT;
        __syncthreads();
#pragma unroll
        for (int u = 0; u < PR; ++u) dys[(wv + NW * u) * XF + lane] = pf[u];
        if (tid < 2 * C) dys[hc * XF + hpp] = pfh;
        __syncthreads();
        const int tq = t0 + m0 + 4 * lk;
        f32x4v hcur[NH], xcur[NX];
#pragma unroll
        for (int n = 0; n < NH; ++n) hcur[n] = hv[n];
#pragma unroll
        for (int n = 0; n < NX; ++n) xcur[n] = xv[n];
        const float hhcur = hh;
        if (tile + (int)gridDim.x < ntiles) fetch(tile + gridDim.x);
        // ---- dh^T[p][j] = ELU'(h) * sum_o dy[o][p] W2[j][o] for p < TT ...
        {
            f32x4v acc[NH];
#pragma unroll
            for (int n = 0; n < NH; ++n) acc[n] = (f32x4v){0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int o4 = 0; o4 < C / 4; ++o4) {
                const float av = dys[(4 * o4 + lk) * XF + m0 + lc];
#pragma unroll
                for (int n = 0; n < NH; ++n) acc[n] = mfma16(av, bh[o4][n], acc[n]);
            }
#pragma unroll
            for (int n = 0; n < NH; ++n) {
                const int j = (g * NH + n) * 16 + lc;
                f32x4v d;
#pragma unroll
                for (int i = 0; i < 4; ++i) d[i] = tq + i < T ? acc[n][i] * elu_grad(hcur[n][i]) : 0.f;
                *(f32x4v*)(dhs + j * XF + m0 + 4 * lk) = d;
                st4(a.dh + ((int64_t)b * HD + j) * T, tq, T, d);
            }
        }
        // ... and the right halo TT, TT + 1
        {
            float s = 0.f;
#pragma unroll
            for (int u = 0; u < U; ++u) s = fmaf(dys[(hr * U + u) * XF + hp], hw[u], s);
            s += __shfl_xor(s, 4, 64);
            s += __shfl_xor(s, 2, 64);
            s += __shfl_xor(s, 1, 64);
            if (hr == 0) {
                const int t = t0 + hp;
                dhs[hj * XF + hp] = t < T ? s * elu_grad(hhcur) : 0.f;
            }
        }
        __syncthreads();
        // ---- dx^T[m][c] = sum_o dy[o][m] Ws[c][o] + ELU'(x[c][m]) * sum_{j,k} dh[j][m + 2 - k] W1[c][k][j]
        f32x4v asc[NX], ak3[NX];
#pragma unroll
        for (int n = 0; n < NX; ++n) asc[n] = ak3[n] = (f32x4v){0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int o4 = 0; o4 < C / 4; ++o4) {
            const float av = dys[(4 * o4 + lk) * XF + m0 + lc];
#pragma unroll
            for (int n = 0; n < NX; ++n) asc[n] = mfma16(av, bs[o4][n], asc[n]);
        }
#pragma unroll
        for (int k = 0; k < 3; ++k)
#pragma unroll
            for (int j4 = 0; j4 < HD / 4; ++j4) {
                const float av = dhs[(4 * j4 + lk) * XF + m0 + lc + 2 - k];
#pragma unroll
                for (int n = 0; n < NX; ++n) ak3[n] = mfma16(av, b3[k][j4][n], ak3[n]);
            }
        // reflect pad: ELU(x) at t = -1, -2 is ELU(x[1]), ELU(x[2]); their grads fold into t = 1, 2
        if (t0 == 0 && m0 == 0 && lk == 0) {
#pragma unroll
            for (int n = 0; n < NX; ++n) {
                const int c = (g * NX + n) * 16 + lc;
                float v1 = 0.f, v2 = 0.f;
#pragma unroll 1
                for (int j = 0; j < HD; ++j) {
                    const float w0 = a.w1[(c * 3) * HD + j], w1v = a.w1[(c * 3 + 1) * HD + j];
                    v1 = fmaf(w0, dhs[j * XF + 1], fmaf(w1v, dhs[j * XF + 0], v1));
                    v2 = fmaf(w0, dhs[j * XF + 0], v2);
                }
                ak3[n][1] += v1;
                ak3[n][2] += v2;
            }
        }
#pragma unroll
        for (int n = 0; n < NX; ++n) {
            const int c = (g * NX + n) * 16 + lc;
            f32x4v v;
#pragma unroll
            for (int i = 0; i < 4; ++i) v[i] = asc[n][i] + elu_grad(xcur[n][i]) * ak3[n][i];
            st4(a.dx + ((int64_t)b * C + c) * T, tq, T, v);
        }
    }
}

// -------------------------------------------------------------------------- backward: weights
// One 32 x 32 output tile of a weight grad, K = the tile's positions: acc += A[m][q] B[q][n] with
// A rows / B rows read channel-major from LDS (lane l: row l & 31 at position q + (l >> 5)).
struct WTile {
    const float* bp;  // this lane's B row pointer (incl. the position shift)
    int kind;         // 0 dWs[o][c], 1 dW2[o][j], 2 dW1[j][c][k]
    int ro, co, k;    // tile origin (rows, columns), tap
};

template <int NTL>
ENCX_DEV void wgemm(const float* ap, const WTile* t, f32x16* acc) {
#pragma unroll 4
    for (int q = 0; q < TT; q += 2) {
        const float av = ap[q];
#pragma unroll
        for (int i = 0; i < NTL; ++i) acc[i] = mfma32(av, t[i].bp[q], acc[i]);
    }
}

// waves: C = 64 -- w0 / w1: A = dy rows 0-31 / 32-63 x {x rows 0-31, x rows 32-63, ELU(h)}
// (dWs, dW2); w2 / w3: A = dh x ELU(x) rows {0-31, 32-63} at taps {0, 0, 1} / {1, 2, 2} (dW1).
// C = 32 -- w0: A = dy x {x, ELU(h)}; w1..w3: A = dh x ELU(x) at tap w - 1 (16-row operands
// read twice, the duplicate rows / columns of the tile dropped at the store).
template <int C>
__global__ __launch_bounds__(256) void rb_wgrad_kernel(RbArgs a) {
    constexpr int HD = C / 2, NTL = C == 64 ? 3 : 2;
    extern __shared__ float sm[];
    float* dys = sm;            // [C][XW]: dy at t0 + q (0 past T)
    float* dhs = dys + C * XW;  // [HD][XW]: dh at t0 + q (0 past T)
    float* hes = dhs + HD * XW; // [HD][XW]: ELU(h) at t0 + q
    float* xs = hes + HD * XW;  // [C][XW]: x at t0 - 2 + p (reflect)
    float* exs = xs + C * XW;   // ELU(xs)
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, lr = lane & 31, lq = lane >> 5;
    const int lh = lr & (HD - 1);  // row of a HD-row operand (C = 32: rows 16-31 repeat 0-15)
    const float* ap;
    WTile tl[NTL];
    int ntl = NTL;
    if (C == 64) {
        if (wv < 2) {
            ap = dys + (32 * wv + lr) * XW;
            tl[0] = {xs + lr * XW + 2, 0, 32 * wv, 0, 0};
            tl[1] = {xs + (32 + lr) * XW + 2, 0, 32 * wv, 32, 0};
            tl[2] = {hes + lh * XW, 1, 32 * wv, 0, 0};
        } else {
            ap = dhs + lh * XW;
#pragma unroll
            for (int i = 0; i < 3; ++i) {  // dW1 tile u = (tap u / 2, column half u % 2)
                const int u = 3 * (wv - 2) + i, k = u >> 1, co = 32 * (u & 1);
                tl[i] = {exs + (co + lr) * XW + k, 2, 0, co, k};
            }
        }
    } else {
        if (wv == 0) {
            ap = dys + lr * XW;
            tl[0] = {xs + lr * XW + 2, 0, 0, 0, 0};
            tl[1] = {hes + lh * XW, 1, 0, 0, 0};
        } else {
            ap = dhs + lh * XW;
            tl[0] = {exs + lr * XW + (wv - 1), 2, 0, 0, wv - 1};
            tl[1] = tl[0];
            ntl = 1;
        }
    }
    ap += lq;
#pragma unroll
    for (int i = 0; i < NTL; ++i) tl[i].bp += lq;
    f32x16 acc[NTL];
#pragma unroll
    for (int i = 0; i < NTL; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][r] = 0.f;
    const int T = a.T, ntiles = a.B * a.NT;
    // the next tile in registers, loaded while the current tile computes: dy, dh (0 past T), h,
    // x (reflect) as rows wv + 4 u at positions lane; x's last two halo columns by threads < 2 C
    constexpr int PD = C / 4, PH = HD / 4;
    float pd[PD], pdh[PH], ph[PH], px[PD], pxh = 0.f;
    float bacc[PD + PH];  // this lane's partial bias sums: dy rows wv + 4 u, then dh rows
#pragma unroll
    for (int u = 0; u < PD + PH; ++u) bacc[u] = 0.f;
    const int hc = tid >> 1, hp = TT + (tid & 1);
    auto fetch = [&](int tile) {
        const int b = tile / a.NT, t0 = (tile - b * a.NT) * TT, t = t0 + lane;
        const rsrc_t rdy = rsrc(a.dy + (int64_t)b * C * T, (int64_t)C * T);
        const rsrc_t rdh = rsrc(a.dh + (int64_t)b * HD * T, (int64_t)HD * T);
        const rsrc_t rh = rsrc(a.h + (int64_t)b * HD * T, (int64_t)HD * T);
        const rsrc_t rx = rsrc(a.x + (int64_t)b * C * T, (int64_t)C * T);
        const int vo = (wv * T + (t < T ? t : T - 1)) * 4, vx = (wv * T + reflect_clamp(t0 - 2 + lane, T)) * 4;
#pragma unroll
        for (int u = 0; u < PD; ++u) {
            const float v = bload(rdy, vo, u * 4 * T * 4);
            pd[u] = t < T ? v : 0.f;
            px[u] = bload(rx, vx, u * 4 * T * 4);
        }
#pragma unroll
        for (int u = 0; u < PH; ++u) {
            const float v = bload(rdh, vo, u * 4 * T * 4);
            pdh[u] = t < T ? v : 0.f;
            ph[u] = bload(rh, vo, u * 4 * T * 4);
        }
        if (tid < 2 * C) pxh = bload(rx, (hc * T + reflect_clamp(t0 - 2 + hp, T)) * 4, 0);
    };
    if ((int)blockIdx.x < ntiles) fetch(blockIdx.x);
    for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        __syncthreads();
#pragma unroll
        for (int u = 0; u < PD; ++u) {
            dys[(wv + 4 * u) * XW + lane] = pd[u];
            xs[(wv + 4 * u) * XW + lane] = px[u];
            exs[(wv + 4 * u) * XW + lane] = elu(px[u]);
            bacc[u] += pd[u];
        }
#pragma unroll
        for (int u = 0; u < PH; ++u) {
            dhs[(wv + 4 * u) * XW + lane] = pdh[u];
            hes[(wv + 4 * u) * XW + lane] = elu(ph[u]);
            bacc[PD + u] += pdh[u];
        }
        if (tid < 2 * C) {
            xs[hc * XW + hp] = pxh;
            exs[hc * XW + hp] = elu(pxh);
        }
        __syncthreads();
        if (tile + (int)gridDim.x < ntiles) fetch(tile + gridDim.x);
        if (C == 64 || ntl == NTL) wgemm<NTL>(ap, tl, acc);
        else wgemm<1>(ap, tl, acc);
    }
    // ---- this workgroup's partial weight grads -> slab [dWs C x C][dW2 C x HD][dW1 HD x C x 3][db C][db1 HD]
    // (natural layouts: dWs[o][c], dW2[o][j], dW1[j][c][k])
    float* sl = a.slab + (int64_t)blockIdx.x * Rb<C>::SLAB;
#pragma unroll
    for (int i = 0; i < NTL; ++i) {
        if (i >= ntl) break;
        const WTile& t = tl[i];
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int row = t.ro + mfma_row(r, lane), col = t.co + lr;
            if (t.kind == 0) sl[row * C + col] = acc[i][r];
            else if (t.kind == 1) {
                if (col < HD) sl[C * C + row * HD + col] = acc[i][r];
            } else if (row < HD) {
                sl[C * C + C * HD + (row * C + col) * 3 + t.k] = acc[i][r];
            }
        }
    }
#pragma unroll
    for (int u = 0; u < PD + PH; ++u) {  // db rows wv + 4 u, then db1 rows wv + 4 u
        const float v = wave_sum(bacc[u]);
        if (lane == 0) sl[C * C + C * HD + HD * 3 * C + (u < PD ? wv + 4 * u : C + wv + 4 * (u - PD))] = v;
    }
}

// out[i] (+)= sum_{g < G} slab[g][i] in ascending g (fp64 accumulation), for the slab's sections: dWs -> dws, dW2 ->
// dw2, dW1 -> dw1, db -> db2 and dbs (the same sum), db1 -> db1. Null outputs are skipped.
template <int C>
__global__ __launch_bounds__(256) void rb_wgrad_reduce(const float* slab, int G, float* dws, float* dw2, float* dw1,
                                                       float* db2, float* dbs, float* db1, int acc_w, int acc_b) {
    constexpr int HD = C / 2, S = Rb<C>::SLAB;
    __shared__ double red[256];
    const int64_t i = (int64_t)blockIdx.x * 64 + (threadIdx.x & 63);
    const bool valid = i < S;
    const float v = slab_sum_256_d(slab + (valid ? i : 0), G, S, valid, red);
    if (threadIdx.x >= 64 || !valid) return;
    auto put = [](float* p, float v, int acc) {
        if (p) *p = acc ? *p + v : v;
    };
    int k = (int)i;
    if (k < C * C) { put(dws ? dws + k : nullptr, v, acc_w); return; }
    k -= C * C;
    if (k < C * HD) { put(dw2 ? dw2 + k : nullptr, v, acc_w); return; }
    k -= C * HD;
    if (k < HD * 3 * C) { put(dw1 ? dw1 + k : nullptr, v, acc_w); return; }
    k -= HD * 3 * C;
    if (k < C) {
        put(db2 ? db2 + k : nullptr, v, acc_b);
        put(dbs ? dbs + k : nullptr, v, acc_b);
        return;
    }
    k -= C;
    put(db1 ? db1 + k : nullptr, v, acc_b);
}

size_t rb_fwd_lds(int C) { return (size_t)(2 * C + C / 2) * XF * sizeof(float); }
size_t rb_dgrad_lds(int C) { return (size_t)(C + C / 2) * XF * sizeof(float); }
size_t rb_wgrad_lds(int C) { return (size_t)(3 * C + C) * XW * sizeof(float); }

int num_cus() {
    static int n = 0;
    if (!n) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
            n = 256;
    }
    return n;
}
// persistent grid: whole rounds of the workgroups resident per CU (occupancy from the runtime,
// cached per kernel), at most one workgroup per tile
template <typename K>
int rb_grid(K kernel, int threads, size_t lds, int64_t tiles) {
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, threads, lds) != hipSuccess || per_cu < 1)
        per_cu = 1;
    const int64_t g = (int64_t)per_cu * num_cus();
    return (int)(tiles < g ? tiles : g);
}
bool rb_ok(int64_t C, int64_t T) { return (C == 32 || C == 64) && T >= 3; }

// cached (the workspace size must not move between the size query and the launch)
template <int C>
int rb_wgrad_grid(int64_t tiles) {
    static int g = 0;
    if (!g) g = rb_grid(rb_wgrad_kernel<C>, 256, rb_wgrad_lds(C), (int64_t)1 << 40);
    return (int)(tiles < g ? tiles : g);
}

template <int C>
void launch_bwd(const RbArgs& a, float* dws, float* dw2, float* dw1, float* db2, float* dbs, float* db1, int acc_w,
                int acc_b, hipStream_t st) {
    const int64_t tiles = (int64_t)a.B * a.NT;
    static int gd = 0;
    if (!gd) gd = rb_grid(rb_dgrad_kernel<C>, Rb<C>::NT, rb_dgrad_lds(C), (int64_t)1 << 40);
    hipLaunchKernelGGL((rb_dgrad_kernel<C>), dim3((unsigned)(tiles < gd ? tiles : gd)), dim3(Rb<C>::NT),
                       rb_dgrad_lds(C), st, a);
    const int gw = rb_wgrad_grid<C>(tiles);
    hipLaunchKernelGGL((rb_wgrad_kernel<C>), dim3(gw), dim3(256), rb_wgrad_lds(C), st, a);
    hipLaunchKernelGGL(rb_wgrad_reduce<C>, dim3((unsigned)cdiv(Rb<C>::SLAB, 64)), dim3(256), 0, st, a.slab, gw, dws,
                       dw2, dw1, db2, dbs, db1, acc_w, acc_b);
}

template <int C>
void launch_fwd(const RbArgs& a, int64_t tiles, hipStream_t st) {
    static int g = 0;
    if (!g) g = rb_grid(rb_fwd_kernel<C>, Rb<C>::NT, rb_fwd_lds(C), (int64_t)1 << 40);
    hipLaunchKernelGGL((rb_fwd_kernel<C>), dim3((unsigned)(tiles < g ? tiles : g)), dim3(Rb<C>::NT), rb_fwd_lds(C),
                       st, a);
}

}  // namespace

extern "C" {

int encx_resblock_fwd(const float* x, const float* w1, const float* b1, const float* w2, const float* b2,
                      const float* ws, const float* bs, float* h, float* y, int64_t B, int64_t C, int64_t T,
                      encx_stream_t stream) {
    ENCX_REQUIRE(x && w1 && b1 && w2 && b2 && ws && bs && y && B > 0 && rb_ok(C, T));
    hipStream_t st = (hipStream_t)stream;
    const int64_t HD = C / 2;
    encx_prof_scope ps(st, 2.0 * B * T * (3 * C * HD + (HD + C) * C), 4.0 * B * T * (2 * C + HD), "conv_rb_fwd");
    ps.tag(" C%ld T%ld", (long)C, (long)T);
    RbArgs a{x, w1, b1, w2, b2, ws, bs, h, y, nullptr, nullptr, nullptr, nullptr, (int)B, (int)T, (int)cdiv(T, TT)};
    const int64_t tiles = B * a.NT;
    if (C == 32) launch_fwd<32>(a, tiles, st);
    else launch_fwd<64>(a, tiles, st);
    ENCX_CHECK_LAUNCH();
    return 0;
}

// workspace: dh [B][C/2][T], then the weight-grad slab
size_t encx_resblock_bwd_workspace(int64_t B, int64_t C, int64_t T) {
    if (!rb_ok(C, T) || B <= 0) return 0;
    const int64_t tiles = B * cdiv(T, TT);
    const size_t slab = C == 32 ? (size_t)rb_wgrad_grid<32>(tiles) * Rb<32>::SLAB
                                : (size_t)rb_wgrad_grid<64>(tiles) * Rb<64>::SLAB;
    return ((size_t)B * (C / 2) * T + slab) * sizeof(float);
}

int encx_resblock_bwd(const float* dy, const float* x, const float* h, const float* w1, const float* w2,
                      const float* ws, float* dx, float* dw1, float* db1, float* dw2, float* db2, float* dws,
                      float* dbs, int acc_w, int acc_b, float* wsp, int64_t B, int64_t C, int64_t T,
                      encx_stream_t stream) {
    ENCX_REQUIRE(dy && x && h && w1 && w2 && ws && dx && wsp && B > 0 && rb_ok(C, T));
    hipStream_t st = (hipStream_t)stream;
    const int64_t HD = C / 2;
    encx_prof_scope ps(st, 4.0 * B * T * (3 * C * HD + (HD + C) * C), 4.0 * B * T * (4 * C + 2 * HD), "conv_rb_bwd");
    ps.tag(" C%ld T%ld", (long)C, (long)T);
    float* dh = wsp;
    float* slab = wsp + (size_t)B * HD * T;
    RbArgs a{x, w1, nullptr, w2, nullptr, ws, nullptr, const_cast<float*>(h), nullptr, dy, dx, dh, slab, (int)B, (int)T,
             (int)cdiv(T, TT)};
    if (C == 32) launch_bwd<32>(a, dws, dw2, dw1, db2, dbs, db1, acc_w, acc_b, st);
    else launch_bwd<64>(a, dws, dw2, dw1, db2, dbs, db1, acc_w, acc_b, st);
    ENCX_CHECK_LAUNCH();
    return 0;
}

}  // extern "C"
