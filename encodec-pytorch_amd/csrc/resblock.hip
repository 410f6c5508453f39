// Fused SEANet residual block for the high-rate stages (modules/seanet.py:21-63 with the EnCodec
// defaults: kernel_sizes [3, 1], dilations [1, 1], compress 2, true_skip False, causal reflect
// padding, weight_norm):
//     y = Ws x + bs  +  W2 ELU(h) + b2,    h = W1 * ELU(xpad) + b1  (k3, causal, reflect pad 2)
// At T = 24000 / 12000 (C = 32 / 64) the three convs are HBM-bound one by one: the unfused
// forward reads x twice and writes / re-reads the shortcut and the hidden tensor, the backward
// moves dy, x, h and their grads through HBM six times. Here one kernel per direction keeps a
// 64-position tile of every operand in LDS:
//   forward : x tile (+2 left halo) -> h (k3 GEMM) -> y ([ELU(h) | x] x [W2 | Ws] GEMM);
//             writes y and h (the backward's saved tensor), reads x once;
//   backward: dy, h (+2 right halo), x (+2 left halo) -> dh = W2^T dy * ELU'(h) ->
//             dx = Ws^T dy + ELU'(x) * (W1^T * dh)  (the reflect pad folded back at t = 1, 2)
//             and the weight grads dWs, dW2, dW1 and biases, accumulated in registers over the
//             workgroup's tiles (persistent grid), stored once per workgroup as a slab and summed
//             in a fixed order by rb_wgrad_reduce.
// Matrix work on v_mfma_f32_16x16x4_f32 (exact fp32; lane l: A[l&15][k=l>>4], B[k=l>>4][l&15],
// D[row 4(l>>4)+i][col l&15]); the position-major GEMMs put 16 positions of a wave on the rows,
// so a lane's 4 accumulator rows are 4 consecutive t of one channel: one 16-byte store.
#include "common.h"
#include "prof.h"

namespace {

typedef float f32x4v __attribute__((ext_vector_type(4)));
ENCX_DEV f32x4v mfma16(float a, float b, f32x4v c) { return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0); }

constexpr int TT = 64;       // positions per tile
constexpr int XS = TT + 4;   // LDS row stride of the position-indexed tiles
constexpr int DS = TT + 20;  // dh rows: positions 0 .. TT + 1 (+ padding to 16-position blocks)
constexpr int RB_NT = 256;

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
    float* slab;      // [grid][RB_SLAB(C)] backward weight-grad partials
    int B, T, NT;     // NT = tiles per batch item
};

template <int C>
struct RbSz {
    static constexpr int HD = C / 2;
    static constexpr int SLAB = C * C + C * HD + HD * 3 * C + C + HD;
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

// ------------------------------------------------------------------------------------ forward
template <int C>
__global__ __launch_bounds__(RB_NT) void rb_fwd_kernel(RbArgs a) {
    constexpr int HD = C / 2;
    extern __shared__ float sm[];
    float* xs = sm;                    // [C][XS]: x at t0 - 2 + p
    float* es = xs + C * XS;           // ELU(xs)
    float* w1 = es + C * XS;           // [C*3][HD]
    float* w2 = w1 + 3 * C * HD;       // [HD + C][C]: W2 rows then Ws rows (both wf [in][out])
    float* hs = w2 + (HD + C) * C;     // [HD][XS]: ELU(h) of the tile
    float* bo = hs + HD * XS;          // [C]: b2 + bs
    float* b1 = bo + C;                // [HD]
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, lc = lane & 15, lk = lane >> 4;
    for (int i = tid; i < 3 * C * HD; i += RB_NT) w1[i] = a.w1[i];
    for (int i = tid; i < HD * C; i += RB_NT) w2[i] = a.w2[i];
    for (int i = tid; i < C * C; i += RB_NT) w2[HD * C + i] = a.ws[i];
    for (int i = tid; i < C; i += RB_NT) bo[i] = a.b2[i] + a.bs[i];
    for (int i = tid; i < HD; i += RB_NT) b1[i] = a.b1[i];
    const int T = a.T, m0 = 16 * wv;
    const int ntiles = a.B * a.NT;
    for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        const int b = tile / a.NT, t0 = (tile - b * a.NT) * TT;
        __syncthreads();  // the previous tile's LDS reads are done (and the weights are staged)
        const float* xb = a.x + (int64_t)b * C * T;
        for (int i = tid; i < C * (TT + 2); i += RB_NT) {
            const int c = i / (TT + 2), p = i - c * (TT + 2);
            int t = t0 - 2 + p;
            t = t < 0 ? -t : (t < T ? t : T - 1);  // causal reflect pad (pad1d); past T: unused
            const float v = xb[(int64_t)c * T + t];
            xs[c * XS + p] = v;
            es[c * XS + p] = elu(v);
        }
        __syncthreads();
        // h^T[m][j] = b1[j] + sum_{c,k} ELU(x)[c][t - 2 + k] W1[c][k][j]   (rows = positions)
        f32x4v acc1[HD / 16];
#pragma unroll
        for (int n = 0; n < HD / 16; ++n) acc1[n] = (f32x4v){0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int k = 0; k < 3; ++k)
#pragma unroll
            for (int c0 = 0; c0 < C; c0 += 4) {
                const int c = c0 + lk;
                const float av = es[c * XS + m0 + lc + k];
#pragma unroll
                for (int n = 0; n < HD / 16; ++n) acc1[n] = mfma16(av, w1[(c * 3 + k) * HD + n * 16 + lc], acc1[n]);
            }
        float* hb = a.h + (int64_t)b * HD * T;
        const int tq = t0 + m0 + 4 * lk;  // this lane's 4 positions
#pragma unroll
        for (int n = 0; n < HD / 16; ++n) {
            const int j = n * 16 + lc;
            f32x4v hv;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                hv[i] = acc1[n][i] + b1[j];
                hs[j * XS + m0 + 4 * lk + i] = elu(hv[i]);
            }
            st4(hb + (int64_t)j * T, tq, T, hv);
        }
        __syncthreads();
        // y^T[m][o] = (b2 + bs)[o] + sum_j ELU(h)[j][m] W2[j][o] + sum_c x[c][m] Ws[c][o]
        f32x4v acc2[C / 16];
#pragma unroll
        for (int n = 0; n < C / 16; ++n) acc2[n] = (f32x4v){0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int j0 = 0; j0 < HD; j0 += 4) {
            const float av = hs[(j0 + lk) * XS + m0 + lc];
#pragma unroll
            for (int n = 0; n < C / 16; ++n) acc2[n] = mfma16(av, w2[(j0 + lk) * C + n * 16 + lc], acc2[n]);
        }
#pragma unroll
        for (int c0 = 0; c0 < C; c0 += 4) {
            const float av = xs[(c0 + lk) * XS + m0 + lc + 2];
#pragma unroll
            for (int n = 0; n < C / 16; ++n) acc2[n] = mfma16(av, w2[(HD + c0 + lk) * C + n * 16 + lc], acc2[n]);
        }
        float* yb = a.y + (int64_t)b * C * T;
#pragma unroll
        for (int n = 0; n < C / 16; ++n) {
            const int o = n * 16 + lc;
            f32x4v v;
#pragma unroll
            for (int i = 0; i < 4; ++i) v[i] = acc2[n][i] + bo[o];
            st4(yb + (int64_t)o * T, tq, T, v);
        }
    }
}

// ----------------------------------------------------------------------------------- backward
// weight-grad tiles (16 x 16) per workgroup: dWs (C/16)^2, dW2 (C/16)(HD/16), dW1 (HD/16)(3C/16),
// dealt round-robin to the 4 waves
template <int C>
struct RbTiles {
    static constexpr int HD = C / 2, NS = (C / 16) * (C / 16), N2 = (C / 16) * (HD / 16),
                         N1 = (HD / 16) * (3 * C / 16), N = NS + N2 + N1, PER = (N + 3) / 4;
};

template <int C>
__global__ __launch_bounds__(RB_NT) void rb_bwd_kernel(RbArgs a) {
    constexpr int HD = C / 2;
    using TL = RbTiles<C>;
    extern __shared__ float sm[];
    float* dys = sm;                 // [C][XS]: dy at t0 + p, p < TT + 2 (0 past T)
    float* hr = dys + C * XS;        // [HD][XS]: h (pre-ELU) at t0 + p
    float* he = hr + HD * XS;        // [HD][XS]: ELU(h)
    float* xs = he + HD * XS;        // [C][XS]: x at t0 - 2 + p (reflect)
    float* es = xs + C * XS;         // ELU(xs)
    float* dhs = es + C * XS;        // [HD][DS]: dh at t0 + p
    float* w1 = dhs + HD * DS;       // [C*3][HD]
    float* w2 = w1 + 3 * C * HD;     // [HD][C]
    float* wsm = w2 + HD * C;        // [C][C]
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, lc = lane & 15, lk = lane >> 4;
    for (int i = tid; i < 3 * C * HD; i += RB_NT) w1[i] = a.w1[i];
    for (int i = tid; i < HD * C; i += RB_NT) w2[i] = a.w2[i];
    for (int i = tid; i < C * C; i += RB_NT) wsm[i] = a.ws[i];
    const int T = a.T, m0 = 16 * wv;
    const int ntiles = a.B * a.NT;
    f32x4v accw[TL::PER];
#pragma unroll
    for (int q = 0; q < TL::PER; ++q) accw[q] = (f32x4v){0.f, 0.f, 0.f, 0.f};
    float bsum = 0.f;  // tid < C: sum of dy[o = tid]; C <= tid < C + HD: sum of dh[j = tid - C]
    for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        const int b = tile / a.NT, t0 = (tile - b * a.NT) * TT;
        __syncthreads();
        const float* dyb = a.dy + (int64_t)b * C * T;
        const float* hb = a.h + (int64_t)b * HD * T;
        const float* xb = a.x + (int64_t)b * C * T;
        for (int i = tid; i < C * (TT + 2); i += RB_NT) {
            const int c = i / (TT + 2), p = i - c * (TT + 2);
            const int t = t0 + p;
            const float v = dyb[(int64_t)c * T + (t < T ? t : T - 1)];
            dys[c * XS + p] = t < T ? v : 0.f;
            int tx = t - 2;
            tx = tx < 0 ? -tx : (tx < T ? tx : T - 1);
            const float u = xb[(int64_t)c * T + tx];
            xs[c * XS + p] = u;
            es[c * XS + p] = elu(u);
        }
        for (int i = tid; i < HD * (TT + 2); i += RB_NT) {
            const int j = i / (TT + 2), p = i - j * (TT + 2);
            const int t = t0 + p;
            const float v = hb[(int64_t)j * T + (t < T ? t : T - 1)];
            hr[j * XS + p] = v;
            he[j * XS + p] = elu(v);
        }
        __syncthreads();
        // ---- dh^T[p][j] = ELU'(h) * sum_o dy[o][p] W2[j][o], positions 0 .. TT - 1 (MFMA) ...
        {
            f32x4v acc[HD / 16];
#pragma unroll
            for (int n = 0; n < HD / 16; ++n) acc[n] = (f32x4v){0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int o0 = 0; o0 < C; o0 += 4) {
                const float av = dys[(o0 + lk) * XS + m0 + lc];
#pragma unroll
                for (int n = 0; n < HD / 16; ++n) acc[n] = mfma16(av, w2[(n * 16 + lc) * C + o0 + lk], acc[n]);
            }
#pragma unroll
            for (int n = 0; n < HD / 16; ++n) {
                const int j = n * 16 + lc;
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int p = m0 + 4 * lk + i;
                    dhs[j * DS + p] = t0 + p < T ? acc[n][i] * elu_grad(hr[j * XS + p]) : 0.f;
                }
            }
        }
        // ... and the right halo TT, TT + 1 on the vector ALU
        for (int i = tid; i < 2 * HD; i += RB_NT) {
            const int j = i >> 1, p = TT + (i & 1);
            float s = 0.f;
            for (int o = 0; o < C; ++o) s = fmaf(dys[o * XS + p], w2[j * C + o], s);
            dhs[j * DS + p] = t0 + p < T ? s * elu_grad(hr[j * XS + p]) : 0.f;
        }
        __syncthreads();
        // ---- dx^T[m][c] = sum_o dy[o][m] Ws[c][o] + ELU'(x[c][m]) * sum_{j,k} dh[j][m + 2 - k] W1[c][k][j]
        {
            f32x4v asc[C / 16], ak3[C / 16];
#pragma unroll
            for (int n = 0; n < C / 16; ++n) asc[n] = ak3[n] = (f32x4v){0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int o0 = 0; o0 < C; o0 += 4) {
                const float av = dys[(o0 + lk) * XS + m0 + lc];
#pragma unroll
                for (int n = 0; n < C / 16; ++n) asc[n] = mfma16(av, wsm[(n * 16 + lc) * C + o0 + lk], asc[n]);
            }
#pragma unroll
            for (int k = 0; k < 3; ++k)
#pragma unroll
                for (int j0 = 0; j0 < HD; j0 += 4) {
                    const int j = j0 + lk;
                    const float av = dhs[j * DS + m0 + lc + 2 - k];
#pragma unroll
                    for (int n = 0; n < C / 16; ++n) ak3[n] = mfma16(av, w1[((n * 16 + lc) * 3 + k) * HD + j], ak3[n]);
                }
            // reflect pad: ELU(x) at t = -1, -2 is ELU(x[1]), ELU(x[2]); their grads fold into t = 1, 2
            if (t0 == 0 && wv == 0 && lk == 0) {
#pragma unroll
                for (int n = 0; n < C / 16; ++n) {
                    const int c = n * 16 + lc;
                    float v1 = 0.f, v2 = 0.f;
                    for (int j = 0; j < HD; ++j) {
                        const float w0 = w1[(c * 3) * HD + j], w1v = w1[(c * 3 + 1) * HD + j];
                        v1 = fmaf(w0, dhs[j * DS + 1], fmaf(w1v, dhs[j * DS + 0], v1));
                        v2 = fmaf(w0, dhs[j * DS + 0], v2);
                    }
                    ak3[n][1] += v1;
                    ak3[n][2] += v2;
                }
            }
            float* dxb = a.dx + (int64_t)b * C * T;
            const int tq = t0 + m0 + 4 * lk;
#pragma unroll
            for (int n = 0; n < C / 16; ++n) {
                const int c = n * 16 + lc;
                f32x4v v;
#pragma unroll
                for (int i = 0; i < 4; ++i) v[i] = asc[n][i] + elu_grad(xs[c * XS + m0 + 4 * lk + i + 2]) * ak3[n][i];
                st4(dxb + (int64_t)c * T, tq, T, v);
            }
        }
        // ---- weight grads over this tile's positions (K = TT; dy and dh are 0 past T)
#pragma unroll
        for (int q = 0; q < TL::PER; ++q) {
            const int tl = wv + 4 * q;
            if (tl >= TL::N) break;
            if (tl < TL::NS) {  // dWs[o][c] = sum_p dy[o][p] x[c][p]
                const int mo = (tl / (C / 16)) * 16, nc = (tl % (C / 16)) * 16;
#pragma unroll
                for (int p0 = 0; p0 < TT; p0 += 4)
                    accw[q] = mfma16(dys[(mo + lc) * XS + p0 + lk], xs[(nc + lc) * XS + p0 + lk + 2], accw[q]);
            } else if (tl < TL::NS + TL::N2) {  // dW2[o][j] = sum_p dy[o][p] ELU(h)[j][p]
                const int t2 = tl - TL::NS, mo = (t2 / (HD / 16)) * 16, nj = (t2 % (HD / 16)) * 16;
#pragma unroll
                for (int p0 = 0; p0 < TT; p0 += 4)
                    accw[q] = mfma16(dys[(mo + lc) * XS + p0 + lk], he[(nj + lc) * XS + p0 + lk], accw[q]);
            } else {  // dW1[j][(k, c)] = sum_p dh[j][p] ELU(x)[c][t - 2 + k]
                const int t1 = tl - TL::NS - TL::N2, mj = (t1 / (3 * C / 16)) * 16, nn = (t1 % (3 * C / 16)) * 16;
                const int k = nn / C, nc = nn - k * C;
#pragma unroll
                for (int p0 = 0; p0 < TT; p0 += 4)
                    accw[q] = mfma16(dhs[(mj + lc) * DS + p0 + lk], es[(nc + lc) * XS + p0 + lk + k], accw[q]);
            }
        }
        if (tid < C) {
            for (int p = 0; p < TT; ++p) bsum += dys[tid * XS + p];
        } else if (tid < C + HD) {
            for (int p = 0; p < TT; ++p) bsum += dhs[(tid - C) * DS + p];
        }
    }
    // ---- this workgroup's partial weight grads -> slab [dWs C x C][dW2 C x HD][dW1 HD x C x 3][db C][db1 HD]
    // (natural layouts: dWs[o][c], dW2[o][j], dW1[j][c][k])
    float* sl = a.slab + (int64_t)blockIdx.x * RbSz<C>::SLAB;
#pragma unroll
    for (int q = 0; q < TL::PER; ++q) {
        const int tl = wv + 4 * q;
        if (tl >= TL::N) break;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int r = 4 * lk + i;  // D row
            if (tl < TL::NS) {
                const int o = (tl / (C / 16)) * 16 + r, c = (tl % (C / 16)) * 16 + lc;
                sl[o * C + c] = accw[q][i];
            } else if (tl < TL::NS + TL::N2) {
                const int t2 = tl - TL::NS, o = (t2 / (HD / 16)) * 16 + r, j = (t2 % (HD / 16)) * 16 + lc;
                sl[C * C + o * HD + j] = accw[q][i];
            } else {
                const int t1 = tl - TL::NS - TL::N2, j = (t1 / (3 * C / 16)) * 16 + r;
                const int nn = (t1 % (3 * C / 16)) * 16 + lc, k = nn / C, c = nn - k * C;
                sl[C * C + C * HD + (j * C + c) * 3 + k] = accw[q][i];
            }
        }
    }
    if (tid < C + HD) sl[C * C + C * HD + HD * 3 * C + tid] = bsum;
}

// out[i] (+)= sum_{g < G} slab[g][i] in ascending g, for the slab's sections: dWs -> dws, dW2 ->
// dw2, dW1 -> dw1, db -> db2 and dbs (the same sum), db1 -> db1. Null outputs are skipped.
template <int C>
__global__ __launch_bounds__(256) void rb_wgrad_reduce(const float* slab, int G, float* dws, float* dw2, float* dw1,
                                                       float* db2, float* dbs, float* db1, int acc_w, int acc_b) {
    constexpr int HD = C / 2, S = RbSz<C>::SLAB;
    __shared__ float red[256];
    const int64_t i = (int64_t)blockIdx.x * 64 + (threadIdx.x & 63);
    const bool valid = i < S;
    const float v = slab_sum_256(slab + (valid ? i : 0), G, S, valid, red);
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

size_t rb_fwd_lds(int C) {
    const int HD = C / 2;
    return (size_t)(2 * C * XS + 3 * C * HD + (HD + C) * C + HD * XS + C + HD) * sizeof(float);
}
size_t rb_bwd_lds(int C) {
    const int HD = C / 2;
    return (size_t)(C * XS + 2 * HD * XS + 2 * C * XS + HD * DS + 3 * C * HD + HD * C + C * C) * sizeof(float);
}
int rb_grid(int64_t tiles, int C) {  // persistent: whole rounds over the CUs (LDS-limited residency)
    const int per_cu = C <= 32 ? 2 : 1;
    return (int)(tiles < 256 * per_cu ? tiles : 256 * per_cu);
}
bool rb_ok(int64_t C, int64_t T) { return (C == 32 || C == 64) && T >= 3; }

}  // namespace

extern "C" {

int encx_resblock_fwd(const float* x, const float* w1, const float* b1, const float* w2, const float* b2,
                      const float* ws, const float* bs, float* h, float* y, int64_t B, int64_t C, int64_t T,
                      encx_stream_t stream) {
    ENCX_REQUIRE(x && w1 && b1 && w2 && b2 && ws && bs && h && y && B > 0 && rb_ok(C, T));
    hipStream_t st = (hipStream_t)stream;
    const int64_t HD = C / 2;
    encx_prof_scope ps(st, 2.0 * B * T * (3 * C * HD + (HD + C) * C), 4.0 * B * T * (2 * C + HD), "conv_rb_fwd");
    ps.tag(" C%ld T%ld", (long)C, (long)T);
    RbArgs a{x, w1, b1, w2, b2, ws, bs, h, y, nullptr, nullptr, nullptr, (int)B, (int)T, (int)cdiv(T, TT)};
    const int grid = rb_grid(B * a.NT, (int)C);
    if (C == 32) hipLaunchKernelGGL(rb_fwd_kernel<32>, dim3(grid), dim3(RB_NT), rb_fwd_lds(32), st, a);
    else hipLaunchKernelGGL(rb_fwd_kernel<64>, dim3(grid), dim3(RB_NT), rb_fwd_lds(64), st, a);
    ENCX_CHECK_LAUNCH();
    return 0;
}

size_t encx_resblock_bwd_workspace(int64_t B, int64_t C, int64_t T) {
    if (!rb_ok(C, T) || B <= 0) return 0;
    const int grid = rb_grid(B * cdiv(T, TT), (int)C);
    return (size_t)grid * (C == 32 ? RbSz<32>::SLAB : RbSz<64>::SLAB) * sizeof(float);
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
    RbArgs a{x, w1, nullptr, w2, nullptr, ws, nullptr, const_cast<float*>(h), nullptr, dy, dx, wsp, (int)B, (int)T,
             (int)cdiv(T, TT)};
    const int grid = rb_grid(B * a.NT, (int)C);
    if (C == 32) {
        hipLaunchKernelGGL(rb_bwd_kernel<32>, dim3(grid), dim3(RB_NT), rb_bwd_lds(32), st, a);
        ENCX_CHECK_LAUNCH();
        hipLaunchKernelGGL(rb_wgrad_reduce<32>, dim3((unsigned)cdiv(RbSz<32>::SLAB, 64)), dim3(256), 0, st, wsp, grid,
                           dws, dw2, dw1, db2, dbs, db1, acc_w, acc_b);
    } else {
        hipLaunchKernelGGL(rb_bwd_kernel<64>, dim3(grid), dim3(RB_NT), rb_bwd_lds(64), st, a);
        ENCX_CHECK_LAUNCH();
        hipLaunchKernelGGL(rb_wgrad_reduce<64>, dim3((unsigned)cdiv(RbSz<64>::SLAB, 64)), dim3(256), 0, st, wsp, grid,
                           dws, dw2, dw1, db2, dbs, db1, acc_w, acc_b);
    }
    ENCX_CHECK_LAUNCH();
    return 0;
}

}  // extern "C"
