// SEANet 1-D convolution family on gfx950 (modules/conv.py SConv1d / SConvTranspose1d).
//
// Three MFMA kernels (v_mfma_f32_32x32x2_f32, exact fp32), 4 waves per workgroup, each wave
// owning a (32*TM) x (32*TN) output sub-tile:
//   conv_fwd     implicit GEMM  Y[co, t]  = W[co, (ci,k)] * act(Xpad)[(ci,k), t]
//                The X window of a channel chunk is staged once in LDS (act applied once per
//                element) and stored phase-major, Xs[ci][t mod s][t div s], so strided taps
//                read consecutive LDS words.
//   conv_poly    polyphase transposed conv: rows (o, r), columns u, reduction (i, q):
//                out[o][u*s + r] = sum_{i,q} Wp[i][q][o*s+r] * in[i][u-q]. Serves
//                ConvTranspose1d forward and Conv1d backward-data (with the reflect pad
//                folded back and act' applied in the epilogue; pad positions go to a side
//                buffer that conv_fold_edges adds in a fixed order).
//   conv_wgrad   dW[a][(c,k)] = sum_{b,t} L[b][a][t] * R[b][c][t*s + k*d - pl], split over
//                (b, t) ranges into a workspace and summed by wgrad_reduce in a fixed order;
//                for narrow weights (Cin*K <= 32) the 4 waves split the t range of one 32x32
//                tile instead of tiling N.
// Low-rate layers (T = 75 / 600 at B = 32) would launch fewer workgroups than the chip has
// CUs, so conv_fwd / conv_poly split the channel reduction (split-K) into a workspace and a
// fixed-order reduce kernel applies the epilogue: deterministic, no float atomics.
// Plus VALU kernels for the 1-channel ends of the stack (Cout = 1 forward, tiny wgrads).
#include <stdlib.h>

#include <algorithm>
#include <cstdlib>

#include "common.h"
#include "gemm.h"
#include "prof.h"

namespace {

constexpr int NT = 256;  // threads per workgroup (4 waves)
#ifndef ENCX_SPER
#define ENCX_SPER 4
#endif
constexpr int SPER = ENCX_SPER;  // staging items (float4) in flight per thread
constexpr int FLAT_T = 128;  // layers with T_out <= this run as one (b, t)-flattened GEMM

// LDS staging: position lanes per channel lane for a window of `len` positions (QP | NT)

// ------------------------------------------------------------------------- conv forward
struct FwdArgs {
    const float* x;
    const float* wf;  // [Cin][K][Cout]
    const float* bias;
    const float* res;
    float* y;
    const float* xact;  // epilogue act' source (backward-data use), or null
    float* part;        // split-K partials [KS][B][Cout][Tout]
    int B, Cin, Tin, Cout, Tout, K, s, d, pl, e, mode, act;
    int epi_act, accumulate;
    int vec;  // x rows and wf rows 16-B aligned: float4 staging loads
    int CK;   // channels per LDS chunk (even)
    int Up;   // LDS words per (ci, phase) row
    int KS;   // channel splits
    int cps;  // channels per split (multiple of CK)
    FastDiv fs;  // division by s (set by launch_fwd): the phase split of every staged element
};

// y = [acc ? y : 0] + act'(xact) * (v + bias) + res
ENCX_DEV void fwd_store(const FwdArgs& a, int64_t o, int co, float v) {
    v += a.bias ? a.bias[co] : 0.f;
    if (a.xact) v *= act_grad(a.epi_act, a.xact[o]);
    if (a.res) v += a.res[o];
    if (a.accumulate) v += a.y[o];
    a.y[o] = v;
}

// Epilogue operands are compile-time (EPI bits): runtime-null operand pointers tested per
// element compile to exec-masked branches around every load and cost ~3x on the HBM-bound
// layers. EPI_RES: + residual; EPI_XACT: * act'(xact); EPI_ACC: + y; EPI_PART: split-K
// partial store (no bias, no operands).
enum { EPI_RES = 1, EPI_XACT = 2, EPI_ACC = 4, EPI_PART = 8 };
template <int BM, int BN, int WM, int WN, int EPI>
__global__ __launch_bounds__(NT) void conv_fwd_kernel(FwdArgs a) {
    constexpr int TM = BM / WM / 32, TN = BN / WN / 32;
    extern __shared__ float smem[];
    const int CK = a.CK, S = a.s, Up = a.Up, K = a.K;
    float* Xs = smem;                       // [CK][S][Up]
    float* Ws = smem + ((CK * S * Up + 3) & ~3);  // [CK][K][BM], 16-B aligned
    float* Bsm = Ws + K * CK * BM;          // [BM] bias of the block's rows
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm0 = (wave / WN) * TM * 32, wn0 = (wave % WN) * TN * 32;
    const int t0 = blockIdx.x * BN, co0 = blockIdx.y * BM;
    if (tid < BM) Bsm[tid] = (a.bias && co0 + tid < a.Cout) ? a.bias[co0 + tid] : 0.f;
    const int b = blockIdx.z / a.KS, ks = blockIdx.z - (blockIdx.z / a.KS) * a.KS;
    const float* xb = a.x + (int64_t)b * a.Cin * a.Tin;
    const int span = S * Up;
    const int cbeg = ks * a.cps, cend = min(a.Cin, cbeg + a.cps);

    f32x16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = (f32x16){0};

    // The chunk's window of every channel row is [wb, wb + span) in input coordinates
    // (wb = t0*S - pl), staged as 4-position items from the 4-aligned floor of wb: one float4
    // load per interior item (VEC: rows 16-B aligned), per-element pad_src only for the items
    // that straddle a row end. The loop is kept simple (one item per iteration): unrolled,
    // predicated staging compiles to divergent branch ladders that cost more than the loads.
    const int wb = t0 * S - a.pl;
    const int ab = wb & ~3, woff = wb - ab;
    const int nv = (woff + span + 3) >> 2;
    const int nitems = CK * nv;
    const int BM4 = BM / 4, nw = K * CK * BM4;
    // item (cl, vi) of thread tid advances by NT items per step: no per-item division
    const int dcl = NT / nv, dvi = NT - dcl * nv, cl_init = tid / nv, vi_init = tid - cl_init * nv;
    for (int c0 = cbeg; c0 < cend; c0 += CK) {
        __syncthreads();
        // SPER items per thread in flight: interior items load as float4 from a clamped address
        // (value selected after the load), the rare items straddling a row end are patched
        // per element afterwards, then everything goes to LDS
        int cl_n = cl_init, vi_n = vi_init;
        for (int it0 = 0; it0 < nitems; it0 += NT * SPER) {
            f32x4 v[SPER];
            int clq[SPER], viq[SPER];
#pragma unroll
            for (int q = 0; q < SPER; ++q) {
                clq[q] = cl_n;
                viq[q] = vi_n;
                vi_n += dvi;
                cl_n += dcl;
                if (vi_n >= nv) {
                    vi_n -= nv;
                    ++cl_n;
                }
            }
#pragma unroll
            for (int q = 0; q < SPER; ++q) {
                const int c = c0 + clq[q], p = ab + 4 * viq[q];
                const bool ok = clq[q] < CK && c < cend;
                v[q] = (f32x4){0.f, 0.f, 0.f, 0.f};
                if (a.vec) {
                    const int pc = p < 0 ? 0 : (p > a.Tin - 4 ? a.Tin - 4 : p);
                    const f32x4 t = *(const f32x4*)(xb + (int64_t)(ok ? c : cbeg) * a.Tin + pc);
                    if (ok && p >= 0 && p + 3 < a.Tin) v[q] = t;
                }
            }
#pragma unroll
            for (int q = 0; q < SPER; ++q) {
                const int c = c0 + clq[q], p = ab + 4 * viq[q];
                if (clq[q] < CK && c < cend && !(a.vec && p >= 0 && p + 3 < a.Tin)) {
                    const float* xr = xb + (int64_t)c * a.Tin;
                    for (int e = 0; e < 4; ++e) {
                        const int m = pad_src(p + e + a.pl, a.pl, a.Tin, a.e, a.mode);
                        v[q][e] = m >= 0 ? xr[m] : 0.f;
                    }
                }
            }
#pragma unroll
            for (int q = 0; q < SPER; ++q) {
                if (clq[q] >= CK) continue;
                float* xs = Xs + clq[q] * span;
                const int q0 = 4 * viq[q] - woff;
                if (S == 1 && q0 >= 0 && q0 + 3 < span) {
                    xs[q0] = act_apply(a.act, v[q][0]);
                    xs[q0 + 1] = act_apply(a.act, v[q][1]);
                    xs[q0 + 2] = act_apply(a.act, v[q][2]);
                    xs[q0 + 3] = act_apply(a.act, v[q][3]);
                } else {
                    for (int e = 0; e < 4; ++e) {
                        const int qq = q0 + e;
                        if (qq >= 0 && qq < span) {
                            const int u = (int)fdiv((uint32_t)qq, a.fs), ph = qq - u * S;
                            xs[ph * Up + u] = act_apply(a.act, v[q][e]);
                        }
                    }
                }
            }
        }
        // weights Ws[cl][k][co] = wf[c0 + cl][k][co0 + co]: rows (cl, k) are consecutive rows of
        // wf, BM contiguous co per row, float4 items
        const int wrows = (min(cend, c0 + CK) - c0) * K;
        for (int it0 = 0; it0 < nw; it0 += NT * SPER) {
            f32x4 v[SPER];
#pragma unroll
            for (int q = 0; q < SPER; ++q) {
                const int it = it0 + q * NT + tid;
                const int r = it / BM4, c4 = it - r * BM4, co = co0 + 4 * c4;
                const bool ok = r < wrows;
                const float* wr = a.wf + ((int64_t)c0 * K + (ok ? r : 0)) * a.Cout;
                v[q] = (f32x4){0.f, 0.f, 0.f, 0.f};
                if (a.vec) {
                    const int coc = co + 3 < a.Cout ? co : a.Cout - 4;
                    const f32x4 t = *(const f32x4*)(wr + coc);
                    if (ok && co + 3 < a.Cout) v[q] = t;
                } else if (ok) {
                    for (int e = 0; e < 4; ++e) v[q][e] = co + e < a.Cout ? wr[co + e] : 0.f;
                }
            }
#pragma unroll
            for (int q = 0; q < SPER; ++q) {
                const int it = it0 + q * NT + tid;
                if (it < nw) *(f32x4*)(Ws + 4 * it) = v[q];
            }
        }
        __syncthreads();
        const int h = lane >> 5, l32 = lane & 31;
        for (int k = 0; k < K; ++k) {
            const int kd = k * a.d, ph = kd % S, off = kd / S;
            const float* wk = Ws + (h * K + k) * BM + wm0 + l32;
            const float* xk = Xs + (h * S + ph) * Up + wn0 + l32 + off;
#pragma unroll 4
            for (int cp = 0; cp < CK; cp += 2) {
                float av[TM], bv[TN];
#pragma unroll
                for (int i = 0; i < TM; ++i) av[i] = wk[cp * K * BM + i * 32];
#pragma unroll
                for (int j = 0; j < TN; ++j) bv[j] = xk[cp * S * Up + j * 32];
#pragma unroll
                for (int i = 0; i < TM; ++i)
#pragma unroll
                    for (int j = 0; j < TN; ++j) acc[i][j] = mfma32(av[i], bv[j], acc[i][j]);
            }
        }
    }
    // epilogue: bias from LDS (staged at entry); the operands of a 32 x 32 sub-tile are all
    // loaded before its stores (y may alias them, so the compiler cannot hoist them itself)
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int t = t0 + wn0 + j * 32 + (lane & 31);
            const int64_t ob = ((int64_t)b * a.Cout + co0 + wm0 + i * 32) * a.Tout + t;
            float e0[16], e1[16];
            const bool tok = t < a.Tout;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const bool ok = tok && co0 + wm0 + i * 32 + mfma_row(r, lane) < a.Cout;
                const int64_t o = ok ? ob + (int64_t)mfma_row(r, lane) * a.Tout : 0;
                e0[r] = (EPI & EPI_XACT) ? a.xact[o] : 0.f;
                e1[r] = (EPI & EPI_RES) ? a.res[o] : 0.f;
                if (EPI & EPI_ACC) e1[r] += a.y[o];
            }
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int cl = wm0 + i * 32 + mfma_row(r, lane), co = co0 + cl;
                if (co >= a.Cout || t >= a.Tout) continue;
                const int64_t o = ob + (int64_t)mfma_row(r, lane) * a.Tout;
                float w = acc[i][j][r];
                if (EPI & EPI_PART) {
                    a.part[(int64_t)ks * a.B * a.Cout * a.Tout + o] = w;
                } else {
                    w += Bsm[cl];
                    if (EPI & EPI_XACT) w *= act_grad(a.epi_act, e0[r]);
                    a.y[o] = w + e1[r];
                }
            }
        }
}

__global__ void conv_fwd_reduce(FwdArgs a) {
    const int64_t n = (int64_t)a.B * a.Cout * a.Tout;
    int64_t o = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (o >= n) return;
    const float v = sum_strided(a.part + o, a.KS, n);
    const int co = (int)((o / a.Tout) % a.Cout);
    fwd_store(a, o, co, v);
}

// ------------------------------------------------------------------------- polyphase
struct PolyArgs {
    const float* in;   // [B][Ci][Tin]
    const float* wp;   // [Ci][J][Co*s]
    const float* bias; // convtr mode
    const float* xact; // dgrad mode: pre-activation input for act'
    float* out;        // convtr: y [B][Co][Tout]; dgrad: dx [B][Co][Tx]
    float* side;       // dgrad: [B][Co][pl+pr]
    float* part;       // split-K partials [KS][B][Co][Q], Q = ncols * s
    int B, Ci, Tin, Co, s, J;
    int mode;          // 0 convtr store, 1 dgrad fold
    int trim;          // convtr: trim_left
    int Tout;          // convtr output length
    int pl, pr, Tx;    // dgrad: pads, unpadded length
    int act, in_act, accumulate;
    int CK, Ub;        // chunk channels, LDS row length (BN + J - 1 [+pad])
    int KS, cps, Q;
    int vec;           // in rows and wp rows 16-B aligned: float4 staging loads
};

ENCX_DEV void poly_store(const PolyArgs& a, int b, int o, int qpos, float v) {
    if (a.mode == 0) {
        const int p = qpos - a.trim;
        if (p >= 0 && p < a.Tout)
            a.out[((int64_t)b * a.Co + o) * a.Tout + p] = v + (a.bias ? a.bias[o] : 0.f);
    } else {
        const int m = qpos - a.pl;
        if (m >= 0 && m < a.Tx) {
            const int64_t idx = ((int64_t)b * a.Co + o) * a.Tx + m;
            float g = v;
            if (a.act != ENCX_ACT_NONE) g *= act_grad(a.act, a.xact[idx]);
            a.out[idx] = a.accumulate ? a.out[idx] + g : g;
        } else if (qpos >= 0 && qpos < a.pl + a.Tx + a.pr) {
            const int slot = m < 0 ? qpos : a.pl + (m - a.Tx);
            a.side[((int64_t)b * a.Co + o) * (a.pl + a.pr) + slot] = v;
        }
    }
}

// Epilogue bits (compile-time, see conv_fwd_kernel): P_DGRAD: backward-data fold (else the
// ConvTranspose1d store with bias and trim); P_XACT: * act'(xact); P_ACC: + out; P_PART:
// split-K partial store.
enum { P_DGRAD = 1, P_XACT = 2, P_ACC = 4, P_PART = 8 };
template <int BM, int BN, int WM, int WN, int EPI>
__global__ __launch_bounds__(NT) void conv_poly_kernel(PolyArgs a) {
    constexpr int TM = BM / WM / 32, TN = BN / WN / 32;
    extern __shared__ float smem[];
    const int CK = a.CK, J = a.J, Ub = a.Ub, S = a.s;
    const int M = a.Co * S;
    float* Xs = smem;                               // [CK][Ub]
    float* As = smem + ((CK * Ub + 3) & ~3);        // [CK][J][BM], 16-B aligned
    float* Bsm = As + J * CK * BM;                  // [BM] per-row bias (ConvTranspose1d mode)
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm0 = (wave / WN) * TM * 32, wn0 = (wave % WN) * TN * 32;
    const int u0 = blockIdx.x * BN, m0 = blockIdx.y * BM;
    if (tid < BM) Bsm[tid] = (!(EPI & P_DGRAD) && a.bias && m0 + tid < M) ? a.bias[(m0 + tid) / S] : 0.f;
    const int b = blockIdx.z / a.KS, ks = blockIdx.z - (blockIdx.z / a.KS) * a.KS;
    const float* ib = a.in + (int64_t)b * a.Ci * a.Tin;
    const int cbeg = ks * a.cps, cend = min(a.Ci, cbeg + a.cps);

    f32x16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = (f32x16){0};

    // input window of the tile: positions w in [0, wlen) are in[u0 - (J-1) + w] (zero outside
    // [0, Tin)), staged as 4-position items from the 4-aligned floor (see conv_fwd_kernel)
    const int wlen = BN + J - 1;
    const int wb = u0 - (J - 1), ab = wb & ~3, woff = wb - ab;
    const int nv = (woff + wlen + 3) >> 2, nitems = CK * nv;
    const int BM4 = BM / 4, nw = J * CK * BM4;
    const int dcl = NT / nv, dvi = NT - dcl * nv, cl_init = tid / nv, vi_init = tid - cl_init * nv;
    for (int c0 = cbeg; c0 < cend; c0 += CK) {
        __syncthreads();
        // batched staging as in conv_fwd_kernel: SPER float4 loads in flight per thread, items
        // walked by a fixed step (no per-item division)
        int cl_n = cl_init, vi_n = vi_init;
        for (int it0 = 0; it0 < nitems; it0 += NT * SPER) {
            f32x4 v[SPER];
            int clq[SPER], viq[SPER];
#pragma unroll
            for (int q = 0; q < SPER; ++q) {
                clq[q] = cl_n;
                viq[q] = vi_n;
                vi_n += dvi;
                cl_n += dcl;
                if (vi_n >= nv) {
                    vi_n -= nv;
                    ++cl_n;
                }
            }
#pragma unroll
            for (int q = 0; q < SPER; ++q) {
                const int c = c0 + clq[q], p = ab + 4 * viq[q];
                const bool ok = clq[q] < CK && c < cend;
                v[q] = (f32x4){0.f, 0.f, 0.f, 0.f};
                if (a.vec) {
                    const int pc = p < 0 ? 0 : (p > a.Tin - 4 ? a.Tin - 4 : p);
                    const f32x4 t = *(const f32x4*)(ib + (int64_t)(ok ? c : cbeg) * a.Tin + pc);
                    if (ok && p >= 0 && p + 3 < a.Tin) v[q] = t;
                }
            }
#pragma unroll
            for (int q = 0; q < SPER; ++q) {
                const int c = c0 + clq[q], p = ab + 4 * viq[q];
                if (clq[q] < CK && c < cend && !(a.vec && p >= 0 && p + 3 < a.Tin)) {
                    const float* ir = ib + (int64_t)c * a.Tin;
                    for (int e = 0; e < 4; ++e) v[q][e] = (p + e >= 0 && p + e < a.Tin) ? ir[p + e] : 0.f;
                }
            }
#pragma unroll
            for (int q = 0; q < SPER; ++q) {
                if (clq[q] >= CK) continue;
                float* xs = Xs + clq[q] * Ub;
                const int q0 = 4 * viq[q] - woff;
                for (int e = 0; e < 4; ++e) {
                    const int qq = q0 + e;
                    if (qq >= 0 && qq < wlen) xs[qq] = act_apply(a.in_act, v[q][e]);
                }
            }
        }
        // As[cl][q][m] = wp[c0 + cl][q][m0 + m]: consecutive rows of wp, float4 items
        const int wrows = (min(cend, c0 + CK) - c0) * J;
        for (int it0 = 0; it0 < nw; it0 += NT * SPER) {
            f32x4 v[SPER];
#pragma unroll
            for (int q = 0; q < SPER; ++q) {
                const int it = it0 + q * NT + tid;
                const int r = it / BM4, c4 = it - r * BM4, m = m0 + 4 * c4;
                const bool ok = r < wrows;
                const float* wr = a.wp + ((int64_t)c0 * J + (ok ? r : 0)) * M;
                v[q] = (f32x4){0.f, 0.f, 0.f, 0.f};
                if (a.vec) {
                    const int mc = m + 3 < M ? m : M - 4;
                    const f32x4 t = *(const f32x4*)(wr + mc);
                    if (ok && m + 3 < M) v[q] = t;
                } else if (ok) {
                    for (int e = 0; e < 4; ++e) v[q][e] = m + e < M ? wr[m + e] : 0.f;
                }
            }
#pragma unroll
            for (int q = 0; q < SPER; ++q) {
                const int it = it0 + q * NT + tid;
                if (it < nw) *(f32x4*)(As + 4 * it) = v[q];
            }
        }
        __syncthreads();
        const int h = lane >> 5, l32 = lane & 31;
        for (int q = 0; q < J; ++q) {
            const float* aq = As + (h * J + q) * BM + wm0 + l32;
            const float* xq = Xs + h * Ub + wn0 + l32 + (J - 1) - q;
#pragma unroll 4
            for (int cp = 0; cp < CK; cp += 2) {
                float av[TM], bv[TN];
#pragma unroll
                for (int i = 0; i < TM; ++i) av[i] = aq[cp * J * BM + i * 32];
#pragma unroll
                for (int j = 0; j < TN; ++j) bv[j] = xq[cp * Ub + j * 32];
#pragma unroll
                for (int i = 0; i < TM; ++i)
#pragma unroll
                    for (int j = 0; j < TN; ++j) acc[i][j] = mfma32(av[i], bv[j], acc[i][j]);
            }
        }
    }
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int u = u0 + wn0 + j * 32 + (lane & 31);
            if (EPI & P_PART) {
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int row = m0 + wm0 + i * 32 + mfma_row(r, lane);
                    if (row >= M) continue;
                    const int o = row / S, rr = row - o * S, qpos = u * S + rr;
                    if (qpos < a.Q) a.part[(((int64_t)ks * a.B + b) * a.Co + o) * a.Q + qpos] = acc[i][j][r];
                }
                continue;
            }
            if (!(EPI & P_DGRAD)) {  // ConvTranspose1d: bias from LDS, trim
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int rl = wm0 + i * 32 + mfma_row(r, lane), row = m0 + rl;
                    if (row >= M) continue;
                    const int o = row / S, p = u * S + (row - o * S) - a.trim;
                    if (p >= 0 && p < a.Tout) a.out[((int64_t)b * a.Co + o) * a.Tout + p] = acc[i][j][r] + Bsm[rl];
                }
                continue;
            }
            // backward-data: act' source / accumulated value loaded for the whole sub-tile first
            float e0[16], e1[16];
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int row = m0 + wm0 + i * 32 + mfma_row(r, lane);
                const int o = row / S, m = u * S + (row - o * S) - a.pl;
                const bool ok = row < M && m >= 0 && m < a.Tx;
                const int64_t idx = ok ? ((int64_t)b * a.Co + o) * a.Tx + m : 0;
                e0[r] = (EPI & P_XACT) ? a.xact[idx] : 0.f;
                e1[r] = (EPI & P_ACC) ? a.out[idx] : 0.f;
            }
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int row = m0 + wm0 + i * 32 + mfma_row(r, lane);
                if (row >= M) continue;
                const int o = row / S, qpos = u * S + (row - o * S), m = qpos - a.pl;
                const float v = acc[i][j][r];
                if (m >= 0 && m < a.Tx) {
                    float g = v;
                    if (EPI & P_XACT) g *= act_grad(a.act, e0[r]);
                    a.out[((int64_t)b * a.Co + o) * a.Tx + m] = g + e1[r];
                } else if (qpos >= 0 && qpos < a.pl + a.Tx + a.pr) {
                    const int slot = m < 0 ? qpos : a.pl + (m - a.Tx);
                    a.side[((int64_t)b * a.Co + o) * (a.pl + a.pr) + slot] = v;
                }
            }
        }
}

__global__ void conv_poly_reduce(PolyArgs a) {
    const int64_t n = (int64_t)a.B * a.Co * a.Q;
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float v = sum_strided(a.part + i, a.KS, n);
    const int qpos = (int)(i % a.Q);
    const int64_t bo = i / a.Q;
    poly_store(a, (int)(bo / a.Co), (int)(bo % a.Co), qpos, v);
}

// Add the gradients that landed on pad positions back onto their reflect sources, in slot
// order (deterministic). One thread per (b, channel) row.
__global__ void conv_fold_edges(const float* side, const float* xact, float* dx, int rows, int Tx,
                                int pl, int pr, int e, int mode, int act) {
    int row = blockIdx.x * blockDim.x + threadIdx.x;
    if (row >= rows) return;
    const int np = pl + pr;
    for (int slot = 0; slot < np; ++slot) {
        int qpos = slot < pl ? slot : pl + Tx + (slot - pl);
        int m = pad_src(qpos, pl, Tx, e, mode);
        if (m < 0) continue;
        int64_t idx = (int64_t)row * Tx + m;
        float g = side[(int64_t)row * np + slot];
        if (act != ENCX_ACT_NONE) g *= act_grad(act, xact[idx]);
        dx[idx] += g;
    }
}

// ------------------------------------------------------------------------- weight grad
struct WgArgs {
    const float* L;  // [B][A][Tl]
    const float* R;  // [B][C][Tr]
    float* ws;       // [S][A][C*K]
    int B, A, Tl, C, Tr, K, s, d, pl, e, mode, actL, actR;
    int BT;          // t per LDS chunk (even)
    int items;       // total work items = B * ceil(Tl / BT)
    int per_split;   // work items per split
    int WLp;         // LDS row length of the R window
    int NCmax;       // R window rows
    int vec;         // L / R rows 16-B aligned: float4 staging loads
    float* wsb;      // non-null: also sum L over t (the bias grad of a conv, L = dy) into
                     // wsb[split][A] (the ones column of the GEMM, on the vector ALU)
};

// WK > 1: the WK waves share one (32*TM) x (32*TN) tile and split each chunk's t range.
// L is staged as Ls[a][t] (row stride BT + 1: the MFMA A reads, 32 lanes down a column, hit
// 32 banks; the staging writes run along t) and R as Rs[c][window]; both from float4 items.
template <int BM, int BN, int WM, int WN, int WK>
__global__ __launch_bounds__(NT) void conv_wgrad_kernel(WgArgs a) {
    constexpr int TM = BM / WM / 32, TN = BN / WN / 32;
    static_assert(WM * WN * WK == 4, "4 waves");
    extern __shared__ float smem[];
    const int BT = a.BT, BTp = BT + 1, WLp = a.WLp, K = a.K, N = a.C * a.K;
    float* Ls = smem;              // [BM][BTp]
    float* Rs = smem + BM * BTp;   // [NCmax][WLp]
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wk = wave % WK, wmn = wave / WK;
    const int wm0 = (wmn / WN) * TM * 32, wn0 = (wmn % WN) * TN * 32;
    const int a0 = blockIdx.y * BM, n0 = blockIdx.x * BN, split = blockIdx.z;
    const int c_first = n0 / K;
    const int nchunks_t = (a.Tl + BT - 1) / BT;
    const int h = lane >> 5, l32 = lane & 31;

    int boff[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) {
        int n = n0 + wn0 + j * 32 + l32;
        int c = n / K, k = n - c * K;
        boff[j] = (c - c_first) * WLp + k * a.d;
        if (n >= N) boff[j] = 0;
    }
    f32x16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = (f32x16){0};
    // bias grad: the first column tile's waves that hold column 0 sum the A operand they load
    const bool bias_blk = a.wsb && blockIdx.x == 0;
    const bool do_bias = bias_blk && wn0 == 0;
    float bsum[TM];
#pragma unroll
    for (int i = 0; i < TM; ++i) bsum[i] = 0.f;

    const int it_beg = split * a.per_split;
    const int it_end = min(a.items, it_beg + a.per_split);
    const int WL = (BT - 1) * a.s + (K - 1) * a.d + 1;
    const int tw = BT / WK;  // t per wave per chunk
    const int BT4 = BT / 4, nl = BM * BT4;
    // R window items: tc*s is a multiple of 4, so the window's offset from its aligned floor
    // is the same for every chunk
    const int woff = (4 - (a.pl & 3)) & 3;
    const int nv = (woff + WL + 3) >> 2, nr = a.NCmax * nv;
    const int dal = NT / BT4, dti = NT - dal * BT4, lal0 = tid / BT4, lti0 = tid - lal0 * BT4;
    const int dcr = NT / nv, dvr = NT - dcr * nv, rcr0 = tid / nv, rvi0 = tid - rcr0 * nv;
    for (int it = it_beg; it < it_end; ++it) {
        const int b = it / nchunks_t, tc = (it - b * nchunks_t) * BT;
        const float* Lb = a.L + (int64_t)b * a.A * a.Tl;
        const float* Rb = a.R + (int64_t)b * a.C * a.Tr;
        __syncthreads();
        // batched staging as in conv_fwd_kernel: SPER float4 loads in flight per thread; items
        // (row, column) walked by a fixed step of NT (no per-item division)
        {
            int al_n = lal0, ti_n = lti0;
            for (int i0 = 0; i0 < nl; i0 += NT * SPER) {
                f32x4 v[SPER];
                int alq[SPER], tq[SPER];
#pragma unroll
                for (int q = 0; q < SPER; ++q) {
                    alq[q] = al_n;
                    tq[q] = tc + 4 * ti_n;
                    ti_n += dti;
                    al_n += dal;
                    if (ti_n >= BT4) {
                        ti_n -= BT4;
                        ++al_n;
                    }
                }
#pragma unroll
                for (int q = 0; q < SPER; ++q) {
                    const int t = tq[q], aa = a0 + alq[q];
                    const bool ok = alq[q] < BM && aa < a.A;
                    v[q] = (f32x4){0.f, 0.f, 0.f, 0.f};
                    if (a.vec) {
                        const int tcl = t + 3 < a.Tl ? t : a.Tl - 4;
                        const f32x4 x = *(const f32x4*)(Lb + (int64_t)(ok ? aa : a0) * a.Tl + tcl);
                        if (ok && t + 3 < a.Tl) v[q] = x;
                    }
                }
#pragma unroll
                for (int q = 0; q < SPER; ++q) {
                    const int t = tq[q], aa = a0 + alq[q];
                    if (alq[q] < BM && aa < a.A && !(a.vec && t + 3 < a.Tl)) {
                        const float* lr = Lb + (int64_t)aa * a.Tl;
                        for (int e = 0; e < 4; ++e) v[q][e] = t + e < a.Tl ? lr[t + e] : 0.f;
                    }
                }
#pragma unroll
                for (int q = 0; q < SPER; ++q) {
                    if (alq[q] >= BM) continue;
                    float* ls = Ls + alq[q] * BTp + (tq[q] - tc);
                    ls[0] = act_apply(a.actL, v[q][0]);
                    ls[1] = act_apply(a.actL, v[q][1]);
                    ls[2] = act_apply(a.actL, v[q][2]);
                    ls[3] = act_apply(a.actL, v[q][3]);
                }
            }
        }
        const int base = tc * a.s - a.pl - woff;  // input index of the first item's element 0
        {
            int cr_n = rcr0, vi_n = rvi0;
            for (int i0 = 0; i0 < nr; i0 += NT * SPER) {
                f32x4 v[SPER];
                int crq[SPER], viq[SPER];
#pragma unroll
                for (int q = 0; q < SPER; ++q) {
                    crq[q] = cr_n;
                    viq[q] = vi_n;
                    vi_n += dvr;
                    cr_n += dcr;
                    if (vi_n >= nv) {
                        vi_n -= nv;
                        ++cr_n;
                    }
                }
#pragma unroll
                for (int q = 0; q < SPER; ++q) {
                    const int c = c_first + crq[q], p = base + 4 * viq[q];
                    const bool ok = crq[q] < a.NCmax && c < a.C;
                    v[q] = (f32x4){0.f, 0.f, 0.f, 0.f};
                    if (a.vec) {
                        const int pc = p < 0 ? 0 : (p > a.Tr - 4 ? a.Tr - 4 : p);
                        const f32x4 x = *(const f32x4*)(Rb + (int64_t)(ok ? c : c_first) * a.Tr + pc);
                        if (ok && p >= 0 && p + 3 < a.Tr) v[q] = x;
                    }
                }
#pragma unroll
                for (int q = 0; q < SPER; ++q) {
                    const int c = c_first + crq[q], p = base + 4 * viq[q];
                    if (crq[q] < a.NCmax && c < a.C && !(a.vec && p >= 0 && p + 3 < a.Tr)) {
                        const float* rr = Rb + (int64_t)c * a.Tr;
                        for (int e = 0; e < 4; ++e) {
                            const int m = pad_src(p + e + a.pl, a.pl, a.Tr, a.e, a.mode);
                            v[q][e] = m >= 0 ? rr[m] : 0.f;
                        }
                    }
                }
#pragma unroll
                for (int q = 0; q < SPER; ++q) {
                    if (crq[q] >= a.NCmax) continue;
                    float* rs = Rs + crq[q] * WLp;
                    const int q0 = 4 * viq[q] - woff;
                    for (int e = 0; e < 4; ++e) {
                        const int qq = q0 + e;
                        if (qq >= 0 && qq < WL) rs[qq] = act_apply(a.actR, v[q][e]);
                    }
                }
            }
        }
        __syncthreads();
#pragma unroll 4
        for (int tp = wk * tw; tp < (wk + 1) * tw; tp += 2) {
            const int tl = tp + h;
            float av[TM], bv[TN];
#pragma unroll
            for (int i = 0; i < TM; ++i) av[i] = Ls[(wm0 + i * 32 + l32) * BTp + tl];
            if (do_bias)
#pragma unroll
                for (int i = 0; i < TM; ++i) bsum[i] += av[i];
#pragma unroll
            for (int j = 0; j < TN; ++j) bv[j] = Rs[boff[j] + tl * a.s];
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j) acc[i][j] = mfma32(av[i], bv[j], acc[i][j]);
        }
    }
    if (bias_blk) {  // the bias column: halves (even / odd t), then the WK waves in order
        __shared__ float bred[4][128];
        __syncthreads();
        if (do_bias)
#pragma unroll
            for (int i = 0; i < TM; ++i) {
                const float v = bsum[i] + __shfl_xor(bsum[i], 32, 64);
                if (h == 0) bred[wave][wm0 + i * 32 + l32] = v;
            }
        __syncthreads();
        if (tid < BM && a0 + tid < a.A) {
            const int wrow = tid / (TM * 32);  // the wave row (of WM) holding this tile row
            float v = 0.f;
            for (int w = 0; w < WK; ++w) v += bred[(wrow * WN) * WK + w][tid];
            a.wsb[(int64_t)split * a.A + a0 + tid] = v;
        }
    }
    if (WK > 1) {  // combine the waves' partial tiles in wave order (deterministic)
        __syncthreads();
        float* red = smem;  // [WM*WN][WK][TM*TN*16][64]
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j)
#pragma unroll
                for (int r = 0; r < 16; ++r)
                    red[(((wmn * WK + wk) * TM * TN + i * TN + j) * 16 + r) * 64 + lane] = acc[i][j][r];
        __syncthreads();
        if (wk != 0) return;
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    float v = red[(((wmn * WK) * TM * TN + i * TN + j) * 16 + r) * 64 + lane];
                    for (int w = 1; w < WK; ++w)
                        v += red[(((wmn * WK + w) * TM * TN + i * TN + j) * 16 + r) * 64 + lane];
                    acc[i][j][r] = v;
                }
    }
    float* wsb = a.ws + (int64_t)split * a.A * N;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int n = n0 + wn0 + j * 32 + l32;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int aa = a0 + wm0 + i * 32 + mfma_row(r, lane);
                if (aa < a.A && n < N) wsb[(int64_t)aa * N + n] = acc[i][j][r];
            }
        }
}

// VALU weight grad for tiny A*N (first / last conv of the stack): thread per output element.
// The chunk's L and R windows are staged SB elements per thread at a time, every load issued
// before the first is used (a loop of single loads waited out one memory round trip per element:
// 33 in a row per thread for the R window of the last conv).
// KW > 0 (stride 1, dilation 1, K == KW, A*C <= NT): thread (pair p = tid % P of (a, c), segment
// sg = tid / P of the chunk's t range) keeps a KW-wide window of its R row in registers and
// accumulates all KW taps of its pair: 2 LDS reads per t instead of 2 per (t, tap); the segments'
// partials are summed in segment order at the end (deterministic).
constexpr int SMALL_BT = 256;  // t per chunk (plan_wgrad's kind 0)
constexpr int SB = 8;
template <int KW>
__global__ __launch_bounds__(NT) void conv_wgrad_small_kernel(WgArgs a) {
    extern __shared__ float smem[];
    constexpr int BT = SMALL_BT;
    const int K = a.K, N = a.C * K, AN = a.A * N;
    constexpr int LST = BT + 1;     // Ls row stride: the rows of one wave's threads on distinct banks
    float* Ls = smem;               // [A][LST]
    float* Rs = smem + a.A * LST;   // [C][WLp]
    const int split = blockIdx.x, tid = threadIdx.x;
    const int nchunks_t = (a.Tl + BT - 1) / BT;
    const int WL = (BT - 1) * a.s + (K - 1) * a.d + 1;
    const int nl = a.A * BT, nr = a.C * WL;
    float acc = 0.f, bacc = 0.f;  // AN (+ A with the bias) <= NT
    float wacc[KW > 0 ? KW : 1];
#pragma unroll
    for (int k = 0; k < (KW > 0 ? KW : 1); ++k) wacc[k] = 0.f;
    const int it_beg = split * a.per_split, it_end = min(a.items, it_beg + a.per_split);
    for (int it = it_beg; it < it_end; ++it) {
        const int b = it / nchunks_t, tc = (it - b * nchunks_t) * BT;
        const float* Lb = a.L + (int64_t)b * a.A * a.Tl;
        const float* Rb = a.R + (int64_t)b * a.C * a.Tr;
        __syncthreads();
        for (int i0 = 0; i0 < nl; i0 += NT * SB) {
            float v[SB];
            bool ok[SB];
#pragma unroll
            for (int q = 0; q < SB; ++q) {
                const int i = i0 + q * NT + tid, al = i / BT, t = tc + (i - al * BT);
                ok[q] = i < nl && t < a.Tl;
                v[q] = Lb[ok[q] ? (int64_t)al * a.Tl + t : 0];  // no branch around the load
            }
#pragma unroll
            for (int q = 0; q < SB; ++q) {
                const int i = i0 + q * NT + tid, al = i / BT;
                if (i < nl) Ls[i + al] = ok[q] ? act_apply(a.actL, v[q]) : 0.f;
            }
        }
        // (c, w) of element i0 + tid, advanced by NT elements per step without a division
        const int dc = NT / WL, dw = NT - dc * WL;
        int c_n = tid / WL, w_n = tid - (tid / WL) * WL;
        for (int i0 = 0; i0 < nr; i0 += NT * SB) {
            float v[SB];
            int cq[SB], wq[SB], mq[SB];
#pragma unroll
            for (int q = 0; q < SB; ++q) {
                cq[q] = c_n;
                wq[q] = w_n;
                w_n += dw;
                c_n += dc;
                if (w_n >= WL) {
                    w_n -= WL;
                    ++c_n;
                }
                const int m = cq[q] < a.C ? pad_src(tc * a.s + wq[q], a.pl, a.Tr, a.e, a.mode) : -1;
                mq[q] = m;
                v[q] = Rb[m >= 0 ? (int64_t)cq[q] * a.Tr + m : 0];
            }
#pragma unroll
            for (int q = 0; q < SB; ++q)
                if (cq[q] < a.C) Rs[cq[q] * a.WLp + wq[q]] = mq[q] >= 0 ? act_apply(a.actR, v[q]) : 0.f;
        }
        __syncthreads();
        if (KW > 0) {
            const int P = a.A * a.C, seg = NT / P, TS = (BT + seg - 1) / seg;
            const int pp = tid % P, sg = tid / P, aa = pp / a.C, c = pp - aa * a.C;
            if (sg < seg) {
                const int tb = sg * TS, te = min(BT, tb + TS);
                const float* lp = Ls + aa * LST;
                const float* rp = Rs + c * a.WLp;
                float win[KW > 0 ? KW : 1];
#pragma unroll
                for (int k = 0; k + 1 < KW; ++k) win[k] = rp[tb + k];
                for (int tl = tb; tl < te; ++tl) {
                    win[KW - 1] = rp[tl + KW - 1];
                    const float l = lp[tl];
#pragma unroll
                    for (int k = 0; k < KW; ++k) wacc[k] = fmaf(l, win[k], wacc[k]);
                    bacc += l;
#pragma unroll
                    for (int k = 0; k + 1 < KW; ++k) win[k] = win[k + 1];
                }
            }
            continue;
        }
        if (a.wsb && tid >= AN && tid < AN + a.A) {  // bias: sum of the L row over the chunk
            const float* lp = Ls + (tid - AN) * LST;
            float s0 = 0.f, s1 = 0.f;
            for (int tl = 0; tl < BT; tl += 2) {
                s0 += lp[tl];
                s1 += lp[tl + 1];
            }
            bacc += s0 + s1;
        }
        if (tid < AN) {
            int aa = tid / N, n = tid - aa * N, c = n / K, k = n - c * K;
            const float* lp = Ls + aa * LST;
            const float* rp = Rs + c * a.WLp + k * a.d;
            float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;  // 4 independent chains
            for (int tl = 0; tl < BT; tl += 4) {
                s0 = fmaf(lp[tl], rp[tl * a.s], s0);
                s1 = fmaf(lp[tl + 1], rp[(tl + 1) * a.s], s1);
                s2 = fmaf(lp[tl + 2], rp[(tl + 2) * a.s], s2);
                s3 = fmaf(lp[tl + 3], rp[(tl + 3) * a.s], s3);
            }
            acc += (s0 + s1) + (s2 + s3);
        }
    }
    if (KW > 0) {  // the segments' partials: red[sg][pp][k] (k = KW: the bias sum), summed in sg order
        const int P = a.A * a.C, seg = NT / P;
        __syncthreads();
        float* red = smem;
        if (tid < seg * P) {
#pragma unroll
            for (int k = 0; k < KW; ++k) red[tid * (KW + 1) + k] = wacc[k];
            red[tid * (KW + 1) + KW] = bacc;
        }
        __syncthreads();
        if (tid < P * KW) {  // output tid = pp * K + k (= aa * N + c * K + k)
            const int pp = tid / KW, k = tid - pp * KW;
            float v = 0.f;
            for (int sg = 0; sg < seg; ++sg) v += red[(sg * P + pp) * (KW + 1) + k];
            a.ws[(int64_t)split * AN + tid] = v;
        }
        if (a.wsb && tid < a.A) {  // bias of row aa: the pairs (aa, c = 0)
            float v = 0.f;
            for (int sg = 0; sg < seg; ++sg) v += red[(sg * P + tid * a.C) * (KW + 1) + KW];
            a.wsb[(int64_t)split * a.A + tid] = v;
        }
        return;
    }
    if (tid < AN) a.ws[(int64_t)split * AN + tid] = acc;
    if (a.wsb && tid >= AN && tid < AN + a.A) a.wsb[(int64_t)split * a.A + (tid - AN)] = bacc;
}

// dw[i] = [acc ? dw : 0] + sum_s ws[s][i] (slab_sum_256_d: 64 outputs per block, 4 split slices,
// fixed order, fp64 accumulation: at B 32 the high-rate layers' grads sum 768 k positions through
// hundreds of slabs); blocks past cdiv(AN, 64) reduce the bias slabs wsb[s][A] into db the same way.
__global__ __launch_bounds__(256) void wgrad_reduce(const float* ws, float* dw, int64_t AN, int S, int accumulate,
                                                    const float* wsb, float* db, int A, int acc_b) {
    __shared__ double red[256];
    const int64_t nbw = (AN + 63) / 64;
    if (blockIdx.x >= nbw) {
        const int i = (int)((blockIdx.x - nbw) * 64) + (threadIdx.x & 63);
        const bool valid = i < A;
        const float v = slab_sum_256_d(wsb + (valid ? i : 0), S, A, valid, red);
        if (threadIdx.x < 64 && valid) db[i] = acc_b ? db[i] + v : v;
        return;
    }
    const int64_t i = (int64_t)blockIdx.x * 64 + (threadIdx.x & 63);
    const bool valid = i < AN;
    const float v = slab_sum_256_d(ws + (valid ? i : 0), S, AN, valid, red);
    if (threadIdx.x < 64 && valid) dw[i] = accumulate ? dw[i] + v : v;
}

// VALU forward for Cout <= 4 (decoder's final 32 -> 1 conv): thread per output sample.
__global__ __launch_bounds__(NT) void conv_fwd_small_kernel(FwdArgs a) {
    extern __shared__ float smem[];
    const int K = a.K, S = a.s, CK = a.CK;
    const int WL = (NT - 1) * S + (K - 1) * a.d + 1;
    float* Xs = smem;            // [CK][WL]
    float* Wsm = smem + CK * WL; // [Cout][CK][K]
    const int tid = threadIdx.x, t0 = blockIdx.x * NT, b = blockIdx.z;
    const float* xb = a.x + (int64_t)b * a.Cin * a.Tin;
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    for (int c0 = 0; c0 < a.Cin; c0 += CK) {
        __syncthreads();
        // SB loads in flight per thread (as conv_wgrad_small_kernel); (cl, w) stepped without a division
        {
            const int dc = NT / WL, dw = NT - dc * WL;
            int cl_n = tid / WL, w_n = tid - (tid / WL) * WL;
            for (int i0 = 0; i0 < CK * WL; i0 += NT * SB) {
                float v[SB];
                int iq[SB], mq[SB];
#pragma unroll
                for (int q = 0; q < SB; ++q) {
                    const int cl = cl_n, w = w_n, c = c0 + cl;
                    w_n += dw;
                    cl_n += dc;
                    if (w_n >= WL) {
                        w_n -= WL;
                        ++cl_n;
                    }
                    iq[q] = cl < CK ? cl * WL + w : -1;
                    const int m = (cl < CK && c < a.Cin) ? pad_src(t0 * S + w, a.pl, a.Tin, a.e, a.mode) : -1;
                    mq[q] = m;
                    v[q] = xb[m >= 0 ? (int64_t)c * a.Tin + m : 0];  // no branch around the load
                }
#pragma unroll
                for (int q = 0; q < SB; ++q)
                    if (iq[q] >= 0) Xs[iq[q]] = mq[q] >= 0 ? act_apply(a.act, v[q]) : 0.f;
            }
        }
        for (int i = tid; i < a.Cout * CK * K; i += NT) {
            int co = i / (CK * K), r = i - co * CK * K, cl = r / K, k = r - cl * K, c = c0 + cl;
            Wsm[i] = c < a.Cin ? a.wf[((int64_t)c * K + k) * a.Cout + co] : 0.f;
        }
        __syncthreads();
        for (int co = 0; co < a.Cout; ++co) {
            float s = acc[co];
            for (int cl = 0; cl < CK; ++cl) {
                const float* xr = Xs + cl * WL + tid * S;
                const float* wr = Wsm + (co * CK + cl) * K;
                for (int k = 0; k < K; ++k) s = fmaf(wr[k], xr[k * a.d], s);
            }
            acc[co] = s;
        }
    }
    const int t = t0 + tid;
    if (t < a.Tout)
        for (int co = 0; co < a.Cout; ++co)
            fwd_store(a, ((int64_t)b * a.Cout + co) * a.Tout + t, co, acc[co]);
}

// ------------------------------------------------------------------------- low-rate layers
// At T = 75 (B = 32) a per-item time tile is mostly padding and the weights are re-staged for
// every 32 columns. These layers run instead as one GEMM over the flattened (b, t) columns
// (N = B*T = 2400) with an im2col B operand gathered from L2 while staging, split over the
// reduction into fixed slabs (conv_fwd_reduce / conv_poly_reduce apply the epilogue).
// (the flattened indices split by FastDiv: a runtime integer division per staged element made
// these GEMMs VALU-bound)
struct LdConvFlat {
    static constexpr bool A_K_FAST = false, B_N_FAST = true;
    FwdArgs p;
    FastDiv fk, ft;  // by K, by Tout
    ENCX_DEV float a(int m, int k) const { return p.wf[(int64_t)k * p.Cout + m]; }
    ENCX_DEV float b(int k, int n) const {
        const int ci = (int)fdiv((uint32_t)k, fk), tap = k - ci * p.K;
        const int bb = (int)fdiv((uint32_t)n, ft), t = n - bb * p.Tout;
        const int m = pad_src(t * p.s + tap * p.d, p.pl, p.Tin, p.e, p.mode);
        const float v = p.x[((int64_t)bb * p.Cin + ci) * p.Tin + (m >= 0 ? m : 0)];  // no branch around the load
        return m >= 0 ? act_apply(p.act, v) : 0.f;
    }
};
struct EpConvFlat {
    FwdArgs p;
    int slabs;
    FastDiv ft;
    ENCX_DEV void pre(int co, int n, float* l) const {
        const int bb = (int)fdiv((uint32_t)n, ft), t = n - bb * p.Tout;
        const int64_t o = ((int64_t)bb * p.Cout + co) * p.Tout + t;
        const bool fin = slabs == 1;
        l[0] = (fin && p.bias) ? p.bias[co] : 0.f;
        l[1] = (fin && p.xact) ? p.xact[o] : 0.f;
        l[2] = (fin && p.res) ? p.res[o] : 0.f;
        l[3] = (fin && p.accumulate) ? p.y[o] : 0.f;
    }
    ENCX_DEV void post(int co, int n, float v, const float* l) const {
        const int bb = (int)fdiv((uint32_t)n, ft), t = n - bb * p.Tout;
        const int64_t o = ((int64_t)bb * p.Cout + co) * p.Tout + t;
        if (slabs > 1) {
            p.part[(int64_t)blockIdx.z * p.B * p.Cout * p.Tout + o] = v;
            return;
        }
        v += l[0];
        if (p.xact) v *= act_grad(p.epi_act, l[1]);
        p.y[o] = v + l[2] + l[3];
    }
    ENCX_DEV void operator()(int co, int n, float v) const {
        float l[4];
        pre(co, n, l);
        post(co, n, v, l);
    }
};
struct LdPolyFlat {
    static constexpr bool A_K_FAST = false, B_N_FAST = true;
    PolyArgs p;
    int M, ncols;
    FastDiv fj, fc;  // by J, by ncols
    ENCX_DEV float a(int m, int k) const { return p.wp[(int64_t)k * M + m]; }
    ENCX_DEV float b(int k, int n) const {
        const int i = (int)fdiv((uint32_t)k, fj), q = k - i * p.J;
        const int bb = (int)fdiv((uint32_t)n, fc), u = n - bb * ncols, t = u - q;
        const bool in = t >= 0 && t < p.Tin;
        const float v = p.in[((int64_t)bb * p.Ci + i) * p.Tin + (in ? t : 0)];  // no branch around the load
        return in ? act_apply(p.in_act, v) : 0.f;
    }
};
struct EpPolyFlat {
    PolyArgs p;
    int ncols, slabs;
    FastDiv fs, fc;  // by s, by ncols
    ENCX_DEV void pre(int row, int n, float* l) const {
        const int o = (int)fdiv((uint32_t)row, fs), rr = row - o * p.s;
        const int bb = (int)fdiv((uint32_t)n, fc), u = n - bb * ncols, qpos = u * p.s + rr;
        l[0] = l[1] = 0.f;
        if (slabs > 1) return;
        if (p.mode == 0) {
            l[0] = p.bias ? p.bias[o] : 0.f;
        } else {
            const int m = qpos - p.pl;
            if (m >= 0 && m < p.Tx) {
                const int64_t idx = ((int64_t)bb * p.Co + o) * p.Tx + m;
                if (p.act != ENCX_ACT_NONE) l[0] = p.xact[idx];
                if (p.accumulate) l[1] = p.out[idx];
            }
        }
    }
    ENCX_DEV void post(int row, int n, float v, const float* l) const {
        const int o = (int)fdiv((uint32_t)row, fs), rr = row - o * p.s;
        const int bb = (int)fdiv((uint32_t)n, fc), u = n - bb * ncols, qpos = u * p.s + rr;
        if (slabs > 1) {
            if (qpos < p.Q) p.part[(((int64_t)blockIdx.z * p.B + bb) * p.Co + o) * p.Q + qpos] = v;
            return;
        }
        if (p.mode == 0) {
            const int q = qpos - p.trim;
            if (q >= 0 && q < p.Tout) p.out[((int64_t)bb * p.Co + o) * p.Tout + q] = v + l[0];
        } else {
            const int m = qpos - p.pl;
            if (m >= 0 && m < p.Tx) {
                float g = v;
                if (p.act != ENCX_ACT_NONE) g *= act_grad(p.act, l[0]);
                p.out[((int64_t)bb * p.Co + o) * p.Tx + m] = g + l[1];
            } else if (qpos >= 0 && qpos < p.pl + p.Tx + p.pr) {
                const int slot = m < 0 ? qpos : p.pl + (m - p.Tx);
                p.side[((int64_t)bb * p.Co + o) * (p.pl + p.pr) + slot] = v;
            }
        }
    }
    ENCX_DEV void operator()(int row, int n, float v) const {
        float l[2];
        pre(row, n, l);
        post(row, n, v, l);
    }
};

// ------------------------------------------------------------------------- short-T layers, library GEMM
// The flattened layers with a large reduction (the k16 s8 stage at T 75: forward 512 x 2400 x
// 4096, bwd-data and the transposed conv's polyphase 2048 x 2400 x 1024, their weight grads) as
// im2col -> hipBLASLt -> epilogue: the flat loaders' gathers (pad modes, pre-activation) written
// once into the workspace as a plain [N][Kred] matrix, the library's fp32 GEMM (blas.hip: 107-119
// TF/s at these shapes against ~45 for the flattened implicit GEMM), then the flat epilogues
// (bias, act'(xact), residual, accumulate, the polyphase fold and side columns) applied while
// transposing the [N][M] product back through LDS.
constexpr int WGB_ROWS = 160;  // positions per bias-partial chunk (blas_wgrad_run)
static bool blas_flat_ok(int64_t M, int64_t N, int64_t Kred) {
    return (encx_opt(OPT_BLAS) & 2) && M >= 256 && Kred >= 512 && 2.0 * M * N * Kred >= 2.0e9;
}
// the longer layers (option BLAS & 4): 256+ output rows, a reduction of 512+, an im2col of at
// most 128 MB and 8+ GFLOP (the k10 s5 stage at T 600: 256 x 19200 x 1280 and 640 x 19200 x 512)
static bool blas_big_ok(int64_t M, int64_t N, int64_t Kred) {
    return (encx_opt(OPT_BLAS) & 4) && M >= 256 && Kred >= 512 && N * Kred <= (32ll << 20) &&
           2.0 * M * N * Kred >= 8.0e9;
}
// The reduction is cut into KB equal chunks (a strided batch of library GEMMs into KB product
// slabs, summed in order in fp64 by the epilogue / reduce): one library accumulation chain over
// all 4096 reduction elements (or 2400 positions) was 5-7x the error of plain fp32 in the config-3
// step check. KB: up to 8, chunks of at least 256, at most 48 MB of slabs.
static int blas_chunks(int64_t K, int64_t slab_elems) {
    for (const int c : {8, 6, 4, 3, 2})
        if (K % c == 0 && K / c >= 256 && (size_t)c * slab_elems * sizeof(float) <= (48ull << 20)) return c;
    return 1;
}
static size_t blas_flat_ws(int64_t M, int64_t N, int64_t Kred) {
    if (!blas_flat_ok(M, N, Kred) && !blas_big_ok(M, N, Kred)) return 0;
    return (size_t)(N * Kred + (int64_t)blas_chunks(Kred, N * M) * N * M) * sizeof(float);
}
// out[n][k] = ld.b(k, n): a wave per 4 columns n, lanes along k (one (ci, tap) run per lane group)
template <class Ld>
__global__ __launch_bounds__(256) void im2col_kernel(Ld ld, int Kred, int N, float* out) {
    const int k = blockIdx.x * 64 + (threadIdx.x & 63), n0 = blockIdx.y * 16 + (threadIdx.x >> 6) * 4;
    if (k >= Kred) return;
#pragma unroll
    for (int j = 0; j < 4; ++j)
        if (n0 + j < N) out[(int64_t)(n0 + j) * Kred + k] = ld.b(k, n0 + j);
}
// ep(m, n, sum_s Cm[s][n][m]) for the KB slabs of the [N][M] product (summed in slab order in
// fp64), a 32 x 32 tile transposed through LDS so that the epilogue's stores run along n (t)
template <class Ep>
__global__ __launch_bounds__(256) void gemm_epi_kernel(Ep ep, const float* Cm, int M, int N, int KB) {
    __shared__ float tile[32][33];
    const int m0 = blockIdx.x * 32, n0 = blockIdx.y * 32, tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
    const int64_t NM = (int64_t)N * M;
#pragma unroll
    for (int r = ty; r < 32; r += 8) {
        double v = 0.0;
        if (n0 + r < N && m0 + tx < M) {
            const float* c = Cm + (int64_t)(n0 + r) * M + m0 + tx;
            for (int sl = 0; sl < KB; ++sl) v += (double)c[sl * NM];
        }
        tile[r][tx] = (float)v;
    }
    __syncthreads();
#pragma unroll
    for (int r = ty; r < 32; r += 8)
        if (m0 + r < M && n0 + tx < N) ep(m0 + r, n0 + tx, tile[tx][r]);
}
template <class Ld, class Ep>
static int blas_flat_run(const Ld& ld, const Ep& ep, const float* wA, int M, int N, int Kred, float* ws,
                         hipStream_t st) {
    float* Xc = ws;
    float* Cm = ws + (int64_t)N * Kred;
    hipLaunchKernelGGL(im2col_kernel<Ld>, dim3((unsigned)cdiv(Kred, 64), (unsigned)cdiv(N, 16)), dim3(256), 0, st,
                       ld, Kred, N, Xc);
    ENCX_CHECK_LAUNCH();
    // slab c of Cm (M x N, column-major) = wA (M x Kred, column-major: the weights [Kred][M]) Xc^T
    // over reduction chunk c
    const int KB = blas_chunks(Kred, (int64_t)N * M), kc = Kred / KB;
    if (encx_sgemm(st, false, false, M, N, kc, wA, M, Xc, Kred, Cm, M, false, KB, (int64_t)kc * M, kc,
                   (int64_t)N * M))
        return -1;
    hipLaunchKernelGGL(gemm_epi_kernel<Ep>, dim3((unsigned)cdiv(M, 32), (unsigned)cdiv(N, 32)), dim3(256), 0, st,
                       ep, Cm, M, N, KB);
    ENCX_CHECK_LAUNCH();
    return 0;
}

// ------------------------------------------------------------------------- planning
static int even_up(int v) { return (v + 1) & ~1; }

// channels per LDS stage: ~64 reduction elements, even, and preferably dividing C exactly
// (a ragged last chunk is zero-padded MFMA work)
static int pick_ck(int C, int taps) {
    int cap = (int)encx_opt(OPT_CONV_CK) / taps;  // default 64 reduction elements
    if (cap < 2) cap = 2;
    cap = even_up(cap);
    if (cap >= C) return even_up(C);
    for (int ck = cap & ~1; ck >= 2; ck -= 2)
        if (C % ck == 0 && ck * 2 >= cap) return ck;
    return cap & ~1;
}

enum Tile { T32x128, T64x64, T64x128, T128x32, T128x64, T128x128 };
static Tile pick_tile(int64_t M, int64_t N) {
    if (N <= 96) return T128x32;
    if (M <= 32) return T32x128;
    if (M <= 64) return T64x128;
    return T128x128;
}
static int tile_bm(Tile t) { return (t == T32x128) ? 32 : (t == T64x64 || t == T64x128) ? 64 : 128; }
static int tile_bn(Tile t) { return (t == T128x32) ? 32 : (t == T64x64 || t == T128x64) ? 64 : 128; }

// Split the channel reduction (split-K into partial slabs + a fixed-order reduce that applies the
// epilogue) when the plain grid would underfill the chip. The slabs cost KS x the output in
// writes and reads, so (round 5, tools/conv_sweep.py on every config-3 layer):
//  * split only below CONV_SPLIT / 2 workgroups (default 512: two per CU) -- or below CONV_SPLIT
//    (1024) when the direct epilogue reads operands (act'(x), residual, accumulate: its loads
//    wait out a round trip per sub-tile at the end of every workgroup, which the streaming
//    reduce does not);
//  * keep >= 192 reduction elements (channels x taps) per split and <= 1536 workgroups;
//  * split evenly: KS divides the channel chunks (an uneven last split idles the others).
// Measured against the round-4 rule (split up to 1024 workgroups): 8.76 -> 8.3-8.5 ms per step.
static void plan_split(int64_t blocks, int C, int CK, int red, bool heavy_epi, int* KS, int* cps) {
    const int nch = (C + CK - 1) / CK;
    const int64_t target = encx_opt(OPT_CONV_SPLIT);
    int ks = 1;
    if (blocks < (heavy_epi ? target : target / 2) && nch >= 4) {
        int64_t cap = red / 192;
        if (cap > (3 * target / 2) / blocks) cap = (3 * target / 2) / blocks;
        if (cap > nch / 2) cap = nch / 2;
        if (cap > 16) cap = 16;
        for (ks = (int)(cap < 1 ? 1 : cap); ks > 1 && nch % ks; --ks) {
        }
    }
    const int per = (int)cdiv(nch, ks);
    *cps = per * CK;
    *KS = (int)cdiv(C, *cps);
}

struct FwdPlan { Tile t; int CK, Up, KS, cps; bool small; };
static FwdPlan plan_fwd(int64_t B, int64_t Cin, int64_t Cout, int64_t Tout, int64_t K, int64_t s,
                        int64_t d, bool heavy_epi) {
    FwdPlan p;
    p.small = Cout <= 4;
    const int ck = pick_ck((int)Cin, (int)K);
    p.CK = ck;
    p.t = pick_tile(Cout, Tout);
    int BN = tile_bn(p.t);
    p.Up = BN + (int)(((K - 1) * d) / s) + 1;
    if ((p.Up & 31) == 0) p.Up += 1;
    int64_t blocks = cdiv(Tout, BN) * cdiv(Cout, tile_bm(p.t)) * B;
    p.KS = 1;
    p.cps = (int)Cin;
    if (!p.small) plan_split(blocks, (int)Cin, ck, (int)(Cin * K), heavy_epi, &p.KS, &p.cps);
    return p;
}

struct PolyPlan { Tile t; int CK, Ub, KS, cps; };
static PolyPlan plan_poly(int64_t B, int64_t Ci, int64_t M, int64_t ncols, int64_t J, bool heavy_epi) {
    PolyPlan p;
    const int ck = pick_ck((int)Ci, (int)J);
    p.CK = ck;
    p.t = pick_tile(M, ncols);
    int BN = tile_bn(p.t);
    p.Ub = BN + (int)J - 1;
    if ((p.Ub & 31) == 0) p.Ub += 1;
    int64_t blocks = cdiv(ncols, BN) * cdiv(M, tile_bm(p.t)) * B;
    plan_split(blocks, (int)Ci, ck, (int)(Ci * J), heavy_epi, &p.KS, &p.cps);
    return p;
}

// ------------------------------------------------------------------------- launch helpers
template <int BM, int BN, int WM, int WN>
void launch_fwd(FwdArgs a, hipStream_t st) {
    dim3 grid(cdiv(a.Tout, BN), cdiv(a.Cout, BM), a.B * a.KS);
    size_t lds = (size_t)(((a.CK * a.s * a.Up + 3) & ~3) + a.K * a.CK * BM + BM) * sizeof(float);
    a.vec = (a.Tin % 4 == 0) && (a.Cout % 4 == 0) && ((uintptr_t)a.x % 16 == 0) && ((uintptr_t)a.wf % 16 == 0);
    a.fs = make_fastdiv((uint32_t)a.s);
    const int epi = a.KS > 1 ? EPI_PART
                             : ((a.res ? EPI_RES : 0) | (a.xact ? EPI_XACT : 0) | (a.accumulate ? EPI_ACC : 0));
#define ENCX_FWD_EPI(E) \
    case E: hipLaunchKernelGGL((conv_fwd_kernel<BM, BN, WM, WN, E>), grid, dim3(NT), lds, st, a); break
    switch (epi) {
        ENCX_FWD_EPI(0); ENCX_FWD_EPI(1); ENCX_FWD_EPI(2); ENCX_FWD_EPI(3); ENCX_FWD_EPI(4);
        ENCX_FWD_EPI(5); ENCX_FWD_EPI(6); ENCX_FWD_EPI(7); ENCX_FWD_EPI(8);
    }
#undef ENCX_FWD_EPI
}

template <int BM, int BN, int WM, int WN>
void launch_poly(PolyArgs a, int ncols, hipStream_t st) {
    dim3 grid(cdiv(ncols, BN), cdiv((int64_t)a.Co * a.s, BM), a.B * a.KS);
    size_t lds = (size_t)(((a.CK * a.Ub + 3) & ~3) + a.J * a.CK * BM + BM) * sizeof(float);
    a.vec = (a.Tin % 4 == 0) && ((a.Co * a.s) % 4 == 0) && ((uintptr_t)a.in % 16 == 0) &&
            ((uintptr_t)a.wp % 16 == 0);
    int epi;
    if (a.KS > 1) epi = P_PART;
    else if (a.mode == 0) epi = 0;
    else epi = P_DGRAD | (a.act != ENCX_ACT_NONE ? P_XACT : 0) | (a.accumulate ? P_ACC : 0);
#define ENCX_POLY_EPI(E) \
    case E: hipLaunchKernelGGL((conv_poly_kernel<BM, BN, WM, WN, E>), grid, dim3(NT), lds, st, a); break
    switch (epi) {
        ENCX_POLY_EPI(0); ENCX_POLY_EPI(1); ENCX_POLY_EPI(3); ENCX_POLY_EPI(5); ENCX_POLY_EPI(7);
        ENCX_POLY_EPI(8);
    }
#undef ENCX_POLY_EPI
}

static bool fwd_flat(int64_t Cout, int64_t Tout) { return Cout > 4 && Tout <= FLAT_T; }
static int fwd_flat_slabs(int64_t B, int64_t Cin, int64_t Cout, int64_t Tout, int64_t K) {
    const int Kred = (int)(Cin * K);
    return gemm_slabs(Kred, gemm_splits((int)Cout, (int)(B * Tout), Kred));
}

// ---------------------------------------------------------------------------- 1x1 convs
// The pointwise convs of the residual blocks (seanet.py:59-60, kernel 1, stride 1, no padding)
// as a batched GEMM: C[b][m][n] = sum_k A[k][m] Bm[b][k][n], A the weight in k-major layout
// (forward: wf [Cin][Cout]; backward-data: wp [Cout][Cin]) and Bm the [B][C][T] activation
// (forward: ELU(x) when pre-activated; backward-data: dy). Both operands are staged as float4
// quads along their contiguous dim (m for A, n = t for Bm), register-prefetched one BK slice
// ahead; the epilogue is fwd_store's (bias, act'(xact), residual, accumulate).
struct PwArgs {
    const float* w;     // A [K][M]
    const float* x;     // Bm [B][K][N]
    const float* bias;  // [M] or null
    const float* res;   // [B][M][N] (PW_RES)
    const float* xact;  // [B][M][N] (PW_XACT): y *= act'(xact)
    float* y;           // [B][M][N]
    int M, K, N, in_act, epi_act;
};
enum { PW_RES = 1, PW_XACT = 2, PW_ACC = 4 };
typedef float f32x4u_pw __attribute__((ext_vector_type(4), aligned(4)));

template <int BM, int BN, int WM, int WN, int EPI>
__global__ __launch_bounds__(256) void pw_kernel(PwArgs a) {
    constexpr int BK = 32, TM = BM / WM / 32, TN = BN / WN / 32;
    constexpr int QA = BM * BK / 4 / 256, QB = BN * BK / 4 / 256;  // quads per thread
    static_assert(QA * 1024 == BM * BK && QB * 1024 == BN * BK, "tile / thread mismatch");
    __shared__ float As[BK][BM + 4];
    __shared__ float Bs[BK][BN + 4];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm0 = (wave / WN) * TM * 32, wn0 = (wave % WN) * TN * 32;
    const TileId tile = xcd_tile();
    const int n0 = tile.x * BN, m0 = tile.y * BM, b = tile.z;
    const int h = lane >> 5, l32 = lane & 31;
    const float* xb = a.x + (int64_t)b * a.K * a.N;
    f32x16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = (f32x16){0};
    f32x4 ra[QA], rb[QB];
    auto fetch = [&](int k0) {
#pragma unroll
        for (int e = 0; e < QA; ++e) {
            const int i = tid + e * 256, k = i / (BM / 4), mq = (i - k * (BM / 4)) * 4;
            const bool ok = k0 + k < a.K && m0 + mq < a.M;  // M % 4 == 0: whole quads
            ra[e] = *(const f32x4u_pw*)(a.w + (ok ? (int64_t)(k0 + k) * a.M + m0 + mq : 0));
            if (!ok) ra[e] = (f32x4){0.f, 0.f, 0.f, 0.f};
        }
#pragma unroll
        for (int e = 0; e < QB; ++e) {
            const int i = tid + e * 256, k = i / (BN / 4), nq = (i - k * (BN / 4)) * 4;
            const bool ok = k0 + k < a.K && n0 + nq < a.N;  // N % 4 == 0
            rb[e] = *(const f32x4u_pw*)(xb + (ok ? (int64_t)(k0 + k) * a.N + n0 + nq : 0));
            if (!ok) rb[e] = (f32x4){0.f, 0.f, 0.f, 0.f};
        }
    };
    fetch(0);
    for (int k0 = 0; k0 < a.K; k0 += BK) {
        __syncthreads();
#pragma unroll
        for (int e = 0; e < QA; ++e) {
            const int i = tid + e * 256, k = i / (BM / 4), mq = (i - k * (BM / 4)) * 4;
            *(f32x4*)&As[k][mq] = ra[e];
        }
#pragma unroll
        for (int e = 0; e < QB; ++e) {
            const int i = tid + e * 256, k = i / (BN / 4), nq = (i - k * (BN / 4)) * 4;
            f32x4 v = rb[e];
            if (a.in_act == ENCX_ACT_ELU)
#pragma unroll
                for (int c = 0; c < 4; ++c) v[c] = elu(v[c]);  // elu(0) = 0 keeps the padding
            *(f32x4*)&Bs[k][nq] = v;
        }
        __syncthreads();
        if (k0 + BK < a.K) fetch(k0 + BK);
#pragma unroll
        for (int kp = 0; kp < BK; kp += 2) {
            float av[TM], bv[TN];
#pragma unroll
            for (int i = 0; i < TM; ++i) av[i] = As[kp + h][wm0 + i * 32 + l32];
#pragma unroll
            for (int j = 0; j < TN; ++j) bv[j] = Bs[kp + h][wn0 + j * 32 + l32];
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j) acc[i][j] = mfma32(av[i], bv[j], acc[i][j]);
        }
    }
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int n = n0 + wn0 + j * 32 + l32;
            if (n >= a.N) continue;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int m = m0 + wm0 + i * 32 + mfma_row(r, lane);
                if (m >= a.M) continue;
                const int64_t o = ((int64_t)b * a.M + m) * a.N + n;
                float v = acc[i][j][r];
                if (a.bias) v += a.bias[m];
                if (EPI & PW_XACT) v *= act_grad(a.epi_act, a.xact[o]);
                if (EPI & PW_RES) v += a.res[o];
                if (EPI & PW_ACC) v += a.y[o];
                a.y[o] = v;
            }
        }
}

template <int EPI>
static void pw_launch_epi(const PwArgs& a, int B, hipStream_t st) {
    // largest tile that still gives >= 640 workgroups (2.5 rounds over 256 CUs)
    const int64_t nb128 = cdiv(a.N, 128), nb64 = cdiv(a.N, 64);
    if (a.M > 64 && cdiv(a.M, 128) * nb128 * B >= 640) {
        hipLaunchKernelGGL((pw_kernel<128, 128, 2, 2, EPI>), dim3(nb128, cdiv(a.M, 128), B), dim3(256), 0, st, a);
    } else if (a.M > 64 && cdiv(a.M, 128) * nb64 * B >= 640) {
        hipLaunchKernelGGL((pw_kernel<128, 64, 2, 2, EPI>), dim3(nb64, cdiv(a.M, 128), B), dim3(256), 0, st, a);
    } else if (a.M > 32 && cdiv(a.M, 64) * nb128 * B >= 640) {
        hipLaunchKernelGGL((pw_kernel<64, 128, 2, 2, EPI>), dim3(nb128, cdiv(a.M, 64), B), dim3(256), 0, st, a);
    } else if (a.M > 32) {
        hipLaunchKernelGGL((pw_kernel<64, 64, 2, 2, EPI>), dim3(nb64, cdiv(a.M, 64), B), dim3(256), 0, st, a);
    } else {
        hipLaunchKernelGGL((pw_kernel<32, 128, 1, 4, EPI>), dim3(nb128, cdiv(a.M, 32), B), dim3(256), 0, st, a);
    }
}
static int pw_launch(const PwArgs& a, int B, int epi, hipStream_t st) {
    switch (epi) {
        case 0: pw_launch_epi<0>(a, B, st); break;
        case PW_RES: pw_launch_epi<PW_RES>(a, B, st); break;
        case PW_XACT: pw_launch_epi<PW_XACT>(a, B, st); break;
        case PW_ACC: pw_launch_epi<PW_ACC>(a, B, st); break;
        case PW_XACT | PW_ACC: pw_launch_epi<PW_XACT | PW_ACC>(a, B, st); break;
        case PW_RES | PW_ACC: pw_launch_epi<PW_RES | PW_ACC>(a, B, st); break;
        default: return ENCX_EINVAL;
    }
    ENCX_CHECK_LAUNCH();
    return 0;
}
// the 1x1 layers the pointwise kernel serves (ENCX_PW=0 keeps the implicit-GEMM path): the
// short, wide ones (T <= 1024). tools/mb/conv_mb: 256x256 at T 600 101 -> 59 us, 128x256 53 -> 42
// us; the long, HBM-bound ones (T >= 3000) stay on conv_fwd_kernel, whose epilogue streams
// the residual better (64x64 at T 12000: 108 us there, 145 here)
// red: the GEMM's reduction length (Cin forward, Cout backward-data). Above PW_TMAX positions the
// GEMM still wins when it reduces over >= 128 channels (round 5 sweep at T 3000: 128 -> 128
// forward 168 -> 134 us, bwd-data 198 -> 160 and 135 -> 85 us; but the 64 -> 128 forward 129 -> 196)
static bool pw_ok(int K, int s, int d, int pl, int pr, int e, int Tin, int Tout, int Cin, int Cout, int red) {
    return encx_opt(OPT_PW) != 0 && K == 1 && s == 1 && d == 1 && pl == 0 && pr == 0 && e == 0 && Tin == Tout && Tout % 4 == 0 &&
           (Tout <= encx_opt(OPT_PW_TMAX) || red >= 128) && Cin % 4 == 0 && Cout % 4 == 0;
}

// weight grad of the short, wide 1x1 convs: dW[m=co][n=ci] = sum_{b,t} dy[b][co][t] act(x[b][ci][t])
// over positions k = b*T + t (T % 4 == 0: a quad never straddles two clips), split over k into
// slabs [S][M][N] (+ bias slabs [S][M] = sum dy, from the staged A operand) that wgrad_reduce
// adds in a fixed order
struct PwWgArgs {
    const float* dy;  // [B][M][T]
    const float* x;   // [B][N][T]
    float* ws;        // [S][M][N], then [S][M]
    int M, N, T, Ktot, kchunk, in_act, do_bias, S;
};
template <int BM, int BN, int WM, int WN>
__global__ __launch_bounds__(256) void pw_wgrad_kernel(PwWgArgs a) {
    constexpr int BK = 32, TM = BM / WM / 32, TN = BN / WN / 32;
    constexpr int QA = BM * BK / 4 / 256, QB = BN * BK / 4 / 256;
    static_assert(QA * 1024 == BM * BK && QB * 1024 == BN * BK, "tile / thread mismatch");
    __shared__ float As[BK][BM + 1];
    __shared__ float Bs[BK][BN + 1];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm0 = (wave / WN) * TM * 32, wn0 = (wave % WN) * TN * 32;
    const int n0 = blockIdx.x * BN, m0 = blockIdx.y * BM, z = blockIdx.z;
    const int h = lane >> 5, l32 = lane & 31;
    const int kbeg = z * a.kchunk, kend = min(a.Ktot, kbeg + a.kchunk);
    const bool bias_wave = a.do_bias && blockIdx.x == 0 && (wave % WN) == 0;
    f32x16 acc[TM][TN];
    float bsum[TM];
#pragma unroll
    for (int i = 0; i < TM; ++i) {
        bsum[i] = 0.f;
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = (f32x16){0};
    }
    f32x4 ra[QA], rb[QB];
    auto fetch = [&](int k0) {
#pragma unroll
        for (int e = 0; e < QA; ++e) {
            const int i = tid + e * 256, m = i / (BK / 4), k4 = (i - m * (BK / 4)) * 4, gk = k0 + k4;
            const bool ok = m0 + m < a.M && gk < kend;
            const int b = gk / a.T, t = gk - b * a.T;
            ra[e] = ld4u(a.dy + (ok ? ((int64_t)b * a.M + m0 + m) * a.T + t : 0));
            if (!ok) ra[e] = (f32x4){0.f, 0.f, 0.f, 0.f};
        }
#pragma unroll
        for (int e = 0; e < QB; ++e) {
            const int i = tid + e * 256, n = i / (BK / 4), k4 = (i - n * (BK / 4)) * 4, gk = k0 + k4;
            const bool ok = n0 + n < a.N && gk < kend;
            const int b = gk / a.T, t = gk - b * a.T;
            rb[e] = ld4u(a.x + (ok ? ((int64_t)b * a.N + n0 + n) * a.T + t : 0));
            if (!ok) rb[e] = (f32x4){0.f, 0.f, 0.f, 0.f};
        }
    };
    if (kbeg < kend) fetch(kbeg);
    for (int k0 = kbeg; k0 < kend; k0 += BK) {
        __syncthreads();
#pragma unroll
        for (int e = 0; e < QA; ++e) {
            const int i = tid + e * 256, m = i / (BK / 4), k4 = (i - m * (BK / 4)) * 4;
#pragma unroll
            for (int c = 0; c < 4; ++c) As[k4 + c][m] = ra[e][c];
        }
#pragma unroll
        for (int e = 0; e < QB; ++e) {
            const int i = tid + e * 256, n = i / (BK / 4), k4 = (i - n * (BK / 4)) * 4;
#pragma unroll
            for (int c = 0; c < 4; ++c) Bs[k4 + c][n] = a.in_act == ENCX_ACT_ELU ? elu(rb[e][c]) : rb[e][c];
        }
        __syncthreads();
        if (k0 + BK < kend) fetch(k0 + BK);
#pragma unroll
        for (int kp = 0; kp < BK; kp += 2) {
            float av[TM], bv[TN];
#pragma unroll
            for (int i = 0; i < TM; ++i) av[i] = As[kp + h][wm0 + i * 32 + l32];
#pragma unroll
            for (int j = 0; j < TN; ++j) bv[j] = Bs[kp + h][wn0 + j * 32 + l32];
            if (bias_wave)
#pragma unroll
                for (int i = 0; i < TM; ++i) bsum[i] += av[i];
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j) acc[i][j] = mfma32(av[i], bv[j], acc[i][j]);
        }
    }
    float* slab = a.ws + (int64_t)z * a.M * a.N;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int n = n0 + wn0 + j * 32 + l32;
            if (n >= a.N) continue;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int m = m0 + wm0 + i * 32 + mfma_row(r, lane);
                if (m < a.M) slab[(int64_t)m * a.N + n] = acc[i][j][r];
            }
        }
    if (bias_wave) {
        float* bslab = a.ws + (int64_t)a.S * a.M * a.N + (int64_t)z * a.M;
#pragma unroll
        for (int i = 0; i < TM; ++i) {
            const float v = bsum[i] + __shfl_xor(bsum[i], 32, 64);
            const int m = m0 + wm0 + i * 32 + l32;
            if (h == 0 && m < a.M) bslab[m] = v;
        }
    }
}

struct PwWgPlan {
    int BM, BN, S, kchunk;
};
static PwWgPlan plan_pw_wgrad(int64_t B, int64_t M, int64_t N, int64_t T) {
    PwWgPlan p;
    p.BM = M >= 128 ? 128 : 64;
    p.BN = N >= 128 ? 128 : 64;
    const int64_t tiles = cdiv(M, p.BM) * cdiv(N, p.BN), Ktot = B * T;
    int64_t S = cdiv(768, tiles);
    const int64_t cap = Ktot / 128;  // >= 4 k-stages per workgroup
    if (S > cap) S = cap;
    if (S < 1) S = 1;
    p.kchunk = (int)(cdiv(cdiv(Ktot, S), 32) * 32);
    p.S = (int)cdiv(Ktot, p.kchunk);
    return p;
}
static size_t pw_wgrad_ws_bytes(int64_t B, int64_t M, int64_t N, int64_t T) {
    const PwWgPlan p = plan_pw_wgrad(B, M, N, T);
    return (size_t)p.S * M * (N + 1) * sizeof(float);
}
// the layers pw_wgrad serves: 1x1, T <= 12000 (A/B: 3000 -> 12000 +0.2 %), at least 64 x 64
static bool pw_wgrad_ok(int64_t K, int64_t s, int64_t d, int64_t pl, int64_t e, int64_t Tin, int64_t Tout, int64_t Cin,
                        int64_t Cout) {
    const int64_t tmax = encx_opt(OPT_PW_WG_TMAX);
    return encx_opt(OPT_PW) != 0 && K == 1 && s == 1 && d == 1 && pl == 0 && e == 0 && Tin == Tout && Tout % 4 == 0 && Tout <= tmax &&
           Cin >= 64 && Cout >= 64 && Cin % 4 == 0 && Cout % 4 == 0;
}
static void pw_wgrad_run(const float* dy, const float* x, float* dw, float* db, float* ws, int64_t B, int64_t M,
                         int64_t N, int64_t T, int in_act, int acc_w, int acc_b, hipStream_t st) {
    const PwWgPlan p = plan_pw_wgrad(B, M, N, T);
    PwWgArgs a{dy, x, ws, (int)M, (int)N, (int)T, (int)(B * T), p.kchunk, in_act, db != nullptr, p.S};
    const dim3 grid((unsigned)cdiv(N, p.BN), (unsigned)cdiv(M, p.BM), (unsigned)p.S);
    if (p.BM == 128 && p.BN == 128) hipLaunchKernelGGL((pw_wgrad_kernel<128, 128, 2, 2>), grid, dim3(256), 0, st, a);
    else if (p.BM == 128) hipLaunchKernelGGL((pw_wgrad_kernel<128, 64, 2, 2>), grid, dim3(256), 0, st, a);
    else if (p.BN == 128) hipLaunchKernelGGL((pw_wgrad_kernel<64, 128, 2, 2>), grid, dim3(256), 0, st, a);
    else hipLaunchKernelGGL((pw_wgrad_kernel<64, 64, 2, 2>), grid, dim3(256), 0, st, a);
    const int64_t AN = M * N;
    hipLaunchKernelGGL(wgrad_reduce, dim3((unsigned)(cdiv(AN, 64) + (db ? cdiv(M, 64) : 0))), dim3(256), 0, st, ws, dw,
                       AN, p.S, acc_w, ws + (int64_t)p.S * AN, db, (int)M, acc_b);
}

// ------------------------------------------------------------------------- conv v2 main loop
// Round 6 (option CONV2): the implicit-GEMM forward and polyphase kernels rebuilt around one
// software-pipelined main loop. Per channel chunk the operands live in TWO LDS buffers: while the
// MFMAs run on chunk c, the weight rows of chunk c + 1 stream into the other buffer by LDS-DMA
// (global_load_lds_dwordx4: no VGPRs, one instruction per 64 quads) and its input window streams
// into registers (a few quads per thread), which are written to LDS -- with the pre-activation
// ELU applied once per element and the pad positions patched -- after the chunk's MFMAs: one
// barrier per chunk and no exposed memory round trip (the round-5 kernels staged synchronously
// between two barriers: MFMA busy 0.30-0.42). The window keeps its global order (stride-S taps
// read S words apart: at most 8-way bank conflicts, cheap beside the fp32 MFMA's 64 cycles). The
// reduction runs per lane half over half the chunk's channels (k slot 0: channels [0, CK/2), slot
// 1: [CK/2, CK)), so every operand address is a lane base plus a compile-time offset.
enum { EPI2_ELU = 16 };
// ELU without a branch: expm1 by its Taylor series to x^10 on [-1, 0] (truncation < 3e-8
// relative), exp2 - 1 below (|result| > 0.63, a few ulp); ocml's expm1f branches per element
ENCX_DEV float elu_nb(float x) {
    const float n = fminf(x, 0.f);
    float p = 1.f / 3628800.f;
    p = fmaf(p, n, 1.f / 362880.f);
    p = fmaf(p, n, 1.f / 40320.f);
    p = fmaf(p, n, 1.f / 5040.f);
    p = fmaf(p, n, 1.f / 720.f);
    p = fmaf(p, n, 1.f / 120.f);
    p = fmaf(p, n, 1.f / 24.f);
    p = fmaf(p, n, 1.f / 6.f);
    p = fmaf(p, n, 0.5f);
    p = fmaf(p * n, n, n);
    const float e = __builtin_amdgcn_exp2f(n * 1.44269504088896341f) - 1.f;
    return x > 0.f ? x : (n >= -1.f ? p : e);
}
typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) const void glb_void_t;
ENCX_DEV void glds16(const float* src, float* lds_wave_base) {
    __builtin_amdgcn_global_load_lds((glb_void_t*)src, (lds_void_t*)lds_wave_base, 16, 0, 0);
}
constexpr int C2X_MAXQ = 4;  // input-window quads per thread per chunk (registers in flight)
template <int BN, int K, int S> struct C1Geo {
    static constexpr int XW = ((BN - 1) * S + K + 3 + 3) & ~3;  // window positions per channel row
    static constexpr int XQ = XW / 4;
};
static size_t c1_lds(int XW, int CK, int K, int BM) {
    return (size_t)2 * (((CK * XW + 3) & ~3) + ((CK * K * BM + 255) & ~255)) * sizeof(float);
}

// The operand geometry of one tile: input rows xrow(c, cl) = xb + (cbeg + c CK + cl) Tin, window
// [ab, ab + XW) (ab 4-aligned; positions outside [0, Tin) come from pad_src(p + pl, pl, Tin, e,
// mode)), weight rows (cl, k) of chunk c at wsrc + ((c CK + cl) K + k) wstride, BM floats each.
// Tap k of output column n reads window position n S + k + woff (REV: tap K - 1 - k, the
// polyphase form's in[u - q]).
struct C1Tile {
    const float* xb;
    int Tin, ab, woff, pl, e, mode;
    int vec;  // input rows 16-B aligned (Tin % 4 == 0): quad loads; else 4 scalar loads per quad
    const float* wsrc;
    int wstride, CK, nch;
};
template <int BM, int BN, int WM, int K, int S, bool REV, bool ELU>
ENCX_DEV void c1_mainloop(f32x16 (&acc)[BM / WM / 32][BN / (4 / WM) / 32], const C1Tile& g) {
    constexpr int WN = 4 / WM, TM = BM / WM / 32, TN = BN / WN / 32;
    constexpr int XW = C1Geo<BN, K, S>::XW, XQ = C1Geo<BN, K, S>::XQ;
    extern __shared__ float smem[];
    const int CK = g.CK, CKH = CK >> 1, Tin = g.Tin;
    const int xsz = (CK * XW + 3) & ~3, bsz = xsz + ((CK * K * BM + 255) & ~255);
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm0 = (wave / WN) * TM * 32, wn0 = (wave % WN) * TN * 32;
    const int h = lane >> 5, l32 = lane & 31;
    const int nxq = CK * XQ, nwq = CK * K * (BM / 4);
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = (f32x16){0};
    f32x4 rx[C2X_MAXQ];
    auto load_x = [&](int c) {
        const float* xc = g.xb + (int64_t)(c * CK) * Tin;
        if (g.vec) {
#pragma unroll
            for (int e = 0; e < C2X_MAXQ; ++e) {
                const int q = tid + NT * e;
                const int row = q / XQ, p = g.ab + 4 * (q - row * XQ);
                const bool ok = q < nxq && p >= 0 && p + 4 <= Tin;
                rx[e] = *(const f32x4*)(xc + (ok ? (int64_t)row * Tin + p : 0));
            }
        } else {  // rows not 16-B aligned (T 75): the quad's elements one by one (the edges patched later)
#pragma unroll
            for (int e = 0; e < C2X_MAXQ; ++e) {
                const int q = tid + NT * e;
                const int row = q / XQ, p = g.ab + 4 * (q - row * XQ);
                const bool ok = q < nxq && p >= 0 && p + 4 <= Tin;
                const float* src = xc + (ok ? (int64_t)row * Tin + p : 0);
#pragma unroll
                for (int i = 0; i < 4; ++i) rx[e][i] = src[ok ? i : 0];
            }
        }
    };
    auto store_x = [&](int c, float* xs) {
        const float* xc = g.xb + (int64_t)(c * CK) * Tin;
#pragma unroll
        for (int e = 0; e < C2X_MAXQ; ++e) {
            const int q = tid + NT * e;
            if (q < nxq) {
                const int row = q / XQ, p = g.ab + 4 * (q - row * XQ);
                f32x4 v = rx[e];
                if (p < 0 || p + 4 > Tin) {
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        const int m = pad_src(p + i + g.pl, g.pl, Tin, g.e, g.mode);
                        v[i] = m >= 0 ? xc[(int64_t)row * Tin + m] : 0.f;
                    }
                }
                if (ELU) {
#pragma unroll
                    for (int i = 0; i < 4; ++i) v[i] = elu_nb(v[i]);
                }
                *(f32x4*)(xs + 4 * q) = v;
            }
        }
    };
    auto stage_w = [&](int c, float* ws) {
        const float* wc = g.wsrc + (int64_t)(c * CK) * K * g.wstride;
        for (int q0 = wave * 64; q0 < nwq; q0 += NT) {
            const int q = q0 + lane;
            const int row = q / (BM / 4), c4 = q - row * (BM / 4);
            glds16(wc + (q < nwq ? (int64_t)row * g.wstride + 4 * c4 : 0), ws + 4 * q0);
        }
    };
    if (g.nch <= 0) return;
    load_x(0);
    stage_w(0, smem + xsz);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    store_x(0, smem);
    __syncthreads();
    for (int c = 0; c < g.nch; ++c) {
        float* cur = smem + (c & 1) * bsz;
        float* nxt = smem + ((c + 1) & 1) * bsz;
        const bool more = c + 1 < g.nch;
        if (more) {
            stage_w(c + 1, nxt + xsz);
            load_x(c + 1);
        }
        const float* xs = cur + h * CKH * XW + g.woff + (wn0 + l32) * S;
        const float* ws = cur + xsz + h * CKH * K * BM + wm0 + l32;
        for (int cl = 0; cl < CKH; ++cl) {
#pragma unroll
            for (int kk = 0; kk < K; ++kk) {
                float av[TM], bv[TN];
                const int wk = REV ? K - 1 - kk : kk;
#pragma unroll
                for (int i = 0; i < TM; ++i) av[i] = ws[(cl * K + wk) * BM + i * 32];
#pragma unroll
                for (int j = 0; j < TN; ++j) bv[j] = xs[cl * XW + kk + j * 32 * S];
#pragma unroll
                for (int i = 0; i < TM; ++i)
#pragma unroll
                    for (int j = 0; j < TN; ++j) acc[i][j] = mfma32(av[i], bv[j], acc[i][j]);
            }
        }
        if (more) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            store_x(c + 1, nxt);
        }
        __syncthreads();
    }
}

// ------------------------------------------------------------------------- conv forward, v2
template <int BM, int BN, int WM, int K, int S, int EPI>
__global__ __launch_bounds__(NT) void conv_fwd2_kernel(FwdArgs a) {
    constexpr int WN = 4 / WM, TM = BM / WM / 32, TN = BN / WN / 32;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm0 = (wave / WN) * TM * 32, wn0 = (wave % WN) * TN * 32;
    // tile order: co block fastest (the blocks of one (b, t) tile share its x window), XCD-remapped
    const int nco = a.Cout / BM, ntt = (a.Tout + BN - 1) / BN;
    int id = xcd_linear_id();
    const int cb = id % nco;
    id /= nco;
    const int tt = id % ntt;
    id /= ntt;
    const int ks = id % a.KS, b = id / a.KS;
    const int co0 = cb * BM, t0 = tt * BN;
    const int cbeg = ks * a.cps, cend = min(a.Cin, cbeg + a.cps);
    const int wb = t0 * S - a.pl;
    C1Tile g;
    g.xb = a.x + ((int64_t)b * a.Cin + cbeg) * a.Tin;
    g.Tin = a.Tin;
    g.ab = wb & ~3;
    g.woff = wb - g.ab;
    g.pl = a.pl;
    g.e = a.e;
    g.mode = a.mode;
    g.vec = (a.Tin & 3) == 0;
    g.wsrc = a.wf + (int64_t)cbeg * K * a.Cout + co0;
    g.wstride = a.Cout;
    g.CK = a.CK;
    g.nch = (cend - cbeg) / a.CK;
    f32x16 acc[TM][TN];
    c1_mainloop<BM, BN, WM, K, S, false, (EPI & EPI2_ELU) != 0>(acc, g);
    // epilogue (conv_fwd_kernel's): the operands of a 32 x 32 sub-tile are loaded before its stores
    const int l32 = lane & 31;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int t = t0 + wn0 + j * 32 + l32;
            const int cr = co0 + wm0 + i * 32;
            const int64_t ob = ((int64_t)b * a.Cout + cr) * a.Tout + t;
            const bool tok = t < a.Tout;
            float e0[16], e1[16];
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int64_t o = tok ? ob + (int64_t)mfma_row(r, lane) * a.Tout : 0;
                e0[r] = (EPI & EPI_XACT) ? a.xact[o] : 0.f;
                e1[r] = (EPI & EPI_RES) ? a.res[o] : 0.f;
                if (EPI & EPI_ACC) e1[r] += a.y[o];
            }
            if (!tok) continue;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int co = cr + mfma_row(r, lane);
                const int64_t o = ob + (int64_t)mfma_row(r, lane) * a.Tout;
                float w = acc[i][j][r];
                if (EPI & EPI_PART) {
                    a.part[(int64_t)ks * a.B * a.Cout * a.Tout + o] = w;
                } else {
                    if (a.bias) w += a.bias[co];
                    if (EPI & EPI_XACT) w *= act_grad(a.epi_act, e0[r]);
                    a.y[o] = w + e1[r];
                }
            }
        }
}

// v2 planning: channels per chunk (even, dividing the channels of a split, about CONV2_RED
// reduction elements, the window within C2X_MAXQ quads per thread) and, over the tiles
// {128, 64} x {128, 64} and channel splits, the least estimated time: rounds of the grid over
// 256 CUs x the workgroups per CU the LDS admits (each sharing its CU), times the tile's MFMA
// time at an efficiency per tile shape, plus the split partials' HBM round trip.
struct C1Plan { int BM, BN, CK, KS, cps; size_t lds; double est; };
// Per tile shape and channel chunk: the workgroups one CU holds (LDS, and the VGPRs of the ELU
// variants: 224 -> 2 waves per SIMD) and the MFMA utilisation measured at that occupancy (round
// 6 sweeps: one workgroup per CU leaves the chunk hand-overs exposed, ~0.55; two ~0.8), the
// rounds of the grid over the CUs, a fixed cost per chunk, and the split partials' round trip.
static bool c1_plan(int B, int Cin, int M, int ncols, int K, int S, int out_elems_per_b, bool elu, C1Plan* best) {
    const int64_t force_tile = encx_opt(OPT_CONV2_TILE), force_ks = encx_opt(OPT_CONV2_KS);
    const int64_t red_cap = encx_opt(OPT_CONV2_RED);
    best->est = -1;
    for (int BM : {128, 64})
        for (int BN : {128, 64}) {
            const int tile = BM == 128 ? (BN == 128 ? 1 : 2) : (BN == 128 ? 3 : 4);
            if (force_tile && force_tile != tile) continue;
            if (M % BM) continue;
            const int XW = (((BN - 1) * S + K + 3 + 3) & ~3);
            const int wave_cap = elu ? 2 : 4;
            for (int CK = 2; CK <= Cin; CK += 2) {
                if (Cin % CK || CK * XW / 4 > NT * C2X_MAXQ || (int64_t)CK * K > red_cap) continue;
                const size_t lds = c1_lds(XW, CK, K, BM);
                if (lds > 160 * 1024) continue;
                const int occ = std::min<int>(wave_cap, (int)((160 * 1024) / lds));
                const double util = occ == 1 ? 0.55 : (occ == 2 ? 0.8 : 0.85);
                // relative rates per tile shape from the round-6 per-layer sweeps: the 64 x 128 tile
                // (each wave 64 rows x 32 columns) leads; 128-row tiles hold twice the weight rows
                // in LDS and, with the ELU, 224 VGPRs
                const double eff = BM == 64 ? (BN == 128 ? 1.0 : 0.95) : 0.85;
                const int nch = Cin / CK;
                for (int ks = 1; ks <= 8; ++ks) {
                    if (nch % ks || (force_ks && ks != force_ks)) continue;
                    if (ks > 1 && nch / ks < 2) continue;
                    const int64_t tiles = (int64_t)(M / BM) * cdiv(ncols, BN) * B * ks;
                    const int64_t slots = 256LL * occ;
                    // one CU: 0.614 TFLOP/s of fp32 MFMA (157.3 / 256), shared by occ workgroups
                    const double tile_us = 2.0 * BM * BN * (double)(Cin / ks) * K / (0.614e6 * util * eff) * occ;
                    const double rounds = (double)cdiv(tiles, slots);
                    double est = rounds * (tile_us + 0.25 * (nch / ks));
                    if (ks > 1) est += (double)ks * B * out_elems_per_b * 8.0 / 4.0e6 + 4.0;
                    if (best->est < 0 || est < best->est) {
                        best->BM = BM; best->BN = BN; best->CK = CK; best->KS = ks;
                        best->cps = (nch / ks) * CK; best->lds = lds; best->est = est;
                    }
                }
            }
        }
    return best->est >= 0;
}
template <int BM, int BN, int WM, int K, int S>
static int launch_fwd2_tile(FwdArgs a, size_t lds, hipStream_t st) {
    const int64_t nwg = (int64_t)(a.Cout / BM) * cdiv(a.Tout, BN) * a.B * a.KS;
    const int elu = a.act == ENCX_ACT_ELU ? EPI2_ELU : 0;
    const int epi = a.KS > 1 ? (EPI_PART | elu)
                             : elu | (a.res ? EPI_RES : 0) | (a.xact ? EPI_XACT : 0) | (a.accumulate ? EPI_ACC : 0);
#define ENCX_FWD2(E) \
    case E: hipLaunchKernelGGL((conv_fwd2_kernel<BM, BN, WM, K, S, E>), dim3((unsigned)nwg), dim3(NT), lds, st, a); break
    switch (epi) {
        ENCX_FWD2(0); ENCX_FWD2(EPI2_ELU); ENCX_FWD2(EPI_RES); ENCX_FWD2(EPI_RES | EPI2_ELU); ENCX_FWD2(EPI_XACT);
        ENCX_FWD2(EPI_PART); ENCX_FWD2(EPI_PART | EPI2_ELU);
        default: return -1;
    }
#undef ENCX_FWD2
    return 0;
}
static bool fwd2_shape_ok(const FwdArgs& a) {
    // (T <= 64: the flattened GEMM; between that and FLAT_T the v2 tiles of 64 columns, option CONV2_LOWT)
    const int64_t tmin = encx_opt(OPT_CONV2_LOWT) ? 64 : FLAT_T;
    return (encx_opt(OPT_CONV2) & 1) && a.d == 1 && a.e == 0 && a.Cout > 4 && a.Tout > tmin &&
           ((uintptr_t)a.x | (uintptr_t)a.wf) % 16 == 0 && a.Cout % 4 == 0;
}
template <int K, int S>
static int launch_fwd2_ks(FwdArgs a, float* ws, hipStream_t st) {
    C1Plan p;
    if (!c1_plan(a.B, a.Cin, a.Cout, a.Tout, K, S, a.Cout * a.Tout, a.act == ENCX_ACT_ELU, &p)) return -1;
    a.CK = p.CK;
    a.KS = p.KS;
    a.cps = p.cps;
    a.part = ws;
    if (p.KS > 1 && !ws) return -1;
    int rc;
    // waves side by side along t (WM 1) for the 128-column tiles
    if (p.BM == 128 && p.BN == 128) rc = launch_fwd2_tile<128, 128, 1, K, S>(a, p.lds, st);
    else if (p.BM == 128) rc = launch_fwd2_tile<128, 64, 2, K, S>(a, p.lds, st);
    else if (p.BN == 128) rc = launch_fwd2_tile<64, 128, 1, K, S>(a, p.lds, st);
    else rc = launch_fwd2_tile<64, 64, 2, K, S>(a, p.lds, st);
    if (rc) return rc;
    ENCX_CHECK_LAUNCH();
    if (a.KS > 1) {
        const int64_t n = (int64_t)a.B * a.Cout * a.Tout;
        hipLaunchKernelGGL(conv_fwd_reduce, dim3((unsigned)cdiv(n, 256)), dim3(256), 0, st, a);
        ENCX_CHECK_LAUNCH();
    }
    return 0;
}
#define ENCX_C1_KS_LIST(X) X(7, 1) X(3, 1) X(1, 1) X(4, 2) X(8, 4) X(10, 5) X(16, 8)
// -1: shape not served by v2 (the caller runs the round-5 kernels)
static int conv_fwd2_run(const FwdArgs& a, float* ws, hipStream_t st) {
    if (!fwd2_shape_ok(a)) return -1;
    switch (a.K * 16 + a.s) {
#define ENCX_C1_CASE(K_, S_) \
    case K_ * 16 + S_: return launch_fwd2_ks<K_, S_>(a, ws, st);
        ENCX_C1_KS_LIST(ENCX_C1_CASE)
#undef ENCX_C1_CASE
        default: return -1;
    }
}
static size_t conv_fwd2_ws(int64_t B, int64_t Cin, int64_t Cout, int64_t Tout, int64_t K, int64_t s) {
    if (!(encx_opt(OPT_CONV2) & 1)) return 0;
    C1Plan p;
    C1Plan q;
    if (!c1_plan((int)B, (int)Cin, (int)Cout, (int)Tout, (int)K, (int)s, (int)(Cout * Tout), true, &p)) p.KS = 1;
    if (!c1_plan((int)B, (int)Cin, (int)Cout, (int)Tout, (int)K, (int)s, (int)(Cout * Tout), false, &q)) q.KS = 1;
    if (p.KS < q.KS) p.KS = q.KS;
    if (p.KS == 1) return 0;
    return (size_t)p.KS * B * Cout * Tout * sizeof(float);
}

// ------------------------------------------------------------------------- polyphase, v2
// conv_poly_kernel on the v2 main loop: K = J taps, S = 1, the window read backwards (REV: tap kk
// of column n is in[u0 + n - (J - 1 - kk)] with the weight row of q = J - 1 - kk), zero outside
// [0, Tin); the ConvTranspose1d input ELU (in_act) applied as the window is written to LDS.
template <int BM, int BN, int WM, int J, int EPI>
__global__ __launch_bounds__(NT) void conv_poly2_kernel(PolyArgs a) {
    constexpr int WN = 4 / WM, TM = BM / WM / 32, TN = BN / WN / 32;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm0 = (wave / WN) * TM * 32, wn0 = (wave % WN) * TN * 32;
    const int S = a.s, M = a.Co * S;
    const int nmb = M / BM, ncols = a.Q / S, ntt = (ncols + BN - 1) / BN;
    int id = xcd_linear_id();
    const int mb = id % nmb;
    id /= nmb;
    const int tt = id % ntt;
    id /= ntt;
    const int ks = id % a.KS, b = id / a.KS;
    const int m0 = mb * BM, u0 = tt * BN;
    const int cbeg = ks * a.cps, cend = min(a.Ci, cbeg + a.cps);
    const int wb = u0 - (J - 1);
    C1Tile g;
    g.xb = a.in + ((int64_t)b * a.Ci + cbeg) * a.Tin;
    g.Tin = a.Tin;
    g.ab = wb & ~3;
    g.woff = wb - g.ab;
    g.pl = 0;
    g.e = 0;
    g.mode = ENCX_PAD_ZERO;
    g.vec = (a.Tin & 3) == 0;
    g.wsrc = a.wp + (int64_t)cbeg * J * M + m0;
    g.wstride = M;
    g.CK = a.CK;
    g.nch = (cend - cbeg) / a.CK;
    f32x16 acc[TM][TN];
    c1_mainloop<BM, BN, WM, J, 1, true, (EPI & EPI2_ELU) != 0>(acc, g);
    const int l32 = lane & 31;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int u = u0 + wn0 + j * 32 + l32;
            if (EPI & P_PART) {
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int row = m0 + wm0 + i * 32 + mfma_row(r, lane);
                    const int o = row / S, qpos = u * S + (row - o * S);
                    if (qpos < a.Q) a.part[(((int64_t)ks * a.B + b) * a.Co + o) * a.Q + qpos] = acc[i][j][r];
                }
                continue;
            }
            if (!(EPI & P_DGRAD)) {  // ConvTranspose1d: bias, trim
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int row = m0 + wm0 + i * 32 + mfma_row(r, lane);
                    const int o = row / S, p = u * S + (row - o * S) - a.trim;
                    if (p >= 0 && p < a.Tout)
                        a.out[((int64_t)b * a.Co + o) * a.Tout + p] = acc[i][j][r] + (a.bias ? a.bias[o] : 0.f);
                }
                continue;
            }
            float e0[16], e1[16];
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int row = m0 + wm0 + i * 32 + mfma_row(r, lane);
                const int o = row / S, m = u * S + (row - o * S) - a.pl;
                const bool ok = m >= 0 && m < a.Tx;
                const int64_t idx = ok ? ((int64_t)b * a.Co + o) * a.Tx + m : 0;
                e0[r] = (EPI & P_XACT) ? a.xact[idx] : 0.f;
                e1[r] = (EPI & P_ACC) ? a.out[idx] : 0.f;
            }
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int row = m0 + wm0 + i * 32 + mfma_row(r, lane);
                const int o = row / S, qpos = u * S + (row - o * S), m = qpos - a.pl;
                const float v = acc[i][j][r];
                if (m >= 0 && m < a.Tx) {
                    float gv = v;
                    if (EPI & P_XACT) gv *= act_grad(a.act, e0[r]);
                    a.out[((int64_t)b * a.Co + o) * a.Tx + m] = gv + e1[r];
                } else if (qpos >= 0 && qpos < a.pl + a.Tx + a.pr) {
                    const int slot = m < 0 ? qpos : a.pl + (m - a.Tx);
                    a.side[((int64_t)b * a.Co + o) * (a.pl + a.pr) + slot] = v;
                }
            }
        }
}
template <int BM, int BN, int WM, int J>
static int launch_poly2_tile(PolyArgs a, size_t lds, hipStream_t st) {
    const int M = a.Co * a.s;
    const int64_t nwg = (int64_t)(M / BM) * cdiv(a.Q / a.s, BN) * a.B * a.KS;
    const int elu = a.in_act == ENCX_ACT_ELU ? EPI2_ELU : 0;
    int epi;
    if (a.KS > 1) epi = P_PART | elu;
    else if (a.mode == 0) epi = elu;
    else epi = elu | P_DGRAD | (a.act != ENCX_ACT_NONE ? P_XACT : 0) | (a.accumulate ? P_ACC : 0);
#define ENCX_POLY2(E) \
    case E: hipLaunchKernelGGL((conv_poly2_kernel<BM, BN, WM, J, E>), dim3((unsigned)nwg), dim3(NT), lds, st, a); break
    switch (epi) {
        ENCX_POLY2(0); ENCX_POLY2(EPI2_ELU); ENCX_POLY2(P_DGRAD); ENCX_POLY2(P_DGRAD | P_XACT);
        ENCX_POLY2(P_DGRAD | P_ACC); ENCX_POLY2(P_DGRAD | P_XACT | P_ACC); ENCX_POLY2(P_PART);
        ENCX_POLY2(P_PART | EPI2_ELU);
        default: return -1;
    }
#undef ENCX_POLY2
    return 0;
}
template <int J>
static int launch_poly2_j(PolyArgs a, int ncols, float* ws, hipStream_t st) {
    C1Plan p;
    const int M = a.Co * a.s;
    if (!c1_plan(a.B, a.Ci, M, ncols, J, 1, a.Co * a.Q, a.in_act == ENCX_ACT_ELU, &p)) return -1;
    if (p.KS > 1 && !ws) return -1;
    a.CK = p.CK;
    a.KS = p.KS;
    a.cps = p.cps;
    a.part = ws;
    int rc;
    if (p.BM == 128 && p.BN == 128) rc = launch_poly2_tile<128, 128, 1, J>(a, p.lds, st);
    else if (p.BM == 128) rc = launch_poly2_tile<128, 64, 2, J>(a, p.lds, st);
    else if (p.BN == 128) rc = launch_poly2_tile<64, 128, 1, J>(a, p.lds, st);
    else rc = launch_poly2_tile<64, 64, 2, J>(a, p.lds, st);
    if (rc) return rc;
    ENCX_CHECK_LAUNCH();
    if (a.KS > 1) {
        const int64_t n = (int64_t)a.B * a.Co * a.Q;
        hipLaunchKernelGGL(conv_poly_reduce, dim3((unsigned)cdiv(n, 256)), dim3(256), 0, st, a);
        ENCX_CHECK_LAUNCH();
    }
    return 0;
}
// -1: not served by v2. a.Q must be set (ncols * s).
static int poly2_run(const PolyArgs& a, int ncols, float* ws, hipStream_t st) {
    if (!(encx_opt(OPT_CONV2) & 2) || ncols <= (encx_opt(OPT_CONV2_LOWT) ? 64 : FLAT_T) ||
        ((uintptr_t)a.in | (uintptr_t)a.wp) % 16 || (a.Co * a.s) % 4)
        return -1;
    switch (a.J) {
        case 1: return launch_poly2_j<1>(a, ncols, ws, st);
        case 2: return launch_poly2_j<2>(a, ncols, ws, st);
        case 3: return launch_poly2_j<3>(a, ncols, ws, st);
        case 7: return launch_poly2_j<7>(a, ncols, ws, st);
        default: return -1;
    }
}
static size_t poly2_ws(int64_t B, int64_t Ci, int64_t Co, int64_t s, int64_t ncols, int64_t J) {
    if (!(encx_opt(OPT_CONV2) & 2) || ncols <= 64) return 0;
    C1Plan p;
    C1Plan q;
    if (!c1_plan((int)B, (int)Ci, (int)(Co * s), (int)ncols, (int)J, 1, (int)(Co * ncols * s), true, &p)) p.KS = 1;
    if (!c1_plan((int)B, (int)Ci, (int)(Co * s), (int)ncols, (int)J, 1, (int)(Co * ncols * s), false, &q)) q.KS = 1;
    if (p.KS < q.KS) p.KS = q.KS;
    if (p.KS == 1) return 0;
    return (size_t)p.KS * B * Co * ncols * s * sizeof(float);
}

int conv_fwd_run(FwdArgs a, float* ws, hipStream_t st) {
    if (ws && !a.part && !fwd_flat(a.Cout, a.Tout) &&
        blas_big_ok(a.Cout, (int64_t)a.B * a.Tout, (int64_t)a.Cin * a.K) &&
        blas_flat_run(LdConvFlat{a, make_fastdiv(a.K), make_fastdiv(a.Tout)}, EpConvFlat{a, 1, make_fastdiv(a.Tout)},
                      a.wf, a.Cout, a.B * a.Tout, a.Cin * a.K, ws, st) == 0)
        return 0;
    if (!(encx_opt(OPT_PW) && a.K == 1 && a.Tout <= encx_opt(OPT_PW_TMAX)) && !a.part) {
        const int rc = conv_fwd2_run(a, ws, st);
        if (rc >= 0) return rc;
    }
    if (pw_ok(a.K, a.s, a.d, a.pl, 0, a.e, a.Tin, a.Tout, a.Cin, a.Cout, a.Cin) && !a.part) {
        PwArgs p{a.wf, a.x, a.bias, a.res, a.xact, a.y, a.Cout, a.Cin, a.Tout, a.act, a.epi_act};
        const int epi = (a.res ? PW_RES : 0) | (a.xact ? PW_XACT : 0) | (a.accumulate ? PW_ACC : 0);
        if (pw_launch(p, a.B, epi, st) == 0) return 0;
    }
    if (fwd_flat(a.Cout, a.Tout)) {
        const int Kred = a.Cin * a.K, N = a.B * a.Tout;
        if (ws && blas_flat_ok(a.Cout, N, Kred) &&
            blas_flat_run(LdConvFlat{a, make_fastdiv(a.K), make_fastdiv(a.Tout)}, EpConvFlat{a, 1, make_fastdiv(a.Tout)},
                          a.wf, a.Cout, N, Kred, ws, st) == 0)
            return 0;
        const int splits = gemm_splits(a.Cout, N, Kred);
        const int slabs = gemm_slabs(Kred, splits);
        a.part = ws;
        a.KS = slabs;
        ENCX_REQUIRE(slabs == 1 || ws);
        int rc = gemm_launch(LdConvFlat{a, make_fastdiv(a.K), make_fastdiv(a.Tout)},
                             EpConvFlat{a, slabs, make_fastdiv(a.Tout)}, a.Cout, N, Kred, st, splits);
        if (rc) return rc;
        if (slabs > 1) {
            int64_t n = (int64_t)a.B * a.Cout * a.Tout;
            hipLaunchKernelGGL(conv_fwd_reduce, dim3(cdiv(n, 256)), dim3(256), 0, st, a);
            ENCX_CHECK_LAUNCH();
        }
        return 0;
    }
    FwdPlan p = plan_fwd(a.B, a.Cin, a.Cout, a.Tout, a.K, a.s, a.d, a.res || a.xact || a.accumulate);
    if (p.small) {
        // as many channels per LDS stage as ~48 KB hold (the stages are sequential round trips;
        // the per-thread sum runs over the channels in order either way)
        const int WL = (NT - 1) * a.s + (a.K - 1) * a.d + 1;
        int ck = 12288 / (WL + a.Cout * a.K);
        if (ck < 1) ck = 1;
        if (ck > a.Cin) ck = a.Cin;
        a.CK = ck;
        a.KS = 1;
        a.cps = a.Cin;
        size_t lds = (size_t)(ck * WL + a.Cout * ck * a.K) * sizeof(float);
        ENCX_REQUIRE(lds <= 160 * 1024);
        hipLaunchKernelGGL(conv_fwd_small_kernel, dim3(cdiv(a.Tout, NT), 1, a.B), dim3(NT), lds, st, a);
        ENCX_CHECK_LAUNCH();
        return 0;
    }
    a.CK = p.CK; a.Up = p.Up; a.KS = p.KS; a.cps = p.cps; a.part = ws;
    ENCX_REQUIRE(a.KS == 1 || ws);
    switch (p.t) {
        case T32x128: launch_fwd<32, 128, 1, 4>(a, st); break;
        case T64x128: launch_fwd<64, 128, 2, 2>(a, st); break;
        case T128x32: launch_fwd<128, 32, 4, 1>(a, st); break;
        default: launch_fwd<128, 128, 2, 2>(a, st); break;
    }
    ENCX_CHECK_LAUNCH();
    if (a.KS > 1) {
        int64_t n = (int64_t)a.B * a.Cout * a.Tout;
        hipLaunchKernelGGL(conv_fwd_reduce, dim3(cdiv(n, 256)), dim3(256), 0, st, a);
        ENCX_CHECK_LAUNCH();
    }
    return 0;
}

size_t conv_fwd_ws(int64_t B, int64_t Cin, int64_t Cout, int64_t Tout, int64_t K, int64_t s, int64_t d) {
    const size_t v2 = std::max(conv_fwd2_ws(B, Cin, Cout, Tout, K, s), blas_flat_ws(Cout, B * Tout, Cin * K));
    if (fwd_flat(Cout, Tout)) {
        const int slabs = fwd_flat_slabs(B, Cin, Cout, Tout, K);
        return std::max({v2, slabs > 1 ? (size_t)slabs * B * Cout * Tout * sizeof(float) : (size_t)0,
                         blas_flat_ws(Cout, B * Tout, Cin * K)});
    }
    // (the epilogue's operands are not known here: the larger of the two plans)
    size_t ws = 0;
    for (const bool heavy : {false, true}) {
        const FwdPlan p = plan_fwd(B, Cin, Cout, Tout, K, s, d, heavy);
        if (!p.small && p.KS > 1) ws = std::max(ws, (size_t)p.KS * B * Cout * Tout * sizeof(float));
    }
    return std::max(ws, v2);
}

int poly_run(PolyArgs a, int ncols, float* ws, hipStream_t st) {
    if (ws && ncols > FLAT_T && blas_big_ok((int64_t)a.Co * a.s, (int64_t)a.B * ncols, (int64_t)a.Ci * a.J)) {
        PolyArgs ab = a;
        ab.Q = ncols * a.s;
        if (blas_flat_run(LdPolyFlat{ab, ab.Co * ab.s, ncols, make_fastdiv(ab.J), make_fastdiv(ncols)},
                          EpPolyFlat{ab, ncols, 1, make_fastdiv(ab.s), make_fastdiv(ncols)}, ab.wp, ab.Co * ab.s,
                          ab.B * ncols, ab.Ci * ab.J, ws, st) == 0)
            return 0;
    }
    {
        PolyArgs a2 = a;
        a2.Q = ncols * a.s;
        const int rc = poly2_run(a2, ncols, ws, st);
        if (rc >= 0) return rc;
    }
    if (ncols <= FLAT_T) {
        const int M = a.Co * a.s, Kred = a.Ci * a.J, N = a.B * ncols;
        a.Q = ncols * a.s;
        if (ws && blas_flat_ok(M, N, Kred) &&
            blas_flat_run(LdPolyFlat{a, M, ncols, make_fastdiv(a.J), make_fastdiv(ncols)},
                          EpPolyFlat{a, ncols, 1, make_fastdiv(a.s), make_fastdiv(ncols)}, a.wp, M, N, Kred, ws,
                          st) == 0)
            return 0;
        const int splits = gemm_splits(M, N, Kred);
        const int slabs = gemm_slabs(Kred, splits);
        a.part = ws;
        a.KS = slabs;
        ENCX_REQUIRE(slabs == 1 || ws);
        int rc = gemm_launch(LdPolyFlat{a, M, ncols, make_fastdiv(a.J), make_fastdiv(ncols)},
                             EpPolyFlat{a, ncols, slabs, make_fastdiv(a.s), make_fastdiv(ncols)}, M, N, Kred, st,
                             splits);
        if (rc) return rc;
        if (slabs > 1) {
            int64_t n = (int64_t)a.B * a.Co * a.Q;
            hipLaunchKernelGGL(conv_poly_reduce, dim3(cdiv(n, 256)), dim3(256), 0, st, a);
            ENCX_CHECK_LAUNCH();
        }
        return 0;
    }
    PolyPlan p = plan_poly(a.B, a.Ci, (int64_t)a.Co * a.s, ncols, a.J,
                           a.mode != 0 && (a.act != ENCX_ACT_NONE || a.accumulate));
    a.CK = p.CK; a.Ub = p.Ub; a.KS = p.KS; a.cps = p.cps; a.Q = ncols * a.s; a.part = ws;
    ENCX_REQUIRE(a.KS == 1 || ws);
    switch (p.t) {
        case T32x128: launch_poly<32, 128, 1, 4>(a, ncols, st); break;
        case T64x128: launch_poly<64, 128, 2, 2>(a, ncols, st); break;
        case T128x32: launch_poly<128, 32, 4, 1>(a, ncols, st); break;
        default: launch_poly<128, 128, 2, 2>(a, ncols, st); break;
    }
    ENCX_CHECK_LAUNCH();
    if (a.KS > 1) {
        int64_t n = (int64_t)a.B * a.Co * a.Q;
        hipLaunchKernelGGL(conv_poly_reduce, dim3(cdiv(n, 256)), dim3(256), 0, st, a);
        ENCX_CHECK_LAUNCH();
    }
    return 0;
}

size_t poly_ws(int64_t B, int64_t Ci, int64_t Co, int64_t s, int64_t ncols, int64_t J) {
    const size_t v2 = std::max(poly2_ws(B, Ci, Co, s, ncols, J), blas_flat_ws(Co * s, B * ncols, Ci * J));
    if (ncols <= FLAT_T) {
        const int Kred = (int)(Ci * J);
        const int slabs = gemm_slabs(Kred, gemm_splits((int)(Co * s), (int)(B * ncols), Kred));
        return std::max({v2, slabs > 1 ? (size_t)slabs * B * Co * ncols * s * sizeof(float) : (size_t)0,
                         blas_flat_ws(Co * s, B * ncols, Kred)});
    }
    size_t ws = 0;
    for (const bool heavy : {false, true}) {
        const PolyPlan p = plan_poly(B, Ci, Co * s, ncols, J, heavy);
        if (p.KS > 1) ws = std::max(ws, (size_t)p.KS * B * Co * ncols * s * sizeof(float));
    }
    return std::max(ws, v2);
}

// wgrad planning shared by the launcher and the workspace query
struct WgPlan {
    int kind;  // 0 VALU small, 1 narrow (32x32, waves split t), 2 tiled
    int BM, BN, BT, splits, items, per_split, tiles;
};
static WgPlan plan_wgrad(int64_t B, int64_t A, int64_t Tl, int64_t C, int64_t K) {
    WgPlan p;
    const int64_t N = C * K;
    if (A * N <= NT) {
        p.kind = 0; p.BT = SMALL_BT; p.BM = p.BN = 0; p.tiles = 1;
    } else if (N <= 32 && A <= 64) {
        p.kind = 1; p.BT = 64; p.BM = A <= 32 ? 32 : 64; p.BN = 32;
        p.tiles = (int)cdiv(A, p.BM);
    } else {
        p.kind = 2;
        // the row in equal chunks of <= 64 positions, a multiple of 4 each: T 75 -> 2 x 40
        // (fixed 32-position chunks padded it to 96), T 600 -> 10 x 60 (64: 640)
        const int64_t nch = cdiv(Tl, 64);
        p.BT = (int)(cdiv(cdiv(Tl, nch), 4) * 4);
        Tile t = (A <= 32) ? T32x128 : (A <= 64 ? T64x128 : T128x128);
        p.BM = tile_bm(t); p.BN = 128;
        p.tiles = (int)(cdiv(N, p.BN) * cdiv(A, p.BM));
    }
    p.items = (int)(B * cdiv(Tl, p.BT));
    const int64_t target = encx_opt(OPT_CONV_WG_SPLIT);  // ~1024 workgroups in flight
    int64_t want = cdiv(target, p.tiles);
    // <= 32 MB of partials: the slabs are written and read back once each (64 MB cost the big
    // weights 10 % over 32 MB, round 5 sweep; the small ones never reach the cap)
    int64_t cap = (32ll << 20) / (4 * A * N);
    if (cap < 1) cap = 1;
    int64_t sp = want < cap ? want : cap;
    if (sp > p.items / 4) sp = p.items / 4;              // >= 4 chunks of t per workgroup
    if (sp < 1) sp = 1;
    p.per_split = (int)cdiv(p.items, sp);
    p.splits = (int)cdiv(p.items, p.per_split);
    return p;
}

static int wlp_for(int WL, int K) {
    // row stride == K (mod 32) so 32 consecutive (c,k) columns hit 32 distinct banks
    int r = ((K % 32) - (WL % 32) + 32) % 32;
    return WL + r;
}

template <int BM, int BN, int WM, int WN, int WK>
void launch_wg(WgArgs a, int splits, hipStream_t st) {
    dim3 grid(cdiv((int64_t)a.C * a.K, BN), cdiv(a.A, BM), splits);
    size_t lds = (size_t)((a.BT + 1) * BM + a.NCmax * a.WLp) * sizeof(float);
    a.vec = (a.Tl % 4 == 0) && (a.Tr % 4 == 0) && ((uintptr_t)a.L % 16 == 0) && ((uintptr_t)a.R % 16 == 0);
    size_t red = (size_t)4 * (BM / WM / 32) * (BN / WN / 32) * 16 * 64 * sizeof(float);  // all 4 waves
    if (WK > 1 && red > lds) lds = red;
    hipLaunchKernelGGL((conv_wgrad_kernel<BM, BN, WM, WN, WK>), grid, dim3(NT), lds, st, a);
}

// whether wgrad_run can also produce the bias grad (sum over t of L) for this shape
static bool wgrad_bias_ok(int64_t B, int64_t A, int64_t Tl, int64_t C, int64_t K) {
    const WgPlan p = plan_wgrad(B, A, Tl, C, K);
    return p.kind != 0 || A * C * K + A <= NT;
}

// ------------------------------------------------------------------------- weight grad, v2
// dW[a][(c, k)] = sum_{b,t} L[b][a][t] * R~[b][c][t s + k - pl] (conv: L = dy, R = x; convtr: L = x,
// R = dy) on the v2 pipeline: a workgroup owns a BM x BN tile of dW and walks a contiguous run of
// (b, 64-position) chunks; per chunk L is staged transposed, Ls[t][a] (the MFMA A reads 32 rows
// of one position: consecutive words), and R as the window rows of the tile's channels, both
// through registers (the next chunk's loads in flight while the current chunk's MFMAs run, the
// activation applied once per element and the pad patched on the way into LDS), two LDS buffers,
// one barrier per chunk. Partial tiles go to slabs [split][A][C K] (+ the bias sums of L, conv
// only, by the column-0 tiles) for wgrad_reduce.
constexpr int W2_PT = 64;       // positions per chunk
constexpr int W2_LQ = 4;        // L quads per thread per chunk (BM <= 64)
constexpr int W2_RQ = 6;        // R-window quads per thread per chunk
struct Wg2Args {
    const float* L;
    const float* R;
    float* ws;
    float* wsb;
    int B, A, Tl, C, Tr, K, s, pl, e, mode, actL, actR;
    int items, per_split;  // items = B * ceil(Tl / PT)
    int NC, WLp;            // window rows per tile, LDS row length
};
static int w2_wl(int K, int S) { return (W2_PT - 1) * S + K + 3 + 3; }
template <int BM, int BN, int K, int S, bool ELU_L, bool ELU_R, bool BIAS>
__global__ __launch_bounds__(NT) void conv_wgrad2_kernel(Wg2Args a) {
    constexpr int TM = BM / 64, TN = BN / 64;  // 4 waves as 2 x 2
    constexpr int LS = BM + 1;                 // Ls row stride (odd: the transposing writes)
    extern __shared__ float smem[];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm0 = (wave >> 1) * TM * 32, wn0 = (wave & 1) * TN * 32;
    const int h = lane >> 5, l32 = lane & 31;
    const int N = a.C * K;
    const int n0 = blockIdx.x * BN, a0 = blockIdx.y * BM, split = blockIdx.z;
    const int c_lo = n0 / K;
    const int WLp = a.WLp, NC = a.NC;
    const int lsz = W2_PT * LS, rsz = NC * WLp, bsz = ((lsz + rsz) + 3) & ~3;
    const int it0 = split * a.per_split, it1 = min(a.items, it0 + a.per_split);
    const int tch = (a.Tl + W2_PT - 1) / W2_PT;
    // this lane's B columns: n = n0 + wn0 + j 32 + l32 -> (channel row, tap) of the staged window
    int bbase[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) {
        const int n = min(n0 + wn0 + j * 32 + l32, N - 1);
        const int c = n / K, kk = n - c * K;
        bbase[j] = (c - c_lo) * WLp + kk;
    }
    f32x16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = (f32x16){0};
    f32x4 rl[W2_LQ], rr[W2_RQ];
    float bacc[W2_LQ];
#pragma unroll
    for (int e = 0; e < W2_LQ; ++e) bacc[e] = 0.f;
    constexpr int LQR = W2_PT / 4;  // L quads per row
    const int nlq = BM * LQR;
    const int RQ = WLp / 4, nrq = NC * RQ;
    auto load = [&](int it) {
        const int b = it / tch, t0 = (it - b * tch) * W2_PT;
        const float* Lb = a.L + ((int64_t)b * a.A + a0) * a.Tl;
#pragma unroll
        for (int e = 0; e < W2_LQ; ++e) {
            const int q = tid + NT * e;
            const int row = q / LQR, t = t0 + 4 * (q - row * LQR);
            const bool ok = q < nlq && t + 4 <= a.Tl;
            rl[e] = *(const f32x4*)(Lb + (ok ? (int64_t)row * a.Tl + t : 0));
            if (!ok) rl[e] = (f32x4){0.f, 0.f, 0.f, 0.f};
        }
        const int wb = t0 * S - a.pl, ab = wb & ~3;
        const float* Rb = a.R + ((int64_t)b * a.C + c_lo) * a.Tr;
#pragma unroll
        for (int e = 0; e < W2_RQ; ++e) {
            const int q = tid + NT * e;
            const int row = q / RQ, p = ab + 4 * (q - row * RQ);
            const bool ok = q < nrq && c_lo + row < a.C && p >= 0 && p + 4 <= a.Tr;
            rr[e] = *(const f32x4*)(Rb + (ok ? (int64_t)row * a.Tr + p : 0));
        }
    };
    auto store = [&](int it, float* buf) {
        const int b = it / tch, t0 = (it - b * tch) * W2_PT;
        float* Ls = buf;
        float* Rs = buf + lsz;
#pragma unroll
        for (int e = 0; e < W2_LQ; ++e) {
            const int q = tid + NT * e;
            if (q < nlq) {
                const int row = q / LQR, tq = 4 * (q - row * LQR);
                f32x4 v = rl[e];
                if (BIAS) bacc[e] += (v[0] + v[1]) + (v[2] + v[3]);
#pragma unroll
                for (int i = 0; i < 4; ++i) Ls[(tq + i) * LS + row] = ELU_L ? elu_nb(v[i]) : v[i];
            }
        }
        const int wb = t0 * S - a.pl, ab = wb & ~3;
        const float* Rb = a.R + ((int64_t)b * a.C + c_lo) * a.Tr;
#pragma unroll
        for (int e = 0; e < W2_RQ; ++e) {
            const int q = tid + NT * e;
            if (q < nrq) {
                const int row = q / RQ, p = ab + 4 * (q - row * RQ);
                f32x4 v = rr[e];
                if (c_lo + row >= a.C) {
                    v = (f32x4){0.f, 0.f, 0.f, 0.f};
                } else if (p < 0 || p + 4 > a.Tr) {
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        const int m = pad_src(p + i + a.pl, a.pl, a.Tr, a.e, a.mode);
                        v[i] = m >= 0 ? Rb[(int64_t)row * a.Tr + m] : 0.f;
                    }
                }
                if (ELU_R) {
#pragma unroll
                    for (int i = 0; i < 4; ++i) v[i] = elu_nb(v[i]);
                }
                *(f32x4*)(Rs + row * WLp + 4 * (q - row * RQ)) = v;
            }
        }
    };
    if (it0 < it1) {
        load(it0);
        store(it0, smem);
        __syncthreads();
    }
    for (int it = it0; it < it1; ++it) {
        float* cur = smem + ((it - it0) & 1) * bsz;
        float* nxt = smem + ((it - it0 + 1) & 1) * bsz;
        const bool more = it + 1 < it1;
        if (more) load(it + 1);
        const int t0 = (it % tch) * W2_PT, wb = t0 * S - a.pl, woff = wb - (wb & ~3);
        const float* Ls = cur + wm0 + l32;
        const float* Rs = cur + lsz + woff;
#pragma unroll 8
        for (int p = 0; p < W2_PT; p += 2) {
            float av[TM], bv[TN];
#pragma unroll
            for (int i = 0; i < TM; ++i) av[i] = Ls[(p + h) * LS + i * 32];
#pragma unroll
            for (int j = 0; j < TN; ++j) bv[j] = Rs[bbase[j] + (p + h) * S];
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j) acc[i][j] = mfma32(av[i], bv[j], acc[i][j]);
        }
        if (more) store(it + 1, nxt);
        __syncthreads();
    }
    // the slab of this split: ws[split][a][n]
    float* slab = a.ws + (int64_t)split * a.A * N;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int n = n0 + wn0 + j * 32 + l32;
            if (n >= N) continue;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int row = a0 + wm0 + i * 32 + mfma_row(r, lane);
                slab[(int64_t)row * N + n] = acc[i][j][r];
            }
        }
    if (BIAS && blockIdx.x == 0) {
        // rows' bias partials: the LQR threads of a row sum theirs through LDS (after the loop's
        // final barrier nothing reads the buffers)
        float* red = smem;
#pragma unroll
        for (int e = 0; e < W2_LQ; ++e) {
            const int q = tid + NT * e;
            if (q < nlq) red[q] = bacc[e];
        }
        __syncthreads();
        if (tid < BM) {
            float v = 0.f;
            for (int k = 0; k < LQR; ++k) v += red[tid * LQR + k];
            a.wsb[(int64_t)split * a.A + a0 + tid] = v;
        }
    }
}
struct Wg2Plan { int BM, BN, splits, per_split, items, NC, WLp; size_t lds; };
static bool plan_wgrad2(int64_t B, int64_t A, int64_t Tl, int64_t C, int64_t K, int64_t S, Wg2Plan* p) {
    if (!(encx_opt(OPT_CONV2) & 4) || Tl % 4 || Tl < W2_PT || A % 64) return false;
    p->BM = 64;
    const int64_t N = C * K;
    p->BN = N >= 128 ? 128 : 64;
    p->WLp = w2_wl((int)K, (int)S) & ~3;
    p->NC = (int)std::min<int64_t>(C, (p->BN + K - 1) / K + 1);
    if ((int64_t)p->NC * (p->WLp / 4) > NT * W2_RQ) return false;
    p->lds = (size_t)2 * (((W2_PT * (p->BM + 1) + p->NC * p->WLp) + 3) & ~3) * sizeof(float);
    if (p->lds > 160 * 1024) return false;
    p->items = (int)(B * cdiv(Tl, W2_PT));
    const int64_t tiles = (A / p->BM) * cdiv(N, p->BN);
    const int64_t target = encx_opt(OPT_CONV2_WGS);
    int64_t splits = std::max<int64_t>(1, target / tiles);
    splits = std::min<int64_t>(splits, p->items / 4 > 0 ? p->items / 4 : 1);
    p->per_split = (int)cdiv(p->items, splits);
    p->splits = (int)cdiv(p->items, p->per_split);
    return true;
}
template <int K, int S>
static int wgrad2_launch(const Wg2Args& a, const Wg2Plan& p, bool bias, hipStream_t st) {
    const dim3 grid((unsigned)cdiv((int64_t)a.C * K, p.BN), (unsigned)(a.A / p.BM), (unsigned)p.splits);
    const bool eL = a.actL == ENCX_ACT_ELU, eR = a.actR == ENCX_ACT_ELU;
#define ENCX_W2(BN_, EL, ER, BI) \
    hipLaunchKernelGGL((conv_wgrad2_kernel<64, BN_, K, S, EL, ER, BI>), grid, dim3(NT), p.lds, st, a)
#define ENCX_W2B(BN_)                                   \
    do {                                                \
        if (bias) ENCX_W2(BN_, false, true, true);      \
        else if (eL) ENCX_W2(BN_, true, false, false);  \
        else if (eR) ENCX_W2(BN_, false, true, false);  \
        else ENCX_W2(BN_, false, false, false);         \
    } while (0)
    if (bias && (eL || !eR)) return -1;
    if (p.BN == 128) ENCX_W2B(128);
    else ENCX_W2B(64);
#undef ENCX_W2B
#undef ENCX_W2
    return 0;
}
// -1: not served (the caller runs the round-5 kernels). db (conv only: L = dy, no activation).
static int wgrad2_run(const float* L, const float* R, float* dw, float* ws, int64_t B, int64_t A, int64_t Tl,
                      int64_t C, int64_t Tr, int64_t K, int64_t s, int64_t d, int64_t pl, int64_t e, int mode,
                      int actL, int actR, int accumulate, hipStream_t st, float* db, int acc_b) {
    Wg2Plan p;
    if (d != 1 || !plan_wgrad2(B, A, Tl, C, K, s, &p)) return -1;
    if (((uintptr_t)L | (uintptr_t)R) % 16 || Tr % 4) return -1;
    Wg2Args a;
    a.L = L; a.R = R; a.ws = ws;
    const int64_t AN = A * C * K;
    a.wsb = db ? ws + (int64_t)p.splits * AN : nullptr;
    a.B = (int)B; a.A = (int)A; a.Tl = (int)Tl; a.C = (int)C; a.Tr = (int)Tr; a.K = (int)K; a.s = (int)s;
    a.pl = (int)pl; a.e = (int)e; a.mode = mode; a.actL = actL; a.actR = actR;
    a.items = p.items; a.per_split = p.per_split; a.NC = p.NC; a.WLp = p.WLp;
    int rc = -1;
    switch (K * 16 + s) {
#define ENCX_C1_CASE(K_, S_) \
    case K_ * 16 + S_: rc = wgrad2_launch<K_, S_>(a, p, db != nullptr, st); break;
        ENCX_C1_KS_LIST(ENCX_C1_CASE)
#undef ENCX_C1_CASE
        default: break;
    }
    if (rc) return rc;
    ENCX_CHECK_LAUNCH();
    hipLaunchKernelGGL(wgrad_reduce, dim3((unsigned)(cdiv(AN, 64) + (db ? cdiv(A, 64) : 0))), dim3(256), 0, st, ws, dw,
                       AN, p.splits, accumulate, a.wsb, db, (int)A, acc_b);
    ENCX_CHECK_LAUNCH();
    return 0;
}
static size_t wgrad2_ws(int64_t B, int64_t A, int64_t Tl, int64_t C, int64_t K, int64_t s) {
    Wg2Plan p;
    if (!plan_wgrad2(B, A, Tl, C, K, s, &p)) return 0;
    return (size_t)p.splits * A * (C * K + 1) * sizeof(float);
}

// ---- weight grads of the short-T layers through hipBLASLt: dw (A x C K) = L^T-rows x im2col(R)
// over the N = B Tl positions: L transposed to [N][A] (with its pre-activation), R gathered as the
// forward's im2col [N][C K], one library GEMM straight into dw (accumulating when asked); the
// bias (db = sum of L over positions) as fixed-order column sums of the transposed L
static bool blas_wgrad_ok(int64_t A, int64_t Tl, int64_t N, int64_t CK) {
    if (A < 64) return false;
    if (Tl <= FLAT_T) return blas_flat_ok(CK, A, N);
    return (encx_opt(OPT_BLAS) & 8) && CK >= 256 && N * CK <= (32ll << 20) && 2.0 * A * N * CK >= 8.0e9;
}
static size_t blas_wgrad_ws(int64_t B, int64_t A, int64_t Tl, int64_t C, int64_t K) {
    const int64_t N = B * Tl;
    if (!blas_wgrad_ok(A, Tl, N, C * K)) return 0;
    return (size_t)(N * A + N * C * K + cdiv(N, WGB_ROWS) * A + blas_chunks(N, A * C * K) * A * C * K) *
           sizeof(float);
}
// Lt[b Tl + t][a] = act(L[b][a][t]), 32 x 32 tiles through LDS
__global__ __launch_bounds__(256) void wg_transpose_kernel(const float* L, float* Lt, int A, int Tl, int act) {
    __shared__ float tile[32][33];
    const int t0 = blockIdx.x * 32, a0 = blockIdx.y * 32, b = blockIdx.z, tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
#pragma unroll
    for (int r = ty; r < 32; r += 8)
        tile[r][tx] = (a0 + r < A && t0 + tx < Tl) ? act_apply(act, L[((int64_t)b * A + a0 + r) * Tl + t0 + tx]) : 0.f;
    __syncthreads();
#pragma unroll
    for (int r = ty; r < 32; r += 8)
        if (t0 + r < Tl && a0 + tx < A) Lt[((int64_t)b * Tl + t0 + r) * A + a0 + tx] = tile[tx][r];
}
// db[a] (+)= sum over n of Lt[n][a]: chunk c of WGB_ROWS rows per workgroup column block (4 row
// lanes, each ascending, then the lanes in order), then the chunks in order
__global__ __launch_bounds__(256) void wg_colsum_part(const float* Lt, int N, int A, float* part) {
    __shared__ float red[4][65];
    const int c = threadIdx.x & 63, r = threadIdx.x >> 6;
    const int j = blockIdx.x * 64 + c, n0 = blockIdx.y * WGB_ROWS, n1 = min(N, n0 + WGB_ROWS);
    float sum = 0.f;
    if (j < A)
        for (int n = n0 + r; n < n1; n += 4) sum += Lt[(int64_t)n * A + j];
    red[r][c] = sum;
    __syncthreads();
    if (r == 0 && j < A) part[(int64_t)blockIdx.y * A + j] = ((red[0][c] + red[1][c]) + red[2][c]) + red[3][c];
}
__global__ __launch_bounds__(256) void wg_colsum_fin(const float* part, int nch, int A, float* db, int acc) {
    const int j = blockIdx.x * 256 + threadIdx.x;
    if (j >= A) return;
    float v = part[j];
    for (int c = 1; c < nch; ++c) v += part[(int64_t)c * A + j];
    db[j] = acc ? db[j] + v : v;
}
static int blas_wgrad_run(const float* L, const float* R, float* dw, float* ws, int64_t B, int64_t A, int64_t Tl,
                          int64_t C, int64_t Tr, int64_t K, int64_t s, int64_t d, int64_t pl, int64_t e, int mode,
                          int actL, int actR, int accumulate, hipStream_t st, float* db, int acc_b) {
    const int64_t N = B * Tl, CK = C * K;
    if (!ws || !blas_wgrad_ok(A, Tl, N, CK)) return -1;
    if (db && actL != ENCX_ACT_NONE) return -1;
    float* Lt = ws;
    float* Rc = ws + N * A;
    float* part = Rc + N * CK;
    float* slabs = part + cdiv(N, WGB_ROWS) * A;
    hipLaunchKernelGGL(wg_transpose_kernel, dim3((unsigned)cdiv(Tl, 32), (unsigned)cdiv(A, 32), (unsigned)B), dim3(256),
                       0, st, L, Lt, (int)A, (int)Tl, actL);
    ENCX_CHECK_LAUNCH();
    FwdArgs r{};
    r.x = R; r.B = (int)B; r.Cin = (int)C; r.Tin = (int)Tr; r.K = (int)K; r.s = (int)s; r.d = (int)d; r.pl = (int)pl;
    r.e = (int)e; r.mode = mode; r.act = actR; r.Tout = (int)Tl;
    const LdConvFlat ld{r, make_fastdiv((int)K), make_fastdiv((int)Tl)};
    hipLaunchKernelGGL(im2col_kernel<LdConvFlat>, dim3((unsigned)cdiv(CK, 64), (unsigned)cdiv(N, 16)), dim3(256), 0,
                       st, ld, (int)CK, (int)N, Rc);
    ENCX_CHECK_LAUNCH();
    // slab c (C K x A, column-major = [A][C][K]) = Rc (C K x N) Lt (A x N)^T over position chunk c,
    // then the slabs in order into dw (wgrad_reduce, fp64)
    const int KB = blas_chunks(N, A * CK), kc = (int)(N / KB);
    if (encx_sgemm(st, false, true, (int)CK, (int)A, kc, Rc, (int)CK, Lt, (int)A, slabs, (int)CK, false, KB,
                   (int64_t)kc * CK, (int64_t)kc * A, A * CK))
        return -1;
    hipLaunchKernelGGL(wgrad_reduce, dim3((unsigned)cdiv(A * CK, 64)), dim3(256), 0, st, slabs, dw, A * CK, KB,
                       accumulate, nullptr, nullptr, (int)A, 0);
    ENCX_CHECK_LAUNCH();
    if (db) {
        const int nch = (int)cdiv(N, WGB_ROWS);
        hipLaunchKernelGGL(wg_colsum_part, dim3((unsigned)cdiv(A, 64), (unsigned)nch), dim3(256), 0, st, Lt, (int)N,
                           (int)A, part);
        hipLaunchKernelGGL(wg_colsum_fin, dim3((unsigned)cdiv(A, 256)), dim3(256), 0, st, part, nch, (int)A, db, acc_b);
        ENCX_CHECK_LAUNCH();
    }
    return 0;
}

int wgrad_run(const float* L, const float* R, float* dw, float* ws, int64_t B, int64_t A,
              int64_t Tl, int64_t C, int64_t Tr, int64_t K, int64_t s, int64_t d, int64_t pl,
              int64_t e, int mode, int actL, int actR, int accumulate, hipStream_t st,
              float* db = nullptr, int acc_b = 0) {
    {
        const int rc = blas_wgrad_run(L, R, dw, ws, B, A, Tl, C, Tr, K, s, d, pl, e, mode, actL, actR, accumulate, st,
                                      db, acc_b);
        if (rc >= 0) return rc;
    }
    {
        const int rc = wgrad2_run(L, R, dw, ws, B, A, Tl, C, Tr, K, s, d, pl, e, mode, actL, actR, accumulate, st, db,
                                  acc_b);
        if (rc >= 0) return rc;
    }
    WgPlan p = plan_wgrad(B, A, Tl, C, K);
    WgArgs a;
    a.L = L; a.R = R; a.ws = ws;
    // the bias slabs follow the weight slabs (db = sum over t of L: L must be the conv's dy, act none)
    if (db && (actL != ENCX_ACT_NONE || (p.kind == 0 && A * C * K + A > NT))) return ENCX_EINVAL;
    a.wsb = db ? ws + (int64_t)p.splits * A * C * K : nullptr;
    a.B = (int)B; a.A = (int)A; a.Tl = (int)Tl; a.C = (int)C; a.Tr = (int)Tr; a.K = (int)K;
    a.s = (int)s; a.d = (int)d; a.pl = (int)pl; a.e = (int)e; a.mode = mode; a.actL = actL;
    a.actR = actR; a.BT = p.BT; a.items = p.items; a.per_split = p.per_split;
    const int WL = (p.BT - 1) * a.s + (a.K - 1) * a.d + 1;
    const int64_t AN = A * C * K;
    if (p.kind == 0) {
        const bool win7 = s == 1 && d == 1 && K == 7 && A * C <= NT;
        a.WLp = win7 ? (WL | 1) : WL;  // (odd: the window rows of a wave's pairs on distinct banks)
        a.NCmax = (int)C;
        size_t lds = (size_t)(A * (p.BT + 1) + C * a.WLp) * sizeof(float);
        if (win7) lds = std::max(lds, (size_t)NT * 8 * sizeof(float));  // the segment reduction
        if (lds > 160 * 1024) return ENCX_EINVAL;
        if (win7) hipLaunchKernelGGL(conv_wgrad_small_kernel<7>, dim3(p.splits), dim3(NT), lds, st, a);
        else hipLaunchKernelGGL(conv_wgrad_small_kernel<0>, dim3(p.splits), dim3(NT), lds, st, a);
    } else {
        a.WLp = wlp_for(WL, a.K);
        a.NCmax = (int)((p.BN + a.K - 1) / a.K + 1);
        if (a.NCmax > C) a.NCmax = (int)C;
        if (p.kind == 1) {
            if (p.BM == 32) launch_wg<32, 32, 1, 1, 4>(a, p.splits, st);
            else launch_wg<64, 32, 2, 1, 2>(a, p.splits, st);
        } else if (p.BM == 32) launch_wg<32, 128, 1, 4, 1>(a, p.splits, st);
        else if (p.BM == 64) launch_wg<64, 128, 2, 2, 1>(a, p.splits, st);
        else launch_wg<128, 128, 2, 2, 1>(a, p.splits, st);
    }
    ENCX_CHECK_LAUNCH();
    hipLaunchKernelGGL(wgrad_reduce, dim3(cdiv(AN, 64) + (db ? cdiv(A, 64) : 0)), dim3(256), 0, st, ws, dw, AN,
                       p.splits, accumulate, a.wsb, db, (int)A, acc_b);
    ENCX_CHECK_LAUNCH();
    return 0;
}

size_t wgrad_ws_bytes(int64_t B, int64_t A, int64_t Tl, int64_t C, int64_t K) {
    WgPlan p = plan_wgrad(B, A, Tl, C, K);
    // (+ the bias slabs; the v2 plan's splits do not depend on the stride)
    return std::max({(size_t)p.splits * A * (C * K + 1) * sizeof(float), wgrad2_ws(B, A, Tl, C, K, 1),
                     blas_wgrad_ws(B, A, Tl, C, K)});
}

static size_t maxz(size_t a, size_t b) { return a > b ? a : b; }

// Backward-data of a dilated Conv1d (any stride): the gradient of every padded input position,
// g[p] = sum_{co,k : p = t*s + k*d} wf[ci][k][co] * dy[co][t], one thread per position (the
// block's (b, ci) row is uniform, so the weight loads are scalar). Interior positions take
// act'(x) (+ dx) and land in dx; pad positions go to the side buffer for conv_fold_edges. A direct
// VALU form: EnCodec's configurations use d = 1 (modules/seanet.py:114-117 dilates only with
// n_residual_layers > 1), so this is the general path, not a hot one.
__global__ void conv_dgrad_dilated_kernel(const float* __restrict__ dy, const float* __restrict__ wf,
                                          const float* __restrict__ xact, float* __restrict__ dx,
                                          float* __restrict__ side, int Cin, int Tx, int Cout, int Tout,
                                          int K, int s, int d, int pl, int pr, int act, int accumulate) {
    const int row = blockIdx.y;  // b * Cin + ci
    const int b = row / Cin, ci = row - b * Cin;
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    const int Tpad = pl + Tx + pr;
    if (p >= Tpad) return;
    const float* dyb = dy + (int64_t)b * Cout * Tout;
    const float* w = wf + (int64_t)ci * K * Cout;
    float g = 0.f;
    for (int k = 0; k < K; ++k) {
        const int q = p - k * d;
        if (q < 0 || q % s) continue;
        const int t = q / s;
        if (t >= Tout) continue;
        for (int co = 0; co < Cout; ++co) g = fmaf(w[k * Cout + co], dyb[(int64_t)co * Tout + t], g);
    }
    const int m = p - pl;
    if (m >= 0 && m < Tx) {
        const int64_t idx = (int64_t)row * Tx + m;
        if (act != ENCX_ACT_NONE) g *= act_grad(act, xact[idx]);
        dx[idx] = accumulate ? dx[idx] + g : g;
    } else if (side) {
        side[(int64_t)row * (pl + pr) + (m < 0 ? p : p - Tx)] = g;
    }
}

}  // namespace

// ============================================================================ C ABI
extern "C" {

size_t encx_conv1d_fwd_workspace(int64_t B, int64_t Cin, int64_t Cout, int64_t Tout, int64_t K,
                                 int64_t stride, int64_t dilation) {
    return conv_fwd_ws(B, Cin, Cout, Tout, K, stride, dilation);
}

int encx_conv1d_fwd(const float* x, const float* wf, const float* bias, const float* residual,
                    float* y, float* ws, int64_t B, int64_t Cin, int64_t Tin, int64_t Cout,
                    int64_t Tout, int64_t K, int64_t stride, int64_t dilation, int64_t pad_left,
                    int64_t short_ext, int pad_mode, int pre_act, encx_stream_t stream) {
    ENCX_REQUIRE(x && wf && y && B > 0 && Cin > 0 && Cout > 0 && Tin > 0 && Tout > 0);
    ENCX_REQUIRE(K > 0 && stride > 0 && dilation > 0 && pad_left >= 0 && short_ext >= 0);
    hipStream_t st = (hipStream_t)stream;
    FwdArgs a;
    a.x = x; a.wf = wf; a.bias = bias; a.res = residual; a.y = y; a.xact = nullptr; a.part = nullptr;
    a.B = (int)B; a.Cin = (int)Cin; a.Tin = (int)Tin; a.Cout = (int)Cout; a.Tout = (int)Tout;
    a.K = (int)K; a.s = (int)stride; a.d = (int)dilation; a.pl = (int)pad_left; a.e = (int)short_ext;
    a.mode = pad_mode; a.act = pre_act; a.epi_act = ENCX_ACT_NONE; a.accumulate = 0;
    encx_prof_scope ps(st, 2.0 * B * Cout * Tout * Cin * K,
                       4.0 * (B * Cin * Tin + B * Cout * Tout * (residual ? 2 : 1) + Cin * K * Cout), "conv_fwd");
    ps.tag(" %ldx%ld k%ld s%ld T%ld", (long)Cin, (long)Cout, (long)K, (long)stride, (long)Tout);
    return conv_fwd_run(a, ws, st);
}

size_t encx_conv1d_bwd_data_workspace(int64_t B, int64_t Cin, int64_t Tin, int64_t Cout,
                                      int64_t Tout, int64_t K, int64_t stride, int64_t pad_left,
                                      int64_t pad_right) {
    const int64_t Tpad = pad_left + Tin + pad_right;
    const int64_t ncols = cdiv(Tpad, stride);
    size_t side = (size_t)(B * Cin * (pad_left + pad_right) + 1) * sizeof(float);
    side = (side + 255) & ~(size_t)255;
    return side + poly_ws(B, Cout, Cin, stride, ncols, cdiv(K, stride));
}

int encx_conv1d_bwd_data(const float* dy, const float* wp, const float* x, float* dx, float* ws,
                         int64_t B, int64_t Cin, int64_t Tin, int64_t Cout, int64_t Tout,
                         int64_t K, int64_t stride, int64_t pad_left, int64_t pad_right,
                         int64_t short_ext, int pad_mode, int pre_act, int accumulate,
                         encx_stream_t stream) {
    ENCX_REQUIRE(dy && wp && dx && ws && B > 0 && Cin > 0 && Cout > 0 && Tin > 0 && Tout > 0);
    ENCX_REQUIRE(pre_act == ENCX_ACT_NONE || x);
    hipStream_t st = (hipStream_t)stream;
    size_t side_b = (size_t)(B * Cin * (pad_left + pad_right) + 1) * sizeof(float);
    side_b = (side_b + 255) & ~(size_t)255;
    float* side = ws;
    float* part = (float*)((char*)ws + side_b);
    PolyArgs a;
    a.in = dy; a.wp = wp; a.bias = nullptr; a.xact = x; a.out = dx; a.side = side;
    a.B = (int)B; a.Ci = (int)Cout; a.Tin = (int)Tout; a.Co = (int)Cin; a.s = (int)stride;
    a.J = (int)cdiv(K, stride); a.mode = 1; a.trim = 0; a.Tout = 0;
    a.pl = (int)pad_left; a.pr = (int)pad_right; a.Tx = (int)Tin;
    a.act = pre_act; a.in_act = ENCX_ACT_NONE; a.accumulate = accumulate;
    const int64_t Tpad = pad_left + Tin + pad_right;
    const int ncols = (int)cdiv(Tpad, stride);
    encx_prof_scope ps(st, 2.0 * B * Cout * Tout * Cin * K,
                       4.0 * (B * Cout * Tout + B * Cin * Tin * (1 + (pre_act ? 1 : 0) + (accumulate ? 1 : 0)) + Cin * K * Cout), "conv_dgrad");
    ps.tag(" %ldx%ld k%ld s%ld T%ld", (long)Cin, (long)Cout, (long)K, (long)stride, (long)Tout);
    // (the long 1x1 layers go to the v2 polyphase kernel when it is on)
    if (pw_ok((int)K, (int)stride, 1, (int)pad_left, (int)pad_right, (int)short_ext, (int)Tin, (int)Tout, (int)Cin,
              (int)Cout, (int)Cout) &&
        !((encx_opt(OPT_CONV2) & 2) && Tout > encx_opt(OPT_PW_TMAX))) {
        // dx[b][ci][t] = sum_co wp[co][ci] dy[b][co][t], * act'(x), (+ dx)
        PwArgs p{wp, dy, nullptr, nullptr, x, dx, (int)Cin, (int)Cout, (int)Tout, ENCX_ACT_NONE, pre_act};
        const int epi = (pre_act != ENCX_ACT_NONE ? PW_XACT : 0) | (accumulate ? PW_ACC : 0);
        if (pw_launch(p, (int)B, epi, st) == 0) return 0;
    }
    int rc = poly_run(a, ncols, part, st);
    if (rc) return rc;
    if (pad_left + pad_right > 0 && pad_mode == ENCX_PAD_REFLECT) {
        int rows = (int)(B * Cin);
        hipLaunchKernelGGL(conv_fold_edges, dim3(cdiv(rows, 256)), dim3(256), 0, st, side, x, dx,
                           rows, (int)Tin, (int)pad_left, (int)pad_right, (int)short_ext, pad_mode,
                           pre_act);
        ENCX_CHECK_LAUNCH();
    }
    return 0;
}

int encx_conv1d_bwd_data_dilated(const float* dy, const float* wf, const float* x, float* dx, float* ws,
                                 int64_t B, int64_t Cin, int64_t Tin, int64_t Cout, int64_t Tout,
                                 int64_t K, int64_t stride, int64_t dilation, int64_t pad_left,
                                 int64_t pad_right, int64_t short_ext, int pad_mode, int pre_act,
                                 int accumulate, encx_stream_t stream) {
    ENCX_REQUIRE(dy && wf && dx && B > 0 && Cin > 0 && Cout > 0 && Tin > 0 && Tout > 0 && K > 0);
    ENCX_REQUIRE(stride > 0 && dilation > 0 && pad_left >= 0 && pad_right >= 0 && short_ext >= 0);
    ENCX_REQUIRE(pre_act == ENCX_ACT_NONE || x);
    const int64_t Tpad = pad_left + Tin + pad_right;
    ENCX_REQUIRE((Tout - 1) * stride + (K - 1) * dilation < Tpad && B * Cin <= 65535);
    const bool fold = pad_left + pad_right > 0 && pad_mode == ENCX_PAD_REFLECT;
    ENCX_REQUIRE(!fold || ws);
    hipStream_t st = (hipStream_t)stream;
    encx_prof_scope ps(st, 2.0 * B * Cout * Tout * Cin * K,
                       4.0 * (B * Cout * Tout + B * Cin * Tin * (1 + (pre_act ? 1 : 0) + (accumulate ? 1 : 0)) + Cin * K * Cout),
                       "conv_dgrad");
    ps.tag(" %ldx%ld k%ld s%ld d%ld T%ld", (long)Cin, (long)Cout, (long)K, (long)stride, (long)dilation, (long)Tout);
    hipLaunchKernelGGL(conv_dgrad_dilated_kernel, dim3(cdiv(Tpad, 256), B * Cin), dim3(256), 0, st, dy, wf, x, dx,
                       fold ? ws : nullptr, (int)Cin, (int)Tin, (int)Cout, (int)Tout, (int)K, (int)stride,
                       (int)dilation, (int)pad_left, (int)pad_right, pre_act, accumulate);
    ENCX_CHECK_LAUNCH();
    if (fold) {
        const int rows = (int)(B * Cin);
        hipLaunchKernelGGL(conv_fold_edges, dim3(cdiv(rows, 256)), dim3(256), 0, st, ws, x, dx, rows, (int)Tin,
                           (int)pad_left, (int)pad_right, (int)short_ext, pad_mode, pre_act);
        ENCX_CHECK_LAUNCH();
    }
    return 0;
}

int encx_conv1d_bwd_weight(const float* dy, const float* x, float* dw, float* db, float* ws,
                           int64_t B, int64_t Cin, int64_t Tin, int64_t Cout, int64_t Tout,
                           int64_t K, int64_t stride, int64_t dilation, int64_t pad_left,
                           int64_t short_ext, int pad_mode, int pre_act, int accumulate,
                           encx_stream_t stream) {
    return encx_conv1d_bwd_weight_bias(dy, x, dw, db, ws, B, Cin, Tin, Cout, Tout, K, stride, dilation, pad_left,
                                       short_ext, pad_mode, pre_act, accumulate, accumulate, stream);
}

int encx_conv1d_bwd_weight_bias(const float* dy, const float* x, float* dw, float* db, float* ws, int64_t B,
                                int64_t Cin, int64_t Tin, int64_t Cout, int64_t Tout, int64_t K, int64_t stride,
                                int64_t dilation, int64_t pad_left, int64_t short_ext, int pad_mode, int pre_act,
                                int acc_w, int acc_b, encx_stream_t stream) {
    ENCX_REQUIRE(dy && x && dw && ws && B > 0);
    hipStream_t st = (hipStream_t)stream;
    encx_prof_scope ps(st, 2.0 * B * Cout * Tout * Cin * K, 4.0 * (B * Cout * Tout + B * Cin * Tin + Cin * K * Cout), "conv_wgrad");
    ps.tag(" %ldx%ld k%ld s%ld T%ld", (long)Cin, (long)Cout, (long)K, (long)stride, (long)Tout);
    if (pw_wgrad_ok(K, stride, dilation, pad_left, short_ext, Tin, Tout, Cin, Cout)) {
        pw_wgrad_run(dy, x, dw, db, ws, B, Cout, Cin, Tout, pre_act, acc_w, acc_b, st);
        ENCX_CHECK_LAUNCH();
        return 0;
    }
    const bool fused = db && wgrad_bias_ok(B, Cout, Tout, Cin, K);
    int rc = wgrad_run(dy, x, dw, ws, B, Cout, Tout, Cin, Tin, K, stride, dilation, pad_left, short_ext, pad_mode,
                       ENCX_ACT_NONE, pre_act, acc_w, st, fused ? db : nullptr, acc_b);
    if (rc || !db || fused) return rc;
    return encx_channel_sum(dy, db, ws, B, Cout, Tout, acc_b, stream);
}

size_t encx_conv1d_bwd_weight_workspace(int64_t B, int64_t Cin, int64_t Cout, int64_t Tout,
                                        int64_t K) {
    return maxz(maxz(wgrad_ws_bytes(B, Cout, Tout, Cin, K), encx_channel_sum_workspace(Cout)),
                K == 1 ? pw_wgrad_ws_bytes(B, Cout, Cin, Tout) : 0);
}

size_t encx_convtr1d_fwd_workspace(int64_t B, int64_t Cin, int64_t Cout, int64_t Tout, int64_t K,
                                   int64_t stride, int64_t trim_left) {
    return poly_ws(B, Cin, Cout, stride, cdiv(Tout + trim_left, stride), cdiv(K, stride));
}

int encx_convtr1d_fwd(const float* x, const float* wp, const float* bias, float* y, float* ws,
                      int64_t B, int64_t Cin, int64_t Tin, int64_t Cout, int64_t Tout, int64_t K,
                      int64_t stride, int64_t trim_left, int pre_act, encx_stream_t stream) {
    ENCX_REQUIRE(x && wp && y && B > 0 && Cin > 0 && Cout > 0 && Tin > 0 && Tout > 0);
    hipStream_t st = (hipStream_t)stream;
    PolyArgs a;
    a.in = x; a.wp = wp; a.bias = bias; a.xact = nullptr; a.out = y; a.side = nullptr;
    a.B = (int)B; a.Ci = (int)Cin; a.Tin = (int)Tin; a.Co = (int)Cout; a.s = (int)stride;
    a.J = (int)cdiv(K, stride); a.mode = 0; a.trim = (int)trim_left; a.Tout = (int)Tout;
    a.pl = a.pr = a.Tx = 0; a.act = ENCX_ACT_NONE; a.in_act = pre_act; a.accumulate = 0;
    const int ncols = (int)cdiv(Tout + trim_left, stride);
    encx_prof_scope ps(st, 2.0 * B * Cin * Tin * Cout * K, 4.0 * (B * Cin * Tin + B * Cout * Tout + Cin * K * Cout), "convtr_fwd");
    ps.tag(" %ldx%ld k%ld s%ld T%ld", (long)Cin, (long)Cout, (long)K, (long)stride, (long)Tout);
    return poly_run(a, ncols, ws, st);
}

size_t encx_convtr1d_bwd_data_workspace(int64_t B, int64_t Cin, int64_t Tin, int64_t Cout,
                                        int64_t K, int64_t stride) {
    return conv_fwd_ws(B, Cout, Cin, Tin, K, stride, 1);
}

int encx_convtr1d_bwd_data(const float* dy, const float* wf, const float* x, float* dx, float* ws,
                           int64_t B, int64_t Cin, int64_t Tin, int64_t Cout, int64_t Tout,
                           int64_t K, int64_t stride, int64_t trim_left, int pre_act,
                           int accumulate, encx_stream_t stream) {
    // dx[ci,t] = [acc ? dx : 0] + act'(x) * sum_{co,k} Wt[ci,co,k] dy[co, t*s+k-trim_left]
    // (zero outside [0,Tout)): a forward conv of dy with zero padding pad_left = trim_left.
    ENCX_REQUIRE(dy && wf && dx && B > 0 && Cin > 0 && Cout > 0 && Tin > 0 && Tout > 0);
    ENCX_REQUIRE(pre_act == ENCX_ACT_NONE || x);
    hipStream_t st = (hipStream_t)stream;
    FwdArgs a;
    a.x = dy; a.wf = wf; a.bias = nullptr; a.res = nullptr; a.y = dx; a.part = nullptr;
    a.xact = pre_act != ENCX_ACT_NONE ? x : nullptr;
    a.B = (int)B; a.Cin = (int)Cout; a.Tin = (int)Tout; a.Cout = (int)Cin; a.Tout = (int)Tin;
    a.K = (int)K; a.s = (int)stride; a.d = 1; a.pl = (int)trim_left; a.e = 0;
    a.mode = ENCX_PAD_ZERO; a.act = ENCX_ACT_NONE; a.epi_act = pre_act; a.accumulate = accumulate;
    encx_prof_scope ps(st, 2.0 * B * Cin * Tin * Cout * K,
                       4.0 * (B * Cout * Tout + B * Cin * Tin * (1 + (pre_act ? 1 : 0) + (accumulate ? 1 : 0)) + Cin * K * Cout), "convtr_dgrad");
    ps.tag(" %ldx%ld k%ld s%ld T%ld", (long)Cin, (long)Cout, (long)K, (long)stride, (long)Tout);
    return conv_fwd_run(a, ws, st);
}

int encx_convtr1d_bwd_weight(const float* x, const float* dy, float* dw, float* db, float* ws,
                             int64_t B, int64_t Cin, int64_t Tin, int64_t Cout, int64_t Tout,
                             int64_t K, int64_t stride, int64_t trim_left, int pre_act,
                             int accumulate, encx_stream_t stream) {
    ENCX_REQUIRE(x && dy && dw && ws && B > 0);
    hipStream_t st = (hipStream_t)stream;
    encx_prof_scope ps(st, 2.0 * B * Cin * Tin * Cout * K, 4.0 * (B * Cout * Tout + B * Cin * Tin + Cin * K * Cout), "convtr_wgrad");
    ps.tag(" %ldx%ld k%ld s%ld T%ld", (long)Cin, (long)Cout, (long)K, (long)stride, (long)Tout);
    // L = act(x) [ci][t], R = dy [co][t*s + k - trim_left] zero-padded
    int rc = wgrad_run(x, dy, dw, ws, B, Cin, Tin, Cout, Tout, K, stride, 1, trim_left, 0,
                       ENCX_PAD_ZERO, pre_act, ENCX_ACT_NONE, accumulate, st);
    if (rc) return rc;
    if (db) return encx_channel_sum(dy, db, ws, B, Cout, Tout, accumulate, stream);
    return 0;
}

size_t encx_convtr1d_bwd_weight_workspace(int64_t B, int64_t Cin, int64_t Cout, int64_t Tin,
                                          int64_t K) {
    return maxz(wgrad_ws_bytes(B, Cin, Tin, Cout, K), encx_channel_sum_workspace(Cout));
}

}  // extern "C"
