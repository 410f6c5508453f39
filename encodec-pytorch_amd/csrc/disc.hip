// MS-STFT discriminator (msstftd.py:28-149) and its losses (losses.py:44-80) on gfx950.
//
//   spectrogram  torchaudio Spectrogram(normalized, center=False, power=None) as a DFT GEMM:
//                frames gathered from the waveform while staging, [w cos | -w sin] table
//                shared with the mel loss; the epilogue writes the cat([re, im]) and
//                'b c w t -> b c t w' layout directly. Backward: the transposed GEMM + a
//                fixed-order overlap-add.
//   NormConv2d   (modules/conv.py:125-139) as three implicit GEMMs over v_mfma_f32_32x32x2_f32:
//     fwd    Y[co][(t,f)]  = sum_{(ci,kt),kf} W * X[ci][t+kt*dt-pt][f*sf+kf-pf]; the (t, f)
//            output positions of a batch item are flattened into one GEMM column space so
//            narrow late layers (F = 33..65) still fill 32-wide MFMA tiles; every tile stages
//            the input rows it touches (one window per (ci, kt) and output row) in LDS.
//            Bias + LeakyReLU(0.2) fused in the epilogue.
//     dgrad  polyphase along f (rows (ci, r), columns (t, u), reduction ((co, kt), q)), the
//            output-grad mask LeakyReLU'(y) applied while staging, the input's LeakyReLU'
//            applied in the epilogue; every dX element is written exactly once.
//     wgrad  dW[co][((ci,kt),kf)] + the bias as a ones column, split over (b, position chunk)
//            work items into slabs, summed in a fixed order (deterministic).
#include "common.h"
#include "gemm.h"
#include "fft.h"
#include "prof.h"

namespace {

constexpr int NT = 256;
constexpr int DPER = 8;  // staging loads in flight per thread
constexpr int WG_BT = 64;  // wgrad: output positions per work item

struct C2Geo {
    int B, Ci, T2, Fi, Co, Fo, KT, KF, sf, dt, pt, pf;
};

// ------------------------------------------------------------------------------- forward
struct C2Fwd {
    C2Geo g;
    const float* x;
    const float* wf;  // [(ci,kt)][kf][co]
    const float* bias;
    float* y;
    int act;
    int CK, NR, RL;
};

template <int BM, int BN, int WM, int WN, int KFC = 0>
__global__ __launch_bounds__(NT) void c2_fwd_kernel(C2Fwd a) {
    constexpr int TM = BM / WM / 32, TN = BN / WN / 32;
    extern __shared__ float smem[];
    const C2Geo g = a.g;
    const int CK = a.CK, NR = a.NR, RL = a.RL, KF = g.KF, S = g.sf;
    const int VC = g.Ci * g.KT, XR = NR * RL;
    float* Xs = smem;           // [CK][NR][RL]
    float* Ws = smem + CK * XR; // [CK][KF][BM]
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm0 = (wave / WN) * TM * 32, wn0 = (wave % WN) * TN * 32;
    const int h = lane >> 5, l32 = lane & 31;
    const int b = blockIdx.z, n0 = blockIdx.x * BN, co0 = blockIdx.y * BM;
    const int Nall = g.T2 * g.Fo, nend = min(Nall, n0 + BN);
    const int tf = n0 / g.Fo, f0 = n0 - tf * g.Fo;
    const int nr = (nend - 1) / g.Fo - tf + 1;
    int boff[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) {
        const int n = n0 + wn0 + j * 32 + l32;
        boff[j] = 0;
        if (n < nend) {
            const int tr = n / g.Fo, f = n - tr * g.Fo, rs = tr - tf;
            boff[j] = rs * RL + (f - (rs ? 0 : f0)) * S;
        }
    }
    f32x16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = (f32x16){0};
    const float* xb = a.x + (int64_t)b * g.Ci * g.T2 * g.Fi;
    // Staging without per-element division: a table of the window rows (global row
    // gr = vc*NR + rs -> source offset of column 0, first column position or "invalid"), built
    // once; each thread walks its items (row r, column w) by a fixed step of NT; the weight
    // items keep their column (NT is a multiple of BM) and step the (kf, cl) row.
    int2* rtab = (int2*)(Ws + KF * CK * BM);  // {source offset of column 0, first position}
    for (int gr = tid; gr < VC * NR; gr += NT) {
        const int vc = gr / NR, rs = gr - vc * NR, ci = vc / g.KT, kt = vc - ci * g.KT;
        const int row = tf + rs + kt * g.dt - g.pt, pos0 = (rs ? 0 : f0) * S - g.pf;
        const bool ok = rs < nr && row >= 0 && row < g.T2;
        rtab[gr] = make_int2(ok ? (ci * g.T2 + row) * g.Fi + pos0 : 0, ok ? pos0 : -(1 << 30));
    }
    const int dr = NT / RL, dw = NT - dr * RL, r_init = tid / RL, w_init = tid - r_init * RL;
    const int wcol = tid & (BM - 1);
    for (int c0 = 0; c0 < VC; c0 += CK) {
        __syncthreads();
        {
            const int nrows = min(CK, VC - c0) * NR, items = CK * XR;
            int r = r_init, w = w_init;
            for (int i0 = 0; i0 < items; i0 += NT * DPER) {
                // (row, column) of the DPER items, then their table entries, then the loads
                int rq[DPER], wq[DPER];
#pragma unroll
                for (int q = 0; q < DPER; ++q) {
                    rq[q] = r;
                    wq[q] = w;
                    w += dw;
                    r += dr;
                    if (w >= RL) {
                        w -= RL;
                        ++r;
                    }
                }
                int2 e[DPER];
#pragma unroll
                for (int q = 0; q < DPER; ++q) e[q] = rtab[c0 * NR + (rq[q] < nrows ? rq[q] : 0)];
                float v[DPER];
#pragma unroll
                for (int q = 0; q < DPER; ++q) {
                    const int pos = e[q].y + wq[q];
                    const bool ok = rq[q] < nrows && pos >= 0 && pos < g.Fi;
                    const float t = xb[ok ? e[q].x + wq[q] : 0];
                    v[q] = ok ? t : 0.f;
                }
#pragma unroll
                for (int q = 0; q < DPER; ++q) {
                    const int i = i0 + q * NT + tid;
                    if (i < items) Xs[i] = v[q];
                }
            }
        }
        {
            // Ws[cl][kf][col] = wf[(c0 + cl, kf)][co0 + col]: rows (cl, kf) are consecutive rows
            // of wf, so an item's source needs no division
            const int items = KF * CK * BM, rows = (VC - c0) * KF, co = co0 + wcol;
            const float* wsrc = a.wf + (int64_t)c0 * KF * g.Co + co;
            for (int i0 = 0; i0 < items; i0 += NT * DPER) {
                float v[DPER];
#pragma unroll
                for (int q = 0; q < DPER; ++q) {
                    const int rr = (i0 + q * NT + tid) / BM;
                    const bool ok = rr < rows && co < g.Co;
                    const float t = wsrc[ok ? (int64_t)rr * g.Co : 0];
                    v[q] = ok ? t : 0.f;
                }
#pragma unroll
                for (int q = 0; q < DPER; ++q) {
                    const int i = i0 + q * NT + tid;
                    if (i < items) Ws[i] = v[q];
                }
            }
        }
        __syncthreads();
        if constexpr (KFC > 0) {
            // k-pairs = combo pairs (cp, cp+1); the KF taps of a pair unrolled, so every
            // accumulator sees KFC independent MFMAs per loop trip and the loads run ahead
            for (int cp = 0; cp < CK; cp += 2) {
                const float* wk = Ws + (cp + h) * KFC * BM + wm0 + l32;
                const float* xk = Xs + (cp + h) * XR;
#pragma unroll
                for (int kf = 0; kf < KFC; ++kf) {
                    float av[TM], bv[TN];
#pragma unroll
                    for (int i = 0; i < TM; ++i) av[i] = wk[kf * BM + i * 32];
#pragma unroll
                    for (int j = 0; j < TN; ++j) bv[j] = xk[boff[j] + kf];
#pragma unroll
                    for (int i = 0; i < TM; ++i)
#pragma unroll
                        for (int j = 0; j < TN; ++j) acc[i][j] = mfma32(av[i], bv[j], acc[i][j]);
                }
            }
        } else {
            for (int kf = 0; kf < KF; ++kf) {
                const float* wk = Ws + (h * KF + kf) * BM + wm0 + l32;
                const float* xk = Xs + h * XR + kf;
                for (int cp = 0; cp < CK; cp += 2) {
                    float av[TM], bv[TN];
#pragma unroll
                    for (int i = 0; i < TM; ++i) av[i] = wk[cp * KF * BM + i * 32];
#pragma unroll
                    for (int j = 0; j < TN; ++j) bv[j] = xk[cp * XR + boff[j]];
#pragma unroll
                    for (int i = 0; i < TM; ++i)
#pragma unroll
                        for (int j = 0; j < TN; ++j) acc[i][j] = mfma32(av[i], bv[j], acc[i][j]);
                }
            }
        }
    }
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int n = n0 + wn0 + j * 32 + l32;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int co = co0 + wm0 + i * 32 + mfma_row(r, lane);
                const float bco = a.bias ? a.bias[co < g.Co ? co : g.Co - 1] : 0.f;  // unconditional load
                if (co < g.Co && n < nend) {
                    float v = acc[i][j][r] + bco;
                    if (a.act) v = lrelu(v);
                    a.y[((int64_t)b * g.Co + co) * Nall + n] = v;
                }
            }
        }
}

// Forward, register-pipelined. Same implicit GEMM and LDS image as c2_fwd_kernel (BM = 32 rows,
// BN columns, CK combos of (ci, kt) per chunk, KF taps unrolled), but the next chunk's window
// and weights are fetched into registers (MX + MW values per thread, every load issued from a
// clamped address and selected afterwards) before the current chunk's MFMAs run: the staging
// latency hides behind the matrix work instead of stalling every workgroup of a CU in step.
template <int BN, int KFC, int CK, int MX>
__global__ __launch_bounds__(NT) void c2_fwdp_kernel(C2Fwd a) {
    constexpr int BM = 32, TN = BN / 128, WI = KFC * CK * BM, MW = (WI + NT - 1) / NT;
    extern __shared__ float smem[];
    const C2Geo g = a.g;
    const int NR = a.NR, RL = a.RL, S = g.sf;
    const int VC = g.Ci * g.KT, XR = NR * RL, XI = CK * XR;
    float* Xs = smem;                  // [CK][NR][RL]
    float* Ws = smem + XI;             // [CK][KFC][BM]
    int2* rtab = (int2*)(Ws + WI);     // [VC*NR]
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int h = lane >> 5, l32 = lane & 31;
    const int b = blockIdx.z, n0 = blockIdx.x * BN, co0 = blockIdx.y * BM;
    const int wn0 = wave * TN * 32;
    const int Nall = g.T2 * g.Fo, nend = min(Nall, n0 + BN);
    const int tf = n0 / g.Fo, f0 = n0 - tf * g.Fo;
    const int nr = (nend - 1) / g.Fo - tf + 1;
    int boff[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) {
        const int n = n0 + wn0 + j * 32 + l32;
        boff[j] = 0;
        if (n < nend) {
            const int tr = n / g.Fo, f = n - tr * g.Fo, rs = tr - tf;
            boff[j] = rs * RL + (f - (rs ? 0 : f0)) * S;
        }
    }
    f32x16 acc[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[j] = (f32x16){0};
    const float* xb = a.x + (int64_t)b * g.Ci * g.T2 * g.Fi;
    for (int gr = tid; gr < VC * NR; gr += NT) {
        const int vc = gr / NR, rs = gr - vc * NR, ci = vc / g.KT, kt = vc - ci * g.KT;
        const int row = tf + rs + kt * g.dt - g.pt, pos0 = (rs ? 0 : f0) * S - g.pf;
        const bool ok = rs < nr && row >= 0 && row < g.T2;
        rtab[gr] = make_int2(ok ? (ci * g.T2 + row) * g.Fi + pos0 : 0, ok ? pos0 : -(1 << 30));
    }
    __syncthreads();
    const int dr = NT / RL, dw = NT - dr * RL, r_init = tid / RL, w_init = tid - r_init * RL;
    float rx[MX], rw[MW];
    auto fetch = [&](int c0) {
        const int nrows = min(CK, VC - c0) * NR;
        int r = r_init, w = w_init;
#pragma unroll
        for (int q = 0; q < MX; ++q) {
            const int2 e = rtab[c0 * NR + (r < nrows ? r : 0)];
            const int pos = e.y + w;
            const bool ok = r < nrows && pos >= 0 && pos < g.Fi;
            const float t = xb[ok ? e.x + w : 0];
            rx[q] = ok ? t : 0.f;
            w += dw;
            r += dr;
            if (w >= RL) {
                w -= RL;
                ++r;
            }
        }
        const float* wsrc = a.wf + (int64_t)c0 * KFC * g.Co + co0;
        const int wrows = (VC - c0) * KFC;
#pragma unroll
        for (int q = 0; q < MW; ++q) {
            const int j = q * NT + tid, rr = j / BM, col = j & (BM - 1);
            const bool ok = j < WI && rr < wrows && co0 + col < g.Co;
            const float t = wsrc[ok ? (int64_t)rr * g.Co + col : 0];
            rw[q] = ok ? t : 0.f;
        }
    };
    fetch(0);
    for (int c0 = 0; c0 < VC; c0 += CK) {
        __syncthreads();
#pragma unroll
        for (int q = 0; q < MX; ++q)
            if (q * NT + tid < XI) Xs[q * NT + tid] = rx[q];
#pragma unroll
        for (int q = 0; q < MW; ++q)
            if (q * NT + tid < WI) Ws[q * NT + tid] = rw[q];
        __syncthreads();
        if (c0 + CK < VC) fetch(c0 + CK);
#pragma unroll 2
        for (int cp = 0; cp < CK; cp += 2) {
            const float* wk = Ws + (cp + h) * KFC * BM + l32;
            const float* xk = Xs + (cp + h) * XR;
#pragma unroll
            for (int kf = 0; kf < KFC; ++kf) {
                const float av = wk[kf * BM];
                float bv[TN];
#pragma unroll
                for (int j = 0; j < TN; ++j) bv[j] = xk[boff[j] + kf];
#pragma unroll
                for (int j = 0; j < TN; ++j) acc[j] = mfma32(av, bv[j], acc[j]);
            }
        }
    }
#pragma unroll
    for (int j = 0; j < TN; ++j) {
        const int n = n0 + wn0 + j * 32 + l32;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int co = co0 + mfma_row(r, lane);
            const float bco = a.bias ? a.bias[co < g.Co ? co : g.Co - 1] : 0.f;
            if (co < g.Co && n < nend) {
                float v = acc[j][r] + bco;
                if (a.act) v = lrelu(v);
                a.y[((int64_t)b * g.Co + co) * Nall + n] = v;
            }
        }
    }
}

// 4 floats from a dword-aligned global address (one global_load_dwordx4: the HSA target runs in
// unaligned-access mode)

// One window row of the LDS image, as float4 quads: src = global offset of window column 0,
// pos0 = its input column (-2^30 when the row lies outside the input), lim = input width.
// Interior quads are one 16-byte load; quads that straddle the zero padding load per element
// from clamped addresses.
ENCX_DEV f32x4 window_quad(const float* base, int src, int pos0, int w, int lim) {
    const int pos = pos0 + w;
    if (pos >= 0 && pos + 3 < lim) return ld4u(base + src + w);
    f32x4 v;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        const bool ok = pos + e >= 0 && pos + e < lim;
        const float t = base[ok ? src + w + e : 0];
        v[e] = ok ? t : 0.f;
    }
    return v;
}

// Forward with vectorised staging: the implicit GEMM of c2_fwd_kernel (rows co, BN flattened
// (t, f) columns, CK combos (ci, kt) x KFC taps per chunk, 4 waves x TN column tiles), but every
// window row is moved as float4 quads (row stride RLp = RL rounded up to 4, so each quad is one
// ds_write_b128) and the weights as float4 rows: ~10 vector instructions per 4 staged values
// instead of ~12 per value, which left the matrix pipe idle behind the address arithmetic.
template <int BN, int KFC, int CK>
__global__ __launch_bounds__(NT) void c2_fwdv_kernel(C2Fwd a) {
    constexpr int BM = 32, TN = BN / 128, WQ = KFC * CK * BM / 4, QU = 4;
    extern __shared__ float smem[];
    const C2Geo g = a.g;
    const int NR = a.NR, RL = a.RL, S = g.sf;
    const int RLp = (RL + 3) & ~3, NQ = RLp >> 2;
    const int VC = g.Ci * g.KT, XR = NR * RLp;
    float* Xs = smem;                      // [CK][NR][RLp]
    float* Ws = smem + CK * XR;            // [CK][KFC][BM]
    int2* rtab = (int2*)(Ws + KFC * CK * BM);  // [VC*NR]
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int h = lane >> 5, l32 = lane & 31;
    const int b = blockIdx.z, n0 = blockIdx.x * BN, co0 = blockIdx.y * BM;
    const int wn0 = wave * TN * 32;
    const int Nall = g.T2 * g.Fo, nend = min(Nall, n0 + BN);
    const int tf = n0 / g.Fo, f0 = n0 - tf * g.Fo;
    const int nr = (nend - 1) / g.Fo - tf + 1;
    int boff[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) {
        const int n = n0 + wn0 + j * 32 + l32;
        boff[j] = 0;
        if (n < nend) {
            const int tr = n / g.Fo, f = n - tr * g.Fo, rs = tr - tf;
            boff[j] = rs * RLp + (f - (rs ? 0 : f0)) * S;
        }
    }
    f32x16 acc[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[j] = (f32x16){0};
    const float* xb = a.x + (int64_t)b * g.Ci * g.T2 * g.Fi;
    for (int gr = tid; gr < VC * NR; gr += NT) {
        const int vc = gr / NR, rs = gr - vc * NR, ci = vc / g.KT, kt = vc - ci * g.KT;
        const int row = tf + rs + kt * g.dt - g.pt, pos0 = (rs ? 0 : f0) * S - g.pf;
        const bool ok = rs < nr && row >= 0 && row < g.T2;
        rtab[gr] = make_int2(ok ? (ci * g.T2 + row) * g.Fi + pos0 : 0, ok ? pos0 : -(1 << 30));
    }
    // quad items (row, q) walked by a fixed step of NT: no division per item
    const int dr = NT / NQ, dq = NT - dr * NQ, r_init = tid / NQ, q_init = tid - r_init * NQ;
    for (int c0 = 0; c0 < VC; c0 += CK) {
        __syncthreads();
        {
            // QU quads per thread in flight: interior quads are one 16-byte load from their own
            // address; the rest load nothing here and are patched per element below (the row's
            // ends, next to the zero padding)
            const int nrows = min(CK, VC - c0) * NR, rows = CK * NR;
            int r = r_init, q = q_init;
            while (r < rows) {
                int rq[QU], wq[QU];
                bool in[QU];
                int2 e[QU];
                f32x4 v[QU];
#pragma unroll
                for (int u = 0; u < QU; ++u) {
                    rq[u] = r;
                    wq[u] = 4 * q;
                    q += dq;
                    r += dr;
                    if (q >= NQ) {
                        q -= NQ;
                        ++r;
                    }
                    e[u] = rtab[c0 * NR + (rq[u] < nrows ? rq[u] : 0)];
                    const int pos = e[u].y + wq[u];
                    in[u] = rq[u] < nrows && pos >= 0 && pos + 3 < g.Fi;
                    v[u] = ld4u(xb + (in[u] ? e[u].x + wq[u] : 0));
                }
#pragma unroll
                for (int u = 0; u < QU; ++u) {
                    if (!in[u]) {
                        const int pos = e[u].y + wq[u];
#pragma unroll
                        for (int k = 0; k < 4; ++k) {
                            const bool ok = rq[u] < nrows && pos + k >= 0 && pos + k < g.Fi;
                            v[u][k] = ok ? xb[e[u].x + wq[u] + k] : 0.f;
                        }
                    }
                    if (rq[u] < rows) *(f32x4*)(Xs + rq[u] * RLp + wq[u]) = v[u];
                }
            }
        }
        {
            // Ws[cl][kf][col] = wf[(c0 + cl) * KFC + kf][co0 + col]: rows of BM floats, 8 quads each
            const float* wsrc = a.wf + (int64_t)c0 * KFC * g.Co + co0;
            const int wrows = (VC - c0) * KFC;
            constexpr int WU = (WQ + NT - 1) / NT;
            f32x4 v[WU];
#pragma unroll
            for (int u = 0; u < WU; ++u) {
                const int j = u * NT + tid, rr = j >> 3, col = (j & 7) * 4;
                const bool ok = j < WQ && rr < wrows && co0 + col + 3 < g.Co;
                v[u] = ld4u(wsrc + (ok ? (int64_t)rr * g.Co + col : 0));
                if (!ok) v[u] = (f32x4){0.f, 0.f, 0.f, 0.f};
            }
#pragma unroll
            for (int u = 0; u < WU; ++u) {
                const int j = u * NT + tid, rr = j >> 3, col = (j & 7) * 4;
                if (j < WQ && rr < wrows && co0 + col + 3 >= g.Co)  // a partial last row tile (Co % 4 != 0)
                    for (int k = 0; k < 4; ++k)
                        v[u][k] = co0 + col + k < g.Co ? wsrc[(int64_t)rr * g.Co + col + k] : 0.f;
                if (j < WQ) *(f32x4*)(Ws + rr * BM + col) = v[u];
            }
        }
        __syncthreads();
#pragma unroll 2
        for (int cp = 0; cp < CK; cp += 2) {
            const float* wk = Ws + (cp + h) * KFC * BM + l32;
            const float* xk = Xs + (cp + h) * XR;
#pragma unroll
            for (int kf = 0; kf < KFC; ++kf) {
                const float av = wk[kf * BM];
                float bv[TN];
#pragma unroll
                for (int j = 0; j < TN; ++j) bv[j] = xk[boff[j] + kf];
#pragma unroll
                for (int j = 0; j < TN; ++j) acc[j] = mfma32(av, bv[j], acc[j]);
            }
        }
    }
#pragma unroll
    for (int j = 0; j < TN; ++j) {
        const int n = n0 + wn0 + j * 32 + l32;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int co = co0 + mfma_row(r, lane);
            const float bco = a.bias ? a.bias[co < g.Co ? co : g.Co - 1] : 0.f;
            if (co < g.Co && n < nend) {
                float v = acc[j][r] + bco;
                if (a.act) v = lrelu(v);
                a.y[((int64_t)b * g.Co + co) * Nall + n] = v;
            }
        }
    }
}

// Window quad through a CLAMPED 16-byte load: the load always reads 4 in-row floats starting at
// c = clamp(pos, 0, lim - 4) (so it never leaves the row, whatever the padding), and the quad
// for columns pos..pos+3 is recovered in registers: shift by s = pos - c, zeros outside
// [0, lim). Every quad issues the same one load; only straddling quads run the (register-only)
// fix-up, so a batch of quads keeps all its loads in flight.
struct QuadSrc {
    int addr;  // element offset of the clamped load (0 for a row outside the input)
    int pos;   // first column of the quad; INT_MIN/2 -> the quad is all padding
};
ENCX_DEV QuadSrc quad_src(int2 e, int w, int lim, bool live) {
    QuadSrc q;
    const bool rowok = live && e.y > -(1 << 29);
    const int pos = e.y + w;
    const int c = min(max(pos, 0), lim - 4);
    q.addr = rowok ? e.x - e.y + c : 0;
    q.pos = rowok ? pos : -(1 << 30);
    return q;
}
ENCX_DEV f32x4 quad_fix(f32x4 v, int pos, int lim) {
    const int c = min(max(pos, 0), lim - 4), s = pos - c;
    if (s == 0) return v;  // interior quad (also: every row outside the input has pos = -2^30)
    f32x4 o;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        const int k = e + s;
        const float t = k == 0 ? v[0] : k == 1 ? v[1] : k == 2 ? v[2] : v[3];
        o[e] = (k >= 0 && k < 4 && pos + e >= 0 && pos + e < lim) ? t : 0.f;
    }
    return o;
}

// Forward, vectorised AND register-pipelined: c2_fwdv_kernel's LDS image and compute loop, with
// the next chunk's quads (window: MQ per thread, clamped loads; weights: MW) fetched into
// registers before the current chunk's MFMAs, so each chunk costs one overlapped memory round
// trip. CK (runtime, even) is sized so a chunk's window fits MQ quads per thread.
template <int BN, int KFC, int MQ, int CKM, int DBG = 0>  // DBG: microbenchmark ablations only
__global__ __launch_bounds__(NT) void c2_fwdq_kernel(C2Fwd a) {
    constexpr int BM = 32, TN = BN / 128, MW = (KFC * CKM * BM / 4 + NT - 1) / NT;
    extern __shared__ float smem[];
    const C2Geo g = a.g;
    const int CK = a.CK, NR = a.NR, RL = a.RL, S = g.sf;
    const int RLp = (RL + 3) & ~3, NQ = RLp >> 2;
    const int VC = g.Ci * g.KT, XR = NR * RLp, WQ = KFC * CK * BM / 4;
    float* Xs = smem;                      // [CK][NR][RLp]
    float* Ws = smem + CK * XR;            // [CK][KFC][BM]
    int2* rtab = (int2*)(Ws + KFC * CK * BM);  // [VC*NR]
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int h = lane >> 5, l32 = lane & 31;
    const int b = blockIdx.z, n0 = blockIdx.x * BN, co0 = blockIdx.y * BM;
    const int wn0 = wave * TN * 32;
    const int Nall = g.T2 * g.Fo, nend = min(Nall, n0 + BN);
    const int tf = n0 / g.Fo, f0 = n0 - tf * g.Fo;
    const int nr = (nend - 1) / g.Fo - tf + 1;
    int boff[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) {
        const int n = n0 + wn0 + j * 32 + l32;
        boff[j] = 0;
        if (n < nend) {
            const int tr = n / g.Fo, f = n - tr * g.Fo, rs = tr - tf;
            boff[j] = rs * RLp + (f - (rs ? 0 : f0)) * S;
        }
    }
    f32x16 acc[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[j] = (f32x16){0};
    const float* xb = a.x + (int64_t)b * g.Ci * g.T2 * g.Fi;
    for (int gr = tid; gr < VC * NR; gr += NT) {
        const int vc = gr / NR, rs = gr - vc * NR, ci = vc / g.KT, kt = vc - ci * g.KT;
        const int row = tf + rs + kt * g.dt - g.pt, pos0 = (rs ? 0 : f0) * S - g.pf;
        const bool ok = rs < nr && row >= 0 && row < g.T2;
        rtab[gr] = make_int2(ok ? (ci * g.T2 + row) * g.Fi + pos0 : 0, ok ? pos0 : -(1 << 30));
    }
    __syncthreads();
    const int rows = CK * NR;
    const int dr = NT / NQ, dq = NT - dr * NQ, r_init = tid / NQ, q_init = tid - r_init * NQ;
    f32x4 xv[MQ], wv[MW];
    int xpos[MQ], xdst[MQ];
    auto fetch = [&](int c0) {
        const int nrows = min(CK, VC - c0) * NR;
        int r = r_init, q = q_init;
#pragma unroll
        for (int u = 0; u < MQ; ++u) {
            const bool live = r < nrows;
            const QuadSrc s = quad_src(rtab[c0 * NR + (live ? r : 0)], 4 * q, g.Fi, live);
            if (DBG & 1) xv[u] = (f32x4){1.f, 1.f, 1.f, (float)s.addr};
            else xv[u] = ld4u(xb + s.addr);
            xpos[u] = s.pos;
            xdst[u] = r < rows ? r * RLp + 4 * q : -1;
            q += dq;
            r += dr;
            if (q >= NQ) {
                q -= NQ;
                ++r;
            }
        }
        const float* wsrc = a.wf + (int64_t)c0 * KFC * g.Co + co0;
        const int wrows = (VC - c0) * KFC;
#pragma unroll
        for (int u = 0; u < MW; ++u) {
            const int j = u * NT + tid, rr = j >> 3, col = (j & 7) * 4;
            const bool ok = j < WQ && rr < wrows && co0 + col + 3 < g.Co;
            wv[u] = ld4u(wsrc + (ok ? (int64_t)rr * g.Co + col : 0));
            if (!ok) wv[u] = (f32x4){0.f, 0.f, 0.f, 0.f};
        }
    };
    fetch(0);
    for (int c0 = 0; c0 < VC; c0 += CK) {
        __syncthreads();
#pragma unroll
        for (int u = 0; u < MQ; ++u)
            if (!(DBG & 2) && xdst[u] >= 0) *(f32x4*)(Xs + xdst[u]) = quad_fix(xv[u], xpos[u], g.Fi);
#pragma unroll
        for (int u = 0; u < MW; ++u) {
            const int j = u * NT + tid, rr = j >> 3, col = (j & 7) * 4;
            if (j < WQ && rr < (VC - c0) * KFC && co0 + col + 3 >= g.Co)  // partial co tile (Co % 4)
                for (int k = 0; k < 4; ++k)
                    wv[u][k] = co0 + col + k < g.Co ? a.wf[((int64_t)c0 * KFC + rr) * g.Co + co0 + col + k] : 0.f;
            if (j < WQ) *(f32x4*)(Ws + rr * BM + col) = wv[u];
        }
        __syncthreads();
        if (c0 + CK < VC) fetch(c0 + CK);
#pragma unroll 2
        for (int cp = 0; cp < CK; cp += 2) {
            const float* wk = Ws + (cp + h) * KFC * BM + l32;
            const float* xk = Xs + (cp + h) * XR;
#pragma unroll
            for (int kf = 0; kf < KFC; ++kf) {
                const float av = wk[kf * BM];
                float bv[TN];
#pragma unroll
                for (int j = 0; j < TN; ++j) bv[j] = xk[boff[j] + kf];
#pragma unroll
                for (int j = 0; j < TN; ++j) acc[j] = mfma32(av, bv[j], acc[j]);
            }
        }
    }
#pragma unroll
    for (int j = 0; j < TN; ++j) {
        const int n = n0 + wn0 + j * 32 + l32;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int co = co0 + mfma_row(r, lane);
            const float bco = a.bias ? a.bias[co < g.Co ? co : g.Co - 1] : 0.f;
            if (co < g.Co && n < nend && (!(DBG & 4) || acc[j][r] == 1234.5f)) {
                float v = acc[j][r] + bco;
                if (a.act) v = lrelu(v);
                a.y[((int64_t)b * g.Co + co) * Nall + n] = v;
            }
        }
    }
}

// Forward with column-aligned window quads. A window row holds input columns [base, base + RLp)
// of one input row, base = the row's first needed column rounded DOWN to a multiple of 4 (the
// compute reads at an offset of col - base), so every quad is aligned to input columns: a quad
// is entirely padding (left of column 0, or a row outside the input: a select, no load),
// entirely interior, or the one quad holding column Fi - 1 whose tail lanes are masked. The
// loads are issued for the next chunk before the current chunk's MFMAs (MQ quads per thread),
// and the commit is a masked select + ds_write_b128: no per-element paths, no shifts.
template <int BN, int KFC, int MQ, int CKM, int OCC = 1>  // OCC: min waves per SIMD (register cap)
__global__ __launch_bounds__(NT, OCC) void c2_fwdr_kernel(C2Fwd a) {
    constexpr int BM = 32, TN = BN / 128, MW = (KFC * CKM * BM / 4 + NT - 1) / NT;
    extern __shared__ float smem[];
    const C2Geo g = a.g;
    const int CK = a.CK, NR = a.NR, RL = a.RL, S = g.sf;
    const int RLp = (RL + 3) & ~3, NQ = RLp >> 2;
    const int VC = g.Ci * g.KT, XR = NR * RLp, WQ = KFC * CK * BM / 4;
    float* Xs = smem;                      // [CK][NR][RLp]
    float* Ws = smem + CK * XR;            // [CK][KFC][BM]
    int2* rtab = (int2*)(Ws + KFC * CK * BM);  // [VC*NR]: {offset of column `base`, base} / invalid
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int h = lane >> 5, l32 = lane & 31;
    const TileId tile = xcd_tile();
    const int b = tile.z, n0 = tile.x * BN, co0 = tile.y * BM;
    const int wn0 = wave * TN * 32;
    const int Nall = g.T2 * g.Fo, nend = min(Nall, n0 + BN);
    const int tf = n0 / g.Fo, f0 = n0 - tf * g.Fo;
    const int nr = (nend - 1) / g.Fo - tf + 1;
    const int base0 = ((f0 * S - g.pf) & ~3), baseN = ((-g.pf) & ~3);  // floor to a multiple of 4
    int boff[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) {
        const int n = n0 + wn0 + j * 32 + l32;
        boff[j] = 0;
        if (n < nend) {
            const int tr = n / g.Fo, f = n - tr * g.Fo, rs = tr - tf;
            boff[j] = rs * RLp + f * S - g.pf - (rs ? baseN : base0);
        }
    }
    f32x16 acc[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[j] = (f32x16){0};
    const int64_t xtot = (int64_t)g.B * g.Ci * g.T2 * g.Fi;
    const float* xb = a.x + (int64_t)b * g.Ci * g.T2 * g.Fi;
    const int64_t xleft = xtot - (int64_t)b * g.Ci * g.T2 * g.Fi;  // floats from xb to the tensor end
    for (int gr = tid; gr < VC * NR; gr += NT) {
        const int vc = gr / NR, rs = gr - vc * NR, ci = vc / g.KT, kt = vc - ci * g.KT;
        const int row = tf + rs + kt * g.dt - g.pt, base = rs ? baseN : base0;
        const bool ok = rs < nr && row >= 0 && row < g.T2;
        rtab[gr] = make_int2(ok ? (ci * g.T2 + row) * g.Fi + base : 0, ok ? base : -(1 << 30));
    }
    __syncthreads();
    const int rows = CK * NR;
    const int dr = NT / NQ, dq = NT - dr * NQ, r_init = tid / NQ, q_init = tid - r_init * NQ;
    f32x4 xv[MQ], wv[MW];
    int xmask[MQ], xdst[MQ];
    auto fetch = [&](int c0) {
        const int nrows = min(CK, VC - c0) * NR;
        int r = r_init, q = q_init;
#pragma unroll
        for (int u = 0; u < MQ; ++u) {
            const bool live = r < nrows;
            const int2 e = rtab[c0 * NR + (live ? r : 0)];
            const int col = e.y + 4 * q;  // first input column of the quad
            const bool any = live && col >= 0 && col < g.Fi;  // e.y = -2^30 for rows outside
            int off = any ? e.x + 4 * q : 0;
            // the last quad of the tensor may run past its end: read it one quad earlier
            // (only columns < Fi are kept, and those are then at lanes shifted... see mask)
            if (off > xleft - 4) off = (int)xleft - 4;
            xv[u] = ld4u(xb + off);
            const int sh = (any ? e.x + 4 * q : 0) - off;  // 0 except at the tensor's very end
            xmask[u] = any ? (min(g.Fi - col, 4) | (sh << 4)) : 0;  // valid lanes, shift
            xdst[u] = r < rows ? r * RLp + 4 * q : -1;
            q += dq;
            r += dr;
            if (q >= NQ) {
                q -= NQ;
                ++r;
            }
        }
        const float* wsrc = a.wf + (int64_t)c0 * KFC * g.Co + co0;
        const int wrows = (VC - c0) * KFC;
#pragma unroll
        for (int u = 0; u < MW; ++u) {
            const int j = u * NT + tid, rr = j >> 3, col = (j & 7) * 4;
            const bool ok = j < WQ && rr < wrows && co0 + col + 3 < g.Co;
            wv[u] = ld4u(wsrc + (ok ? (int64_t)rr * g.Co + col : 0));
            if (!ok) wv[u] = (f32x4){0.f, 0.f, 0.f, 0.f};
        }
    };
    fetch(0);
    for (int c0 = 0; c0 < VC; c0 += CK) {
        __syncthreads();
#pragma unroll
        for (int u = 0; u < MQ; ++u) {
            const int m = xmask[u], nv = m & 15, sh = m >> 4;
            f32x4 v = xv[u];
            if (sh) {  // the tensor's last quad, read shifted back by sh lanes (one quad in all)
                const f32x4 t = v;
#pragma unroll
                for (int k = 0; k < 4; ++k) v[k] = k + sh < 4 ? (k + sh == 1 ? t[1] : k + sh == 2 ? t[2] : t[3]) : 0.f;
            }
#pragma unroll
            for (int k = 0; k < 4; ++k) v[k] = k < nv ? v[k] : 0.f;
            if (xdst[u] >= 0) *(f32x4*)(Xs + xdst[u]) = v;
        }
#pragma unroll
        for (int u = 0; u < MW; ++u) {
            const int j = u * NT + tid, rr = j >> 3, col = (j & 7) * 4;
            if (j < WQ && rr < (VC - c0) * KFC && co0 + col + 3 >= g.Co)  // partial co tile (Co % 4)
                for (int k = 0; k < 4; ++k)
                    wv[u][k] = co0 + col + k < g.Co ? a.wf[((int64_t)c0 * KFC + rr) * g.Co + co0 + col + k] : 0.f;
            if (j < WQ) *(f32x4*)(Ws + rr * BM + col) = wv[u];
        }
        __syncthreads();
        if (c0 + CK < VC) fetch(c0 + CK);
#pragma unroll 2
        for (int cp = 0; cp < CK; cp += 2) {
            const float* wk = Ws + (cp + h) * KFC * BM + l32;
            const float* xk = Xs + (cp + h) * XR;
#pragma unroll
            for (int kf = 0; kf < KFC; ++kf) {
                const float av = wk[kf * BM];
                float bv[TN];
#pragma unroll
                for (int j = 0; j < TN; ++j) bv[j] = xk[boff[j] + kf];
#pragma unroll
                for (int j = 0; j < TN; ++j) acc[j] = mfma32(av, bv[j], acc[j]);
            }
        }
    }
#pragma unroll
    for (int j = 0; j < TN; ++j) {
        const int n = n0 + wn0 + j * 32 + l32;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int co = co0 + mfma_row(r, lane);
            const float bco = a.bias ? a.bias[co < g.Co ? co : g.Co - 1] : 0.f;
            if (co < g.Co && n < nend) {
                float v = acc[j][r] + bco;
                if (a.act) v = lrelu(v);
                a.y[((int64_t)b * g.Co + co) * Nall + n] = v;
            }
        }
    }
}

// A quad meant to start at element offset o of a tensor whose last quad starts at `last` is
// loaded from min(max(o, 0), last) (never outside the tensor); quad_abs moves it into place:
// o[e] = v[e + sh], sh = o - clamped, zero where e + sh leaves the quad. Only the tensor's first
// and last quads are ever clamped, and there |sh| < 4 matters: the rest is padding, masked by
// the caller. Two select layers on the bits of |sh| (a select chain on sh == k compiles to
// branches).
ENCX_DEV f32x4 quad_abs(f32x4 v, int o, int last) {
    const int sh = o < 0 ? o : (o > last ? o - last : 0);
    const int n = sh < 0 ? -sh : sh;
    const bool b1 = n & 1, b2 = n & 2;
    f32x4 r;
    if (sh >= 0) {  // down: r[e] = v[e + n]
        const float t0 = b1 ? v[1] : v[0], t1 = b1 ? v[2] : v[1], t2 = b1 ? v[3] : v[2], t3 = b1 ? 0.f : v[3];
        r[0] = b2 ? t2 : t0;
        r[1] = b2 ? t3 : t1;
        r[2] = b2 ? 0.f : t2;
        r[3] = b2 ? 0.f : t3;
    } else {  // up: r[e] = v[e - n]
        const float t0 = b1 ? 0.f : v[0], t1 = b1 ? v[0] : v[1], t2 = b1 ? v[1] : v[2], t3 = b1 ? v[2] : v[3];
        r[0] = b2 ? 0.f : t0;
        r[1] = b2 ? 0.f : t1;
        r[2] = b2 ? t0 : t2;
        r[3] = b2 ? t1 : t3;
    }
    return r;
}

// Forward, register-window form. The 32 x (Ci*KT*KF) weights of the layer are staged ONCE per
// workgroup into LDS ([(ci,kt)][kf][32 co], the wf layout), then each wave loops over tiles of
// 32 output-position QUADS (128 positions; rows padded to whole quads, F4 = ceil(Fo/4) quads
// per row). Lane l of a wave owns quad l: its 4 consecutive output columns f0..f0+3 are the
// MFMA columns of its 4 accumulators (jb = 0..3). The MFMA's two k slots are two input channels
// (ci = 2c + h), so per (c, kt) step each lane loads ONE contiguous input window
// x[ci][t + kt*dt - pt][S*f0 - pf .. + 3S + KF - 1] (WQ quads, straight from global memory into
// registers) which holds the operand of all KF taps x 4 columns: 4 * KF MFMAs per step, each
// with no address arithmetic, the A operand (weights) one ds_read_b32 per tap shared by the 4
// columns. The next step's window is loaded before this step's MFMAs. Window elements outside
// the input (padding, rows outside [0, T2), the tensor's ends) are zeroed by a per-lane
// element mask, only in waves that have such a lane. Bias + LeakyReLU(0.2) in the epilogue.
struct C2FwdR {
    C2Geo g;
    const float* x;
    const float* wf;  // [(ci,kt)][kf][co]
    const float* bias;
    float* y;
    int act;
    int F4;     // quads per output row
    int tiles;  // ceil(B * T2 * F4 / 32)
};
// Slot order of the persistent register-window loops (one NWV-wave workgroup per CU): item j of
// a round goes to wave j / gridDim.x of the j % gridDim.x-th workgroup in XCD order. A partial last
// round thus hands out one item per SIMD (waves w and w + 4 share one) before any SIMD takes a second
// -- the workgroup-major order piled it onto the first CUs, costing a whole extra round on layers
// with 1.5x or 2.9x as many items as wave slots -- and neighbouring items still share an XCD's L2.
ENCX_DEV int rw_first_slot(int wave) { return wave * (int)gridDim.x + xcd_linear_id(); }

template <int KF, int S, int WQ, int NWV>
__global__ __launch_bounds__(NWV * 64) void c2_fwd_rw_kernel(C2FwdR a) {
    constexpr int NE = 4 * WQ, KT = 3;  // window elements per lane; kernel rows (host-checked)
    extern __shared__ float smem[];
    const C2Geo g = a.g;
    float* Ws = smem;                          // [Ci*KT][KF][32]
    float* Bs = smem + g.Ci * KT * KF * 32;    // [32] bias
    for (int i = threadIdx.x; i < g.Ci * KT * KF * 32; i += NWV * 64) {
        const int co = i & 31, r = i >> 5;
        Ws[i] = co < g.Co ? a.wf[r * g.Co + co] : 0.f;
    }
    if (threadIdx.x < 32) Bs[threadIdx.x] = (a.bias && (int)threadIdx.x < g.Co) ? a.bias[threadIdx.x] : 0.f;
    __syncthreads();
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, h = lane >> 5, l = lane & 31;
    // element offsets fit in 32 bits (checked on the host)
    const int quads = g.B * g.T2 * a.F4;
    const int plane = g.T2 * g.Fi, xlast = g.B * g.Ci * plane - 4;
    const int CP = g.Ci >> 1;  // channel pairs
    const int cstride = 2 * plane;
    // one item's geometry: window element e of step (c, kt) is x[b][2c + h][row(kt)][col0 + e]
    struct Geo {
        int t, b, f0;
        int rb[KT];
        uint32_t msk[KT];
        bool fix;  // wave-uniform: some lane's window leaves the input
    };
    auto geo = [&](int tile) {
        Geo q;
        const int qd = min(tile * 32 + l, quads - 1);
        const int fq = qd % a.F4, bt = qd / a.F4;
        q.t = bt % g.T2;
        q.b = bt / g.T2;
        q.f0 = 4 * fq;
        const int col0 = S * q.f0 - g.pf;
        uint32_t cmask = 0;
#pragma unroll
        for (int e = 0; e < NE; ++e) cmask |= (col0 + e >= 0 && col0 + e < g.Fi) ? (1u << e) : 0u;
        bool clean = true;  // every element of every window of this lane is in the input
#pragma unroll
        for (int kt = 0; kt < KT; ++kt) {
            const int row = q.t + kt * g.dt - g.pt;
            const bool ok = row >= 0 && row < g.T2;
            q.rb[kt] = (q.b * g.Ci + h) * plane + (ok ? row : 0) * g.Fi + col0;
            q.msk[kt] = ok ? cmask : 0u;
            clean = clean && q.msk[kt] == (1u << NE) - 1;
        }
        q.fix = !__all(clean);
        return q;
    };
    auto load = [&](f32x4* w, const Geo& q, int c, int kt) {
        const int base = q.rb[kt] + c * cstride;
#pragma unroll
        for (int w4 = 0; w4 < WQ; ++w4) w[w4] = ld4u(a.x + min(max(base + 4 * w4, 0), xlast));
    };
    // three register windows, one per kt: step (c, kt) multiplies window kt with the weight
    // columns of (c, kt), read from LDS just in time, while the next step's window is in flight
    // (the prefetch is unconditional, so every wait is exact). The last step of an item loads the
    // NEXT item's first window, so it is in flight during this item's epilogue stores and the
    // next item does not start by waiting out a memory round trip behind them (vmcnt counts the
    // stores too). Measured against reading the weights a step ahead or one tap ahead: none is
    // faster (profiles/r05).
    f32x4 wb[KT][WQ];
    auto wcol = [&](int c, int kt) { return Ws + ((2 * c + h) * KT + kt) * KF * 32 + l; };
    const int stride = gridDim.x * NWV;
    int tile = rw_first_slot(wave);
    if (tile < a.tiles) load(wb[0], geo(tile), 0, 0);
    for (; tile < a.tiles; tile += stride) {
        const Geo cur = geo(tile);  // (recomputed: cheaper than holding the next item's in registers)
        const int t = cur.t, b = cur.b, f0 = cur.f0;
        f32x16 acc[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[j] = (f32x16){0};
        for (int c = 0; c < CP; ++c) {
#pragma unroll
            for (int kt = 0; kt < KT; ++kt) {
                const int nk = kt + 1 < KT ? kt + 1 : 0;
                if (kt + 1 < KT) load(wb[nk], cur, c, nk);
                else if (c + 1 < CP) load(wb[0], cur, c + 1, 0);
                else load(wb[0], geo(tile + stride < a.tiles ? tile + stride : tile), 0, 0);  // (past the last: own)
                f32x4* w = wb[kt];
                if (cur.fix) {
                    const int base = cur.rb[kt] + c * cstride;
#pragma unroll
                    for (int q = 0; q < WQ; ++q) {
                        const int o = base + 4 * q;
                        if (__any(o < 0 || o > xlast)) w[q] = quad_abs(w[q], o, xlast);  // tensor ends
#pragma unroll
                        for (int e = 0; e < 4; ++e)
                            if (!((cur.msk[kt] >> (4 * q + e)) & 1u)) w[q][e] = 0.f;
                    }
                }
                const float* wk = wcol(c, kt);
#pragma unroll
                for (int kf = 0; kf < KF; ++kf) {
                    const float av = wk[kf * 32];
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        const int r = S * j + kf;
                        acc[j] = mfma32(av, w[r >> 2][r & 3], acc[j]);
                    }
                }
            }
        }
        // ---- epilogue: rows co, columns f0 + j of this lane's quad
        if (tile * 32 + l < quads) {
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int co = mfma_row(r, lane);
                if (co >= g.Co) continue;
                const float bco = Bs[co];
                f32x4 v;
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const float u = acc[j][r] + bco;
                    v[j] = a.act ? lrelu(u) : u;
                }
                float* dst = a.y + (((int64_t)b * g.Co + co) * g.T2 + t) * g.Fo + f0;
                if (f0 + 4 <= g.Fo) {
                    *(f32x4u*)dst = v;
                } else {
#pragma unroll
                    for (int j = 0; j < 4; ++j)
                        if (f0 + j < g.Fo) dst[j] = v[j];
                }
            }
        }
    }
}

// ------------------------------------------------------------------------ backward data
struct C2Dg {
    C2Geo g;
    const float* dy;    // [B][Co][T2][Fo]
    const float* yact;  // post-activation output (LeakyReLU' mask of dy) or null
    const float* wp;    // [(co,kt)][J][ci*S + r]
    const float* xact;  // input (LeakyReLU' of the previous layer) or null
    float* dx;          // [B][Ci][T2][Fi]
    int J, U, CK, NR, RL, accumulate;
    // optional feature-matching term added to dx (FeatFn's grad of this input map, fused here
    // instead of a separate grad tensor + add): c * sign(ffx - ffr), c = fg[0] * fscale / fden[0]
    const float* ffr;   // real map [B][Ci][T2][Fi] or null
    const float* ffx;   // fake map (this layer's input)
    const float* fden;  // mean |fr| of the pair
    const float* fg;    // upstream grad of the loss (null: 1)
    float fscale;
    // optional per-element code of the pair (encx_feat_loss_code): bit 0 ffx > ffr, bit 1
    // ffx < ffr, bit 2 ffx > 0. The register-window and tiled epilogues read it (1 byte) instead
    // of ffx / ffr (8 bytes) when the mask comes from ffx or is absent
    const uint8_t* fcode;
};
ENCX_DEV float code_term(uint32_t c, float fc) { return (c & 1u) ? fc : ((c & 2u) ? -fc : 0.f); }
ENCX_DEV float code_mask(uint32_t c) { return (c & 4u) ? 1.f : 0.2f; }

ENCX_DEV float feat_coef(const C2Dg& a) {
    return a.ffr ? (a.fg ? a.fg[0] : 1.f) * a.fscale / a.fden[0] : 0.f;
}
// same value as feat_grad_kernel's dff for element o
ENCX_DEV float feat_term(const C2Dg& a, float c, int64_t o) {
    const float d = a.ffx[o] - a.ffr[o];
    return d > 0.f ? c : (d < 0.f ? -c : 0.f);
}

// dx element o (+ masks / feature term) for the epilogues below
// (the grad of the input map is completed by the feature term first; xact then turns it into
// the grad of the input's pre-activation, so the producing layer reads dy without its mask)
ENCX_DEV float dg_out(const C2Dg& a, float fc, int64_t o, float v) {
    if (a.ffr) v += feat_term(a, fc, o);
    if (a.xact) v *= lrelu_grad(a.xact[o]);
    return a.accumulate ? a.dx[o] + v : v;
}
typedef float f32x2u __attribute__((ext_vector_type(2), aligned(4)));

template <int BM, int BN, int WM, int WN, int JC = 0>
__global__ __launch_bounds__(NT) void c2_dgrad_kernel(C2Dg a) {
    constexpr int TM = BM / WM / 32, TN = BN / WN / 32;
    extern __shared__ float smem[];
    const C2Geo g = a.g;
    const int CK = a.CK, NR = a.NR, RL = a.RL, J = a.J, U = a.U, S = g.sf;
    const int VC = g.Co * g.KT, XR = NR * RL, M = g.Ci * S;
    float* Xs = smem;            // [CK][NR][RL]
    float* As = smem + CK * XR;  // [CK][J][BM]
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm0 = (wave / WN) * TM * 32, wn0 = (wave % WN) * TN * 32;
    const int h = lane >> 5, l32 = lane & 31;
    const int b = blockIdx.z, n0 = blockIdx.x * BN, m0 = blockIdx.y * BM;
    const int Nall = g.T2 * U, nend = min(Nall, n0 + BN);
    const int tf = n0 / U, u0 = n0 - tf * U;
    const int nr = (nend - 1) / U - tf + 1;
    int boff[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) {
        const int n = n0 + wn0 + j * 32 + l32;
        boff[j] = J - 1;  // in-range LDS reads for masked columns
        if (n < nend) {
            const int tr = n / U, u = n - tr * U, rs = tr - tf;
            boff[j] = rs * RL + (u - (rs ? 0 : u0)) + (J - 1);
        }
    }
    f32x16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = (f32x16){0};
    const int64_t plane = (int64_t)g.T2 * g.Fo;
    const float* dyb = a.dy + (int64_t)b * g.Co * plane;
    const float* yab = a.yact ? a.yact + (int64_t)b * g.Co * plane : nullptr;
    // staging as in c2_fwd_kernel: window-row table {offset, first position}, items walked by
    // a fixed step, weights in source order As[cl][q][m]
    int2* rtab = (int2*)(As + J * CK * BM);
    for (int gr = tid; gr < VC * NR; gr += NT) {
        const int vc = gr / NR, rs = gr - vc * NR, co = vc / g.KT, kt = vc - co * g.KT;
        const int row = tf + rs + g.pt - kt * g.dt, pos0 = (rs ? 0 : u0) - (J - 1);
        const bool ok = rs < nr && row >= 0 && row < g.T2;
        rtab[gr] = make_int2(ok ? co * (int)plane + row * g.Fo + pos0 : 0, ok ? pos0 : -(1 << 30));
    }
    const int dr = NT / RL, dw = NT - dr * RL, r_init = tid / RL, w_init = tid - r_init * RL;
    const int wcol = tid & (BM - 1);
    const float* ysrc = yab ? yab : dyb;
    for (int c0 = 0; c0 < VC; c0 += CK) {
        __syncthreads();
        {
            const int nrows = min(CK, VC - c0) * NR, items = CK * XR;
            int r = r_init, w = w_init;
            for (int i0 = 0; i0 < items; i0 += NT * DPER) {
                int rq[DPER], wq[DPER];
#pragma unroll
                for (int q = 0; q < DPER; ++q) {
                    rq[q] = r;
                    wq[q] = w;
                    w += dw;
                    r += dr;
                    if (w >= RL) {
                        w -= RL;
                        ++r;
                    }
                }
                int2 e[DPER];
#pragma unroll
                for (int q = 0; q < DPER; ++q) e[q] = rtab[c0 * NR + (rq[q] < nrows ? rq[q] : 0)];
                float v[DPER], ym[DPER];
#pragma unroll
                for (int q = 0; q < DPER; ++q) {
                    const int pos = e[q].y + wq[q];
                    const bool ok = rq[q] < nrows && pos >= 0 && pos < g.Fo;
                    const int o = ok ? e[q].x + wq[q] : 0;
                    const float t = dyb[o];
                    if (yab) ym[q] = ysrc[o];
                    v[q] = ok ? t : 0.f;
                }
#pragma unroll
                for (int q = 0; q < DPER; ++q) {
                    const int i = i0 + q * NT + tid;
                    if (i < items) Xs[i] = yab ? v[q] * lrelu_grad(ym[q]) : v[q];
                }
            }
        }
        {
            const int items = J * CK * BM, rows = (VC - c0) * J, m = m0 + wcol;
            const float* wsrc = a.wp + (int64_t)c0 * J * M + m;
            for (int i0 = 0; i0 < items; i0 += NT * DPER) {
                float v[DPER];
#pragma unroll
                for (int q = 0; q < DPER; ++q) {
                    const int rr = (i0 + q * NT + tid) / BM;
                    const bool ok = rr < rows && m < M;
                    const float t = wsrc[ok ? (int64_t)rr * M : 0];
                    v[q] = ok ? t : 0.f;
                }
#pragma unroll
                for (int q = 0; q < DPER; ++q) {
                    const int i = i0 + q * NT + tid;
                    if (i < items) As[i] = v[q];
                }
            }
        }
        __syncthreads();
        if constexpr (JC > 0) {
            for (int cp = 0; cp < CK; cp += 2) {
                const float* aq = As + (cp + h) * JC * BM + wm0 + l32;
                const float* xq = Xs + (cp + h) * XR;
#pragma unroll
                for (int q = 0; q < JC; ++q) {
                    float av[TM], bv[TN];
#pragma unroll
                    for (int i = 0; i < TM; ++i) av[i] = aq[q * BM + i * 32];
#pragma unroll
                    for (int j = 0; j < TN; ++j) bv[j] = xq[boff[j] - q];
#pragma unroll
                    for (int i = 0; i < TM; ++i)
#pragma unroll
                        for (int j = 0; j < TN; ++j) acc[i][j] = mfma32(av[i], bv[j], acc[i][j]);
                }
            }
        } else {
            for (int q = 0; q < J; ++q) {
                const float* aq = As + (h * J + q) * BM + wm0 + l32;
                const float* xq = Xs + h * XR - q;
                for (int cp = 0; cp < CK; cp += 2) {
                    float av[TM], bv[TN];
#pragma unroll
                    for (int i = 0; i < TM; ++i) av[i] = aq[cp * J * BM + i * 32];
#pragma unroll
                    for (int j = 0; j < TN; ++j) bv[j] = xq[cp * XR + boff[j]];
#pragma unroll
                    for (int i = 0; i < TM; ++i)
#pragma unroll
                        for (int j = 0; j < TN; ++j) acc[i][j] = mfma32(av[i], bv[j], acc[i][j]);
                }
            }
        }
    }
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int n = n0 + wn0 + j * 32 + l32;
            if (n >= nend) continue;
            const int tr = n / U, u = n - tr * U;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int m = m0 + wm0 + i * 32 + mfma_row(r, lane);
                if (m >= M) continue;
                const int ci = m / S, rr = m - ci * S;
                const int f = u * S + rr - g.pf;
                if (f < 0 || f >= g.Fi) continue;
                const int64_t o = (((int64_t)b * g.Ci + ci) * g.T2 + tr) * g.Fi + f;
                float v = acc[i][j][r];
                if (a.ffr) v += feat_term(a, feat_coef(a), o);
                if (a.xact) v *= lrelu_grad(a.xact[o]);
                a.dx[o] = a.accumulate ? a.dx[o] + v : v;
            }
        }
}

// Backward-data with column-aligned quads and register pipelining (c2_fwdr_kernel's staging
// applied to c2_dgrad_kernel's polyphase GEMM): rows m = (ci, r) (BM = 32 * TM), columns
// (t, u), reduction (co, kt) pairs x JC taps; the staged B image is dy * LeakyReLU'(y), both
// read as aligned quads (dy columns [base, base + RLp), base = the window start rounded down to
// a multiple of 4) and masked in the commit.
// c2_dgradr_kernel's epilogue, its terms fixed at compile time (MODE bits as rw_dg_epi): no
// branches around the loads, and the output never aliases the maps read, so the 8 row pairs of a
// (row tile, column tile) are loaded together, then combined and stored.
template <int TM, int TN, int MODE, bool PS = false>
ENCX_DEV void dgr_epi(const C2Dg& a, const f32x16 (&acc)[TM][TN], int b, int m0, int nl, int nend, int U, int M,
                      int S, int lane, float fc, bool ps = false) {
    constexpr bool C = MODE & 16, F = (MODE & 1) && !C, XM = (MODE & 2) && !C, XL = MODE & 4, A = MODE & 8,
                   LX = F || XL, CX = C && (MODE & 2);
    const C2Geo& g = a.g;
    const float* __restrict__ xs = XL ? a.xact : a.ffx;
    const float* __restrict__ rs = a.ffr;
    const uint8_t* __restrict__ cs = a.fcode;
    float* __restrict__ dx = a.dx;
    auto combine = [&](float u, float x, float r, float d, uint32_t c) {
        if (F) {
            const float e = x - r;
            u += e > 0.f ? fc : (e < 0.f ? -fc : 0.f);
        }
        if (XM) u *= lrelu_grad(x);
        if (C) u += code_term(c, fc);
        if (CX) u *= code_mask(c);
        return A ? d + u : u;
    };
    if (PS && ps) {
        // phase-major rows (c2_dgradr_kernel with TM 2 at the 3x9 stride-2 layers): tile 0 holds
        // phase 0 and tile 1 phase 1 of the 32 ci, register r of both the same ci
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int n = nl + j * 32;
            if (n >= nend) continue;
            const int tr = n / U, u = n - tr * U, f = 2 * u - g.pf;
            if (f >= 0 && f + 1 < g.Fi) {
#pragma unroll
                for (int h8 = 0; h8 < 16; h8 += 8) {
                    int64_t o[8];
                    f32x2u X[8], R[8], D[8];
                    uint32_t Cc[8][2];
#pragma unroll
                    for (int p = 0; p < 8; ++p) {
                        o[p] = (((int64_t)b * g.Ci + mfma_row(h8 + p, lane)) * g.T2 + tr) * g.Fi + f;
                        if (LX) X[p] = *(const f32x2u*)(xs + o[p]);
                        if (F) R[p] = *(const f32x2u*)(rs + o[p]);
                        if (A) D[p] = *(const f32x2u*)(dx + o[p]);
                        if (C) {
                            Cc[p][0] = cs[o[p]];
                            Cc[p][1] = cs[o[p] + 1];
                        }
                    }
#pragma unroll
                    for (int p = 0; p < 8; ++p) {
                        f32x2u s2;
#pragma unroll
                        for (int e = 0; e < 2; ++e)
                            s2[e] = combine(acc[e][j][h8 + p], LX ? X[p][e] : 0.f, F ? R[p][e] : 0.f,
                                            A ? D[p][e] : 0.f, C ? Cc[p][e] : 0u);
                        *(f32x2u*)(dx + o[p]) = s2;
                    }
                }
            } else {
#pragma unroll
                for (int e = 0; e < 2; ++e)
#pragma unroll
                    for (int r = 0; r < 16; ++r) {
                        const int fe = f + e;
                        if (fe < 0 || fe >= g.Fi) continue;
                        const int64_t q = (((int64_t)b * g.Ci + mfma_row(r, lane)) * g.T2 + tr) * g.Fi + fe;
                        dx[q] = combine(acc[e][j][r], LX ? xs[q] : 0.f, F ? rs[q] : 0.f, A ? dx[q] : 0.f,
                                        C ? (uint32_t)cs[q] : 0u);
                    }
            }
        }
        return;
    }
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int n = nl + j * 32;
            if (n >= nend) continue;
            const int tr = n / U, u = n - tr * U;
            if (S == 2) {
                // rows m, m + 1 (registers r, r + 1) are phases 0 / 1 of the same ci: the two
                // adjacent f of this column, one 8-byte access
                const int f = 2 * u - g.pf;
                if (f >= 0 && f + 1 < g.Fi && m0 + i * 32 + 32 <= M) {
                    int64_t o[8];
                    f32x2u X[8], R[8], D[8];
                    uint32_t Cc[8][2];
#pragma unroll
                    for (int p = 0; p < 8; ++p) {
                        const int m = m0 + i * 32 + mfma_row(2 * p, lane);
                        o[p] = (((int64_t)b * g.Ci + (m >> 1)) * g.T2 + tr) * g.Fi + f;
                        if (LX) X[p] = *(const f32x2u*)(xs + o[p]);
                        if (F) R[p] = *(const f32x2u*)(rs + o[p]);
                        if (A) D[p] = *(const f32x2u*)(dx + o[p]);
                        if (C) {
                            Cc[p][0] = cs[o[p]];
                            Cc[p][1] = cs[o[p] + 1];
                        }
                    }
#pragma unroll
                    for (int p = 0; p < 8; ++p) {
                        f32x2u s2;
#pragma unroll
                        for (int e = 0; e < 2; ++e)
                            s2[e] = combine(acc[i][j][2 * p + e], LX ? X[p][e] : 0.f, F ? R[p][e] : 0.f,
                                            A ? D[p][e] : 0.f, C ? Cc[p][e] : 0u);
                        *(f32x2u*)(dx + o[p]) = s2;
                    }
                } else {
#pragma unroll
                    for (int r = 0; r < 16; ++r) {
                        const int m = m0 + i * 32 + mfma_row(r, lane);
                        const int fe = f + (r & 1);
                        if (m >= M || fe < 0 || fe >= g.Fi) continue;
                        const int64_t q = (((int64_t)b * g.Ci + (m >> 1)) * g.T2 + tr) * g.Fi + fe;
                        dx[q] = combine(acc[i][j][r], LX ? xs[q] : 0.f, F ? rs[q] : 0.f, A ? dx[q] : 0.f,
                                        C ? (uint32_t)cs[q] : 0u);
                    }
                }
                continue;
            }
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int m = m0 + i * 32 + mfma_row(r, lane);
                if (m >= M) continue;
                const int ci = m / S, rr = m - ci * S;
                const int f = u * S + rr - g.pf;
                if (f < 0 || f >= g.Fi) continue;
                const int64_t q = (((int64_t)b * g.Ci + ci) * g.T2 + tr) * g.Fi + f;
                dx[q] = combine(acc[i][j][r], LX ? xs[q] : 0.f, F ? rs[q] : 0.f, A ? dx[q] : 0.f,
                                C ? (uint32_t)cs[q] : 0u);
            }
        }
}

template <int TM, int BN, int JC, int MQ, int CKM, int OCC = 1, int DB = 0, bool YM = true>
__global__ __launch_bounds__(NT, OCC) void c2_dgradr_kernel(C2Dg a) {
    constexpr int BM = 32 * TM, TN = BN / 128, MW = (JC * CKM * BM / 4 + NT - 1) / NT;
    // phase-major rows at the 3x9 stride-2 layers (both 32-row tiles in one workgroup): the fifth
    // polyphase tap, zero for every phase-1 row (kf = 2 q + 1 = 9), is skipped for tile 1
    constexpr bool PS = TM == 2 && JC == 5;
    extern __shared__ float smem[];
    const C2Geo g = a.g;
    const int CK = a.CK, NR = a.NR, RL = a.RL, U = a.U, S = g.sf;
    const int RLp = (RL + 3) & ~3, NQ = RLp >> 2;
    const int VC = g.Co * g.KT, XR = NR * RLp, M = g.Ci * S, WQ = JC * CK * BM / 4;
    // DB: two LDS images; chunk i + 1 is committed into the idle one while chunk i is
    // multiplied, so one barrier per chunk instead of two
    float* Xs = smem;                     // [CK][NR][RLp]
    float* As = smem + CK * XR;           // [CK][JC][BM]
    float* Xs2 = As + JC * CK * BM;       // DB: second image
    float* As2 = Xs2 + CK * XR;
    int2* rtab = (int2*)(DB ? As2 + JC * CK * BM : Xs2);  // [VC*NR]
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int h = lane >> 5, l32 = lane & 31;
    const TileId tile = xcd_tile();
    const int b = tile.z, n0 = tile.x * BN, m0 = tile.y * BM;
    const bool ps = PS && S == 2 && M == 64 && m0 == 0;
    const int wn0 = wave * TN * 32;
    const int Nall = g.T2 * U, nend = min(Nall, n0 + BN);
    const int tf = n0 / U, u0 = n0 - tf * U;
    const int nr = (nend - 1) / U - tf + 1;
    const int base0 = (u0 - (JC - 1)) & ~3, baseN = (-(JC - 1)) & ~3;
    int boff[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) {
        const int n = n0 + wn0 + j * 32 + l32;
        boff[j] = JC - 1;  // in-range reads for masked columns
        if (n < nend) {
            const int tr = n / U, u = n - tr * U, rs = tr - tf;
            boff[j] = rs * RLp + u - (rs ? baseN : base0);
        }
    }
    f32x16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = (f32x16){0};
    const int64_t plane = (int64_t)g.T2 * g.Fo;
    const float* dyb = a.dy + (int64_t)b * g.Co * plane;
    const float* yab = YM ? a.yact + (int64_t)b * g.Co * plane : dyb;
    const int64_t left = (int64_t)(g.B - b) * g.Co * plane;  // floats from dyb to the tensor end
    const float fc = feat_coef(a);
    for (int gr = tid; gr < VC * NR; gr += NT) {
        const int vc = gr / NR, rs = gr - vc * NR, co = vc / g.KT, kt = vc - co * g.KT;
        const int row = tf + rs + g.pt - kt * g.dt, base = rs ? baseN : base0;
        const bool ok = rs < nr && row >= 0 && row < g.T2;
        rtab[gr] = make_int2(ok ? co * (int)plane + row * g.Fo + base : 0, ok ? base : -(1 << 30));
    }
    __syncthreads();
    const int rows = CK * NR;
    const int dr = NT / NQ, dq = NT - dr * NQ, r_init = tid / NQ, q_init = tid - r_init * NQ;
    f32x4 xv[MQ], yv[MQ], wv[MW];
    int xmask[MQ], xdst[MQ];
    auto fetch = [&](int c0) {
        const int nrows = min(CK, VC - c0) * NR;
        int r = r_init, q = q_init;
#pragma unroll
        for (int u = 0; u < MQ; ++u) {
            const bool live = r < nrows;
            const int2 e = rtab[c0 * NR + (live ? r : 0)];
            const int col = e.y + 4 * q;
            const bool any = live && col >= 0 && col < g.Fo;
            int off = any ? e.x + 4 * q : 0;
            if (off > left - 4) off = (int)left - 4;
            xv[u] = ld4u(dyb + off);
            if (YM) yv[u] = ld4u(yab + off);
            const int sh = (any ? e.x + 4 * q : 0) - off;
            xmask[u] = any ? (min(g.Fo - col, 4) | (sh << 4)) : 0;
            xdst[u] = r < rows ? r * RLp + 4 * q : -1;
            q += dq;
            r += dr;
            if (q >= NQ) {
                q -= NQ;
                ++r;
            }
        }
        const float* wsrc = a.wp + (int64_t)c0 * JC * M + m0;
        const int wrows = (VC - c0) * JC;
#pragma unroll
        for (int u = 0; u < MW; ++u) {
            const int j = u * NT + tid, rr = j / (BM / 4), col = (j % (BM / 4)) * 4;
            const bool ok = j < WQ && rr < wrows && m0 + col + 3 < M;
            wv[u] = ld4u(wsrc + (ok ? (int64_t)rr * M + col : 0));
            if (!ok) wv[u] = (f32x4){0.f, 0.f, 0.f, 0.f};
        }
    };
    auto commit = [&](int c0, float* X, float* A) {
#pragma unroll
        for (int u = 0; u < MQ; ++u) {
            const int m = xmask[u], nv = m & 15, sh = m >> 4;
            f32x4 v = xv[u], y = yv[u];
            if (sh) {
                const f32x4 t = v, ty = y;
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    v[k] = k + sh < 4 ? (k + sh == 1 ? t[1] : k + sh == 2 ? t[2] : t[3]) : 0.f;
                    y[k] = k + sh < 4 ? (k + sh == 1 ? ty[1] : k + sh == 2 ? ty[2] : ty[3]) : 0.f;
                }
            }
#pragma unroll
            for (int k = 0; k < 4; ++k) v[k] = k < nv ? (YM ? v[k] * lrelu_grad(y[k]) : v[k]) : 0.f;
            if (xdst[u] >= 0) *(f32x4*)(X + xdst[u]) = v;
        }
#pragma unroll
        for (int u = 0; u < MW; ++u) {
            const int j = u * NT + tid, rr = j / (BM / 4), col = (j % (BM / 4)) * 4;
            if (j < WQ && rr < (VC - c0) * JC && m0 + col + 3 >= M)
                for (int k = 0; k < 4; ++k)
                    wv[u][k] = m0 + col + k < M ? a.wp[((int64_t)c0 * JC + rr) * M + m0 + col + k] : 0.f;
            if (j < WQ) {
                if (PS && ps) {  // rows col .. col + 3 = (ci, 0), (ci, 1), (ci + 1, 0), (ci + 1, 1)
                    const int ci = col >> 1;
                    *(f32x2*)(A + rr * BM + ci) = (f32x2){wv[u][0], wv[u][2]};
                    *(f32x2*)(A + rr * BM + 32 + ci) = (f32x2){wv[u][1], wv[u][3]};
                } else {
                    *(f32x4*)(A + rr * BM + col) = wv[u];
                }
            }
        }
    };
    auto compute = [&](const float* X, const float* A) {
        if (DB & 2) {  // operands of the next k-pair group read before this group's MFMAs
            float ca[TM], cb[TN], na[TM], nb[TN];
            auto rd = [&](int cp, int q, float* va, float* vb) {
                const float* aq = A + (cp + h) * JC * BM + l32;
                const float* xq = X + (cp + h) * XR;
#pragma unroll
                for (int i = 0; i < TM; ++i) va[i] = aq[q * BM + i * 32];
#pragma unroll
                for (int j = 0; j < TN; ++j) vb[j] = xq[boff[j] - q];
            };
            rd(0, 0, ca, cb);
            for (int cp = 0; cp < CK; cp += 2) {
#pragma unroll
                for (int q = 0; q < JC; ++q) {
                    if (q + 1 < JC) rd(cp, q + 1, na, nb);
                    else if (cp + 2 < CK) rd(cp + 2, 0, na, nb);
#pragma unroll
                    for (int i = 0; i < TM; ++i)
                        if (!(PS && ps && i == 1 && q == JC - 1))
#pragma unroll
                            for (int j = 0; j < TN; ++j) acc[i][j] = mfma32(ca[i], cb[j], acc[i][j]);
#pragma unroll
                    for (int i = 0; i < TM; ++i) ca[i] = na[i];
#pragma unroll
                    for (int j = 0; j < TN; ++j) cb[j] = nb[j];
                }
            }
            return;
        }
#pragma unroll 2
        for (int cp = 0; cp < CK; cp += 2) {
            const float* aq = A + (cp + h) * JC * BM + l32;
            const float* xq = X + (cp + h) * XR;
#pragma unroll
            for (int q = 0; q < JC; ++q) {
                float av[TM], bv[TN];
#pragma unroll
                for (int i = 0; i < TM; ++i) av[i] = aq[q * BM + i * 32];
#pragma unroll
                for (int j = 0; j < TN; ++j) bv[j] = xq[boff[j] - q];
#pragma unroll
                for (int i = 0; i < TM; ++i)
                    if (!(PS && ps && i == 1 && q == JC - 1))
#pragma unroll
                        for (int j = 0; j < TN; ++j) acc[i][j] = mfma32(av[i], bv[j], acc[i][j]);
            }
        }
    };
    fetch(0);
    if (DB) {
        commit(0, Xs, As);
        if (CK < VC) fetch(CK);
        __syncthreads();
        int i = 0;
        for (int c0 = 0; c0 < VC; c0 += CK, ++i) {
            float* Xc = (i & 1) ? Xs2 : Xs;
            float* Ac = (i & 1) ? As2 : As;
            if (c0 + CK < VC) {  // the idle image was last read before the previous barrier
                commit(c0 + CK, (i & 1) ? Xs : Xs2, (i & 1) ? As : As2);
                if (c0 + 2 * CK < VC) fetch(c0 + 2 * CK);
            }
            compute(Xc, Ac);
            __syncthreads();
        }
    } else {
        for (int c0 = 0; c0 < VC; c0 += CK) {
            __syncthreads();
            commit(c0, Xs, As);
            __syncthreads();
            if (c0 + CK < VC) fetch(c0 + CK);
            compute(Xs, As);
        }
    }
    // epilogue (dgr_epi): the feature-matching term, LeakyReLU'(x), accumulate
    const bool ldx = a.xact && !(a.ffr && a.ffx == a.xact);
    const int mode = (a.ffr ? 1 : 0) | (a.xact ? 2 : 0) | (ldx ? 4 : 0) | (a.accumulate ? 8 : 0) |
                     (a.fcode && a.ffr && !ldx ? 16 : 0);
    switch (mode) {
#define ENCX_EPI(m) \
    case m: dgr_epi<TM, TN, m, PS>(a, acc, b, m0, n0 + wn0 + l32, nend, U, M, S, lane, fc, ps); break;
        ENCX_EPI(0) ENCX_EPI(1) ENCX_EPI(3) ENCX_EPI(6) ENCX_EPI(7)
        ENCX_EPI(8) ENCX_EPI(9) ENCX_EPI(11) ENCX_EPI(14) ENCX_EPI(15)
        ENCX_EPI(17) ENCX_EPI(19) ENCX_EPI(25) ENCX_EPI(27)
#undef ENCX_EPI
        default: break;
    }
}


// Backward-data, register-window form (c2_fwd_rw_kernel's scheme on c2_dgradr_kernel's
// polyphase GEMM): rows m = (ci, r) (M = Ci*S: TM tiles of 32), columns = output-column QUADS
// of the polyphase grid (t, u), rows padded to whole quads (U4 per row); lane l of a wave owns
// quad l, its 4 accumulators per row tile are the columns u0..u0+3. The k slots are two output
// channels (co = 2c + h): per (c, kt) step each lane loads ONE window of the output grad
// dy[co][t + pt - kt*dt][u0 - J + 1 .. u0 + 3] (+ the same window of y for LeakyReLU'(y)),
// which holds the operand of all J taps x 4 columns: J * 4 * TM MFMAs per step, the polyphase
// weights (staged once per workgroup in LDS, wp layout) one ds_read_b32 per tap and row tile.
// Epilogue: the feature-matching term, LeakyReLU'(x), accumulate, as c2_dgradr_kernel; the
// 2S consecutive input columns a lane holds per ci are written as quads.
struct C2DgR {
    C2Dg d;
    int U4;     // quads per polyphase row
    int tiles;  // column tiles (32 quads each): ceil(B * T2 * U4 / 32)
};
// c2_dgrad_rw_kernel's epilogue for one item, the combination of its terms fixed at compile time
// (MODE bits: 1 feature term, 2 LeakyReLU'(x), 4 x read from xact (else from ffx), 8 accumulate),
// so the per-quad code has no branches around its loads: with them, every load sat in its own
// basic block behind a wait, one memory round trip per quad. The output never aliases the maps
// read here, so the loads of EP rows are issued together, then combined and stored.
template <int S, int TM, int MODE>
ENCX_DEV void rw_dg_epi(const C2Dg& a, const f32x16 (&acc)[TM][4], int rt, int lane, int b, int t, int u0, float fc) {
    // MODE 16: the feature term (and LeakyReLU'(ffx)) from the 1-byte pair code
    constexpr bool C = MODE & 16, F = (MODE & 1) && !C, XM = (MODE & 2) && !C, XL = MODE & 4, A = MODE & 8,
                   LX = F || XL, CX = C && (MODE & 2);
    constexpr int EP = 2;  // S == 2: ci rows (2 phases x 2 quads each) per batch; S == 1: 2 EP rows
    const C2Geo& g = a.g;
    const float* __restrict__ xs = XL ? a.xact : a.ffx;
    const float* __restrict__ rs = a.ffr;
    const uint8_t* __restrict__ cs = a.fcode;
    float* __restrict__ dx = a.dx;
    auto combine = [&](float u, float x, float r, float d, uint32_t c) {
        if (F) {
            const float e = x - r;
            u += e > 0.f ? fc : (e < 0.f ? -fc : 0.f);
        }
        if (XM) u *= lrelu_grad(x);
        if (C) u += code_term(c, fc);
        if (CX) u *= code_mask(c);
        return A ? d + u : u;
    };
    if (S == 2) {
        // TM == 2 (phase-split rows, c2_dgrad_rw_kernel): tile 0 holds phase 0 and tile 1 phase 1
        // of the same 32 ci, register r of both the same ci; otherwise registers r, r + 1 of a tile
        // are phases 0 / 1 of one ci. Either way the 4 columns give 8 consecutive f.
        constexpr bool PS = TM == 2;
        const int f = 2 * u0 - g.pf;
        const bool inb = f >= 0 && f + 8 <= g.Fi;
        if constexpr (PS && C && !LX && !F && !A) {
            // the premasked feature-code epilogue (the map's only input is its 1-byte code): the
            // codes of four row pairs as unaligned dwords (8 bytes per row, two loads) issued
            // together, then combined and stored; one round trip per four pairs instead of one
            // per pair of 16 byte loads
            if (inb) {
                typedef uint32_t u32u __attribute__((aligned(1)));
#pragma unroll
                for (int hb = 0; hb < 16; hb += 4 * EP) {
                    uint32_t cw[4][EP][2];
                    int64_t oo[4][EP];
#pragma unroll
                    for (int j = 0; j < 4; ++j)
#pragma unroll
                        for (int p = 0; p < EP; ++p) {
                            const int ci = mfma_row(hb + j * EP + p, lane);
                            oo[j][p] = (((int64_t)b * g.Ci + ci) * g.T2 + t) * g.Fi + f;
                            cw[j][p][0] = *(const u32u*)(cs + oo[j][p]);
                            cw[j][p][1] = *(const u32u*)(cs + oo[j][p] + 4);
                        }
#pragma unroll
                    for (int j = 0; j < 4; ++j)
#pragma unroll
                        for (int p = 0; p < EP; ++p)
#pragma unroll
                            for (int h = 0; h < 2; ++h) {
                                f32x4 s4;
#pragma unroll
                                for (int e = 0; e < 4; ++e) {
                                    const int e8 = 4 * h + e, r = hb + j * EP + p;
                                    s4[e] = combine(acc[e8 & 1][e8 >> 1][r], 0.f, 0.f, 0.f, (cw[j][p][h] >> (8 * e)) & 255u);
                                }
                                *(f32x4u*)(dx + oo[j][p] + 4 * h) = s4;
                            }
                }
                return;
            }
        }
#pragma unroll
        for (int i = 0; i < (PS ? 1 : TM); ++i)
#pragma unroll
            for (int r0 = 0; r0 < 16; r0 += PS ? EP : 2 * EP) {
                int64_t o[EP];
#pragma unroll
                for (int p = 0; p < EP; ++p) {
                    const int ci = PS ? mfma_row(r0 + p, lane) : ((rt * TM + i) * 32 + mfma_row(r0 + 2 * p, lane)) >> 1;
                    o[p] = (((int64_t)b * g.Ci + ci) * g.T2 + t) * g.Fi + f;
                }
                auto val = [&](int p, int e8) {
                    return PS ? acc[e8 & 1][e8 >> 1][r0 + p] : acc[i][e8 >> 1][r0 + 2 * p + (e8 & 1)];
                };
                if (inb) {
                    f32x4 X[EP][2], R[EP][2], D[EP][2];
                    uint32_t Cc[EP][8];
#pragma unroll
                    for (int p = 0; p < EP; ++p) {
#pragma unroll
                        for (int h = 0; h < 2; ++h) {
                            if (LX) X[p][h] = ld4u(xs + o[p] + 4 * h);
                            if (F) R[p][h] = ld4u(rs + o[p] + 4 * h);
                            if (A) D[p][h] = ld4u(dx + o[p] + 4 * h);
                        }
                        if (C) {
#pragma unroll
                            for (int e = 0; e < 8; ++e) Cc[p][e] = cs[o[p] + e];
                        }
                    }
#pragma unroll
                    for (int p = 0; p < EP; ++p)
#pragma unroll
                        for (int h = 0; h < 2; ++h) {
                            f32x4 s4;
#pragma unroll
                            for (int e = 0; e < 4; ++e)
                                s4[e] = combine(val(p, 4 * h + e), LX ? X[p][h][e] : 0.f, F ? R[p][h][e] : 0.f,
                                                A ? D[p][h][e] : 0.f, C ? Cc[p][4 * h + e] : 0u);
                            *(f32x4u*)(dx + o[p] + 4 * h) = s4;
                        }
                } else {
#pragma unroll
                    for (int p = 0; p < EP; ++p)
#pragma unroll
                        for (int e = 0; e < 8; ++e)
                            if (f + e >= 0 && f + e < g.Fi) {
                                const int64_t q = o[p] + e;
                                dx[q] = combine(val(p, e), LX ? xs[q] : 0.f, F ? rs[q] : 0.f, A ? dx[q] : 0.f,
                                                C ? (uint32_t)cs[q] : 0u);
                            }
                }
            }
    } else {
        const int f = u0 - g.pf;
        const bool inb = f >= 0 && f + 4 <= g.Fi;
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int r0 = 0; r0 < 16; r0 += 2 * EP) {
                int64_t o[2 * EP];
#pragma unroll
                for (int p = 0; p < 2 * EP; ++p) {
                    const int ci = (rt * TM + i) * 32 + mfma_row(r0 + p, lane);
                    o[p] = (((int64_t)b * g.Ci + ci) * g.T2 + t) * g.Fi + f;
                }
                if (inb) {
                    f32x4 X[2 * EP], R[2 * EP], D[2 * EP];
                    uint32_t Cc[2 * EP][4];
#pragma unroll
                    for (int p = 0; p < 2 * EP; ++p) {
                        if (LX) X[p] = ld4u(xs + o[p]);
                        if (F) R[p] = ld4u(rs + o[p]);
                        if (A) D[p] = ld4u(dx + o[p]);
                        if (C) {
#pragma unroll
                            for (int e = 0; e < 4; ++e) Cc[p][e] = cs[o[p] + e];
                        }
                    }
#pragma unroll
                    for (int p = 0; p < 2 * EP; ++p) {
                        f32x4 s4;
#pragma unroll
                        for (int e = 0; e < 4; ++e)
                            s4[e] = combine(acc[i][e][r0 + p], LX ? X[p][e] : 0.f, F ? R[p][e] : 0.f, A ? D[p][e] : 0.f,
                                            C ? Cc[p][e] : 0u);
                        *(f32x4u*)(dx + o[p]) = s4;
                    }
                } else {
#pragma unroll
                    for (int p = 0; p < 2 * EP; ++p)
#pragma unroll
                        for (int e = 0; e < 4; ++e)
                            if (f + e >= 0 && f + e < g.Fi) {
                                const int64_t q = o[p] + e;
                                dx[q] = combine(acc[i][e][r0 + p], LX ? xs[q] : 0.f, F ? rs[q] : 0.f, A ? dx[q] : 0.f,
                                                C ? (uint32_t)cs[q] : 0u);
                            }
                }
            }
    }
}

template <int J, int S, int RT, int WQ, bool YM, int NWV, int TM>
__global__ __launch_bounds__(NWV * 64) void c2_dgrad_rw_kernel(C2DgR R) {
    // RT row tiles of 32 (M = Ci*S = 32 RT); a work item is (column tile, TM row tiles); the
    // weight columns are read from LDS just in time (measured against reading them a step ahead,
    // one tap ahead, and one row tile per item: none is faster, profiles/r05)
    constexpr int NE = 4 * WQ, KT = 3, M = 32 * RT, RG = RT / TM;
    const C2Dg& a = R.d;
    extern __shared__ float smem[];
    const C2Geo g = a.g;
    // phase-split rows (the 3x9 stride-2 layers with both row tiles per item): tile 0 = phase 0,
    // tile 1 = phase 1 of the 32 ci, so the fifth polyphase tap, zero for every phase-1 row
    // (kf = 2 q + 1 = 9 >= KF), is skipped for tile 1: 10 % fewer MFMAs
    constexpr bool PS = S == 2 && J == 5 && RT == 2 && TM == 2;
    float* As = smem;  // [(co,kt)][J][M]: the wp layout (M == Ci*S, host-checked), rows phase-major if PS
    for (int i = threadIdx.x; i < g.Co * KT * J * M; i += NWV * 64) {
        if (PS) {
            const int mn = i % M;
            As[i] = a.wp[i - mn + (mn & 31) * S + (mn >> 5)];
        } else {
            As[i] = a.wp[i];
        }
    }
    __syncthreads();
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, h = lane >> 5, l = lane & 31;
    // element offsets fit in 32 bits (checked on the host)
    const int quads = g.B * g.T2 * R.U4;
    const int plane = g.T2 * g.Fo, ylast = g.B * g.Co * plane - 4;
    const int CP = g.Co >> 1, cstride = 2 * plane;
    const float fc = feat_coef(a);
    // one item's geometry: window element e of step (c, kt) is dy[b][2c + h][row(kt)][e0 + e]
    struct Geo {
        int rt, tile, t, b, u0;
        int rb[KT];
        uint32_t msk[KT];
        bool fix;  // wave-uniform: some lane's window leaves the map
    };
    auto geo = [&](int item) {
        Geo q;
        q.rt = item % RG;
        q.tile = item / RG;  // rows rt*TM*32 .. + TM*32
        const int qd = min(q.tile * 32 + l, quads - 1);
        const int uq = qd % R.U4, bt = qd / R.U4;
        q.t = bt % g.T2;
        q.b = bt / g.T2;
        q.u0 = 4 * uq;
        const int e0 = q.u0 - (J - 1);  // dy column of window element 0
        uint32_t cmask = 0;
#pragma unroll
        for (int e = 0; e < NE; ++e) cmask |= (e0 + e >= 0 && e0 + e < g.Fo) ? (1u << e) : 0u;
        bool clean = true;
#pragma unroll
        for (int kt = 0; kt < KT; ++kt) {
            const int row = q.t + g.pt - kt * g.dt;
            const bool ok = row >= 0 && row < g.T2;
            q.rb[kt] = (q.b * g.Co + h) * plane + (ok ? row : 0) * g.Fo + e0;
            q.msk[kt] = ok ? cmask : 0u;
            clean = clean && q.msk[kt] == (1u << NE) - 1;
        }
        q.fix = !__all(clean);
        return q;
    };
    // two register buffers of windows, alternating over the (c, kt) steps: step s + 1 is in
    // flight while step s multiplies. The loop body is 2 channel pairs x 3 kt = 6 steps, so
    // every buffer / kt index is a compile-time constant (Co % 4 == 0). The last step of an item
    // loads the NEXT item's first window, so it is in flight during this item's epilogue and the
    // next item does not start by waiting out a round trip behind the epilogue's stores.
    f32x4 wb[2][WQ], yb[2][WQ];
    auto load = [&](int k, const Geo& q, int c, int kt) {
        const int base = q.rb[kt] + c * cstride;
#pragma unroll
        for (int w4 = 0; w4 < WQ; ++w4) {
            const int o = min(max(base + 4 * w4, 0), ylast);
            wb[k][w4] = ld4u(a.dy + o);
            if (YM) yb[k][w4] = ld4u(a.yact + o);
        }
    };
    const int stride = gridDim.x * NWV, nitems = R.tiles * RG;
    int item = rw_first_slot(wave);
    if (item < nitems) load(0, geo(item), 0, 0);
    for (; item < nitems; item += stride) {
        const Geo cur = geo(item);  // (recomputed: cheaper than holding the next item's in registers)
        const int rt = cur.rt, tile = cur.tile, t = cur.t, b = cur.b, u0 = cur.u0;
        auto acol = [&](int c, int kt) { return As + ((2 * c + h) * KT + kt) * J * M + rt * TM * 32 + l; };
        f32x16 acc[TM][4];
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[i][j] = (f32x16){0};
        for (int c0 = 0; c0 < CP; c0 += 2) {
#pragma unroll
            for (int u = 0; u < 2 * KT; ++u) {
                const int kt = u % KT, c = c0 + u / KT, k = u & 1;
                // the next step: within the item, or the next item's first (past the last item
                // its own first again, never used)
                const int nu = u + 1 < 2 * KT ? u + 1 : 0;
                if (u + 1 < 2 * KT || c0 + 2 < CP) load(k ^ 1, cur, u + 1 < 2 * KT ? c0 + nu / KT : c0 + 2, nu % KT);
                else load(k ^ 1, geo(item + stride < nitems ? item + stride : item), 0, 0);
                // keep the next step's loads HERE, a whole step ahead of their use: without the
                // barrier the scheduler sinks them to the end of the step (one register buffer
                // instead of two) and every step waits out the load latency (measured: the
                // round-3 kernel without it is slower, profiles/r05)
                __builtin_amdgcn_sched_barrier(0);
                f32x4* w = wb[k];
                if (YM) {
#pragma unroll
                    for (int q = 0; q < WQ; ++q)
#pragma unroll
                        for (int e = 0; e < 4; ++e) w[q][e] *= lrelu_grad(yb[k][q][e]);
                }
                if (cur.fix) {
                    const int base = cur.rb[kt] + c * cstride;
#pragma unroll
                    for (int q = 0; q < WQ; ++q) {
                        const int o = base + 4 * q;
                        if (__any(o < 0 || o > ylast)) w[q] = quad_abs(w[q], o, ylast);  // tensor ends
#pragma unroll
                        for (int e = 0; e < 4; ++e)
                            if (!((cur.msk[kt] >> (4 * q + e)) & 1u)) w[q][e] = 0.f;
                    }
                }
                const float* ak = acol(c, kt);
#pragma unroll
                for (int q = 0; q < J; ++q) {
                    float av[TM];
#pragma unroll
                    for (int i = 0; i < TM; ++i) av[i] = (PS && i == 1 && q == J - 1) ? 0.f : ak[q * M + i * 32];
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        const int r = j - q + J - 1;  // window element of column u0 + j, tap q
#pragma unroll
                        for (int i = 0; i < TM; ++i)
                            if (!(PS && i == 1 && q == J - 1)) acc[i][j] = mfma32(av[i], w[r >> 2][r & 3], acc[i][j]);
                    }
                }
            }
        }
        // ---- epilogue (rw_dg_epi): the feature-matching term, LeakyReLU'(x), accumulate
        const bool live = tile * 32 + l < quads;
        const bool ldx = a.xact && !(a.ffr && a.ffx == a.xact);  // x from xact (else from ffx)
        const int mode = (a.ffr ? 1 : 0) | (a.xact ? 2 : 0) | (ldx ? 4 : 0) | (a.accumulate ? 8 : 0) |
                         (a.fcode && a.ffr && !ldx ? 16 : 0);
        switch (mode) {
#define ENCX_EPI(m) \
    case m: if (live) rw_dg_epi<S, TM, m>(a, acc, rt, lane, b, t, u0, fc); break;
            ENCX_EPI(0) ENCX_EPI(1) ENCX_EPI(3) ENCX_EPI(6) ENCX_EPI(7)
            ENCX_EPI(8) ENCX_EPI(9) ENCX_EPI(11) ENCX_EPI(14) ENCX_EPI(15)
            ENCX_EPI(17) ENCX_EPI(19) ENCX_EPI(25) ENCX_EPI(27)
#undef ENCX_EPI
            default: break;  // (xact without its own load needs ffr: modes 2, 10 do not occur)
        }
    }
}

// Narrow backward-data (M = Ci <= 4 rows, stride 1 along f: the first layer's grad into the
// spectrogram). A 32-row MFMA tile would carry 2 useful rows, so this runs on the vector ALU:
// a workgroup owns 16 t rows x 64 f columns of one batch item; the masked output grad for
// NC_CO channels is staged in LDS with its (KT-1)*dt row and KF-1 column halo; a thread keeps
// CI x 4 accumulators for 4 adjacent f and slides a 4+KF-1 window over its LDS row per tap;
// the weights are wave-uniform (scalar loads).
#ifndef ENCX_DN_QP
#define ENCX_DN_QP 4  // staging quads in flight per thread and tensor (compile-time A/B knob)
#endif
constexpr int DN_ROWS = 16, DN_COLS = 64, DN_FPT = 4, DN_CC = 8, DN_MAXHALO = 4;
// DT: the time dilation at compile time (the staging's index splits then divide by constants:
// with a runtime row count they were integer divisions, and the staging's VALU work rivalled the
// FMAs'); interior quads (the whole quad inside the row) skip the edge shift / mask.
template <int CI, int KT, int KF, bool YM = true, bool VQ = true, int DT = 1>
__global__ __launch_bounds__(NT) void c2_dgrad_narrow(C2Dg a) {
    constexpr int RC = (DN_COLS + KF - 1 + 3) & ~3;  // LDS row length (float4 aligned)
    constexpr int WIN4 = (DN_FPT + KF - 1 + 3) / 4;
    __shared__ float Xs[DN_CC * (DN_ROWS + DN_MAXHALO) * RC];
    const C2Geo g = a.g;
    const int tid = threadIdx.x, tx = tid & 15, ty = tid >> 4;
    const int f0 = blockIdx.x * DN_COLS, t0 = blockIdx.y * DN_ROWS, b = blockIdx.z;
    constexpr int halo = (KT - 1) * DT, NRW = DN_ROWS + halo;
    const int tbase = t0 + g.pt - halo, fbase = f0 + g.pf - (KF - 1);
    const int64_t plane = (int64_t)g.T2 * g.Fo;
    const float* dyb = a.dy + (int64_t)b * g.Co * plane;
    const float* yab = YM ? a.yact + (int64_t)b * g.Co * plane : dyb;
    const int items = DN_CC * NRW * RC;
    // accumulators as (ci, ci + 1) pairs: one packed FMA (v_pk_fma_f32, the weight pair from
    // SGPRs) per two channels
    static_assert(CI % 2 == 0, "channel pairs");
    f32x2 acc[CI / 2][DN_FPT];
#pragma unroll
    for (int c = 0; c < CI / 2; ++c)
#pragma unroll
        for (int e = 0; e < DN_FPT; ++e) acc[c][e] = (f32x2){0.f, 0.f};
    // VQ: the tile is staged as quads along f (ld4u; lanes outside [0, Fo) or outside the
    // tensor masked), one index split per 4 elements instead of per element
    constexpr int RQ = RC / 4, QP = ENCX_DN_QP;
    constexpr int nq = DN_CC * NRW * RQ;
    const int64_t left = (int64_t)(g.B - b) * g.Co * plane;  // floats from dyb to the tensor end
    for (int c0 = 0; c0 < g.Co; c0 += DN_CC) {
        __syncthreads();
        if (VQ) {
            for (int i0 = 0; i0 < nq; i0 += NT * QP) {
                f32x4 v[QP], ym[QP];
                int mk[QP];
#pragma unroll
                for (int q = 0; q < QP; ++q) {
                    const int i = i0 + q * NT + tid;
                    const int cl = i / (NRW * RQ), rem = i - cl * (NRW * RQ), r = rem / RQ, cq = rem - r * RQ;
                    const int tr = tbase + r, fc = fbase + 4 * cq;
                    const bool ok = i < nq && c0 + cl < g.Co && tr >= 0 && tr < g.T2 && fc + 4 > 0 && fc < g.Fo;
                    const int64_t o = ok ? (int64_t)(c0 + cl) * plane + (int64_t)tr * g.Fo + fc : 0;
                    int64_t oc = o < 0 ? 0 : o;
                    if (oc > left - 4) oc = left - 4;
                    v[q] = ld4u(dyb + oc);
                    if (YM) ym[q] = ld4u(yab + oc);
                    // lanes [lo, hi) hold columns inside [0, Fo); sh = the shift of a clamped load
                    const int lo = fc < 0 ? -fc : 0, hi = min(g.Fo - fc, 4), sh = (int)(o - oc);
                    // 1: the plain quad (inside the row and the tensor), no shift or mask
                    mk[q] = ok ? ((lo == 0 && hi == 4 && sh == 0) ? 1 : (lo | (hi << 4) | ((sh + 4) << 8))) : 0;
                }
#pragma unroll
                for (int q = 0; q < QP; ++q) {
                    const int i = i0 + q * NT + tid;
                    if (i >= nq) continue;
                    const int m = mk[q];
                    if (m == 1) {
                        f32x4 u = v[q];
                        if (YM)
#pragma unroll
                            for (int k = 0; k < 4; ++k) u[k] *= lrelu_grad(ym[q][k]);
                        *(f32x4*)(Xs + i * 4) = u;
                        continue;
                    }
                    const int lo = m & 15, hi = (m >> 4) & 15, sh = (m >> 8) - 4;
                    f32x4 t = v[q], ty = ym[q], u;
#pragma unroll
                    for (int k = 0; k < 4; ++k) {
                        const int src = k + sh;  // lane of the loaded quad holding column fc + k
                        float dv = 0.f, yv = 0.f;
#pragma unroll
                        for (int j = 0; j < 4; ++j)
                            if (src == j) {
                                dv = t[j];
                                if (YM) yv = ty[j];
                            }
                        const bool in = m && k >= lo && k < hi && src >= 0 && src < 4;
                        u[k] = in ? (YM ? dv * lrelu_grad(yv) : dv) : 0.f;
                    }
                    *(f32x4*)(Xs + i * 4) = u;
                }
            }
        } else
        for (int i0 = 0; i0 < items; i0 += NT * DPER) {
            float v[DPER], ym[DPER];
#pragma unroll
            for (int q = 0; q < DPER; ++q) {
                const int i = i0 + q * NT + tid;
                const int cl = i / (NRW * RC), rem = i - cl * (NRW * RC), r = rem / RC, c = rem - r * RC;
                const int tr = tbase + r, fc = fbase + c;
                const bool ok = i < items && tr >= 0 && tr < g.T2 && fc >= 0 && fc < g.Fo;
                const int64_t o = ok ? (int64_t)(c0 + cl) * plane + (int64_t)tr * g.Fo + fc : 0;
                const float t = dyb[o];
                if (YM) ym[q] = yab[o];
                v[q] = ok ? t : 0.f;
            }
#pragma unroll
            for (int q = 0; q < DPER; ++q) {
                const int i = i0 + q * NT + tid;
                if (i < items) Xs[i] = YM ? v[q] * lrelu_grad(ym[q]) : v[q];
            }
        }
        __syncthreads();
        for (int cl = 0; cl < DN_CC; ++cl) {
            const int co = c0 + cl;
#pragma unroll
            for (int kt = 0; kt < KT; ++kt) {
                const float* row = Xs + (cl * NRW + ty + (KT - 1 - kt) * DT) * RC + 4 * tx;
                float win[WIN4 * 4];
#pragma unroll
                for (int j = 0; j < WIN4; ++j) {
                    const f32x4 t = *(const f32x4*)(row + 4 * j);
                    win[4 * j] = t[0];
                    win[4 * j + 1] = t[1];
                    win[4 * j + 2] = t[2];
                    win[4 * j + 3] = t[3];
                }
                const float* wr = a.wp + (int64_t)(co * KT + kt) * KF * CI;
#pragma unroll
                for (int kf = 0; kf < KF; ++kf)
#pragma unroll
                    for (int c = 0; c < CI / 2; ++c) {
                        const f32x2 w = {wr[kf * CI + 2 * c], wr[kf * CI + 2 * c + 1]};
#pragma unroll
                        for (int e = 0; e < DN_FPT; ++e) {
                            const float xv = win[e + KF - 1 - kf];
                            acc[c][e] = __builtin_elementwise_fma(w, (f32x2){xv, xv}, acc[c][e]);
                        }
                    }
            }
        }
    }
    const int t = t0 + ty;
    if (t >= g.T2) return;
#pragma unroll
    for (int c = 0; c < CI; ++c)
#pragma unroll
        for (int e = 0; e < DN_FPT; ++e) {
            const int f = f0 + 4 * tx + e;
            if (f >= g.Fi) continue;
            const int64_t o = (((int64_t)b * CI + c) * g.T2 + t) * g.Fi + f;
            float v = acc[c / 2][e][c % 2];
            if (a.ffr) v += feat_term(a, feat_coef(a), o);
            if (a.xact) v *= lrelu_grad(a.xact[o]);
            a.dx[o] = a.accumulate ? a.dx[o] + v : v;
        }
}

// ------------------------------------------------------------------------ weight grad
struct C2Wg {
    C2Geo g;
    const float* dy;
    const float* yact;
    const float* x;
    float* ws;  // [S][Co][N], N = VC*KF + 1 (bias column last)
    int BT, NR, RL, NCmax, items, per_split, chunks;
};

template <int BM, int BN, int WM, int WN, int WK, bool YM = true>
__global__ __launch_bounds__(NT) void c2_wgrad_kernel(C2Wg a) {
    constexpr int TM = BM / WM / 32, TN = BN / WN / 32;
    static_assert(WM * WN * WK == 4, "4 waves");
    extern __shared__ float smem[];
    const C2Geo g = a.g;
    constexpr int BT = WG_BT;
    const int NR = a.NR, RL = a.RL, KF = g.KF, S = g.sf;
    const int VC = g.Ci * g.KT, Nw = VC * KF, N = Nw + 1, XR = NR * RL;
    int4* rtab = (int4*)smem;                         // [NCmax*NR]: window-row table
    float* Ls = smem + 4 * a.NCmax * NR;              // [BT][BM]
    float* Rs = Ls + BT * BM;                         // [NCmax][NR][RL]
    int* poff = (int*)(Rs + a.NCmax * XR);            // [BT]
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wk = wave % WK, wmn = wave / WK;
    const int wm0 = (wmn / WN) * TM * 32, wn0 = (wmn % WN) * TN * 32;
    const int h = lane >> 5, l32 = lane & 31;
    const int co0 = blockIdx.y * BM, n0 = blockIdx.x * BN, split = blockIdx.z;
    const int c_first = n0 / KF;
    const int Nall = g.T2 * g.Fo;
    const int64_t plane_y = (int64_t)Nall, plane_x = (int64_t)g.T2 * g.Fi;
    int cbase[TN];
    bool isb[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) {
        const int n = n0 + wn0 + j * 32 + l32;
        const int vc = n / KF, kf = n - vc * KF;
        isb[j] = n == Nw;
        cbase[j] = (n < Nw) ? (vc - c_first) * XR + kf : 0;
    }
    f32x16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = (f32x16){0};
    // rows r = cl*NR + rs of the x window: {offset relative to row tf, row relative to tf, rs,
    // vc in range}; per item only tf / f0 / nr change, so the staging needs no division
    for (int r = tid; r < a.NCmax * NR; r += NT) {
        const int cl = r / NR, rs = r - cl * NR, vc = c_first + cl, ci = vc / g.KT, kt = vc - ci * g.KT;
        const int rrel = rs + kt * g.dt - g.pt;
        rtab[r] = make_int4(ci * (int)plane_x + rrel * g.Fi, rrel, rs, vc < VC);
    }
    const int dr = NT / RL, dw = NT - dr * RL, r_init = tid / RL, w_init = tid - r_init * RL;
    const int it_beg = split * a.per_split, it_end = min(a.items, it_beg + a.per_split);
    const int tw = BT / WK;
    for (int it = it_beg; it < it_end; ++it) {
        const int b = it / a.chunks, p0 = (it - b * a.chunks) * BT;
        const int pend = min(Nall, p0 + BT);
        const int tf = p0 / g.Fo, f0 = p0 - tf * g.Fo;
        const int nr = (pend - 1) / g.Fo - tf + 1;
        const float* dyb = a.dy + (int64_t)b * g.Co * plane_y;
        const float* yab = YM ? a.yact + (int64_t)b * g.Co * plane_y : nullptr;
        const float* xb = a.x + (int64_t)b * g.Ci * plane_x;
        __syncthreads();
        const float* ysrc = yab ? yab : dyb;
        for (int i0 = 0; i0 < BT * BM; i0 += NT * DPER) {
            float v[DPER], ym[DPER];
#pragma unroll
            for (int q = 0; q < DPER; ++q) {
                const int i = i0 + q * NT + tid;
                const int tl = i % BT, col = i / BT, p = p0 + tl, co = co0 + col;
                const bool ok = i < BT * BM && p < pend && co < g.Co;
                const int64_t o = ok ? (int64_t)co * plane_y + p : 0;
                const float t = dyb[o];
                if (YM) ym[q] = ysrc[o];
                v[q] = ok ? t : 0.f;
            }
#pragma unroll
            for (int q = 0; q < DPER; ++q) {
                const int i = i0 + q * NT + tid;
                if (i < BT * BM) {
                    const int tl = i % BT, col = i / BT;
                    Ls[tl * BM + col] = YM ? v[q] * lrelu_grad(ym[q]) : v[q];
                }
            }
        }
        {
            const int items = a.NCmax * XR, nrows = a.NCmax * NR, tfo = tf * g.Fi;
            int r = r_init, w = w_init;
            for (int i0 = 0; i0 < items; i0 += NT * DPER) {
                int rq[DPER], wq[DPER];
#pragma unroll
                for (int q = 0; q < DPER; ++q) {
                    rq[q] = r;
                    wq[q] = w;
                    w += dw;
                    r += dr;
                    if (w >= RL) {
                        w -= RL;
                        ++r;
                    }
                }
                int4 e[DPER];
#pragma unroll
                for (int q = 0; q < DPER; ++q) e[q] = rtab[rq[q] < nrows ? rq[q] : 0];
                float v[DPER];
#pragma unroll
                for (int q = 0; q < DPER; ++q) {
                    const int row = tf + e[q].y, pos = (e[q].z ? 0 : f0) * S - g.pf + wq[q];
                    const bool ok = rq[q] < nrows && e[q].w && e[q].z < nr && row >= 0 && row < g.T2 && pos >= 0 &&
                                    pos < g.Fi;
                    const float t = xb[ok ? e[q].x + tfo + pos : 0];
                    v[q] = ok ? t : 0.f;
                }
#pragma unroll
                for (int q = 0; q < DPER; ++q) {
                    const int i = i0 + q * NT + tid;
                    if (i < items) Rs[i] = v[q];
                }
            }
        }
        for (int tl = tid; tl < BT; tl += NT) {
            const int p = p0 + tl;
            int off = 0;
            if (p < pend) {
                const int tr = p / g.Fo, f = p - tr * g.Fo, rs = tr - tf;
                off = rs * RL + (f - (rs ? 0 : f0)) * S;
            }
            poff[tl] = off;
        }
        __syncthreads();
        for (int tp = wk * tw; tp < (wk + 1) * tw; tp += 2) {
            const int tl = tp + h;
            const int po = poff[tl];
            float av[TM], bv[TN];
#pragma unroll
            for (int i = 0; i < TM; ++i) av[i] = Ls[tl * BM + wm0 + i * 32 + l32];
#pragma unroll
            for (int j = 0; j < TN; ++j) bv[j] = isb[j] ? 1.f : Rs[cbase[j] + po];
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j) acc[i][j] = mfma32(av[i], bv[j], acc[i][j]);
        }
    }
    if (WK > 1) {
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
    float* wsb = a.ws + (int64_t)split * g.Co * N;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int n = n0 + wn0 + j * 32 + l32;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int co = co0 + wm0 + i * 32 + mfma_row(r, lane);
                if (co < g.Co && n < N) wsb[(int64_t)co * N + n] = acc[i][j][r];
            }
        }
}

// Weight grad, column-group form. dW[co][n] (n = vc*KF + kf, vc = ci*KT + kt) as a GEMM over
// the positions (b, t, f). A workgroup owns GC combos = GC*KF columns = NW*NTW tiles of 32 and
// all Co <= 32 rows; wave w keeps NTW column tiles, so the masked dy value a lane reads once per
// k-pair (the A operand) feeds NTW independent MFMA chains. Positions are staged W2_P at a time
// (one batch item per chunk): dy' = dy * LeakyReLU'(y) transposed into Ls[p][33] (the pad keeps
// the transposing store conflict-free) and the x window of the GC combos, Rs[GC][NR][RL]. A
// workgroup walks a contiguous range of chunks and writes one partial slab [Co][N + 1] (column
// Nw = the bias, summed by wave 0 of group 0 on the vector ALU); c2_wg_reduce adds the slabs in
// a fixed order.
constexpr int W2_P = 64;
struct C2Wg2 {
    C2Geo g;
    const float* dy;
    const float* yact;
    const float* x;
    float* ws;  // [splits][Co][N], N = VC*KF + 1
    int NR, RL, GC, items, per_split, chunks;
};

template <int KF, int NTW, int NW>
__global__ __launch_bounds__(NW * 64) void c2_wgrad2_kernel(C2Wg2 a) {
    constexpr int NTH = NW * 64, P = W2_P, LDA = 33;
    extern __shared__ float smem[];
    const C2Geo g = a.g;
    const int NR = a.NR, RL = a.RL, GC = a.GC, S = g.sf, XR = NR * RL;
    const int VC = g.Ci * g.KT, Nw = VC * KF, N = Nw + 1;
    int4* rtab = (int4*)smem;                  // [GC*NR]: {offset at row tf, row - tf, rs, valid}
    float* Ls = smem + 4 * GC * NR;            // [P][LDA]
    int* poff = (int*)(Ls + P * LDA);          // [P]
    float* Rs = (float*)(poff + P);            // [GC][NR][RL]
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int h = lane >> 5, l32 = lane & 31;
    const int vc0 = blockIdx.x * GC, split = blockIdx.y;
    const int n0 = vc0 * KF + wave * NTW * 32;
    const int Nall = g.T2 * g.Fo;
    const int64_t plane_y = (int64_t)Nall, plane_x = (int64_t)g.T2 * g.Fi;
    const bool do_bias = blockIdx.x == 0 && wave == 0;
    int cbase[NTW];
#pragma unroll
    for (int j = 0; j < NTW; ++j) {
        const int n = n0 + j * 32 + l32;
        const int vc = n / KF, kf = n - vc * KF;
        cbase[j] = (n < Nw) ? (vc - vc0) * XR + kf : 0;
    }
    f32x16 acc[NTW];
#pragma unroll
    for (int j = 0; j < NTW; ++j) acc[j] = (f32x16){0};
    float bsum = 0.f;
    for (int r = tid; r < GC * NR; r += NTH) {
        const int cl = r / NR, rs = r - cl * NR, vc = vc0 + cl, ci = vc / g.KT, kt = vc - ci * g.KT;
        const int rrel = rs + kt * g.dt - g.pt;
        rtab[r] = make_int4(ci * (int)plane_x + rrel * g.Fi, rrel, rs, vc < VC);
    }
    const int dr = NTH / RL, dw = NTH - dr * RL, r_init = tid / RL, w_init = tid - r_init * RL;
    const int it_beg = split * a.per_split, it_end = min(a.items, it_beg + a.per_split);
    for (int it = it_beg; it < it_end; ++it) {
        const int b = it / a.chunks, p0 = (it - b * a.chunks) * P;
        const int pend = min(Nall, p0 + P);
        const int tf = p0 / g.Fo, f0 = p0 - tf * g.Fo;
        const int nr = (pend - 1) / g.Fo - tf + 1;
        const float* dyb = a.dy + (int64_t)b * g.Co * plane_y;
        const float* yab = a.yact ? a.yact + (int64_t)b * g.Co * plane_y : dyb;
        const float* xb = a.x + (int64_t)b * g.Ci * plane_x;
        __syncthreads();
        // dy' chunk, read along positions (coalesced), stored transposed
        for (int i0 = 0; i0 < P * 32; i0 += NTH * DPER) {
            float v[DPER], ym[DPER];
#pragma unroll
            for (int q = 0; q < DPER; ++q) {
                const int i = i0 + q * NTH + tid;
                const int co = i / P, tl = i - co * P, p = p0 + tl;
                const bool ok = i < P * 32 && p < pend && co < g.Co;
                const int64_t o = ok ? (int64_t)co * plane_y + p : 0;
                const float t = dyb[o];
                ym[q] = yab[o];
                v[q] = ok ? t : 0.f;
            }
#pragma unroll
            for (int q = 0; q < DPER; ++q) {
                const int i = i0 + q * NTH + tid;
                if (i < P * 32) {
                    const int co = i / P, tl = i - co * P;
                    Ls[tl * LDA + co] = a.yact ? v[q] * lrelu_grad(ym[q]) : v[q];
                }
            }
        }
        {  // x window of the group's combos
            const int items = GC * XR, nrows = GC * NR, tfo = tf * g.Fi;
            int r = r_init, w = w_init;
            for (int i0 = 0; i0 < items; i0 += NTH * DPER) {
                int rq[DPER], wq[DPER];
#pragma unroll
                for (int q = 0; q < DPER; ++q) {
                    rq[q] = r;
                    wq[q] = w;
                    w += dw;
                    r += dr;
                    if (w >= RL) {
                        w -= RL;
                        ++r;
                    }
                }
                int4 e[DPER];
#pragma unroll
                for (int q = 0; q < DPER; ++q) e[q] = rtab[rq[q] < nrows ? rq[q] : 0];
                float v[DPER];
#pragma unroll
                for (int q = 0; q < DPER; ++q) {
                    const int row = tf + e[q].y, pos = (e[q].z ? 0 : f0) * S - g.pf + wq[q];
                    const bool ok = rq[q] < nrows && e[q].w && e[q].z < nr && row >= 0 && row < g.T2 && pos >= 0 &&
                                    pos < g.Fi;
                    const float t = xb[ok ? e[q].x + tfo + pos : 0];
                    v[q] = ok ? t : 0.f;
                }
#pragma unroll
                for (int q = 0; q < DPER; ++q) {
                    const int i = i0 + q * NTH + tid;
                    if (i < items) Rs[i] = v[q];
                }
            }
        }
        for (int tl = tid; tl < P; tl += NTH) {
            const int p = p0 + tl;
            int off = 0;
            if (p < pend) {
                const int tr = p / g.Fo, f = p - tr * g.Fo, rs = tr - tf;
                off = rs * RL + (f - (rs ? 0 : f0)) * S;
            }
            poff[tl] = off;
        }
        __syncthreads();
#pragma unroll 4
        for (int kp = 0; kp < P / 2; ++kp) {
            const int tl = 2 * kp + h;
            const int po = poff[tl];
            const float av = Ls[tl * LDA + l32];
            if (do_bias) bsum += av;
            float bv[NTW];
#pragma unroll
            for (int j = 0; j < NTW; ++j) bv[j] = Rs[cbase[j] + po];
#pragma unroll
            for (int j = 0; j < NTW; ++j) acc[j] = mfma32(av, bv[j], acc[j]);
        }
    }
    float* wsb = a.ws + (int64_t)split * g.Co * N;
#pragma unroll
    for (int j = 0; j < NTW; ++j) {
        const int n = n0 + j * 32 + l32;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int co = mfma_row(r, lane);
            if (co < g.Co && n < Nw) wsb[(int64_t)co * N + n] = acc[j][r];
        }
    }
    if (do_bias) {
        bsum += __shfl_xor(bsum, 32, 64);
        if (h == 0 && l32 < g.Co) wsb[(int64_t)l32 * N + Nw] = bsum;
    }
}

// Weight grad, column-group form with vectorised staging: c2_wgrad2_kernel's GEMM (a
// workgroup owns GC combos = NW * NTW column tiles and all Co <= 32 rows, positions staged
// W3_P per chunk), but every staged value moves in aligned quads: dy and y along the positions
// (then transposed into Ls[p][33] by four ds_write_b32), the x window as column-aligned quads
// (c2_fwdr_kernel). All of a chunk's loads are issued before any of its LDS stores.
constexpr int W3_P = 64;
struct C2Wg3 {
    C2Geo g;
    const float* dy;
    const float* yact;
    const float* x;
    float* ws;  // [splits][Co][N], N = VC*KF + 1
    int NR, RL, GC, items, per_split, chunks;
};
template <int KF, int NTW, int NW, int MQ, int ML, int OCC = 1, int PF = 0, bool YM = true>
__global__ __launch_bounds__(NW * 64, OCC) void c2_wgrad3_kernel(C2Wg3 a) {
    // PF: the next chunk's global loads are issued before this chunk's MFMA loop (register
    // pipelining, as c2_dgradr_kernel), so their latency hides under the 32 k-pairs
    constexpr int NTH = NW * 64, P = W3_P, LDA = 33, PQ = P / 4;
    extern __shared__ float smem[];
    const C2Geo g = a.g;
    const int NR = a.NR, RL = a.RL, GC = a.GC, S = g.sf;
    const int RLp = (RL + 3) & ~3, NQ = RLp >> 2, XR = NR * RLp;
    const int VC = g.Ci * g.KT, Nw = VC * KF, N = Nw + 1;
    int4* rtab = (int4*)smem;                  // [GC*NR]: {offset at row tf, row - tf, rs, valid}
    float* Ls = smem + 4 * GC * NR;            // [P][LDA]
    int* poff = (int*)(Ls + P * LDA);          // [P]
    float* Rs = (float*)(poff + P);            // [GC][NR][RLp] (16-byte aligned: see plan_wg3r)
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int h = lane >> 5, l32 = lane & 31;
    const TileId tile = xcd_tile();  // the combo groups of one split share its dy chunks
    const int vc0 = tile.x * GC, split = tile.y;
    const int n0 = vc0 * KF + wave * NTW * 32;
    const int Nall = g.T2 * g.Fo;
    const int64_t plane_y = (int64_t)Nall, plane_x = (int64_t)g.T2 * g.Fi;
    const int64_t ytot = (int64_t)g.B * g.Co * plane_y, xtot = (int64_t)g.B * g.Ci * plane_x;
    const bool do_bias = tile.x == 0 && wave == 0;
    const int baseN = (-g.pf) & ~3;
    int cbase[NTW];
#pragma unroll
    for (int j = 0; j < NTW; ++j) {
        const int n = n0 + j * 32 + l32;
        const int vc = n / KF, kf = n - vc * KF;
        cbase[j] = (n < Nw) ? (vc - vc0) * XR + kf : 0;
    }
    f32x16 acc[NTW];
#pragma unroll
    for (int j = 0; j < NTW; ++j) acc[j] = (f32x16){0};
    float bsum = 0.f;
    for (int r = tid; r < GC * NR; r += NTH) {
        const int cl = r / NR, rs = r - cl * NR, vc = vc0 + cl, ci = vc / g.KT, kt = vc - ci * g.KT;
        const int rrel = rs + kt * g.dt - g.pt;
        rtab[r] = make_int4(ci * (int)plane_x + rrel * g.Fi, rrel, rs, vc < VC);
    }
    const int dr = NTH / NQ, dq = NTH - dr * NQ, r_init = tid / NQ, q_init = tid - r_init * NQ;
    const int it_beg = split * a.per_split, it_end = min(a.items, it_beg + a.per_split);
    __syncthreads();
    f32x4 dv[ML], yv[ML], xv[MQ];
    int dmask[ML], xmask[MQ];
    // ---- loads of chunk it: dy / y quads along positions, x window quads
    auto load = [&](int it) {
        const int b = it / a.chunks, p0 = (it - b * a.chunks) * P;
        const int pend = min(Nall, p0 + P);
        const int tf = p0 / g.Fo, f0 = p0 - tf * g.Fo;
        const int nr = (pend - 1) / g.Fo - tf + 1;
        const int base0 = (f0 * S - g.pf) & ~3;
        const int64_t yb = (int64_t)b * g.Co * plane_y, xbo = (int64_t)b * g.Ci * plane_x;
#pragma unroll
        for (int u = 0; u < ML; ++u) {
            const int i = u * NTH + tid, co = i / PQ, k = i - co * PQ, p = p0 + 4 * k;
            const bool any = i < 32 * PQ && co < g.Co && p < pend;
            int64_t off = any ? yb + (int64_t)co * plane_y + p : 0;
            const int64_t offc = off > ytot - 4 ? ytot - 4 : off;
            dv[u] = ld4u(a.dy + offc);
            if (YM) yv[u] = ld4u(a.yact + offc);
            dmask[u] = any ? (min(pend - p, 4) | ((int)(off - offc) << 4)) : 0;
        }
        int r = r_init, q = q_init;
#pragma unroll
        for (int u = 0; u < MQ; ++u) {
            const int rr = r < GC * NR ? r : 0;
            const int4 e = rtab[rr];
            const int base = e.z ? baseN : base0, col = base + 4 * q;
            const int row = tf + e.y;
            const bool any = r < GC * NR && e.w && e.z < nr && row >= 0 && row < g.T2 && col >= 0 && col < g.Fi;
            int64_t off = any ? xbo + e.x + (int64_t)tf * g.Fi + col : 0;
            const int64_t offc = off > xtot - 4 ? xtot - 4 : off;
            xv[u] = ld4u(a.x + offc);
            xmask[u] = any ? (min(g.Fi - col, 4) | ((int)(off - offc) << 4)) : 0;
            q += dq;
            r += dr;
            if (q >= NQ) {
                q -= NQ;
                ++r;
            }
        }
    };
    // ---- LDS image of chunk it from the loaded registers
    auto store = [&](int it) {
        const int b = it / a.chunks, p0 = (it - b * a.chunks) * P;
        const int pend = min(Nall, p0 + P);
        const int tf = p0 / g.Fo, f0 = p0 - tf * g.Fo;
        const int base0 = (f0 * S - g.pf) & ~3;
#pragma unroll
        for (int u = 0; u < ML; ++u) {
            const int i = u * NTH + tid, co = i / PQ, k = i - co * PQ;
            if (i < 32 * PQ) {
                const int m = dmask[u], nv = m & 15, sh = m >> 4;
                f32x4 v = dv[u], y = yv[u];
                if (sh) {
                    const f32x4 t = v, ty = y;
#pragma unroll
                    for (int c = 0; c < 4; ++c) {
                        v[c] = c + sh < 4 ? (c + sh == 1 ? t[1] : c + sh == 2 ? t[2] : t[3]) : 0.f;
                        y[c] = c + sh < 4 ? (c + sh == 1 ? ty[1] : c + sh == 2 ? ty[2] : ty[3]) : 0.f;
                    }
                }
#pragma unroll
                for (int c = 0; c < 4; ++c)
                    Ls[(4 * k + c) * LDA + co] = c < nv ? (YM ? v[c] * lrelu_grad(y[c]) : v[c]) : 0.f;
            }
        }
        int r = r_init, q = q_init;
#pragma unroll
        for (int u = 0; u < MQ; ++u) {
            const int m = xmask[u], nv = m & 15, sh = m >> 4;
            f32x4 v = xv[u];
            if (sh) {
                const f32x4 t = v;
#pragma unroll
                for (int c = 0; c < 4; ++c) v[c] = c + sh < 4 ? (c + sh == 1 ? t[1] : c + sh == 2 ? t[2] : t[3]) : 0.f;
            }
#pragma unroll
            for (int c = 0; c < 4; ++c) v[c] = c < nv ? v[c] : 0.f;
            if (r < GC * NR) *(f32x4*)(Rs + r * RLp + 4 * q) = v;
            q += dq;
            r += dr;
            if (q >= NQ) {
                q -= NQ;
                ++r;
            }
        }
        for (int tl = tid; tl < P; tl += NTH) {
            const int p = p0 + tl;
            int off = 0;
            if (p < pend) {
                const int tr = p / g.Fo, f = p - tr * g.Fo, rs = tr - tf;
                off = rs * RLp + f * S - g.pf - (rs ? baseN : base0);
            }
            poff[tl] = off;
        }
    };
    if (PF && it_beg < it_end) load(it_beg);
    for (int it = it_beg; it < it_end; ++it) {
        if (!PF) load(it);
        __syncthreads();  // the previous chunk's MFMAs are done with Ls / Rs
        store(it);
        __syncthreads();
        if (PF && it + 1 < it_end) load(it + 1);
#pragma unroll 4
        for (int kp = 0; kp < P / 2; ++kp) {
            const int tl = 2 * kp + h;
            const int po = poff[tl];
            const float av = Ls[tl * LDA + l32];
            bsum += av;  // every wave (no branch in the loop); only the bias wave stores it
            float bv[NTW];
#pragma unroll
            for (int j = 0; j < NTW; ++j) bv[j] = Rs[cbase[j] + po];
#pragma unroll
            for (int j = 0; j < NTW; ++j) acc[j] = mfma32(av, bv[j], acc[j]);
        }
    }
    float* wsb = a.ws + (int64_t)split * g.Co * N;
#pragma unroll
    for (int j = 0; j < NTW; ++j) {
        const int n = n0 + j * 32 + l32;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int co = mfma_row(r, lane);
            if (co < g.Co && n < Nw) wsb[(int64_t)co * N + n] = acc[j][r];
        }
    }
    if (do_bias) {
        bsum += __shfl_xor(bsum, 32, 64);
        if (h == 0 && l32 < g.Co) wsb[(int64_t)l32 * N + Nw] = bsum;
    }
}

// Weight grad, register-window form: no LDS, no staging. The GEMM's reduction index is the
// output position, and the MFMA's two k slots are two positions, so the 32 x 32 tile of one tap
// (kt, kf) is D[co][ci] = sum_p dy'[co][p] x[ci][row(p, kt)][S p + kf - pf]. A wave owns 9 taps
// (one kt of a 3x9 layer, or all of a 3x3 layer) and walks (b, t, 8-position chunk) items; half
// h of the wave takes positions f0 + 4h .. f0 + 4h + 3 of a chunk, so
//   A: lane (h, co) needs dy'[co][t][f0 + 4h + q], q < 4: ONE quad load (+ the y quad for
//      LeakyReLU'(y)),
//   B: lane (h, ci) needs, for all 9 taps and the 4 positions, x[ci][row][S (f0 + 4h) - pf + r],
//      r < 3S + KF: one contiguous window of WQ quads per kt row,
// and a chunk is 9 taps x 4 positions = 36 MFMAs on 9 accumulator chains (one per tap), with
// no LDS read and no address arithmetic between them. The next item's quads are loaded before the
// current item's MFMAs (register double buffer). Each wave writes its 32 x 32 x 9 partial to
// the split slab ws[split][co][n] (c2_wg_reduce sums the slabs in a fixed order).
struct C2WgR {
    C2Geo g;
    const float* dy;
    const float* yact;
    const float* x;
    float* ws;      // [splits][Co][N], N = Ci*KT*KF + 1
    int NC;         // 8-position chunks per output row
    int items;      // B * T2 * NC
    int per_split;  // items per wave
    int ktg;        // kt groups (tasks per split per ci block): KT for KF = 9, 1 for KF = 3
    int cib;        // 32-channel ci blocks
    int SW, NCS;    // item order: strips of SW chunks (SW | NC, NCS = NC / SW), t within a strip
};
template <int KTW, int WQ>
struct RwStage {  // one item's operands, loaded a whole item ahead of their MFMAs
    f32x4 av, yv, xw[KTW][WQ];
    int p, col0;  // this lane's first position / first input column (for the edge masks)
    int sha;      // the dy / y quad's shift (nonzero only at the very end of the tensor)
    int xo[KTW];  // this lane's first window element offset per kt row (unclamped)
    bool edge;    // wave-uniform: some element of this item lies outside its row
    bool rok[KTW];
};
// NW > 1 (c2_wgrad_rwg): NW waves per workgroup share one (kt group, ci block, split) task and
// take its items interleaved (wave w: items it_beg + w, + NW, ...; neighbouring waves read
// neighbouring windows), then sum their 32 x 32 x NTAP accumulators through LDS in a fixed
// order (waves 0..3 store, waves 4..7 add, one pass sums the four) and store ONE task partial,
// contiguous, in the task-major slab ws[split][kt group][ci block][co][ci][tap] (+ 32 biases),
// which c2_wgr_reduce sums: NW x fewer slab bytes than the one-wave form, and coalesced.
template <int KF, int S, int KTW, int WQ, bool YM, int NW = 1>
__global__ __launch_bounds__(NW * 64, NW == 1 ? 2 : 1) void c2_wgrad_rw_kernel(C2WgR a) {
    constexpr int NTAP = KTW * KF;
    static_assert(NW == 1 || NW == 8, "one-wave or 8-wave workgroups");
    const C2Geo g = a.g;
    const int lane = threadIdx.x & 63, h = lane >> 5, l = lane & 31, wv = threadIdx.x >> 6;
    const int id = xcd_linear_id();
    const int kg = id % a.ktg, rest = id / a.ktg, cb = rest % a.cib, split = rest / a.cib;
    const int kt0 = kg * KTW, ci = cb * 32 + l;
    const bool ci_ok = ci < g.Ci, co_ok = l < g.Co;
    const bool full = g.Co >= 32 && (cb + 1) * 32 <= g.Ci;  // every lane's row and column exist
    const int it_beg = split * a.per_split, it_end = min(a.items, it_beg + a.per_split);
    // element offsets fit in 32 bits (checked on the host)
    const int plane_y = g.T2 * g.Fo, plane_x = g.T2 * g.Fi;
    const int ylast = g.B * g.Co * plane_y - 4, xlast = g.B * g.Ci * plane_x - 4;
    f32x16 acc[NTAP];
#pragma unroll
    for (int j = 0; j < NTAP; ++j) acc[j] = (f32x16){0};
    float bsum = 0.f;
    // ---- issue the loads of item it; nothing waits for them until compute(). Every quad is one
    // (unaligned) load at its own address, so every item issues the same loads: elements past a
    // row's ends read the neighbouring row (in bounds) and compute() zeroes them; only a quad
    // past the END of the tensor is read from a clamped address and shifted.
    auto load = [&](RwStage<KTW, WQ>& st, int it) {
        // items run (b, strip, t, chunk in strip), the chunk fastest: the kt-group workgroups of a
        // task (same ci block and split, same XCD) read the same dy / y quads at the same time and
        // x rows one or two steps of t apart, a reuse distance of a strip's bytes, not a row's
        const int cs = it % a.SW, r1 = it / a.SW, t = r1 % g.T2, r2 = r1 / g.T2;
        const int c = (r2 % a.NCS) * a.SW + cs, b = r2 / a.NCS;
        const int f0 = c * 8, p = f0 + 4 * h;
        const int oa = (b * g.Co + (co_ok ? l : 0)) * plane_y + t * g.Fo + p;
        const int oac = min(oa, ylast);
        st.av = ld4u(a.dy + oac);
        if (YM) st.yv = ld4u(a.yact + oac);
        st.sha = oa - oac;
        const int col0 = S * p - g.pf;
        const int xb = (b * g.Ci + (ci_ok ? ci : 0)) * plane_x + col0;
#pragma unroll
        for (int k = 0; k < KTW; ++k) {
            const int row = t + (kt0 + k) * g.dt - g.pt;
            st.rok[k] = row >= 0 && row < g.T2;
            const int rb = xb + (st.rok[k] ? row : 0) * g.Fi;
#pragma unroll
            for (int w = 0; w < WQ; ++w) st.xw[k][w] = ld4u(a.x + min(max(rb + 4 * w, 0), xlast));
            st.xo[k] = rb;
        }
        st.p = p;
        st.col0 = col0;
        st.edge = f0 + 8 > g.Fo || S * f0 - g.pf < 0 || S * (f0 + 4) - g.pf + 4 * WQ > g.Fi;
    };
    // ---- the 9 taps x 4 positions of one item
    auto compute = [&](RwStage<KTW, WQ>& st) {
        if (st.edge) {
            if (__any(st.sha != 0)) {
                st.av = quad_abs(st.av, ylast + st.sha, ylast);
                if (YM) st.yv = quad_abs(st.yv, ylast + st.sha, ylast);
            }
#pragma unroll
            for (int e = 0; e < 4; ++e)
                if (st.p + e >= g.Fo) st.av[e] = 0.f;
#pragma unroll
            for (int w = 0; w < WQ; ++w) {
#pragma unroll
                for (int k = 0; k < KTW; ++k) {  // the tensor's first / last quad
                    const int o = st.xo[k] + 4 * w;
                    if (__any(o < 0 || o > xlast)) st.xw[k][w] = quad_abs(st.xw[k][w], o, xlast);
                }
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int col = st.col0 + 4 * w + e;
                    if (col < 0 || col >= g.Fi) {
#pragma unroll
                        for (int k = 0; k < KTW; ++k) st.xw[k][w][e] = 0.f;
                    }
                }
            }
        }
        if (!full) {
            if (!co_ok) st.av = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int k = 0; k < KTW; ++k)
#pragma unroll
                for (int w = 0; w < WQ; ++w)
                    if (!ci_ok) st.xw[k][w] = (f32x4){0.f, 0.f, 0.f, 0.f};
        }
        f32x4 ca = st.av;
        if (YM) {
#pragma unroll
            for (int e = 0; e < 4; ++e) ca[e] *= lrelu_grad(st.yv[e]);
        }
        bsum += (ca[0] + ca[1]) + (ca[2] + ca[3]);
#pragma unroll
        for (int k = 0; k < KTW; ++k) {
            if (!st.rok[k]) continue;  // a kt row outside the input contributes zero
#pragma unroll
            for (int q = 0; q < 4; ++q)
#pragma unroll
                for (int kf = 0; kf < KF; ++kf) {
                    const int r = S * q + kf;
                    acc[k * KF + kf] = mfma32(ca[q], st.xw[k][r >> 2][r & 3], acc[k * KF + kf]);
                }
        }
    };
    // two register stages, alternating: item it + 1 is in flight while item it computes
    // The prefetches are unconditional (past the end they re-load the last item and are never
    // used), so every path issues the same loads and each wait is for exactly the older item.
    RwStage<KTW, WQ> s0, s1;
    const int it0 = it_beg + wv;
    if (it0 < it_end) load(s0, it0);
    for (int it = it0; it < it_end; it += 2 * NW) {
        load(s1, min(it + NW, it_end - 1));
        compute(s0);
        if (it + NW >= it_end) break;
        load(s0, min(it + 2 * NW, it_end - 1));
        compute(s1);
    }
    if constexpr (NW > 1) {
        // ---- fixed-order workgroup sum through LDS, then one contiguous task partial
        extern __shared__ float red[];  // [4][32 co][32 ci][NTAP] + [NW][32] biases
        constexpr int TS = 32 * 32 * NTAP;
        float* bred = red + 4 * TS;
        bsum += __shfl_xor(bsum, 32, 64);
        if (h == 0) bred[wv * 32 + l] = bsum;
#pragma unroll
        for (int pass = 0; pass < 2; ++pass) {
            if ((wv >> 2) == pass) {
                float* reg = red + (wv & 3) * TS;
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int co = mfma_row(r, lane);
#pragma unroll
                    for (int j = 0; j < NTAP; ++j) {
                        float* q = reg + (co * 32 + l) * NTAP + j;
                        *q = pass == 0 ? acc[j][r] : *q + acc[j][r];
                    }
                }
            }
            __syncthreads();
        }
        const int64_t SZ = (int64_t)a.ktg * a.cib * TS + 32;
        float* dst = a.ws + (int64_t)split * SZ + (int64_t)(kg * a.cib + cb) * TS;
        for (int d = threadIdx.x; d < TS; d += NW * 64)
            dst[d] = ((red[d] + red[TS + d]) + red[2 * TS + d]) + red[3 * TS + d];
        if (kg == 0 && cb == 0 && threadIdx.x < 32) {
            float b = 0.f;
#pragma unroll
            for (int w = 0; w < NW; ++w) b += bred[w * 32 + threadIdx.x];
            a.ws[(int64_t)split * SZ + (SZ - 32) + threadIdx.x] = b;
        }
        return;
    }
    // ---- the partial: D[co][ci] of tap (kt0 + k, kf) -> ws[split][co][(ci*KT + kt)*KF + kf]
    const int N = g.Ci * g.KT * KF + 1;
    float* wsb = a.ws + (int64_t)split * g.Co * N;
    if (ci_ok) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int co = mfma_row(r, lane);
            if (co < g.Co) {
                float* dst = wsb + (int64_t)co * N + (ci * g.KT + kt0) * KF;
#pragma unroll
                for (int j = 0; j < NTAP; ++j) dst[j] = acc[j][r];
            }
        }
    }
    if (kg == 0 && cb == 0) {
        bsum += __shfl_xor(bsum, 32, 64);
        if (h == 0 && co_ok) wsb[(int64_t)l * N + N - 1] = bsum;
    }
}

// part[g][i] = sum of slabs s in [g*G, (g+1)*G) of ws[s][i], ascending: the first stage of a
// two-stage slab sum when the slabs far outnumber the outputs (c2_wg_reduce alone would run a
// few dozen workgroups, each adding hundreds of slabs in sequence)
__global__ __launch_bounds__(256) void c2_slab_group_sum(const float* ws, int S, int G, int64_t n, float* part) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const int g = blockIdx.y, s0 = g * G, cnt = min(G, S - s0);
    part[(int64_t)g * n + i] = (float)sum_strided_d(ws + (int64_t)s0 * n + i, cnt, n);
}

// dw[co][n] (+)= sum_s ws[s][co][n] for n < Nw; db[co] (+)= sum_s ws[s][co][Nw]. Fixed order
// (slab_sum_256_d: 64 outputs per block, 4 split slices, fp64 accumulation: at B 32 the bias
// grads sum ~10^5 positions through up to ~1500 slabs, and an fp32 sum of the slabs lost ~4x the
// accuracy of a pairwise fp32 sum, test_config3_b32_step_vs_oracle_fp64).
__global__ __launch_bounds__(256) void c2_wg_reduce(const float* ws, int S, int Co, int N, float* dw, float* db,
                                                    int acc_w, int acc_b) {
    __shared__ double red[256];
    const int64_t i = (int64_t)blockIdx.x * 64 + (threadIdx.x & 63);
    const bool valid = i < (int64_t)Co * N;
    const float v = slab_sum_256_d(ws + (valid ? i : 0), S, (int64_t)Co * N, valid, red);
    if (threadIdx.x >= 64 || !valid) return;
    const int co = (int)(i / N), n = (int)(i - (int64_t)co * N);
    const int Nw = N - 1;
    if (n < Nw) {
        if (dw) {
            float* p = dw + (int64_t)co * Nw + n;
            *p = acc_w ? *p + v : v;
        }
    } else if (db) {
        db[co] = acc_b ? db[co] + v : v;
    }
}

// dw[co][(ci*KT + kt)*KF + kf] (+)= sum_s of the task-major slabs of c2_wgrad_rw_kernel<.., NW > 1>
// (ws[s][kg][cb][co][ci % 32][k*KF + kf], kt = kg*KTW + k, cb = ci / 32; the biases at SZ - 32 + co),
// db[co] likewise. Fixed order (slab_sum_256_d).
__global__ __launch_bounds__(256) void c2_wgr_reduce(const float* ws, int S, int64_t SZ, int Co, int Ci, int KT,
                                                     int KF, int KTW, int cib, float* dw, float* db, int acc_w,
                                                     int acc_b) {
    __shared__ double red[256];
    const int N = Ci * KT * KF + 1;
    const int64_t i = (int64_t)blockIdx.x * 64 + (threadIdx.x & 63);
    const bool valid = i < (int64_t)Co * N;
    int64_t off = 0;
    int co = 0, n = 0;
    if (valid) {
        co = (int)(i / N);
        n = (int)(i - (int64_t)co * N);
        if (n < N - 1) {
            const int ci = n / (KT * KF), kt = (n / KF) % KT, kf = n % KF;
            const int kg = kt / KTW, k = kt % KTW, NTAP = KTW * KF;
            off = ((((int64_t)kg * cib + ci / 32) * 32 + co) * 32 + (ci & 31)) * NTAP + k * KF + kf;
        } else {
            off = SZ - 32 + co;
        }
    }
    const float v = slab_sum_256_d(ws + off, S, SZ, valid, red);
    if (threadIdx.x >= 64 || !valid) return;
    if (n < N - 1) {
        if (dw) {
            float* p = dw + (int64_t)co * (N - 1) + n;
            *p = acc_w ? *p + v : v;
        }
    } else if (db) {
        db[co] = acc_b ? db[co] + v : v;
    }
}

// wp[(co,kt)][q][ci*S + r] = W[co][ci][kt][q*S + r] from wf[((ci,kt))*KF + kf][co]
__global__ void c2_wpoly_kernel(const float* wf, float* wp, int Co, int Ci, int KT, int KF, int S, int J) {
    const int64_t total = (int64_t)Co * KT * J * Ci * S;
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= total) return;
    const int M = Ci * S;
    const int m = (int)(i % M);
    const int64_t rq = i / M;
    const int q = (int)(rq % J), vc = (int)(rq / J);
    const int co = vc / KT, kt = vc - co * KT;
    const int ci = m / S, r = m - ci * S, kf = q * S + r;
    wp[i] = kf < KF ? wf[(((int64_t)ci * KT + kt) * KF + kf) * Co + co] : 0.f;
}

// ---------------------------------------------------------------------------- spectrogram
struct LdSpecD {  // A(m = (bc, fr), k) = x[bc][fr*hop + k]; B = DFT table [n][2nb]
    // (scalar staging: the quad form measured 4 % slower here)
    static constexpr bool A_K_FAST = true, B_N_FAST = true, VEC = false;
    const float* x;
    const float* bt;
    int T, Fr, hop, nb2;
    FastDiv fFr;
    ENCX_DEV float a(int m, int k) const {
        const int bc = (int)fdiv((uint32_t)m, fFr), fr = m - bc * Fr;
        return x[(int64_t)bc * T + (int64_t)fr * hop + k];
    }
    ENCX_DEV float b(int k, int n) const { return bt[(int64_t)k * nb2 + n]; }
    ENCX_DEV f32x4 a4(int m, int k) const {  // k..k+3 of one frame (k + 3 < n_fft)
        const int bc = (int)fdiv((uint32_t)m, fFr), fr = m - bc * Fr;
        return ld4u(x + (int64_t)bc * T + (int64_t)fr * hop + k);
    }
    ENCX_DEV f32x4 b4(int k, int n) const { return ld4u(bt + (int64_t)k * nb2 + n); }
};
struct EpSpecD {  // z[b][ch][fr][k], ch = c (re) or C + c (im)
    float* z;
    int C, Fr, nb;
    float inv;
    ENCX_DEV void operator()(int m, int n, float v) const {
        const int bc = m / Fr, fr = m - bc * Fr, b = bc / C, c = bc - b * C;
        const int im = n >= nb, k = im ? n - nb : n, ch = im ? C + c : c;
        z[(((int64_t)b * 2 * C + ch) * Fr + fr) * nb + k] = v * inv;
    }
};
struct LdSpecDB {  // A(m = (bc, fr), col) = dz at col; B(col, t) = bt[t][col]
    static constexpr bool A_K_FAST = true, B_N_FAST = false, VEC = true;
    const float* dz;
    const float* bt;
    int C, Fr, nb, nb2;
    float inv;
    ENCX_DEV float a(int m, int col) const {
        const int bc = m / Fr, fr = m - bc * Fr, b = bc / C, c = bc - b * C;
        const int im = col >= nb, k = im ? col - nb : col, ch = im ? C + c : c;
        return dz[(((int64_t)b * 2 * C + ch) * Fr + fr) * nb + k] * inv;
    }
    ENCX_DEV float b(int col, int t) const { return bt[(int64_t)t * nb2 + col]; }
    ENCX_DEV f32x4 a4(int m, int col) const {
        if (col < nb && col + 3 >= nb) {  // the quad straddles the re / im boundary
            f32x4 v;
#pragma unroll
            for (int q = 0; q < 4; ++q) v[q] = a(m, col + q);
            return v;
        }
        const int bc = m / Fr, fr = m - bc * Fr, b = bc / C, c = bc - b * C;
        const int im = col >= nb, k = im ? col - nb : col, ch = im ? C + c : c;
        const f32x4 v = ld4u(dz + (((int64_t)b * 2 * C + ch) * Fr + fr) * nb + k);
        return (f32x4){v[0] * inv, v[1] * inv, v[2] * inv, v[3] * inv};
    }
    ENCX_DEV f32x4 b4(int col, int t) const { return ld4u(bt + (int64_t)t * nb2 + col); }
};
struct EpFrames {
    float* out;
    int n;
    ENCX_DEV void operator()(int m, int t, float v) const { out[(int64_t)m * n + t] = v; }
};
// dx[bc][t] (+)= sum_{fr: 0 <= t - fr*hop < n} frames[bc*Fr + fr][t - fr*hop], fr ascending
__global__ void spec_overlap_add(const float* frames, float* dx, int BC, int T, int Fr, int n, int hop,
                                 int acc) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (int64_t)BC * T) return;
    const int bc = (int)(i / T), t = (int)(i - (int64_t)bc * T);
    int lo = t - n + 1;
    lo = lo <= 0 ? 0 : (lo + hop - 1) / hop;
    const int hi = min(Fr - 1, t / hop);
    float s = 0.f;
    for (int fr = lo; fr <= hi; ++fr) s += frames[((int64_t)bc * Fr + fr) * n + (t - fr * hop)];
    dx[i] = acc ? dx[i] + s : s;
}

// ---------------------------------------------------------------------------- losses
// sums[0] += sum relu(1 + s*x) over n (s = -1: generator / real term, +1: fake term)
__global__ __launch_bounds__(256) void hinge_kernel(const float* x, int64_t n, float s, float* parts) {
    __shared__ float red[16];
    float acc = 0.f;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
        acc += fmaxf(1.f + s * x[i], 0.f);
    acc = block_sum(acc, red);
    if (threadIdx.x == 0) parts[blockIdx.x] = acc;
}
// parts[b] = (sum |fr - ff|, sum |fr|) over a grid-stride slice: float4 loads, 4 in flight per
// operand and thread (n % 4 == 0, 16-byte aligned maps: torch allocations of 32-channel maps)
template <bool CODE>
__global__ __launch_bounds__(256) void feat_kernel(const float* fr, const float* ff, int64_t n, float* parts,
                                                   uint32_t* code) {
    __shared__ float red[16];
    const f32x4* r4 = (const f32x4*)fr;
    const f32x4* f4 = (const f32x4*)ff;
    const int64_t n4 = n >> 2, stride = (int64_t)gridDim.x * 256;
    float s1 = 0.f, s2 = 0.f;
    for (int64_t i0 = (int64_t)blockIdx.x * 256 + threadIdx.x; i0 < n4; i0 += 4 * stride) {
        f32x4 rv[4], fv[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int64_t i = i0 + u * stride;
            const int64_t ic = i < n4 ? i : 0;
            rv[u] = r4[ic];
            fv[u] = f4[ic];
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            if (i0 + u * stride < n4) {
                uint32_t cw = 0;  // CODE: 4 bytes, one per element (code_term / code_mask)
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    const float d = fv[u][c] - rv[u][c];
                    s1 += fabsf(rv[u][c] - fv[u][c]);
                    s2 += fabsf(rv[u][c]);
                    cw |= ((d > 0.f ? 1u : (d < 0.f ? 2u : 0u)) | (fv[u][c] > 0.f ? 4u : 0u)) << (8 * c);
                }
                if (CODE) code[i0 + u * stride] = cw;
            }
        }
    }
    s1 = block_sum(s1, red);
    s2 = block_sum(s2, red);
    if (threadIdx.x == 0) {
        parts[2 * blockIdx.x] = s1;
        parts[2 * blockIdx.x + 1] = s2;
    }
}
constexpr int LP = 512;  // partial blocks of the loss reductions
// out[0] (+)= scale * sum(parts[0::stride]) / (stride == 2 ? sum(parts[1::2]) : n)
__global__ __launch_bounds__(256) void loss_finish(const float* parts, int np, int stride, double n,
                                                   float scale, float* out, float* denom, int acc) {
    __shared__ float red[16];
    float a = 0.f, d = 0.f;
    for (int i = threadIdx.x; i < np; i += 256) {
        a += parts[i * stride];
        if (stride == 2) d += parts[i * stride + 1];
    }
    a = block_sum(a, red);
    d = block_sum(d, red);
    if (threadIdx.x == 0) {
        const float den = stride == 2 ? d : (float)n;
        const float v = scale * (a / den);
        out[0] = acc ? out[0] + v : v;
        if (denom) denom[0] = den;
    }
}
// grad of scale * mean(relu(1 + s*x)): scale * s / n where 1 + s*x > 0; g0 = upstream scalar
__global__ void hinge_grad_kernel(const float* x, int64_t n, float s, float scale, const float* g0,
                                  float* dx) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float g = (g0 ? g0[0] : 1.f) * scale * s / (float)n;
    dx[i] = (1.f + s * x[i] > 0.f) ? g : 0.f;
}
// grad wrt ff of scale * sum|fr - ff| / sum|fr| (the reference's l1 / mean|fr| ratio)
__global__ void feat_grad_kernel(const float* fr, const float* ff, int64_t n, float scale,
                                 const float* denom, const float* g0, float* dff) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float g = (g0 ? g0[0] : 1.f) * scale / denom[0];
    const float d = ff[i] - fr[i];
    dff[i] = d > 0.f ? g : (d < 0.f ? -g : 0.f);
}

// ------------------------------------------------------------- single output channel (Co = 1)
// The post conv of each DiscriminatorSTFT (msstftd.py:80-81, 32 -> 1, 3x3) has one output
// channel, so an MFMA tile would idle 31 of its 32 rows. These are VALU kernels with the taps
// unrolled (KT, KF, stride compile-time) and clamped loads, so every lane keeps its KT*KF loads in
// flight; lanes run along the frequency axis (coalesced). Each input element is read KT*KF
// times through L1/L2; the HBM traffic is the algorithmic |x| + |y| (+ |dx|).
constexpr int C1_ROWS = 4;  // fwd: ci groups per block (waves); dgrad: rows per block

// y[b][0][t][fo]: block = 64 output columns x 4 ci groups of one (b, t); the 4 partial sums meet
// in LDS in a fixed order.
template <int KT, int KF, int S>
__global__ __launch_bounds__(256) void c2_co1_fwd(C2Fwd a) {
    const C2Geo g = a.g;
    __shared__ float part[4][64];
    const int lane = threadIdx.x & 63, cg = threadIdx.x >> 6;
    const int plane = g.T2 * g.Fo, p = blockIdx.x * 64 + lane, b = blockIdx.y;
    const int pc = p < plane ? p : plane - 1;
    const int t = pc / g.Fo, fo = pc - t * g.Fo;
    const int64_t xplane = (int64_t)g.T2 * g.Fi;
    const int cper = (g.Ci + 3) >> 2, c0 = cg * cper, c1 = min(g.Ci, c0 + cper);
    const int fb = fo * S - g.pf;
    float acc = 0.f;
    for (int ci = c0; ci < c1; ++ci) {
        const float* xc = a.x + ((int64_t)b * g.Ci + ci) * xplane;
        const float* w = a.wf + ci * KT * KF;
#pragma unroll
        for (int kt = 0; kt < KT; ++kt) {
            const int tr = t + kt * g.dt - g.pt;
            const bool rok = tr >= 0 && tr < g.T2;
            const float* row = xc + (int64_t)(rok ? tr : 0) * g.Fi;
#pragma unroll
            for (int kf = 0; kf < KF; ++kf) {
                const int f = fb + kf;
                const bool ok = rok && f >= 0 && f < g.Fi;
                const float v = row[ok ? f : 0];
                acc = fmaf(w[kt * KF + kf], ok ? v : 0.f, acc);
            }
        }
    }
    part[cg][lane] = acc;
    __syncthreads();
    if (cg == 0 && p < plane) {
        float v = ((part[0][lane] + part[1][lane]) + part[2][lane]) + part[3][lane];
        if (a.bias) v += a.bias[0];
        a.y[(int64_t)b * plane + p] = a.act ? lrelu(v) : v;
    }
}

// dx[b][ci][ti][fi] = sum_{kt,kf} W[ci][kt][kf] * dy'[b][ti - kt*dt + pt][(fi - kf + pf)/S]
// (terms whose output column is fractional or out of range drop), dy' = dy * LeakyReLU'(yact).
// Block = 64 columns x 4 rows of one (b, ci) plane.
// CPT input channels per thread share the KT*KF loads of dy' (blockIdx.y = (b, channel group));
// per channel the taps are summed in the same order as one channel per thread.
template <int KT, int KF, int S, int CPT = 1>
__global__ __launch_bounds__(256) void c2_co1_dgrad(C2Dg a) {
    const C2Geo g = a.g;
    const int xplane = g.T2 * g.Fi, p = blockIdx.x * 256 + threadIdx.x;
    if (p >= xplane) return;
    const int ti = p / g.Fi, fi = p - ti * g.Fi;
    const int groups = g.Ci / CPT, b = blockIdx.y / groups, ci0 = (blockIdx.y - b * groups) * CPT;
    const int64_t plane = (int64_t)g.T2 * g.Fo;
    const float* dyb = a.dy + (int64_t)b * plane;
    const float* yab = a.yact ? a.yact + (int64_t)b * plane : dyb;
    const int M = g.Ci * S;
    float dv[KT * KF];
#pragma unroll
    for (int kt = 0; kt < KT; ++kt) {
        const int to = ti - kt * g.dt + g.pt;
        const bool rok = to >= 0 && to < g.T2;
#pragma unroll
        for (int kf = 0; kf < KF; ++kf) {
            const int fs = fi - kf + g.pf;
            const int fo = fs / S;  // S is 1 or 2: a shift
            const bool ok = rok && fs >= 0 && (S == 1 || fs % S == 0) && fo < g.Fo;
            const int64_t o = ok ? (int64_t)to * g.Fo + fo : 0;
            float d = dyb[o];
            if (a.yact) d *= lrelu_grad(yab[o]);
            dv[kt * KF + kf] = ok ? d : 0.f;
        }
    }
    const float fc = feat_coef(a);
#pragma unroll
    for (int c = 0; c < CPT; ++c) {
        const int ci = ci0 + c;
        float acc = 0.f;
#pragma unroll
        for (int kt = 0; kt < KT; ++kt)
#pragma unroll
            for (int kf = 0; kf < KF; ++kf)
                acc = fmaf(a.wp[(kt * a.J + kf / S) * M + ci * S + kf % S], dv[kt * KF + kf], acc);
        const int64_t i = ((int64_t)b * g.Ci + ci) * xplane + p;
        if (a.ffr) acc += feat_term(a, fc, i);
        if (a.xact) acc *= lrelu_grad(a.xact[i]);
        a.dx[i] = a.accumulate ? a.dx[i] + acc : acc;
    }
}

// ws[s][0][n], s = (b, row chunk): n = (ci*KT + kt)*KF + kf -> sum over the chunk's output
// positions of dy'[b][to][fo] * x[b][ci][to + kt*dt - pt][fo*S + kf - pf]; n = Ci*KT*KF -> the
// chunk's sum of dy' (bias). Block = 4 waves (one ci each, blockIdx.z picks the ci group) x 64
// lanes along fo; per-lane partials are summed over the wave in a fixed order through LDS.
template <int KT, int KF, int S>
__global__ __launch_bounds__(256) void c2_co1_wgrad(C2Wg a) {
    constexpr int K = KT * KF;
    const C2Geo g = a.g;
    __shared__ float red[4][K + 1][65];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int rc = blockIdx.x, b = blockIdx.y, ci = blockIdx.z * 4 + wave;
    const int N = g.Ci * K + 1, rows = a.BT;
    const int to0 = rc * rows, to1 = min(g.T2, to0 + rows);
    const int64_t plane = (int64_t)g.T2 * g.Fo, xplane = (int64_t)g.T2 * g.Fi;
    const float* dyb = a.dy + (int64_t)b * plane;
    const float* yab = a.yact ? a.yact + (int64_t)b * plane : dyb;
    const float* xc = a.x + ((int64_t)b * g.Ci + (ci < g.Ci ? ci : 0)) * xplane;
    float acc[K], bacc = 0.f;
#pragma unroll
    for (int k = 0; k < K; ++k) acc[k] = 0.f;
    const int p1 = to1 * g.Fo;
    for (int base = to0 * g.Fo; base < p1; base += 64) {
        {
            const int p = base + lane;
            const bool cok = p < p1;
            const int pc = cok ? p : p1 - 1;
            const int to = pc / g.Fo, fo = pc - to * g.Fo;
            const int64_t o = pc;
            float d = dyb[o];
            if (a.yact) d *= lrelu_grad(yab[o]);
            d = cok ? d : 0.f;
            bacc += d;
#pragma unroll
            for (int kt = 0; kt < KT; ++kt) {
                const int tr = to + kt * g.dt - g.pt;
                const bool rok = tr >= 0 && tr < g.T2;
                const float* row = xc + (int64_t)(rok ? tr : 0) * g.Fi;
#pragma unroll
                for (int kf = 0; kf < KF; ++kf) {
                    const int f = fo * S + kf - g.pf;
                    const bool ok = rok && f >= 0 && f < g.Fi;
                    const float v = row[ok ? f : 0];
                    acc[kt * KF + kf] = fmaf(d, ok ? v : 0.f, acc[kt * KF + kf]);
                }
            }
        }
    }
#pragma unroll
    for (int k = 0; k < K; ++k) red[wave][k][lane] = acc[k];
    red[wave][K][lane] = bacc;
    __syncthreads();
    if (lane <= K) {
        float v = 0.f;
        for (int l = 0; l < 64; ++l) v += red[wave][lane][l];
        float* out = a.ws + ((int64_t)b * gridDim.x + rc) * N;
        if (lane < K && ci < g.Ci) out[ci * K + lane] = v;
        if (lane == K && blockIdx.z == 0 && wave == 0) out[N - 1] = v;
    }
}

// ---------------------------------------------------------------------------- planning
static int c2_rows(int BN, int len) { return (len + BN - 2) / len + 1; }

template <int BM, int BN, int WM, int WN, int KFC = 0>
int launch_fwd(C2Fwd a, hipStream_t st) {
    const size_t lds = ((size_t)a.CK * a.NR * a.RL + (size_t)a.g.KF * a.CK * BM +
                        (size_t)2 * a.g.Ci * a.g.KT * a.NR + 2) * sizeof(float);
    dim3 grid((unsigned)cdiv((int64_t)a.g.T2 * a.g.Fo, BN), (unsigned)cdiv(a.g.Co, BM), (unsigned)a.g.B);
    hipLaunchKernelGGL((c2_fwd_kernel<BM, BN, WM, WN, KFC>), grid, dim3(NT), lds, st, a);
    ENCX_CHECK_LAUNCH();
    return 0;
}
template <int BM, int BN, int WM, int WN, int JC = 0>
int launch_dgrad(C2Dg a, hipStream_t st) {
    const size_t lds = ((size_t)a.CK * a.NR * a.RL + (size_t)a.J * a.CK * BM +
                        (size_t)2 * a.g.Co * a.g.KT * a.NR + 2) * sizeof(float);
    dim3 grid((unsigned)cdiv((int64_t)a.g.T2 * a.U, BN), (unsigned)cdiv(a.g.Ci * a.g.sf, BM), (unsigned)a.g.B);
    hipLaunchKernelGGL((c2_dgrad_kernel<BM, BN, WM, WN, JC>), grid, dim3(NT), lds, st, a);
    ENCX_CHECK_LAUNCH();
    return 0;
}

// channels per LDS chunk: even, <= VC rounded up to even, LDS <= budget floats
static int c2_ck(int VC, int per_ch, int budget = 12288);

// planned launches: window geometry and LDS chunking for the column tile BN
template <int BM, int BN, int WM, int WN, int KFC = 0>
int run_fwd(C2Fwd a, hipStream_t st, int budget = 12288) {
    a.NR = c2_rows(BN, a.g.Fo);
    a.RL = (min(BN, a.g.Fo) - 1) * a.g.sf + a.g.KF;
    a.CK = c2_ck(a.g.Ci * a.g.KT, a.NR * a.RL + a.g.KF * BM, budget);
    return launch_fwd<BM, BN, WM, WN, KFC>(a, st);
}
template <int BM, int BN, int WM, int WN, int JC = 0>
int run_dgrad(C2Dg a, hipStream_t st, int budget = 12288) {
    a.J = (int)cdiv(a.g.KF, a.g.sf);
    a.U = (a.g.Fi - 1 + a.g.pf) / a.g.sf + 1;
    a.NR = c2_rows(BN, a.U);
    a.RL = min(BN, a.U) - 1 + a.J;
    a.CK = c2_ck(a.g.Co * a.g.KT, a.NR * a.RL + a.J * BM, budget);
    return launch_dgrad<BM, BN, WM, WN, JC>(a, st);
}

template <int BN, int KFC, int CK, int MX>
int run_fwdp(C2Fwd a, hipStream_t st) {
    a.NR = c2_rows(BN, a.g.Fo);
    a.RL = (min(BN, a.g.Fo) - 1) * a.g.sf + a.g.KF;
    a.CK = CK;
    if (a.g.KF != KFC || (int64_t)CK * a.NR * a.RL > (int64_t)MX * NT) return ENCX_EINVAL;
    const size_t lds = ((size_t)CK * a.NR * a.RL + (size_t)KFC * CK * 32 + (size_t)2 * a.g.Ci * a.g.KT * a.NR) *
                       sizeof(float);
    dim3 grid((unsigned)cdiv((int64_t)a.g.T2 * a.g.Fo, BN), (unsigned)cdiv(a.g.Co, 32), (unsigned)a.g.B);
    hipLaunchKernelGGL((c2_fwdp_kernel<BN, KFC, CK, MX>), grid, dim3(NT), lds, st, a);
    ENCX_CHECK_LAUNCH();
    return 0;
}

template <int BN, int KFC, int CK>
int run_fwdv(C2Fwd a, hipStream_t st) {
    a.NR = c2_rows(BN, a.g.Fo);
    a.RL = (min(BN, a.g.Fo) - 1) * a.g.sf + a.g.KF;
    a.CK = CK;
    if (a.g.KF != KFC) return ENCX_EINVAL;
    const int RLp = (a.RL + 3) & ~3;
    const size_t lds = ((size_t)CK * a.NR * RLp + (size_t)KFC * CK * 32 + (size_t)2 * a.g.Ci * a.g.KT * a.NR) *
                       sizeof(float);
    dim3 grid((unsigned)cdiv((int64_t)a.g.T2 * a.g.Fo, BN), (unsigned)cdiv(a.g.Co, 32), (unsigned)a.g.B);
    hipLaunchKernelGGL((c2_fwdv_kernel<BN, KFC, CK>), grid, dim3(NT), lds, st, a);
    ENCX_CHECK_LAUNCH();
    return 0;
}

// CK for c2_fwdq_kernel: the largest even combo count (<= CKM, <= VC rounded up to even) whose
// window fits MQ quads per thread; 0 when not even 2 combos fit
static int fwdq_ck(int VC, int NR, int RL, int MQ, int CKM) {
    const int quads = NR * (((RL + 3) & ~3) >> 2);
    int ck = MQ * NT / quads;
    ck = min(ck, CKM);
    ck = min(ck, (VC + 1) & ~1);
    ck &= ~1;
    return ck;
}
template <int BN, int KFC, int MQ, int CKM, int DBG = 0>
int run_fwdq(C2Fwd a, hipStream_t st) {
    a.NR = c2_rows(BN, a.g.Fo);
    a.RL = (min(BN, a.g.Fo) - 1) * a.g.sf + a.g.KF;
    a.CK = fwdq_ck(a.g.Ci * a.g.KT, a.NR, a.RL, MQ, CKM);
    if (a.g.KF != KFC || a.CK < 2 || a.g.Fi < 4) return ENCX_EINVAL;
    const int RLp = (a.RL + 3) & ~3;
    const size_t lds = ((size_t)a.CK * a.NR * RLp + (size_t)KFC * a.CK * 32 + (size_t)2 * a.g.Ci * a.g.KT * a.NR) *
                       sizeof(float);
    dim3 grid((unsigned)cdiv((int64_t)a.g.T2 * a.g.Fo, BN), (unsigned)cdiv(a.g.Co, 32), (unsigned)a.g.B);
    hipLaunchKernelGGL((c2_fwdq_kernel<BN, KFC, MQ, CKM, DBG>), grid, dim3(NT), lds, st, a);
    ENCX_CHECK_LAUNCH();
    return 0;
}

// register-window backward-data (c2_dgrad_rw_kernel): 3x9 stride 2 (M = 64) and 3x3 stride 1
// (M = 32) layers with Co % 4 == 0; the polyphase weights in LDS
static bool dgr_ok(const C2Geo& g) {
    if ((g.Co & 3) || g.KT != 3 || g.Fi < 4 || g.Fo < 4) return false;
    if (!((g.KF == 9 && g.sf == 2 && g.Ci == 32) || (g.KF == 3 && g.sf == 1 && g.Ci == 32))) return false;
    if ((int64_t)g.B * g.Co * g.T2 * g.Fo >= (1ll << 31) - 64) return false;
    const int J = (g.KF + g.sf - 1) / g.sf;
    return (size_t)g.Co * 3 * J * g.Ci * g.sf * sizeof(float) <= 150 * 1024;
}
template <int TM>
static void launch_dgrad_rw(const C2DgR& R, int grid, size_t lds, hipStream_t st) {
    constexpr int NWV = 8;
    const bool ym = R.d.yact != nullptr;
    if (R.d.g.KF == 9) {
        if (ym) hipLaunchKernelGGL((c2_dgrad_rw_kernel<5, 2, 2, 2, true, NWV, TM>), dim3(grid), dim3(NWV * 64), lds, st, R);
        else hipLaunchKernelGGL((c2_dgrad_rw_kernel<5, 2, 2, 2, false, NWV, TM>), dim3(grid), dim3(NWV * 64), lds, st, R);
    } else {
        if (ym) hipLaunchKernelGGL((c2_dgrad_rw_kernel<3, 1, 1, 2, true, NWV, 1>), dim3(grid), dim3(NWV * 64), lds, st, R);
        else hipLaunchKernelGGL((c2_dgrad_rw_kernel<3, 1, 1, 2, false, NWV, 1>), dim3(grid), dim3(NWV * 64), lds, st, R);
    }
}
// 8 waves per workgroup, items of both row tiles of the 3x9 layers (TM = 2). Measured and
// dropped (round 5): a half-full last round of items handed to a second launch as one-row-tile
// items (TM = 1, twice the items at half the work): 799.0 vs 802.0 audio-s/s.
static int run_dgrad_rw(const C2Dg& d, int wgs, hipStream_t st) {
    if (!dgr_ok(d.g)) return ENCX_EINVAL;
    constexpr int NWV = 8;
    const C2Geo& g = d.g;
    C2DgR R{d, 0, 0};
    R.d.U = (g.Fi - 1 + g.pf) / g.sf + 1;
    R.U4 = (int)cdiv(R.d.U, 4);
    const int tiles = (int)cdiv((int64_t)g.B * g.T2 * R.U4, 32);
    const int J = (g.KF + g.sf - 1) / g.sf;
    const size_t lds = (size_t)g.Co * 3 * J * g.Ci * g.sf * sizeof(float);
    const int grid = (int)min((int64_t)wgs, cdiv((int64_t)tiles, NWV));
    R.tiles = tiles;
    launch_dgrad_rw<2>(R, grid, lds, st);
    ENCX_CHECK_LAUNCH();
    return 0;
}

// register-window forward (c2_fwd_rw_kernel): 32-wide output-channel tile, even Ci, KT <= 3,
// the layer's weights in LDS (<= 128 KB)
static bool fwr_ok(const C2Geo& g) {
    if (g.Co > 32 || (g.Ci & 1) || g.KT != 3 || g.Fo < 1 || g.Fi < 4) return false;
    if ((int64_t)g.B * g.Ci * g.T2 * g.Fi >= (1ll << 31) || (int64_t)g.B * g.T2 * cdiv(g.Fo, 4) >= (1ll << 31) - 64)
        return false;
    if (!((g.KF == 9 && (g.sf == 2 || g.sf == 1)) || (g.KF == 3 && g.sf == 1))) return false;
    return (size_t)g.Ci * g.KT * g.KF * 32 * sizeof(float) <= 128 * 1024;
}
// wgs: workgroups (one per CU holds the layer's weights) of 8 waves
static int run_fwd_rw(const C2Fwd& f, int wgs, hipStream_t st) {
    if (!fwr_ok(f.g)) return ENCX_EINVAL;
    constexpr int NWV = 8;
    const C2Geo& g = f.g;
    C2FwdR a{g, f.x, f.wf, f.bias, f.y, f.act, (int)cdiv(g.Fo, 4), 0};
    a.tiles = (int)cdiv((int64_t)g.B * g.T2 * a.F4, 32);
    const size_t lds = ((size_t)g.Ci * g.KT * g.KF * 32 + 32) * sizeof(float);
    const int grid = (int)min((int64_t)wgs, cdiv(a.tiles, NWV));
    if (g.KF == 9 && g.sf == 2)
        hipLaunchKernelGGL((c2_fwd_rw_kernel<9, 2, 4, NWV>), dim3(grid), dim3(NWV * 64), lds, st, a);
    else if (g.KF == 9)
        hipLaunchKernelGGL((c2_fwd_rw_kernel<9, 1, 3, NWV>), dim3(grid), dim3(NWV * 64), lds, st, a);
    else
        hipLaunchKernelGGL((c2_fwd_rw_kernel<3, 1, 2, NWV>), dim3(grid), dim3(NWV * 64), lds, st, a);
    ENCX_CHECK_LAUNCH();
    return 0;
}
template <int BN, int KFC, int MQ, int CKM, int OCC = 1>
int run_fwdr(C2Fwd a, hipStream_t st) {
    a.NR = c2_rows(BN, a.g.Fo);
    a.RL = (min(BN, a.g.Fo) - 1) * a.g.sf + a.g.KF + 3;  // + alignment slack of the column base
    a.CK = fwdq_ck(a.g.Ci * a.g.KT, a.NR, a.RL, MQ, CKM);
    if (a.g.KF != KFC || a.CK < 2 || a.g.Fi < 4 || a.g.pf > 4) return ENCX_EINVAL;
    const int RLp = (a.RL + 3) & ~3;
    const size_t lds = ((size_t)a.CK * a.NR * RLp + (size_t)KFC * a.CK * 32 + (size_t)2 * a.g.Ci * a.g.KT * a.NR) *
                       sizeof(float);
    dim3 grid((unsigned)cdiv((int64_t)a.g.T2 * a.g.Fo, BN), (unsigned)cdiv(a.g.Co, 32), (unsigned)a.g.B);
    hipLaunchKernelGGL((c2_fwdr_kernel<BN, KFC, MQ, CKM, OCC>), grid, dim3(NT), lds, st, a);
    ENCX_CHECK_LAUNCH();
    return 0;
}

template <int TM, int BN, int JC, int MQ, int CKM, int OCC = 1, int DB = 0>
int run_dgradr(C2Dg a, hipStream_t st) {
    a.J = (int)cdiv(a.g.KF, a.g.sf);
    a.U = (a.g.Fi - 1 + a.g.pf) / a.g.sf + 1;
    a.NR = c2_rows(BN, a.U);
    a.RL = min(BN, a.U) - 1 + a.J + 3;
    a.CK = fwdq_ck(a.g.Co * a.g.KT, a.NR, a.RL, MQ, CKM);
    if (a.J != JC || a.CK < 2 || a.g.Fo < 4 || JC > 5 || a.g.Ci * a.g.sf > 32 * TM) return ENCX_EINVAL;
    const int RLp = (a.RL + 3) & ~3;
    const size_t lds = ((size_t)(DB ? 2 : 1) * ((size_t)a.CK * a.NR * RLp + (size_t)JC * a.CK * 32 * TM) +
                        (size_t)2 * a.g.Co * a.g.KT * a.NR) * sizeof(float);
    dim3 grid((unsigned)cdiv((int64_t)a.g.T2 * a.U, BN), 1, (unsigned)a.g.B);
    if (a.yact) hipLaunchKernelGGL((c2_dgradr_kernel<TM, BN, JC, MQ, CKM, OCC, DB, true>), grid, dim3(NT), lds, st, a);
    else hipLaunchKernelGGL((c2_dgradr_kernel<TM, BN, JC, MQ, CKM, OCC, DB, false>), grid, dim3(NT), lds, st, a);
    ENCX_CHECK_LAUNCH();
    return 0;
}

// weight grad, column-group form (c2_wgrad2_kernel)
struct WgPlan3 {
    int NR, RL, GC, chunks, items, splits, per_split;
    size_t lds;
};
static WgPlan3 plan_wg3(const C2Geo& g, int GC, int target = 1024) {
    WgPlan3 p;
    const int P = W2_P, Nall = g.T2 * g.Fo;
    p.GC = GC;
    p.NR = c2_rows(P, g.Fo);
    p.RL = (min(P, g.Fo) - 1) * g.sf + g.KF;
    p.chunks = (int)cdiv(Nall, P);
    p.items = g.B * p.chunks;
    const int groups = (int)cdiv(g.Ci * g.KT, GC);
    int sp = (int)cdiv(target, groups);
    if (sp > p.items) sp = p.items;
    p.per_split = (int)cdiv(p.items, sp);
    p.splits = (int)cdiv(p.items, p.per_split);
    p.lds = ((size_t)4 * GC * p.NR + (size_t)P * 33 + P + (size_t)GC * p.NR * p.RL) * sizeof(float);
    return p;
}
// combos per workgroup for the column-group wgrad, 0 when the layer does not fit its tiling
static int wg3_gc(const C2Geo& g) {
    const int VC = g.Ci * g.KT;
    if (g.Co > 32) return 0;
    if (g.KF == 9 && VC % 32 == 0) return 32;   // 288 columns = 3 waves x 3 tiles
    if (g.KF == 3 && VC % 96 == 0) return 96;   // 288 columns
    return 0;
}
template <int KF, int NTW, int NW>
int run_wgrad2(const C2Geo& g, const float* dy, const float* yact, const float* x, float* ws, const WgPlan3& p,
               hipStream_t st) {
    C2Wg2 a{g, dy, yact, x, ws, p.NR, p.RL, p.GC, p.items, p.per_split, p.chunks};
    dim3 grid((unsigned)cdiv(g.Ci * g.KT, p.GC), (unsigned)p.splits);
    hipLaunchKernelGGL((c2_wgrad2_kernel<KF, NTW, NW>), grid, dim3(NW * 64), p.lds, st, a);
    ENCX_CHECK_LAUNCH();
    return 0;
}

static WgPlan3 plan_wg3r(const C2Geo& g, int GC, int target = 1024) {
    WgPlan3 p;
    const int P = W3_P, Nall = g.T2 * g.Fo;
    p.GC = GC;
    p.NR = c2_rows(P, g.Fo);
    p.RL = (min(P, g.Fo) - 1) * g.sf + g.KF + 3;
    p.chunks = (int)cdiv(Nall, P);
    p.items = g.B * p.chunks;
    const int groups = (int)cdiv(g.Ci * g.KT, GC);
    int sp = (int)cdiv(target, groups);
    if (sp > p.items) sp = p.items;
    p.per_split = (int)cdiv(p.items, sp);
    p.splits = (int)cdiv(p.items, p.per_split);
    // rtab int4 [GC*NR] + Ls [P][33] + poff [P]: P*33 + P = 34*64 floats keeps Rs 16-byte aligned
    p.lds = ((size_t)4 * GC * p.NR + (size_t)P * 33 + P + (size_t)GC * p.NR * (((p.RL + 3) & ~3))) * sizeof(float);
    return p;
}
// workgroups per launch: 768 = 3 combo groups x 256 splits, whole rounds over the 256 CUs
// (tools/mb/c2_mb sweep: 768 within 2 % of the best target on all nine strided layers; targets
// that leave a partial last round, 512 = 3 x 171, lose up to 35 %)
static int wg3r_target(const C2Geo& g) {
    (void)g;
    return 768;
}
// the layers c2_wgrad3_kernel<9, 1, 9, *, 1> serves: 3x9 taps, 32-combo groups, <= 32 rows
static bool wg3r_ok(const C2Geo& g) {
    if (g.KF != 9 || (g.Ci * g.KT) % 32 != 0 || g.Co > 32 || g.Fi < 4 || g.pf > 4) return false;
    const WgPlan3 q = plan_wg3r(g, 32, 512);
    return q.GC * q.NR * (((q.RL + 3) & ~3) >> 2) <= 4 * 9 * 64;
}
// the narrow first layer (Ci*KT <= 14 combos, 3x9 taps): all combos in one column group of
// 2 or 4 waves (tools/mb/c2_mb: 1536 workgroups, 4 waves/SIMD cap; 1.5x the generic kernel)
static bool wg3n_ok(const C2Geo& g) {
    return g.KF == 9 && g.Ci * g.KT <= 14 && g.Co <= 32 && g.Fi >= 4 && g.pf <= 4;
}
static WgPlan3 plan_wg3n(const C2Geo& g) { return plan_wg3r(g, g.Ci * g.KT, 1536); }
template <int KF, int NTW, int NW, int MQ, int ML, int OCC = 1, int PF = 0>
int run_wgrad3(const C2Geo& g, const float* dy, const float* yact, const float* x, float* ws, const WgPlan3& p,
               hipStream_t st) {
    const int quads = p.GC * p.NR * (((p.RL + 3) & ~3) >> 2);
    if (quads > MQ * NW * 64 || 32 * (W3_P / 4) > ML * NW * 64 || g.Co > 32 || g.Fi < 4 || g.pf > 4) return ENCX_EINVAL;
    C2Wg3 a{g, dy, yact, x, ws, p.NR, p.RL, p.GC, p.items, p.per_split, p.chunks};
    dim3 grid((unsigned)cdiv(g.Ci * g.KT, p.GC), (unsigned)p.splits);
    if (yact) hipLaunchKernelGGL((c2_wgrad3_kernel<KF, NTW, NW, MQ, ML, OCC, PF, true>), grid, dim3(NW * 64), p.lds, st, a);
    else hipLaunchKernelGGL((c2_wgrad3_kernel<KF, NTW, NW, MQ, ML, OCC, PF, false>), grid, dim3(NW * 64), p.lds, st, a);
    ENCX_CHECK_LAUNCH();
    return 0;
}


// register-window weight grad (c2_wgrad_rw_kernel): 3x9 stride-2 and 3x3 stride-1 layers with
// 32-channel blocks of input channels and <= 32 output channels
struct WgPlanR {
    int NC, items, ktg, cib, splits, per_split, SW, NCS;
};
static bool wgr_ok(const C2Geo& g) {
    if (g.Co > 32 || g.Ci < 16 || g.KT != 3 || g.Fo < 4 || g.Fi < 4) return false;
    if ((int64_t)g.B * g.Ci * g.T2 * g.Fi >= (1ll << 31) - 64 || (int64_t)g.B * g.Co * g.T2 * g.Fo >= (1ll << 31) - 64)
        return false;
    return (g.KF == 9 && g.sf == 2) || (g.KF == 3 && g.sf == 1);
}
// waves: the one-wave form's wave count; wgs > 0: the 8-wave workgroup form with at most that
// many workgroups (one per CU: its 144 KB of reduction LDS), whole rounds over the CUs
static WgPlanR plan_wgr(const C2Geo& g, int waves = 2048, int wgs = 0) {
    WgPlanR p;
    p.NC = (int)cdiv(g.Fo, 8);
    p.items = g.B * g.T2 * p.NC;
    // strip width: NC itself up to 17 chunks, else its largest divisor <= 16 (65 -> 13, 33 -> 11)
    p.SW = p.NC;
    if (p.NC > 17)
        for (int w = 16; w >= 1; --w)
            if (p.NC % w == 0) {
                p.SW = w;
                break;
            }
    p.NCS = p.NC / p.SW;
    p.ktg = g.KF == 9 ? g.KT : 1;
    p.cib = (int)cdiv(g.Ci, 32);
    const int per = p.ktg * p.cib;
    int sp = wgs > 0 ? max(1, wgs / per) : (int)cdiv(waves, per);
    if (sp > p.items) sp = p.items;
    p.per_split = (int)cdiv(p.items, sp);
    p.splits = (int)cdiv(p.items, p.per_split);
    return p;
}
static int64_t wgr_slab(const C2Geo& g, const WgPlanR& p) {  // task-major slab floats (8-wave form)
    return (int64_t)p.ktg * p.cib * 32 * 32 * 9 + 32;  // NTAP = 9 taps per task (1 x 9 or 3 x 3)
}
static int run_wgrad_rw(const C2Geo& g, const float* dy, const float* yact, const float* x, float* ws,
                        const WgPlanR& p, hipStream_t st, bool wg8 = false) {
    if (!wgr_ok(g)) return ENCX_EINVAL;
    C2WgR a{g, dy, yact, x, ws, p.NC, p.items, p.per_split, p.ktg, p.cib, p.SW, p.NCS};
    const dim3 grid((unsigned)(p.splits * p.ktg * p.cib));
    if (wg8) {
        const size_t lds = (4 * 32 * 32 * 9 + 8 * 32) * sizeof(float);
        if (g.KF == 9) {
            if (yact) hipLaunchKernelGGL((c2_wgrad_rw_kernel<9, 2, 1, 4, true, 8>), grid, dim3(512), lds, st, a);
            else hipLaunchKernelGGL((c2_wgrad_rw_kernel<9, 2, 1, 4, false, 8>), grid, dim3(512), lds, st, a);
        } else {
            if (yact) hipLaunchKernelGGL((c2_wgrad_rw_kernel<3, 1, 3, 2, true, 8>), grid, dim3(512), lds, st, a);
            else hipLaunchKernelGGL((c2_wgrad_rw_kernel<3, 1, 3, 2, false, 8>), grid, dim3(512), lds, st, a);
        }
        ENCX_CHECK_LAUNCH();
        return 0;
    }
    const dim3 blk(64);
    if (g.KF == 9) {
        if (yact) hipLaunchKernelGGL((c2_wgrad_rw_kernel<9, 2, 1, 4, true>), grid, blk, 0, st, a);
        else hipLaunchKernelGGL((c2_wgrad_rw_kernel<9, 2, 1, 4, false>), grid, blk, 0, st, a);
    } else {
        if (yact) hipLaunchKernelGGL((c2_wgrad_rw_kernel<3, 1, 3, 2, true>), grid, blk, 0, st, a);
        else hipLaunchKernelGGL((c2_wgrad_rw_kernel<3, 1, 3, 2, false>), grid, blk, 0, st, a);
    }
    ENCX_CHECK_LAUNCH();
    return 0;
}

static int c2_ck(int VC, int per_ch, int budget) {
    int ck = budget / per_ch;
    if (ck > 32) ck = 32;
    int vce = (VC + 1) & ~1;
    if (ck > vce) ck = vce;
    ck &= ~1;
    if (ck < 2) ck = 2;
    // prefer an exact (even) divisor of VC near ck
    for (int c = ck; c >= 2; c -= 2)
        if (VC % c == 0 && c * 2 >= ck) return c;
    return ck;
}

struct WgPlan2 {
    int BT, NR, RL, NCmax, chunks, items, splits, per_split, narrow;
};
static WgPlan2 plan_wg2(const C2Geo& g) {
    WgPlan2 p;
    p.BT = WG_BT;
    const int Nall = g.T2 * g.Fo;
    p.NR = c2_rows(p.BT, g.Fo);
    p.RL = (min(p.BT, g.Fo) - 1) * g.sf + g.KF;
    const int N = g.Ci * g.KT * g.KF + 1;
    p.narrow = N <= 64;
    const int BN = p.narrow ? 64 : 128;
    p.NCmax = (BN - 1) / g.KF + 2;
    p.chunks = (int)cdiv(Nall, p.BT);
    p.items = g.B * p.chunks;
    const int tiles = (int)(cdiv(N, BN) * cdiv(g.Co, 32));
    int sp = (int)cdiv(1024, tiles);
    if (sp > p.items) sp = p.items;
    p.per_split = (int)cdiv(p.items, sp);
    p.splits = (int)cdiv(p.items, p.per_split);
    return p;
}

// Co = 1 wgrad: splits = (b, row chunk), about 512 of them
struct WgPlanC1 {
    int rows, chunks, splits;
};
static bool co1_ok(const C2Geo& g) { return g.Co == 1 && g.KT == 3 && g.KF == 3 && (g.sf == 1 || g.sf == 2); }
static WgPlanC1 plan_co1(const C2Geo& g) {
    WgPlanC1 p;
    const int per_b = max(1, 512 / g.B);
    p.rows = (int)cdiv(g.T2, per_b);
    p.chunks = (int)cdiv(g.T2, p.rows);
    p.splits = g.B * p.chunks;
    return p;
}

static bool geo_ok(const C2Geo& g) {
    return g.B > 0 && g.Ci > 0 && g.T2 > 0 && g.Fi > 0 && g.Co > 0 && g.Fo > 0 && g.KT > 0 && g.KF > 0 &&
           g.sf > 0 && g.dt > 0 && g.pt >= 0 && g.pf >= 0 &&
           g.Fo == (g.Fi + 2 * g.pf - g.KF) / g.sf + 1 && g.T2 + 2 * g.pt - g.dt * (g.KT - 1) == g.T2;
}

}  // namespace

extern "C" {

/* NormConv2d geometry as used by DiscriminatorSTFT (msstftd.py:67-84): input [B][Ci][T2][Fi]
 * (time frames x freq bins), kernel (KT, KF), stride (1, sf), dilation (dt, 1), zero padding
 * (pt, pf) with T2 preserved; Fo = (Fi + 2 pf - KF)/sf + 1. */
int encx_conv2d_wpoly(const float* wf, float* wp, int64_t Co, int64_t Ci, int64_t KT, int64_t KF, int64_t sf,
                      encx_stream_t stream) {
    ENCX_REQUIRE(wf && wp && Co > 0 && Ci > 0 && KT > 0 && KF > 0 && sf > 0);
    const int J = (int)cdiv(KF, sf);
    const int64_t total = Co * KT * J * Ci * sf;
    hipLaunchKernelGGL(c2_wpoly_kernel, dim3((unsigned)cdiv(total, 256)), dim3(256), 0, (hipStream_t)stream, wf,
                       wp, (int)Co, (int)Ci, (int)KT, (int)KF, (int)sf, J);
    ENCX_CHECK_LAUNCH();
    return 0;
}

// Register-window or tiled kernel for a layer. The register-window kernels hand whole 128-position
// items to SIMDs (rw_first_slot), so their time follows ceil(items / SIMDs) item rounds; the tiled
// kernels' time follows the positions. Per round / per 128 x SIMDs positions, measured on the
// config-3 layers (tools/mb/c2_mb, profiles/r03/mb_rw.md): forward 66 vs 87 us, bwd-data 78 vs 92
// us -- so the register-window form loses on layers whose last round is mostly idle (Fo 65 at
// T2 90, Fo 65 at T2 184) and wins everywhere else. `ratio` = tiled / register-window cost.
static int g_c2_select = [] {  // encx_conv2d_select; ENCX_C2 sets the initial mode
    const char* v = getenv("ENCX_C2");
    return v ? atoi(v) : 0;
}();
static bool rw_pays(int64_t items, int64_t positions, double ratio) {
    if (g_c2_select != 0) return g_c2_select == 1;
    static const int simds = [] {
        int cus = 0;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0) != hipSuccess || cus <= 0) cus = 256;
        return 4 * cus;
    }();
    const double rounds = std::ceil((double)items / simds), tiled = (double)positions / (128.0 * simds);
    return rounds < ratio * tiled;
}

int encx_conv2d_select(int mode) {
    const int prev = g_c2_select;
    if (mode >= 0 && mode <= 2) g_c2_select = mode;
    return prev;
}

int encx_conv2d_fwd(const float* x, const float* wf, const float* bias, float* y, int64_t B, int64_t Ci,
                    int64_t T2, int64_t Fi, int64_t Co, int64_t Fo, int64_t KT, int64_t KF, int64_t sf,
                    int64_t dt, int64_t pt, int64_t pf, int act, encx_stream_t stream) {
    ENCX_REQUIRE(x && wf && y);
    C2Geo g{(int)B, (int)Ci, (int)T2, (int)Fi, (int)Co, (int)Fo, (int)KT, (int)KF, (int)sf, (int)dt, (int)pt, (int)pf};
    ENCX_REQUIRE(geo_ok(g));
    hipStream_t st = (hipStream_t)stream;
    encx_prof_scope ps(st, 2.0 * B * Co * T2 * Fo * Ci * KT * KF, 4.0 * (B * Ci * T2 * Fi + B * Co * T2 * Fo), "c2_fwd");
    ps.tag(" %ldx%ld %ldx%ld s%ld T%ld F%ld", (long)Ci, (long)Co, (long)KT, (long)KF, (long)sf, (long)T2, (long)Fo);
    C2Fwd a{g, x, wf, bias, y, act, 0, 0, 0};
    // register-window form (c2_fwd_rw_kernel); option FWR = workgroups (0: off)
    const int fw_wgs = (int)encx_opt(OPT_FWR);
    if (fw_wgs > 0 && fwr_ok(g) &&
        ((Ci * KT < 16 && g_c2_select != 2) || rw_pays(cdiv(B * T2 * cdiv(Fo, 4), 32), B * T2 * Fo, 87.0 / 66.0)) &&
        run_fwd_rw(a, fw_wgs, st) == 0)
        return 0;
    if (Co == 1 && KT == 3 && KF == 3 && (sf == 1 || sf == 2)) {
        dim3 grid((unsigned)cdiv(T2 * Fo, 64), (unsigned)B);
        if (sf == 1) hipLaunchKernelGGL((c2_co1_fwd<3, 3, 1>), grid, dim3(256), 0, st, a);
        else hipLaunchKernelGGL((c2_co1_fwd<3, 3, 2>), grid, dim3(256), 0, st, a);
        ENCX_CHECK_LAUNCH();
        return 0;
    }
    // column-aligned, register-pipelined staging (c2_fwdr_kernel) for the 32-channel layers; the
    // 2-channel first layer (K = 54) keeps the round-1 kernel, which is faster there
    if (Co <= 32 && Ci * KT >= 16) {
        if (KF == 9 && run_fwdr<256, 9, 6, 16>(a, st) == 0) return 0;
        if (KF == 3 && run_fwdr<256, 3, 6, 32>(a, st) == 0) return 0;
    }
    constexpr int BN = 128;
    a.NR = c2_rows(BN, (int)Fo);
    a.RL = (min(BN, (int)Fo) - 1) * (int)sf + (int)KF;
    a.CK = c2_ck((int)(Ci * KT), a.NR * a.RL + (int)KF * 32);
    if (Co <= 32) return launch_fwd<32, 128, 1, 4>(a, st);
    a.CK = c2_ck((int)(Ci * KT), a.NR * a.RL + (int)KF * 64);
    return launch_fwd<64, 128, 2, 2>(a, st);
}

int encx_conv2d_bwd_data(const float* dy, const float* yact, const float* wp, const float* xact, float* dx,
                         int accumulate, int64_t B, int64_t Ci, int64_t T2, int64_t Fi, int64_t Co, int64_t Fo,
                         int64_t KT, int64_t KF, int64_t sf, int64_t dt, int64_t pt, int64_t pf,
                         encx_stream_t stream) {
    return encx_conv2d_bwd_data_feat(dy, yact, wp, xact, dx, accumulate, nullptr, nullptr, nullptr, nullptr, 0.0,
                                     nullptr, B,
                                     Ci, T2, Fi, Co, Fo, KT, KF, sf, dt, pt, pf, stream);
}

int encx_conv2d_bwd_data_feat(const float* dy, const float* yact, const float* wp, const float* xact, float* dx,
                              int accumulate, const float* feat_real, const float* feat_fake, const float* feat_denom,
                              const float* feat_g, double feat_scale, const uint8_t* feat_code, int64_t B, int64_t Ci,
                              int64_t T2, int64_t Fi, int64_t Co, int64_t Fo, int64_t KT, int64_t KF, int64_t sf,
                              int64_t dt, int64_t pt, int64_t pf, encx_stream_t stream) {
    ENCX_REQUIRE(dy && wp && dx);
    ENCX_REQUIRE(!feat_real || (feat_fake && feat_denom));
    // the epilogues with a feature term take sign(x - feat_real) from the map they load as x: the
    // xact map when there is one (the compile-time epilogues dgr_epi / rw_dg_epi), so it must BE
    // the fake map
    ENCX_REQUIRE(!feat_real || !xact || xact == feat_fake);
    C2Geo g{(int)B, (int)Ci, (int)T2, (int)Fi, (int)Co, (int)Fo, (int)KT, (int)KF, (int)sf, (int)dt, (int)pt, (int)pf};
    ENCX_REQUIRE(geo_ok(g));
    hipStream_t st = (hipStream_t)stream;
    encx_prof_scope ps(st, 2.0 * B * Co * T2 * Fo * Ci * KT * KF,
                       4.0 * (B * Ci * T2 * Fi * (feat_real ? 3 : 1) + 2 * B * Co * T2 * Fo), "c2_dgrad");
    ps.tag(" %ldx%ld %ldx%ld s%ld T%ld F%ld", (long)Ci, (long)Co, (long)KT, (long)KF, (long)sf, (long)T2, (long)Fo);
    C2Dg a{g, dy, yact, wp, xact, dx, 0, 0, 0, 0, 0, accumulate, feat_real, feat_fake, feat_denom, feat_g,
           (float)feat_scale, feat_real && encx_opt(OPT_FEAT_CODE) ? feat_code : nullptr};
    constexpr int BN = 128;
    a.J = (int)cdiv(KF, sf);
    a.U = (int)((Fi - 1 + pf) / sf + 1);
    a.NR = c2_rows(BN, a.U);
    a.RL = min(BN, a.U) - 1 + a.J;
    const int M = (int)(Ci * sf);
    if (Co == 1 && KT == 3 && KF == 3 && (sf == 1 || sf == 2)) {
        dim3 grid((unsigned)cdiv(T2 * Fi, 256), (unsigned)(B * Ci));
        if (Ci % 4 == 0) {
            const dim3 g4((unsigned)cdiv(T2 * Fi, 256), (unsigned)(B * Ci / 4));
            if (sf == 1) hipLaunchKernelGGL((c2_co1_dgrad<3, 3, 1, 4>), g4, dim3(256), 0, st, a);
            else hipLaunchKernelGGL((c2_co1_dgrad<3, 3, 2, 4>), g4, dim3(256), 0, st, a);
        } else if (sf == 1) hipLaunchKernelGGL((c2_co1_dgrad<3, 3, 1>), grid, dim3(256), 0, st, a);
        else hipLaunchKernelGGL((c2_co1_dgrad<3, 3, 2>), grid, dim3(256), 0, st, a);
        ENCX_CHECK_LAUNCH();
        return 0;
    }
    // register-window form (c2_dgrad_rw_kernel); option DGR = workgroups (0: off)
    const int dg_wgs = (int)encx_opt(OPT_DGR);
    if (dg_wgs > 0 && dgr_ok(g) && rw_pays(cdiv(B * T2 * cdiv(a.U, 4), 32), B * T2 * a.U, 92.0 / 78.0) &&
        run_dgrad_rw(a, dg_wgs, st) == 0)
        return 0;
    // tile choice from tools/mb/c2_mb sweeps: 128-column tiles for the narrowest layers (Fo 33;
    // at Fo 65 the 256-column tile is 4-7 % faster), 8-combo
    // chunks + a 3-waves/SIMD register cap for the wide ones
    if (M == 64 && KF == 9 && sf == 2) {
        if (Fo <= 33 ? run_dgradr<2, 128, 5, 4, 16, 3>(a, st) == 0 : run_dgradr<2, 256, 5, 4, 8, 3>(a, st) == 0)
            return 0;
    }
    if (M <= 32 && KF == 3 && sf == 1 && run_dgradr<1, 256, 3, 6, 32>(a, st) == 0) return 0;
    if (sf == 1 && KT == 3 && KF == 9 && (Ci == 2 || Ci == 4) && Co % DN_CC == 0 && (KT - 1) * dt <= DN_MAXHALO) {
        dim3 grid((unsigned)cdiv(Fi, DN_COLS), (unsigned)cdiv(T2, DN_ROWS), (unsigned)B);
#define ENCX_DN(ci, ym, dt) hipLaunchKernelGGL((c2_dgrad_narrow<ci, 3, 9, ym, true, dt>), grid, dim3(NT), 0, st, a)
        if (dt == 1) {
            if (Ci == 2 && yact) ENCX_DN(2, true, 1);
            else if (Ci == 2) ENCX_DN(2, false, 1);
            else if (yact) ENCX_DN(4, true, 1);
            else ENCX_DN(4, false, 1);
        } else {
            if (Ci == 2 && yact) ENCX_DN(2, true, 2);
            else if (Ci == 2) ENCX_DN(2, false, 2);
            else if (yact) ENCX_DN(4, true, 2);
            else ENCX_DN(4, false, 2);
        }
#undef ENCX_DN
        ENCX_CHECK_LAUNCH();
        return 0;
    }
    if (M <= 32) {
        a.CK = c2_ck((int)(Co * KT), a.NR * a.RL + a.J * 32);
        return launch_dgrad<32, 128, 1, 4>(a, st);
    }
    a.CK = c2_ck((int)(Co * KT), a.NR * a.RL + a.J * 64);
    return launch_dgrad<64, 128, 2, 2>(a, st);
}

size_t encx_conv2d_bwd_weight_workspace(int64_t B, int64_t Ci, int64_t T2, int64_t Fi, int64_t Co, int64_t Fo,
                                        int64_t KT, int64_t KF, int64_t sf, int64_t dt, int64_t pt, int64_t pf) {
    C2Geo g{(int)B, (int)Ci, (int)T2, (int)Fi, (int)Co, (int)Fo, (int)KT, (int)KF, (int)sf, (int)dt, (int)pt, (int)pf};
    WgPlan2 p = plan_wg2(g);
    int splits = p.splits;
    if (wg3r_ok(g)) splits = max(splits, plan_wg3r(g, 32, wg3r_target(g)).splits);
    if (wgr_ok(g)) splits = max(splits, plan_wgr(g, 4096).splits);  // ENCX_WGR up to 4096 waves
    if (co1_ok(g)) splits = max(splits, plan_co1(g).splits);
    if (wg3n_ok(g)) splits = max(splits, plan_wg3n(g).splits + (int)cdiv(plan_wg3n(g).splits, 32));
    size_t bytes = (size_t)splits * Co * (Ci * KT * KF + 1) * sizeof(float);
    if (wgr_ok(g)) {  // the 8-wave form's task-major slabs (ENCX_WGR_WGS up to 1024 workgroups)
        const WgPlanR q = plan_wgr(g, 0, 1024);
        bytes = max(bytes, (size_t)q.splits * wgr_slab(g, q) * sizeof(float));
    }
    return bytes;
}

/* dw [Co][Ci][KT][KF] and db [Co] (either may be NULL) of the layer whose output grad is dy,
 * masked by LeakyReLU'(yact) when yact != NULL. acc_w / acc_b: add into dw / db. */
int encx_conv2d_bwd_weight(const float* dy, const float* yact, const float* x, float* dw, float* db,
                           int acc_w, int acc_b, float* ws, int64_t B, int64_t Ci, int64_t T2, int64_t Fi, int64_t Co,
                           int64_t Fo, int64_t KT, int64_t KF, int64_t sf, int64_t dt, int64_t pt, int64_t pf,
                           encx_stream_t stream) {
    ENCX_REQUIRE(dy && x && ws);
    C2Geo g{(int)B, (int)Ci, (int)T2, (int)Fi, (int)Co, (int)Fo, (int)KT, (int)KF, (int)sf, (int)dt, (int)pt, (int)pf};
    ENCX_REQUIRE(geo_ok(g));
    hipStream_t st = (hipStream_t)stream;
    encx_prof_scope ps(st, 2.0 * B * Co * T2 * Fo * Ci * KT * KF, 4.0 * (B * Ci * T2 * Fi + 2 * B * Co * T2 * Fo), "c2_wgrad");
    ps.tag(" %ldx%ld %ldx%ld s%ld T%ld F%ld", (long)Ci, (long)Co, (long)KT, (long)KF, (long)sf, (long)T2, (long)Fo);
    const int N = (int)(Ci * KT * KF + 1);
    if (co1_ok(g)) {
        const WgPlanC1 q = plan_co1(g);
        C2Wg a{g, dy, yact, x, ws, q.rows, 0, 0, 0, 0, 0, 0};
        dim3 grid((unsigned)q.chunks, (unsigned)B, (unsigned)cdiv(Ci, 4));
        if (sf == 1) hipLaunchKernelGGL((c2_co1_wgrad<3, 3, 1>), grid, dim3(256), 0, st, a);
        else hipLaunchKernelGGL((c2_co1_wgrad<3, 3, 2>), grid, dim3(256), 0, st, a);
        ENCX_CHECK_LAUNCH();
        hipLaunchKernelGGL(c2_wg_reduce, dim3((unsigned)cdiv(N, 64)), dim3(256), 0, st, ws, q.splits, 1, N, dw, db,
                           acc_w, acc_b);
        ENCX_CHECK_LAUNCH();
        return 0;
    }
    const int rw_waves = (int)min(encx_opt(OPT_WGR), (int64_t)4096);
    // 8-wave workgroups summing their partials in LDS (one per CU); option WGR_WGS = 0: one-wave form
    const int rw_wgs = (int)min(encx_opt(OPT_WGR_WGS), (int64_t)1024);
    if (rw_waves > 0 && rw_wgs > 0 && wgr_ok(g) && g_c2_select != 2) {
        const WgPlanR q = plan_wgr(g, 0, rw_wgs);
        if (run_wgrad_rw(g, dy, yact, x, ws, q, st, true) == 0) {
            hipLaunchKernelGGL(c2_wgr_reduce, dim3((unsigned)cdiv(Co * N, 64)), dim3(256), 0, st, ws, q.splits,
                               wgr_slab(g, q), (int)Co, (int)Ci, (int)KT, (int)KF, KF == 9 ? 1 : 3, q.cib, dw, db,
                               acc_w, acc_b);
            ENCX_CHECK_LAUNCH();
            return 0;
        }
    }
    if (rw_waves > 0 && wgr_ok(g) && g_c2_select != 2) {  // register-window form (c2_wgrad_rw_kernel); ENCX_WGR=0 off
        const WgPlanR q = plan_wgr(g, rw_waves);
        if (run_wgrad_rw(g, dy, yact, x, ws, q, st) == 0) {
            hipLaunchKernelGGL(c2_wg_reduce, dim3((unsigned)cdiv(Co * N, 64)), dim3(256), 0, st, ws, q.splits, (int)Co,
                               N, dw, db, acc_w, acc_b);
            ENCX_CHECK_LAUNCH();
            return 0;
        }
    }
    if (wg3r_ok(g)) {  // 9 waves x one 32-column tile each, vectorised staging (c2_wgrad3_kernel)
        const WgPlan3 q = plan_wg3r(g, 32, wg3r_target(g));
        if (run_wgrad3<9, 1, 9, 4, 1, 5>(g, dy, yact, x, ws, q, st) == 0) {
            hipLaunchKernelGGL(c2_wg_reduce, dim3((unsigned)cdiv(Co * N, 64)), dim3(256), 0, st, ws, q.splits, (int)Co,
                               N, dw, db, acc_w, acc_b);
            ENCX_CHECK_LAUNCH();
            return 0;
        }
    }
    if (wg3n_ok(g)) {
        const WgPlan3 q = plan_wg3n(g);
        const int rc = Ci * KT <= 7 ? run_wgrad3<9, 1, 2, 2, 4, 4>(g, dy, yact, x, ws, q, st)
                                    : run_wgrad3<9, 1, 4, 2, 2, 4>(g, dy, yact, x, ws, q, st);
        if (rc == 0) {
            // ~1500 slabs of Co x N outputs: groups of 32 slabs first, then the fixed-order sum
            const int G = 32, S2 = (int)cdiv(q.splits, G);
            const int64_t n = Co * N;
            float* part = ws + (int64_t)q.splits * n;
            hipLaunchKernelGGL(c2_slab_group_sum, dim3((unsigned)cdiv(n, 256), (unsigned)S2), dim3(256), 0, st, ws,
                               q.splits, G, n, part);
            hipLaunchKernelGGL(c2_wg_reduce, dim3((unsigned)cdiv(n, 64)), dim3(256), 0, st, part, S2, (int)Co, N, dw,
                               db, acc_w, acc_b);
            ENCX_CHECK_LAUNCH();
            return 0;
        }
    }
    WgPlan2 p = plan_wg2(g);
    C2Wg a{g, dy, yact, x, ws, p.BT, p.NR, p.RL, p.NCmax, p.items, p.per_split, p.chunks};
    const size_t lds = ((size_t)4 * p.NCmax * p.NR + (size_t)p.BT * 32 + (size_t)p.NCmax * p.NR * p.RL) * sizeof(float) +
                       p.BT * sizeof(int);
    if (p.narrow) {
        const size_t red = (size_t)4 * 16 * 64 * sizeof(float);  // all 4 waves' tiles
        const dim3 grid((unsigned)cdiv(N, 64), (unsigned)cdiv(Co, 32), p.splits);
        if (yact) hipLaunchKernelGGL((c2_wgrad_kernel<32, 64, 1, 2, 2, true>), grid, dim3(NT), lds > red ? lds : red, st, a);
        else hipLaunchKernelGGL((c2_wgrad_kernel<32, 64, 1, 2, 2, false>), grid, dim3(NT), lds > red ? lds : red, st, a);
    } else {
        const dim3 grid((unsigned)cdiv(N, 128), (unsigned)cdiv(Co, 32), p.splits);
        if (yact) hipLaunchKernelGGL((c2_wgrad_kernel<32, 128, 1, 4, 1, true>), grid, dim3(NT), lds, st, a);
        else hipLaunchKernelGGL((c2_wgrad_kernel<32, 128, 1, 4, 1, false>), grid, dim3(NT), lds, st, a);
    }
    ENCX_CHECK_LAUNCH();
    hipLaunchKernelGGL(c2_wg_reduce, dim3((unsigned)cdiv(Co * N, 64)), dim3(256), 0, st, ws, p.splits, (int)Co, N,
                       dw, db, acc_w, acc_b);
    ENCX_CHECK_LAUNCH();
    return 0;
}

/* Spectrogram of DiscriminatorSTFT (msstftd.py:62-64, 97-99): x [B][C][T] -> z [B][2C][Fr][nb]
 * (channels re_0..re_{C-1}, im_0..im_{C-1}), Fr = (T - n)/hop + 1, nb = n/2 + 1, scaled by
 * 1/sqrt(sum w^2) (normalized=True). tables: the mel-table layout of n (encx_mel_tables_init). */
// option FFT = 0: the spectrogram as the framed DFT GEMM (round 3) instead of the real FFT (fft.h)
static bool disc_fft(int64_t n) {
    return encx_opt(OPT_FFT) != 0 && encx_fft::fft_ok(n);
}

static double hann_norm(int64_t n) { return 1.0 / sqrt(3.0 * (double)n / 8.0); }  // sum of periodic hann^2 = 3n/8

int encx_disc_spec_fwd(const float* x, const float* tables, float* z, int64_t B, int64_t C, int64_t T,
                       int64_t n_fft, int64_t hop, encx_stream_t stream) {
    return encx_disc_spec_fwd_scaled(x, tables, z, B, C, T, n_fft, hop, hann_norm(n_fft), stream);
}

int encx_disc_spec_fwd_scaled(const float* x, const float* tables, float* z, int64_t B, int64_t C, int64_t T,
                              int64_t n_fft, int64_t hop, double scale, encx_stream_t stream) {
    ENCX_REQUIRE(x && tables && z && T >= n_fft && hop > 0);
    hipStream_t st = (hipStream_t)stream;
    const int Fr = (int)((T - n_fft) / hop + 1), nb = (int)(n_fft / 2 + 1);
    const float inv = (float)scale;
    const int M = (int)(B * C * Fr), N = 2 * nb, K = (int)n_fft;
    const bool fft = disc_fft(n_fft);
    encx_prof_scope ps(st, fft ? 2.5 * M * K * log2((double)K) : 2.0 * M * N * K, 4.0 * (B * C * T + (int64_t)M * N), "spec_fwd");
    ps.tag(" n%ld", (long)n_fft);
    if (fft) {  // real FFT of each hann-windowed frame (fft.h), written in the (t, f) channel layout
        encx_fft::FftArgs a{x, tables, N, z, (int)T, Fr, (int)hop, 0, M, 1, (int)C, inv};
        return encx_fft::r2c(a, (int)n_fft, st);
    }
    return gemm_launch(LdSpecD{x, tables, (int)T, Fr, (int)hop, N, make_fastdiv((uint32_t)Fr)}, EpSpecD{z, (int)C, Fr, nb, inv}, M, N, K, st);
}

size_t encx_disc_spec_bwd_workspace(int64_t B, int64_t C, int64_t T, int64_t n_fft, int64_t hop) {
    const int64_t Fr = (T - n_fft) / hop + 1;
    return (size_t)(B * C * Fr * n_fft) * sizeof(float);
}

/* dx (+)= d spectrogram^T dz (accumulate: add into dx). ws: encx_disc_spec_bwd_workspace. */
int encx_disc_spec_bwd(const float* dz, const float* tables, float* dx, float* ws, int accumulate, int64_t B,
                       int64_t C, int64_t T, int64_t n_fft, int64_t hop, encx_stream_t stream) {
    return encx_disc_spec_bwd_scaled(dz, tables, dx, ws, accumulate, B, C, T, n_fft, hop, hann_norm(n_fft), stream);
}

int encx_disc_spec_bwd_scaled(const float* dz, const float* tables, float* dx, float* ws, int accumulate,
                              int64_t B, int64_t C, int64_t T, int64_t n_fft, int64_t hop, double scale,
                              encx_stream_t stream) {
    ENCX_REQUIRE(dz && tables && dx && ws && T >= n_fft && hop > 0);
    hipStream_t st = (hipStream_t)stream;
    const int Fr = (int)((T - n_fft) / hop + 1), nb = (int)(n_fft / 2 + 1);
    const float inv = (float)scale;
    const int M = (int)(B * C * Fr), N = (int)n_fft, K = 2 * nb;
    {
        const bool fft = disc_fft(n_fft);
        encx_prof_scope ps(st, fft ? 2.5 * M * N * log2((double)N) : 2.0 * M * N * K,
                           4.0 * ((int64_t)M * K + (int64_t)M * N), "spec_bwd");
        ps.tag(" n%ld", (long)n_fft);
        int rc;
        if (fft) {  // the transpose of the windowed real DFT per frame (fft.h c2r)
            encx_fft::FftArgs a{dz, tables, K, ws, (int)T, Fr, (int)hop, 0, M, 1, (int)C, inv};
            rc = encx_fft::c2r(a, (int)n_fft, st);
        } else {
            rc = gemm_launch(LdSpecDB{dz, tables, (int)C, Fr, nb, K, inv}, EpFrames{ws, N}, M, N, K, st);
        }
        if (rc) return rc;
    }
    const int64_t tot = B * C * T;
    hipLaunchKernelGGL(spec_overlap_add, dim3((unsigned)cdiv(tot, 256)), dim3(256), 0, st, ws, dx, (int)(B * C),
                       (int)T, Fr, (int)n_fft, (int)hop, accumulate);
    ENCX_CHECK_LAUNCH();
    return 0;
}

size_t encx_disc_loss_workspace(void) { return (size_t)2 * LP * sizeof(float); }

/* out[0] (+)= scale * mean(relu(1 + s*x)) over n elements (losses.py:48, 78-79). */
int encx_hinge_loss(const float* x, int64_t n, double s, double scale, float* out, int accumulate, float* ws,
                    encx_stream_t stream) {
    ENCX_REQUIRE(x && out && ws && n > 0);
    encx_prof_scope ps((hipStream_t)stream, 2.0 * n, 4.0 * n, "hinge", false);
    hipStream_t st = (hipStream_t)stream;
    const int nb = (int)min((int64_t)LP, cdiv(n, 256));
    hipLaunchKernelGGL(hinge_kernel, dim3(nb), dim3(256), 0, st, x, n, (float)s, ws);
    hipLaunchKernelGGL(loss_finish, dim3(1), dim3(256), 0, st, ws, nb, 1, (double)n, (float)scale, out,
                       (float*)nullptr, accumulate);
    ENCX_CHECK_LAUNCH();
    return 0;
}

/* out[0] (+)= scale * mean|fr - ff| / mean|fr| (losses.py:53); denom[0] = sum|fr| for the
 * backward. */
int encx_feat_loss(const float* fr, const float* ff, int64_t n, double scale, float* out, float* denom,
                   int accumulate, float* ws, encx_stream_t stream) {
    ENCX_REQUIRE(fr && ff && out && ws && n > 0 && n % 4 == 0 && ((uintptr_t)fr & 15) == 0 && ((uintptr_t)ff & 15) == 0);
    encx_prof_scope ps((hipStream_t)stream, 4.0 * n, 8.0 * n, "feat", false);
    hipStream_t st = (hipStream_t)stream;
    const int nb = (int)min((int64_t)LP, cdiv(n, 1024));
    hipLaunchKernelGGL(feat_kernel<false>, dim3(nb), dim3(256), 0, st, fr, ff, n, ws, (uint32_t*)nullptr);
    hipLaunchKernelGGL(loss_finish, dim3(1), dim3(256), 0, st, ws, nb, 2, (double)n, (float)scale, out, denom,
                       accumulate);
    ENCX_CHECK_LAUNCH();
    return 0;
}

/* encx_feat_loss + the pair's per-element code (code[i] = [ff > fr] | 2 [ff < fr] | 4 [ff > 0], one
 * byte per element, 4-byte aligned), which encx_conv2d_bwd_data_feat reads instead of the two maps. */
int encx_feat_loss_code(const float* fr, const float* ff, int64_t n, double scale, float* out, float* denom,
                        int accumulate, float* ws, uint8_t* code, encx_stream_t stream) {
    ENCX_REQUIRE(fr && ff && out && ws && code && n > 0 && n % 4 == 0 && ((uintptr_t)fr & 15) == 0 &&
                 ((uintptr_t)ff & 15) == 0 && ((uintptr_t)code & 3) == 0);
    encx_prof_scope ps((hipStream_t)stream, 4.0 * n, 9.0 * n, "feat", false);
    hipStream_t st = (hipStream_t)stream;
    const int nb = (int)min((int64_t)LP, cdiv(n, 1024));
    hipLaunchKernelGGL(feat_kernel<true>, dim3(nb), dim3(256), 0, st, fr, ff, n, ws, (uint32_t*)code);
    hipLaunchKernelGGL(loss_finish, dim3(1), dim3(256), 0, st, ws, nb, 2, (double)n, (float)scale, out, denom,
                       accumulate);
    ENCX_CHECK_LAUNCH();
    return 0;
}

/* dx = g0[0] * scale * s / n * [1 + s*x > 0]  (g0 may be NULL: 1) */
int encx_hinge_loss_bwd(const float* x, int64_t n, double s, double scale, const float* g0, float* dx,
                        encx_stream_t stream) {
    ENCX_REQUIRE(x && dx && n > 0);
    encx_prof_scope ps((hipStream_t)stream, 2.0 * n, 8.0 * n, "hinge_bwd", false);
    hipLaunchKernelGGL(hinge_grad_kernel, dim3((unsigned)cdiv(n, 256)), dim3(256), 0, (hipStream_t)stream, x, n,
                       (float)s, (float)scale, g0, dx);
    ENCX_CHECK_LAUNCH();
    return 0;
}

/* dff = g0[0] * scale * sign(ff - fr) / denom[0] */
int encx_feat_loss_bwd(const float* fr, const float* ff, int64_t n, double scale, const float* denom,
                       const float* g0, float* dff, encx_stream_t stream) {
    ENCX_REQUIRE(fr && ff && denom && dff && n > 0);
    encx_prof_scope ps((hipStream_t)stream, 2.0 * n, 12.0 * n, "feat_bwd", false);
    hipLaunchKernelGGL(feat_grad_kernel, dim3((unsigned)cdiv(n, 256)), dim3(256), 0, (hipStream_t)stream, fr, ff, n,
                       (float)scale, denom, g0, dff);
    ENCX_CHECK_LAUNCH();
    return 0;
}

}  // extern "C"
