// Microbenchmark for the high-rate 1-D conv layers: times the library's encx_conv1d_fwd on a
// layer shape against bandwidth probes with the same traffic (build: make -C tools/mb).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>
#include "../../include/encx.h"

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

// probe A: y[b][co][t] = res[b][co][t] + x[b][co % Cin][t], float4, grid-stride
__global__ void probe_rowmix(const float* x, const float* res, float* y, int Cin, int Cout, int T, long n4) {
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x) {
        long e = i * 4;
        long t = e % T, row = e / T;
        long b = row / Cout, co = row % Cout;
        f32x4 r = *(const f32x4*)(res + e);
        f32x4 v = *(const f32x4*)(x + ((b * Cin + co % Cin) * (long)T + t));
        *(f32x4*)(y + e) = r + v;
    }
}
// probe B: pure copy of n floats (float4)
__global__ void probe_copy(const float* x, float* y, long n4) {
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x)
        ((f32x4*)y)[i] = ((const f32x4*)x)[i];
}

// probe C: the conv epilogue's access shape -- one wave per 32 x 32 (co, t) tile, lane l owns
// column t = l & 31 and rows (r & 3) + 8 (r >> 2) + 4 (l >> 5) (v_mfma_f32_32x32x2 layout);
// y = res + x[co % Cin] with scalar loads / stores as in conv_fwd_kernel's epilogue
__global__ __launch_bounds__(256) void probe_mfma_layout(const float* x, const float* res, float* y, int Cin,
                                                         int Cout, int T) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int t = (blockIdx.x * 4 + wave) * 32 + (lane & 31);
    const int co0 = blockIdx.y * 32, b = blockIdx.z;
    if (t >= T) return;
    float e[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int co = co0 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        e[r] = res[((long)b * Cout + co) * T + t] + x[((long)b * Cin + co % Cin) * T + t];
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int co = co0 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        y[((long)b * Cout + co) * T + t] = e[r];
    }
}

// experimental 1x1 / k-tap stride-1 conv (zero pad), tile BM(co) x 128(t), 4 waves 2x2,
// FLAGS: 1 = skip MFMA, 2 = skip staging loads, 4 = skip epilogue residual loads
template <int BM, int FLAGS>
__global__ __launch_bounds__(256) void xconv(const float* x, const float* wf, const float* bias, const float* res,
                                             float* y, int Cin, int Cout, int T, int K) {
    constexpr int BN = 128, WM = 2, WN = 2, TM = BM / WM / 32, TN = BN / WN / 32;
    extern __shared__ float smem[];
    const int Up = BN + K;  // window length (<= BN + K - 1, padded)
    float* Xs = smem;                       // [Cin][Up]
    float* Ws = smem + ((Cin * Up + 3) & ~3);  // [K][Cin][BM]
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm0 = (wave / WN) * TM * 32, wn0 = (wave % WN) * TN * 32;
    const int t0 = blockIdx.x * BN, co0 = blockIdx.y * BM, b = blockIdx.z;
    const int h = lane >> 5, l32 = lane & 31;
    const float* xb = x + (long)b * Cin * T;
    // stage window [t0 - (K-1), t0 + BN) as float4 items from the aligned floor
    const int wb = t0 - (K - 1), ab = wb & ~3, off = wb - ab, nv = (off + BN + K - 1 + 3) >> 2;
    const int nitems = Cin * nv;
    for (int it = tid; it < nitems; it += 256) {
        const int c = it / nv, p = ab + 4 * (it - c * nv);
        f32x4 v = (f32x4){0.f, 0.f, 0.f, 0.f};
        if (!(FLAGS & 2)) {
            if (p >= 0 && p + 3 < T) v = *(const f32x4*)(xb + (long)c * T + p);
            else for (int e = 0; e < 4; ++e) v[e] = (p + e >= 0 && p + e < T) ? xb[(long)c * T + p + e] : 0.f;
        }
        const int q0 = 4 * (it - c * nv) - off;
        for (int e = 0; e < 4; ++e)
            if (q0 + e >= 0 && q0 + e < Up) Xs[c * Up + q0 + e] = v[e];
    }
    for (int it = tid; it < K * Cin * BM / 4; it += 256) {
        const int r = it / (BM / 4), c4 = it - r * (BM / 4), k = r / Cin, c = r - k * Cin;
        *(f32x4*)(Ws + r * BM + 4 * c4) = *(const f32x4*)(wf + ((long)c * K + k) * Cout + co0 + 4 * c4);
    }
    __syncthreads();
    f32x16 acc[TM][TN];
    for (int i = 0; i < TM; ++i) for (int j = 0; j < TN; ++j) acc[i][j] = (f32x16){0};
    if (!(FLAGS & 1)) {
        for (int k = 0; k < K; ++k) {
            const float* wk = Ws + (k * Cin + h) * BM + wm0 + l32;
            const float* xk = Xs + h * Up + wn0 + l32 + k;
            for (int cp = 0; cp < Cin; cp += 2) {
                float av[TM], bv[TN];
#pragma unroll
                for (int i = 0; i < TM; ++i) av[i] = wk[cp * BM + i * 32];
#pragma unroll
                for (int j = 0; j < TN; ++j) bv[j] = xk[cp * Up + j * 32];
#pragma unroll
                for (int i = 0; i < TM; ++i)
#pragma unroll
                    for (int j = 0; j < TN; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[i], bv[j], acc[i][j], 0, 0, 0);
            }
        }
    }
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int t = t0 + wn0 + j * 32 + l32;
            float e1[16];
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int co = co0 + wm0 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
                e1[r] = (!(FLAGS & 4) && res && t < T) ? res[((long)b * Cout + co) * T + t] : 0.f;
            }
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int co = co0 + wm0 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
                if (t < T) y[((long)b * Cout + co) * T + t] = acc[i][j][r] + bias[co] + e1[r];
            }
        }
}

// ---- verbatim copy of the library's conv_fwd_kernel (bisect target)
constexpr int NT = 256;
#define ENCX_DEV __device__ __forceinline__
ENCX_DEV float elu(float x) { return x > 0.f ? x : expm1f(x); }
ENCX_DEV float elu_grad(float x) { return x > 0.f ? 1.f : expf(x); }
ENCX_DEV float act_apply(int act, float x) { return act == ENCX_ACT_ELU ? elu(x) : x; }
ENCX_DEV float act_grad(int act, float x) { return act == ENCX_ACT_ELU ? elu_grad(x) : 1.f; }
ENCX_DEV int pad_src(int p, int pl, int T, int e, int mode) {
    int i = p - pl;
    if (mode == ENCX_PAD_REFLECT) {
        int L = T + e;
        if (i < 0) i = -i;
        else if (i >= L) i = 2 * (L - 1) - i;
        return (i >= 0 && i < T) ? i : -1;
    }
    return (i >= 0 && i < T) ? i : -1;
}
ENCX_DEV f32x16 mfma32(float a, float b, f32x16 c) { return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0); }
ENCX_DEV int mfma_row(int r, int lane) { return (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5); }
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
    int CK;   // channels per LDS chunk (even)
    int Up;   // LDS words per (ci, phase) row
    int KS;   // channel splits
    int cps;  // channels per split (multiple of CK)
};

// y = [acc ? y : 0] + act'(xact) * (v + bias) + res
ENCX_DEV void fwd_store(const FwdArgs& a, int64_t o, int co, float v) {
    v += a.bias ? a.bias[co] : 0.f;
    if (a.xact) v *= act_grad(a.epi_act, a.xact[o]);
    if (a.res) v += a.res[o];
    if (a.accumulate) v += a.y[o];
    a.y[o] = v;
}

// EPI = 0: bias-only epilogue (no operand loads); EPI = 1: act' source / residual / accumulate.
// VEC: input rows and the weight rows are 16-B aligned (float4 staging loads).
template <int BM, int BN, int WM, int WN, int EPI, bool VEC>
__global__ __launch_bounds__(NT, 4) void lconv(FwdArgs a) {
    constexpr int TM = BM / WM / 32, TN = BN / WN / 32;
    extern __shared__ float smem[];
    const int CK = a.CK, S = a.s, Up = a.Up, K = a.K;
    float* Xs = smem;                       // [CK][S][Up]
    float* Ws = smem + ((CK * S * Up + 3) & ~3);  // [K][CK][BM], 16-B aligned
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
    for (int c0 = cbeg; c0 < cend; c0 += CK) {
        __syncthreads();
        for (int it = tid; it < nitems; it += NT) {
            const int cl = it / nv, vi = it - cl * nv, c = c0 + cl;
            const int p = ab + 4 * vi;
            f32x4 v = (f32x4){0.f, 0.f, 0.f, 0.f};
            if (c < cend) {
                const float* xr = xb + (int64_t)c * a.Tin;
                if (VEC && p >= 0 && p + 3 < a.Tin) {
                    v = *(const f32x4*)(xr + p);
                } else {
                    for (int e = 0; e < 4; ++e) {
                        const int m = pad_src(p + e + a.pl, a.pl, a.Tin, a.e, a.mode);
                        v[e] = m >= 0 ? xr[m] : 0.f;
                    }
                }
            }
            float* xs = Xs + cl * span;
            const int q0 = 4 * vi - woff;
            if (S == 1 && q0 >= 0 && q0 + 3 < span) {
                xs[q0] = act_apply(a.act, v[0]);
                xs[q0 + 1] = act_apply(a.act, v[1]);
                xs[q0 + 2] = act_apply(a.act, v[2]);
                xs[q0 + 3] = act_apply(a.act, v[3]);
            } else {
                for (int e = 0; e < 4; ++e) {
                    const int q = q0 + e;
                    if (q >= 0 && q < span) {
                        const int u = q / S, ph = q - u * S;
                        xs[ph * Up + u] = act_apply(a.act, v[e]);
                    }
                }
            }
        }
        // weights [k][ci][co] from wf[ci][k][co]: BM contiguous co per row, float4 items
        for (int it = tid; it < nw; it += NT) {
            const int r = it / BM4, c4 = it - r * BM4, k = r / CK, cl = r - k * CK;
            const int c = c0 + cl, co = co0 + 4 * c4;
            f32x4 v = (f32x4){0.f, 0.f, 0.f, 0.f};
            if (c < cend) {
                const float* wr = a.wf + ((int64_t)c * K + k) * a.Cout + co;
                if (VEC && co + 3 < a.Cout) {
                    v = *(const f32x4*)wr;
                } else {
                    for (int e = 0; e < 4; ++e) v[e] = co + e < a.Cout ? wr[e] : 0.f;
                }
            }
            *(f32x4*)(Ws + r * BM + 4 * c4) = v;
        }
        __syncthreads();
        const int h = lane >> 5, l32 = lane & 31;
        for (int k = 0; k < K; ++k) {
            const int kd = k * a.d, ph = kd % S, off = kd / S;
            const float* wk = Ws + (k * CK + h) * BM + wm0 + l32;
            const float* xk = Xs + (h * S + ph) * Up + wn0 + l32 + off;
#pragma unroll 4
            for (int cp = 0; cp < CK; cp += 2) {
                float av[TM], bv[TN];
#pragma unroll
                for (int i = 0; i < TM; ++i) av[i] = wk[cp * BM + i * 32];
#pragma unroll
                for (int j = 0; j < TN; ++j) bv[j] = xk[cp * S * Up + j * 32];
#pragma unroll
                for (int i = 0; i < TM; ++i)
#pragma unroll
                    for (int j = 0; j < TN; ++j) acc[i][j] = mfma32(av[i], bv[j], acc[i][j]);
            }
        }
    }
    // epilogue: bias from LDS (staged at entry); the residual / act' source / accumulated y of
    // a whole 32 x 32 sub-tile are loaded before any of its stores (y may alias them, so the
    // compiler cannot hoist loads over stores itself)
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int t = t0 + wn0 + j * 32 + (lane & 31);
            const int64_t ob = ((int64_t)b * a.Cout + co0 + wm0 + i * 32) * a.Tout + t;
            // EPI bits: 1 residual, 2 act' source, 4 accumulate into y
            float e0[16], e1[16];
            const bool tok = t < a.Tout;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const bool ok = tok && co0 + wm0 + i * 32 + mfma_row(r, lane) < a.Cout;
                const int64_t o = ok ? ob + (int64_t)mfma_row(r, lane) * a.Tout : 0;
                e0[r] = (EPI & 2) ? a.xact[o] : 0.f;
                e1[r] = (EPI & 1) ? a.res[o] : 0.f;
                if (EPI & 4) e1[r] += a.y[o];
            }
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int cl = wm0 + i * 32 + mfma_row(r, lane), co = co0 + cl;
                if (co >= a.Cout || t >= a.Tout) continue;
                const int64_t o = ob + (int64_t)mfma_row(r, lane) * a.Tout;
                float w = acc[i][j][r];
                if (EPI == 8) {
                    a.part[(int64_t)ks * a.B * a.Cout * a.Tout + o] = w;
                } else {
                    w += Bsm[cl];
                    if (EPI & 2) w *= act_grad(a.epi_act, e0[r]);
                    a.y[o] = w + e1[r];
                }
            }
        }
}


int main(int argc, char** argv) {
    int B = 32, Cin = argc > 1 ? atoi(argv[1]) : 32, Cout = argc > 2 ? atoi(argv[2]) : 64;
    int T = argc > 3 ? atoi(argv[3]) : 12000, K = argc > 4 ? atoi(argv[4]) : 1;
    int resid = argc > 5 ? atoi(argv[5]) : 1;
    int reps = 20;
    size_t nx = (size_t)B * Cin * T, ny = (size_t)B * Cout * T;
    float *x, *y, *res, *wf, *bias, *ws;
    CK(hipMalloc(&x, nx * 4)); CK(hipMalloc(&y, ny * 4)); CK(hipMalloc(&res, ny * 4));
    CK(hipMalloc(&wf, (size_t)Cin * K * Cout * 4)); CK(hipMalloc(&bias, Cout * 4));
    size_t wsb = encx_conv1d_fwd_workspace(B, Cin, Cout, T, K, 1, 1);
    CK(hipMalloc(&ws, wsb + 256));
    std::vector<float> h(ny);
    for (size_t i = 0; i < ny; ++i) h[i] = (float)((i * 2654435761u) % 1000) * 1e-3f - 0.5f;
    CK(hipMemcpy(x, h.data(), nx * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(res, h.data(), ny * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(wf, h.data(), (size_t)Cin * K * Cout * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(bias, h.data(), Cout * 4, hipMemcpyHostToDevice));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    double bytes = 4.0 * (nx + ny * (resid ? 2 : 1));
    auto timeit = [&](const char* name, auto fn) {
        fn();
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0, 0));
        for (int r = 0; r < reps; ++r) fn();
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1));
        double us = ms * 1e3 / reps;
        printf("%-28s %8.1f us  %7.0f GB/s\n", name, us, bytes / us * 1e-3);
    };
    int pl = K - 1;
    printf("B %d Cin %d Cout %d T %d K %d residual %d: %.1f MB\n", B, Cin, Cout, T, K, resid, bytes / 1e6);
    timeit("encx_conv1d_fwd", [&] {
        int rc = encx_conv1d_fwd(x, wf, bias, resid ? res : nullptr, y, ws, B, Cin, T, Cout, T, K, 1, 1, pl, 0,
                                 ENCX_PAD_REFLECT, ENCX_ACT_ELU, 0);
        if (rc) { printf("rc %d\n", rc); exit(1); }
    });
    if (Cout % 64 == 0) {
        const int Up = 128 + K;
        size_t lds = (((Cin * Up + 3) & ~3) + K * Cin * 64) * 4;
        dim3 g((T + 127) / 128, Cout / 64, B);
        timeit("xconv full", [&] { hipLaunchKernelGGL((xconv<64, 0>), g, dim3(256), lds, 0, x, wf, bias, resid ? res : nullptr, y, Cin, Cout, T, K); });
        timeit("xconv no-mfma", [&] { hipLaunchKernelGGL((xconv<64, 1>), g, dim3(256), lds, 0, x, wf, bias, resid ? res : nullptr, y, Cin, Cout, T, K); });
        timeit("xconv no-stage-loads", [&] { hipLaunchKernelGGL((xconv<64, 2>), g, dim3(256), lds, 0, x, wf, bias, resid ? res : nullptr, y, Cin, Cout, T, K); });
        timeit("xconv no-res-loads", [&] { hipLaunchKernelGGL((xconv<64, 4>), g, dim3(256), lds, 0, x, wf, bias, resid ? res : nullptr, y, Cin, Cout, T, K); });
        timeit("xconv stores only", [&] { hipLaunchKernelGGL((xconv<64, 7>), g, dim3(256), lds, 0, x, wf, bias, resid ? res : nullptr, y, Cin, Cout, T, K); });
    }
    timeit("encx_conv1d_fwd act=none", [&] {
        int rc = encx_conv1d_fwd(x, wf, bias, resid ? res : nullptr, y, ws, B, Cin, T, Cout, T, K, 1, 1, pl, 0,
                                 ENCX_PAD_REFLECT, ENCX_ACT_NONE, 0);
        if (rc) { printf("rc %d\n", rc); exit(1); }
    });
    timeit("encx_conv1d_fwd zero-pad", [&] {
        int rc = encx_conv1d_fwd(x, wf, bias, resid ? res : nullptr, y, ws, B, Cin, T, Cout, T, K, 1, 1, pl, 0,
                                 ENCX_PAD_ZERO, ENCX_ACT_NONE, 0);
        if (rc) { printf("rc %d\n", rc); exit(1); }
    });
    {
        FwdArgs a;
        a.x = x; a.wf = wf; a.bias = bias; a.res = resid ? res : nullptr; a.y = y; a.xact = nullptr; a.part = nullptr;
        a.B = B; a.Cin = Cin; a.Tin = T; a.Cout = Cout; a.Tout = T; a.K = K; a.s = 1; a.d = 1; a.pl = pl; a.e = 0;
        a.mode = ENCX_PAD_REFLECT; a.act = ENCX_ACT_ELU; a.epi_act = 0; a.accumulate = 0;
        a.CK = Cin; a.Up = 128 + (K - 1) + 1; if ((a.Up & 31) == 0) a.Up += 1; a.KS = 1; a.cps = Cin;
        size_t lds = (size_t)(((a.CK * a.Up + 3) & ~3) + K * a.CK * 64 + 64) * 4;
        dim3 g((T + 127) / 128, (Cout + 63) / 64, B);
        if (Cout % 64 == 0) {
            timeit("lconv copy EPI", [&] { hipLaunchKernelGGL((lconv<64, 128, 2, 2, 1, true>), g, dim3(256), lds, 0, a); });
            a.res = nullptr;
            timeit("lconv copy EPI0 nores", [&] { hipLaunchKernelGGL((lconv<64, 128, 2, 2, 0, true>), g, dim3(256), lds, 0, a); });
            a.act = 0;
            timeit("lconv copy EPI0 nores noact", [&] { hipLaunchKernelGGL((lconv<64, 128, 2, 2, 0, true>), g, dim3(256), lds, 0, a); });
        }
    }
    timeit("probe rowmix (same bytes)", [&] {
        hipLaunchKernelGGL(probe_rowmix, dim3(2048), dim3(256), 0, 0, x, res, y, Cin, Cout, T, (long)(ny / 4));
    });
    timeit("probe mfma-layout rowmix", [&] {
        hipLaunchKernelGGL(probe_mfma_layout, dim3((T + 127) / 128, Cout / 32, B), dim3(256), 0, 0, x, res, y, Cin,
                           Cout, T);
    });
    timeit("probe copy res->y (2/3 bytes)", [&] {
        hipLaunchKernelGGL(probe_copy, dim3(2048), dim3(256), 0, 0, res, y, (long)(ny / 4));
    });
    return 0;
}
