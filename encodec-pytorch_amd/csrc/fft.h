// Batched real FFTs of windowed frames for the spectrogram front-ends (round 4): the multi-scale
// mel loss (audio_to_mel.py:34-55: torch.stft, center=False after a reflect pad, hann window) and
// the discriminator's Spectrogram (msstftd.py:62-64: normalized, center=False). They replace the
// framed DFT-as-GEMM (2 n (n + 2) flops per frame) by an n log n transform:
//   r2c: frame f of row bc is w[t] * x_pad[bc][f*hop + t], t < n (x_pad: reflect pad p both sides,
//        or none); X_k = sum_t frame[t] e^{-2 pi i k t / n}, k <= n/2, written as (re | im) rows
//        [row][2 nb] (mel) or to the discriminator layout z[b][re c | im c][f][k] * scale.
//   c2r: the transpose (the spectrogram backward): y[t] = w[t] * scale * sum_{k <= n/2} Re(D_k e^{+2 pi i k t / n})
//        from (re | im) rows (mel) or the discriminator layout, written as frames [row][n]; the
//        callers' overlap-add kernels fold the frames back onto the waveform.
// Both run the n-point real transform as an m = n/2-point complex Stockham radix-2 FFT in LDS
// (one workgroup: max(1, 1024/m) frames), packed z[j] = x[2j] + i x[2j+1], with the real/complex
// pre/post twiddle; twiddles e^{-pi i k/m} from fp64 sincospi per workgroup. Accuracy: O(log n)
// roundings per output instead of the GEMM's O(n)-term fp32 sums.
#pragma once
#include "common.h"

namespace encx_fft {

typedef float f2v __attribute__((ext_vector_type(2)));

ENCX_DEV f2v cmul(f2v a, f2v b) { return (f2v){a[0] * b[0] - a[1] * b[1], a[0] * b[1] + a[1] * b[0]}; }
ENCX_DEV f2v cconj(f2v a) { return (f2v){a[0], -a[1]}; }

constexpr int FFT_NT = 256;

struct FftArgs {
    const float* x;     // r2c: waveform [BC][T]; c2r: spectrum (layout per `layout`)
    const float* win;   // window w[t] = win[t * wstride] (the DFT table's cos column 0)
    int wstride;
    float* out;         // r2c: spectrum; c2r: frames [rows][n]
    int T, F, hop, pad; // frames per row F, reflect pad `pad` (r2c input)
    int rows;           // BC * F
    int layout;         // 0: [row][2nb] (re | im); 1: z[b][2C][F][nb] (re channels, then im)
    int C;              // layout 1: channels
    float scale;        // layout 1: 1 / sqrt(sum w^2)
};

// Twiddles e^{-pi i k / M}, k <= M, for M = 2^4 .. 2^10, from fp64 sincospi once per module and
// device (tw_ready: a setup launch before the first transform) at g_tw[tw_base(M) + k]; each
// workgroup copies its M + 1 into LDS (computing them per workgroup, 1025 fp64 sincospi at M 1024,
// was a third of a frame's work). One copy per translation unit (static).
constexpr int tw_base(int M) { return 2 * M + 16; }
constexpr int TW_SIZE = tw_base(1024) + 1025;
static __device__ f2v g_tw[TW_SIZE];
static __global__ void tw_init_kernel(int M) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k > M) return;
    double s, c;
    sincospi((double)k / (double)M, &s, &c);
    g_tw[tw_base(M) + k] = (f2v){(float)c, (float)(-s)};
}
static inline int tw_ready(hipStream_t st) {
    static bool done[64];
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return ENCX_EINVAL;
    if (done[dev]) return 0;
    for (int M = 16; M <= 1024; M <<= 1)
        hipLaunchKernelGGL(tw_init_kernel, dim3((unsigned)((M + 256) / 256)), dim3(256), 0, st, M);
    const hipError_t e = hipGetLastError();
    if (e == hipSuccess) done[dev] = true;
    return (int)e;
}
// twiddles e^{sign * pi i k / M}, k <= M, into tw (LDS)
template <int M>
ENCX_DEV void make_twiddles(f2v* tw, float sign) {
    for (int k = threadIdx.x; k <= M; k += FFT_NT) {
        const f2v v = g_tw[tw_base(M) + k];
        tw[k] = sign < 0.f ? v : cconj(v);
    }
}

// Stockham over FPW frames of M points in buf[0] (result in buf[RES]); tw[k] = e^{-pi i k/M}, k <= M
// (CONJ: the conjugate twiddles, the inverse transform from the forward table). Radix-4 stages
// (one radix-2 stage first when log2 M is odd): half the passes, and so half the workgroup
// barriers, of a radix-2 transform -- the barriers, not the arithmetic, set the pace of these
// one-to-few-frame workgroups.
template <int M, bool CONJ>
ENCX_DEV f2v tw_at(const f2v* tw, int k) {  // e^{-+pi i k / M} for 0 <= k < 2M (e^{-pi i} = -1)
    const f2v t = k <= M ? tw[k] : -tw[k - M];
    return CONJ ? cconj(t) : t;
}
template <int M, int FPW, bool CONJ = false>
ENCX_DEV int stockham(f2v* buf, const f2v* tw) {
    int cur = 0;
    int ns = 1;
    if (__builtin_ctz(M) & 1) {  // radix-2 stage
        const f2v* src = buf;
        f2v* dst = buf + FPW * M;
        for (int q = threadIdx.x; q < FPW * (M / 2); q += FFT_NT) {
            const int f = q / (M / 2), j = q - f * (M / 2);
            const f2v a = src[f * M + j], b = src[f * M + j + M / 2];
            dst[f * M + 2 * j] = a + b;
            dst[f * M + 2 * j + 1] = a - b;
        }
        __syncthreads();
        cur = 1;
        ns = 2;
    }
#pragma unroll 1
    for (; ns < M; ns <<= 2) {
        const f2v* src = buf + cur * (FPW * M);
        f2v* dst = buf + (cur ^ 1) * (FPW * M);
        const int tstep = M / (2 * ns);  // twiddle index per unit of jm: e^{-2 pi i jm / (4 ns)}
        for (int q = threadIdx.x; q < FPW * (M / 4); q += FFT_NT) {
            const int f = q / (M / 4), j = q - f * (M / 4);
            const int jm = j & (ns - 1);
            const f2v* s0 = src + f * M + j;
            const f2v a0 = s0[0];
            const f2v a1 = cmul(s0[M / 4], tw_at<M, CONJ>(tw, jm * tstep));
            const f2v a2 = cmul(s0[M / 2], tw_at<M, CONJ>(tw, 2 * jm * tstep));
            const f2v a3 = cmul(s0[3 * M / 4], tw_at<M, CONJ>(tw, 3 * jm * tstep));
            const f2v b0 = a0 + a2, b1 = a0 - a2, b2 = a1 + a3, b3 = a1 - a3;
            // -i b3 (forward) / +i b3 (inverse)
            const f2v ib3 = CONJ ? (f2v){-b3[1], b3[0]} : (f2v){b3[1], -b3[0]};
            const int d = f * M + ((j - jm) << 2) + jm;
            dst[d] = b0 + b2;
            dst[d + ns] = b1 + ib3;
            dst[d + 2 * ns] = b0 - b2;
            dst[d + 3 * ns] = b1 - ib3;
        }
        __syncthreads();
        cur ^= 1;
    }
    return cur;
}

template <int LOGM>
__global__ __launch_bounds__(FFT_NT) void r2c_kernel(FftArgs a) {
    constexpr int M = 1 << LOGM, N = 2 * M, FPW = M >= 1024 ? 1 : 1024 / M;
    __shared__ f2v buf[2 * FPW * M];
    __shared__ f2v tw[M + 1];
    __shared__ float Win[N];  // the window, gathered once (a strided table column)
    make_twiddles<M>(tw, -1.f);
    for (int t = threadIdx.x; t < N; t += FFT_NT) Win[t] = a.win[(int64_t)t * a.wstride];
    __syncthreads();
    const int row0 = blockIdx.x * FPW;
    // load: packed z[j] = (w x)[2j] + i (w x)[2j + 1]
    float* bufr = reinterpret_cast<float*>(buf);
    for (int i = threadIdx.x; i < FPW * N; i += FFT_NT) {
        const int f = i / N, t = i - f * N, row = row0 + f;
        float v = 0.f;
        if (row < a.rows) {
            const int bc = row / a.F, fr = row - bc * a.F;
            int s = fr * a.hop + t - a.pad;
            s = s < 0 ? -s : (s >= a.T ? 2 * (a.T - 1) - s : s);
            v = a.x[(int64_t)bc * a.T + s] * Win[t];
        }
        bufr[i] = v;
    }
    __syncthreads();
    const int res = stockham<M, FPW>(buf, tw);
    const f2v* Z = buf + res * (FPW * M);
    constexpr int NB = M + 1;
    for (int q = threadIdx.x; q < FPW * NB; q += FFT_NT) {
        const int f = q / NB, k = q - f * NB, row = row0 + f;
        if (row >= a.rows) continue;
        const f2v zk = Z[f * M + (k & (M - 1))], zm = cconj(Z[f * M + ((M - k) & (M - 1))]);
        const f2v e = (zk + zm) * 0.5f, o = (zk - zm) * 0.5f;  // even / odd spectra (o times i)
        // X_k = e - i e^{-pi i k/M} o
        const f2v t = cmul(tw[k], o);
        const float re = e[0] + t[1], im = e[1] - t[0];
        if (a.layout == 0) {
            a.out[(int64_t)row * 2 * NB + k] = re;
            a.out[(int64_t)row * 2 * NB + NB + k] = im;
        } else {
            const int bc = row / a.F, fr = row - bc * a.F, b = bc / a.C, c = bc - b * a.C;
            a.out[(((int64_t)b * 2 * a.C + c) * a.F + fr) * NB + k] = re * a.scale;
            a.out[(((int64_t)b * 2 * a.C + a.C + c) * a.F + fr) * NB + k] = im * a.scale;
        }
    }
}

template <int LOGM>
__global__ __launch_bounds__(FFT_NT) void c2r_kernel(FftArgs a) {
    constexpr int M = 1 << LOGM, N = 2 * M, FPW = M >= 1024 ? 1 : 1024 / M, NB = M + 1;
    __shared__ f2v buf[2 * FPW * M];
    __shared__ f2v tw[M + 1];
    __shared__ f2v Ys[FPW * NB];
    __shared__ float Win[N];
    make_twiddles<M>(tw, -1.f);  // e^{-pi i k / M}; the inverse conjugates them
    for (int t = threadIdx.x; t < N; t += FFT_NT) Win[t] = a.win[(int64_t)t * a.wstride];
    const int row0 = blockIdx.x * FPW;
    for (int q = threadIdx.x; q < FPW * NB; q += FFT_NT) {
        const int f = q / NB, k = q - f * NB, row = row0 + f;
        f2v d = (f2v){0.f, 0.f};
        if (row < a.rows) {
            if (a.layout == 0) {
                d = (f2v){a.x[(int64_t)row * 2 * NB + k], a.x[(int64_t)row * 2 * NB + NB + k]};
            } else {
                const int bc = row / a.F, fr = row - bc * a.F, b = bc / a.C, c = bc - b * a.C;
                d = (f2v){a.x[(((int64_t)b * 2 * a.C + c) * a.F + fr) * NB + k],
                          a.x[(((int64_t)b * 2 * a.C + a.C + c) * a.F + fr) * NB + k]} * a.scale;
            }
        }
        // Hermitian spectrum of y = sum_{k<=M} Re(D_k e^{+i theta}): Y_0 = Re D_0, Y_M = Re D_M,
        // Y_k = D_k / 2 otherwise
        Ys[q] = (k == 0 || k == M) ? (f2v){d[0], 0.f} : d * 0.5f;
    }
    __syncthreads();
    // Z'_k = A_k + i B_k, A_k = Y_k + conj(Y_{M-k}), B_k = (Y_k - conj(Y_{M-k})) e^{+pi i k/M}
    for (int q = threadIdx.x; q < FPW * M; q += FFT_NT) {
        const int f = q / M, k = q - f * M;
        const f2v yk = Ys[f * NB + k], ym = cconj(Ys[f * NB + M - k]);
        const f2v A = yk + ym, Bv = cmul(yk - ym, cconj(tw[k]));
        buf[q] = (f2v){A[0] - Bv[1], A[1] + Bv[0]};
    }
    __syncthreads();
    const int res = stockham<M, FPW, true>(buf, tw);  // inverse (e^{+}), unnormalised
    const float* c = reinterpret_cast<const float*>(buf + res * (FPW * M));  // y[2j], y[2j+1] interleaved
    for (int i = threadIdx.x; i < FPW * N; i += FFT_NT) {
        const int f = i / N, t = i - f * N, row = row0 + f;
        if (row < a.rows) a.out[(int64_t)row * N + t] = c[i] * Win[t];
    }
}

// host launchers: n = 2^k, 32 <= n <= 2048
#define ENCX_FFT_SWITCH(KERNEL)                                                                   \
    {                                                                                             \
        if (const int rc_ = tw_ready(st)) return rc_;                                             \
        const int m = n / 2, fpw = m >= 1024 ? 1 : 1024 / m;                                      \
        const dim3 grid((unsigned)cdiv(a.rows, fpw));                                             \
        switch (m) {                                                                              \
            case 16: hipLaunchKernelGGL(KERNEL<4>, grid, dim3(FFT_NT), 0, st, a); break;          \
            case 32: hipLaunchKernelGGL(KERNEL<5>, grid, dim3(FFT_NT), 0, st, a); break;          \
            case 64: hipLaunchKernelGGL(KERNEL<6>, grid, dim3(FFT_NT), 0, st, a); break;          \
            case 128: hipLaunchKernelGGL(KERNEL<7>, grid, dim3(FFT_NT), 0, st, a); break;         \
            case 256: hipLaunchKernelGGL(KERNEL<8>, grid, dim3(FFT_NT), 0, st, a); break;         \
            case 512: hipLaunchKernelGGL(KERNEL<9>, grid, dim3(FFT_NT), 0, st, a); break;         \
            case 1024: hipLaunchKernelGGL(KERNEL<10>, grid, dim3(FFT_NT), 0, st, a); break;       \
            default: return ENCX_EINVAL;                                                          \
        }                                                                                         \
        return (int)hipGetLastError();                                                            \
    }
inline bool fft_ok(int64_t n) { return n >= 32 && n <= 2048 && (n & (n - 1)) == 0; }
inline int r2c(const FftArgs& a, int n, hipStream_t st) ENCX_FFT_SWITCH(r2c_kernel)
inline int c2r(const FftArgs& a, int n, hipStream_t st) ENCX_FFT_SWITCH(c2r_kernel)
#undef ENCX_FFT_SWITCH

}  // namespace encx_fft
