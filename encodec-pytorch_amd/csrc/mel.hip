// Multi-scale mel-spectrogram loss (audio_to_mel.py:34-55, losses.py:40-42), forward and the
// gradient w.r.t. the generator output, on the generic MFMA GEMM skeleton of gemm.h.
//
// Per scale n (hop h = n/4, reflect pad p = (n-h)/2, nb = n/2+1 bins, F frames):
//   spec  [B*F][2nb] = frames(reflect_pad(wav)) @ [w*cos | -w*sin]      (DFT as a GEMM; frames
//                      are gathered from the waveform while staging: no im2col in HBM)
//   mel   [B*F][nm]  = (re^2 + im^2) @ mel_basis^T                       (power built on load)
//   loss  += mean|lx - ly| + mean (lx - ly)^2, l = log10(clamp(mel, 1e-5))
// and for d/dy: dmel = (sign(d) + 2d)/Nel / (mel ln10) [mel >= 1e-5]; dP = dmel @ mel_basis;
// G = [2 re dP | 2 im dP]; dframe = G @ [w*cos | -w*sin]^T; overlap-add + reflect fold -> dy.
#include "common.h"
#include "prof.h"
#include "gemm.h"
#include "fft.h"

namespace {

struct Tab {  // device table pointers for one scale
    const float* bt;  // [n][2nb]
    const float* mt;  // [nb][nm]
    const float* mb;  // [nm][nb]
};
ENCX_DEV Tab tab_at(const float* t, int n, int nm) {
    const int nb = n / 2 + 1;
    Tab r;
    r.bt = t;
    r.mt = t + (int64_t)n * 2 * nb;
    r.mb = r.mt + (int64_t)nb * nm;
    return r;
}

// ---------------------------------------------------------------- loaders / epilogues
struct LdSpec {  // A: framed reflect-padded audio, B: DFT table
    static constexpr bool A_K_FAST = true, B_N_FAST = true, VEC = true;
    const float* wav; const float* bt;
    int T, F, h, p, nb2;
    FastDiv fF;  // m -> (clip, frame) without an integer division per staged element
    ENCX_DEV float a(int m, int k) const {
        const int b = (int)fdiv((uint32_t)m, fF), f = m - b * F;
        int src = pad_src(f * h + k, p, T, 0, ENCX_PAD_REFLECT);
        return wav[(int64_t)b * T + src];
    }
    ENCX_DEV float b(int k, int n) const { return bt[(int64_t)k * nb2 + n]; }
    ENCX_DEV f32x4 a4(int m, int k) const {  // one quad load unless it touches the reflected pad
        const int b = (int)fdiv((uint32_t)m, fF), f = m - b * F;
        const int i = f * h + k - p;
        if (i >= 0 && i + 3 < T) return ld4u(wav + (int64_t)b * T + i);
        f32x4 v;
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] = wav[(int64_t)b * T + pad_src(f * h + k + q, p, T, 0, ENCX_PAD_REFLECT)];
        return v;
    }
    ENCX_DEV f32x4 b4(int k, int n) const { return ld4u(bt + (int64_t)k * nb2 + n); }
};
struct EpStore {
    float* out; int ld;
    ENCX_DEV void operator()(int m, int n, float v) const { out[(int64_t)m * ld + n] = v; }
};
struct LdMel {  // A: |X|^2 built from (re, im); B: mel basis^T (scalar staging: the quad form
    // measured 20 % slower, its odd row length 2 nb splits every quad across cache lines)
    static constexpr bool A_K_FAST = true, B_N_FAST = true, VEC = false;
    const float* spec; const float* mt;
    int nb, nm;
    ENCX_DEV float a(int m, int k) const {
        const float* r = spec + (int64_t)m * 2 * nb;
        float re = r[k], im = r[nb + k];
        return re * re + im * im;
    }
    ENCX_DEV float b(int k, int n) const { return mt[(int64_t)k * nm + n]; }
    ENCX_DEV f32x4 a4(int m, int k) const {
        const float* r = spec + (int64_t)m * 2 * nb;
        const f32x4 re = ld4u(r + k), im = ld4u(r + nb + k);
        f32x4 v;
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] = re[q] * re[q] + im[q] * im[q];
        return v;
    }
    ENCX_DEV f32x4 b4(int k, int n) const { return ld4u(mt + (int64_t)k * nm + n); }
};
struct EpLog {
    float* out; int nm;
    ENCX_DEV void operator()(int m, int n, float v) const {
        out[(int64_t)m * nm + n] = log10f(fmaxf(v, 1e-5f));
    }
};
struct EpLogT {  // log-mel in the reference layout [B][nm][F]
    float* out; int nm, F;
    ENCX_DEV void operator()(int m, int n, float v) const {
        int b = m / F, f = m - b * F;
        out[((int64_t)b * nm + n) * F + f] = log10f(fmaxf(v, 1e-5f));
    }
};
struct LdDP {  // A: dmel [rows][nm]; B: mel basis [nm][nb]
    static constexpr bool A_K_FAST = true, B_N_FAST = true, VEC = true;
    const float* dmel; const float* mb;
    int nb, nm;
    ENCX_DEV float a(int m, int k) const { return dmel[(int64_t)m * nm + k]; }
    ENCX_DEV float b(int k, int n) const { return mb[(int64_t)k * nb + n]; }
    ENCX_DEV f32x4 a4(int m, int k) const { return ld4u(dmel + (int64_t)m * nm + k); }
    ENCX_DEV f32x4 b4(int k, int n) const { return ld4u(mb + (int64_t)k * nb + n); }
};
struct EpG {  // spec (re, im) -> (2 re dP, 2 im dP) in place
    float* spec; int nb;
    ENCX_DEV void operator()(int m, int n, float v) const {
        float* r = spec + (int64_t)m * 2 * nb;
        float re = r[n], im = r[nb + n];
        r[n] = 2.f * re * v;
        r[nb + n] = 2.f * im * v;
    }
};
struct LdDF {  // A: G [rows][2nb]; B(k, t) = bt[t][k]
    static constexpr bool A_K_FAST = true, B_N_FAST = false, VEC = true;
    const float* g; const float* bt;
    int nb2;
    ENCX_DEV float a(int m, int k) const { return g[(int64_t)m * nb2 + k]; }
    ENCX_DEV float b(int k, int n) const { return bt[(int64_t)n * nb2 + k]; }
    ENCX_DEV f32x4 a4(int m, int k) const { return ld4u(g + (int64_t)m * nb2 + k); }
    ENCX_DEV f32x4 b4(int k, int n) const { return ld4u(bt + (int64_t)n * nb2 + k); }
};

// ---------------------------------------------------------------- element kernels
__global__ void tables_kernel(float* t, const float* mel, int n, int nm) {
    const int nb = n / 2 + 1, nb2 = 2 * nb;
    Tab tb = tab_at(t, n, nm);
    float* bt = (float*)tb.bt;
    float* mt = (float*)tb.mt;
    float* mb = (float*)tb.mb;
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t nbt = (int64_t)n * nb2;
    if (i < nbt) {
        int tt = (int)(i / nb2), c = (int)(i - (int64_t)tt * nb2);
        int k = c < nb ? c : c - nb;
        // torch.hann_window(n) (periodic): 0.5 - 0.5 cos(2 pi t / n)
        double w = 0.5 - 0.5 * cos(2.0 * M_PI * (double)tt / (double)n);
        double ang = 2.0 * M_PI * (double)(((int64_t)k * tt) % n) / (double)n;
        bt[i] = (float)(c < nb ? w * cos(ang) : -w * sin(ang));
        return;
    }
    i -= nbt;
    if (i < (int64_t)nb * nm) {
        int k = (int)(i / nm), m = (int)(i - (int64_t)k * nm);
        mt[i] = mel[(int64_t)m * nb + k];
        mb[(int64_t)m * nb + k] = mel[(int64_t)m * nb + k];
    }
}

// DFT table of an arbitrary window (a DiscriminatorSTFT whose win_length < n_fft: torch.stft
// centres the window in n_fft zeros): bt[t][c] = win[t] cos / -win[t] sin of the same angle
__global__ void window_table_kernel(float* bt, const float* win, int n) {
    const int nb = n / 2 + 1, nb2 = 2 * nb;
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (int64_t)n * nb2) return;
    const int tt = (int)(i / nb2), c = (int)(i - (int64_t)tt * nb2);
    const int k = c < nb ? c : c - nb;
    const double w = (double)win[tt];
    const double ang = 2.0 * M_PI * (double)(((int64_t)k * tt) % n) / (double)n;
    bt[i] = (float)(c < nb ? w * cos(ang) : -w * sin(ang));
}

// Audio2Mel with any hop / window (encx_mel_logmel_framed): the reflect pad of each row, and the
// log-mel of a spectrogram in the discriminator's layout z [row][re | im][f][k]: one workgroup per
// frame stages its power spectrum in LDS, a thread per mel sums its filter over all bins in order.
__global__ void reflect_pad_kernel(const float* x, float* xp, int64_t rows, int T, int p) {
    const int Tp = T + 2 * p;
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= rows * Tp) return;
    const int64_t r = i / Tp;
    int j = (int)(i - r * Tp) - p;
    j = j < 0 ? -j : (j >= T ? 2 * (T - 1) - j : j);
    xp[i] = x[r * T + j];
}
__global__ void logmel_from_spec_kernel(const float* z, const float* basis, float* out, int Fr, int nb, int nm) {
    extern __shared__ float pw[];
    const int r = blockIdx.y, f = blockIdx.x;
    const float* re = z + ((int64_t)r * 2 * Fr + f) * nb;
    const float* im = re + (int64_t)Fr * nb;
    for (int k = threadIdx.x; k < nb; k += blockDim.x) pw[k] = re[k] * re[k] + im[k] * im[k];
    __syncthreads();
    for (int m = threadIdx.x; m < nm; m += blockDim.x) {
        const float* w = basis + (int64_t)m * nb;
        float s = 0.f;
        for (int k = 0; k < nb; ++k) s = fmaf(w[k], pw[k], s);
        out[((int64_t)r * nm + m) * Fr + f] = log10f(fmaxf(s, 1e-5f));
    }
}

constexpr int LB = 1024;  // loss partial blocks

// ly = log10(clamp(mel_y)); d = ly - lx; parts; dmel (in place over mel_y)
__global__ __launch_bounds__(256) void mel_loss_kernel(const float* lx, float* mel_y, float* parts,
                                                       int64_t total, float inv_n, int want_grad) {
    __shared__ float red[16];
    float s1 = 0.f, s2 = 0.f;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
        float mel = mel_y[i];
        float ly = log10f(fmaxf(mel, 1e-5f));
        float d = lx[i] - ly;  // l1Loss(mel(x), mel(y)): input = mel(x), target = mel(y)
        s1 += fabsf(d);
        s2 = fmaf(d, d, s2);
        if (want_grad) {
            float g = ((d < 0.f ? 1.f : (d > 0.f ? -1.f : 0.f)) - 2.f * d) * inv_n;  // d/d ly
            mel_y[i] = mel >= 1e-5f ? g / (mel * 2.302585092994046f) : 0.f;
        }
    }
    s1 = block_sum(s1, red);
    s2 = block_sum(s2, red);
    if (threadIdx.x == 0) {
        parts[blockIdx.x] = s1;
        parts[LB + blockIdx.x] = s2;
    }
}

__global__ __launch_bounds__(256) void loss_add(const float* parts, int nblk, float inv_n, float* loss) {
    __shared__ float red[16];
    float s1 = 0.f, s2 = 0.f;
    for (int i = threadIdx.x; i < nblk; i += 256) {
        s1 += parts[i];
        s2 += parts[LB + i];
    }
    s1 = block_sum(s1, red);
    s2 = block_sum(s2, red);
    if (threadIdx.x == 0) loss[0] = (loss[0] + s1 * inv_n) + s2 * inv_n;
}

// dy[b][m] += sum over padded positions j mapping to m (reflect) of the overlapping frames
__global__ void overlap_add(const float* dframe, float* grad, int Bn, int T, int n, int h, int p,
                            int F) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (int64_t)Bn * T) return;
    int b = (int)(i / T), m = (int)(i - (int64_t)b * T);
    int js[3];
    int nj = 0;
    js[nj++] = m + p;
    if (m >= 1 && m <= p) js[nj++] = p - m;
    if (m >= T - 1 - p && m <= T - 2) js[nj++] = p + 2 * (T - 1) - m;
    float s = 0.f;
    for (int q = 0; q < nj; ++q) {
        int j = js[q];
        int flo = j - n + 1 > 0 ? (j - n + 1 + h - 1) / h : 0;
        int fhi = j / h;
        if (fhi > F - 1) fhi = F - 1;
        for (int f = flo; f <= fhi; ++f) s += dframe[((int64_t)b * F + f) * n + (j - f * h)];
    }
    grad[i] += s;
}

// option FFT = 0: the spectrogram as the framed DFT GEMM (round 3) instead of the real FFT (fft.h)
static bool use_fft(int64_t n) {
    return encx_opt(OPT_FFT) != 0 && encx_fft::fft_ok(n);
}
// spec [rows][2nb] (re | im) of the reflect-padded, hann-windowed frames of wav
static int spec_rows(const float* wav, const float* bt, float* spec, int64_t B, int64_t T, int n, int h, int p,
                     int F, hipStream_t st) {
    const int nb2 = 2 * (n / 2 + 1);
    if (use_fft(n)) {
        encx_fft::FftArgs a{wav, bt, nb2, spec, (int)T, F, h, p, (int)(B * F), 0, 1, 1.f};
        return encx_fft::r2c(a, n, st);
    }
    return gemm_launch(LdSpec{wav, bt, (int)T, F, h, p, nb2, make_fastdiv((uint32_t)F)}, EpStore{spec, nb2},
                       (int)(B * F), nb2, n, st);
}

struct Geo {
    int n, h, p, nb, F, rows;
    int64_t spec, lmx, mely, dframe;  // workspace offsets (floats)
    int64_t parts, total;
};
Geo geo(int64_t B, int64_t T, int64_t n, int64_t nm) {
    Geo g;
    g.n = (int)n; g.h = (int)(n / 4); g.p = (int)((n - n / 4) / 2); g.nb = (int)(n / 2 + 1);
    g.F = (int)((T + 2 * g.p - n) / g.h + 1);
    g.rows = (int)(B * g.F);
    g.spec = 0;
    g.lmx = g.spec + (int64_t)g.rows * 2 * g.nb;
    g.mely = g.lmx + (int64_t)g.rows * nm;
    g.dframe = g.mely + (int64_t)g.rows * nm;
    g.parts = g.dframe + (int64_t)g.rows * n;
    g.total = g.parts + 2 * LB;
    return g;
}

// the mel filters' supports (tables after mb): per mel m the bins [klo, khi) with a nonzero
// weight, per bin k the mels [mlo, mhi) (the triangular filters overlap pairwise)
ENCX_DEV const int* sup_at(const float* t, int n, int nm) {
    const int nb = n / 2 + 1;
    return reinterpret_cast<const int*>(t + (int64_t)n * 2 * nb + 2 * (int64_t)nb * nm);
}
__global__ void support_kernel(float* t, const float* mel, int n, int nm) {
    const int nb = n / 2 + 1;
    int* sup = const_cast<int*>(sup_at(t, n, nm));
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < nm) {
        int lo = nb, hi = 0;
        for (int k = 0; k < nb; ++k)
            if (mel[(int64_t)i * nb + k] != 0.f) {
                lo = min(lo, k);
                hi = k + 1;
            }
        sup[2 * i] = lo < hi ? lo : 0;
        sup[2 * i + 1] = lo < hi ? hi : 0;
    } else if (i < nm + nb) {
        const int k = i - nm;
        int lo = nm, hi = 0;
        for (int m = 0; m < nm; ++m)
            if (mel[(int64_t)m * nb + k] != 0.f) {
                lo = min(lo, m);
                hi = m + 1;
            }
        sup[2 * nm + 2 * k] = lo < hi ? lo : 0;
        sup[2 * nm + 2 * k + 1] = lo < hi ? hi : 0;
    }
}

// ---------------------------------------------------------------- fused multi-scale loss (round 6)
// One launch per scale does what the nine per-scale launches of encx_mel_loss did: each workgroup
// takes FPW frames of x and the same frames of y through the real FFT in LDS (fft.h), the power
// spectrum through the mel filters (sparse: each bin lies under at most two triangles, so the
// 64 x nb projection costs ~2 nb multiply-adds per frame instead of an MFMA GEMM over a spectrum
// round trip through HBM), log10, the L1 + MSE partial sums and d/d mel(y); then d/d |Y_k|^2 back
// through the filters, G_k = 2 Y_k dP_k, the inverse real FFT and the window: the frame gradients
// for one overlap-add launch over all scales. Loss partials per workgroup, summed by one finish
// launch in a fixed order.
struct MelScale {
    const float* tables;
    float* dframe;  // [rows][n] frame gradients (null: no gradient)
    float* parts;   // [2][nblk] L1 / MSE partial sums
    int T, F, hop, pad, rows;
    float inv_n;    // 1 / (rows * nm)
};
template <int LOGM, bool GRAD>
__global__ __launch_bounds__(encx_fft::FFT_NT) void mel_fused_kernel(const float* x, const float* y, MelScale a) {
    using namespace encx_fft;
    constexpr int M = 1 << LOGM, N = 2 * M, FPW = M >= 1024 ? 1 : 1024 / M, NB = M + 1, NM = 64;
    // splits per mel filter of the projection, so that all 256 threads work at the long frames
    constexpr int S = FPW * NM >= FFT_NT ? 1 : FFT_NT / (FPW * NM);
    __shared__ f2v buf[2 * FPW * M];
    __shared__ f2v twf[M + 1];
    __shared__ f2v Xs[FPW * NB];     // Y's spectrum (kept for the backward), then the c2r input
    __shared__ float Ps[FPW * NB];   // power spectrum, then dP
    __shared__ float Lx[FPW * NM];   // log-mel of x, then d mel(y)
    __shared__ float Mp[S > 1 ? FPW * NM * S : 1];  // split partial sums of the projection
    // the filters' nonzero weights packed per filter (each bin lies under at most two triangles):
    // filter m's weights for bins Wlo[m] + j at Wp[Woff[m] + j], gathered once per workgroup
    __shared__ float Wp[2 * NB];
    __shared__ int Woff[NM + 1], Wlo[NM];
    __shared__ float Win[N];         // the window (a column of the table: one line per element)
    __shared__ float red[16];
    const int nb2 = 2 * NB;
    const float* bt = a.tables;      // window = bt[t * nb2] (column 0: w cos 0)
    for (int t = threadIdx.x; t < N; t += FFT_NT) Win[t] = bt[(int64_t)t * nb2];
    const float* mt = a.tables + (int64_t)N * nb2;  // [nb][nm]
    const int* sup = sup_at(a.tables, N, NM);
    make_twiddles<M>(twf, -1.f);
    if (threadIdx.x < NM) {  // wave 0: the packed offsets, an exclusive scan of the widths
        const int m = threadIdx.x, lo = sup[2 * m], w = sup[2 * m + 1] - lo;
        int incl = w;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int v = __shfl_up(incl, o, 64);
            if (m >= o) incl += v;
        }
        Woff[m] = incl - w;
        Wlo[m] = lo;
        if (m == NM - 1) Woff[NM] = incl;
    }
    __syncthreads();
    {
        const int m = threadIdx.x & (NM - 1), lo = Wlo[m], off = Woff[m], w = Woff[m + 1] - off;
        for (int j = threadIdx.x >> 6; j < w; j += FFT_NT / NM) Wp[off + j] = mt[(int64_t)(lo + j) * NM + m];
    }
    const int row0 = blockIdx.x * FPW;
    float* bufr = reinterpret_cast<float*>(buf);
    float s1 = 0.f, s2 = 0.f;
#pragma unroll 1
    for (int pass = 0; pass < 2; ++pass) {
        const float* w = pass == 0 ? x : y;
        __syncthreads();
        for (int i = threadIdx.x; i < FPW * N; i += FFT_NT) {
            const int f = i / N, t = i - f * N, row = row0 + f;
            float v = 0.f;
            if (row < a.rows) {
                const int bc = row / a.F, fr = row - bc * a.F;
                int s = fr * a.hop + t - a.pad;
                s = s < 0 ? -s : (s >= a.T ? 2 * (a.T - 1) - s : s);
                v = w[(int64_t)bc * a.T + s] * Win[t];
            }
            bufr[i] = v;
        }
        __syncthreads();
        const int res = stockham<M, FPW>(buf, twf);
        const f2v* Z = buf + res * (FPW * M);
        for (int q = threadIdx.x; q < FPW * NB; q += FFT_NT) {
            const int f = q / NB, k = q - f * NB;
            const f2v zk = Z[f * M + (k & (M - 1))], zm = cconj(Z[f * M + ((M - k) & (M - 1))]);
            const f2v e = (zk + zm) * 0.5f, o = (zk - zm) * 0.5f;
            const f2v tt = cmul(twf[k], o);
            const float re = e[0] + tt[1], im = e[1] - tt[0];
            Ps[q] = re * re + im * im;
            if (GRAD && pass == 1) Xs[q] = (f2v){re, im};
        }
        __syncthreads();
        if (S > 1) {  // the projection's split partials: filter m's bins in S equal runs
            for (int q = threadIdx.x; q < FPW * NM * S; q += FFT_NT) {
                const int f = q / (NM * S), r = q - f * NM * S, m = r / S, sp = r - m * S;
                const int lo = Wlo[m], off = Woff[m], wd = Woff[m + 1] - off, ch = (wd + S - 1) / S;
                const int j1 = min(wd, (sp + 1) * ch);
                float acc = 0.f;
                for (int j = sp * ch; j < j1; ++j) acc = fmaf(Ps[f * NB + lo + j], Wp[off + j], acc);
                Mp[q] = acc;
            }
            __syncthreads();
        }
        for (int q = threadIdx.x; q < FPW * NM; q += FFT_NT) {
            const int f = q / NM, m = q - f * NM, row = row0 + f;
            float mel = 0.f;
            if (S > 1) {
#pragma unroll
                for (int sp = 0; sp < S; ++sp) mel += Mp[q * S + sp];
            } else {
                const int lo = Wlo[m], off = Woff[m], wd = Woff[m + 1] - off;
                for (int j = 0; j < wd; ++j) mel = fmaf(Ps[f * NB + lo + j], Wp[off + j], mel);
            }
            const float l = log10f(fmaxf(mel, 1e-5f));
            if (pass == 0) {
                Lx[q] = l;
            } else if (row < a.rows) {
                const float d = Lx[q] - l;  // l1Loss(mel(x), mel(y)): input mel(x), target mel(y)
                s1 += fabsf(d);
                s2 = fmaf(d, d, s2);
                if (GRAD) {
                    const float g = ((d < 0.f ? 1.f : (d > 0.f ? -1.f : 0.f)) - 2.f * d) * a.inv_n;
                    Lx[q] = mel >= 1e-5f ? g / (mel * 2.302585092994046f) : 0.f;
                }
            } else if (GRAD) {
                Lx[q] = 0.f;
            }
        }
    }
    s1 = block_sum(s1, red);
    s2 = block_sum(s2, red);
    if (threadIdx.x == 0) {
        a.parts[blockIdx.x] = s1;
        a.parts[gridDim.x + blockIdx.x] = s2;
    }
    if (!GRAD) return;
    __syncthreads();
    // D_k = 2 Y_k dP_k, dP_k = sum over the filters on k of dmel_m w_mk; then the c2r of c2r_kernel
    for (int q = threadIdx.x; q < FPW * NB; q += FFT_NT) {
        const int f = q / NB, k = q - f * NB;
        const int mlo = sup[2 * NM + 2 * k], mhi = sup[2 * NM + 2 * k + 1];
        float dp = 0.f;
        for (int m = mlo; m < mhi; ++m) dp = fmaf(Lx[f * NM + m], Wp[Woff[m] + k - Wlo[m]], dp);
        const f2v d = Xs[q] * (2.f * dp);
        Xs[q] = (k == 0 || k == M) ? (f2v){d[0], 0.f} : d * 0.5f;
    }
    __syncthreads();
    for (int q = threadIdx.x; q < FPW * M; q += FFT_NT) {
        const int f = q / M, k = q - f * M;
        const f2v yk = Xs[f * NB + k], ym = cconj(Xs[f * NB + M - k]);
        const f2v A = yk + ym, Bv = cmul(yk - ym, cconj(twf[k]));
        buf[q] = (f2v){A[0] - Bv[1], A[1] + Bv[0]};
    }
    __syncthreads();
    const int res = stockham<M, FPW, true>(buf, twf);
    const float* c = reinterpret_cast<const float*>(buf + res * (FPW * M));
    for (int i = threadIdx.x; i < FPW * N; i += FFT_NT) {
        const int f = i / N, t = i - f * N, row = row0 + f;
        if (row < a.rows) a.dframe[(int64_t)row * N + t] = c[i] * Win[t];
    }
}
template <bool GRAD>
static int mel_fused_launch(int n, const float* x, const float* y, const MelScale& a, hipStream_t st) {
    if (const int rc = encx_fft::tw_ready(st)) return rc;
    const int m = n / 2, fpw = m >= 1024 ? 1 : 1024 / m;
    const dim3 grid((unsigned)cdiv(a.rows, fpw));
    switch (m) {
        case 16: hipLaunchKernelGGL((mel_fused_kernel<4, GRAD>), grid, dim3(encx_fft::FFT_NT), 0, st, x, y, a); break;
        case 32: hipLaunchKernelGGL((mel_fused_kernel<5, GRAD>), grid, dim3(encx_fft::FFT_NT), 0, st, x, y, a); break;
        case 64: hipLaunchKernelGGL((mel_fused_kernel<6, GRAD>), grid, dim3(encx_fft::FFT_NT), 0, st, x, y, a); break;
        case 128: hipLaunchKernelGGL((mel_fused_kernel<7, GRAD>), grid, dim3(encx_fft::FFT_NT), 0, st, x, y, a); break;
        case 256: hipLaunchKernelGGL((mel_fused_kernel<8, GRAD>), grid, dim3(encx_fft::FFT_NT), 0, st, x, y, a); break;
        case 512: hipLaunchKernelGGL((mel_fused_kernel<9, GRAD>), grid, dim3(encx_fft::FFT_NT), 0, st, x, y, a); break;
        case 1024: hipLaunchKernelGGL((mel_fused_kernel<10, GRAD>), grid, dim3(encx_fft::FFT_NT), 0, st, x, y, a); break;
        default: return ENCX_EINVAL;
    }
    return (int)hipGetLastError();
}
constexpr int MEL_MAXS = 8;
struct MelOla {  // the frame gradients of every scale
    const float* dframe[MEL_MAXS];
    int n[MEL_MAXS], hop[MEL_MAXS], pad[MEL_MAXS], F[MEL_MAXS];
    int lh[MEL_MAXS];  // log2 hop (hop = n / 4, a power of two)
    int ns;
};
// grad[b][m] (+)= sum over scales (in order) of overlap_add's sum for that scale
__global__ void overlap_add_all(MelOla o, float* grad, int Bn, int T) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (int64_t)Bn * T) return;
    const int b = (int)(i / T), m = (int)(i - (int64_t)b * T);
    float tot = 0.f;
    for (int sc = 0; sc < o.ns; ++sc) {
        const int n = o.n[sc], h = o.hop[sc], p = o.pad[sc], F = o.F[sc];
        int js[3];
        int nj = 0;
        js[nj++] = m + p;
        if (m >= 1 && m <= p) js[nj++] = p - m;
        if (m >= T - 1 - p && m <= T - 2) js[nj++] = p + 2 * (T - 1) - m;
        float s = 0.f;
        const int lh = o.lh[sc];
        for (int q = 0; q < nj; ++q) {
            const int j = js[q];
            const int flo = j - n + 1 > 0 ? (j - n + h) >> lh : 0;
            int fhi = j >> lh;
            if (fhi > F - 1) fhi = F - 1;
            // at most n / hop = 4 frames cover j: their loads in flight together, added in f order
            float v[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int f = flo + u;
                v[u] = f <= fhi ? o.dframe[sc][((int64_t)b * F + f) * n + (j - f * h)] : 0.f;
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) s += v[u];
        }
        tot += s;
    }
    grad[i] += tot;
}
// loss[0] += sum over scales (in order) of (sum L1 parts + sum MSE parts) * inv_n
struct MelFin {
    const float* parts[MEL_MAXS];
    int nblk[MEL_MAXS];
    float inv_n[MEL_MAXS];
    int ns;
};
// one wave per scale (MEL_MAXS <= 8 waves), each lane summing its strided share of the scale's
// partials, then the waves' sums in scale order
__global__ __launch_bounds__(512) void mel_loss_finish(MelFin f, float* loss) {
    __shared__ float r1[MEL_MAXS], r2[MEL_MAXS];
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (w < f.ns) {
        const float* p = f.parts[w];
        const int nb = f.nblk[w];
        float a1 = 0.f, a2 = 0.f;
        for (int i = lane; i < nb; i += 64) {
            a1 += p[i];
            a2 += p[nb + i];
        }
        a1 = wave_sum(a1);
        a2 = wave_sum(a2);
        if (lane == 0) {
            r1[w] = a1;
            r2[w] = a2;
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        float tot = loss[0];
        for (int sc = 0; sc < f.ns; ++sc) tot = (tot + r1[sc] * f.inv_n[sc]) + r2[sc] * f.inv_n[sc];
        loss[0] = tot;
    }
}

}  // namespace

extern "C" {

size_t encx_mel_tables_floats(int64_t n_fft, int64_t n_mels) {
    int64_t nb = n_fft / 2 + 1;
    // + the filters' supports: per mel [klo, khi), per bin [mlo, mhi) (ints)
    return (size_t)(n_fft * 2 * nb + 2 * nb * n_mels + 2 * n_mels + 2 * nb);
}

int encx_mel_tables_init(float* tables, const float* mel_basis, int64_t n_fft, int64_t n_mels,
                         encx_stream_t stream) {
    ENCX_REQUIRE(tables && mel_basis && n_fft >= 4 && (n_fft % 4) == 0 && n_mels > 0);
    int64_t tot = n_fft * 2 * (n_fft / 2 + 1) + (n_fft / 2 + 1) * n_mels;
    hipLaunchKernelGGL(tables_kernel, dim3(cdiv(tot, 256)), dim3(256), 0, (hipStream_t)stream, tables,
                       mel_basis, (int)n_fft, (int)n_mels);
    const int64_t nsup = n_mels + n_fft / 2 + 1;
    hipLaunchKernelGGL(support_kernel, dim3(cdiv(nsup, 256)), dim3(256), 0, (hipStream_t)stream, tables, mel_basis,
                       (int)n_fft, (int)n_mels);
    ENCX_CHECK_LAUNCH();
    return 0;
}

int encx_spec_tables_window(float* tables, const float* window, int64_t n_fft, encx_stream_t stream) {
    ENCX_REQUIRE(tables && window && n_fft >= 4 && (n_fft % 4) == 0);
    const int64_t tot = n_fft * 2 * (n_fft / 2 + 1);
    hipLaunchKernelGGL(window_table_kernel, dim3(cdiv(tot, 256)), dim3(256), 0, (hipStream_t)stream, tables, window,
                       (int)n_fft);
    ENCX_CHECK_LAUNCH();
    return 0;
}

size_t encx_mel_logmel_framed_workspace_floats(int64_t B, int64_t T, int64_t n_fft, int64_t hop) {
    const int64_t p = (n_fft - hop) / 2, Tp = T + 2 * p, Fr = Tp >= n_fft ? (Tp - n_fft) / hop + 1 : 0;
    return (size_t)(B * Tp + B * 2 * Fr * (n_fft / 2 + 1) + 64);
}

int encx_mel_logmel_framed(const float* x, const float* win_tables, const float* mel_basis, float* ws, float* out,
                           int64_t B, int64_t T, int64_t n_fft, int64_t hop, int64_t n_mels, encx_stream_t stream) {
    ENCX_REQUIRE(x && win_tables && mel_basis && ws && out && B > 0 && hop > 0 && n_mels > 0 && n_fft >= 4 &&
                 (n_fft % 4) == 0 && hop <= n_fft);
    const int64_t p = (n_fft - hop) / 2, Tp = T + 2 * p, nb = n_fft / 2 + 1;
    ENCX_REQUIRE(p < T && Tp >= n_fft && nb * sizeof(float) <= 64 * 1024 && B <= 65535);
    const int64_t Fr = (Tp - n_fft) / hop + 1;
    hipStream_t st = (hipStream_t)stream;
    float* xp = ws;
    float* z = ws + ((B * Tp + 15) & ~(int64_t)15);
    hipLaunchKernelGGL(reflect_pad_kernel, dim3(cdiv(B * Tp, 256)), dim3(256), 0, st, x, xp, B, (int)T, (int)p);
    ENCX_CHECK_LAUNCH();
    const int rc = encx_disc_spec_fwd_scaled(xp, win_tables, z, B, 1, Tp, n_fft, hop, 1.0, stream);
    if (rc) return rc;
    hipLaunchKernelGGL(logmel_from_spec_kernel, dim3((unsigned)Fr, (unsigned)B), dim3(256), nb * sizeof(float), st, z,
                       mel_basis, out, (int)Fr, (int)nb, (int)n_mels);
    ENCX_CHECK_LAUNCH();
    return 0;
}

size_t encx_mel_workspace_floats(int64_t B, int64_t T, int64_t n_fft, int64_t n_mels) {
    return (size_t)geo(B, T, n_fft, n_mels).total;
}

int64_t encx_mel_frames(int64_t T, int64_t n_fft) { return geo(1, T, n_fft, 1).F; }

int encx_mel_logmel(const float* x, const float* tables, float* ws, float* out, int64_t B,
                    int64_t T, int64_t n_fft, int64_t n_mels, encx_stream_t stream) {
    ENCX_REQUIRE(x && tables && ws && out && B > 0 && n_fft >= 4 && (n_fft % 4) == 0);
    hipStream_t st = (hipStream_t)stream;
    const int nm = (int)n_mels;
    Geo g = geo(B, T, n_fft, n_mels);
    ENCX_REQUIRE(g.p < T && g.F > 0);
    const float* bt = tables;
    const float* mt = tables + (int64_t)g.n * 2 * g.nb;
    const int nb2 = 2 * g.nb;
    int rc = spec_rows(x, bt, ws + g.spec, B, T, g.n, g.h, g.p, g.F, st);
    if (rc) return rc;
    return gemm_launch(LdMel{ws + g.spec, mt, g.nb, nm}, EpLogT{out, nm, g.F}, g.rows, nm, g.nb, st);
}

int encx_mel_loss(const float* x, const float* y, const float* tables, float* ws, float* loss,
                  float* grad, int64_t B, int64_t T, int64_t n_fft, int64_t n_mels,
                  encx_stream_t stream) {
    ENCX_REQUIRE(x && y && tables && ws && loss && B > 0 && n_fft >= 4 && (n_fft % 4) == 0);
    const double rows_ = (double)geo(B, T, n_fft, n_mels).rows, nb_ = (double)(n_fft / 2 + 1);
    // algorithmic flops: the transforms at 5 n log2 n per real frame with the FFT (2 n (n + 2) as the DFT GEMM)
    const double lg = log2((double)n_fft), dft = use_fft(n_fft) ? 2.5 * n_fft * lg : 2.0 * nb_ * n_fft * 2;
    encx_prof_scope ps((hipStream_t)stream, rows_ * (2 * dft + 2.0 * nb_ * n_mels * 2) + (grad ? rows_ * (2.0 * nb_ * n_mels + dft) : 0.0),
                       4.0 * B * T * (grad ? 3 : 2), "mel_loss");
    hipStream_t st = (hipStream_t)stream;
    const int nm = (int)n_mels;
    Geo g = geo(B, T, n_fft, n_mels);
    ENCX_REQUIRE(g.p < T && g.F > 0);
    const float* bt = tables;
    const float* mt = tables + (int64_t)g.n * 2 * g.nb;
    const float* mb = mt + (int64_t)g.nb * nm;
    float* spec = ws + g.spec;
    float* lmx = ws + g.lmx;
    float* mely = ws + g.mely;
    float* dframe = ws + g.dframe;
    float* parts = ws + g.parts;
    const int nb2 = 2 * g.nb;
    int rc;
    // target: logmel(x)
    rc = spec_rows(x, bt, spec, B, T, g.n, g.h, g.p, g.F, st);
    if (rc) return rc;
    rc = gemm_launch(LdMel{spec, mt, g.nb, nm}, EpLog{lmx, nm}, g.rows, nm, g.nb, st);
    if (rc) return rc;
    // output: mel(y)
    rc = spec_rows(y, bt, spec, B, T, g.n, g.h, g.p, g.F, st);
    if (rc) return rc;
    rc = gemm_launch(LdMel{spec, mt, g.nb, nm}, EpStore{mely, nm}, g.rows, nm, g.nb, st);
    if (rc) return rc;
    const int64_t total = (int64_t)g.rows * nm;
    const float inv_n = 1.f / (float)total;
    const int nblk = (int)std::min<int64_t>(LB, cdiv(total, 256 * 4));
    hipLaunchKernelGGL(mel_loss_kernel, dim3(nblk), dim3(256), 0, st, lmx, mely, parts, total, inv_n,
                       grad ? 1 : 0);
    ENCX_CHECK_LAUNCH();
    hipLaunchKernelGGL(loss_add, dim3(1), dim3(256), 0, st, parts, nblk, inv_n, loss);
    ENCX_CHECK_LAUNCH();
    if (!grad) return 0;
    rc = gemm_launch(LdDP{mely, mb, g.nb, nm}, EpG{spec, g.nb}, g.rows, g.nb, nm, st);
    if (rc) return rc;
    if (use_fft(g.n)) {  // dframe = w * Re sum_k G_k e^{+i theta}: the real inverse transform
        encx_fft::FftArgs fa{spec, bt, nb2, dframe, (int)T, g.F, g.h, g.p, g.rows, 0, 1, 1.f};
        rc = encx_fft::c2r(fa, g.n, st);
    } else {
        rc = gemm_launch(LdDF{spec, bt, nb2}, EpStore{dframe, g.n}, g.rows, g.n, nb2, st);
    }
    if (rc) return rc;
    hipLaunchKernelGGL(overlap_add, dim3(cdiv(B * T, 256)), dim3(256), 0, st, dframe, grad, (int)B,
                       (int)T, g.n, g.h, g.p, g.F);
    ENCX_CHECK_LAUNCH();
    return 0;
}

size_t encx_mel_loss_multi_workspace_floats(int64_t B, int64_t T, const int64_t* n_ffts, int64_t nscales) {
    size_t tot = 0;
    for (int64_t i = 0; i < nscales; ++i) {
        const Geo g = geo(B, T, n_ffts[i], 64);
        const int fpw = g.n / 2 >= 1024 ? 1 : 1024 / (g.n / 2);
        tot += (size_t)g.rows * g.n + 2 * (size_t)cdiv(g.rows, fpw) + 64;
    }
    return tot;
}

int encx_mel_loss_multi(const float* x, const float* y, const float* const* tables, const int64_t* n_ffts,
                        int64_t nscales, float* ws, float* loss, float* grad, int64_t B, int64_t T,
                        encx_stream_t stream) {
    ENCX_REQUIRE(x && y && tables && n_ffts && ws && loss && B > 0 && nscales > 0 && nscales <= MEL_MAXS);
    hipStream_t st = (hipStream_t)stream;
    double flops = 0.0;
    for (int64_t i = 0; i < nscales; ++i) {
        const int64_t n = n_ffts[i];
        ENCX_REQUIRE(tables[i] && encx_fft::fft_ok(n));
        const double rows = (double)geo(B, T, n, 64).rows, lg = log2((double)n);
        flops += rows * (2 * 2.5 * n * lg + 2 * 2.0 * (n + 2)) + (grad ? rows * (2.5 * n * lg + 2.0 * (n + 2)) : 0.0);
    }
    encx_prof_scope ps(st, flops, 4.0 * B * T * (grad ? 3 : 2), "mel_loss");
    MelOla o{};
    MelFin fin{};
    o.ns = fin.ns = (int)nscales;
    float* cur = ws;
    for (int64_t i = 0; i < nscales; ++i) {
        const Geo g = geo(B, T, n_ffts[i], 64);
        ENCX_REQUIRE(g.p < T && g.F > 0);
        const int fpw = g.n / 2 >= 1024 ? 1 : 1024 / (g.n / 2);
        const int nblk = (int)cdiv(g.rows, fpw);
        MelScale a;
        a.tables = tables[i];
        a.dframe = grad ? cur : nullptr;
        cur += (size_t)g.rows * g.n;
        a.parts = cur;
        cur += 2 * (size_t)nblk + 64;
        a.T = (int)T; a.F = g.F; a.hop = g.h; a.pad = g.p; a.rows = g.rows;
        a.inv_n = 1.f / (float)((int64_t)g.rows * 64);
        const int rc = grad ? mel_fused_launch<true>(g.n, x, y, a, st) : mel_fused_launch<false>(g.n, x, y, a, st);
        if (rc) return rc;
        o.dframe[i] = a.dframe;
        o.n[i] = g.n; o.hop[i] = g.h; o.pad[i] = g.p; o.F[i] = g.F;
        o.lh[i] = 31 - __builtin_clz((unsigned)g.h);
        fin.parts[i] = a.parts;
        fin.nblk[i] = nblk;
        fin.inv_n[i] = a.inv_n;
    }
    hipLaunchKernelGGL(mel_loss_finish, dim3(1), dim3(512), 0, st, fin, loss);
    ENCX_CHECK_LAUNCH();
    if (grad) {
        hipLaunchKernelGGL(overlap_add_all, dim3((unsigned)cdiv(B * T, 256)), dim3(256), 0, st, o, grad, (int)B, (int)T);
        ENCX_CHECK_LAUNCH();
    }
    return 0;
}

}  // extern "C"
