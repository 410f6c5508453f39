// 48 kHz model pieces (config 5): GroupNorm(1, C) after every conv (modules/conv.py:45-49,
// norm='time_group_norm') and the segment overlap-add of EncodecModel.decode (utils.py:22-61).
//
// GroupNorm(1, C) normalises each sample over (C, T). Both directions make one pass that forms
// per-(b, c) row sums in fp64 (one workgroup per row, fixed-order block reduction), a tiny
// finalise kernel per sample / channel, and one elementwise pass. All reductions run in a fixed
// order (deterministic).
#include "common.h"
#include "prof.h"

namespace {

constexpr int NT = 256;

ENCX_DEV double block_sum_d(double v, double* red /* >= 4 doubles */) {
    v = wave_sum_d(v);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (lane == 0) red[wave] = v;
    __syncthreads();
    double s = 0.0;
    if (threadIdx.x == 0)
        for (int w = 0; w < (int)(blockDim.x >> 6); ++w) s += red[w];
    __syncthreads();
    return s;  // valid in thread 0
}

// rows[(b*C + c)*2 + {0,1}] = (sum x, sum x^2) over t
__global__ __launch_bounds__(NT) void gn_row_stats(const float* x, double* rows, int T) {
    __shared__ double red[4];
    const float* xr = x + (int64_t)blockIdx.x * T;
    double s = 0.0, q = 0.0;
    for (int t = threadIdx.x; t < T; t += NT) {
        const double v = xr[t];
        s += v;
        q += v * v;
    }
    s = block_sum_d(s, red);
    q = block_sum_d(q, red);
    if (threadIdx.x == 0) {
        rows[2 * blockIdx.x] = s;
        rows[2 * blockIdx.x + 1] = q;
    }
}

// stats[2b] = mean, stats[2b+1] = rstd = 1/sqrt(var + eps) (biased variance, torch GroupNorm)
__global__ void gn_finish_stats(const double* rows, float* stats, int B, int C, int T, double eps) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= B) return;
    double s = 0.0, q = 0.0;
    for (int c = 0; c < C; ++c) {
        s += rows[2 * ((int64_t)b * C + c)];
        q += rows[2 * ((int64_t)b * C + c) + 1];
    }
    const double n = (double)C * T, mean = s / n;
    double var = q / n - mean * mean;
    if (var < 0.0) var = 0.0;
    stats[2 * b] = (float)mean;
    stats[2 * b + 1] = (float)(1.0 / sqrt(var + eps));
}

// y[row][t] = norm(x[row][tl + t]) for t < Ty (the statistics cover all T positions)
__global__ void gn_apply(const float* x, const float* stats, const float* gamma, const float* beta, float* y,
                         int C, int T, int tl, int Ty, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int64_t row = i / Ty;
    const int t = (int)(i - row * Ty) + tl;
    const int b = (int)(row / C), c = (int)(row - (int64_t)b * C);
    const float xh = (x[row * T + t] - stats[2 * b]) * stats[2 * b + 1];
    y[i] = xh * (gamma ? gamma[c] : 1.f) + (beta ? beta[c] : 0.f);
}

// rows[(b*C + c)*2 + {0,1}] = (sum dy, sum dy * xhat) over the window (dy is 0 outside it)
__global__ __launch_bounds__(NT) void gn_row_bwd(const float* dy, const float* x, const float* stats,
                                                 double* rows, int C, int T, int tl, int Ty) {
    __shared__ double red[4];
    const int b = blockIdx.x / C;
    const float mean = stats[2 * b], rstd = stats[2 * b + 1];
    const float* dr = dy + (int64_t)blockIdx.x * Ty;
    const float* xr = x + (int64_t)blockIdx.x * T + tl;
    double s = 0.0, q = 0.0;
    for (int t = threadIdx.x; t < Ty; t += NT) {
        const double g = dr[t];
        s += g;
        q += g * (double)((xr[t] - mean) * rstd);
    }
    s = block_sum_d(s, red);
    q = block_sum_d(q, red);
    if (threadIdx.x == 0) {
        rows[2 * blockIdx.x] = s;
        rows[2 * blockIdx.x + 1] = q;
    }
}

// per sample: coef[2b] = mean_ct(g), coef[2b+1] = mean_ct(g * xhat) with g = dy * gamma[c];
// per channel: dgamma[c] (+)= sum_b rows[b][c][1], dbeta[c] (+)= sum_b rows[b][c][0]
__global__ void gn_finish_bwd(const double* rows, const float* gamma, float* coef, float* dgamma, float* dbeta,
                              int B, int C, int T, int acc) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < B) {
        double s = 0.0, q = 0.0;
        for (int c = 0; c < C; ++c) {
            const double gm = gamma ? gamma[c] : 1.0;
            s += gm * rows[2 * ((int64_t)i * C + c)];
            q += gm * rows[2 * ((int64_t)i * C + c) + 1];
        }
        const double n = (double)C * T;
        coef[2 * i] = (float)(s / n);
        coef[2 * i + 1] = (float)(q / n);
    }
    if (i < C) {
        double s = 0.0, q = 0.0;
        for (int b = 0; b < B; ++b) {
            s += rows[2 * ((int64_t)b * C + i)];
            q += rows[2 * ((int64_t)b * C + i) + 1];
        }
        if (dgamma) dgamma[i] = acc ? dgamma[i] + (float)q : (float)q;
        if (dbeta) dbeta[i] = acc ? dbeta[i] + (float)s : (float)s;
    }
}

// dx = rstd * (dy*gamma - mean(g) - xhat * mean(g*xhat)), dy = 0 outside the window
__global__ void gn_dx(const float* dy, const float* x, const float* stats, const float* coef, const float* gamma,
                      float* dx, int C, int T, int tl, int Ty, int64_t n, int acc) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int64_t row = i / T;
    const int t = (int)(i - row * T) - tl;
    const int b = (int)(row / C), c = (int)(row - (int64_t)b * C);
    const float mean = stats[2 * b], rstd = stats[2 * b + 1];
    const float xh = (x[i] - mean) * rstd;
    const float d = (t >= 0 && t < Ty) ? dy[row * Ty + t] : 0.f;
    const float g = d * (gamma ? gamma[c] : 1.f);
    const float v = rstd * (g - coef[2 * b] - xh * coef[2 * b + 1]);
    dx[i] = acc ? dx[i] + v : v;
}

// ------------------------------------------------------------------------- overlap-add
constexpr int MAXF = 32;
struct Frames {
    const float* p[MAXF];
    int len[MAXF];
};
// triangle weight of utils.py:45-46: t = linspace(0, 1, L0 + 2)[1:-1], w = 0.5 - |t - 0.5|
ENCX_DEV float ola_w(int j, int L0) {
    const float t = (float)(j + 1) / (float)(L0 + 1);
    return 0.5f - fabsf(t - 0.5f);
}
__global__ void ola_fwd(Frames f, int nf, int stride, int L0, int64_t BC, int total, float* out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= BC * total) return;
    const int64_t bc = i / total;
    const int t = (int)(i - bc * total);
    float acc = 0.f, sw = 0.f;
    for (int k = 0; k < nf; ++k) {
        const int j = t - k * stride;
        if (j < 0 || j >= f.len[k]) continue;
        const float w = ola_w(j, L0);
        acc += w * f.p[k][bc * f.len[k] + j];
        sw += w;
    }
    out[i] = acc / sw;
}
// d frame_k[bc][j] = w(j) * dout[bc][k*stride + j] / sumw(k*stride + j)
__global__ void ola_bwd(const float* dout, int nf, int stride, int L0, int64_t BC, int total, int k, int len,
                        float* dframe) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= BC * len) return;
    const int64_t bc = i / len;
    const int j = (int)(i - bc * len), t = k * stride + j;
    float sw = 0.f;
    for (int q = 0; q < nf; ++q) {
        const int jj = t - q * stride;
        const int lq = q == nf - 1 ? (total - q * stride) : L0;
        if (jj >= 0 && jj < lq) sw += ola_w(jj, L0);
    }
    dframe[i] = ola_w(j, L0) * dout[bc * total + t] / sw;
}

}  // namespace

extern "C" {

size_t encx_groupnorm_workspace(int64_t B, int64_t C) { return (size_t)(2 * B * C) * sizeof(double); }

int encx_groupnorm_fwd(const float* x, const float* gamma, const float* beta, float* y, float* stats, void* ws,
                       int64_t B, int64_t C, int64_t T, int64_t trim_left, int64_t Ty, double eps,
                       encx_stream_t stream) {
    ENCX_REQUIRE(x && y && stats && ws && B > 0 && C > 0 && T > 0);
    encx_prof_scope ps((hipStream_t)stream, 6.0 * B * C * T, 8.0 * B * C * T, "groupnorm", false);
    ENCX_REQUIRE(trim_left >= 0 && Ty > 0 && trim_left + Ty <= T);
    hipStream_t st = (hipStream_t)stream;
    double* rows = (double*)ws;
    hipLaunchKernelGGL(gn_row_stats, dim3((unsigned)(B * C)), dim3(NT), 0, st, x, rows, (int)T);
    hipLaunchKernelGGL(gn_finish_stats, dim3((unsigned)cdiv(B, 64)), dim3(64), 0, st, rows, stats, (int)B, (int)C,
                       (int)T, eps);
    const int64_t n = B * C * Ty;
    hipLaunchKernelGGL(gn_apply, dim3((unsigned)cdiv(n, 256)), dim3(256), 0, st, x, stats, gamma, beta, y, (int)C,
                       (int)T, (int)trim_left, (int)Ty, n);
    ENCX_CHECK_LAUNCH();
    return 0;
}

int encx_groupnorm_bwd(const float* dy, const float* x, const float* gamma, const float* stats, float* dx,
                       float* dgamma, float* dbeta, int acc_x, int acc_params, void* ws, float* coef, int64_t B,
                       int64_t C, int64_t T, int64_t trim_left, int64_t Ty, encx_stream_t stream) {
    ENCX_REQUIRE(dy && x && stats && ws && coef && B > 0 && C > 0 && T > 0);
    encx_prof_scope ps((hipStream_t)stream, 8.0 * B * C * T, 12.0 * B * C * T, "groupnorm_bwd", false);
    ENCX_REQUIRE(trim_left >= 0 && Ty > 0 && trim_left + Ty <= T);
    hipStream_t st = (hipStream_t)stream;
    double* rows = (double*)ws;
    hipLaunchKernelGGL(gn_row_bwd, dim3((unsigned)(B * C)), dim3(NT), 0, st, dy, x, stats, rows, (int)C, (int)T,
                       (int)trim_left, (int)Ty);
    const int64_t m = B > C ? B : C;
    hipLaunchKernelGGL(gn_finish_bwd, dim3((unsigned)cdiv(m, 64)), dim3(64), 0, st, rows, gamma, coef, dgamma, dbeta,
                       (int)B, (int)C, (int)T, acc_params);
    if (dx) {
        const int64_t n = B * C * T;
        hipLaunchKernelGGL(gn_dx, dim3((unsigned)cdiv(n, 256)), dim3(256), 0, st, dy, x, stats, coef, gamma, dx,
                           (int)C, (int)T, (int)trim_left, (int)Ty, n, acc_x);
    }
    ENCX_CHECK_LAUNCH();
    return 0;
}

int encx_overlap_add(const float* const* frames, const int64_t* lengths, int nf, int64_t stride, int64_t BC,
                     float* out, encx_stream_t stream) {
    ENCX_REQUIRE(frames && lengths && out && nf > 0 && nf <= MAXF && stride > 0 && BC > 0);
    Frames f;
    for (int k = 0; k < nf; ++k) {
        ENCX_REQUIRE(frames[k] && lengths[k] > 0 && (k == nf - 1 || lengths[k] == lengths[0]));
        f.p[k] = frames[k];
        f.len[k] = (int)lengths[k];
    }
    const int total = (int)(stride * (nf - 1) + lengths[nf - 1]);
    ENCX_REQUIRE(nf == 1 || stride <= lengths[0]);
    hipLaunchKernelGGL(ola_fwd, dim3((unsigned)cdiv(BC * total, 256)), dim3(256), 0, (hipStream_t)stream, f, nf,
                       (int)stride, (int)lengths[0], BC, total, out);
    ENCX_CHECK_LAUNCH();
    return 0;
}

int encx_overlap_add_bwd(const float* dout, int nf, int64_t stride, int64_t L0, int64_t BC, int64_t total, int k,
                         int64_t len, float* dframe, encx_stream_t stream) {
    ENCX_REQUIRE(dout && dframe && nf > 0 && k >= 0 && k < nf && len > 0);
    hipLaunchKernelGGL(ola_bwd, dim3((unsigned)cdiv(BC * len, 256)), dim3(256), 0, (hipStream_t)stream, dout, nf,
                       (int)stride, (int)L0, BC, (int)total, k, (int)len, dframe);
    ENCX_CHECK_LAUNCH();
    return 0;
}

}  // extern "C"
