// Small bandwidth-bound kernels around the conv stacks: bias grads, the audio normalisation of
// EncodecModel._encode_frame, output rescale, the L1 time-domain loss, fixed-order reductions.
// All reductions are two-pass with a fixed partition (no float atomics): bit-reproducible.
#include "common.h"
#include "prof.h"

namespace {
constexpr int NT = 256;
constexpr int CS_PARTS = 64;

// db[c] = sum_{b,t} dy[b,c,t]. Block (c, part) sums a contiguous slice of the B*T positions,
// CS_PER loads in flight per thread (clamped addresses, values selected after the load: a
// branch around each load would serialise their latency); (b, t) advance incrementally, no
// division in the loop. parts == 1: the block writes db[c]; else a second pass adds the parts
// in a fixed order (bit-reproducible either way).
constexpr int CS_PER = 8;
__global__ __launch_bounds__(NT) void chan_sum_p1(const float* dy, float* ws, float* db, int B, int C, int T,
                                                  int parts, int acc) {
    __shared__ float red[16];
    const int c = blockIdx.x, part = blockIdx.y;
    const int64_t tot = (int64_t)B * T;
    const int64_t per = (tot + parts - 1) / parts;
    const int64_t beg = part * per, end = min(tot, beg + per);
    const int dq = NT / T, dr = NT - dq * T;  // a step of NT positions as (rows, columns)
    int64_t i = beg + threadIdx.x;
    int b = (int)(i / T), t = (int)(i - (int64_t)b * T);
    float sacc[CS_PER];
#pragma unroll
    for (int q = 0; q < CS_PER; ++q) sacc[q] = 0.f;
    for (; i < end; i += CS_PER * NT) {
        float v[CS_PER];
#pragma unroll
        for (int q = 0; q < CS_PER; ++q) {
            const bool ok = i + (int64_t)q * NT < end;
            const float x = dy[ok ? ((int64_t)b * C + c) * T + t : 0];
            v[q] = ok ? x : 0.f;
            b += dq;
            t += dr;
            if (t >= T) {
                t -= T;
                ++b;
            }
        }
#pragma unroll
        for (int q = 0; q < CS_PER; ++q) sacc[q] += v[q];
    }
    float s = ((sacc[0] + sacc[1]) + (sacc[2] + sacc[3])) + ((sacc[4] + sacc[5]) + (sacc[6] + sacc[7]));
    s = block_sum(s, red);
    if (threadIdx.x == 0) {
        if (parts == 1) db[c] = acc ? db[c] + s : s;
        else ws[c * parts + part] = s;
    }
}

__global__ void chan_sum_p2(const float* ws, float* db, int C, int parts, int acc) {
    int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= C) return;
    const float s = sum_strided(ws + c * parts, parts, 1);
    db[c] = acc ? db[c] + s : s;
}

// model.py:152-157: mono = mean_c x; volume = sqrt(mean_t mono^2); scale = 1e-8 + volume
__global__ __launch_bounds__(1024) void normalize_kernel(const float* x, float* xn, float* scale,
                                                         int C, int T) {
    __shared__ float red[16];
    const int b = blockIdx.x;
    const float* xb = x + (int64_t)b * C * T;
    float s = 0.f;
    for (int t = threadIdx.x; t < T; t += blockDim.x) {
        float m = 0.f;
        for (int c = 0; c < C; ++c) m += xb[(int64_t)c * T + t];
        m = m / (float)C;
        s = fmaf(m, m, s);
    }
    s = block_sum(s, red);
    const float sc = 1e-8f + sqrtf(s / (float)T);
    if (threadIdx.x == 0) scale[b] = sc;
    float* ob = xn + (int64_t)b * C * T;
    for (int64_t i = threadIdx.x; i < (int64_t)C * T; i += blockDim.x) ob[i] = xb[i] / sc;
}

__global__ void scale_rows_kernel(const float* x, const float* scale, float* y, int64_t CT,
                                  int64_t n) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) y[i] = x[i] * scale[i / CT];
}

__global__ void axpby_kernel(const float* x, float* y, int64_t n, float alpha, const float* ad,
                             float beta) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    float a = ad ? ad[0] : alpha;
    float v = a * x[i];
    if (beta != 0.f) v += beta * y[i];
    y[i] = v;
}

// losses.py:37 l_t = mean|x - y|; d/dy = sign(y - x) / n
__global__ __launch_bounds__(NT) void l1_p1(const float* x, const float* y, float* grad, float* ws,
                                            int64_t n, float inv_n) {
    __shared__ float red[16];
    float s = 0.f;
    for (int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x; i < n; i += (int64_t)gridDim.x * NT) {
        float d = x[i] - y[i];
        s += fabsf(d);
        if (grad) grad[i] = (d < 0.f ? 1.f : (d > 0.f ? -1.f : 0.f)) * inv_n;
    }
    s = block_sum(s, red);
    if (threadIdx.x == 0) ws[blockIdx.x] = s;
}

__global__ __launch_bounds__(NT) void reduce_kernel(const float* parts, int64_t n, float scale,
                                                    float* out, int acc) {
    __shared__ float red[16];
    float s = 0.f;
    for (int64_t i = threadIdx.x; i < n; i += NT) s += parts[i];
    s = block_sum(s, red);
    if (threadIdx.x == 0) out[0] = acc ? out[0] + s * scale : s * scale;
}

__global__ void bdt_to_nd_kernel(const float* r, float* o, int D, int Tf, int64_t total) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= total) return;
    int64_t n = i / D;
    int d = (int)(i - n * D);
    int64_t b = n / Tf, t = n - b * Tf;
    o[i] = r[(b * D + d) * Tf + t];
}
}  // namespace

extern "C" {

size_t encx_channel_sum_workspace(int64_t C) { return (size_t)C * CS_PARTS * sizeof(float); }

int encx_channel_sum(const float* dy, float* db, float* ws, int64_t B, int64_t C, int64_t T,
                     int accumulate, encx_stream_t stream) {
    ENCX_REQUIRE(dy && db && ws && B > 0 && C > 0 && T > 0);
    encx_prof_scope ps((hipStream_t)stream, 1.0 * B * C * T, 4.0 * B * C * T, "chan_sum", false);
    hipStream_t st = (hipStream_t)stream;
    // ~4096 positions per block: one pass for the short rows of the low-rate stages
    int64_t parts = B * T / 4096;
    parts = parts < 1 ? 1 : (parts > CS_PARTS ? CS_PARTS : parts);
    hipLaunchKernelGGL(chan_sum_p1, dim3(C, parts), dim3(NT), 0, st, dy, ws, db, (int)B, (int)C, (int)T,
                       (int)parts, accumulate);
    ENCX_CHECK_LAUNCH();
    if (parts > 1) {
        hipLaunchKernelGGL(chan_sum_p2, dim3(cdiv(C, 256)), dim3(256), 0, st, ws, db, (int)C, (int)parts,
                           accumulate);
        ENCX_CHECK_LAUNCH();
    }
    return 0;
}

int encx_normalize_fwd(const float* x, float* xn, float* scale, int64_t B, int64_t C, int64_t T,
                       encx_stream_t stream) {
    ENCX_REQUIRE(x && xn && scale && B > 0 && C > 0 && T > 0);
    encx_prof_scope ps((hipStream_t)stream, 4.0 * B * C * T, 8.0 * B * C * T, "normalize", false);
    hipLaunchKernelGGL(normalize_kernel, dim3(B), dim3(1024), 0, (hipStream_t)stream, x, xn, scale,
                       (int)C, (int)T);
    ENCX_CHECK_LAUNCH();
    return 0;
}

int encx_scale_rows(const float* x, const float* scale, float* y, int64_t B, int64_t CT,
                    encx_stream_t stream) {
    ENCX_REQUIRE(x && scale && y && B > 0 && CT > 0);
    encx_prof_scope ps((hipStream_t)stream, 1.0 * B * CT, 8.0 * B * CT, "scale_rows", false);
    int64_t n = B * CT;
    hipLaunchKernelGGL(scale_rows_kernel, dim3(cdiv(n, 256)), dim3(256), 0, (hipStream_t)stream, x,
                       scale, y, CT, n);
    ENCX_CHECK_LAUNCH();
    return 0;
}

int encx_axpby(const float* x, float* y, int64_t n, float alpha, const float* alpha_dev,
               float beta, encx_stream_t stream) {
    ENCX_REQUIRE(x && y && n >= 0);
    encx_prof_scope ps((hipStream_t)stream, 2.0 * n, (beta != 0.f ? 12.0 : 8.0) * n, "axpby", false);
    if (n == 0) return 0;
    hipLaunchKernelGGL(axpby_kernel, dim3(cdiv(n, 256)), dim3(256), 0, (hipStream_t)stream, x, y, n,
                       alpha, alpha_dev, beta);
    ENCX_CHECK_LAUNCH();
    return 0;
}

int encx_l1_loss(const float* x, const float* y, float* loss, float* grad, float* ws, int64_t n,
                 encx_stream_t stream) {
    ENCX_REQUIRE(x && y && loss && ws && n > 0);
    encx_prof_scope ps((hipStream_t)stream, 3.0 * n, (grad ? 12.0 : 8.0) * n, "l1_loss", false);
    hipStream_t st = (hipStream_t)stream;
    int blocks = (int)std::min<int64_t>(1024, cdiv(n, NT * 8));
    hipLaunchKernelGGL(l1_p1, dim3(blocks), dim3(NT), 0, st, x, y, grad, ws, n, 1.f / (float)n);
    ENCX_CHECK_LAUNCH();
    hipLaunchKernelGGL(reduce_kernel, dim3(1), dim3(NT), 0, st, ws, (int64_t)blocks, 1.f / (float)n,
                       loss, 0);
    ENCX_CHECK_LAUNCH();
    return 0;
}

int encx_reduce_sum(const float* parts, int64_t n, float scale, float* out, int accumulate,
                    encx_stream_t stream) {
    ENCX_REQUIRE(parts && out && n > 0);
    hipLaunchKernelGGL(reduce_kernel, dim3(1), dim3(NT), 0, (hipStream_t)stream, parts, n, scale,
                       out, accumulate);
    ENCX_CHECK_LAUNCH();
    return 0;
}

int encx_bdt_to_nd(const float* res, float* out, int64_t B, int64_t D, int64_t Tf,
                   encx_stream_t stream) {
    ENCX_REQUIRE(res && out && B > 0 && D > 0 && Tf > 0);
    int64_t total = B * D * Tf;
    hipLaunchKernelGGL(bdt_to_nd_kernel, dim3(cdiv(total, 256)), dim3(256), 0, (hipStream_t)stream,
                       res, out, (int)D, (int)Tf, total);
    ENCX_CHECK_LAUNCH();
    return 0;
}

}  // extern "C"
