// Step-level kernels: the RVQ straight-through backward, the device-side loss Balancer
// (balancer.py:83-118) and Adam (torch.optim.Adam as configured at train_multi_gpu.py:295-296).
// Nothing here syncs with the host, so a whole train step can be captured in a hipGraph.
#include "common.h"
#include "prof.h"

namespace {
constexpr int NT = 256;
constexpr int NP = 16;  // partial sums per batch item

// out = a * x + (bdev[0] * bscale) * z
__global__ void lincomb_kernel(const float* x, const float* z, float* out, int64_t n, float a,
                               const float* bdev, float bscale) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float b = bdev ? bdev[0] * bscale : bscale;
    out[i] = a * x[i] + b * z[i];
}

// per-item sum of squares, partial over NP slices
__global__ __launch_bounds__(NT) void item_sq_kernel(const float* g, float* ws, int64_t L) {
    __shared__ float red[16];
    const int b = blockIdx.x, p = blockIdx.y;
    const int64_t per = (L + NP - 1) / NP, beg = p * per, end = min(L, beg + per);
    const float* gb = g + (int64_t)b * L;
    float s = 0.f;
    for (int64_t i = beg + threadIdx.x; i < end; i += NT) s = fmaf(gb[i], gb[i], s);
    s = block_sum(s, red);
    if (threadIdx.x == 0) ws[b * NP + p] = s;
}

// out[0] = mean_b sqrt(sum ws[b][:])  == grad.norm(dim=1..).mean() (balancer.py:88-90)
__global__ __launch_bounds__(NT) void item_norm_mean_kernel(const float* ws, float* out, int B) {
    __shared__ float red[16];
    float s = 0.f;
    for (int b = threadIdx.x; b < B; b += NT) {
        float q = 0.f;
        for (int p = 0; p < NP; ++p) q += ws[b * NP + p];
        s += sqrtf(q);
    }
    s = block_sum(s, red);
    if (threadIdx.x == 0) out[0] = s / (float)B;
}

// averager(beta) (balancer.py:10-28) in fp64 like the reference's Python floats; writes the
// averaged norms (double) and, for average_metrics (distrib.py:112-124), [avg*count.., count]
__global__ void balancer_update_kernel(const float* norms, double* total, double* fix, double* avg,
                                       float* red, int nl, double beta, float count) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    for (int k = 0; k < nl; ++k) {
        total[k] = total[k] * beta + (double)norms[k];
        fix[k] = fix[k] * beta + 1.0;
        avg[k] = total[k] / fix[k];
        red[k] = (float)avg[k] * count;
    }
    red[nl] = count;
}

// scale_k = ratio_k * total_norm / (eps + avg_k) (balancer.py:99-114); from_red: take avg from
// the all-reduced [sum avg*count.., sum count] buffer (fp32 division as average_metrics does)
__global__ void balancer_scales_kernel(const double* avg, const float* red, const double* ratio,
                                       float* scales, int nl, double total_norm, double eps,
                                       int from_red) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    for (int k = 0; k < nl; ++k) {
        double a = from_red ? (double)(red[k] / red[nl]) : avg[k];
        scales[k] = (float)(ratio[k] * total_norm / (eps + a));
    }
}

// out = g0*s0 + g1*s1 + ...  (summed in loss order, balancer.py:110-117)
__global__ void balancer_combine_kernel(const float* g0, const float* g1, const float* g2,
                                        const float* g3, const float* s, float* out, int64_t n) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    {
#pragma clang fp contract(off)  // grad = g * scale, then out_grad += grad: two roundings each
        float v = g0[i] * s[0];
        if (g1) v = v + g1[i] * s[1];
        if (g2) v = v + g2[i] * s[2];
        if (g3) v = v + g3[i] * s[3];
        out[i] = v;
    }
}

// torch.optim.Adam single-tensor step (amsgrad off, no weight decay), flat buffers
__global__ void adam_kernel(float* p, const float* g, float* m, float* v, int64_t n, float w1,
                            float beta2, float one_m_b2, float step_size, float bc2_sqrt,
                            float eps) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float gi = g[i];
    float mi = m[i];
    // exp_avg.lerp_(grad, 1 - beta1): torch's lerp branches on the weight
    mi = w1 < 0.5f ? mi + w1 * (gi - mi) : gi - (gi - mi) * (1.f - w1);
    float vi = v[i] * beta2;
    vi = vi + one_m_b2 * (gi * gi);  // addcmul_(grad, grad, value=1-beta2)
    const float denom = sqrtf(vi) / bc2_sqrt + eps;
    p[i] = p[i] + (-step_size) * (mi / denom);
    m[i] = mi;
    v[i] = vi;
}
// Same update as adam_kernel with the per-step scalars read from device memory (written by
// adam_hyper_kernel), so a HIP graph that captured this launch picks up each step's lr and bias
// corrections on replay.
__global__ void adam_dev_kernel(float* p, const float* g, float* m, float* v, int64_t n,
                                const float* __restrict__ hp) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float w1 = hp[0], beta2 = hp[1], one_m_b2 = hp[2], step_size = hp[3], bc2_sqrt = hp[4],
                eps = hp[5];
    const float gi = g[i];
    float mi = m[i];
    mi = w1 < 0.5f ? mi + w1 * (gi - mi) : gi - (gi - mi) * (1.f - w1);
    float vi = v[i] * beta2;
    vi = vi + one_m_b2 * (gi * gi);
    const float denom = sqrtf(vi) / bc2_sqrt + eps;
    p[i] = p[i] + (-step_size) * (mi / denom);
    m[i] = mi;
    v[i] = vi;
}

__global__ void adam_hyper_kernel(float* hp, float w1, float beta2, float one_m_b2, float step_size,
                                  float bc2_sqrt, float eps) {
    if (threadIdx.x == 0) {
        hp[0] = w1;
        hp[1] = beta2;
        hp[2] = one_m_b2;
        hp[3] = step_size;
        hp[4] = bc2_sqrt;
        hp[5] = eps;
    }
}
}  // namespace

extern "C" {

int encx_lincomb(const float* x, const float* z, float* out, int64_t n, float a, const float* bdev,
                 float bscale, encx_stream_t stream) {
    ENCX_REQUIRE(x && z && out && n >= 0);
    encx_prof_scope ps((hipStream_t)stream, 2.0 * n, 12.0 * n, "lincomb", false);
    if (!n) return 0;
    hipLaunchKernelGGL(lincomb_kernel, dim3(cdiv(n, 256)), dim3(256), 0, (hipStream_t)stream, x, z,
                       out, n, a, bdev, bscale);
    ENCX_CHECK_LAUNCH();
    return 0;
}

size_t encx_item_norm_workspace(int64_t B) { return (size_t)B * NP * sizeof(float); }

int encx_item_norm_mean(const float* g, float* out, float* ws, int64_t B, int64_t L,
                        encx_stream_t stream) {
    ENCX_REQUIRE(g && out && ws && B > 0 && L > 0);
    encx_prof_scope ps((hipStream_t)stream, 2.0 * B * L, 4.0 * B * L, "item_norm", false);
    hipStream_t st = (hipStream_t)stream;
    hipLaunchKernelGGL(item_sq_kernel, dim3(B, NP), dim3(NT), 0, st, g, ws, L);
    ENCX_CHECK_LAUNCH();
    hipLaunchKernelGGL(item_norm_mean_kernel, dim3(1), dim3(NT), 0, st, ws, out, (int)B);
    ENCX_CHECK_LAUNCH();
    return 0;
}

int encx_balancer_update(const float* norms, double* total, double* fix, double* avg, float* red,
                         int nl, double beta, float count, encx_stream_t stream) {
    ENCX_REQUIRE(norms && total && fix && avg && red && nl > 0 && nl <= ENCX_BALANCER_MAX_LOSSES);
    hipLaunchKernelGGL(balancer_update_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, norms,
                       total, fix, avg, red, nl, beta, count);
    ENCX_CHECK_LAUNCH();
    return 0;
}

int encx_balancer_scales(const double* avg, const float* red, const double* ratio, float* scales,
                         int nl, double total_norm, double eps, int from_red,
                         encx_stream_t stream) {
    ENCX_REQUIRE(avg && red && ratio && scales && nl > 0 && nl <= ENCX_BALANCER_MAX_LOSSES);
    hipLaunchKernelGGL(balancer_scales_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, avg, red,
                       ratio, scales, nl, total_norm, eps, from_red);
    ENCX_CHECK_LAUNCH();
    return 0;
}

int encx_balancer_combine(const float* g0, const float* g1, const float* g2, const float* g3,
                          const float* scales, float* out, int64_t n, encx_stream_t stream) {
    ENCX_REQUIRE(g0 && scales && out && n > 0);
    encx_prof_scope ps((hipStream_t)stream, 8.0 * n, 4.0 * n * (1 + (g0 != nullptr) + (g1 != nullptr) + (g2 != nullptr) + (g3 != nullptr)), "balancer_combine", false);
    hipLaunchKernelGGL(balancer_combine_kernel, dim3(cdiv(n, 256)), dim3(256), 0,
                       (hipStream_t)stream, g0, g1, g2, g3, scales, out, n);
    ENCX_CHECK_LAUNCH();
    return 0;
}

int encx_adam_step(float* p, const float* g, float* m, float* v, int64_t n, double lr, double beta1,
                   double beta2, double eps, int64_t step, encx_stream_t stream) {
    ENCX_REQUIRE(p && g && m && v && n >= 0 && step >= 1);
    encx_prof_scope ps((hipStream_t)stream, 10.0 * n, 28.0 * n, "adam");
    if (!n) return 0;
    const double bc1 = 1.0 - pow(beta1, (double)step);
    const double bc2 = 1.0 - pow(beta2, (double)step);
    hipLaunchKernelGGL(adam_kernel, dim3(cdiv(n, 256)), dim3(256), 0, (hipStream_t)stream, p, g, m, v,
                       n, (float)(1.0 - beta1), (float)beta2, (float)(1.0 - beta2),
                       (float)(lr / bc1), (float)sqrt(bc2), (float)eps);
    ENCX_CHECK_LAUNCH();
    return 0;
}

int encx_adam_hyper(float* hp, double lr, double beta1, double beta2, double eps, int64_t step,
                    encx_stream_t stream) {
    ENCX_REQUIRE(hp && step >= 1);
    const double bc1 = 1.0 - pow(beta1, (double)step);
    const double bc2 = 1.0 - pow(beta2, (double)step);
    hipLaunchKernelGGL(adam_hyper_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, hp,
                       (float)(1.0 - beta1), (float)beta2, (float)(1.0 - beta2), (float)(lr / bc1),
                       (float)sqrt(bc2), (float)eps);
    ENCX_CHECK_LAUNCH();
    return 0;
}

int encx_adam_step_dev(float* p, const float* g, float* m, float* v, int64_t n, const float* hp,
                       encx_stream_t stream) {
    ENCX_REQUIRE(p && g && m && v && hp && n >= 0);
    encx_prof_scope ps((hipStream_t)stream, 10.0 * n, 28.0 * n, "adam");
    if (!n) return 0;
    hipLaunchKernelGGL(adam_dev_kernel, dim3(cdiv(n, 256)), dim3(256), 0, (hipStream_t)stream, p, g,
                       m, v, n, hp);
    ENCX_CHECK_LAUNCH();
    return 0;
}

}  // extern "C"
