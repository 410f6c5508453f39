// torch.nn.utils.weight_norm(dim=0) as applied by modules/conv.py:25-34 to every SEANet conv
// (and msstftd.py:73-84 to the discriminator's 2-D convs): w = v * (g / ||v||_row).
// The forward writes the weight directly in the operand layouts of the conv kernels, so the
// normalisation and the per-step re-layout are a single pass over the (small) weight.
#include "common.h"
#include "prof.h"

namespace {

constexpr int NT = 256;

ENCX_DEV void wn_fwd_row(const float* v, const float* g, float* wf, float* wp, int A0, int A1, int K, int s,
                         int J, int a0, float* red) {
    const int cols = A1 * K;
    const float* vr = v + (int64_t)a0 * cols;
    float scale = 1.f;
    if (g) {
        float ss = 0.f;
        for (int i = threadIdx.x; i < cols; i += NT) ss = fmaf(vr[i], vr[i], ss);
        ss = block_sum(ss, red);
        scale = g[a0] / sqrtf(ss);
    }
    if (wf)  // wf[a1][k][a0]
        for (int i = threadIdx.x; i < cols; i += NT) {
            int a1 = i / K, k = i - a1 * K;
            wf[((int64_t)a1 * K + k) * A0 + a0] = vr[i] * scale;
        }
    if (wp) {  // wp[a0][j][a1*s + r] = w[a0][a1][r + s*j]
        const int rows = A1 * s;
        for (int i = threadIdx.x; i < J * rows; i += NT) {
            int j = i / rows, rr = i - j * rows;
            int a1 = rr / s, r = rr - a1 * s, k = r + s * j;
            wp[((int64_t)a0 * J + j) * rows + rr] = k < K ? vr[a1 * K + k] * scale : 0.f;
        }
    }
}

__global__ __launch_bounds__(NT) void wn_fwd_kernel(const float* v, const float* g, float* wf,
                                                    float* wp, int A0, int A1, int K, int s,
                                                    int J) {
    __shared__ float red[16];
    wn_fwd_row(v, g, wf, wp, A0, A1, K, s, J, blockIdx.x, red);
}

// layer of global row r: the last descriptor with row0 <= r (row0 ascending)
template <typename D>
ENCX_DEV int wn_find(const D* d, int n, int64_t r) {
    int lo = 0, hi = n - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (d[mid].row0 <= r) lo = mid;
        else hi = mid - 1;
    }
    return lo;
}

__global__ __launch_bounds__(NT) void wn_fwd_batch_kernel(const encx_wn_fwd_desc* d, int n) {
    __shared__ float red[16];
    const int li = wn_find(d, n, blockIdx.x);
    const encx_wn_fwd_desc e = d[li];
    const int J = (int)((e.K + e.stride - 1) / e.stride);
    wn_fwd_row(e.v, e.g, e.wf, e.wp, (int)e.A0, (int)e.A1, (int)e.K, (int)e.stride, J,
               (int)(blockIdx.x - e.row0), red);
}

ENCX_DEV void wn_bwd_row(const float* v, const float* g, const float* dw, float* dv, float* dg, int cols, int acc,
                         int r, float* red) {
    const float* vr = v + (int64_t)r * cols;
    const float* dr = dw + (int64_t)r * cols;
    float ss = 0.f, dot = 0.f;
    for (int i = threadIdx.x; i < cols; i += NT) {
        ss = fmaf(vr[i], vr[i], ss);
        dot = fmaf(dr[i], vr[i], dot);
    }
    ss = block_sum(ss, red);
    dot = block_sum(dot, red);
    const float nrm = sqrtf(ss);
    const float gg = g[r];
    const float gd = dot / nrm;               // grad_g = sum(dw*v)/||v||
    const float sc = gg / nrm, proj = dot / ss;
    if (threadIdx.x == 0) dg[r] = acc ? dg[r] + gd : gd;
    float* o = dv + (int64_t)r * cols;
    for (int i = threadIdx.x; i < cols; i += NT) {
        float val = sc * (dr[i] - vr[i] * proj);  // (g/||v||)(dw - v * dot/||v||^2)
        o[i] = acc ? o[i] + val : val;
    }
}

__global__ __launch_bounds__(NT) void wn_bwd_kernel(const float* v, const float* g, const float* dw,
                                                    float* dv, float* dg, int cols, int acc) {
    __shared__ float red[16];
    wn_bwd_row(v, g, dw, dv, dg, cols, acc, blockIdx.x, red);
}

__global__ __launch_bounds__(NT) void wn_bwd_batch_kernel(const encx_wn_bwd_desc* d, int n) {
    __shared__ float red[16];
    const int li = wn_find(d, n, blockIdx.x);
    const encx_wn_bwd_desc e = d[li];
    wn_bwd_row(e.v, e.g, e.dw, e.dv, e.dg, (int)e.cols, (int)e.accumulate, (int)(blockIdx.x - e.row0), red);
}

}  // namespace

extern "C" {

int encx_weightnorm_fwd(const float* v, const float* g, float* wf, float* wp, int64_t A0,
                        int64_t A1, int64_t K, int64_t stride, encx_stream_t stream) {
    ENCX_REQUIRE(v && A0 > 0 && A1 > 0 && K > 0 && stride > 0);
    encx_prof_scope ps((hipStream_t)stream, 3.0 * A0 * A1 * K, 4.0 * A0 * A1 * K * (1 + (wf != nullptr) + (wp != nullptr)), "weightnorm", false);
    const int J = (int)cdiv(K, stride);
    hipLaunchKernelGGL(wn_fwd_kernel, dim3(A0), dim3(NT), 0, (hipStream_t)stream, v, g, wf, wp,
                       (int)A0, (int)A1, (int)K, (int)stride, J);
    ENCX_CHECK_LAUNCH();
    return 0;
}

int encx_weightnorm_bwd(const float* v, const float* g, const float* dw, float* dv, float* dg,
                        int64_t rows, int64_t cols, int accumulate, encx_stream_t stream) {
    ENCX_REQUIRE(v && g && dw && dv && dg && rows > 0 && cols > 0);
    encx_prof_scope ps((hipStream_t)stream, 4.0 * rows * cols, 4.0 * rows * cols * (accumulate ? 4 : 3), "weightnorm_bwd", false);
    hipLaunchKernelGGL(wn_bwd_kernel, dim3(rows), dim3(NT), 0, (hipStream_t)stream, v, g, dw, dv,
                       dg, (int)cols, accumulate);
    ENCX_CHECK_LAUNCH();
    return 0;
}

int encx_weightnorm_fwd_batch(const encx_wn_fwd_desc* layers, int64_t n_layers, int64_t rows_total,
                              encx_stream_t stream) {
    ENCX_REQUIRE(layers && n_layers > 0 && rows_total > 0);
    encx_prof_scope ps((hipStream_t)stream, 0.0, 0.0, "weightnorm_batch", false);
    hipLaunchKernelGGL(wn_fwd_batch_kernel, dim3((unsigned)rows_total), dim3(NT), 0, (hipStream_t)stream, layers,
                       (int)n_layers);
    ENCX_CHECK_LAUNCH();
    return 0;
}

int encx_weightnorm_bwd_batch(const encx_wn_bwd_desc* layers, int64_t n_layers, int64_t rows_total,
                              encx_stream_t stream) {
    ENCX_REQUIRE(layers && n_layers > 0 && rows_total > 0);
    encx_prof_scope ps((hipStream_t)stream, 0.0, 0.0, "weightnorm_bwd_batch", false);
    hipLaunchKernelGGL(wn_bwd_batch_kernel, dim3((unsigned)rows_total), dim3(NT), 0, (hipStream_t)stream, layers,
                       (int)n_layers);
    ENCX_CHECK_LAUNCH();
    return 0;
}

}  // extern "C"
