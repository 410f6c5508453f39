// Microbenchmark: where the time of one LSTM forward step launch goes (csrc/lstm.hip
// lstm_fwd_wave at the config-3 size: H 512, L 2, B 32, 256 workgroups of 8 waves). The step body
// is restated with switches that drop one part at a time, and 76 dependent launches are timed
// (the diagonal wavefront of 75 frames x 2 layers) against a chain of empty launches:
//   FLAGS 1: no weight loads (a register constant)   2: no [x | h] loads
//         4: no MFMA chain                           8: no LDS reduction / gates / stores
// hipcc --offload-arch=gfx950 -O3 lstm_step_mb.hip -o lstm_step_mb && ./lstm_step_mb
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)
typedef float f32x4v __attribute__((ext_vector_type(4)));

constexpr int UNITS = 4, FW = 8, H = 512, B = 32, T = 75, L = 2, G = 8, RT = 2;

__device__ __forceinline__ f32x4v mfma16(float a, float b, f32x4v c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ float at4(const float4& v, int s) { return s == 0 ? v.x : s == 1 ? v.y : s == 2 ? v.z : v.w; }
__device__ __forceinline__ float sigm(float x) { return 1.f / (1.f + expf(-x)); }

template <int FLAGS>
__global__ __launch_bounds__(FW * 64) void step(const float* xt, const float* wcat, float* Y, float* C, int k) {
    const int l = blockIdx.y, t = k - l;
    if (t < 0 || t >= T) return;
    __shared__ float red[FW][64][17];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, col = lane & 15, kk = lane >> 4;
    const int u0 = blockIdx.x * UNITS, K = 2 * H;
    const long BTH = (long)B * T * H;
    const float* W = wcat + (long)l * 4 * H * K;
    const float* xin = l == 0 ? xt : Y + (long)(l - 1) * BTH;
    float* Yl = Y + (long)l * BTH;
    const int tp = t > 0 ? t - 1 : 0;
    const int j = (col >> 2) * H + u0 + (col & 3);
    float4 wv[G], hv[RT][G];
#pragma unroll
    for (int g = 0; g < G; ++g) {
        const int kq = (wave + FW * g) * 16 + 4 * kk;
        wv[g] = (FLAGS & 1) ? make_float4(1e-3f, 2e-3f, 3e-3f, 4e-3f) : *(const float4*)(W + (long)j * K + kq);
        const bool rec = kq >= H;
        const float* src = rec ? Yl : xin;
        const int ts = rec ? tp : t, kc = rec ? kq - H : kq;
#pragma unroll
        for (int r = 0; r < RT; ++r) {
            const int row = r * 16 + col;
            hv[r][g] = (FLAGS & 2) ? make_float4(0.5f, 0.25f, 0.125f, 1.f)
                                   : *(const float4*)(src + ((long)row * T + ts) * H + kc);
        }
    }
    f32x4v acc[RT];
#pragma unroll
    for (int r = 0; r < RT; ++r) acc[r] = (f32x4v){0.f, 0.f, 0.f, 0.f};
    if (!(FLAGS & 4)) {
#pragma unroll
        for (int g = 0; g < G; ++g)
#pragma unroll
            for (int s = 0; s < 4; ++s)
#pragma unroll
                for (int r = 0; r < RT; ++r) acc[r] = mfma16(at4(hv[r][g], s), at4(wv[g], s), acc[r]);
    } else {
#pragma unroll
        for (int g = 0; g < G; ++g)
#pragma unroll
            for (int r = 0; r < RT; ++r) acc[r][0] += hv[r][g].x * wv[g].x;
    }
    if (FLAGS & 8) {
        if (acc[0][0] == 12345.f) Yl[tid] = acc[1][1];  // keep the chain live
        return;
    }
#pragma unroll
    for (int r = 0; r < RT; ++r)
#pragma unroll
        for (int q = 0; q < 4; ++q) red[wave][r * 16 + kk * 4 + q][col] = acc[r][q];
    __syncthreads();
    const int pb = tid / UNITS, pu = u0 + (tid - pb * UNITS);
    if (pb < B) {
        float pre[4];
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            float s = 0.f;
            for (int w = 0; w < FW; ++w) s += red[w][pb][g * 4 + pu - u0];
            pre[g] = s;
        }
        const long po = ((long)pb * T + t) * H + pu;
        const float c = sigm(pre[1]) * (t > 0 ? C[po - H] : 0.f) + sigm(pre[0]) * tanhf(pre[2]);
        C[(long)l * BTH + po] = c;
        Yl[po] = sigm(pre[3]) * tanhf(c);
    }
}
__global__ void empty_kernel(float* p, int k) {
    if (p[0] == 12345.f && k < 0) p[1] = 0.f;
}

template <int FLAGS>
float run(const float* xt, const float* w, float* Y, float* C, hipEvent_t e0, hipEvent_t e1, int reps) {
    const dim3 grid(H / UNITS, L);
    for (int k = 0; k < T + L - 1; ++k) hipLaunchKernelGGL(step<FLAGS>, grid, dim3(FW * 64), 0, 0, xt, w, Y, C, k);
    CK(hipEventRecord(e0));
    for (int rr = 0; rr < reps; ++rr)
        for (int k = 0; k < T + L - 1; ++k) hipLaunchKernelGGL(step<FLAGS>, grid, dim3(FW * 64), 0, 0, xt, w, Y, C, k);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    return ms * 1e3f / (reps * (T + L - 1));
}

int main() {
    float *xt, *w, *Y, *C;
    CK(hipMalloc(&xt, (size_t)B * T * H * 4));
    CK(hipMalloc(&w, (size_t)L * 4 * H * 2 * H * 4));
    CK(hipMalloc(&Y, (size_t)L * B * T * H * 4));
    CK(hipMalloc(&C, (size_t)L * B * T * H * 4));
    CK(hipMemset(xt, 0, (size_t)B * T * H * 4));
    CK(hipMemset(w, 0, (size_t)L * 4 * H * 2 * H * 4));
    CK(hipMemset(Y, 0, (size_t)L * B * T * H * 4));
    CK(hipMemset(C, 0, (size_t)L * B * T * H * 4));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int reps = 20;
    // empty launches of the same grid
    {
        const dim3 grid(H / UNITS, L);
        CK(hipEventRecord(e0));
        for (int i = 0; i < reps * (T + L - 1); ++i) hipLaunchKernelGGL(empty_kernel, grid, dim3(FW * 64), 0, 0, Y, i);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        printf("empty launch             %6.2f us\n", ms * 1e3f / (reps * (T + L - 1)));
    }
    printf("full step                %6.2f us\n", run<0>(xt, w, Y, C, e0, e1, reps));
    printf("no weight loads          %6.2f us\n", run<1>(xt, w, Y, C, e0, e1, reps));
    printf("no [x|h] loads           %6.2f us\n", run<2>(xt, w, Y, C, e0, e1, reps));
    printf("no loads                 %6.2f us\n", run<3>(xt, w, Y, C, e0, e1, reps));
    printf("no MFMA                  %6.2f us\n", run<4>(xt, w, Y, C, e0, e1, reps));
    printf("no reduce/gates/stores   %6.2f us\n", run<8>(xt, w, Y, C, e0, e1, reps));
    printf("loads only               %6.2f us\n", run<12>(xt, w, Y, C, e0, e1, reps));
    printf("MFMA only                %6.2f us\n", run<11>(xt, w, Y, C, e0, e1, reps));
    return 0;
}
