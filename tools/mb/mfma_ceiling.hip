// Ceilings of the fp32 MFMA inner loops used by the conv kernels (gfx950): (1) MFMA from
// registers only, (2) the conv2d forward's LDS-operand loop (one A ds_read per k-pair shared by
// TN MFMAs, TN B ds_reads at stride S) with no staging at all. Random operands (DVFS: zeros read
// high). Build: make -C tools/mb mfma_ceiling.
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef float f32x16 __attribute__((ext_vector_type(16)));
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

template <int NACC>
__global__ __launch_bounds__(256) void mfma_regs(const float* in, float* out, int iters) {
    float a = in[threadIdx.x], b = in[threadIdx.x + 256];
    f32x16 acc[NACC];
#pragma unroll
    for (int j = 0; j < NACC; ++j) acc[j] = (f32x16){0};
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int j = 0; j < NACC; ++j) acc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc[j], 0, 0, 0);
        a += 1e-7f;
    }
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < NACC; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) s += acc[j][r];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

// LDS-operand loop of c2_fwd (BM = 32, TN column tiles per wave, KF taps unrolled, stride S)
template <int TN, int S, int KF>
__global__ __launch_bounds__(256) void lds_loop(const float* in, float* out, int iters, int XR) {
    extern __shared__ float sm[];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, h = lane >> 5, l32 = lane & 31;
    for (int i = tid; i < 8 * XR + 8 * KF * 32; i += 256) sm[i] = in[i & 4095];
    __syncthreads();
    const float* Xs = sm;
    const float* Ws = sm + 8 * XR;
    int boff[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) boff[j] = ((wave * TN + j) * 32 + l32) * S;
    f32x16 acc[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[j] = (f32x16){0};
    for (int it = 0; it < iters; ++it) {
        for (int cp = 0; cp < 8; cp += 2) {
            const float* wk = Ws + (cp + h) * KF * 32 + l32;
            const float* xk = Xs + (cp + h) * XR;
#pragma unroll
            for (int kf = 0; kf < KF; ++kf) {
                const float av = wk[kf * 32];
                float bv[TN];
#pragma unroll
                for (int j = 0; j < TN; ++j) bv[j] = xk[boff[j] + kf];
#pragma unroll
                for (int j = 0; j < TN; ++j) acc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bv[j], acc[j], 0, 0, 0);
            }
        }
    }
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) s += acc[j][r];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <class F>
static double run(F f, double flops) {
    f();
    hipDeviceSynchronize();
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0, 0);
    for (int i = 0; i < 5; ++i) f();
    hipEventRecord(e1, 0);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    return flops * 5 / (ms * 1e-3) / 1e12;
}

int main() {
    float *in, *out;
    CK(hipMalloc(&in, 4096 * 4));
    CK(hipMalloc(&out, 4096 * 256 * 4));
    float h[4096];
    for (int i = 0; i < 4096; ++i) h[i] = (float)((i * 2654435761u) % 1000) / 1000.f - 0.5f;
    CK(hipMemcpy(in, h, sizeof h, hipMemcpyHostToDevice));
    const int iters = 2000;
    for (int wg : {256, 512, 1024, 2048}) {
        double f1 = 2.0 * 32 * 32 * 2 * 4.0 * iters * wg * 1;
        printf("regs  1 acc  %4d WGs: %6.1f TF/s\n", wg, run([&] { hipLaunchKernelGGL(mfma_regs<1>, dim3(wg), dim3(256), 0, 0, in, out, iters); }, f1));
        printf("regs  2 acc  %4d WGs: %6.1f TF/s\n", wg, run([&] { hipLaunchKernelGGL(mfma_regs<2>, dim3(wg), dim3(256), 0, 0, in, out, iters); }, 2 * f1));
        printf("regs  4 acc  %4d WGs: %6.1f TF/s\n", wg, run([&] { hipLaunchKernelGGL(mfma_regs<4>, dim3(wg), dim3(256), 0, 0, in, out, iters / 2); }, 2 * f1));
    }
    const int it2 = 200;
    for (int wg : {256, 512, 1024}) {
        // per WG per iteration: 4 waves x 4 cp-pairs x KF x TN MFMAs
        const int XR = 600;
        size_t lds = (8 * XR + 8 * 9 * 32) * 4;
        double f2 = 4096.0 * 4 * 4 * 9 * 2 * it2 * wg;
        printf("lds TN2 S2 KF9 %4d WGs: %6.1f TF/s\n", wg, run([&] { hipLaunchKernelGGL((lds_loop<2, 2, 9>), dim3(wg), dim3(256), lds, 0, in, out, it2, XR); }, f2));
        printf("lds TN4 S2 KF9 %4d WGs: %6.1f TF/s\n", wg, run([&] { hipLaunchKernelGGL((lds_loop<4, 2, 9>), dim3(wg), dim3(256), lds, 0, in, out, it2, XR); }, 2 * f2));
        printf("lds TN2 S1 KF9 %4d WGs: %6.1f TF/s\n", wg, run([&] { hipLaunchKernelGGL((lds_loop<2, 1, 9>), dim3(wg), dim3(256), lds, 0, in, out, it2, XR); }, f2));
        printf("lds TN1 S2 KF9 %4d WGs: %6.1f TF/s\n", wg, run([&] { hipLaunchKernelGGL((lds_loop<1, 2, 9>), dim3(wg), dim3(256), lds, 0, in, out, it2, XR); }, f2 / 2));
    }
    return 0;
}
