// Ceilings of the fp32 MFMA inner loops used by the conv kernels (gfx950): (1) MFMA from
// registers only, (2) the conv2d forward's LDS-operand loop (one A ds_read per k-pair shared by
// TN MFMAs, TN B ds_reads at stride S) with no staging at all. Random operands (DVFS: zeros read
// high). Build: make -C tools/mb mfma_ceiling.
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
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


// chunked version of lds_loop: per chunk optional barrier pair, optional LDS rewrite of Q quads per
// thread from registers, optional global prefetch of Q quads per thread (issued before the
// compute, consumed at the next chunk's rewrite)
template <int TN, int KF, int Q, int MODE>  // MODE bit0: barriers, bit1: LDS writes, bit2: global loads
__global__ __launch_bounds__(256) void chunk_loop(const float* in, float* out, int chunks, int XR, int CK) {
    extern __shared__ float sm[];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, h = lane >> 5, l32 = lane & 31;
    for (int i = tid; i < CK * XR + CK * KF * 32; i += 256) sm[i] = in[i & 4095];
    __syncthreads();
    const float* Xs = sm;
    const float* Ws = sm + CK * XR;
    int boff[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) boff[j] = ((wave * TN + j) * 32 + l32) * 2;
    f32x16 acc[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[j] = (f32x16){0};
    f32x4 rv[Q];
#pragma unroll
    for (int u = 0; u < Q; ++u) rv[u] = (f32x4){0.f, 0.f, 0.f, 0.f};
    const float* src = in + 64 * 1024 * (blockIdx.x & 63);
    for (int c = 0; c < chunks; ++c) {
        if (MODE & 1) __syncthreads();
        if (MODE & 2) {
#pragma unroll
            for (int u = 0; u < Q; ++u) *(f32x4*)(sm + ((u * 256 + tid) * 4) % (CK * XR)) = rv[u];
        }
        if (MODE & 1) __syncthreads();
        if (MODE & 4) {
#pragma unroll
            for (int u = 0; u < Q; ++u) rv[u] = *(const f32x4*)(src + ((c * Q + u) * 256 + tid) * 4 % (64 * 1024 - 4));
        }
        for (int cp = 0; cp < CK; cp += 2) {
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
#pragma unroll
    for (int u = 0; u < Q; ++u) s += rv[u][0] + rv[u][3];
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
    // chunked loops: 2976 WGs (d2 L1 forward), 12 chunks of CK = 8 combos, TN = 2
    {
        float* big;
        CK(hipMalloc(&big, (64 * 1024 * 64 + 4096) * 4));
        CK(hipMemset(big, 0, (64 * 1024 * 64 + 4096) * 4));
        CK(hipMemcpy(big, h, sizeof h, hipMemcpyHostToDevice));  // random MFMA operands (DVFS)
        const int wg = 2976, chunks = 12, CKc = 8, XR = 804;
        size_t lds = (CKc * XR + CKc * 9 * 32) * 4 + 2304;
        double f = 4096.0 * 4 * (CKc / 2) * 9 * 2 * chunks * wg;
        printf("chunk none           : %6.1f TF/s\n", run([&] { hipLaunchKernelGGL((chunk_loop<2, 9, 8, 0>), dim3(wg), dim3(256), lds, 0, big, out, chunks, XR, CKc); }, f));
        printf("chunk barriers       : %6.1f TF/s\n", run([&] { hipLaunchKernelGGL((chunk_loop<2, 9, 8, 1>), dim3(wg), dim3(256), lds, 0, big, out, chunks, XR, CKc); }, f));
        printf("chunk bar+lds        : %6.1f TF/s\n", run([&] { hipLaunchKernelGGL((chunk_loop<2, 9, 8, 3>), dim3(wg), dim3(256), lds, 0, big, out, chunks, XR, CKc); }, f));
        printf("chunk bar+lds+gload  : %6.1f TF/s\n", run([&] { hipLaunchKernelGGL((chunk_loop<2, 9, 8, 7>), dim3(wg), dim3(256), lds, 0, big, out, chunks, XR, CKc); }, f));
        printf("chunk bar+gload      : %6.1f TF/s\n", run([&] { hipLaunchKernelGGL((chunk_loop<2, 9, 8, 5>), dim3(wg), dim3(256), lds, 0, big, out, chunks, XR, CKc); }, f));
        printf("chunk all TN4        : %6.1f TF/s\n", run([&] { hipLaunchKernelGGL((chunk_loop<4, 9, 8, 7>), dim3(wg / 2), dim3(256), lds, 0, big, out, chunks, XR, CKc); }, f));
        printf("chunk all CK16       : %6.1f TF/s\n", run([&] { hipLaunchKernelGGL((chunk_loop<2, 9, 8, 7>), dim3(wg), dim3(256), (16 * XR + 16 * 9 * 32) * 4, 0, big, out, chunks / 2, XR, 16); }, f));
        printf("chunk none 1 WG/CU-ish (lds 100K): %6.1f TF/s\n", run([&] { hipLaunchKernelGGL((chunk_loop<2, 9, 8, 0>), dim3(wg), dim3(256), 100000, 0, big, out, chunks, XR, CKc); }, f));
    }
    return 0;
}
