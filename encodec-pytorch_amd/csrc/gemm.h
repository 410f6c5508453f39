// Generic LDS-staged fp32 MFMA GEMM skeleton, C[M][N] = sum_k A(m,k) B(k,n), with operand
// loaders and the epilogue supplied as functors (implicit-GEMM style): the mel/STFT loss
// kernels build their A operands (framed, reflect-padded audio; |X|^2; d mel) on the fly
// while staging, so no im2col / intermediate tensor ever reaches HBM.
//
// Tiles: BM x BN per 256-thread workgroup (4 waves as WM x WN), BK-deep LDS stages,
// v_mfma_f32_32x32x2_f32 (exact fp32). Loader contract:
//   float a(int m, int k) const; static constexpr bool A_K_FAST;  // coalescing order
//   float b(int k, int n) const; static constexpr bool B_N_FAST;
// Epilogue: void operator()(int m, int n, float v) const  (only for m < M, n < N).
#pragma once
#include "common.h"

template <int BM, int BN, int WM, int WN, int BK, class LD, class EP>
__global__ __launch_bounds__(256) void gemm_kernel(LD ld, EP ep, int M, int N, int Kred) {
    constexpr int TM = BM / WM / 32, TN = BN / WN / 32;
    __shared__ float As[BK][BM + 1];
    __shared__ float Bs[BK][BN + 1];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm0 = (wave / WN) * TM * 32, wn0 = (wave % WN) * TN * 32;
    const int m0 = blockIdx.y * BM, n0 = blockIdx.x * BN;
    const int h = lane >> 5, l32 = lane & 31;
    f32x16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = (f32x16){0};
    for (int k0 = 0; k0 < Kred; k0 += BK) {
        __syncthreads();
        for (int i = tid; i < BM * BK; i += 256) {
            int m, k;
            if (LD::A_K_FAST) { m = i / BK; k = i - m * BK; }
            else { k = i / BM; m = i - k * BM; }
            int gm = m0 + m, gk = k0 + k;
            As[k][m] = (gm < M && gk < Kred) ? ld.a(gm, gk) : 0.f;
        }
        for (int i = tid; i < BN * BK; i += 256) {
            int n, k;
            if (LD::B_N_FAST) { k = i / BN; n = i - k * BN; }
            else { n = i / BK; k = i - n * BK; }
            int gn = n0 + n, gk = k0 + k;
            Bs[k][n] = (gn < N && gk < Kred) ? ld.b(gk, gn) : 0.f;
        }
        __syncthreads();
#pragma unroll
        for (int kp = 0; kp < BK; kp += 2) {
            float av[TM], bv[TN];
#pragma unroll
            for (int i = 0; i < TM; ++i) av[i] = As[kp + h][wm0 + i * 32 + l32];
#pragma unroll
            for (int j = 0; j < TN; ++j) bv[j] = Bs[kp + h][wn0 + j * 32 + l32];
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j) acc[i][j] = mfma32(av[i], bv[j], acc[i][j]);
        }
    }
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int n = n0 + wn0 + j * 32 + l32;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int m = m0 + wm0 + i * 32 + mfma_row(r, lane);
                if (m < M && n < N) ep(m, n, acc[i][j][r]);
            }
        }
}

// launch with a tile picked from the problem shape
template <class LD, class EP>
int gemm_launch(const LD& ld, const EP& ep, int M, int N, int Kred, hipStream_t st) {
    // 128x128 tiles when they still give >= 2 workgroups per CU, else 64x64 (256 CUs)
    const int64_t big = cdiv(N, 128) * cdiv(M, 128);
    if (N <= 48) {
        hipLaunchKernelGGL((gemm_kernel<128, 32, 4, 1, 32, LD, EP>), dim3(cdiv(N, 32), cdiv(M, 128)),
                           dim3(256), 0, st, ld, ep, M, N, Kred);
    } else if (N <= 96) {
        hipLaunchKernelGGL((gemm_kernel<128, 64, 2, 2, 32, LD, EP>), dim3(cdiv(N, 64), cdiv(M, 128)),
                           dim3(256), 0, st, ld, ep, M, N, Kred);
    } else if (big < 512) {
        hipLaunchKernelGGL((gemm_kernel<64, 64, 2, 2, 32, LD, EP>), dim3(cdiv(N, 64), cdiv(M, 64)),
                           dim3(256), 0, st, ld, ep, M, N, Kred);
    } else {
        hipLaunchKernelGGL((gemm_kernel<128, 128, 2, 2, 32, LD, EP>), dim3(cdiv(N, 128), cdiv(M, 128)),
                           dim3(256), 0, st, ld, ep, M, N, Kred);
    }
    ENCX_CHECK_LAUNCH();
    return 0;
}
