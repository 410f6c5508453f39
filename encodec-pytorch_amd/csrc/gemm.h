// Generic LDS-staged fp32 MFMA GEMM skeleton, C[M][N] = sum_k A(m,k) B(k,n), with operand
// loaders and the epilogue supplied as functors (implicit-GEMM style): the mel/STFT loss,
// the EMA codebook sums and the low-rate (T <= 128) conv layers build their operands on the
// fly while staging (framed audio, |X|^2, one-hot codes, im2col windows), so no intermediate
// tensor reaches HBM.
//
// Tiles: BM x BN per 256-thread workgroup (4 waves as WM x WN), BK-deep LDS stages,
// v_mfma_f32_32x32x2_f32 (exact fp32). Split-K: workgroup z covers k in
// [z*kchunk, (z+1)*kchunk); the epilogue sees blockIdx.z and writes its own partial slab.
// Loader contract:
//   float a(int m, int k) const; static constexpr bool A_K_FAST;  // coalescing order
//   float b(int k, int n) const; static constexpr bool B_N_FAST;
// Epilogue: void operator()(int m, int n, float v) const  (only for m < M, n < N).
#pragma once
#include "common.h"

// epilogue functors that load operands declare `static constexpr int NPRE` floats per element
// and split into pre(m, n, float*) / post(m, n, v, const float*)
template <class EP, class = void>
struct ep_npre { static constexpr int value = 0; };
template <class EP>
struct ep_npre<EP, decltype((void)EP::NPRE)> { static constexpr int value = EP::NPRE; };

// loaders that can hand over 4 consecutive elements along their fast dim declare
// `static constexpr bool VEC = true` and a4(m, k) / b4(k, n) (f32x4 of (m..m+3 or k..k+3) /
// (k..k+3 or n..n+3)); the kernel then stages quads (one loader call per 4 elements) and takes
// the scalar path only for quads that cross the matrix edge
template <class LD, class = void>
struct ld_vec { static constexpr bool value = false; };
template <class LD>
struct ld_vec<LD, decltype((void)LD::VEC)> { static constexpr bool value = LD::VEC; };

template <int BM, int BN, int WM, int WN, int BK, class LD, class EP>
__global__ __launch_bounds__(256) void gemm_kernel(LD ld, EP ep, int M, int N, int Kred, int kchunk) {
    constexpr int TM = BM / WM / 32, TN = BN / WN / 32;
    __shared__ float As[BK][BM + 1];
    __shared__ float Bs[BK][BN + 1];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm0 = (wave / WN) * TM * 32, wn0 = (wave % WN) * TN * 32;
    const int m0 = blockIdx.y * BM, n0 = blockIdx.x * BN;
    const int kbeg = blockIdx.z * kchunk, kend = min(Kred, kbeg + kchunk);
    const int h = lane >> 5, l32 = lane & 31;
    f32x16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = (f32x16){0};
    // register-prefetch pipeline: the next BK slice's operands are fetched (through the
    // loaders) while the current slice runs on the MFMA units
    constexpr int EA = BM * BK / 256, EB = BN * BK / 256;
    static_assert(EA * 256 == BM * BK && EB * 256 == BN * BK, "tile/thread mismatch");
    float ra[EA], rb[EB];
    // Every element is loaded from a clamped in-range index and the value selected afterwards:
    // a bounds test around each loader call compiles to an exec-masked branch per element, and
    // a loader that transforms the loaded value (ELU, |X|^2, ...) then waits for each load
    // before issuing the next (one memory round trip per element instead of one per fetch).
    constexpr bool VEC = ld_vec<LD>::value;
    static_assert(!VEC || (EA % 4 == 0 && EB % 4 == 0), "quad staging");
    // quad e of this thread: its first element (m, k) and the fast dim
    auto quad_a = [&](int e, int& m, int& k) {
        const int i = tid + e * 256;
        if (LD::A_K_FAST) { m = i / (BK / 4); k = (i - m * (BK / 4)) * 4; }
        else { k = i / (BM / 4); m = (i - k * (BM / 4)) * 4; }
    };
    auto quad_b = [&](int e, int& k, int& n) {
        const int i = tid + e * 256;
        if (LD::B_N_FAST) { k = i / (BN / 4); n = (i - k * (BN / 4)) * 4; }
        else { n = i / (BK / 4); k = (i - n * (BK / 4)) * 4; }
    };
    auto fetch = [&](int k0) {
        if constexpr (VEC) {
#pragma unroll
            for (int e = 0; e < EA / 4; ++e) {
                int m, k;
                quad_a(e, m, k);
                const int gm = m0 + m, gk = k0 + k;
                const bool whole = LD::A_K_FAST ? (gm < M && gk + 3 < kend) : (gm + 3 < M && gk < kend);
                f32x4 v;
                if (whole) {
                    v = ld.a4(gm, gk);
                } else {
#pragma unroll
                    for (int c = 0; c < 4; ++c) {
                        const int mm = LD::A_K_FAST ? gm : gm + c, kk = LD::A_K_FAST ? gk + c : gk;
                        const float t = ld.a(mm < M ? mm : M - 1, kk < kend ? kk : kend - 1);
                        v[c] = (mm < M && kk < kend) ? t : 0.f;
                    }
                }
#pragma unroll
                for (int c = 0; c < 4; ++c) ra[4 * e + c] = v[c];
            }
#pragma unroll
            for (int e = 0; e < EB / 4; ++e) {
                int k, n;
                quad_b(e, k, n);
                const int gn = n0 + n, gk = k0 + k;
                const bool whole = LD::B_N_FAST ? (gk < kend && gn + 3 < N) : (gk + 3 < kend && gn < N);
                f32x4 v;
                if (whole) {
                    v = ld.b4(gk, gn);
                } else {
#pragma unroll
                    for (int c = 0; c < 4; ++c) {
                        const int nn = LD::B_N_FAST ? gn + c : gn, kk = LD::B_N_FAST ? gk : gk + c;
                        const float t = ld.b(kk < kend ? kk : kend - 1, nn < N ? nn : N - 1);
                        v[c] = (nn < N && kk < kend) ? t : 0.f;
                    }
                }
#pragma unroll
                for (int c = 0; c < 4; ++c) rb[4 * e + c] = v[c];
            }
            return;
        }
#pragma unroll
        for (int e = 0; e < EA; ++e) {
            const int i = tid + e * 256;
            int m, k;
            if (LD::A_K_FAST) { m = i / BK; k = i - m * BK; }
            else { k = i / BM; m = i - k * BM; }
            const int gm = m0 + m, gk = k0 + k;
            const bool ok = gm < M && gk < kend;
            const float v = ld.a(gm < M ? gm : M - 1, gk < kend ? gk : kend - 1);
            ra[e] = ok ? v : 0.f;
        }
#pragma unroll
        for (int e = 0; e < EB; ++e) {
            const int i = tid + e * 256;
            int n, k;
            if (LD::B_N_FAST) { k = i / BN; n = i - k * BN; }
            else { n = i / BK; k = i - n * BK; }
            const int gn = n0 + n, gk = k0 + k;
            const bool ok = gn < N && gk < kend;
            const float v = ld.b(gk < kend ? gk : kend - 1, gn < N ? gn : N - 1);
            rb[e] = ok ? v : 0.f;
        }
    };
    if (kbeg < kend) fetch(kbeg);
    for (int k0 = kbeg; k0 < kend; k0 += BK) {
        __syncthreads();
        if constexpr (VEC) {
#pragma unroll
            for (int e = 0; e < EA / 4; ++e) {
                int m, k;
                quad_a(e, m, k);
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    if (LD::A_K_FAST) As[k + c][m] = ra[4 * e + c];
                    else As[k][m + c] = ra[4 * e + c];
                }
            }
#pragma unroll
            for (int e = 0; e < EB / 4; ++e) {
                int k, n;
                quad_b(e, k, n);
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    if (LD::B_N_FAST) Bs[k][n + c] = rb[4 * e + c];
                    else Bs[k + c][n] = rb[4 * e + c];
                }
            }
        } else {
#pragma unroll
        for (int e = 0; e < EA; ++e) {
            const int i = tid + e * 256;
            int m, k;
            if (LD::A_K_FAST) { m = i / BK; k = i - m * BK; }
            else { k = i / BM; m = i - k * BM; }
            As[k][m] = ra[e];
        }
#pragma unroll
        for (int e = 0; e < EB; ++e) {
            const int i = tid + e * 256;
            int n, k;
            if (LD::B_N_FAST) { k = i / BN; n = i - k * BN; }
            else { n = i / BK; k = i - n * BK; }
            Bs[k][n] = rb[e];
        }
        }
        __syncthreads();
        if (k0 + BK < kend) fetch(k0 + BK);
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
            if constexpr (ep_npre<EP>::value > 0) {
                // two-phase epilogue: all of the tile's operand loads, then all of its stores
                constexpr int NP = ep_npre<EP>::value;
#pragma unroll
                for (int r0 = 0; r0 < 16; r0 += 8) {  // 8 rows' loads in flight together
                    float pl[8][NP];
#pragma unroll
                    for (int q = 0; q < 8; ++q) {
                        const int m = m0 + wm0 + i * 32 + mfma_row(r0 + q, lane);
                        if (m < M && n < N) ep.pre(m, n, pl[q]);
                    }
#pragma unroll
                    for (int q = 0; q < 8; ++q) {
                        const int m = m0 + wm0 + i * 32 + mfma_row(r0 + q, lane);
                        if (m < M && n < N) ep.post(m, n, acc[i][j][r0 + q], pl[q]);
                    }
                }
            } else {
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int m = m0 + wm0 + i * 32 + mfma_row(r, lane);
                    if (m < M && n < N) ep(m, n, acc[i][j][r]);
                }
            }
        }
}

struct GemmShape {
    int BM, BN;
    int64_t blocks;
};

// tile choice shared by gemm_launch and split-K planners: 128x128 while that still gives
// >= 2 workgroups per CU (256 CUs), else 64x64; narrow N gets 128x32 / 128x64
static inline GemmShape gemm_shape(int M, int N) {
    GemmShape s;
    if (N <= 48) { s.BM = 128; s.BN = 32; }
    else if (N <= 96) { s.BM = 128; s.BN = 64; }
    else if (cdiv(N, 128) * cdiv(M, 128) < 512) { s.BM = 64; s.BN = 64; }
    else { s.BM = 128; s.BN = 128; }
    s.blocks = cdiv(N, s.BN) * cdiv(M, s.BM);
    return s;
}

// split count that brings the grid to ~1024 workgroups, each with >= min_k reduction depth
static inline int gemm_splits(int M, int N, int Kred, int min_k = 256, int max_splits = 32) {
    GemmShape s = gemm_shape(M, N);
    int sp = (int)cdiv(1024, s.blocks);
    int cap = Kred / min_k;
    if (sp > cap) sp = cap;
    if (sp > max_splits) sp = max_splits;
    return sp < 1 ? 1 : sp;
}

template <class LD, class EP>
int gemm_launch(const LD& ld, const EP& ep, int M, int N, int Kred, hipStream_t st, int splits = 1) {
    GemmShape s = gemm_shape(M, N);
    const int kchunk = splits > 1 ? (int)(cdiv(cdiv(Kred, splits), 32) * 32) : Kred;
    const int z = (int)cdiv(Kred, kchunk);
    if (s.BN == 32) {
        hipLaunchKernelGGL((gemm_kernel<128, 32, 4, 1, 32, LD, EP>), dim3(cdiv(N, 32), cdiv(M, 128), z),
                           dim3(256), 0, st, ld, ep, M, N, Kred, kchunk);
    } else if (s.BN == 64 && s.BM == 128) {
        hipLaunchKernelGGL((gemm_kernel<128, 64, 2, 2, 32, LD, EP>), dim3(cdiv(N, 64), cdiv(M, 128), z),
                           dim3(256), 0, st, ld, ep, M, N, Kred, kchunk);
    } else if (s.BN == 64) {
        hipLaunchKernelGGL((gemm_kernel<64, 64, 2, 2, 32, LD, EP>), dim3(cdiv(N, 64), cdiv(M, 64), z),
                           dim3(256), 0, st, ld, ep, M, N, Kred, kchunk);
    } else {
        hipLaunchKernelGGL((gemm_kernel<128, 128, 2, 2, 32, LD, EP>), dim3(cdiv(N, 128), cdiv(M, 128), z),
                           dim3(256), 0, st, ld, ep, M, N, Kred, kchunk);
    }
    ENCX_CHECK_LAUNCH();
    return 0;
}

// 128x128 tiles regardless of the grid size, split over k to ~1024 workgroups: for the deep
// weight-gradient GEMMs whose 128-tile grid alone is small (e.g. the LSTM's [4H] x [2H+1] over
// B*T), 128x128 halves the staged bytes per MFMA against the 64x64 tile gemm_shape picks.
static inline int gemm_splits_128(int M, int N, int Kred, int min_k = 256, int max_splits = 32) {
    const int blocks = (int)(cdiv(N, 128) * cdiv(M, 128));
    int sp = (int)cdiv(1024, blocks);
    const int cap = Kred / min_k;
    if (sp > cap) sp = cap;
    if (sp > max_splits) sp = max_splits;
    return sp < 1 ? 1 : sp;
}
template <class LD, class EP>
int gemm_launch_128(const LD& ld, const EP& ep, int M, int N, int Kred, hipStream_t st, int splits) {
    const int kchunk = splits > 1 ? (int)(cdiv(cdiv(Kred, splits), 32) * 32) : Kred;
    const int z = (int)cdiv(Kred, kchunk);
    hipLaunchKernelGGL((gemm_kernel<128, 128, 2, 2, 32, LD, EP>), dim3(cdiv(N, 128), cdiv(M, 128), z),
                       dim3(256), 0, st, ld, ep, M, N, Kred, kchunk);
    ENCX_CHECK_LAUNCH();
    return 0;
}

// number of k-slabs gemm_launch actually uses for a requested split count
static inline int gemm_slabs(int Kred, int splits) {
    if (splits <= 1) return 1;
    const int kchunk = (int)(cdiv(cdiv(Kred, splits), 32) * 32);
    return (int)cdiv(Kred, kchunk);
}
