// Residual vector quantizer kernels (quantization/core_vq.py).
//
//  rvq_argmin_mfma  EuclideanCodebook.quantize (core_vq.py:181-189). A 64-frame x 128-code tile
//                   of dot products on v_mfma_f32_32x32x2_f32, then per element the reference's
//                   own fp32 expression v = (|x|^2 - 2 x.e) + |e|^2, packed into an order-
//                   preserving 64-bit key (dist bits << 32 | code) so that a wave min-reduction
//                   and one 64-bit atomicMin per frame give argmin with FIRST-index tie break
//                   exactly like torch.max(dim=-1) on -v. Integer atomics: order-independent.
//  rvq_argmin_direct kmeans' direct form -sum_d (x-e)^2 (core_vq.py:86-91), VALU.
//  rvq_apply        STE / residual / output / commit-loss pieces of one layer (:301-324,:346-349)
//  bucket_sum       per-code counts and sums of the assigned frames, one wave per code, frames
//                   visited in ascending order (deterministic), used by the EMA update (:227-235)
//                   and by kmeans (:92-100).
#include "common.h"
#include "prof.h"
#include "gemm.h"

namespace {

constexpr int NT = 256;

struct Rows {  // x_n[d] = p[b*sB + t*sT + d*sD], n = b*Tf + t
    const float* p;
    int64_t sB, sT, sD;
    int Tf;
    FastDiv fTf;
    ENCX_DEV float at(int n, int d) const {
        const int b = (int)fdiv((uint32_t)n, fTf), t = n - b * Tf;
        return p[b * sB + t * sT + d * sD];
    }
};

ENCX_DEV uint32_t ord_key(float f) {
    uint32_t u = __float_as_uint(f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
ENCX_DEV uint64_t umin64(uint64_t a, uint64_t b) { return a < b ? a : b; }
ENCX_DEV uint64_t shfl_xor64(uint64_t v, int o) {
    uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
    lo = __shfl_xor(lo, o, 64);
    hi = __shfl_xor(hi, o, 64);
    return ((uint64_t)hi << 32) | lo;
}

// One workgroup = 64 frames x 64 codes with the whole D staged once (no chunk loop): frames
// are loaded along t (the [B][D][T] latent is t-contiguous) into As[d][frame], codes along d
// into Bs[d][code] (row stride 65), so a workgroup does one load phase, one barrier and 64 MFMA
// k-steps; its 4 waves are 2 x 2 tiles of 32 x 32. 66 KB of LDS: two workgroups per CU, so one
// hides the other's LDS and load latency (at 128 codes, 100 KB, one per CU: MFMA busy 0.08).
// 38 x 16 = 608 workgroups at N = 2400.
constexpr int AR_ROWS = 64, AR_CODES = 64, AR_BS = AR_CODES + 1;
constexpr int AR_PER = 8;    // staging loads in flight per thread (scalar code path)
constexpr int AR_XPER = 32;  // frame-element loads in flight per thread
constexpr int AR_EPER = 16;  // code quads in flight per thread

__global__ __launch_bounds__(NT) void rvq_argmin_mfma(Rows x, const float* embed, uint64_t* keys,
                                                      int N, int D, int Kc) {
    extern __shared__ float sm[];
    float* As = sm;                        // [D][AR_ROWS]
    float* Bs = As + D * AR_ROWS;          // [D][AR_BS]
    float* xx = Bs + D * AR_BS;            // [AR_ROWS]
    float* ee = xx + AR_ROWS;              // [AR_CODES]
    __shared__ uint64_t part[2][AR_ROWS];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int n0 = blockIdx.x * AR_ROWS, k0 = blockIdx.y * AR_CODES;
    const int h = lane >> 5, l32 = lane & 31;
    const int wm0 = (wave >> 1) * 32, wn0 = (wave & 1) * 32;
    // staging: AR_XPER (frames) / AR_EPER (code quads) loads in flight per thread from clamped
    // addresses, values selected after the load (a branch around each load serialises the
    // latency: one round trip per element); at D = 128 each operand is ONE round of loads
    {
        const int r = tid & (AR_ROWS - 1), dq = tid / AR_ROWS, n = n0 + r;  // frame fixed per thread
        const bool okn = n < N;
        const int nc = okn ? n : N - 1;
        const int bb = nc / x.Tf, tt = nc - bb * x.Tf;
        const float* xp = x.p + bb * x.sB + tt * x.sT;
        constexpr int DSTEP = NT / AR_ROWS;
        for (int d0 = 0; d0 < D; d0 += DSTEP * AR_XPER) {
            float v[AR_XPER];
#pragma unroll
            for (int q = 0; q < AR_XPER; ++q) {
                const int d = d0 + dq + DSTEP * q;
                const float t = xp[(int64_t)(d < D ? d : D - 1) * x.sD];
                v[q] = (okn && d < D) ? t : 0.f;
            }
#pragma unroll
            for (int q = 0; q < AR_XPER; ++q) {
                const int d = d0 + dq + DSTEP * q;
                if (d < D) As[d * AR_ROWS + r] = v[q];
            }
        }
    }
    if ((D & 3) == 0) {  // codes as 16-byte quads along d, transposed into Bs[d][code]
        const int D4 = D >> 2;
        for (int i0 = 0; i0 < AR_CODES * D4; i0 += NT * AR_EPER) {
            f32x4 v[AR_EPER];
#pragma unroll
            for (int q = 0; q < AR_EPER; ++q) {
                const int i = i0 + q * NT + tid;
                const int c = i / D4, d4 = i - c * D4, k = k0 + c;
                const bool ok = i < AR_CODES * D4 && k < Kc;
                const f32x4 t = ld4u(embed + (ok ? (int64_t)k * D + 4 * d4 : 0));
                v[q] = ok ? t : (f32x4){0.f, 0.f, 0.f, 0.f};
            }
#pragma unroll
            for (int q = 0; q < AR_EPER; ++q) {
                const int i = i0 + q * NT + tid;
                const int c = i / D4, d4 = i - c * D4;
                if (i < AR_CODES * D4) {
#pragma unroll
                    for (int e = 0; e < 4; ++e) Bs[(4 * d4 + e) * AR_BS + c] = v[q][e];
                }
            }
        }
    } else
    for (int i0 = 0; i0 < AR_CODES * D; i0 += NT * AR_PER) {
        float v[AR_PER];
#pragma unroll
        for (int q = 0; q < AR_PER; ++q) {
            const int i = i0 + q * NT + tid;
            const int c = i / D, d = i - c * D, k = k0 + c;
            const bool ok = i < AR_CODES * D && k < Kc;
            const float t = embed[ok ? (int64_t)k * D + d : 0];
            v[q] = ok ? t : 0.f;
        }
#pragma unroll
        for (int q = 0; q < AR_PER; ++q) {
            const int i = i0 + q * NT + tid;
            const int c = i / D, d = i - c * D;
            if (i < AR_CODES * D) Bs[d * AR_BS + c] = v[q];
        }
    }
    __syncthreads();
    // |x|^2 and |e|^2 in ascending d (fmaf chain)
    if (tid < AR_ROWS) {
        float v = 0.f;
        for (int d = 0; d < D; ++d) v = fmaf(As[d * AR_ROWS + tid], As[d * AR_ROWS + tid], v);
        xx[tid] = v;
    } else if (tid < AR_ROWS + AR_CODES) {
        const int c = tid - AR_ROWS;
        float v = 0.f;
        for (int d = 0; d < D; ++d) v = fmaf(Bs[d * AR_BS + c], Bs[d * AR_BS + c], v);
        ee[c] = v;
    }
    f32x16 acc[1];
    acc[0] = (f32x16){0};
    const float* ap = As + h * AR_ROWS + wm0 + l32;
    const float* bp = Bs + h * AR_BS + wn0 + l32;
#pragma unroll 4
    for (int dp = 0; dp < D; dp += 2) {
        const float av = ap[dp * AR_ROWS];
        acc[0] = mfma32(av, bp[dp * AR_BS], acc[0]);
    }
    __syncthreads();  // xx / ee visible
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int row = wm0 + mfma_row(r, lane);
        uint64_t best = ~0ull;
#pragma unroll
        for (int j = 0; j < 1; ++j) {
            const int c = wn0 + j * 32 + l32, k = k0 + c;
            if (k < Kc) {
                const float v = (xx[row] - 2.f * acc[j][r]) + ee[c];
                best = umin64(best, ((uint64_t)ord_key(v) << 32) | (uint32_t)k);
            }
        }
#pragma unroll
        for (int o = 16; o > 0; o >>= 1) best = umin64(best, shfl_xor64(best, o));
        if (l32 == 0) part[wave & 1][row] = best;
    }
    __syncthreads();
    if (tid < AR_ROWS && n0 + tid < N)
        atomicMin((unsigned long long*)&keys[n0 + tid], (unsigned long long)umin64(part[0][tid], part[1][tid]));
}

constexpr int DR_ROWS = 32;

__global__ __launch_bounds__(NT) void rvq_argmin_direct(Rows x, const float* embed, uint64_t* keys,
                                                        int N, int D, int Kc) {
    extern __shared__ float sm[];
    float* es = sm;                        // [256][D+1]
    float* xs = sm + NT * (D + 1);         // [DR_ROWS][D]
    __shared__ uint64_t part[4];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int n0 = blockIdx.x * DR_ROWS, k = blockIdx.y * NT + tid;
    for (int i = tid; i < NT * D; i += NT) {
        int c = i / D, d = i - c * D, kk = blockIdx.y * NT + c;
        es[c * (D + 1) + d] = kk < Kc ? embed[(int64_t)kk * D + d] : 0.f;
    }
    for (int i = tid; i < DR_ROWS * D; i += NT) {
        int r = i / D, d = i - r * D;
        xs[i] = (n0 + r < N) ? x.at(n0 + r, d) : 0.f;
    }
    __syncthreads();
    for (int r = 0; r < DR_ROWS; ++r) {
        float s = 0.f;
        for (int d = 0; d < D; ++d) {
            float df = xs[r * D + d] - es[tid * (D + 1) + d];
            s = fmaf(df, df, s);
        }
        uint64_t key = k < Kc ? (((uint64_t)ord_key(s) << 32) | (uint32_t)k) : ~0ull;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) key = umin64(key, shfl_xor64(key, o));
        if (lane == 0) part[wave] = key;
        __syncthreads();
        if (tid == 0 && n0 + r < N) {
            uint64_t b = umin64(umin64(part[0], part[1]), umin64(part[2], part[3]));
            atomicMin((unsigned long long*)&keys[n0 + r], (unsigned long long)b);
        }
        __syncthreads();
    }
}

__global__ void keys_to_idx(const uint64_t* keys, int64_t* idx, int N) {
    int n = blockIdx.x * blockDim.x + threadIdx.x;
    if (n < N) idx[n] = (int64_t)(uint32_t)(keys[n] & 0xffffffffull);
}

__global__ void fill_u64(uint64_t* p, uint64_t v, int N) {
    int n = blockIdx.x * blockDim.x + threadIdx.x;
    if (n < N) p[n] = v;
}

constexpr int AP_MAXB = 1024;

// one train-mode VQ layer after its argmin; x = res (layer input)
__global__ __launch_bounds__(NT) void rvq_apply_kernel(const float* xin, float* res,
                                                       const float* embed, const int64_t* idx,
                                                       float* out, float* cdir, float* parts, int D,
                                                       int Tf, int64_t total, int first, int ste) {
    __shared__ float red[16];
    float s = 0.f;
    for (int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x; i < total; i += (int64_t)gridDim.x * NT) {
        int64_t bd = i / Tf;
        int t = (int)(i - bd * Tf);
        int64_t b = bd / D;
        int d = (int)(bd - b * D);
        const int64_t k = idx[b * Tf + t];
        const float x = xin[i];
        const float q = embed[k * D + d];
        const float qs = ste ? x + (q - x) : q;  // core_vq.py:309 (train) / exact q (eval encode)
        res[i] = x - qs;                          // :348 residual - quantized.detach()
        if (out) out[i] = first ? qs : out[i] + qs;
        if (cdir) cdir[i] = first ? (x - qs) : cdir[i] + (x - qs);
        const float df = qs - x;
        s = fmaf(df, df, s);
    }
    s = block_sum(s, red);
    if (parts && threadIdx.x == 0) parts[blockIdx.x] = s;
}

// ResidualVectorQuantization.decode (core_vq.py:369-375): out (+)= embed[idx] in [B][D][Tf]
__global__ void rvq_gather_kernel(const float* embed, const int64_t* idx, float* out, int D, int Tf,
                                  int64_t total, int acc) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= total) return;
    int64_t bd = i / Tf;
    int t = (int)(i - bd * Tf);
    int64_t b = bd / D;
    int d = (int)(bd - b * D);
    float q = embed[idx[b * Tf + t] * D + d];
    out[i] = acc ? out[i] + q : q;
}

// Per-code sums of the assigned frames, the reference's own formulation
// embed_sum = x^T @ onehot (core_vq.py:228; kmeans' scatter_add :96-97) as an MFMA GEMM
// [Kc x N] x [N x (D+1)] whose one-hot A operand is generated from the codes while staging and
// whose extra all-ones column yields the counts. Split over frames into fixed slabs, then
// summed in slab order: deterministic and insensitive to how skewed the assignment is.
struct LdOneHot {
    static constexpr bool A_K_FAST = true, B_N_FAST = false;
    Rows x;
    const int64_t* idx;
    int D;
    ENCX_DEV float a(int c, int n) const { return idx[n] == c ? 1.f : 0.f; }
    ENCX_DEV float b(int n, int d) const { return d < D ? x.at(n, d) : 1.f; }
};
struct EpSlab {
    float* ws;
    int Kc, W;
    ENCX_DEV void operator()(int c, int d, float v) const {
        ws[((int64_t)blockIdx.z * Kc + c) * W + d] = v;
    }
};

// MODE 0: EMA (core_vq.py:227-229), 1: kmeans (:92-100), 2: the raw sums into means [Kc][D+1]
template <int MODE>
__global__ void bucket_finish(const float* ws, int S, int Kc, int D, float* cs, float* ea,
                              float* means, int64_t* bins, float decay, float one_m) {
    const int c = blockIdx.x, W = D + 1;
    const float cnt = MODE == 1 ? sum_strided(ws + (int64_t)c * W + D, S, (int64_t)Kc * W) : 0.f;
    for (int d = threadIdx.x; d <= D; d += blockDim.x) {
        const float s = sum_strided(ws + (int64_t)c * W + d, S, (int64_t)Kc * W);
        if (MODE == 2) {
            means[(int64_t)c * W + d] = s;
        } else if (MODE == 0) {
            if (d < D) {
                float* p = ea + (int64_t)c * D + d;
                *p = fmaf(s, one_m, *p * decay);
            } else {
                cs[c] = fmaf(s, one_m, cs[c] * decay);
            }
        } else {
            if (d < D) {
                if (cnt > 0.f) means[(int64_t)c * D + d] = s / cnt;
            } else {
                bins[c] = (int64_t)cnt;
            }
        }
    }
}

template <int MODE>
int bucket_run(Rows x, const int64_t* idx, int N, int D, int Kc, float* ws, float* cs, float* ea,
               float* means, int64_t* bins, float decay, float one_m, hipStream_t st) {
    const int splits = gemm_splits(Kc, D + 1, N);
    const int S = gemm_slabs(N, splits);
    int rc = gemm_launch(LdOneHot{x, idx, D}, EpSlab{ws, Kc, D + 1}, Kc, D + 1, N, st, splits);
    if (rc) return rc;
    hipLaunchKernelGGL(bucket_finish<MODE>, dim3(Kc), dim3(D + 1 < 64 ? 64 : 256), 0, st, ws, S, Kc, D,
                       cs, ea, means, bins, decay, one_m);
    ENCX_CHECK_LAUNCH();
    return 0;
}

// the EMA of core_vq.py:227-229 from precomputed (e.g. all-reduced) sums [Kc][D+1]; the same
// fmaf as bucket_finish<0>, so sums + this == encx_rvq_ema bit for bit
__global__ void ema_from_sums(const float* sums, int D, float* cs, float* ea, float decay, float one_m) {
    const int c = blockIdx.x, W = D + 1;
    for (int d = threadIdx.x; d <= D; d += blockDim.x) {
        const float s = sums[(int64_t)c * W + d];
        if (d < D) {
            float* p = ea + (int64_t)c * D + d;
            *p = fmaf(s, one_m, *p * decay);
        } else {
            cs[c] = fmaf(s, one_m, cs[c] * decay);
        }
    }
}

// embed = embed_avg / (laplace(cluster_size) * sum(cluster_size)), core_vq.py:230-235
__global__ void ema_normalize(const float* cs, const float* ea, float* embed, int D, int Kc,
                              float eps, float keps) {
    __shared__ float red[16];
    float s = 0.f;
    for (int i = threadIdx.x; i < Kc; i += blockDim.x) s += cs[i];
    s = block_sum(s, red);
    const int c = blockIdx.x;
    const float sm = (cs[c] + eps) / (s + keps) * s;
    for (int d = threadIdx.x; d < D; d += blockDim.x)
        embed[(int64_t)c * D + d] = ea[(int64_t)c * D + d] / sm;
}

ENCX_DEV uint64_t splitmix(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// randperm(N)[:num] by rank of random keys (ties by index), or randint when num > N
__global__ __launch_bounds__(NT) void sample_rows_kernel(const float* samples, float* out, int N,
                                                         int D, int num, uint64_t seed) {
    const int i = blockIdx.x * NT + threadIdx.x;
    if (num > N) {  // core_vq.py:74-75 randint
        if (i >= num) return;
        int src = (int)(splitmix(seed ^ (0xA24BAED4963EE407ull * (uint64_t)(i + 1))) % (uint64_t)N);
        for (int d = 0; d < D; ++d) out[(int64_t)i * D + d] = samples[(int64_t)src * D + d];
        return;
    }
    if (i >= N) return;
    const uint64_t ki = splitmix(seed + (uint64_t)i);
    int rank = 0;
    for (int j = 0; j < N; ++j) {
        uint64_t kj = splitmix(seed + (uint64_t)j);
        rank += (kj < ki) || (kj == ki && j < i);
    }
    if (rank < num)
        for (int d = 0; d < D; ++d) out[(int64_t)rank * D + d] = samples[(int64_t)i * D + d];
}

Rows bdt_rows(const float* p, int64_t B, int64_t D, int64_t Tf) {
    Rows r;
    r.p = p; r.sB = D * Tf; r.sT = 1; r.sD = Tf; r.Tf = (int)Tf; r.fTf = make_fastdiv((uint32_t)Tf);
    return r;
}
Rows nd_rows(const float* p, int64_t N, int64_t D) {
    Rows r;
    r.p = p; r.sB = 0; r.sT = D; r.sD = 1; r.Tf = (int)N; r.fTf = make_fastdiv((uint32_t)N);
    return r;
}

int argmin_run(Rows x, const float* embed, int64_t* idx, uint64_t* keys, int N, int D, int Kc,
               int direct, hipStream_t st) {
    hipLaunchKernelGGL(fill_u64, dim3(cdiv(N, 256)), dim3(256), 0, st, keys, ~0ull, N);
    if (!direct) {
        const size_t lds = (size_t)(D * (AR_ROWS + AR_BS) + AR_ROWS + AR_CODES) * sizeof(float);
        if (lds > 150 * 1024) return ENCX_EINVAL;
        hipLaunchKernelGGL(rvq_argmin_mfma, dim3(cdiv(N, AR_ROWS), cdiv(Kc, AR_CODES)), dim3(NT), lds,
                           st, x, embed, keys, N, D, Kc);
    } else {
        size_t lds = (size_t)(NT * (D + 1) + DR_ROWS * D) * sizeof(float);
        if (lds > 160 * 1024) return ENCX_EINVAL;
        hipLaunchKernelGGL(rvq_argmin_direct, dim3(cdiv(N, DR_ROWS), cdiv(Kc, NT)), dim3(NT), lds, st,
                           x, embed, keys, N, D, Kc);
    }
    ENCX_CHECK_LAUNCH();
    hipLaunchKernelGGL(keys_to_idx, dim3(cdiv(N, 256)), dim3(256), 0, st, keys, idx, N);
    ENCX_CHECK_LAUNCH();
    return 0;
}

}  // namespace

extern "C" {

int encx_rvq_argmin(const float* res, const float* embed, int64_t* idx, uint64_t* keys,
                    int64_t B, int64_t D, int64_t Tf, int64_t Kc, int direct,
                    encx_stream_t stream) {
    ENCX_REQUIRE(res && embed && idx && keys && B > 0 && D > 0 && D <= 256 && Tf > 0 && Kc > 0);
    encx_prof_scope ps((hipStream_t)stream, 2.0 * B * Tf * Kc * D, 4.0 * (B * D * Tf + Kc * D) + 8.0 * B * Tf, "rvq_argmin");
    return argmin_run(bdt_rows(res, B, D, Tf), embed, idx, keys, (int)(B * Tf), (int)D, (int)Kc,
                      direct, (hipStream_t)stream);
}

int64_t encx_rvq_apply_parts(int64_t B, int64_t D, int64_t Tf) {
    int64_t total = B * D * Tf;
    int64_t b = cdiv(total, NT);
    return b < AP_MAXB ? b : AP_MAXB;
}

int encx_rvq_apply(const float* x, float* res_out, const float* embed, const int64_t* idx,
                   float* out, float* commit_dir, float* commit_part, int64_t B, int64_t D,
                   int64_t Tf, int first, int ste, encx_stream_t stream) {
    ENCX_REQUIRE(x && res_out && embed && idx && B > 0 && D > 0 && Tf > 0);
    encx_prof_scope ps((hipStream_t)stream, 4.0 * B * D * Tf, 4.0 * B * D * Tf * (2 + (out != nullptr) * 2 + (commit_dir != nullptr) * 2) + 8.0 * B * Tf, "rvq_apply", false);
    int64_t total = B * D * Tf;
    hipLaunchKernelGGL(rvq_apply_kernel, dim3(encx_rvq_apply_parts(B, D, Tf)), dim3(NT), 0,
                       (hipStream_t)stream, x, res_out, embed, idx, out, commit_dir, commit_part,
                       (int)D, (int)Tf, total, first, ste);
    ENCX_CHECK_LAUNCH();
    return 0;
}

int encx_rvq_gather(const float* embed, const int64_t* idx, float* out, int64_t B, int64_t D,
                    int64_t Tf, int accumulate, encx_stream_t stream) {
    ENCX_REQUIRE(embed && idx && out && B > 0 && D > 0 && Tf > 0);
    encx_prof_scope ps((hipStream_t)stream, 0.0, 4.0 * B * D * Tf * (accumulate ? 3 : 2), "rvq_gather", false);
    int64_t total = B * D * Tf;
    hipLaunchKernelGGL(rvq_gather_kernel, dim3(cdiv(total, 256)), dim3(256), 0, (hipStream_t)stream,
                       embed, idx, out, (int)D, (int)Tf, total, accumulate);
    ENCX_CHECK_LAUNCH();
    return 0;
}

size_t encx_rvq_bucket_workspace(int64_t N, int64_t D, int64_t Kc) {
    const int S = gemm_slabs((int)N, gemm_splits((int)Kc, (int)D + 1, (int)N));
    return (size_t)S * Kc * (D + 1) * sizeof(float);
}

int encx_rvq_ema(const float* x, const int64_t* idx, float* cluster_size, float* embed_avg,
                 float* embed, float* ws, int64_t B, int64_t D, int64_t Tf, int64_t Kc,
                 float decay, float eps, encx_stream_t stream) {
    ENCX_REQUIRE(x && idx && cluster_size && embed_avg && embed && ws && D <= 256 && Kc > 0);
    encx_prof_scope ps((hipStream_t)stream, 2.0 * B * Tf * Kc * (D + 1), 4.0 * (B * D * Tf + 4 * Kc * D) + 8.0 * B * Tf, "rvq_ema");
    hipStream_t st = (hipStream_t)stream;
    const float one_m = (float)(1.0 - (double)decay);
    int rc = bucket_run<0>(bdt_rows(x, B, D, Tf), idx, (int)(B * Tf), (int)D, (int)Kc, ws,
                           cluster_size, embed_avg, nullptr, nullptr, decay, one_m, st);
    if (rc) return rc;
    hipLaunchKernelGGL(ema_normalize, dim3(Kc), dim3(D < 64 ? 64 : (D > 256 ? 256 : D)), 0, st,
                       cluster_size, embed_avg, embed, (int)D, (int)Kc, eps,
                       (float)((double)Kc * (double)eps));
    ENCX_CHECK_LAUNCH();
    return 0;
}

int encx_rvq_code_sums(const float* x, const int64_t* idx, float* sums, float* ws, int64_t B,
                       int64_t D, int64_t Tf, int64_t Kc, encx_stream_t stream) {
    ENCX_REQUIRE(x && idx && sums && ws && B > 0 && D > 0 && D <= 256 && Tf > 0 && Kc > 0);
    return bucket_run<2>(bdt_rows(x, B, D, Tf), idx, (int)(B * Tf), (int)D, (int)Kc, ws, nullptr,
                         nullptr, sums, nullptr, 0.f, 0.f, (hipStream_t)stream);
}

int encx_rvq_ema_from_sums(const float* sums, float* cluster_size, float* embed_avg, float* embed,
                           int64_t D, int64_t Kc, float decay, float eps, encx_stream_t stream) {
    ENCX_REQUIRE(sums && cluster_size && embed_avg && embed && D > 0 && D <= 256 && Kc > 0);
    hipStream_t st = (hipStream_t)stream;
    const float one_m = (float)(1.0 - (double)decay);
    hipLaunchKernelGGL(ema_from_sums, dim3(Kc), dim3(D + 1 < 64 ? 64 : 256), 0, st, sums, (int)D,
                       cluster_size, embed_avg, decay, one_m);
    ENCX_CHECK_LAUNCH();
    hipLaunchKernelGGL(ema_normalize, dim3(Kc), dim3(D < 64 ? 64 : (D > 256 ? 256 : D)), 0, st,
                       cluster_size, embed_avg, embed, (int)D, (int)Kc, eps,
                       (float)((double)Kc * (double)eps));
    ENCX_CHECK_LAUNCH();
    return 0;
}

int encx_kmeans_step(const float* samples, float* means, int64_t* bins, int64_t* idx,
                     uint64_t* keys, float* ws, int64_t N, int64_t D, int64_t Kc,
                     encx_stream_t stream) {
    ENCX_REQUIRE(samples && means && bins && idx && keys && ws && N > 0 && D > 0 && D <= 256 && Kc > 0);
    hipStream_t st = (hipStream_t)stream;
    Rows r = nd_rows(samples, N, D);
    int rc = argmin_run(r, means, idx, keys, (int)N, (int)D, (int)Kc, 1, st);
    if (rc) return rc;
    return bucket_run<1>(r, idx, (int)N, (int)D, (int)Kc, ws, nullptr, nullptr, means, bins, 0.f,
                         0.f, st);
}

int encx_sample_rows(const float* samples, float* out, int64_t N, int64_t D, int64_t num,
                     uint64_t seed, encx_stream_t stream) {
    ENCX_REQUIRE(samples && out && N > 0 && D > 0 && num > 0);
    int64_t threads = num > N ? num : N;
    hipLaunchKernelGGL(sample_rows_kernel, dim3(cdiv(threads, NT)), dim3(NT), 0, (hipStream_t)stream,
                       samples, out, (int)N, (int)D, (int)num, seed);
    ENCX_CHECK_LAUNCH();
    return 0;
}

}  // extern "C"
