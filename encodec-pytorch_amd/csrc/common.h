// encx -- MI355X (gfx950) kernels for the EnCodec training hot path.
// Shared device helpers. Every kernel is fp32 in / fp32 accumulate (the reference trains in
// fp32 with AMP off: config/config.yaml:7); matrix work uses the exact-f32 MFMA
// v_mfma_f32_32x32x2_f32 (MI355X_MICROARCH.md: 157 TF/s, bitwise an fmaf chain).
#pragma once
#include <hip/hip_runtime.h>
#include <algorithm>
#include <stdint.h>

#include "../../include/encx.h"

#define ENCX_DEV __device__ __forceinline__

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef float f32x4u __attribute__((ext_vector_type(4), aligned(4)));
ENCX_DEV f32x4 ld4u(const float* p) { return *(const f32x4u*)p; }  // 4-byte aligned quad load

// ---- error plumbing: no exceptions cross the C ABI ---------------------------------------
#define ENCX_CHECK_LAUNCH()                                                    \
    do {                                                                       \
        hipError_t _e = hipGetLastError();                                     \
        if (_e != hipSuccess) return (int)_e;                                  \
    } while (0)
#define ENCX_REQUIRE(cond)                                                     \
    do {                                                                       \
        if (!(cond)) return ENCX_EINVAL;                                       \
    } while (0)

// ---- division by a launch-invariant divisor ---------------------------------------------
// q = n / d for 0 <= n, d < 2^31 as a multiply-high, add and shift (Granlund-Montgomery):
// l = ceil(log2 d), mul = floor(2^32 (2^l - d) / d) + 1, q = (umulhi(n, mul) + n) >> l.
// Loaders that split a flattened index per staged element use it instead of an integer
// division (a ~40-instruction sequence on CDNA).
struct FastDiv {
    uint32_t d, mul, shr;
};
static inline FastDiv make_fastdiv(uint32_t d) {
    uint32_t l = 0;
    while ((1ull << l) < d) ++l;
    FastDiv f;
    f.d = d;
    f.shr = l;
    f.mul = (uint32_t)((((1ull << 32) * ((1ull << l) - d)) / d) + 1);
    return f;
}
ENCX_DEV uint32_t fdiv(uint32_t n, const FastDiv& f) {
    return (__umulhi(n, f.mul) + n) >> f.shr;
}

// ---- activations ---------------------------------------------------------------------------
// nn.ELU(alpha=1) (modules/seanet.py:49 etc.): x > 0 ? x : expm1(x)
ENCX_DEV float elu(float x) { return x > 0.f ? x : expm1f(x); }
// d ELU / dx evaluated at the pre-activation x: 1 or exp(x) (= elu(x) + 1)
ENCX_DEV float elu_grad(float x) { return x > 0.f ? 1.f : expf(x); }
// nn.LeakyReLU(0.2) (msstftd.py:50,61)
ENCX_DEV float lrelu(float x) { return x > 0.f ? x : 0.2f * x; }
ENCX_DEV float lrelu_grad(float y_or_x) { return y_or_x > 0.f ? 1.f : 0.2f; }

ENCX_DEV float act_apply(int act, float x) { return act == ENCX_ACT_ELU ? elu(x) : x; }
ENCX_DEV float act_grad(int act, float x) { return act == ENCX_ACT_ELU ? elu_grad(x) : 1.f; }

// ---- padding -------------------------------------------------------------------------------
// Source index of padded position p for pad1d (modules/conv.py:79-96): reflect (with the
// short-input zero extension `e`, :86-94) or zero padding. Returns -1 for a zero.
ENCX_DEV int pad_src(int p, int pl, int T, int e, int mode) {
    int i = p - pl;
    if (mode == ENCX_PAD_REFLECT) {
        int L = T + e;
        if (i < 0) i = -i;
        else if (i >= L) i = 2 * (L - 1) - i;
        return (i >= 0 && i < T) ? i : -1;
    }
    return (i >= 0 && i < T) ? i : -1;
}

// ---- MFMA ----------------------------------------------------------------------------------
// 32x32x2 f32: lane l holds A[l&31][l>>5], B[l>>5][l&31]; D row = (r&3)+8*(r>>2)+4*(l>>5), col l&31
ENCX_DEV f32x16 mfma32(float a, float b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}
ENCX_DEV int mfma_row(int r, int lane) { return (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5); }

// ---- reductions ----------------------------------------------------------------------------
ENCX_DEV float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
ENCX_DEV double wave_sum_d(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// block-wide sum, blockDim.x multiple of 64 and <= 1024; result valid in every thread
ENCX_DEV float block_sum(float v, float* red /* >= 16 floats of LDS */) {
    v = wave_sum(v);
    int w = threadIdx.x >> 6, l = threadIdx.x & 63;
    __syncthreads();
    if (l == 0) red[w] = v;
    __syncthreads();
    int nw = blockDim.x >> 6;
    float t = 0.f;
    for (int i = 0; i < nw; ++i) t += red[i];
    return t;
}

// sum_{s < n} p[s * stride] in ascending s (bitwise the serial loop) with 8 loads in flight:
// clamped addresses, values selected after the load. A plain `for (s) acc += p[s*stride]`
// compiles to load / s_waitcnt vmcnt(0) / add per iteration, one memory round trip per term.
ENCX_DEV float sum_strided(const float* p, int n, int64_t stride) {
    float acc = 0.f;
    for (int s0 = 0; s0 < n; s0 += 8) {
        float v[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const int s = s0 + q;
            const float t = p[(int64_t)(s < n ? s : 0) * stride];
            v[q] = s < n ? t : 0.f;
        }
#pragma unroll
        for (int q = 0; q < 8; ++q) acc += v[q];
    }
    return acc;
}

// the same sum accumulated in fp64 (one rounding at the end): the weight-grad slab reduces whose
// sums run over up to ~1500 slabs of fp32 partials
ENCX_DEV double sum_strided_d(const float* p, int n, int64_t stride) {
    double acc = 0.0;
    for (int s0 = 0; s0 < n; s0 += 8) {
        float v[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const int s = s0 + q;
            const float t = p[(int64_t)(s < n ? s : 0) * stride];
            v[q] = s < n ? t : 0.f;
        }
#pragma unroll
        for (int q = 0; q < 8; ++q) acc += (double)v[q];
    }
    return acc;
}

// Slab reduction by a 256-thread block: lane l of wave w sums splits s = w, w + 4, ... of output
// i (= the block's 64 consecutive outputs, one per lane: every wave load is one coalesced 256-byte
// row segment), then wave 0 adds the 4 partials in order w = 0..3. Deterministic; the result is
// valid in wave 0 only. red: __shared__ float[4][64].
ENCX_DEV float slab_sum_256(const float* p, int S, int64_t stride, bool valid, float* red) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    float v = 0.f;
    if (valid && w < S) v = sum_strided(p + (int64_t)w * stride, (S - w + 3) >> 2, 4 * stride);
    red[w * 64 + lane] = v;
    __syncthreads();
    return ((red[lane] + red[64 + lane]) + red[128 + lane]) + red[192 + lane];
}
// slab_sum_256 in fp64 (red: __shared__ double[4][64]); the result rounded once to fp32
ENCX_DEV float slab_sum_256_d(const float* p, int S, int64_t stride, bool valid, double* red) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    double v = 0.0;
    if (valid && w < S) v = sum_strided_d(p + (int64_t)w * stride, (S - w + 3) >> 2, 4 * stride);
    red[w * 64 + lane] = v;
    __syncthreads();
    return (float)(((red[lane] + red[64 + lane]) + red[128 + lane]) + red[192 + lane]);
}

// XCD-aware tile order. The dispatcher deals workgroups to the 8 XCDs round-robin by linear id,
// so neighbouring tiles (which share input halo rows or a staged operand) land on different
// XCDs and each re-fetches the shared data into its own L2. Remapped, XCD k works through one
// contiguous run of tiles in order. Returns the remapped linear id of this workgroup.
ENCX_DEV int xcd_linear_id() {
    const int n = (int)(gridDim.x * gridDim.y * gridDim.z);
    const int i = (int)(blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z));
    const int k = i & 7;
    int base = 0;
#pragma unroll
    for (int j = 0; j < 7; ++j)
        if (j < k) base += (n - j + 7) >> 3;  // workgroups dealt to XCD j
    return base + (i >> 3);
}
// the remapped id as (x, y, z) over gridDim
struct TileId {
    int x, y, z;
};
ENCX_DEV TileId xcd_tile() {
    const int id = xcd_linear_id(), gx = (int)gridDim.x, gy = (int)gridDim.y;
    TileId t;
    t.x = id % gx;
    t.y = (id / gx) % gy;
    t.z = id / (gx * gy);
    return t;
}

static inline int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }

// Kernel-selection options (api.hip): each starts from its ENCX_<NAME> environment variable (or
// its default) and is read on every call, so a test or an A/B run can flip it in-process through
// encx_set_option. Set them before sizing workspaces: a workspace query and the launch that uses
// it must see the same options.
enum EncxOpt {
    OPT_FFT,           // spectrograms by real FFT (0: framed-DFT GEMM)
    OPT_PW,            // pointwise GEMM kernels for the short, wide 1x1 convs
    OPT_PW_TMAX,       // longest T served by the 1x1 forward / bwd-data GEMM
    OPT_PW_WG_TMAX,    // longest T served by the 1x1 weight-grad GEMM
    OPT_LSTM_FUSE,     // LSTM backward: elementwise step fused into the next GEMM launch
    OPT_LSTM_PERSIST,  // LSTM: one persistent launch per recurrence (0: a launch per wavefront step)
    OPT_LSTM_WG_SPLITS, // LSTM weight grad: at most this many k-splits (partial slabs) of the GEMM
    OPT_FWR,           // register-window Conv2d forward: workgroups (0: off)
    OPT_DGR,           // register-window Conv2d bwd-data: workgroups (0: off)
    OPT_WGR,           // register-window Conv2d weight grad: waves (0: off)
    OPT_WGR_WGS,       // its 8-wave workgroup form: workgroups (0: one-wave form)
    OPT_FEAT_CODE,     // Conv2d bwd-data feature term from the pair's 1-byte code (else both maps)
    OPT_CONV_CK,       // conv1d fwd / bwd-data: reduction elements (channels x taps) per LDS chunk
    OPT_CONV_SPLIT,    // conv1d fwd / bwd-data: split-K until this many workgroups
    OPT_CONV_WG_SPLIT, // conv1d weight grad: split the positions until this many workgroups
    OPT_CONV2,         // conv1d v2 kernels, bitmask: 1 forward, 2 polyphase (bwd-data / convtr), 4 weight grad
    OPT_CONV2_TILE,    // its tile: 0 auto, 1 128x128, 2 128x64, 3 64x128, 4 64x64 (BM x BN)
    OPT_CONV2_RED,     // its largest reduction (channels x taps) per chunk
    OPT_CONV2_KS,      // its channel splits (0: planned)
    OPT_CONV2_WGS,     // v2 weight grad: about this many workgroups (position splits x tiles)
    OPT_CONV2_LOWT,    // v2 also for 64 < T <= 128 (the T 75 layers), else the flattened GEMMs
    OPT_LSTM_SPIN,     // persistent LSTM: log2 of every poll's spin bound (0: 20, about 1 s)
    OPT_LSTM_FAULT,    // persistent LSTM, tests only: one workgroup never publishes (its consumers time out)
    OPT_BLAS,          // plain GEMMs through hipBLASLt (blas.hip), bitmask: 1 the LSTM weight grads, 2 the
                       // im2col'd T <= 128 convs, 4 the im2col'd larger convs (fwd / polyphase), 8 their weight grads
    OPT_COUNT
};
int64_t encx_opt(EncxOpt id);

// blas.hip: C (m x n, column-major, ldc) = op(A) op(B) (+ C when accumulate), fp32 in, fp32
// compute (HIPBLAS_COMPUTE_32F: the exact-f32 MFMA), on `st`, through hipBLASLt; `batch` > 1:
// that many problems at element strides sa / sb / sc. Nonzero when hipBLASLt has no algorithm for
// the problem or option BLAS is off (the caller runs its own kernels instead); plans and the
// library workspace are cached per shape and device.
int encx_sgemm(hipStream_t st, bool ta, bool tb, int m, int n, int k, const float* A, int lda, const float* B,
               int ldb, float* C, int ldc, bool accumulate, int batch = 1, int64_t sa = 0, int64_t sb = 0,
               int64_t sc = 0);
