// SLSTM (modules/lstm.py:12-28): nn.LSTM(H, H, num_layers) over the 75 latent frames + skip.
//
// All L layers advance together as one diagonal wavefront: launch k moves layer l to frame
// t = k - l (forward) or t = T-1-k+(L-1-l) (backward), so every layer's input for its frame
// was produced by the previous launch. The recurrence costs T+L-1 dependent launches forward
// and 2(T+L)-1 backward, instead of L*T and 2*L*T for layer-after-layer.
//
// Per step the whole gate pre-activation of a layer is one contraction over K = 2H:
//   pre[b][j] = [x_l(b,t) | h_l(b,t-1)] . wcat_l[j] + bsum_l[j]
// with wcat_l = [W_ih | W_hh] ([4H][2H], packed once per call by encx_lstm_pack) and x_l the
// layer input (x transposed for layer 0, h_{l-1} above). The contraction runs on
// v_mfma_f32_16x16x4_f32 with 8 waves splitting K, the partial tiles summed in LDS in wave
// order, then the gates and cell update are fused in the same launch.
//
// Backward per step: an elementwise launch (gate grads of every active layer from the
// recurrent and the upper layer's grads; the input grad of layer 0 for the frame finished one
// step earlier) and one MFMA launch P_l = DA_l(t) . wcat_l over all layers, whose first H
// columns are the grad of layer l's input at frame t (consumed by layer l-1, or dx for l = 0)
// and whose last H columns are the recurrent grad of h_l(t-1). Weight grads are one GEMM per
// layer over all frames afterwards: dwcat_l = sum_{b,t} DA_l^T [x_l | h_l(t-1) | 1].
//
// Sequence tensors are [L][B][T][.] (row m = b*T + t). Gate order i, f, g, o (torch).
// All operand loads use clamped addresses with the value selected afterwards (no branches
// around loads: a branch per load serialises the memory latency).
#include "common.h"
#include "gemm.h"
#include "prof.h"

typedef float f32x4v __attribute__((ext_vector_type(4)));

namespace {

ENCX_DEV f32x4v mfma16(float a, float b, f32x4v c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}
ENCX_DEV float sigm(float x) { return 1.f / (1.f + expf(-x)); }
// The cell forward of one (b, u) point from its gate pre-activations: gates i, f, g, o, the cell c
// (from the previous frame's cp) and h. Shared by the step and the persistent forms, contraction
// limited to single expressions so that both compile to the same arithmetic.
ENCX_DEV void cell_fwd(const float pre[4], float cp, float g4[4], float* c, float* h) {
#pragma clang fp contract(on)
    g4[0] = sigm(pre[0]);
    g4[1] = sigm(pre[1]);
    g4[2] = tanhf(pre[2]);
    g4[3] = sigm(pre[3]);
    *c = g4[1] * cp + g4[0] * g4[2];
    *h = g4[3] * tanhf(*c);
}

constexpr int UNITS = 4;  // hidden units per forward workgroup (16 gate columns)
constexpr int FW = 8;     // waves per forward workgroup (K split)
constexpr int BW = 4;     // waves per backward-GEMM workgroup

// Operand fragments for v_mfma_f32_16x16x4_f32 over a 16-deep k group: lane (col = l&15,
// kk = l>>4) supplies k = 16*grp + 4*kk + s for s = 0..3 in four consecutive MFMAs, so both
// operands come in as one aligned float4 per lane and group (the summation order over k is
// a permutation of the natural one; fp32 accumulate).
ENCX_DEV float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }
ENCX_DEV float at4(const float4& v, int s) { return s == 0 ? v.x : s == 1 ? v.y : s == 2 ? v.z : v.w; }
ENCX_DEV float4 sel4(bool c, const float4& v) {
    return make_float4(c ? v.x : 0.f, c ? v.y : 0.f, c ? v.z : 0.f, c ? v.w : 0.f);
}

// ------------------------------------------------------------------------- forward step
// grid (H/UNITS, L); workgroup = UNITS hidden units (16 gate columns) of layer blockIdx.y.
// G = k-groups per wave (2H/16 groups over FW waves), RT = 16-row batch tiles.
template <int G, int RT>
__global__ __launch_bounds__(FW * 64) void lstm_fwd_wave(const float* xt, const float* wcat,
                                                         const float* bsum, float* Y, float* Cst,
                                                         float* Gs, int B, int T, int H, int k) {
    const int l = blockIdx.y, t = k - l;
    if (t < 0 || t >= T) return;
    __shared__ float red[FW][64][17];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int u0 = blockIdx.x * UNITS;
    const int col = lane & 15, kk = lane >> 4;
    const int K = 2 * H, NG = K >> 4;
    const int64_t BTH = (int64_t)B * T * H;
    const float* W = wcat + (int64_t)l * 4 * H * K;
    const float* xin = l == 0 ? xt : Y + (int64_t)(l - 1) * BTH;  // layer input sequence
    float* Yl = Y + (int64_t)l * BTH;
    float* Cl = Cst + (int64_t)l * BTH;
    const int tp = t > 0 ? t - 1 : 0;
    const int j = (col >> 2) * H + u0 + (col & 3);  // gate column of this lane
    // the gate phase's own operands (B*UNITS <= 256 threads), fetched before the MFMA chain
    const int pb0 = tid / UNITS, pu = u0 + (tid - pb0 * UNITS);
    const bool pact = pb0 < B;
    const int pb = pact ? pb0 : 0;
    const int64_t po = ((int64_t)pb * T + t) * H + pu;
    float bias[4];
#pragma unroll
    for (int g = 0; g < 4; ++g) bias[g] = bsum[(int64_t)l * 4 * H + g * H + pu];
    const float cpl = Cl[((int64_t)pb * T + tp) * H + pu];
    const float cpv = t > 0 ? cpl : 0.f;
    float4 wv[G], hv[RT][G];
#pragma unroll
    for (int g = 0; g < G; ++g) {
        const int gi = wave + FW * g;
        const bool okg = gi < NG;
        const int kq = (okg ? gi : 0) * 16 + 4 * kk;  // first k of this lane's float4
        wv[g] = sel4(okg, ld4(W + (int64_t)j * K + kq));
        const bool rec = kq >= H;  // recurrent half: h_l(t-1), zero at t = 0
        const float* src = rec ? Yl : xin;
        const int ts = rec ? tp : t;
        const int kc = rec ? kq - H : kq;
        const bool keep = !rec || t > 0;
#pragma unroll
        for (int r = 0; r < RT; ++r) {
            int row = r * 16 + col;
            row = row < B ? row : B - 1;  // rows >= B compute garbage that is never read
            hv[r][g] = sel4(keep, ld4(src + ((int64_t)row * T + ts) * H + kc));
        }
    }
    f32x4v acc[RT];
#pragma unroll
    for (int r = 0; r < RT; ++r) acc[r] = (f32x4v){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int g = 0; g < G; ++g)
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
            for (int r = 0; r < RT; ++r) acc[r] = mfma16(at4(hv[r][g], s), at4(wv[g], s), acc[r]);
#pragma unroll
    for (int r = 0; r < RT; ++r)
#pragma unroll
        for (int q = 0; q < 4; ++q) red[wave][r * 16 + kk * 4 + q][col] = acc[r][q];
    __syncthreads();
    if (pact) {
        const int uu = pu - u0;
        float pre[4];
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const int cc = g * 4 + uu;
            float s = red[0][pb][cc];
#pragma unroll
            for (int w = 1; w < FW; ++w) s += red[w][pb][cc];
            pre[g] = s + bias[g];
        }
        float g4[4], c, h;
        cell_fwd(pre, cpv, g4, &c, &h);
        Cl[po] = c;
        Yl[po] = h;
        float* gs = Gs + (int64_t)l * 4 * BTH + ((int64_t)pb * T + t) * 4 * H;
#pragma unroll
        for (int q = 0; q < 4; ++q) gs[q * H + pu] = g4[q];
    }
}

// ------------------------------------------------------------------------- persistent forward
// ONE launch runs the whole recurrence (option LSTM_PERSIST). Workgroup (l, bg, ug) owns the PU
// hidden units u0 = PU ug .. u0 + PU - 1 (4 PU = 32 gate columns, two 16-column MFMA tiles) of
// layer l for the 16 batch rows 16 bg .., and keeps its slice of wcat_l ([32][2H], 64 KB at
// H = 512) in registers for all T frames: the per-frame weight loads and launch boundaries of
// lstm_fwd_wave are gone. Frame t of layer l needs x_l(t) = h_{l-1}(t) and h_l(t-1) of its rows,
// i.e. the outputs of the NUG workgroups of (l-1, bg) and (l, bg). The hand-off is the counter
// form of the write-through protocol (cdna_hip_programming.md Guideline 16 R1; MI355X_MICROARCH.md
// visibility table, first row): h is stored sc1, every storing wave drains (s_waitcnt vmcnt(0)),
// a workgroup barrier, then ONE lane adds 1 to cnt[l][bg]; a consumer's wave 0 polls that word
// with relaxed agent-scope (sc1) loads until it reaches NUG (t + 1), the workgroup joins a
// barrier, and EVERY load of h is an sc1 buffer load (no L1 copy can be stale, no acquire). Layer
// 0 never waits on layer 1, so the layers run as a wavefront with no global step. Every spin is
// bounded: a timeout counts in the error word (encx_lstm_sync_errors) and the launch drains.
// All L NBG NUG workgroups must be resident together: the host uses this form only when they are
// at most one per CU. The arithmetic (k-group order, LDS sum order, gate math) is that of
// lstm_fwd_wave, so both forms give the same bits. Measured (tools/lstm_trace.py, profiles/r05/
// lstm): a frame takes 4.9 us (input part 1.5, recurrent loads + MFMA 1.6, gates 0.7, hand-off
// 0.8). Starting frame t+1's input part during frame t's gate phase (the two storing waves
// signalling through an LDS count) was slower, 389 -> 440 us per forward (frame 7.0 us: the early
// MFMAs delay the gate phase), and plain loads of the handed-off frames instead of sc1 loads
// gained nothing in either direction.
constexpr int PU = 8;           // hidden units per persistent workgroup
constexpr int SYNC_LINE = 32;   // ints per counter: one 128-byte line each
constexpr int SYNC_LINES = 512;
// hand-off counters [SYNC_LINES][SYNC_LINE], then the error word's line and the launch's done count.
// The counters are zero when a launch starts: statically at the first, and the last workgroup of
// every launch zeroes what its launch used (finish_launch). (A hipMemsetAsync node per call
// instead was not ordered before the kernel in graph replays: counts zeroed under running
// workgroups, every spin of the launch timing out.) Launches of the persistent forms must not
// overlap: one stream.
__device__ int g_lstm_sync[(SYNC_LINES + 2) * SYNC_LINE];

// Development tracing (build with -DENCX_LSTM_TRACE; encx_lstm_trace reads it): thread 0 of every
// persistent workgroup stamps the steady clock at up to 8 points of every frame,
// g_lstm_trace[kernel (0 fwd, 1 bwd)][workgroup < 256][frame < 128][point].
#ifdef ENCX_LSTM_TRACE
__device__ long long g_lstm_trace[2 * 256 * 128 * 8];
#define LSTM_TRACE(kern, i, k)                                                               \
    do {                                                                                     \
        if (tid == 0 && blockIdx.x < 256 && (i) < 128)                                       \
            g_lstm_trace[(((kern) * 256 + blockIdx.x) * 128 + (i)) * 8 + (k)] = wall_clock64(); \
    } while (0)
#else
#define LSTM_TRACE(kern, i, k) \
    do {                       \
    } while (0)
#endif

// The persistent kernels' control word (host: pers_ctl): bits 0-4 log2 of the spin bound of every
// poll (0: 20, about 1 s), bit 5 fault injection for tests: workgroup 0 never publishes, so its
// consumers' polls time out (option LSTM_FAULT).
constexpr int CTL_FAULT = 32;
ENCX_DEV int ctl_spins(int ctl) { return (ctl & 31) ? 1 << (ctl & 31) : 1 << 20; }
// wave-wide bounded poll: cnt >= target (relaxed agent loads, sc1); false after `spins` tries
ENCX_DEV bool poll_ge(const int* cnt, int target, int* err, int spins) {
    for (int i = 0; i < spins; ++i) {
        if (__hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= target) return true;
        __builtin_amdgcn_s_sleep(1);
    }
    if ((threadIdx.x & 63) == 0) __hip_atomic_fetch_add(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return false;
}
// end of a persistent launch: the last workgroup to count itself done checks that every counter
// line reached its final count (lines [0, n1) expect e1 arrivals, lines [n1, n1 + n2) expect e2; a
// line off its count -- an arrival lost, or one left over from an earlier launch -- counts in the
// error word), then zeroes the lines and the done count. Every workgroup has passed its last poll
// before it counts itself, and the next launch on the stream starts after this one has ended.
// Ordering: thread 0 made this workgroup's last arrivals; its s_waitcnt vmcnt(0) holds the done
// arrival until those atomics have been performed, so the last workgroup's zeroing (issued after
// its returning done add saw every other workgroup's) follows every arrival of the launch.
ENCX_DEV void finish_launch(int* sync, int n1, int e1, int n2, int e2) {
    __syncthreads();
    if (threadIdx.x == 0) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        int* done = sync + (SYNC_LINES + 1) * SYNC_LINE;
        if (__hip_atomic_fetch_add(done, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (int)gridDim.x - 1) {
            int off = 0;
            for (int i = 0; i < n1 + n2; ++i) {
                const int v = __hip_atomic_load(sync + i * SYNC_LINE, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                off += v != (i < n1 ? e1 : e2);
            }
            if (off) __hip_atomic_fetch_add(sync + SYNC_LINES * SYNC_LINE, off, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            for (int i = 0; i < n1 + n2; ++i)
                __hip_atomic_store(sync + i * SYNC_LINE, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(done, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}
// the error word into a caller's running count, and cleared (encx_lstm_sync_read): stream-ordered,
// capturable
__global__ void sync_read_kernel(int* sync, int* dst) {
    int* err = sync + SYNC_LINES * SYNC_LINE;
    const int v = __hip_atomic_exchange(err, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    dst[0] += v;
}
ENCX_DEV __amdgpu_buffer_rsrc_t buf_rsrc(const float* p, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p), (short)0, (int)bytes, 0x00020000);
}
constexpr int SC1 = 16;  // buffer op cache-policy bit: write-through store / L1-bypassing load
ENCX_DEV float4 ld4_sc1(__amdgpu_buffer_rsrc_t r, uint32_t byte_off) {
    // (the whole vector is bit-cast: clang 20 miscompiles a bit_cast of one element, v[i], into a
    // read of element 0)
    const f32x4v v = __builtin_bit_cast(f32x4v, __builtin_amdgcn_raw_buffer_load_b128(r, (int)byte_off, 0, SC1));
    return make_float4(v[0], v[1], v[2], v[3]);
}

// grid L * NBG * NUG (NUG = H / PU), FW waves; G = 2H / (16 FW) k-groups per wave (H % 128 == 0, so
// groups g < G / 2 of every wave are in the input half of K and the others in the recurrent half)
template <int G>
__global__ __launch_bounds__(FW * 64) void lstm_fwd_pers(const float* xt, const float* wcat, const float* bsum,
                                                         float* Y, float* Cst, float* Gs, int B, int T, int H,
                                                         int NBG, int* sync, int ctl) {
    const int NUG = H / PU;
    const int id = blockIdx.x, ug = id % NUG, bg = (id / NUG) % NBG, l = id / (NUG * NBG);
    __shared__ float red[FW][16][33];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, col = lane & 15, kk = lane >> 4;
    const int u0 = ug * PU, K = 2 * H;
    const int64_t BTH = (int64_t)B * T * H;
    // the resident weight slice: wr[g][c] = wcat_l[j][16 gi + 4 kk ..], gate column n = 16 c + col
    // (gate n / PU, unit u0 + n % PU)
    float4 wr[G][2];
    {
        const float* W = wcat + (int64_t)l * 4 * H * K;
#pragma unroll
        for (int g = 0; g < G; ++g)
#pragma unroll
            for (int c = 0; c < 2; ++c) {
                const int n = 16 * c + col, j = (n / PU) * H + u0 + n % PU;
                wr[g][c] = ld4(W + (int64_t)j * K + (wave + FW * g) * 16 + 4 * kk);
            }
    }
    // every load of a sequence goes through these descriptors with sc1 (the host checks that the
    // byte offsets fit 32 bits)
    const __amdgpu_buffer_rsrc_t rx = buf_rsrc(l == 0 ? xt : Y + (l - 1) * BTH, (uint32_t)(BTH * 4));
    const __amdgpu_buffer_rsrc_t ry = buf_rsrc(Y + l * BTH, (uint32_t)(BTH * 4));
    const int arow = min(bg * 16 + col, B - 1);  // rows >= B compute garbage that is never stored
    // the gate phase: thread p < 16 PU owns (row 16 bg + p / PU, unit u0 + p % PU) for all frames
    const int pr = tid / PU, pu = u0 + tid % PU, pb = bg * 16 + pr;
    const bool pact = tid < 16 * PU && pb < B;
    float bias[4];
#pragma unroll
    for (int g = 0; g < 4; ++g) bias[g] = pact ? bsum[(int64_t)l * 4 * H + g * H + pu] : 0.f;
    float* Cl = Cst + l * BTH;
    int* const cnt_self = sync + (l * NBG + bg) * SYNC_LINE;
    const int* const cnt_in = sync + ((l > 0 ? l - 1 : 0) * NBG + bg) * SYNC_LINE;
    int* const err = sync + SYNC_LINES * SYNC_LINE;
    bool live = true;  // wave 0: no poll has timed out
    const int spins = ctl_spins(ctl);
    const bool silent = (ctl & CTL_FAULT) && blockIdx.x == 0;
    float c = 0.f;
    for (int t = 0; t < T; ++t) {
        LSTM_TRACE(0, t, 0);
        f32x4v acc[2] = {(f32x4v){0.f, 0.f, 0.f, 0.f}, (f32x4v){0.f, 0.f, 0.f, 0.f}};
        // ---- input part x_l(t): layer 0 reads xt (written before this launch), layer l > 0
        // waits for h_{l-1}(t) of all NUG workgroups of (l-1, bg)
        if (l > 0) {
            if (wave == 0 && live) live = poll_ge(cnt_in, NUG * (t + 1), err, spins);
            __syncthreads();
        }
        LSTM_TRACE(0, t, 1);
        {  // k-groups g < G / 2 of every wave lie in the input half (H % 128 == 0)
            float4 a[G / 2];
            const uint32_t rb = (uint32_t)(((int64_t)arow * T + t) * H + 4 * kk) * 4u;
#pragma unroll
            for (int g = 0; g < G / 2; ++g) a[g] = ld4_sc1(rx, rb + (uint32_t)(wave + FW * g) * 64u);
            __builtin_amdgcn_sched_barrier(0);  // every load in flight before the first MFMA waits
#pragma unroll
            for (int g = 0; g < G / 2; ++g)
#pragma unroll
                for (int s = 0; s < 4; ++s)
#pragma unroll
                    for (int cc = 0; cc < 2; ++cc) acc[cc] = mfma16(at4(a[g], s), at4(wr[g][cc], s), acc[cc]);
        }
        // ---- recurrent part h_l(t-1) (zero at t = 0): k-groups g >= G / 2
        if (t > 0) {
            LSTM_TRACE(0, t, 2);
            if (wave == 0 && live) live = poll_ge(cnt_self, NUG * t, err, spins);
            __syncthreads();
            LSTM_TRACE(0, t, 3);
            float4 a[G / 2];
            const uint32_t rb = (uint32_t)(((int64_t)arow * T + t - 1) * H + 4 * kk - H) * 4u;
#pragma unroll
            for (int g = 0; g < G / 2; ++g) a[g] = ld4_sc1(ry, rb + (uint32_t)(wave + FW * (g + G / 2)) * 64u);
            __builtin_amdgcn_sched_barrier(0);  // every load in flight before the first MFMA waits
#pragma unroll
            for (int g = 0; g < G / 2; ++g)
#pragma unroll
                for (int s = 0; s < 4; ++s)
#pragma unroll
                    for (int cc = 0; cc < 2; ++cc)
                        acc[cc] = mfma16(at4(a[g], s), at4(wr[g + G / 2][cc], s), acc[cc]);
        }
#pragma unroll
        for (int cc = 0; cc < 2; ++cc)
#pragma unroll
            for (int q = 0; q < 4; ++q) red[wave][kk * 4 + q][16 * cc + col] = acc[cc][q];
        __syncthreads();
        LSTM_TRACE(0, t, 4);
        if (pact) {
            float pre[4];
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const int n = g * PU + (pu - u0);
                float s = red[0][pr][n];
#pragma unroll
                for (int w = 1; w < FW; ++w) s += red[w][pr][n];
                pre[g] = s + bias[g];
            }
            float g4[4], h;
            cell_fwd(pre, c, g4, &c, &h);
            const int64_t po = ((int64_t)pb * T + t) * H + pu;
            Cl[po] = c;
            // h: handed off inside this launch, so written through (sc1)
            __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, h), ry, (int)((uint32_t)po * 4u), 0,
                                                  SC1);
            float* gs = Gs + (int64_t)l * 4 * BTH + ((int64_t)pb * T + t) * 4 * H;
#pragma unroll
            for (int q = 0; q < 4; ++q) gs[q * H + pu] = g4[q];
        }
        // publish: every storing wave drained, a barrier, one lane's arrival
        LSTM_TRACE(0, t, 5);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        LSTM_TRACE(0, t, 6);
        if (tid == 0 && !silent) __hip_atomic_fetch_add(cnt_self, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    finish_launch(sync, (int)gridDim.x / NUG, NUG * T, 0, 0);  // the L NBG counters
}

// ------------------------------------------------------------------------- backward step
// E(k), grid (cdiv(B*H, 256), L + [dx]): role l < L: layer l at frame t = T-1-k+(L-1-l):
//   dh = (top layer: dout[b][u][t]; else sum_s P_{l+1}[s][b][u])      -- grad of h_l(t) from above
//      + (t < T-1: sum_s P_l[s][b][H+u])                              -- recurrent, from frame t+1
//   dc = dh o (1 - tanh^2 c) + dcn;  da_{i,f,g,o} -> DA_l[b][t];  dcn <- dc f
// role L: dx[b][u][t0] (+)= sum_s P_0[s][b][u] for the frame t0 layer 0 finished in step k-1.
// Partial sums over the split index s are added in ascending s (deterministic).
// The cell backward of one (b, u) point: gate pre-activation grads da[4] and the cell grad carried
// to frame t-1 (dc f), from dh, the carried dcn (rec: t < T-1) and the forward state. Shared by the
// step and the persistent forms, with contraction limited to single expressions so that both
// compile to the same arithmetic.
ENCX_DEV void cell_bwd(float dh, float dcn, bool rec, float ig, float fg, float gg, float og, float c, float cp,
                       float da[4], float* dcn_out) {
#pragma clang fp contract(on)
    const float tc = tanhf(c);
    const float dc = dh * og * (1.f - tc * tc) + (rec ? dcn : 0.f);
    da[0] = dc * gg * ig * (1.f - ig);
    da[1] = dc * cp * fg * (1.f - fg);
    da[2] = dc * ig * (1.f - gg * gg);
    da[3] = dh * tc * og * (1.f - og);
    *dcn_out = dc * fg;
}

// one (b, u) point of E(k) in `role` (the body of lstm_bwd_elem; the fused step's tail)
ENCX_DEV void bwd_elem_point(const float* dout, const float* P, int ns, float* dcn, const float* Cst,
                             const float* Gs, float* DA, float* dx, int acc_x, int B, int T, int H, int L, int k,
                             int role, int b, int u) {
    const int p = b * H + u;
    const int64_t N2 = 2 * H, SB = (int64_t)B * N2;
    if (role == L) {
        const int t0 = T - k + L - 1;
        if (!dx || t0 < 0 || t0 >= T) return;
        const float s = sum_strided(P + (int64_t)b * N2 + u, ns, SB);
        const int64_t o = ((int64_t)b * H + u) * T + t0;
        dx[o] = acc_x ? dx[o] + s : s;
        return;
    }
    const int l = role, t = T - 1 - k + (L - 1 - l);
    if (t < 0 || t >= T) return;
    const bool rec = t < T - 1;
    const int64_t BTH = (int64_t)B * T * H;
    const bool top = l == L - 1;
    // grad from above: dout for the top layer, else the upper layer's input-grad partials
    const float dh = (top ? dout[((int64_t)b * H + u) * T + t]
                          : sum_strided(P + (int64_t)(l + 1) * ns * SB + (int64_t)b * N2 + u, ns, SB)) +
                     (rec ? sum_strided(P + (int64_t)l * ns * SB + (int64_t)b * N2 + H + u, ns, SB) : 0.f);
    const int64_t o = ((int64_t)b * T + t) * H + u;
    const float* Cl = Cst + (int64_t)l * BTH;
    const float* gs = Gs + (int64_t)l * 4 * BTH + ((int64_t)b * T + t) * 4 * H;
    const float ig = gs[u], fg = gs[H + u], gg = gs[2 * H + u], og = gs[3 * H + u];
    const float c = Cl[o], cpl = Cl[t > 0 ? o - H : o], cp = t > 0 ? cpl : 0.f;
    float* dcl = dcn + (int64_t)l * B * H;
    float g4[4];
    cell_bwd(dh, dcl[p], rec, ig, fg, gg, og, c, cp, g4, &dcl[p]);
    float* da = DA + (int64_t)l * 4 * BTH + ((int64_t)b * T + t) * 4 * H;
    da[u] = g4[0];
    da[H + u] = g4[1];
    da[2 * H + u] = g4[2];
    da[3 * H + u] = g4[3];
}

__global__ __launch_bounds__(256) void lstm_bwd_elem(const float* dout, const float* P, int ns, float* dcn,
                                                     const float* Cst, const float* Gs, float* DA, float* dx,
                                                     int acc_x, int B, int T, int H, int L, int k) {
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= B * H) return;
    const int b = p / H;
    bwd_elem_point(dout, P, ns, dcn, Cst, Gs, DA, dx, acc_x, B, T, H, L, k, blockIdx.y, b, p - b * H);
}

// G(k), grid (2H/16, ns, L): P_l[s][b][n] = sum_{j in split s} DA_l[b][t][j] wcat_l[j][n] for the
// frame t of layer l in step k (MFMA 16x16x4 over float4 operands from wcatT [2H][4H]; the 4H
// reduction split over blockIdx.y so the grid covers the CUs, BW waves interleaving k-groups).
//
// FUSE: the same launch also runs E(k + 1). Every P tile feeds exactly one (role, 16-unit) group
// of E(k + 1): columns n >= H are the recurrent grad of layer l's units n - H (role l), columns
// n < H the input grad of layer l, i.e. the grad from above of layer l - 1's units n (role l - 1;
// dx for l = 0). A group has ns (top layer, dx) or 2 ns producing workgroups. Each workgroup,
// active or not, publishes its tile (stores drained, workgroup barrier, agent-scope release) and
// adds 1 to its group's arrival counter; the workgroup whose add completes the group acquires and
// runs E(k + 1) for the group's B x 16 points, then resets the counter for the next launch. No
// workgroup ever waits on another, so the launch cannot deadlock.
template <int G, int RT, bool FUSE>
__global__ __launch_bounds__(BW * 64) void lstm_bwd_gemm(const float* DA, const float* wcatT, float* P,
                                                         int B, int T, int H, int L, int k, int gper,
                                                         const float* dout, float* dcn, const float* Cst,
                                                         const float* Gs, float* DAw, float* dx, int acc_x,
                                                         int* cnt) {
    const int l = blockIdx.z, t = T - 1 - k + (L - 1 - l);
    const bool active = t >= 0 && t < T;
    if (!FUSE && !active) return;
    __shared__ float red[BW][64][17];
    __shared__ int s_last;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int c0 = blockIdx.x * 16, s = blockIdx.y, col = lane & 15, kk = lane >> 4;
    const int K = 4 * H, N2 = 2 * H, g0 = s * gper, ns = gridDim.y;
    if (active) {
        const float* Wt = wcatT + (int64_t)l * N2 * K + (int64_t)(c0 + col) * K;
        const float* D = DA + (int64_t)l * B * T * K;
        float4 wv[G], av[RT][G];
#pragma unroll
        for (int g = 0; g < G; ++g) {
            const int gl = wave + BW * g;
            const bool ok = gl < gper;
            const int kq = (g0 + (ok ? gl : 0)) * 16 + 4 * kk;
            wv[g] = sel4(ok, ld4(Wt + kq));
#pragma unroll
            for (int r = 0; r < RT; ++r) {
                int row = r * 16 + col;
                row = row < B ? row : B - 1;
                av[r][g] = ld4(D + ((int64_t)row * T + t) * K + kq);
            }
        }
        f32x4v acc[RT];
#pragma unroll
        for (int r = 0; r < RT; ++r) acc[r] = (f32x4v){0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int g = 0; g < G; ++g)
#pragma unroll
            for (int q = 0; q < 4; ++q)
#pragma unroll
                for (int r = 0; r < RT; ++r) acc[r] = mfma16(at4(av[r][g], q), at4(wv[g], q), acc[r]);
#pragma unroll
        for (int r = 0; r < RT; ++r)
#pragma unroll
            for (int q = 0; q < 4; ++q) red[wave][r * 16 + kk * 4 + q][col] = acc[r][q];
        __syncthreads();
        float* Pl = P + ((int64_t)l * ns + s) * B * N2;
        for (int p = tid; p < B * 16; p += BW * 64) {
            const int b = p >> 4, cc = p & 15;
            float v = red[0][b][cc];
#pragma unroll
            for (int w = 1; w < BW; ++w) v += red[w][b][cc];
            Pl[(int64_t)b * N2 + c0 + cc] = v;
        }
    }
    if (!FUSE) return;
    // ---- publish the tile, arrive; the last arriver of a group runs E(k + 1) for it
    const int HX = H >> 4, x = blockIdx.x;
    const int role = x >= HX ? l : (l >= 1 ? l - 1 : L), ux = x >= HX ? x - HX : x;
    const int need = (role >= L - 1) ? ns : 2 * ns;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        int* c = cnt + role * HX + ux;
        const int old = __hip_atomic_fetch_add(c, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const int last = old == need - 1;
        if (last) {
            __hip_atomic_store(c, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        s_last = last;
    }
    __syncthreads();
    if (!s_last) return;
    for (int q = tid; q < B * 16; q += BW * 64)
        bwd_elem_point(dout, P, ns, dcn, Cst, Gs, DAw, dx, acc_x, B, T, H, L, k + 1, role, q >> 4,
                       ux * 16 + (q & 15));
}

// ------------------------------------------------------------------------- persistent backward
// ONE launch runs the backward recurrence of all layers (option LSTM_PERSIST). Workgroup
// (l, bg, ct) owns the 16 columns n = 16 ct .. of P_l = DA_l . wcat_l (K = 4H) for the 16 batch
// rows of bg, with its slice of wcatT_l ([16][4H], 128 KB at H = 512) resident in registers:
//   ct >= H/16 (recurrent tile, units u = 16 (ct - H/16) ..): frame t takes the recurrent grad of
//     h_l(t) from DA_l(t+1), adds the grad from above (dout for the top layer, else the input-grad
//     tile of layer l+1 for the same units and frame, handed over by workgroup (l+1, bg, ct - H/16)),
//     runs the cell backward of its 16 x 16 points (dc kept in registers across frames) and
//     publishes DA_l(t) of its units;
//   ct < H/16 (input tile): frame t contracts DA_l(t) into the input grad of layer l (dx for l = 0,
//     else handed to the recurrent tile of layer l-1).
// The hand-offs are those of lstm_fwd_pers (write-through stores, drain, barrier, one arrival;
// sc1 loads after a bounded poll). The contraction keeps the exact split structure of
// lstm_bwd_gemm + lstm_bwd_elem (4 splits of the 4H/16 k-groups, each 4 interleaved chains summed
// in chain order, the splits summed in ascending order), so both forms give the same bits: wave w
// runs chains (s, c) = (w / 2, 2 (w % 2) + h), h = 0, 1, of G k-groups each (H % 128 == 0, G = H/64).
// grid L * NBG * 2H/16, FW waves. XP [L-1][B][T][H]: the input-grad tiles between layers.
template <int G>
__global__ __launch_bounds__(FW * 64) void lstm_bwd_pers(const float* dout, const float* wcatT, const float* Cst,
                                                         const float* Gs, float* DA, float* dx, int acc_x,
                                                         float* XP, int B, int T, int H, int L, int NBG,
                                                         int* sync, int ctl) {
    const int NRT = H / 16, NCT = 2 * NRT;
    const int id = blockIdx.x, ct = id % NCT, bg = (id / NCT) % NBG, l = id / (NCT * NBG);
    const bool recw = ct >= NRT;
    const int ut = recw ? ct - NRT : ct;
    __shared__ float red[16][16][17];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, col = lane & 15, kk = lane >> 4;
    const int K = 4 * H, gper = 4 * G;
    const int64_t BTH = (int64_t)B * T * H;
    float4 wr[2][G];
    {
        const float* Wt = wcatT + (int64_t)l * 2 * H * K + (int64_t)(ct * 16 + col) * K;
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int g = 0; g < G; ++g)
                wr[h][g] = ld4(Wt + ((wave >> 1) * gper + 2 * (wave & 1) + h + 4 * g) * 16 + 4 * kk);
    }
    const __amdgpu_buffer_rsrc_t rda = buf_rsrc(DA + l * 4 * BTH, (uint32_t)(BTH * 16));
    const __amdgpu_buffer_rsrc_t rxp = buf_rsrc(XP, (uint32_t)((L > 1 ? L - 1 : 1) * BTH * 4));
    const int arow = min(bg * 16 + col, B - 1);
    // point phase: thread p < 256 owns (row 16 bg + p / 16, unit 16 ut + p % 16)
    const int pr = tid >> 4, pu = ut * 16 + (tid & 15), pb = bg * 16 + pr;
    const bool pact = tid < 256 && pb < B;
    const int pbc = min(pb, B - 1);
    const float* Cl = Cst + l * BTH;
    const float* Gl = Gs + l * 4 * BTH;
    int* const cnt_da = sync + (l * NBG + bg) * SYNC_LINE;  // DA_l rows of bg: NRT arrivals per frame
    int* const xf_out = sync + (L * NBG + ((l > 0 ? l - 1 : 0) * NBG + bg) * NRT + ut) * SYNC_LINE;
    const int* const xf_in = sync + (L * NBG + (l * NBG + bg) * NRT + ut) * SYNC_LINE;
    int* const err = sync + SYNC_LINES * SYNC_LINE;
    const bool top = l == L - 1;
    bool live = true;
    const int spins = ctl_spins(ctl);
    const bool silent = (ctl & CTL_FAULT) && blockIdx.x == NRT;  // layer 0's first recurrent tile
    float dcn = 0.f;
    for (int i = 0; i < T; ++i) {
        const int t = T - 1 - i;
        LSTM_TRACE(1, i, 0);
        // the point phase's own operands (forward state, dout): loaded after the poll (a poll's
        // wait would otherwise wait for them), ahead of the DA loads
        float ig = 0.f, fg = 0.f, gg = 0.f, og = 0.f, c = 0.f, cpl = 0.f, dtop = 0.f;
        const int64_t o = ((int64_t)pbc * T + t) * H + pu;
        auto load_point = [&]() {
            if (recw && tid < 256) {
                const float* gs = Gl + ((int64_t)pbc * T + t) * 4 * H;
                ig = gs[pu];
                fg = gs[H + pu];
                gg = gs[2 * H + pu];
                og = gs[3 * H + pu];
                c = Cl[o];
                cpl = Cl[t > 0 ? o - H : o];
                if (top) dtop = dout[((int64_t)pbc * H + pu) * T + t];
            }
        };
        // ---- the contraction over DA_l(tf): tf = t + 1 for the recurrent tile, t for the input tile
        const int tf = recw ? t + 1 : t;
        float tile = 0.f;
        if (tf < T) {
            if (wave == 0 && live) live = poll_ge(cnt_da, NRT * (T - tf), err, spins);
            __syncthreads();
            LSTM_TRACE(1, i, 1);
            load_point();  // (older than the DA loads: the MFMAs' in-order waits are not pushed back)
            float4 a[2][G];
            const uint32_t rb = (uint32_t)(((int64_t)arow * T + tf) * K + 4 * kk) * 4u;
            // issued in the order the MFMAs consume them (k-group g of both chains), so the chains
            // start as the first loads land instead of after half of them
#pragma unroll
            for (int g = 0; g < G; ++g)
#pragma unroll
                for (int h = 0; h < 2; ++h)
                    a[h][g] = ld4_sc1(rda, rb + (uint32_t)((wave >> 1) * gper + 2 * (wave & 1) + h + 4 * g) * 64u);
            __builtin_amdgcn_sched_barrier(0);
            f32x4v acc[2] = {(f32x4v){0.f, 0.f, 0.f, 0.f}, (f32x4v){0.f, 0.f, 0.f, 0.f}};
#pragma unroll
            for (int g = 0; g < G; ++g)
#pragma unroll
                for (int q = 0; q < 4; ++q)
#pragma unroll
                    for (int h = 0; h < 2; ++h) acc[h] = mfma16(at4(a[h][g], q), at4(wr[h][g], q), acc[h]);
#pragma unroll
            for (int h = 0; h < 2; ++h)
#pragma unroll
                for (int q = 0; q < 4; ++q) red[2 * wave + h][kk * 4 + q][col] = acc[h][q];
            __syncthreads();
            LSTM_TRACE(1, i, 2);
            if (tid < 256) {
                const int r = tid >> 4, cc = tid & 15;
                float tot = 0.f;
#pragma unroll
                for (int s = 0; s < 4; ++s) {
                    float v = red[4 * s][r][cc];
#pragma unroll
                    for (int w = 1; w < 4; ++w) v += red[4 * s + w][r][cc];
                    tot += v;
                }
                tile = tot;
            }
        } else {
            load_point();
        }
        bool publish = false;
        int* pub = cnt_da;
        if (!recw) {
            // ---- input tile: dx (layer 0) or the grad from above of layer l-1
            if (l == 0) {
                if (dx && pact) {
                    const int64_t ox = ((int64_t)pb * H + pu) * T + t;
                    dx[ox] = acc_x ? dx[ox] + tile : tile;
                }
            } else {
                if (pact)
                    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, tile), rxp,
                                                          (int)((uint32_t)((l - 1) * BTH + o) * 4u), 0, SC1);
                publish = true;
                pub = xf_out;
            }
        } else {
            // ---- recurrent tile: the cell backward of frame t
            float above = dtop;
            if (!top) {
                if (wave == 0 && live) live = poll_ge(xf_in, i + 1, err, spins);
                __syncthreads();
                LSTM_TRACE(1, i, 3);
                if (tid < 256)
                    above = __builtin_bit_cast(
                        float, __builtin_amdgcn_raw_buffer_load_b32(rxp, (int)((uint32_t)(l * BTH + o) * 4u), 0, SC1));
            }
            const bool rec = t < T - 1;
            const float dh = above + (rec ? tile : 0.f);
            float g4[4];
            cell_bwd(dh, dcn, rec, ig, fg, gg, og, c, t > 0 ? cpl : 0.f, g4, &dcn);
            if (pact) {
                const uint32_t ob = (uint32_t)(((int64_t)pb * T + t) * 4 * H + pu) * 4u;
#pragma unroll
                for (int q = 0; q < 4; ++q)
                    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, g4[q]), rda,
                                                          (int)(ob + (uint32_t)(q * H) * 4u), 0, SC1);
            }
            publish = true;
        }
        // publish: every storing wave drained, a barrier (also ends this frame's reads of red), one
        // lane's arrival
        LSTM_TRACE(1, i, 4);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        LSTM_TRACE(1, i, 5);
        if (publish && tid == 0 && !silent) __hip_atomic_fetch_add(pub, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    // the DA counters (NRT arrivals per frame) and the input-tile flags (one per frame)
    finish_launch(sync, L * NBG, NRT * T, (L - 1) * NBG * NRT, T);
}

// ------------------------------------------------------------------------- layout kernels
// wcat[j] = [w_ih[j] | w_hh[j]] ([4H][2H]), wcatT its transpose ([2H][4H]), bsum = b_ih + b_hh
__global__ void lstm_pack_kernel(const float* wih, const float* whh, const float* bih, const float* bhh,
                                 float* wcat, float* wcatT, float* bsum, int H) {
    __shared__ float tile[32][33];
    const int n0 = blockIdx.x * 32, j0 = blockIdx.y * 32;  // n over 2H, j over 4H (both % 32 == 0)
    const int N2 = 2 * H, K4 = 4 * H;
    for (int i = threadIdx.y; i < 32; i += 8) {
        const int jj = j0 + i, n = n0 + threadIdx.x;
        const float v = n < H ? wih[(int64_t)jj * H + n] : whh[(int64_t)jj * H + n - H];
        wcat[(int64_t)jj * N2 + n] = v;
        tile[i][threadIdx.x] = v;
    }
    __syncthreads();
    for (int i = threadIdx.y; i < 32; i += 8) {
        const int n = n0 + i, jj = j0 + threadIdx.x;
        wcatT[(int64_t)n * K4 + jj] = tile[threadIdx.x][i];
    }
    if (blockIdx.x == 0 && threadIdx.y == 0) {
        const int jj = j0 + threadIdx.x;
        bsum[jj] = bih[jj] + bhh[jj];
    }
}

// out[z][c][r] = in[z][r][c]: in [R][Cc] per batch z
__global__ void transpose_kernel(const float* in, float* out, int R, int Cc) {
    __shared__ float tile[32][33];
    const int64_t zo = (int64_t)blockIdx.z * R * Cc;
    in += zo;
    out += zo;
    const int r0 = blockIdx.y * 32, c0 = blockIdx.x * 32;
    for (int i = threadIdx.y; i < 32; i += 8) {
        const int r = r0 + i, c = c0 + threadIdx.x;
        if (r < R && c < Cc) tile[i][threadIdx.x] = in[(int64_t)r * Cc + c];
    }
    __syncthreads();
    for (int i = threadIdx.y; i < 32; i += 8) {
        const int c = c0 + i, r = r0 + threadIdx.x;
        if (r < R && c < Cc) out[(int64_t)c * R + r] = tile[threadIdx.x][i];
    }
}

// out[b][u][t] = Y[b][t][u] (+ x[b][u][t]) (lstm.py:24-27 skip, back to [B][C][T])
__global__ void lstm_out_skip(const float* Y, const float* x, float* out, int B, int T, int H, int skip) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (int64_t)B * H * T) return;
    const int t = (int)(i % T);
    const int64_t bu = i / T;
    const int b = (int)(bu / H), u = (int)(bu - (int64_t)b * H);
    const float y = Y[((int64_t)b * T + t) * H + u];
    out[i] = skip ? y + x[i] : y;
}

// ------------------------------------------------------------------------- weight grads
// dwcat_l[j][n] = sum_m DA_l[m][j] Z(m, n), Z = [x_l(m, :) | h_l(m-1, :) (0 at t = 0) | 1]
struct LdWcat {
    static constexpr bool A_K_FAST = false, B_N_FAST = true, VEC = true;
    const float* DA;
    const float* in;
    const float* Yl;
    int H, T;
    FastDiv fT;
    ENCX_DEV float a(int j, int m) const { return DA[(int64_t)m * 4 * H + j]; }
    ENCX_DEV float b(int m, int n) const {
        // one load from a clamped address, the value chosen afterwards (no branch around it)
        const bool rec = n >= H;
        const int u = rec ? (n - H < H ? n - H : H - 1) : n;
        const int mm = rec ? (m > 0 ? m - 1 : 0) : m;
        const float v = (rec ? Yl : in)[(int64_t)mm * H + u];
        const int t = m - (int)fdiv((uint32_t)m, fT) * T;
        return rec && t == 0 ? 0.f : v;
    }
    // quads (H % 4 == 0, so a quad never straddles the x | h boundary)
    ENCX_DEV f32x4 a4(int j, int m) const { return ld4u(DA + (int64_t)m * 4 * H + j); }
    ENCX_DEV f32x4 b4(int m, int n) const {
        if (n + 3 >= 2 * H) {
            f32x4 v;
#pragma unroll
            for (int q = 0; q < 4; ++q) v[q] = b(m, n + q);
            return v;
        }
        const bool rec = n >= H;
        const int t = m - (int)fdiv((uint32_t)m, fT) * T;
        const f32x4 v = ld4u(rec ? Yl + (int64_t)(m > 0 ? m - 1 : 0) * H + (n - H) : in + (int64_t)m * H + n);
        return rec && t == 0 ? (f32x4){0.f, 0.f, 0.f, 0.f} : v;
    }
};
struct EpSlabs {  // split-K partial slabs [z][M][N]
    float* ws;
    int M, N;
    ENCX_DEV void operator()(int m, int n, float v) const {
        ws[((int64_t)blockIdx.z * M + m) * N + n] = v;
    }
};
// unsplit weight grad: the GEMM's element straight into dw_ih (n < H) or dw_hh (n < 2H); += when
// acc (the same bits as one slab through lstm_slab_reduce)
struct EpDWcat {
    float* dwi;
    float* dwh;
    int H, acc;
    ENCX_DEV void operator()(int m, int n, float v) const {
        if (n >= 2 * H) return;
        float* p = n < H ? dwi + (int64_t)m * H + n : dwh + (int64_t)m * H + (n - H);
        *p = acc ? *p + v : v;
    }
};
// sum split slabs [S][4H][2H] in ascending slab order into dw_ih (n < H) and dw_hh; += when acc
__global__ __launch_bounds__(256) void lstm_slab_reduce(const float* ws, int S, int H, float* dwi, float* dwh,
                                                        int acc) {
    __shared__ float red[256];
    const int M = 4 * H, N = 2 * H;
    const int64_t i = (int64_t)blockIdx.x * 64 + (threadIdx.x & 63);
    const bool valid = i < (int64_t)M * N;
    const float s = slab_sum_256(ws + (valid ? i : 0), S, (int64_t)M * N, valid, red);
    if (threadIdx.x >= 64 || !valid) return;
    const int m = (int)(i / N), n = (int)(i - (int64_t)m * N);
    float* p = n < H ? dwi + (int64_t)m * H + n : dwh + (int64_t)m * H + (n - H);
    *p = acc ? *p + s : s;
}
// the bias grads (b_ih and b_hh get the same): db[j] = sum over the B T positions m of DA[m][j],
// as a column sum beside the weight-grad GEMM (in the GEMM, as a ones column, 2H + 1 columns took
// a ninth 128-column tile for one column). Fixed order: part[c][j] sums the rows of chunk c of
// BIAS_ROWS (4 row lanes, each ascending, then the lanes in order); lstm_bias_fin sums the chunks
// in order.
constexpr int BIAS_ROWS = 160;
__global__ __launch_bounds__(256) void lstm_bias_part(const float* DA, int M, int N4, float* part) {
    __shared__ float red[4][65];
    const int c = threadIdx.x & 63, r = threadIdx.x >> 6;
    const int j = blockIdx.x * 64 + c, m0 = blockIdx.y * BIAS_ROWS, m1 = min(M, m0 + BIAS_ROWS);
    float s = 0.f;
    if (j < N4) {
        const float* p = DA + j;
        int m = m0 + r;
        for (; m + 12 < m1; m += 16) {  // four rows in flight, added in row order
            const float v0 = p[(int64_t)m * N4], v1 = p[(int64_t)(m + 4) * N4];
            const float v2 = p[(int64_t)(m + 8) * N4], v3 = p[(int64_t)(m + 12) * N4];
            s += v0;
            s += v1;
            s += v2;
            s += v3;
        }
        for (; m < m1; m += 4) s += p[(int64_t)m * N4];
    }
    red[r][c] = s;
    __syncthreads();
    if (r == 0 && j < N4) part[(int64_t)blockIdx.y * N4 + j] = ((red[0][c] + red[1][c]) + red[2][c]) + red[3][c];
}
__global__ __launch_bounds__(256) void lstm_bias_fin(const float* part, int nchunk, int N4, float* db1, float* db2,
                                                     int acc) {
    const int j = blockIdx.x * 256 + threadIdx.x;
    if (j >= N4) return;
    float v = part[j];
    for (int c = 1; c < nchunk; ++c) v += part[(int64_t)c * N4 + j];
    if (db1) db1[j] = acc ? db1[j] + v : v;
    if (db2) db2[j] = acc ? db2[j] + v : v;
}
// the weight grad's operand as one plain matrix xh[b T + t] = [x_l(t) | h_l(t - 1)] ([M][2H]; h 0 at
// t = 0), so dW_ih and dW_hh come out of ONE library GEMM (2H output rows instead of two of H)
__global__ __launch_bounds__(256) void lstm_xh(const float* in, const float* Yl, float* xh, int T, int H, int64_t n4) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;  // quad index
    if (i >= n4) return;
    const int64_t e = i * 4, row = e / (2 * H);
    const int c = (int)(e - row * 2 * H), t = (int)(row % T);
    f32x4 v;
    if (c < H) v = *(const f32x4*)(in + row * H + c);
    else v = t > 0 ? *(const f32x4*)(Yl + (row - 1) * H + (c - H)) : (f32x4){0.f, 0.f, 0.f, 0.f};
    *(f32x4*)(xh + e) = v;
}

// ------------------------------------------------------------------------- dispatch
template <int G>
static void fwd_rt(int RT, dim3 grid, hipStream_t st, const float* xt, const float* wcat, const float* bsum,
                   float* Y, float* C, float* Gs, int B, int T, int H, int k) {
    switch (RT) {
        case 1: hipLaunchKernelGGL((lstm_fwd_wave<G, 1>), grid, dim3(FW * 64), 0, st, xt, wcat, bsum, Y, C, Gs, B, T, H, k); break;
        case 2: hipLaunchKernelGGL((lstm_fwd_wave<G, 2>), grid, dim3(FW * 64), 0, st, xt, wcat, bsum, Y, C, Gs, B, T, H, k); break;
        case 3: hipLaunchKernelGGL((lstm_fwd_wave<G, 3>), grid, dim3(FW * 64), 0, st, xt, wcat, bsum, Y, C, Gs, B, T, H, k); break;
        default: hipLaunchKernelGGL((lstm_fwd_wave<G, 4>), grid, dim3(FW * 64), 0, st, xt, wcat, bsum, Y, C, Gs, B, T, H, k); break;
    }
}
static void fwd_step(int G, int RT, dim3 grid, hipStream_t st, const float* xt, const float* wcat,
                     const float* bsum, float* Y, float* C, float* Gs, int B, int T, int H, int k) {
    if (G <= 1) fwd_rt<1>(RT, grid, st, xt, wcat, bsum, Y, C, Gs, B, T, H, k);
    else if (G <= 2) fwd_rt<2>(RT, grid, st, xt, wcat, bsum, Y, C, Gs, B, T, H, k);
    else if (G <= 4) fwd_rt<4>(RT, grid, st, xt, wcat, bsum, Y, C, Gs, B, T, H, k);
    else if (G <= 8) fwd_rt<8>(RT, grid, st, xt, wcat, bsum, Y, C, Gs, B, T, H, k);
    else fwd_rt<16>(RT, grid, st, xt, wcat, bsum, Y, C, Gs, B, T, H, k);
}
struct BwdArgs {
    const float* DA;
    const float* wcatT;
    float* P;
    int B, T, H, L, k, gper;
    const float* dout;
    float* dcn;
    const float* Cst;
    const float* Gs;
    float* dx;
    int acc_x;
    int* cnt;  // non-NULL: fused with E(k + 1)
};
template <int G, int RT>
static void bwd_launch(dim3 grid, hipStream_t st, const BwdArgs& a) {
    if (a.cnt)
        hipLaunchKernelGGL((lstm_bwd_gemm<G, RT, true>), grid, dim3(BW * 64), 0, st, a.DA, a.wcatT, a.P, a.B, a.T, a.H,
                           a.L, a.k, a.gper, a.dout, a.dcn, a.Cst, a.Gs, (float*)a.DA, a.dx, a.acc_x, a.cnt);
    else
        hipLaunchKernelGGL((lstm_bwd_gemm<G, RT, false>), grid, dim3(BW * 64), 0, st, a.DA, a.wcatT, a.P, a.B, a.T,
                           a.H, a.L, a.k, a.gper, a.dout, a.dcn, a.Cst, a.Gs, (float*)a.DA, a.dx, a.acc_x, a.cnt);
}
template <int G>
static void bwd_rt(int RT, dim3 grid, hipStream_t st, const BwdArgs& a) {
    switch (RT) {
        case 1: bwd_launch<G, 1>(grid, st, a); break;
        case 2: bwd_launch<G, 2>(grid, st, a); break;
        case 3: bwd_launch<G, 3>(grid, st, a); break;
        default: bwd_launch<G, 4>(grid, st, a); break;
    }
}
static void bwd_gemm(int G, int RT, dim3 grid, hipStream_t st, const BwdArgs& a) {
    if (G <= 1) bwd_rt<1>(RT, grid, st, a);
    else if (G <= 2) bwd_rt<2>(RT, grid, st, a);
    else if (G <= 4) bwd_rt<4>(RT, grid, st, a);
    else if (G <= 8) bwd_rt<8>(RT, grid, st, a);
    else bwd_rt<16>(RT, grid, st, a);
}
// k-splits of the backward step GEMM (K = 4H in H/4 groups of 16): <= 4, dividing the groups,
// >= 8 groups each
static int bwd_splits(int64_t H) {
    const int groups = (int)(H / 4);
    int ns = groups / 8 < 4 ? groups / 8 : 4;
    if (ns < 1) ns = 1;
    while (groups % ns) --ns;
    return ns;
}
// ---- the persistent forms: residency and the hand-off words
static int device_cus() {
    static int cus[64];
    int d = 0;
    if (hipGetDevice(&d) != hipSuccess || d < 0 || d >= 64) return 0;
    if (!cus[d] && hipDeviceGetAttribute(&cus[d], hipDeviceAttributeMultiprocessorCount, d) != hipSuccess) cus[d] = 0;
    return cus[d];
}
// the persistent kernels' control word from the options (see ctl_spins)
static int pers_ctl() {
    const int64_t sp = encx_opt(OPT_LSTM_SPIN);
    return (int)((sp > 0 && sp < 31 ? sp : 0) | (encx_opt(OPT_LSTM_FAULT) ? CTL_FAULT : 0));
}
// every workgroup of a persistent launch must be resident at once: nwg within what the kernel's
// occupancy (registers, LDS, waves) admits on the device's CUs
static bool coresident(const void* kern, int64_t nwg) {
    int per = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kern, FW * 64, 0) != hipSuccess) return false;
    return per > 0 && nwg <= (int64_t)per * device_cus();
}
static int* sync_words() {
    static int* addr[64];
    int d = 0;
    if (hipGetDevice(&d) != hipSuccess || d < 0 || d >= 64) return nullptr;
    if (!addr[d] && hipGetSymbolAddress((void**)&addr[d], HIP_SYMBOL(g_lstm_sync)) != hipSuccess) addr[d] = nullptr;
    return addr[d];
}
// workgroups of the persistent forward, or 0 when the shape or the device does not admit it (the
// workgroups must be resident together: at most one per CU; the sequences' byte offsets 32-bit)
template <int G> static int fwd_pers_grid(int64_t B, int64_t T, int64_t H, int64_t L) {
    if (encx_opt(OPT_LSTM_PERSIST) == 0 || H % 128 || H > 512 || B * T * H * 4 >= ((int64_t)1 << 31)) return 0;
    const int64_t nbg = cdiv(B, 16), nwg = L * nbg * (H / PU);
    if (L * nbg > SYNC_LINES || nwg > device_cus() || !sync_words()) return 0;
    if (!coresident((const void*)lstm_fwd_pers<G>, nwg)) return 0;
    return (int)nwg;
}
// workgroups of the persistent backward, or 0 (as fwd_pers_grid; plus the hand-off lines)
// (DA's buffer offsets cover B T 4H floats, XP's (L - 1) B T H: both must fit the 32-bit offsets)
template <int G> static int bwd_pers_grid(int64_t B, int64_t T, int64_t H, int64_t L) {
    if (encx_opt(OPT_LSTM_PERSIST) == 0 || H % 128 || H > 512 || B * T * H * 16 >= ((int64_t)1 << 31) ||
        (L - 1) * B * T * H * 4 >= ((int64_t)1 << 31))
        return 0;
    const int64_t nbg = cdiv(B, 16), nwg = L * nbg * (2 * H / 16);
    if (L * nbg + (L - 1) * nbg * (H / 16) > SYNC_LINES || nwg > device_cus() || !sync_words()) return 0;
    if (!coresident((const void*)lstm_bwd_pers<G>, nwg)) return 0;
    return (int)nwg;
}
template <int G>
static bool fwd_pers_launch(hipStream_t st, const float* xt, const float* wcat, const float* bsum, float* Y,
                            float* C, float* Gs, int B, int T, int H, int L) {
    const int nwg = fwd_pers_grid<G>(B, T, H, L);
    if (!nwg) return false;
    hipLaunchKernelGGL((lstm_fwd_pers<G>), dim3((unsigned)nwg), dim3(FW * 64), 0, st, xt, wcat, bsum, Y, C, Gs, B, T,
                       H, (int)cdiv(B, 16), sync_words(), pers_ctl());
    return true;
}
template <int G>
static bool bwd_pers_launch(hipStream_t st, const float* dout, const float* wcatT, const float* Cst, const float* Gs,
                            float* DA, float* dx, int acc_x, float* XP, int B, int T, int H, int L) {
    const int nwg = bwd_pers_grid<G>(B, T, H, L);
    if (!nwg) return false;
    hipLaunchKernelGGL((lstm_bwd_pers<G>), dim3((unsigned)nwg), dim3(FW * 64), 0, st, dout, wcatT, Cst, Gs, DA, dx,
                       acc_x, XP, B, T, H, L, (int)cdiv(B, 16), sync_words(), pers_ctl());
    return true;
}

static bool lstm_shape_ok(int64_t B, int64_t T, int64_t H, int64_t L) {
    return B > 0 && B <= 64 && T > 0 && H >= 16 && (H % 16) == 0 && H <= 1024 && L >= 1 && L <= 16 &&
           B * T * 4 * H < ((int64_t)1 << 31);
}

__global__ void zero_ints(int* p, int n) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i < n) p[i] = 0;
}

}  // namespace

extern "C" {

int encx_lstm_pack(const float* w_ih, const float* w_hh, const float* b_ih, const float* b_hh, float* wcat,
                   float* wcatT, float* bsum, int64_t H, int64_t layer, encx_stream_t stream) {
    ENCX_REQUIRE(w_ih && w_hh && b_ih && b_hh && wcat && wcatT && bsum);
    ENCX_REQUIRE(H >= 16 && (H % 16) == 0 && H <= 1024 && layer >= 0);
    const int64_t wl = 8 * H * H;
    hipLaunchKernelGGL(lstm_pack_kernel, dim3((unsigned)(2 * H / 32), (unsigned)(4 * H / 32)), dim3(32, 8), 0,
                       (hipStream_t)stream, w_ih, w_hh, b_ih, b_hh, wcat + layer * wl, wcatT + layer * wl,
                       bsum + layer * 4 * H, (int)H);
    ENCX_CHECK_LAUNCH();
    return 0;
}

int encx_lstm_fwd(const float* x, const float* wcat, const float* bsum, float* xt, float* Y, float* Cst,
                  float* Gs, float* out, int skip, int64_t B, int64_t T, int64_t H, int64_t L,
                  encx_stream_t stream) {
    ENCX_REQUIRE(x && wcat && bsum && xt && Y && Cst && Gs && out);
    ENCX_REQUIRE(lstm_shape_ok(B, T, H, L));
    hipStream_t st = (hipStream_t)stream;
    encx_prof_scope ps(st, 2.0 * L * B * T * 4 * H * 2 * H, 4.0 * (L * 8 * H * H + B * T * H * (2 + 7 * L)),
                       "lstm_fwd");
    ps.tag(" H%ld L%ld T%ld", (long)H, (long)L, (long)T);
    hipLaunchKernelGGL(transpose_kernel, dim3((unsigned)cdiv(T, 32), (unsigned)cdiv(H, 32), (unsigned)B),
                       dim3(32, 8), 0, st, x, xt, (int)H, (int)T);
    const int RT = (int)cdiv(B, 16), G = (int)cdiv(H / 8, FW);
    bool pers = false;
    switch (G) {  // H / 64 (the persistent form needs H % 128 == 0)
        case 2: pers = fwd_pers_launch<2>(st, xt, wcat, bsum, Y, Cst, Gs, (int)B, (int)T, (int)H, (int)L); break;
        case 4: pers = fwd_pers_launch<4>(st, xt, wcat, bsum, Y, Cst, Gs, (int)B, (int)T, (int)H, (int)L); break;
        case 6: pers = fwd_pers_launch<6>(st, xt, wcat, bsum, Y, Cst, Gs, (int)B, (int)T, (int)H, (int)L); break;
        case 8: pers = fwd_pers_launch<8>(st, xt, wcat, bsum, Y, Cst, Gs, (int)B, (int)T, (int)H, (int)L); break;
        default: break;
    }
    if (pers) {
        ps.tag(" persist");
    } else {
        const dim3 grid((unsigned)(H / UNITS), (unsigned)L);
        for (int k = 0; k < (int)(T + L - 1); ++k)
            fwd_step(G, RT, grid, st, xt, wcat, bsum, Y, Cst, Gs, (int)B, (int)T, (int)H, k);
    }
    const int64_t n = B * H * T;
    hipLaunchKernelGGL(lstm_out_skip, dim3((unsigned)cdiv(n, 256)), dim3(256), 0, st, Y + (L - 1) * B * T * H, x,
                       out, (int)B, (int)T, (int)H, skip);
    ENCX_CHECK_LAUNCH();
    return 0;
}

int encx_lstm_trace(int64_t* out, int64_t n) {
#ifdef ENCX_LSTM_TRACE
    ENCX_REQUIRE(out && n >= 0 && n <= 2 * 256 * 128 * 8);
    hipError_t e = hipDeviceSynchronize();
    if (e == hipSuccess) e = hipMemcpyFromSymbol(out, HIP_SYMBOL(g_lstm_trace), (size_t)n * sizeof(int64_t));
    return (int)e;
#else
    (void)out;
    (void)n;
    return ENCX_EINVAL;
#endif
}

int encx_lstm_sync_errors(int64_t* count) {
    ENCX_REQUIRE(count);
    int* w = sync_words();
    ENCX_REQUIRE(w);
    hipError_t e = hipDeviceSynchronize();
    int v = 0;
    if (e == hipSuccess) e = hipMemcpy(&v, w + SYNC_LINES * SYNC_LINE, sizeof(int), hipMemcpyDeviceToHost);
    if (e == hipSuccess) e = hipMemset(w + SYNC_LINES * SYNC_LINE, 0, sizeof(int));
    if (e == hipSuccess) e = hipDeviceSynchronize();
    *count = v;
    return (int)e;
}

int encx_lstm_sync_read(int32_t* count, encx_stream_t stream) {
    ENCX_REQUIRE(count);
    int* w = sync_words();
    ENCX_REQUIRE(w);
    hipLaunchKernelGGL(sync_read_kernel, dim3(1), dim3(1), 0, (hipStream_t)stream, w, (int*)count);
    ENCX_CHECK_LAUNCH();
    return 0;
}

size_t encx_lstm_bwd_workspace(int64_t B, int64_t T, int64_t H, int64_t L) {
    // step form: dcn [L][B][H], P [L][ns][B][2H], the fused step's arrival counters [(L + 1) * H/16]
    // (int); persistent form: XP [L-1][B][T][H]
    const size_t step = (size_t)L * B * H + (size_t)L * bwd_splits(H) * B * 2 * H + (size_t)(L + 1) * (H / 16);
    const size_t pers = (size_t)(L > 1 ? L - 1 : 1) * B * T * H;
    return (step > pers ? step : pers) * sizeof(float);
}

int encx_lstm_bwd(const float* dout, const float* wcatT, const float* Cst, const float* Gs, float* DA, float* dx,
                  int acc_x, float* ws, int64_t B, int64_t T, int64_t H, int64_t L, encx_stream_t stream) {
    ENCX_REQUIRE(dout && wcatT && Cst && Gs && DA && ws);
    ENCX_REQUIRE(lstm_shape_ok(B, T, H, L));
    hipStream_t st = (hipStream_t)stream;
    encx_prof_scope ps(st, 2.0 * L * B * T * 4 * H * 2 * H, 4.0 * (L * 8 * H * H + B * T * H * (2 + 10 * L)),
                       "lstm_bwd");
    ps.tag(" H%ld L%ld T%ld", (long)H, (long)L, (long)T);
    float* dcn = ws;
    float* P = ws + L * B * H;
    const int ns = bwd_splits(H), gper = (int)(H / 4) / ns, G = (int)cdiv(gper, BW), RT = (int)cdiv(B, 16);
    int* cnt = (int*)(P + L * ns * B * 2 * H);
    const int BH = (int)(B * H);
    const dim3 egrid((unsigned)cdiv(BH, 256), (unsigned)(L + (dx ? 1 : 0)));
    const dim3 ggrid((unsigned)(2 * H / 16), (unsigned)ns, (unsigned)L);
    {
        bool pers = false;
#define BWD_PERS(G_) \
    bwd_pers_launch<G_>(st, dout, wcatT, Cst, Gs, DA, dx, acc_x, ws, (int)B, (int)T, (int)H, (int)L)
        if (H % 64 == 0) switch (H / 64) {
                case 2: pers = BWD_PERS(2); break;
                case 4: pers = BWD_PERS(4); break;
                case 6: pers = BWD_PERS(6); break;
                case 8: pers = BWD_PERS(8); break;
                default: break;
            }
#undef BWD_PERS
        if (pers) {
            ps.tag(" persist");
            ENCX_CHECK_LAUNCH();
            return 0;
        }
    }
    const int steps = (int)(T + L);
    // E(k + 1) fused into G(k): opt-in (ENCX_LSTM_FUSE=1). Measured slower in the config-3 step:
    // 21.7 us per fused launch against 9.0 + 4.9 us for G(k) and E(k + 1) (profiles/r03): each
    // workgroup's agent-scope release (L2 write-back) and the last arriver's acquire cost more
    // than the launch they save.
    const bool fuse = encx_opt(OPT_LSTM_FUSE) != 0;
    BwdArgs a{DA, wcatT, P, (int)B, (int)T, (int)H, (int)L, 0, gper, dout, dcn, Cst, Gs, dx, acc_x,
              fuse ? cnt : nullptr};
    if (fuse) {
        // the arrival counters zeroed by a kernel, not a hipMemsetAsync: a memset node captured into
        // a HIP graph was not ordered before the next kernel in replays (round 5, the persistent
        // form's counters; see g_lstm_sync)
        const int ncnt = (int)((L + 1) * (H / 16));
        hipLaunchKernelGGL(zero_ints, dim3((unsigned)cdiv(ncnt, 256)), dim3(256), 0, st, cnt, ncnt);
        hipLaunchKernelGGL(lstm_bwd_elem, egrid, dim3(256), 0, st, dout, P, ns, dcn, Cst, Gs, DA, dx, acc_x,
                           (int)B, (int)T, (int)H, (int)L, 0);
        for (int k = 0; k < steps - 1; ++k) {
            a.k = k;
            bwd_gemm(G, RT, ggrid, st, a);
        }
    } else {
        for (int k = 0; k < steps; ++k) {
            hipLaunchKernelGGL(lstm_bwd_elem, egrid, dim3(256), 0, st, dout, P, ns, dcn, Cst, Gs, DA, dx, acc_x,
                               (int)B, (int)T, (int)H, (int)L, k);
            a.k = k;
            if (k < steps - 1) bwd_gemm(G, RT, ggrid, st, a);
        }
    }
    ENCX_CHECK_LAUNCH();
    return 0;
}

}  // extern "C"
// floats of the weight grad's main workspace: the own GEMM's split slabs, or the library GEMM's
// 8 position-chunk slabs and the [x | h(t-1)] matrix; the bias partials follow
static size_t wsl_main(int64_t B, int64_t T, int64_t H) {
    const int M = (int)(B * T), N4 = (int)(4 * H), Nw = (int)(2 * H);
    const int S = gemm_slabs(M, gemm_splits_128(N4, Nw, M, 256, (int)encx_opt(OPT_LSTM_WG_SPLITS)));
    return std::max((size_t)S * N4 * Nw, (size_t)8 * N4 * Nw + (size_t)B * T * 2 * H);
}
extern "C" {
size_t encx_lstm_bwd_weight_workspace(int64_t B, int64_t T, int64_t H) {
    const int M = (int)(B * T), N4 = (int)(4 * H);
    return (wsl_main(B, T, H) + (size_t)cdiv(M, BIAS_ROWS) * N4) * sizeof(float);
}

int encx_lstm_bwd_weight(const float* DA, const float* xt, const float* Y, float* dw_ih, float* dw_hh,
                         float* db_ih, float* db_hh, int acc, float* ws, int64_t B, int64_t T, int64_t H,
                         int64_t L, int64_t layer, encx_stream_t stream) {
    ENCX_REQUIRE(DA && xt && Y && dw_ih && dw_hh && ws);
    ENCX_REQUIRE(lstm_shape_ok(B, T, H, L) && layer >= 0 && layer < L);
    hipStream_t st = (hipStream_t)stream;
    // (flops: the GEMM's 2 BT 4H 2H and the bias grads' BT 4H adds)
    encx_prof_scope ps(st, 2.0 * B * T * 4 * H * 2 * H + (double)B * T * 4 * H, 4.0 * (B * T * H * 7 + 8 * H * H),
                       "lstm_wgrad");
    ps.tag(" H%ld T%ld", (long)H, (long)T);
    const int64_t BTH = B * T * H;
    const float* in = layer == 0 ? xt : Y + (layer - 1) * BTH;
    const int M = (int)(B * T), N4 = (int)(4 * H), Nw = (int)(2 * H);
    const int sp = gemm_splits_128(N4, Nw, M, 256, (int)encx_opt(OPT_LSTM_WG_SPLITS));
    const int S = gemm_slabs(M, sp);
    const float* DAl = DA + layer * 4 * BTH;
    const LdWcat ld{DAl, in, Y + layer * BTH, (int)H, (int)T, make_fastdiv((uint32_t)T)};
    int rc;
    // [dW_ih | dW_hh]^T (2H x 4H, column-major) = [x | h(t-1)]^T DA through hipBLASLt (blas.hip),
    // else the own GEMM. The B T positions are cut into KB equal chunks of about 300 (a strided
    // batch: one slab [4H][2H] per chunk) summed in order by lstm_slab_reduce:
    // one library accumulation chain over all 2400 positions of config 3 was 5x the error of plain
    // fp32 (test_lstm_vs_oracle), the chunked form is within it.
    int KB = 0;
    for (const int c : {8, 6, 5, 4, 3, 2, 1})
        if (M % c == 0 && M / c >= 64) {
            KB = c;
            break;
        }
    bool lib = KB > 0 && H % 4 == 0 && (encx_opt(OPT_BLAS) & 1) && (size_t)KB * N4 * Nw <= wsl_main(B, T, H);
    if (lib) {
        const int kc = M / KB;
        float* xh = ws + (size_t)KB * N4 * Nw;
        hipLaunchKernelGGL(lstm_xh, dim3((unsigned)cdiv(2 * BTH / 4, 256)), dim3(256), 0, st, in, Y + layer * BTH, xh,
                           (int)T, (int)H, 2 * BTH / 4);
        ENCX_CHECK_LAUNCH();
        // slab c (2H x 4H, column-major = [4H][2H]) = xh^T DA over position chunk c
        lib = encx_sgemm(st, false, true, Nw, N4, kc, xh, Nw, DAl, N4, ws, Nw, false, KB, (int64_t)kc * Nw,
                         (int64_t)kc * N4, (int64_t)N4 * Nw) == 0;
        if (lib) {
            hipLaunchKernelGGL(lstm_slab_reduce, dim3((unsigned)cdiv((int64_t)N4 * Nw, 64)), dim3(256), 0, st, ws,
                               KB, (int)H, dw_ih, dw_hh, acc);
            ENCX_CHECK_LAUNCH();
        }
    }
    if (!lib && S == 1) {
        rc = gemm_launch_128(ld, EpDWcat{dw_ih, dw_hh, (int)H, acc}, N4, Nw, M, st, 1);
        if (rc) return rc;
    } else if (!lib) {
        rc = gemm_launch_128(ld, EpSlabs{ws, N4, Nw}, N4, Nw, M, st, sp);
        if (rc) return rc;
        hipLaunchKernelGGL(lstm_slab_reduce, dim3((unsigned)cdiv((int64_t)N4 * Nw, 64)), dim3(256), 0, st, ws, S,
                           (int)H, dw_ih, dw_hh, acc);
        ENCX_CHECK_LAUNCH();
    }
    if (db_ih || db_hh) {
        const int nch = (int)cdiv(M, BIAS_ROWS);
        float* part = ws + wsl_main(B, T, H);
        hipLaunchKernelGGL(lstm_bias_part, dim3((unsigned)cdiv(N4, 64), (unsigned)nch), dim3(256), 0, st, DAl, M, N4,
                           part);
        hipLaunchKernelGGL(lstm_bias_fin, dim3((unsigned)cdiv(N4, 256)), dim3(256), 0, st, part, nch, N4, db_ih,
                           db_hh, acc);
        ENCX_CHECK_LAUNCH();
    }
    return 0;
}

}  // extern "C"
