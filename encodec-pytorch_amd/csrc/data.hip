// encx -- batch assembly for training from clips resident in HBM (customAudioDataset.py).
//
// The reference loads each file per item on the host, crops a random tensor_cut window
// (customAudioDataset.py:64-69), expands mono to `channels` (:51-54) and zero-pads the batch
// to its longest item (pad_sequence / collate_fn, :72-91). Here the decoded clips stay in HBM
// as one pool and one launch writes the whole [B][C][Tmax] batch as a coalesced row-by-row
// copy (4 B read + 4 B written per sample; padding is write-only), HBM-bound.
#include "common.h"

namespace {

constexpr int CC_THREADS = 256, CC_PER = 4;  // 1024 samples of one row per workgroup

// grid (ceil(Tmax / 1024), B*C): blockIdx.y is the output row (b, c), so the per-row metadata
// is read once into scalars and no lane divides; each lane copies 4 samples 256 apart, so
// every wave load / store instruction covers 64 consecutive samples.
__global__ __launch_bounds__(CC_THREADS) void crop_collate_kernel(
    const float* __restrict__ pool, const int64_t* __restrict__ offsets,
    const int64_t* __restrict__ lengths, const int64_t* __restrict__ src_ch,
    const int64_t* __restrict__ starts, const int64_t* __restrict__ out_len,
    float* __restrict__ out, int C, int64_t Tmax) {
    const int row = blockIdx.y;
    const int b = row / C;
    const int c = row - b * C;
    const int64_t n = out_len[b];
    const int64_t cs = src_ch[b] == 1 ? 0 : c;  // mono -> expand (customAudioDataset.py:51-54)
    const float* src = pool + offsets[b] + cs * lengths[b] + starts[b];
    float* dst = out + (int64_t)row * Tmax;
    const int64_t t0 = (int64_t)blockIdx.x * (CC_THREADS * CC_PER) + threadIdx.x;
    float v[CC_PER];
#pragma unroll
    for (int q = 0; q < CC_PER; ++q) {
        const int64_t t = t0 + q * CC_THREADS;
        v[q] = t < n ? src[t] : 0.f;
    }
#pragma unroll
    for (int q = 0; q < CC_PER; ++q) {
        const int64_t t = t0 + q * CC_THREADS;
        if (t < Tmax) dst[t] = v[q];
    }
}

}  // namespace

extern "C" {

int encx_crop_collate(const float* pool, const int64_t* offsets, const int64_t* lengths,
                      const int64_t* src_channels, const int64_t* starts, const int64_t* out_len,
                      float* out, int64_t B, int64_t C, int64_t Tmax, encx_stream_t stream) {
    ENCX_REQUIRE(B >= 0 && C >= 1 && C <= 64 && Tmax >= 0);
    const int64_t total = B * C * Tmax;
    if (total == 0) return 0;
    ENCX_REQUIRE(pool && offsets && lengths && src_channels && starts && out_len && out);
    ENCX_REQUIRE(B * C <= 65535);
    hipLaunchKernelGGL(crop_collate_kernel, dim3((unsigned)cdiv(Tmax, CC_THREADS * CC_PER), (unsigned)(B * C)),
                       dim3(CC_THREADS), 0, (hipStream_t)stream, pool, offsets, lengths, src_channels, starts,
                       out_len, out, (int)C, Tmax);
    ENCX_CHECK_LAUNCH();
    return 0;
}

}  // extern "C"
