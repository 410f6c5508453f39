// encx -- `.ecdc` payload bit packing (binary.py:55-123) for whole encoded frames.
//
// The reference pushes the codes of a frame one at a time, t-major then codebook
// (compress.py:88-98): value v = t*K + k occupies bits [v*bits, (v+1)*bits) of a little-endian
// bit stream (BitPacker.push adds value << current_bits, binary.py:69-78), and flush() emits the
// final partial byte (binary.py:80-88), so a frame of n values is exactly ceil(n*bits/8) bytes.
// BitUnpacker.pull (binary.py:105-123) is the inverse. Both are pure byte/integer work and
// HBM-bound: no LDS, no MFMA. Each output byte (pack) or code (unpack) is one lane; adjacent
// lanes touch adjacent codes and bytes, so every wave's loads and stores are contiguous.
// Several frames of equal (K, T) are handled by one launch at a fixed byte stride per frame.
#include "common.h"

namespace {

// One lane per output byte j of frame b: the byte covers stream bits [8j, 8j+8), i.e. codes
// v0 = 8j/bits .. v1 = (8j+7)/bits (at most 8 of them for bits = 1, 2 for bits >= 8).
__global__ void bitpack_kernel(const int64_t* __restrict__ codes, int64_t s_item, int64_t s_k,
                               int64_t s_t, int K, int64_t n, int bits, uint8_t* __restrict__ out,
                               int64_t nbytes, int64_t out_stride, int64_t total,
                               int* __restrict__ err) {
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= total) return;
    const int64_t b = j / nbytes;
    const int64_t jb = j - b * nbytes;
    const int64_t bit0 = jb * 8;
    const int64_t v0 = bit0 / bits;
    int64_t v1 = (bit0 + 7) / bits;
    if (v1 > n - 1) v1 = n - 1;
    const int64_t* src = codes + b * s_item;
    uint64_t acc = 0;
    int bad = 0;
    for (int64_t v = v0; v <= v1; ++v) {
        const int64_t t = v / K;
        const int64_t k = v - t * K;
        const uint64_t val = (uint64_t)src[k * s_k + t * s_t];
        // the reference adds without masking; a code >= 2^bits would corrupt its neighbours
        bad |= (val >> bits) != 0;
        const int64_t sh = v * bits - bit0;
        acc |= sh >= 0 ? (val << sh) : (val >> (-sh));
    }
    out[b * out_stride + jb] = (uint8_t)(acc & 0xff);
    if (bad) atomicOr(err, 1);
}

// One lane per code v of frame b: gather the <= 5 bytes spanning bits [v*bits, (v+1)*bits).
__global__ void bitunpack_kernel(const uint8_t* __restrict__ in, int64_t in_stride, int K, int64_t n,
                                 int bits, int64_t* __restrict__ codes, int64_t s_item, int64_t s_k,
                                 int64_t s_t, int64_t total) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= total) return;
    const int64_t b = i / n;
    const int64_t v = i - b * n;
    const int64_t bit0 = v * bits;
    const uint8_t* src = in + b * in_stride + (bit0 >> 3);
    const int sh = (int)(bit0 & 7);
    const int nb = (sh + bits + 7) >> 3;
    uint64_t acc = 0;
    for (int q = 0; q < nb; ++q) acc |= (uint64_t)src[q] << (8 * q);
    const uint64_t mask = (bits == 64) ? ~0ull : ((1ull << bits) - 1);
    const int64_t t = v / K;
    const int64_t k = v - t * K;
    codes[b * s_item + k * s_k + t * s_t] = (int64_t)((acc >> sh) & mask);
}

}  // namespace

extern "C" {

int64_t encx_bitpack_bytes(int64_t n_values, int bits) {
    if (n_values < 0 || bits < 1 || bits > 32) return -1;
    return (n_values * bits + 7) / 8;
}

int encx_bitpack(const int64_t* codes, int64_t s_item, int64_t s_k, int64_t s_t, int64_t items,
                 int64_t K, int64_t T, int bits, uint8_t* out, int64_t out_stride, int* err,
                 encx_stream_t stream) {
    ENCX_REQUIRE(bits >= 1 && bits <= 32 && items >= 0 && K >= 0 && T >= 0);
    const int64_t n = K * T;
    const int64_t nbytes = encx_bitpack_bytes(n, bits);
    ENCX_REQUIRE(out_stride >= nbytes);
    const int64_t total = items * nbytes;
    if (total == 0) return 0;  // BitPacker.flush with nothing pushed writes nothing
    ENCX_REQUIRE(codes && out && err && K <= INT32_MAX);
    hipLaunchKernelGGL(bitpack_kernel, dim3((unsigned)cdiv(total, 256)), dim3(256), 0,
                       (hipStream_t)stream, codes, s_item, s_k, s_t, (int)K, n, bits, out, nbytes,
                       out_stride, total, err);
    ENCX_CHECK_LAUNCH();
    return 0;
}

int encx_bitunpack(const uint8_t* in, int64_t in_stride, int64_t items, int64_t K, int64_t T,
                   int bits, int64_t* codes, int64_t s_item, int64_t s_k, int64_t s_t,
                   encx_stream_t stream) {
    ENCX_REQUIRE(bits >= 1 && bits <= 32 && items >= 0 && K >= 0 && T >= 0);
    const int64_t n = K * T;
    ENCX_REQUIRE(in_stride >= encx_bitpack_bytes(n, bits));
    const int64_t total = items * n;
    if (total == 0) return 0;
    ENCX_REQUIRE(in && codes && K <= INT32_MAX);
    hipLaunchKernelGGL(bitunpack_kernel, dim3((unsigned)cdiv(total, 256)), dim3(256), 0,
                       (hipStream_t)stream, in, in_stride, (int)K, n, bits, codes, s_item, s_k, s_t,
                       total);
    ENCX_CHECK_LAUNCH();
    return 0;
}

}  // extern "C"
