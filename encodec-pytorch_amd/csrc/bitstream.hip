// encx -- `.ecdc` payload bit packing (binary.py:55-123) for whole encoded frames.
//
// The reference pushes the codes of a frame one at a time, t-major then codebook
// (compress.py:88-98): value v = t*K + k occupies bits [v*bits, (v+1)*bits) of a little-endian
// bit stream (BitPacker.push adds value << current_bits, binary.py:69-78), and flush() emits the
// final partial byte (binary.py:80-88), so a frame of n values is exactly ceil(n*bits/8) bytes.
// BitUnpacker.pull (binary.py:105-123) is the inverse. Both are pure byte/integer work and
// HBM-bound: no LDS, no MFMA.
// Several frames of equal (K, T) are handled by one launch at a fixed byte stride per frame.
#include "common.h"

namespace {

// Eight consecutive codes are exactly `bits` whole bytes of the stream, so lane g owns codes
// 8g..8g+7 and bytes [g*bits, (g+1)*bits): no byte is shared between lanes, and (v -> t, k) is
// one division per lane, then a carried increment. The tail lane (n % 8 codes) emits the
// flush's partial byte. Reads: each of the K codebook rows is walked contiguously across the
// wave (t advances with the lane); writes: the wave covers 64*bits contiguous bytes.
__global__ void bitpack_kernel(const int64_t* __restrict__ codes, int64_t s_item, int64_t s_k,
                               int64_t s_t, int K, int64_t n, int bits, uint8_t* __restrict__ out,
                               int64_t groups, int64_t out_stride, int64_t total,
                               int* __restrict__ err) {
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= total) return;
    const int64_t b = j / groups;
    const int64_t g = j - b * groups;
    const int64_t v0 = g * 8;
    const int cnt = (int)((n - v0) < 8 ? (n - v0) : 8);
    int64_t t = v0 / K;
    int k = (int)(v0 - t * K);
    const int64_t* src = codes + b * s_item;
    uint8_t* dst = out + b * out_stride + g * bits;
    uint64_t acc = 0;
    int nb = 0;
    uint64_t bad = 0;
    for (int i = 0; i < cnt; ++i) {
        const uint64_t val = (uint64_t)src[k * s_k + t * s_t];
        // the reference adds without masking; a code >= 2^bits would corrupt its neighbours
        bad |= val >> bits;
        acc |= val << nb;
        nb += bits;
        while (nb >= 8) {
            *dst++ = (uint8_t)(acc & 0xff);
            acc >>= 8;
            nb -= 8;
        }
        if (++k == K) { k = 0; ++t; }
    }
    if (nb) *dst = (uint8_t)(acc & 0xff);  // flush (binary.py:80-85); only the tail lane
    if (bad) atomicOr(err, 1);
}

// The inverse: lane g reads its `bits` bytes (fewer on the tail) and emits codes 8g..8g+7.
__global__ void bitunpack_kernel(const uint8_t* __restrict__ in, int64_t in_stride, int K, int64_t n,
                                 int bits, int64_t* __restrict__ codes, int64_t s_item, int64_t s_k,
                                 int64_t s_t, int64_t groups, int64_t total) {
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= total) return;
    const int64_t b = j / groups;
    const int64_t g = j - b * groups;
    const int64_t v0 = g * 8;
    const int cnt = (int)((n - v0) < 8 ? (n - v0) : 8);
    int64_t t = v0 / K;
    int k = (int)(v0 - t * K);
    const uint8_t* src = in + b * in_stride + g * bits;
    int64_t* dst = codes + b * s_item;
    const uint64_t mask = (1ull << bits) - 1;
    uint64_t acc = 0;
    int nb = 0;
    for (int i = 0; i < cnt; ++i) {
        while (nb < bits) {
            acc |= (uint64_t)(*src++) << nb;
            nb += 8;
        }
        dst[k * s_k + t * s_t] = (int64_t)(acc & mask);
        acc >>= bits;
        nb -= bits;
        if (++k == K) { k = 0; ++t; }
    }
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
    const int64_t groups = cdiv(n, 8);
    const int64_t total = items * groups;
    if (total == 0) return 0;  // BitPacker.flush with nothing pushed writes nothing
    ENCX_REQUIRE(codes && out && err && K <= INT32_MAX);
    hipLaunchKernelGGL(bitpack_kernel, dim3((unsigned)cdiv(total, 256)), dim3(256), 0,
                       (hipStream_t)stream, codes, s_item, s_k, s_t, (int)K, n, bits, out, groups,
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
    const int64_t groups = cdiv(n, 8);
    const int64_t total = items * groups;
    if (total == 0) return 0;
    ENCX_REQUIRE(in && codes && K <= INT32_MAX);
    hipLaunchKernelGGL(bitunpack_kernel, dim3((unsigned)cdiv(total, 256)), dim3(256), 0,
                       (hipStream_t)stream, in, in_stride, (int)K, n, bits, codes, s_item, s_k, s_t,
                       groups, total);
    ENCX_CHECK_LAUNCH();
    return 0;
}

}  // extern "C"
