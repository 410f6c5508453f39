// encx -- the LM entropy coder's arithmetic coder (quantization/ac.py) on the GPU.
//
// * softmax_cdf_kernel: build_stable_quantized_cdf (ac.py:18-53), optionally fused with the
//   softmax over the codebook that produces its pdf (model.py:64). One 256-thread workgroup per
//   row; the float32 steps are the reference's own (pdf / roundoff, floor, * roundoff, then
//   floor(float32((1 - alpha) 2^bits) * pdf) + min_range) with correctly rounded division and
//   no contraction, and the cumulative sum is an exact integer block scan. For an encoder row
//   the thread that produces cdf[sym - 1] / cdf[sym] also writes the symbol's coding interval
//   (lo, hi), so the serial coder reads two integers per symbol instead of a whole cdf.
// * ac_encode_kernel: ArithmeticCoder.push / flush (ac.py:130-167), one thread per stream.
//   The reference's float64 `ceil(range_low * (delta / 2^bits))` is exact (range_low < 2^bits,
//   delta < 2^(bits+1)), so it is computed as the integer ceil / floor of range_low * delta /
//   2^bits. The doubling loop (ac.py:139-142) is one shift by bits - floor(log2 delta); the
//   common-prefix flush (ac.py:111-128) emits the bits above the highest bit where low and high
//   differ in one go. Bits go out LSB-first within bytes, as BitPacker(bits=1) writes them.
// * ac_decode_kernel: ArithmeticDecoder.pull (ac.py:217-260), one wave per stream, K symbols
//   (one cdf row each) per launch. The state is uniform across the wave; the 64 lanes test the
//   codebook entries in parallel for the one interval containing `current`. The intervals are
//   disjoint and ordered, so this finds exactly the symbol the reference's binary search finds,
//   and finds none exactly when that search fails (ac.py:238).
#include "common.h"

// No mul+add contraction anywhere in this file: the same quantity computed by two kernels (e.g.
// a score scaled, stored, then offset by the max, against the same expression inline) must round
// identically, and __fmul_rn alone does not stop clang fusing it into a following add.
#pragma clang fp contract(off)

namespace {

constexpr int CDF_THREADS = 256;

ENCX_DEV uint64_t lowmask(int n) { return n <= 0 ? 0ull : (n >= 64 ? ~0ull : ((1ull << n) - 1ull)); }

// inclusive scan of one int per thread over the 256-thread block; *total = block sum
ENCX_DEV int block_scan_incl(int v, int* red, int* total) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int u = __shfl_up(v, o, 64);
        if (lane >= o) v += u;
    }
    __syncthreads();
    if (lane == 63) red[w] = v;
    __syncthreads();
    int pre = 0;
    for (int i = 0; i < w; ++i) pre += red[i];
    *total = red[0] + red[1] + red[2] + red[3];
    return v + pre;
}

ENCX_DEV float block_max(float v, float* red) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    __syncthreads();
    if (lane == 0) red[w] = v;
    __syncthreads();
    return fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
}

// One row per workgroup: row r = n*K + k of a [N][K][card] problem (n = b*T + t).
template <bool LOGITS>
__global__ __launch_bounds__(CDF_THREADS) void softmax_cdf_kernel(
    const float* __restrict__ in, int64_t ld_in, int card, float* __restrict__ probas,
    int32_t* __restrict__ cdf, float roundoff, float qscale, int min_range, int64_t total_range,
    const int64_t* __restrict__ sym, int64_t s_b, int64_t s_k, int64_t s_t, int K, int T,
    int32_t* __restrict__ lohi, int* __restrict__ err) {
    __shared__ float redf[4];
    __shared__ int redi[4];
    const int64_t row = blockIdx.x;
    const int tid = threadIdx.x;
    const float* x = in + row * ld_in;
    float mx = 0.f, sum = 1.f;
    if (LOGITS) {
        float m = -INFINITY;
        for (int i = tid; i < card; i += CDF_THREADS) m = fmaxf(m, x[i]);
        mx = block_max(m, redf);
        float s = 0.f;
        for (int i = tid; i < card; i += CDF_THREADS) s += expf(x[i] - mx);
        sum = block_sum(s, redf);
    }
    int64_t symv = -1;
    if (sym) {
        const int64_t n = row / K;
        const int k = (int)(row - n * K);
        const int64_t b = n / T, t = n - b * T;
        symv = sym[b * s_b + k * s_k + t * s_t];
        if (tid == 0 && err && (symv < 0 || symv >= card)) atomicOr(err, 2);
        if (tid == 0 && symv == 0) lohi[row * 2] = 0;
    }
    int carry = 0;
    for (int c0 = 0; c0 < card; c0 += CDF_THREADS) {
        const int i = c0 + tid;
        int r = 0;
        if (i < card) {
            float p = LOGITS ? expf(x[i] - mx) / sum : x[i];
            if (probas) probas[row * card + i] = p;
            float q = p;
            if (roundoff > 0.f) q = __fmul_rn(floorf(__fdiv_rn(p, roundoff)), roundoff);  // ac.py:37-38
            r = (int)floorf(__fmul_rn(qscale, q)) + min_range;                              // ac.py:44-45
        }
        int tot;
        const int incl = block_scan_incl(r, redi, &tot) + carry;                             // ac.py:46
        if (i < card) {
            if (cdf) cdf[row * card + i] = incl;
            if (i == symv - 1) lohi[row * 2] = incl;
            if (i == symv) lohi[row * 2 + 1] = incl - 1;
        }
        carry += tot;
        __syncthreads();
    }
    // a total above 2^bits: check=True would reject it (ac.py:50) and the coder asserts (:116)
    if (tid == 0 && err && (int64_t)carry > total_range) atomicOr(err, 1);
}

struct BitOut {
    uint8_t* o;
    int64_t cap, pos;
    uint64_t acc;
    int nb;
    // append n bits, first bit in bit 0 of `rev`
    ENCX_DEV void put(uint64_t rev, int n) {
        while (n > 0) {
            const int k = n > 32 ? 32 : n;
            acc |= (rev & lowmask(k)) << nb;
            nb += k;
            rev >>= k;
            n -= k;
            while (nb >= 8) {
                if (pos < cap) o[pos] = (uint8_t)(acc & 0xff);
                ++pos;
                acc >>= 8;
                nb -= 8;
            }
        }
    }
    // append the n low bits of v most-significant first (the order _flush_common_prefix pushes)
    ENCX_DEV void put_msb_first(uint64_t v, int n) {
        if (n > 0) put(__builtin_bitreverse64(v) >> (64 - n), n);
    }
};

// The reference's coder state is Python ints (ac.py:56-260): within a push, low / high grow by
// up to total_range_bits (<= 30) bits past max_bit (<= 61 after every flush, ac.py:157), so
// they are held in 128 bits here (never more than 93 used); every interval width (delta, at
// most 2^(bits+1)) and every product of a cdf value with it fits in 64.
typedef unsigned __int128 u128;
ENCX_DEV u128 lowmask128(int n) { return n <= 0 ? (u128)0 : (n >= 128 ? ~(u128)0 : (((u128)1 << n) - 1)); }
ENCX_DEV int hibit128(u128 x) {  // index of the highest set bit, -1 for 0
    const uint64_t h = (uint64_t)(x >> 64), l = (uint64_t)x;
    return h ? 127 - __builtin_clzll(h) : (l ? 63 - __builtin_clzll(l) : -1);
}

__global__ void ac_encode_kernel(const int32_t* __restrict__ lohi, int64_t n, int S, int bits,
                                 uint8_t* __restrict__ out, int64_t cap, int64_t* __restrict__ nbytes,
                                 int* __restrict__ err) {
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= S) return;
    const int32_t* lh = lohi + (int64_t)s * n * 2;
    BitOut bo{out + (int64_t)s * cap, cap, 0, 0ull, 0};
    const uint64_t R = 1ull << bits;
    u128 low = 0, high = 0;
    int max_bit = -1, e = 0;
    // the intervals do not depend on the coder state: fetch them 8 symbols at a time (one
    // memory round trip per 8 pushes instead of one per push)
    for (int64_t i0 = 0; i0 < n && !e; i0 += 8) {
        uint32_t iv[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) {
            const int64_t q = 2 * i0 + u;
            iv[u] = (uint32_t)lh[q < 2 * n ? q : 2 * n - 1];
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            if (i0 + u >= n || e) break;
            const uint64_t rl = iv[2 * u], rh = iv[2 * u + 1];
            uint64_t delta = (uint64_t)(high - low) + 1;  // < 2^62 (both < 2^(max_bit+1))
            if (delta < R) {  // ac.py:139-142
                const int sh = bits - (63 - __builtin_clzll(delta));
                low <<= sh;
                high = (high << sh) | lowmask128(sh);
                max_bit += sh;
                delta = (uint64_t)(high - low) + 1;
            }
            const uint64_t el = (rl * delta + R - 1) >> bits, eh = (rh * delta) >> bits;  // ac.py:146-147
            high = low + eh;
            low = low + el;
            if (high >> (max_bit + 1)) { e = 1; break; }  // ac.py:116
            const int hb = hibit128(low ^ high);           // ac.py:111-128
            const int nf = max_bit - hb;
            if (nf > 0) {
                const u128 pre = low >> (hb + 1);  // the nf-bit common prefix, pushed msb first
                if (nf > 64) bo.put_msb_first((uint64_t)(pre >> 64), nf - 64);
                bo.put_msb_first((uint64_t)pre, nf > 64 ? 64 : nf);
                low &= lowmask128(hb + 1);
                high &= lowmask128(hb + 1);
                max_bit = hb;
            }
            if (max_bit > 61) { e = 3; break; }  // ac.py:157
        }
    }
    if (!e) {
        bo.put_msb_first((uint64_t)low, max_bit + 1);  // flush (ac.py:160-167); max_bit <= 61
        if (bo.nb) {
            if (bo.pos < cap) bo.o[bo.pos] = (uint8_t)(bo.acc & 0xff);
            ++bo.pos;
        }
        if (bo.pos > cap) e = 2;
    }
    nbytes[s] = bo.pos;
    err[s] = e;
}

// decoder state per stream (ENCX_AC_STATE int64 words): low, high, current (128 bits each,
// low word first), max_bit, bits consumed
__global__ __launch_bounds__(64) void ac_decode_kernel(
    const uint8_t* __restrict__ data, int64_t stride, const int64_t* __restrict__ nbytes,
    int64_t* __restrict__ state, const int32_t* __restrict__ cdf, int K, int card, int bits,
    int64_t* __restrict__ codes, int64_t c_s, int64_t c_k, int64_t c_t, int64_t t,
    const int64_t* __restrict__ dstep, int64_t* __restrict__ next_idx, int* __restrict__ err) {
    const int s = blockIdx.x, lane = threadIdx.x;
    if (err[s]) return;  // the stream already failed; later steps leave it as it is
    if (dstep) t += *dstep;
    int64_t* stt = state + (int64_t)s * ENCX_AC_STATE;
    auto ld128 = [&](int i) { return ((u128)(uint64_t)stt[2 * i + 1] << 64) | (u128)(uint64_t)stt[2 * i]; };
    u128 low = ld128(0), high = ld128(1), cur = ld128(2);
    int max_bit = (int)stt[6];
    int64_t pos = stt[7];
    const int64_t nbits = nbytes[s] * 8;
    const uint8_t* src = data + (int64_t)s * stride;
    const uint64_t R = 1ull << bits;
    int e = 0;
    for (int k = 0; k < K; ++k) {
        // the reference decoder has no bound on max_bit (ac.py:217-260); a stream its encoder
        // wrote keeps it <= 61 after every pull, so past 96 the stream is not one it could write
        if (max_bit > 96) { e = 3; break; }
        uint64_t delta = (uint64_t)(high - low) + 1;
        if (delta < R) {  // ac.py:226-233
            const int sh = bits - (63 - __builtin_clzll(delta));
            if (pos + sh > nbits) { e = 1; break; }  // BitUnpacker ran dry: pull returns None
            // the sh (<= 31) stream bits from `pos` span at most 5 bytes: load them together
            const int64_t b0 = pos >> 3, last = (nbits >> 3) - 1;
            uint64_t win = 0;
#pragma unroll
            for (int u = 0; u < 5; ++u) {
                const int64_t bi = b0 + u <= last ? b0 + u : last;
                win |= (uint64_t)src[bi] << (8 * u);
            }
            const uint64_t chunk = (win >> (pos & 7)) & lowmask(sh);   // stream bit pos at bit 0
            cur = (cur << sh) | (u128)(__builtin_bitreverse64(chunk) >> (64 - sh));
            pos += sh;
            low <<= sh;
            high = (high << sh) | lowmask128(sh);
            max_bit += sh;
            delta = (uint64_t)(high - low) + 1;
        }
        const int32_t* row = cdf + ((int64_t)s * K + k) * card;
        const uint64_t off = (uint64_t)(cur - low);  // < delta when the stream is consistent
        int found = -1;
        for (int j0 = 0; j0 < card; j0 += 64 * 16) {   // 16 entries per lane in flight together
            int32_t cl[16], ch[16];
#pragma unroll
            for (int u = 0; u < 16; ++u) {
                const int j = j0 + lane + 64 * u;
                const int jc = j < card ? j : card - 1;
                ch[u] = row[jc];
                cl[u] = jc > 0 ? row[jc - 1] : 0;
            }
#pragma unroll
            for (int u = 0; u < 16; ++u) {
                const int j = j0 + lane + 64 * u;
                // an empty or negative interval (ch - 1 < cl, e.g. the zero cdf ac.py:288 pulls
                // with) has effective_high < effective_low and can never hold `current`
                if (j >= card || cl[u] < 0 || ch[u] - 1 < cl[u]) continue;
                const uint64_t rl = (uint64_t)cl[u], rh = (uint64_t)(ch[u] - 1);
                const uint64_t el = (rl * delta + R - 1) >> bits, eh = (rh * delta) >> bits;
                if (off >= el && off <= eh) found = j;
            }
        }
        const uint64_t hit = __ballot(found >= 0);
        if (!hit) { e = 2; break; }  // ac.py:238 "Binary search failed"
        const int sym = __shfl(found, __ffsll((long long)hit) - 1, 64);
        const uint64_t rl = sym ? (uint64_t)(uint32_t)row[sym - 1] : 0ull;
        const uint64_t rh = (uint64_t)(uint32_t)row[sym] - 1;
        const uint64_t el = (rl * delta + R - 1) >> bits, eh = (rh * delta) >> bits;
        high = low + eh;
        low = low + el;
        const int hb = hibit128(low ^ high);  // ac.py:201-215
        if (max_bit > hb) {
            low &= lowmask128(hb + 1);
            high &= lowmask128(hb + 1);
            cur &= lowmask128(hb + 1);
            max_bit = hb;
        }
        if (lane == 0) {
            if (codes) codes[s * c_s + k * c_k + t * c_t] = sym;
            if (next_idx) next_idx[(int64_t)s * K + k] = sym + 1;
        }
    }
    if (lane == 0) {
        const u128 w[3] = {low, high, cur};
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            stt[2 * i] = (int64_t)(uint64_t)w[i];
            stt[2 * i + 1] = (int64_t)(uint64_t)(w[i] >> 64);
        }
        stt[6] = max_bit;
        stt[7] = pos;
        err[s] = e;
    }
}

__global__ void ac_lohi_kernel(const int32_t* __restrict__ cdf, int64_t ld, const int64_t* __restrict__ sym,
                               int64_t rows, int card, int32_t* __restrict__ lohi, int* __restrict__ err) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= rows) return;
    const int64_t s = sym[r];
    if (s < 0 || s >= card) {
        atomicOr(err, 2);
        lohi[2 * r] = 0;
        lohi[2 * r + 1] = 0;
        return;
    }
    const int32_t* c = cdf + r * ld;
    lohi[2 * r] = s ? c[s - 1] : 0;
    lohi[2 * r + 1] = c[s] - 1;
}

}  // namespace

// shared with lm.hip (encx_lm_heads)
int encx_lm_softmax_cdf_launch(const float* in, int64_t rows, int card, int64_t ld_in, int from_logits,
                               float* probas, int32_t* cdf, int total_range_bits, float roundoff,
                               int min_range, const int64_t* sym, int64_t s_b, int64_t s_k, int64_t s_t,
                               int K, int T, int32_t* lohi, int* err, hipStream_t st) {
    ENCX_REQUIRE(total_range_bits >= 1 && total_range_bits <= 30 && min_range >= 2 && card >= 1);
    const double total = (double)(1ll << total_range_bits);
    const double alpha = (double)min_range * card / total;  // ac.py:42-43
    ENCX_REQUIRE(alpha <= 1.0);
    const float qscale = (float)((1.0 - alpha) * total);
    if (rows == 0) return 0;
    ENCX_REQUIRE(in && rows <= INT32_MAX && (!sym || (lohi && T >= 1 && K >= 1)));
    if (from_logits)
        hipLaunchKernelGGL(softmax_cdf_kernel<true>, dim3((unsigned)rows), dim3(CDF_THREADS), 0, st, in, ld_in,
                           card, probas, cdf, roundoff, qscale, min_range, (int64_t)1 << total_range_bits,
                           sym, s_b, s_k, s_t, K, T, lohi, err);
    else
        hipLaunchKernelGGL(softmax_cdf_kernel<false>, dim3((unsigned)rows), dim3(CDF_THREADS), 0, st, in, ld_in,
                           card, probas, cdf, roundoff, qscale, min_range, (int64_t)1 << total_range_bits,
                           sym, s_b, s_k, s_t, K, T, lohi, err);
    ENCX_CHECK_LAUNCH();
    return 0;
}

extern "C" {

int encx_ac_cdf(const float* pdf, int64_t rows, int64_t card, int64_t ld, int total_range_bits, float roundoff,
                int min_range, int32_t* cdf, int* err, encx_stream_t stream) {
    ENCX_REQUIRE(rows >= 0 && card >= 1 && card <= INT32_MAX && ld >= card && cdf);
    return encx_lm_softmax_cdf_launch(pdf, rows, (int)card, ld, 0, nullptr, cdf, total_range_bits, roundoff,
                                      min_range, nullptr, 0, 0, 0, 1, 1, nullptr, err, (hipStream_t)stream);
}

int encx_ac_lohi(const int32_t* cdf, int64_t ld, const int64_t* sym, int64_t rows, int64_t card, int32_t* lohi,
                 int* err, encx_stream_t stream) {
    ENCX_REQUIRE(rows >= 0 && card >= 1 && card <= INT32_MAX && ld >= card);
    if (rows == 0) return 0;
    ENCX_REQUIRE(cdf && sym && lohi && err);
    hipLaunchKernelGGL(ac_lohi_kernel, dim3((unsigned)cdiv(rows, 256)), dim3(256), 0, (hipStream_t)stream, cdf, ld,
                       sym, rows, (int)card, lohi, err);
    ENCX_CHECK_LAUNCH();
    return 0;
}

int64_t encx_ac_encode_capacity(int64_t n_symbols, int total_range_bits) {
    // each push emits at most bits + 1 bits beyond the <= 62 held back, plus the final flush
    if (n_symbols < 0 || total_range_bits < 1 || total_range_bits > 30) return -1;
    return (n_symbols * (total_range_bits + 1) + 64 + 7) / 8;
}

int encx_ac_encode(const int32_t* lohi, int64_t streams, int64_t n, int total_range_bits, uint8_t* out,
                   int64_t cap, int64_t* nbytes, int* err, encx_stream_t stream) {
    ENCX_REQUIRE(streams >= 0 && n >= 0 && total_range_bits >= 1 && total_range_bits <= 30 && cap >= 0);
    if (streams == 0) return 0;
    ENCX_REQUIRE((lohi || n == 0) && out && nbytes && err && streams <= INT32_MAX);
    hipLaunchKernelGGL(ac_encode_kernel, dim3((unsigned)cdiv(streams, 64)), dim3(64), 0, (hipStream_t)stream,
                       lohi, n, (int)streams, total_range_bits, out, cap, nbytes, err);
    ENCX_CHECK_LAUNCH();
    return 0;
}

int encx_ac_decode(const uint8_t* data, int64_t stride, const int64_t* nbytes, int64_t streams, int64_t* state,
                   const int32_t* cdf, int64_t K, int64_t card, int total_range_bits, int64_t* codes, int64_t c_s,
                   int64_t c_k, int64_t c_t, int64_t t, const int64_t* dev_step, int64_t* next_idx, int* err,
                   encx_stream_t stream) {
    ENCX_REQUIRE(streams >= 0 && K >= 1 && card >= 1 && card <= INT32_MAX && total_range_bits >= 1 &&
                 total_range_bits <= 30);
    if (streams == 0) return 0;
    ENCX_REQUIRE(data && nbytes && state && cdf && err && streams <= INT32_MAX && K <= INT32_MAX);
    hipLaunchKernelGGL(ac_decode_kernel, dim3((unsigned)streams), dim3(64), 0, (hipStream_t)stream, data, stride,
                       nbytes, state, cdf, (int)K, (int)card, total_range_bits, codes, c_s, c_k, c_t, t, dev_step,
                       next_idx, err);
    ENCX_CHECK_LAUNCH();
    return 0;
}

}  // extern "C"
