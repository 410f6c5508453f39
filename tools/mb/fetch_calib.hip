// FETCH_SIZE / WRITE_SIZE calibration on gfx950: kernels that read (or write) a known number of
// HBM bytes once, each with one access width, so `rocprofv3 --pmc FETCH_SIZE` (KiB) divided by
// the bytes moved gives the counter's factor per width:
//   rd_x4      aligned 16-B loads (global_load_dwordx4)
//   rd_x4u     16-B loads at 4-byte-aligned, not 16-B-aligned addresses (the ld4u windows)
//   rd_x2      8-B loads
//   rd_x1      4-B loads
//   wr_x4 / wr_x1   the same for stores (WRITE_SIZE)
// Each kernel touches N floats once (grid-stride, coalesced), from a buffer far larger than the
// caches (512 MiB), flushed between kernels by a 1 GiB streaming write. Prints the bytes per kernel.
// Build: hipcc -O3 --offload-arch=gfx950 fetch_calib.hip -o fetch_calib
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x4u __attribute__((ext_vector_type(4), aligned(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

// the sums go to one float per thread (negligible, counted) so the loads are not dead
__global__ void rd_x4(const float* x, float* out, long n4) {
    f32x4 s = {0, 0, 0, 0};
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x)
        s += ((const f32x4*)x)[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s[0] + s[1] + s[2] + s[3];
}
__global__ void rd_x4u(const float* x, float* out, long n4) {  // x + 1: every quad straddles
    f32x4 s = {0, 0, 0, 0};
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x)
        s += *(const f32x4u*)(x + 1 + 4 * i);
    out[blockIdx.x * blockDim.x + threadIdx.x] = s[0] + s[1] + s[2] + s[3];
}
__global__ void rd_x2(const float* x, float* out, long n2) {
    f32x2 s = {0, 0};
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n2; i += (long)gridDim.x * blockDim.x)
        s += ((const f32x2*)x)[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s[0] + s[1];
}
__global__ void rd_x1(const float* x, float* out, long n) {
    float s = 0.f;
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) s += x[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void wr_x4(float* y, long n4) {
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x)
        ((f32x4*)y)[i] = (f32x4){1.f, 2.f, 3.f, (float)i};
}
__global__ void wr_x1(float* y, long n) {
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) y[i] = (float)i;
}
__global__ void flush(float* y, long n4) {  // streams 1 GiB through the caches
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x)
        ((f32x4*)y)[i] = (f32x4){0.f, 0.f, 0.f, 0.f};
}

int main() {
    const long N = 128l << 20;  // floats: 512 MiB
    const int G = 4096, T = 256;
    float *x, *y, *fl, *out;
    CK(hipMalloc(&x, (N + 64) * sizeof(float)));
    CK(hipMalloc(&y, N * sizeof(float)));
    CK(hipMalloc(&fl, (256l << 20) * sizeof(float)));
    CK(hipMalloc(&out, (long)G * T * sizeof(float)));
    CK(hipMemset(x, 0, (N + 64) * sizeof(float)));
    auto fl_ = [&] { hipLaunchKernelGGL(flush, dim3(G), dim3(T), 0, 0, fl, (256l << 20) / 4); };
    const double MiB = 1 << 20;
    for (int rep = 0; rep < 2; ++rep) {
        fl_(); hipLaunchKernelGGL(rd_x4, dim3(G), dim3(T), 0, 0, x, out, N / 4);
        fl_(); hipLaunchKernelGGL(rd_x4u, dim3(G), dim3(T), 0, 0, x, out, N / 4);
        fl_(); hipLaunchKernelGGL(rd_x2, dim3(G), dim3(T), 0, 0, x, out, N / 2);
        fl_(); hipLaunchKernelGGL(rd_x1, dim3(G), dim3(T), 0, 0, x, out, N);
        fl_(); hipLaunchKernelGGL(wr_x4, dim3(G), dim3(T), 0, 0, y, N / 4);
        fl_(); hipLaunchKernelGGL(wr_x1, dim3(G), dim3(T), 0, 0, y, N);
    }
    CK(hipDeviceSynchronize());
    printf("bytes per kernel: read %.1f MiB (+ %.1f MiB of sums written), write %.1f MiB\n", N * 4 / MiB,
           (double)G * T * 4 / MiB, N * 4 / MiB);
    return 0;
}
