// Microbenchmark: cost of a device-wide barrier between the steps of a persistent kernel (the
// question behind a weights-stationary LSTM). NB workgroups (one per CU) run S
// steps; each step every workgroup writes a row of 512 floats, crosses the barrier (release
// fence + atomic arrive, bounded spin on the counter + acquire fence), then reads the row another
// workgroup (on another XCD) wrote and checks it. Reports us per step, against a baseline of S
// separate launches of the same write/read work. A spin that exceeds its bound sets a flag and
// exits, so a missing workgroup can never hang the device.
//
// hipcc --offload-arch=gfx950 -O3 grid_barrier.hip -o grid_barrier && ./grid_barrier
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

constexpr int ROW = 512;

__device__ void grid_barrier(unsigned* count, unsigned target, int* fail) {
    __syncthreads();
    if (threadIdx.x == 0) {
        __threadfence();                 // release this workgroup's writes (agent scope)
        atomicAdd(count, 1u);
        long spins = 0;
        while (__hip_atomic_load(count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
            if (++spins > (1l << 24)) { atomicOr(fail, 1); break; }
            __builtin_amdgcn_s_sleep(1);
        }
        __threadfence();                 // acquire the others' writes
    }
    __syncthreads();
}

// two-level: the 8 XCDs' workgroups (dispatched round-robin, blockIdx % 8) arrive on their own
// counter; the last arriver of each XCD arrives on the top counter, which everyone polls
__device__ void grid_barrier2(unsigned* count, unsigned step, int* fail) {
    __syncthreads();
    if (threadIdx.x == 0) {
        const int nb = gridDim.x, x = blockIdx.x & 7;
        const unsigned per = (unsigned)((nb - x + 7) >> 3);
        __threadfence();
        const unsigned old = atomicAdd(count + 64 * (1 + x), 1u);
        if (old == per * (step + 1) - 1) atomicAdd(count, 1u);
        long spins = 0;
        while (__hip_atomic_load(count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < 8u * (step + 1)) {
            if (++spins > (1l << 26)) { atomicOr(fail, 1); break; }
        }
        __threadfence();
    }
    __syncthreads();
}

template <int TWO>
__global__ __launch_bounds__(512) void persistent(float* buf, unsigned* count, int* fail, int* bad, int S) {
    const int nb = gridDim.x, b = blockIdx.x;
    for (int s = 0; s < S; ++s) {
        float* row = buf + ((size_t)(s & 1) * nb + b) * ROW;
        row[threadIdx.x] = (float)(s * 1000 + b) + threadIdx.x * 1e-3f;
        if (TWO) grid_barrier2(count, (unsigned)s, fail);
        else grid_barrier(count, (unsigned)(nb * (s + 1)), fail);
        const int o = (b + 37) % nb;     // a workgroup on another XCD
        const float v = buf[((size_t)(s & 1) * nb + o) * ROW + threadIdx.x];
        if (v != (float)(s * 1000 + o) + threadIdx.x * 1e-3f) atomicAdd(bad, 1);
    }
}

__global__ __launch_bounds__(512) void one_step_write(float* buf, int s) {
    const int nb = gridDim.x, b = blockIdx.x;
    buf[((size_t)(s & 1) * nb + b) * ROW + threadIdx.x] = (float)(s * 1000 + b) + threadIdx.x * 1e-3f;
}
__global__ __launch_bounds__(512) void one_step_read(float* buf, int s, int* bad) {
    const int nb = gridDim.x, b = blockIdx.x;
    const int o = (b + 37) % nb;
    const float v = buf[((size_t)(s & 1) * nb + o) * ROW + threadIdx.x];
    if (v != (float)(s * 1000 + o) + threadIdx.x * 1e-3f) atomicAdd(bad, 1);
}

int main(int argc, char** argv) {
    int dev = 0, ncu = 0;
    CK(hipGetDevice(&dev));
    CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
    const int S = 76;
    float* buf;
    unsigned* count;
    int *fail, *bad;
    CK(hipMalloc(&buf, sizeof(float) * 2 * 1024 * ROW));
    CK(hipMalloc(&count, 4 * 64 * 9));
    CK(hipMalloc(&fail, 4));
    CK(hipMalloc(&bad, 4));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int nb : {128, 256}) {
        if (nb > ncu) continue;
        int occ = 0;
        CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, persistent<0>, 512, 0));
        for (int rep = 0; rep < 6; ++rep) {
            const int two = rep >= 3;
            CK(hipMemset(count, 0, 4 * 64 * 9));
            CK(hipMemset(fail, 0, 4));
            CK(hipMemset(bad, 0, 4));
            CK(hipEventRecord(e0));
            if (two) hipLaunchKernelGGL(persistent<1>, dim3(nb), dim3(512), 0, 0, buf, count, fail, bad, S);
            else hipLaunchKernelGGL(persistent<0>, dim3(nb), dim3(512), 0, 0, buf, count, fail, bad, S);
            CK(hipGetLastError());
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            int f, bd;
            CK(hipMemcpy(&f, fail, 4, hipMemcpyDeviceToHost));
            CK(hipMemcpy(&bd, bad, 4, hipMemcpyDeviceToHost));
            printf("persistent %s nb=%d (cus %d, occ %d/CU): %.2f us/step  fail=%d bad=%d\n",
                   two ? "two-level" : "flat", nb, ncu, occ, 1e3 * ms / S, f, bd);
        }
        for (int rep = 0; rep < 2; ++rep) {
            CK(hipMemset(bad, 0, 4));
            CK(hipEventRecord(e0));
            for (int s = 0; s < S; ++s) {
                hipLaunchKernelGGL(one_step_write, dim3(nb), dim3(512), 0, 0, buf, s);
                hipLaunchKernelGGL(one_step_read, dim3(nb), dim3(512), 0, 0, buf, s, bad);
            }
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            int bd;
            CK(hipMemcpy(&bd, bad, 4, hipMemcpyDeviceToHost));
            printf("launches  nb=%d: %.2f us/step (2 launches/step) bad=%d\n", nb, 1e3 * ms / S, bd);
        }
    }
    return 0;
}
