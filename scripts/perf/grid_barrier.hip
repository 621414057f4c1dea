// Grid-barrier microbenchmark (persistent multi-step launches): G workgroups of 1024 threads (84 KB of LDS each, one
// per CU, as worldline_step_fused) run `rounds` rounds of: write own slice, barrier, read another workgroup's slice
// (on another XCD) and check it, barrier.  Reports microseconds per barrier and mismatches (cross-XCD visibility).
// Every spin is bounded (s_memrealtime, 100 MHz): a barrier that does not complete within 20 ms sets err[1] and all
// waits after it give up, so the grid always drains.
//   hipcc --offload-arch=gfx950 -O3 scripts/perf/grid_barrier.hip -o gpurun_out/grid_barrier && ./gpurun_out/grid_barrier 225
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

// mode 0: release add, acquire spin; 1: relaxed add and spin (no cache maintenance: timing only); 2: release add,
// relaxed spin, one acquire fence after it; 3: as 2 without s_sleep
template <int MODE>
__device__ __forceinline__ bool gbar(uint32_t *count, uint32_t target, int *err) {
    __syncthreads();
    __shared__ int ok;
    if (threadIdx.x == 0) {
        if (MODE == 1) __hip_atomic_fetch_add(count, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        else __hip_atomic_fetch_add(count, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        int good = 1;
        while ((MODE == 0 ? __hip_atomic_load(count, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT)
                          : __hip_atomic_load(count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) < target) {
            if (MODE != 3) __builtin_amdgcn_s_sleep(1);
            __builtin_amdgcn_s_sleep(1);
            if (__builtin_amdgcn_s_memrealtime() - t0 > 2000000ull ||
                __hip_atomic_load(&err[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
                __hip_atomic_store(&err[1], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                good = 0;
                break;
            }
        }
        if (MODE >= 2) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        ok = good;
    }
    __syncthreads();
    return ok;
}

template <int MODE>
__global__ __launch_bounds__(1024) void gb_test(int *data, uint32_t *count, int rounds, int *err, int stride) {
    __shared__ double pad[84 * 1024 / 8 - 16];
    pad[threadIdx.x] = threadIdx.x;
    const int G = gridDim.x, w = blockIdx.x;
    const int src = (w + stride) % G;
    int bad = 0;
    for (int r = 0; r < rounds; r++) {
        data[(size_t)w * 1024 + threadIdx.x] = r * 1000003 + w + (int)pad[threadIdx.x & 15] * 0;
        if (!gbar<MODE>(count, (uint32_t)G * (2 * r + 1), err)) break;
        bad += data[(size_t)src * 1024 + threadIdx.x] != r * 1000003 + src;
        if (!gbar<MODE>(count, (uint32_t)G * (2 * r + 2), err)) break;
    }
    if (bad) atomicAdd(&err[0], bad);
}

int main(int argc, char **argv) {
    const int G = argc > 1 ? atoi(argv[1]) : 225, rounds = argc > 2 ? atoi(argv[2]) : 1000;
    int *data, *err;
    uint32_t *count;
    hipMalloc(&data, (size_t)G * 1024 * sizeof(int));
    hipMalloc(&count, sizeof(uint32_t));
    hipMalloc(&err, 2 * sizeof(int));
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    for (int mode = 0; mode < 4; mode++)
    for (int stride : {37}) {
        for (int rep = 0; rep < 2; rep++) {
            hipMemset(count, 0, sizeof(uint32_t));
            hipMemset(err, 0, 2 * sizeof(int));
            hipEventRecord(a);
            if (mode == 0) gb_test<0><<<G, 1024>>>(data, count, rounds, err, stride);
            else if (mode == 1) gb_test<1><<<G, 1024>>>(data, count, rounds, err, stride);
            else if (mode == 2) gb_test<2><<<G, 1024>>>(data, count, rounds, err, stride);
            else gb_test<3><<<G, 1024>>>(data, count, rounds, err, stride);
            hipEventRecord(b);
            if (hipEventSynchronize(b) != hipSuccess) {
                printf("kernel failed\n");
                return 1;
            }
            float ms = 0;
            hipEventElapsedTime(&ms, a, b);
            int e[2];
            hipMemcpy(e, err, sizeof(e), hipMemcpyDeviceToHost);
            printf("G=%d stride=%d rounds=%d mode %d: %.3f us per barrier, mismatches %d, timeout %d\n", G, stride, rounds, mode,
                   ms * 1000.0 / (2 * rounds), e[0], e[1]);
        }
    }
    return 0;
}
