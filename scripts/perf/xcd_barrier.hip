// XCD-local barrier microbenchmark: 256 workgroups of 1024 threads (84 KB of LDS each: one per
// CU); each finds its XCD (HW_REG_XCC_ID) and its place there from a ticket on that XCD's counter, and the P = 32
// workgroups of each XCD run `rounds` rounds of: write own slice, barrier with the XCD's members only, read another
// member's slice and check it, barrier.  The barrier is the band launches' (villain_hot.hip band_barrier): stores
// acknowledged, one workgroup-scope arrival in the XCD's L2, agent-scope polling loads, then `buffer_inv sc0` -- which
// does NOT drop this CU's L1 lines (measured: every re-read of a line after the first is stale; the band launches never
// re-read an address within a launch, and a launch starts with a clean L1).  Mode 0 therefore reads the other member's
// slice with L1-bypassing loads (agent-scope relaxed: global_load sc1), mode 2 invalidates with `buffer_inv sc1` and
// reads plainly.  Mode 1 replaces the barrier by the device-wide form of scripts/perf/grid_barrier.hip mode 0 (release add, acquire spin) over
// all 256 workgroups, for comparison on the same box.  Every spin is bounded (20 ms), so the grid always drains.
//   hipcc --offload-arch=gfx950 -O3 scripts/perf/xcd_barrier.hip -o gpurun_out/xcd_barrier && ./gpurun_out/xcd_barrier
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

__device__ __forceinline__ bool spin_until(uint32_t *cnt, uint32_t target, int *err, bool acquire) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    for (;;) {
        const uint32_t v = acquire ? __hip_atomic_load(cnt, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT)
                                   : __hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (v >= target) return true;
        if (__builtin_amdgcn_s_memrealtime() - t0 > 2000000ull ||
            __hip_atomic_load(&err[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
            __hip_atomic_store(&err[1], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            return false;
        }
        __builtin_amdgcn_s_sleep(1);
    }
}

template <int MODE>
__device__ __forceinline__ bool bar(uint32_t *cnt, uint32_t target, int *err) {
    __shared__ int ok;
    if (MODE != 1) __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    if (threadIdx.x == 0) {
        bool good;
        if (MODE == 0 || MODE == 2) {
            __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            good = spin_until(cnt, target, err, false);
            if (MODE == 0) asm volatile("buffer_inv sc0" ::: "memory");
            else asm volatile("buffer_inv sc1" ::: "memory");
        } else {
            __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
            good = spin_until(cnt, target, err, true);
        }
        ok = good;
    }
    __syncthreads();
    return ok;
}

template <int MODE>
__global__ __launch_bounds__(1024) void xb_test(int *data, uint32_t *ctrl, int rounds, int *err, int P) {
    __shared__ double pad[84 * 1024 / 8 - 16];
    __shared__ int s_slot;
    pad[threadIdx.x] = threadIdx.x;
    if (threadIdx.x == 0) {
        const uint32_t xcc = (uint32_t)__builtin_amdgcn_s_getreg(20 | (31 << 11)) & 0xFu;  // HW_REG_XCC_ID
        const uint32_t t = __hip_atomic_fetch_add(&ctrl[64 * xcc], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s_slot = xcc < 8 && (int)t < P ? (int)(xcc * P + t) : -1;
    }
    __syncthreads();
    const int slot = s_slot;
    if (slot < 0) {
        if (threadIdx.x == 0) atomicAdd(&err[2], 1);
        return;
    }
    const int xcd = slot / P, i = slot % P;
    // MODE 0: the XCD's own counter (its own 256-B line); MODE 1: one counter for the grid
    uint32_t *cnt = MODE != 1 ? &ctrl[64 * (8 + xcd)] : &ctrl[64 * 16];
    const uint32_t members = MODE != 1 ? (uint32_t)P : (uint32_t)(8 * P);
    const int src = MODE != 1 ? xcd * P + (i + 7) % P : (slot + 37) % (8 * P);
    int bad = 0;
    for (int r = 0; r < rounds; r++) {
        data[(size_t)slot * 1024 + threadIdx.x] = r * 1000003 + slot + (int)pad[threadIdx.x & 15] * 0;
        if (!bar<MODE>(cnt, members * (2 * r + 1), err)) break;
        const int got = MODE == 0 ? __hip_atomic_load(&data[(size_t)src * 1024 + threadIdx.x], __ATOMIC_RELAXED,
                                                      __HIP_MEMORY_SCOPE_AGENT)
                                  : data[(size_t)src * 1024 + threadIdx.x];
        bad += got != r * 1000003 + src;
        if (!bar<MODE>(cnt, members * (2 * r + 2), err)) break;
    }
    if (bad) atomicAdd(&err[0], bad);
}

int main(int argc, char **argv) {
    const int P = 32, G = 8 * P, rounds = argc > 1 ? atoi(argv[1]) : 2000;
    int *data, *err;
    uint32_t *ctrl;
    hipMalloc(&data, (size_t)G * 1024 * sizeof(int));
    hipMalloc(&ctrl, 64 * 17 * sizeof(uint32_t));
    hipMalloc(&err, 3 * sizeof(int));
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    for (int mode = 0; mode < 3; mode++)
        for (int rep = 0; rep < 3; rep++) {
            hipMemset(ctrl, 0, 64 * 17 * sizeof(uint32_t));
            hipMemset(err, 0, 3 * sizeof(int));
            hipEventRecord(a);
            if (mode == 0) xb_test<0><<<G, 1024>>>(data, ctrl, rounds, err, P);
            else if (mode == 1) xb_test<1><<<G, 1024>>>(data, ctrl, rounds, err, P);
            else xb_test<2><<<G, 1024>>>(data, ctrl, rounds, err, P);
            hipEventRecord(b);
            if (hipEventSynchronize(b) != hipSuccess) {
                printf("kernel failed\n");
                return 1;
            }
            float ms = 0;
            hipEventElapsedTime(&ms, a, b);
            int e[3];
            hipMemcpy(e, err, sizeof(e), hipMemcpyDeviceToHost);
            printf("%s barrier, %d workgroups, %d rounds: %.3f us per barrier, mismatches %d, timeout %d, unplaced %d\n",
                   mode == 0 ? "XCD-local (32 per XCD), sc1 reads" : mode == 1 ? "device-wide" : "XCD-local, buffer_inv sc1", G, rounds, ms * 1000.0 / (2 * rounds), e[0],
                   e[1], e[2]);
        }
    return 0;
}
