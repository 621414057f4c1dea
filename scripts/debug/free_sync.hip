// Does hipFree (and hipHostFree) wait for work queued on OTHER streams?  A kernel spins ~300 ms on a non-blocking
// stream; the host then frees an UNRELATED buffer and times the call.  ~300 ms: the free drains the device (as the
// header documents); microseconds: it does not, and a free of memory a queued launch still uses is a use-after-free.
// (Safe by construction: the spinning kernel touches only its own buffer, which is freed after a synchronize.)
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>

__global__ void spin(unsigned long long ticks, int *out) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();  // 100 MHz
    while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(100);
    if (threadIdx.x == 0) out[blockIdx.x] = 1;
}

static double ms_since(std::chrono::steady_clock::time_point t) {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t).count();
}

int main() {
    hipStream_t s;
    if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return 1;
    int *own = nullptr;
    void *a = nullptr, *b = nullptr, *h = nullptr;
    if (hipMalloc(&own, 1024 * sizeof(int)) != hipSuccess) return 1;
    for (int trial = 0; trial < 2; trial++) {
        if (hipMalloc(&a, 1 << 20) || hipMalloc(&b, 64 << 20) || hipHostMalloc(&h, 1 << 20, 0)) return 1;
        hipDeviceSynchronize();
        auto t = std::chrono::steady_clock::now();
        spin<<<8, 64, 0, s>>>(30000000ull, own);  // 300 ms
        const double launch = ms_since(t);
        t = std::chrono::steady_clock::now();
        hipError_t e1 = hipFree(a);
        const double f1 = ms_since(t);
        t = std::chrono::steady_clock::now();
        hipError_t e3 = hipHostFree(h);
        const double f3 = ms_since(t);
        t = std::chrono::steady_clock::now();
        hipError_t e2 = hipFree(b);
        const double f2 = ms_since(t);
        t = std::chrono::steady_clock::now();
        hipError_t e4 = hipStreamSynchronize(s);
        const double sy = ms_since(t);
        printf("trial %d: launch %.3f ms; hipFree(1 MiB) %.3f ms rc=%d; hipHostFree %.3f ms rc=%d; hipFree(64 MiB) %.3f ms "
               "rc=%d; then stream sync %.3f ms rc=%d\n", trial, launch, f1, (int)e1, f3, (int)e3, f2, (int)e2, sy, (int)e4);
    }
    hipFree(own);
    hipStreamDestroy(s);
    return 0;
}
