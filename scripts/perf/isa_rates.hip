// isa_rates.hip -- measurement only: issue throughput of the VALU instructions the sweep kernels use
// (cycles per wave-instruction per SIMD, every SIMD of the chip busy), to price kernel rewrites.
//   hipcc --offload-arch=gfx950 -O3 scripts/perf/isa_rates.hip -o gpurun_out/isa_rates && ./gpurun_out/isa_rates
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

constexpr int ITERS = 2048;
constexpr int CH = 8;  // independent chains per lane

// 32-bit VGPR ops: v = op(v, b, c)
#define K32(NAME, ASM)                                                                       \
    __global__ __launch_bounds__(256) void NAME(uint32_t *out, uint32_t seed) {                \
        uint32_t v[CH];                                                                        \
        uint32_t b = seed ^ threadIdx.x, c = seed * 3u + threadIdx.x;                          \
        for (int i = 0; i < CH; i++) v[i] = seed + i * 77u + threadIdx.x;                      \
        for (int it = 0; it < ITERS; it++) {                                                   \
            _Pragma("unroll") for (int i = 0; i < CH; i++) asm volatile(ASM : "+v"(v[i]) : "v"(b), "v"(c) : "vcc"); \
        }                                                                                      \
        uint32_t s = 0;                                                                        \
        for (int i = 0; i < CH; i++) s ^= v[i];                                                \
        out[blockIdx.x * 256 + threadIdx.x] = s;                                               \
    }
// 64-bit VGPR-pair ops: v = op(v, b, c) with 64-bit operands
#define K64(NAME, ASM)                                                                       \
    __global__ __launch_bounds__(256) void NAME(uint32_t *out, uint32_t seed) {                \
        uint64_t v[CH];                                                                        \
        uint64_t b = seed ^ threadIdx.x, c = (uint64_t)seed * 3u + threadIdx.x;                \
        uint32_t b32 = seed + 5, c32 = seed * 7;                                              \
        for (int i = 0; i < CH; i++) v[i] = seed + i * 77u + threadIdx.x;                      \
        for (int it = 0; it < ITERS; it++) {                                                   \
            _Pragma("unroll") for (int i = 0; i < CH; i++) asm volatile(ASM : "+v"(v[i]) : "v"(b), "v"(c), "v"(b32), "v"(c32) : "vcc"); \
        }                                                                                      \
        uint64_t s = 0;                                                                        \
        for (int i = 0; i < CH; i++) s ^= v[i];                                                \
        out[blockIdx.x * 256 + threadIdx.x] = (uint32_t)s ^ (uint32_t)(s >> 32);             \
    }

K32(k_add_u32, "v_add_u32 %0, %0, %1")
K32(k_add3_u32, "v_add3_u32 %0, %0, %1, %2")
K32(k_mov_b32, "v_mov_b32 %0, %1")
K32(k_xor_b32, "v_xor_b32 %0, %0, %1")
K32(k_alignbit, "v_alignbit_b32 %0, %0, %1, %2")
K32(k_cndmask, "v_cndmask_b32 %0, %0, %1, vcc")
K32(k_mul_lo_u32, "v_mul_lo_u32 %0, %0, %1")
K32(k_mul_hi_u32, "v_mul_hi_u32 %0, %0, %1")
K32(k_mul_u32_u24, "v_mul_u32_u24 %0, %0, %1")
K32(k_mul_hi_u32_u24, "v_mul_hi_u32_u24 %0, %0, %1")
K32(k_mad_u32_u24, "v_mad_u32_u24 %0, %0, %1, %2")
K32(k_add_co, "v_add_co_u32 %0, vcc, %0, %1\n v_addc_co_u32 %0, vcc, %0, %2, vcc")
K32(k_fma_f32, "v_fma_f32 %0, %0, %1, %2")
K32(k_exp_f32, "v_exp_f32 %0, %0")
K32(k_cvt_f32_u32, "v_cvt_f32_u32 %0, %0")
K64(k_mad_u64_u32, "v_mad_u64_u32 %0, vcc, %3, %4, %0")
K64(k_lshl_add_u64, "v_lshl_add_u64 %0, %0, 0, %1")
K64(k_lshrrev_b64, "v_lshrrev_b64 %0, 11, %0")
K64(k_mov_b64, "v_mov_b64 %0, %1")
K64(k_add_f64, "v_add_f64 %0, %0, %1")
K64(k_mul_f64, "v_mul_f64 %0, %0, %1")
K64(k_fma_f64, "v_fma_f64 %0, %0, %1, %2")
K64(k_ldexp_f64, "v_ldexp_f64 %0, %0, %3")
K64(k_cvt_f64_i32, "v_cvt_f64_i32 %0, %3")
K64(k_cvt_f64_u32, "v_cvt_f64_u32 %0, %3")
K64(k_cmp_lt_f64, "v_cmp_lt_f64 vcc, %0, %1\n v_add_f64 %0, %0, %2")
K64(k_rndne_f64, "v_rndne_f64 %0, %0")
K64(k_pk_fma_f32, "v_pk_fma_f32 %0, %0, %1, %2")
K64(k_pk_mul_f32, "v_pk_mul_f32 %0, %0, %1")

__global__ void k_clock(uint64_t *o) {
    uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    uint32_t v = threadIdx.x;
    for (int i = 0; i < 2000000; i++) asm volatile("v_add_u32 %0, %0, 1" : "+v"(v));
    uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) { o[2 * blockIdx.x] = t1 - t0; o[2 * blockIdx.x + 1] = r1 - r0; }
    if (v == 12345678) o[0] = v;
}

typedef void (*KF)(uint32_t *, uint32_t);
struct E { const char *name; KF f; int ninstr; };

int main() {
    hipDeviceProp_t p;
    CHK(hipGetDeviceProperties(&p, 0));
    const int cus = p.multiProcessorCount;
    uint32_t *out;
    uint64_t *clk;
    CHK(hipMalloc(&out, (size_t)cus * 8 * 256 * 4 * 4));
    CHK(hipMalloc(&clk, cus * 16 * 8));
    // clock under an all-CU VALU load
    hipLaunchKernelGGL(k_clock, dim3(cus * 4), dim3(256), 0, 0, clk);
    CHK(hipDeviceSynchronize());
    uint64_t h[2];
    CHK(hipMemcpy(h, clk, 16, hipMemcpyDeviceToHost));
    const double ghz = (double)h[0] / (double)h[1] * 0.1;  // memrealtime is 100 MHz
    printf("{\"clock_GHz_under_load\": %.3f, \"cus\": %d}\n", ghz, cus);
    E es[] = {
        {"v_add_u32", k_add_u32, 1}, {"v_add3_u32", k_add3_u32, 1}, {"v_mov_b32", k_mov_b32, 1},
        {"v_xor_b32", k_xor_b32, 1}, {"v_alignbit_b32", k_alignbit, 1}, {"v_cndmask_b32", k_cndmask, 1},
        {"v_mul_lo_u32", k_mul_lo_u32, 1}, {"v_mul_hi_u32", k_mul_hi_u32, 1}, {"v_mul_u32_u24", k_mul_u32_u24, 1},
        {"v_mul_hi_u32_u24", k_mul_hi_u32_u24, 1}, {"v_mad_u32_u24", k_mad_u32_u24, 1},
        {"v_add_co_u32+v_addc_co_u32", k_add_co, 2}, {"v_fma_f32", k_fma_f32, 1}, {"v_exp_f32", k_exp_f32, 1},
        {"v_cvt_f32_u32", k_cvt_f32_u32, 1},
        {"v_mad_u64_u32", k_mad_u64_u32, 1}, {"v_lshl_add_u64", k_lshl_add_u64, 1},
        {"v_lshrrev_b64", k_lshrrev_b64, 1}, {"v_mov_b64", k_mov_b64, 1}, {"v_add_f64", k_add_f64, 1},
        {"v_mul_f64", k_mul_f64, 1}, {"v_fma_f64", k_fma_f64, 1}, {"v_ldexp_f64", k_ldexp_f64, 1},
        {"v_cvt_f64_i32", k_cvt_f64_i32, 1}, {"v_cvt_f64_u32", k_cvt_f64_u32, 1},
        {"v_cmp_lt_f64+v_add_f64", k_cmp_lt_f64, 2}, {"v_rndne_f64", k_rndne_f64, 1},
        {"v_pk_fma_f32", k_pk_fma_f32, 1}, {"v_pk_mul_f32", k_pk_mul_f32, 1},
    };
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    for (int wps : {2, 4}) {  // waves per SIMD
        const int grid = cus * wps;  // 256-thread blocks: 4 waves = one per SIMD
        for (auto &e : es) {
            hipLaunchKernelGGL(e.f, dim3(grid), dim3(256), 0, 0, out, 1u);
            CHK(hipEventRecord(e0));
            for (int r = 0; r < 5; r++) hipLaunchKernelGGL(e.f, dim3(grid), dim3(256), 0, 0, out, 1u);
            CHK(hipEventRecord(e1));
            CHK(hipEventSynchronize(e1));
            float ms;
            CHK(hipEventElapsedTime(&ms, e0, e1));
            const double winstr_per_simd = 5.0 * wps * ITERS * CH * e.ninstr;
            const double cyc = ms * 1e-3 * ghz * 1e9 / winstr_per_simd;
            printf("{\"instr\": \"%s\", \"waves_per_simd\": %d, \"cycles_per_wave_instr\": %.2f}\n", e.name, wps, cyc);
        }
    }
    return 0;
}
