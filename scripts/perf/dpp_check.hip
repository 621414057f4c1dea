// Which lane a DPP wave_ror:1 / wave_rol:1 move reads on this GPU (lane i -> i-1 or i+1), for the paired draws.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(unsigned *a, unsigned *b) {
    const unsigned v = threadIdx.x;
    a[threadIdx.x] = (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x13C, 0xF, 0xF, false);  // wave_ror:1
    b[threadIdx.x] = (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x134, 0xF, 0xF, false);  // wave_rol:1
}
int main() {
    unsigned *a, *b, ha[64], hb[64];
    if (hipMalloc(&a, 256) != hipSuccess || hipMalloc(&b, 256) != hipSuccess) return 1;
    k<<<1, 64>>>(a, b);
    if (hipMemcpy(ha, a, 256, hipMemcpyDeviceToHost) != hipSuccess || hipMemcpy(hb, b, 256, hipMemcpyDeviceToHost) != hipSuccess) return 1;
    printf("wave_ror:1 lanes 0..3, 15..17, 63: %u %u %u %u | %u %u %u | %u\n", ha[0], ha[1], ha[2], ha[3], ha[15], ha[16], ha[17], ha[63]);
    printf("wave_rol:1 lanes 0..3, 15..17, 63: %u %u %u %u | %u %u %u | %u\n", hb[0], hb[1], hb[2], hb[3], hb[15], hb[16], hb[17], hb[63]);
    return 0;
}
