// philox.h -- Philox4x32-10 (Salmon, Moraes, Dror, Shaw, "Parallel random numbers: as easy as 1, 2, 3", SC'11),
// the counter-based generator of the optional fast RNG mode (sv_rng mode 1).  Host and device.
#pragma once
#include <stdint.h>

#ifndef SV_HD
#define SV_HD __host__ __device__ __forceinline__
#endif

namespace sv {

struct P4 {
    uint32_t v[4];
};

// Philox4x32 with R = 10 rounds: round(c, k) = (hi(M1 c2) ^ c1 ^ k0, lo(M1 c2), hi(M0 c0) ^ c3 ^ k1, lo(M0 c0)),
// the key bumped by the Weyl constants before every round after the first
SV_HD P4 philox4x32_10(P4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int i = 0; i < 10; i++) {
        if (i) {
            k0 += 0x9E3779B9u;
            k1 += 0xBB67AE85u;
        }
        const uint64_t p0 = (uint64_t)0xD2511F53u * c.v[0];
        const uint64_t p1 = (uint64_t)0xCD9E8D57u * c.v[2];
        P4 n;
        n.v[0] = (uint32_t)(p1 >> 32) ^ c.v[1] ^ k0;
        n.v[1] = (uint32_t)p1;
        n.v[2] = (uint32_t)(p0 >> 32) ^ c.v[3] ^ k1;
        n.v[3] = (uint32_t)p0;
        c = n;
    }
    return c;
}

}  // namespace sv
