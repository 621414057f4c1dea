// pcg64.h -- NumPy PCG64 stream arithmetic for host and device (gfx950).
//
// The generators replay NumPy's Generator(PCG64) stream exactly (the reference draws every random
// number from `self.rng`, e.g. supervillain/generator/villain/neighborhood.py:87,98,105-107).  A GPU
// lane cannot step the stream serially, so every draw is addressed by its POSITION: PCG64 is an LCG,
// k steps are the affine map  s -> A_k s + C_k  (mod 2^128), and a lane reaches position p of a block
// by composing the block's base state with (A_p, C_p) from small tables.  Output is XSL-RR 128/64 of
// the advanced state (NumPy advances first, then outputs).
#pragma once
#include <stdint.h>

#ifndef SV_HD
#define SV_HD __host__ __device__ __forceinline__
#endif


namespace sv {

struct u128 {
    uint64_t lo, hi;
};

SV_HD uint64_t mulhi64(uint64_t a, uint64_t b) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __umul64hi(a, b);
#else
    return (uint64_t)(((unsigned __int128)a * b) >> 64);
#endif
}

// low 128 bits of a*b
SV_HD u128 mul(u128 a, u128 b) {
    u128 r;
    r.lo = a.lo * b.lo;
    r.hi = mulhi64(a.lo, b.lo) + a.lo * b.hi + a.hi * b.lo;
    return r;
}

SV_HD u128 add(u128 a, u128 b) {
    u128 r;
    r.lo = a.lo + b.lo;
    r.hi = a.hi + b.hi + (r.lo < a.lo ? 1u : 0u);
    return r;
}

// affine map s -> A s + C
struct Affine {
    u128 A, C;
};

#if defined(__HIP_DEVICE_COMPILE__)
// low 128 bits of a*s + c by operand scanning on 32-bit limbs: 6 v_mad_u64_u32 + 4 v_mul_lo_u32 (the
// generic form compiles to 12 multiplies), the addend folded into the partial sums
__device__ __forceinline__ u128 mad128(u128 a, u128 s, u128 c) {
    const uint32_t a0 = (uint32_t)a.lo, a1 = (uint32_t)(a.lo >> 32), a2 = (uint32_t)a.hi, a3 = (uint32_t)(a.hi >> 32);
    const uint32_t s0 = (uint32_t)s.lo, s1 = (uint32_t)(s.lo >> 32), s2 = (uint32_t)s.hi, s3 = (uint32_t)(s.hi >> 32);
    const uint32_t c0 = (uint32_t)c.lo, c1 = (uint32_t)(c.lo >> 32), c2 = (uint32_t)c.hi, c3 = (uint32_t)(c.hi >> 32);
    uint64_t t = (uint64_t)a0 * s0 + c0;
    const uint32_t r0 = (uint32_t)t;
    t = (uint64_t)a0 * s1 + ((t >> 32) + c1);
    uint32_t r1 = (uint32_t)t;
    t = (uint64_t)a0 * s2 + ((t >> 32) + c2);
    uint32_t r2 = (uint32_t)t;
    uint32_t r3 = a0 * s3 + (uint32_t)(t >> 32) + c3;
    t = (uint64_t)a1 * s0 + r1;
    r1 = (uint32_t)t;
    t = (uint64_t)a1 * s1 + ((t >> 32) + r2);
    r2 = (uint32_t)t;
    r3 += a1 * s2 + (uint32_t)(t >> 32);
    t = (uint64_t)a2 * s0 + r2;
    r2 = (uint32_t)t;
    r3 += a2 * s1 + (uint32_t)(t >> 32) + a3 * s0;
    return u128{((uint64_t)r1 << 32) | r0, ((uint64_t)r3 << 32) | r2};
}
SV_HD u128 apply(const Affine &f, u128 s) { return mad128(f.A, s, f.C); }
#else
SV_HD u128 apply(const Affine &f, u128 s) { return add(mul(f.A, s), f.C); }
#endif

// f after g  (apply g first, then f):  A = Af Ag, C = Af Cg + Cf
SV_HD Affine compose(const Affine &f, const Affine &g) {
    Affine r;
    r.A = mul(f.A, g.A);
    r.C = add(mul(f.A, g.C), f.C);
    return r;
}

SV_HD uint64_t xsl_rr(u128 s) {
#if defined(__HIP_DEVICE_COMPILE__)
    // rotate right by 32 as a half swap, then the rest with two 32-bit funnel shifts
    const uint64_t x = s.hi ^ s.lo;
    const uint32_t rot = (uint32_t)(s.hi >> 58);
    const uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
    const bool sw = (rot & 32u) != 0;
    const uint32_t a = sw ? hi : lo, b = sw ? lo : hi;
    const uint32_t nlo = __builtin_amdgcn_alignbit(b, a, rot & 31u);
    const uint32_t nhi = __builtin_amdgcn_alignbit(a, b, rot & 31u);
    return ((uint64_t)nhi << 32) | nlo;
#else
    uint64_t x = s.hi ^ s.lo;
    unsigned rot = (unsigned)(s.hi >> 58);
    return (x >> rot) | (x << ((64u - rot) & 63u));
#endif
}

static constexpr uint64_t MULT_HI = 0x2360ED051FC65DA4ull;
static constexpr uint64_t MULT_LO = 0x4385DF649FCCF645ull;

SV_HD u128 mult() { return u128{MULT_LO, MULT_HI}; }

SV_HD Affine step_map(u128 inc) { return Affine{mult(), inc}; }

SV_HD Affine identity() { return Affine{u128{1, 0}, u128{0, 0}}; }

// NumPy next_double: (u64 >> 11) * 2^-53
SV_HD double to_double(uint64_t x) { return (double)(x >> 11) * (1.0 / 9007199254740992.0); }

// Jump tables for one increment: LEVELS digits of DIGIT_BITS bits, entry [l][d] = map of d * 2^(l*DIGIT_BITS) steps.
// Plus a "small" table of maps for 0..SMALL-1 steps (the per-lane offsets inside a row).
static constexpr int JUMP_LEVELS = 4;
static constexpr int JUMP_DIGIT_BITS = 8;
static constexpr int JUMP_DIGITS = 1 << JUMP_DIGIT_BITS;
static constexpr int SMALL = 256;

struct JumpTables {
    Affine level[JUMP_LEVELS][JUMP_DIGITS];
    Affine small[SMALL];
};

// s advanced by p steps, p < 2^32, using the level tables.
SV_HD u128 jump(const JumpTables *T, u128 s, uint32_t p) {
#pragma unroll
    for (int l = 0; l < JUMP_LEVELS; l++) {
        uint32_t d = (p >> (l * JUMP_DIGIT_BITS)) & (JUMP_DIGITS - 1);
        if (d) s = apply(T->level[l][d], s);
    }
    return s;
}

// Lemire bounded draw on one uint32 (NumPy buffered_bounded_lemire_uint32, 32-bit path):
// returns the index, sets *reject when this uint32 is rejected (leftover < threshold).
SV_HD uint32_t lemire(uint32_t x, uint32_t k, uint32_t thr, bool *reject) {
    uint64_t m = (uint64_t)x * (uint64_t)k;
    *reject = (uint32_t)m < thr;
    return (uint32_t)(m >> 32);
}

}  // namespace sv
