// fused.h -- device helpers shared by the fused sweep kernels (villain.hip: the general fused kernel,
// villain_hot.hip: the fast-draw kernel): NumPy-stream draws by position, rejection reports, statistics,
// the LDS small-offset jump table.
#pragma once
#include "villain.h"

namespace sv {

#ifndef TWO_PI
#define TWO_PI 6.283185307179586
#endif

// Block order inside one sweep's descriptor array:
//   [0] metropolis (uniform V), then per colour c: [1+5c] dphi (uniform), [2+5c] fwd mu=0,
//   [3+5c] bwd mu=0, [4+5c] fwd mu=1, [5+5c] bwd mu=1 (bounded choice).
__device__ __forceinline__ u128 block_base(const Block &b) { return u128{b.base_lo, b.base_hi}; }

__device__ __forceinline__ void report(const DevScratch &S, uint32_t sweep, uint32_t block, uint32_t pos,
                                       uint32_t rep = 0) {
    uint32_t i = atomicAdd(S.nreport, 1u);
    if (i < (uint32_t)MAX_REPORTS) S.reports[i] = Report{sweep, block, pos, rep};
    __hip_atomic_store(S.abort, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (S.gate) __hip_atomic_fetch_min(S.gate, (int32_t)sweep, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (S.hflag) __hip_atomic_store(S.hflag, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    // drain here, on the rare path: a result still pending at the join would make the compiler wait
    // for every outstanding load and store (the row prefetch, the finished-row stores) on the common path
    __builtin_amdgcn_s_waitcnt(0);
}

// a launch of sweep `sweep` has nothing to do: a report came from an earlier sweep (with a gate, DevScratch), or
// from any launch since the batch's reset (without)
// The flag decides correctness, not only speed: the launch of sweep k + 1 writes the buffer sweep k read, so behind a
// failing sweep it must exit (the replay reads that buffer).  Hence a load that bypasses the caches (volatile: every
// XCD sees the report's agent-scope store).  (A scalar-cache read was measured no faster for the drains, r5: ~5.1 us
// per early-exit launch either way, profiles/r05_reject_trace_*.)
__device__ __forceinline__ bool sweep_cancelled(const DevScratch &S, uint32_t sweep) {
    if (S.gate) return *(volatile const int32_t *)S.gate < (int32_t)sweep;
    return *(volatile const int32_t *)S.abort != 0;
}

// stream position of bounded draw d, accounting for known rejected positions (sorted)
__device__ __forceinline__ uint32_t skip_pos(const Block &b, const uint32_t *skips, uint32_t d) {
    uint32_t q = d;
    for (int i = 0; i < b.nskip; i++)
        if (skips[b.skip0 + i] <= q) q++;
    return q;
}

// uint32 at stream position q of a bounded block, by full jump from the block base
__device__ __forceinline__ uint32_t bounded_word(const JumpTables *T, const Block &b, uint32_t q) {
    if (b.has && q == 0) return b.buf;
    uint32_t qq = q - b.has;
    uint64_t X = xsl_rr(jump(T, block_base(b), qq >> 1));
    return (qq & 1) ? (uint32_t)(X >> 32) : (uint32_t)X;
}

// bounded draw d (index into the choice array), any path; reports rejections
__device__ __forceinline__ int64_t bounded_draw(const JumpTables *T, const Block &b, const uint32_t *skips, uint32_t d,
                                                const VParams &P, const DevScratch &S, uint32_t sweep, uint32_t bidx) {
    uint32_t q = skip_pos(b, skips, d);
    bool rej;
    uint32_t idx = lemire(bounded_word(T, b, q), P.k, P.thr, &rej);
    if (rej) report(S, sweep, bidx, q);
    return P.W * ((int64_t)idx - P.interval_n);
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

// One atomic quadruple per WORKGROUP (every thread must call this): same-address atomics from thousands of waves
// serialize in one L2 channel.  psum is the lane's exact acceptance sum (common.h), flushed as three limbs into the
// slot's host-owned words.
template <int MAXW = 16>  // (waves per workgroup: the LDS it takes counts against the replica kernel's 4th workgroup)
__device__ __forceinline__ void flush_stats(sv_stats *st, int64_t acc, const AccFx &psum) {
    __shared__ unsigned long long s_w[4][MAXW];
    unsigned long long w[4];
    w[0] = (unsigned long long)acc;
    fx_limbs(psum, w[1], w[2], w[3]);
    for (int o = 32; o > 0; o >>= 1)
        for (int i = 0; i < 4; i++) w[i] += __shfl_xor(w[i], o);
    if ((threadIdx.x & 63) == 0)
        for (int i = 0; i < 4; i++) s_w[i][threadIdx.x >> 6] = w[i];
    __syncthreads();
    if (threadIdx.x < 4) {
        unsigned long long t = 0;
        for (int v = 0; v < (int)(blockDim.x >> 6); v++) t += s_w[threadIdx.x][v];
        atomicAdd(stat_word(st, threadIdx.x), t);
    }
}

template <int NW>
struct FusedGeom {
    static constexpr int R = 2 * NW + 3;  // ring rows: outputs t.. up to prefetched rows t+2+2NW
};



// v mod N for v in [-2N, 3N) without a division
__device__ __forceinline__ int32_t wrapN(int32_t v, int32_t N) {
    v = v < 0 ? v + N : v;
    v = v < 0 ? v + N : v;
    v = v >= N ? v - N : v;
    v = v >= N ? v - N : v;
    return v;
}

#ifndef SV_ABLATE
#define SV_ABLATE 0  // timing experiments only: 1 = no exp, 2 = no RNG compositions, 4 = no wrapped-column jumps,
                     // 8 = no HBM stores, 16 = no HBM loads, 32 = no barriers, 64 = no choice draws,
                     // 256 / 512 = n kept in HBM as int32 / int16 (villain_sweep_hot; valid from a cold start only)
#endif
// d = a*b + c as the three-address v_fma_f64: the compiler writes ocml's Horner chain as v_fmac_f64 on a copy of
// each hoisted coefficient (one v_mov_b64 per step); written out, the coefficients are read in place
#ifndef SV_EXP_SCOEF
#define SV_EXP_SCOEF 0  // coefficients as SGPR operands: villain_hot.hip sets it (18 VGPRs fewer at 4 waves per SIMD)
#endif
__device__ __forceinline__ double fma3(double a, double b, double c) {
    double d;
#if SV_EXP_SCOEF
    asm("v_fma_f64 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "s"(c));
#else
    asm("v_fma_f64 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "v"(c));
#endif
    return d;
}
// a*b + 1.0 (inline constant operand)
__device__ __forceinline__ double fma3_one(double a, double b) {
    double d;
    asm("v_fma_f64 %0, %1, %2, 1.0" : "=v"(d) : "v"(a), "v"(b));
    return d;
}
// a*b + c, b an SGPR pair
__device__ __forceinline__ double fma3_s(double a, double b, double c) {
    double d;
    asm("v_fma_f64 %0, %1, %2, %3" : "=v"(d) : "v"(a), "s"(b), "v"(c));
    return d;
}
// ocml's __ocml_exp_f64 (ROCm device libs, ocml.bc) restated operation for operation -- the same
// reduction, polynomial, ldexp and range selects, hence the same bits as exp()
__device__ __forceinline__ double exp_ocml(double x) {
    const double t = __builtin_rint(x * 0x1.71547652b82fep+0);
    const double nt = -t;
    double r = __builtin_fma(nt, 0x1.62e42fefa39efp-1, x);
    r = __builtin_fma(nt, 0x1.abc9e3b39803fp-56, r);
    double p = fma3_s(r, 0x1.ade156a5dcb37p-26, 0x1.28af3fca7ab0cp-22);
    p = fma3(r, p, 0x1.71dee623fde64p-19);
    p = fma3(r, p, 0x1.a01997c89e6b0p-16);
    p = fma3(r, p, 0x1.a01a014761f6ep-13);
    p = fma3(r, p, 0x1.6c16c1852b7b0p-10);
    p = fma3(r, p, 0x1.1111111122322p-7);
    p = fma3(r, p, 0x1.55555555502a1p-5);
    p = fma3(r, p, 0x1.5555555555511p-3);
    p = fma3(r, p, 0x1.000000000000bp-1);
    p = fma3_one(r, p);
    p = fma3_one(r, p);
    double e = __builtin_amdgcn_ldexp(p, (int)t);
    e = x > 1024.0 ? __builtin_inf() : e;
    return x < -1075.0 ? 0.0 : e;
}
__device__ __forceinline__ double sv_exp(double x) {
#if SV_ABLATE & 1
    return 1.0 + x * 0.5;
#else
    return exp_ocml(x);
#endif
}
__device__ __forceinline__ u128 sv_apply(const Affine &f, u128 s) {
#if SV_ABLATE & 2
    return u128{s.lo ^ f.A.lo, s.hi + f.C.hi};
#else
    return apply(f, s);
#endif
}

__device__ __forceinline__ u128 readlane128(u128 v, int lane) {
    u128 r;
    const uint32_t a = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v.lo, lane);
    const uint32_t b = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v.lo >> 32), lane);
    const uint32_t c = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v.hi, lane);
    const uint32_t d = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v.hi >> 32), lane);
    r.lo = ((uint64_t)b << 32) | a;
    r.hi = ((uint64_t)d << 32) | c;
    return r;
}

// Row-base position of block type `ty` (0 metropolis, 1 dphi, 2..5 bounded words) for global row gq.
// Bases sit at column xb, the strip's first non-wrapped region column.
__device__ __forceinline__ int64_t base_pos(int ty, int64_t gq, int64_t N, int64_t xb, uint32_t has) {
    const int64_t lin = gq * N + xb;
    if (ty == 0) return lin;
    const int64_t rank = lin >> 1;
    if (ty == 1) return rank;
    const int64_t p = rank - (int64_t)has;
    return p < 0 ? 0 : (p >> 1);
}

// The small-offset maps in LDS as two arrays (A, C) of 16-B entries: lanes read consecutive entries, and
// at a 16-B stride the 16 lanes of a ds_read_b128 group hit 64 distinct banks (the 64-B Affine stride of
// an array of structs put 4 lanes on each bank).
struct alignas(16) SmallTab {
    u128 A[SMALL_LDS];
    u128 C[SMALL_LDS];
    __device__ __forceinline__ Affine operator[](int64_t i) const { return Affine{A[i], C[i]}; }
};

struct Draws {
    double u, dphi;
    int32_t cn[4];  // W * (choice - interval_n); |W * interval_n| < 2^28 on this path
};

// Slow paths (branched around when no lane needs them).  The trailing wait keeps table loads from
// leaving a pending-VMEM hazard on merged values, which would drain the row prefetch early.
__device__ __forceinline__ u128 full_jump(const JumpTables *T, const Block *blk, uint32_t pos) {
    u128 r = jump(T, block_base(*blk), pos);
    __builtin_amdgcn_s_waitcnt(0);
    return r;
}
// The same with the level tables' entries loaded together (digit 0's entry is the identity map): one memory round
// trip instead of up to JUMP_LEVELS dependent ones, for the compositions with the identity maps of zero digits and 32
// more live registers -- for the kernels' prologues (row bases), not their loops
__device__ __forceinline__ u128 full_jump_flat(const JumpTables *T, const Block *blk, uint32_t pos) {
    Affine m[JUMP_LEVELS];
#pragma unroll
    for (int l = 0; l < JUMP_LEVELS; l++) m[l] = T->level[l][(pos >> (l * JUMP_DIGIT_BITS)) & (JUMP_DIGITS - 1)];
    u128 r = block_base(*blk);
#pragma unroll
    for (int l = 0; l < JUMP_LEVELS; l++) r = apply(m[l], r);
    __builtin_amdgcn_s_waitcnt(0);
    return r;
}

__device__ __forceinline__ u128 from_base(const JumpTables *T, const Block *blk, const SmallTab &sm, u128 base,
                                          int64_t bpos, int64_t pos) {
    const int64_t off = pos - bpos;
    u128 st;
    if (off >= 0 && off < SMALL_LDS) st = apply(sm[off], base);
#if SV_ABLATE & 4
    else st = apply(sm[off & (SMALL_LDS - 1)], base);  // timing experiment: no full jumps at wrapped columns
#else
    else st = full_jump(T, blk, (uint32_t)pos);
#endif
    return st;
}

// What one workgroup's replica reads: its sweep descriptors and its PCG64 jump tables.
struct Rep {
    const Block *blocks;
    const JumpTables *T;
    uint32_t id;
};

__device__ __forceinline__ int32_t choice_value(const FArgs &A, const Rep &RP, uint32_t word, uint32_t bidx,
                                                uint32_t spos) {
    bool rej;
    const uint32_t idx = lemire(word, A.P.k, A.P.thr, &rej);
    if (rej) report(A.S, A.sweep, bidx, spos, RP.id);
    return (int32_t)A.P.W * ((int32_t)idx - (int32_t)A.P.interval_n);
}

// General draws: any strip (wrapped columns), skips, mismatched buffers.  6 compositions per site.
// Columns of an edge strip that wrap around the lattice (global columns outside [xb, xb + RW)) draw
// from the wave's second set of row bases `wb`, kept at global column xw, so no lane needs a full jump.
__device__ __forceinline__ Draws draws_general(const FArgs &A, const Rep &RP, int c, bool active, int64_t gq, int64_t gx,
                                               int64_t xb, const u128 *bases, const SmallTab &sm, bool edge,
                                               int64_t xw, const u128 *wb) {
    const JumpTables *T = RP.T;
    const int64_t N = A.G.Nx;  // row length of the global stream layout
    const int bb = 1 + 5 * c;
    const int64_t lin = gq * N + gx, rank = lin >> 1;
    Draws D;
    D.u = 0.0;
    D.dphi = 0.0;
    D.cn[0] = D.cn[1] = D.cn[2] = D.cn[3] = 0;
    if (!active) return D;
    const bool wr = edge && (gx < xb || gx >= xb + RW);
    const int64_t xr = wr ? xw : xb;
    D.u = 0.0 + 1.0 * to_double(xsl_rr(from_base(T, &RP.blocks[0], sm, wr ? wb[0] : bases[0], gq * N + xr, lin)));
    D.dphi = A.P.lo_phi + A.P.range_phi * to_double(xsl_rr(from_base(T, &RP.blocks[bb], sm, wr ? wb[1] : bases[1],
                                                                     (gq * N + xr) >> 1, rank)));
    if (A.P.k > 1) {
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const Block *B = &RP.blocks[bb + 1 + q];
            uint32_t word, spos = (uint32_t)rank;
            {
                // known rejected positions push this draw's stream position forward (skip_pos); the row base sits
                // at the unshifted position of column xr, so the shifted word is still a small offset ahead of it
                // (from_base falls back to a full jump otherwise)
                if (B->nskip) spos = skip_pos(*B, A.skips, (uint32_t)rank);
                const int64_t qq = (int64_t)spos - (int64_t)B->has;
                const int64_t wi = qq < 0 ? 0 : (qq >> 1);
                const uint64_t X = xsl_rr(from_base(T, B, sm, wr ? wb[2 + q] : bases[2 + q], base_pos(2, gq, N, xr, B->has), wi));
                word = (qq & 1) ? (uint32_t)(X >> 32) : (uint32_t)X;
                if (qq < 0) word = B->buf;  // has && rank == 0: the buffered half-word
            }
            D.cn[q] = choice_value(A, RP, word, (uint32_t)(bb + 1 + q), spos);
        }
    }
    return D;
}

// The paired draws swap one 32-bit half with the neighbouring lane: `send` of lane - 1 (half = 1) or lane + 1
// (half = 0), wrapping around the wave.  DPP wave rotates are one VALU move each (on gfx950 wave_ror:1 reads lane
// i - 1 and wave_rol:1 lane i + 1, scripts/perf/dpp_check.hip) where ds_bpermute is an LDS round trip the draw
// waits on.  All 64 lanes execute the draws (inactive sites only discard their results).
__device__ __forceinline__ uint32_t pair_exchange(uint32_t send, uint32_t half, int lane) {
    (void)lane;
    const uint32_t prev = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)send, 0x13C /* wave_ror:1 */, 0xF, 0xF, false);
    const uint32_t next = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)send, 0x134 /* wave_rol:1 */, 0xF, 0xF, false);
    return half ? prev : next;
}

// Fast draws for interior strips (no wrapped columns, no skips, equal buffers within each
// forward/backward pair).  4 compositions per site: the fwd and bwd choice blocks of a direction
// read the SAME u64 word for two adjacent lanes (its two 32-bit halves), so each lane of a pair
// computes one block's word and swaps the other half with its partner.
// Per-lane constants of the fast draws, packed in one register per colour: the small-table offsets of
// the metropolis (bits 0-6), dphi (7-13) and the two choice words (14-20, 21-27) and which half of
// each word pair the lane computes (28, 29).  They are the same for every row a wave visits (rows
// advance NW = 4 at a time, so every parity involved is fixed), hence computed once per kernel.
__device__ __forceinline__ uint32_t fast_pack(const uint32_t *hasw, int32_t lane, uint32_t rowlin, uint32_t xs,
                                              uint32_t gx, uint32_t xb) {
    const uint32_t lin = rowlin + gx, rank = lin >> 1;
    const uint32_t PR = (rowlin + xb) >> 1;
    uint32_t pk = ((gx - xb) & (SMALL_LDS - 1)) | (((rank - PR) & (SMALL_LDS - 1)) << 7);
    const uint32_t R0 = (rowlin + xs) >> 1;  // rank of lane 0
#pragma unroll
    for (int mu = 0; mu < 2; mu++) {
        const uint32_t h = hasw[mu];
        const uint32_t P = (R0 - h) & 1u;   // pairing parity of the row
        const uint32_t PW = (PR - h) >> 1;  // word index of the row base
        uint32_t qq = rank - h;
        if (lane == 63 && P) qq = R0 - h;  // lane 63 serves lane 0's word
        const uint32_t half = (lane == 63 && P) ? 0u : (qq & 1u);
        pk |= (((qq >> 1) - PW) & (SMALL_LDS - 1)) << (14 + 7 * mu);
        pk |= half << (28 + mu);
    }
    return pk;
}

// fast_pack for per-block buffered-half flags (h4: f0, b0, f1, b1), the replay of a sweep that met a NumPy Lemire
// rejection (villain_sweep_hot_split): a rejected word shifts the rest of its block by one half-word, so a direction's
// fwd and bwd blocks can sit at opposite pairing parities.  Then ("mismatched", bit mu of `mism`) every lane computes
// the one word in which it holds the LOW half (the fwd word when its fwd draw is a low half, else the bwd word) and
// passes that word's high half to lane + 1: still one word per lane and direction.  Matched directions pair as in
// fast_pack (bits 28 + mu: the block the lane computes, 0 fwd / 1 bwd).  Lane 63 (never an active site: strips have
// <= 63 colour sites per row) computes the word in which lane 0 holds the high half.
__device__ __forceinline__ uint32_t fast_pack_g(const uint32_t *h4, int32_t lane, uint32_t rowlin, uint32_t xs,
                                                uint32_t gx, uint32_t xb, uint32_t &mism) {
    const uint32_t lin = rowlin + gx, rank = lin >> 1;
    const uint32_t PR = (rowlin + xb) >> 1;
    uint32_t pk = ((gx - xb) & (SMALL_LDS - 1)) | (((rank - PR) & (SMALL_LDS - 1)) << 7);
    const uint32_t R0 = (rowlin + xs) >> 1;  // rank of lane 0
    mism = 0;
#pragma unroll
    for (int mu = 0; mu < 2; mu++) {
        const uint32_t hf = h4[2 * mu], hb = h4[2 * mu + 1];
        if (hf != hb) mism |= 1u << mu;
        uint32_t sel = (rank - hf) & 1u, r = rank;
        if (lane == 63) {
            if ((R0 - hf) & 1u) sel = 0u, r = R0;       // lane 0's fwd draw is a high half
            else if ((R0 - hb) & 1u) sel = 1u, r = R0;  // lane 0's bwd draw is a high half
        }
        const uint32_t h = sel ? hb : hf;
        const uint32_t PW = (PR - h) >> 1;  // word index of the row base (PR >= 1 on interior strips)
        pk |= ((((r - h) >> 1) - PW) & (SMALL_LDS - 1)) << (14 + 7 * mu);
        pk |= sel << (28 + mu);
    }
    return pk;
}

__device__ __forceinline__ Draws draws_fastp(const FArgs &A, const Rep &RP, int c, bool active, int32_t lane,
                                             uint32_t pk, uint32_t rank, const u128 *bases, const SmallTab &sm) {
    const int bb = 1 + 5 * c;
    Draws D;
    {
        const u128 st = sv_apply(sm[pk & (SMALL_LDS - 1)], bases[0]);
        D.u = 0.0 + 1.0 * to_double(xsl_rr(st));
    }
    {
        const u128 st = sv_apply(sm[(pk >> 7) & (SMALL_LDS - 1)], bases[1]);
        D.dphi = A.P.lo_phi + A.P.range_phi * to_double(xsl_rr(st));
    }
    D.cn[0] = D.cn[1] = D.cn[2] = D.cn[3] = 0;
    if (!(SV_ABLATE & 64) && A.P.k > 1) {
#pragma unroll
        for (int mu = 0; mu < 2; mu++) {
            const uint32_t half = (pk >> (28 + mu)) & 1u;
            const u128 st = sv_apply(sm[(pk >> (14 + 7 * mu)) & (SMALL_LDS - 1)], half ? bases[3 + 2 * mu] : bases[2 + 2 * mu]);
            const uint64_t X = xsl_rr(st);
            // lo lanes computed the fwd word (send its high half), hi lanes the bwd word (send its low half)
            const uint32_t send = half ? (uint32_t)X : (uint32_t)(X >> 32);
            const uint32_t got = pair_exchange(send, half, lane);
            const uint32_t wf = half ? got : (uint32_t)X;
            const uint32_t wb = half ? (uint32_t)(X >> 32) : got;
            if (active) {
                D.cn[2 * mu] = choice_value(A, RP, wf, (uint32_t)(bb + 1 + 2 * mu), rank);
                D.cn[2 * mu + 1] = choice_value(A, RP, wb, (uint32_t)(bb + 2 + 2 * mu), rank);
            }
        }
    }
    return D;
}

__device__ __forceinline__ Draws draws_fast(const FArgs &A, const Rep &RP, int c, const uint32_t *hasw, bool active,
                                            int32_t lane, uint32_t rowlin,
                                            uint32_t xs, uint32_t gx, uint32_t xb, const u128 *bases,
                                            const SmallTab &sm) {
    const int bb = 1 + 5 * c;
    const uint32_t lin = rowlin + gx, rank = lin >> 1;
    const uint32_t PM = rowlin + xb, PR = PM >> 1;
    Draws D;
    {
        const u128 st = sv_apply(sm[(gx - xb) & (SMALL_LDS - 1)], bases[0]);
        D.u = 0.0 + 1.0 * to_double(xsl_rr(st));
    }
    {
        const u128 st = sv_apply(sm[(rank - PR) & (SMALL_LDS - 1)], bases[1]);
        D.dphi = A.P.lo_phi + A.P.range_phi * to_double(xsl_rr(st));
    }
    D.cn[0] = D.cn[1] = D.cn[2] = D.cn[3] = 0;
    if (!(SV_ABLATE & 64) && A.P.k > 1) {
        const uint32_t R0 = (rowlin + xs) >> 1;  // rank of lane 0
#pragma unroll
        for (int mu = 0; mu < 2; mu++) {
            const uint32_t h = hasw[mu];  // has of this direction's fwd (= bwd) choice block, preloaded
            const uint32_t P = (R0 - h) & 1u;                        // pairing parity of this row
            const uint32_t PW = (PR - h) >> 1;                       // word index of the row base
            uint32_t qq = rank - h;
            if (lane == 63 && P) qq = R0 - h;                        // lane 63 serves lane 0's word
            const uint32_t half = (lane == 63 && P) ? 0u : (qq & 1u);
            const uint32_t w = qq >> 1;
            const u128 st = sv_apply(sm[(w - PW) & (SMALL_LDS - 1)], half ? bases[3 + 2 * mu] : bases[2 + 2 * mu]);
            const uint64_t X = xsl_rr(st);
            // lo lanes computed the fwd word (send its high half), hi lanes the bwd word (send its low half)
            const uint32_t send = half ? (uint32_t)X : (uint32_t)(X >> 32);
            const uint32_t got = pair_exchange(send, half, lane);
            const uint32_t wf = half ? got : (uint32_t)X;
            const uint32_t wb = half ? (uint32_t)(X >> 32) : got;
            if (active) {
                D.cn[2 * mu] = choice_value(A, RP, wf, (uint32_t)(bb + 1 + 2 * mu), rank);
                D.cn[2 * mu + 1] = choice_value(A, RP, wb, (uint32_t)(bb + 2 + 2 * mu), rank);
            }
        }
    }
    return D;
}

// ---- 128-bit affine step with explicit carries -------------------------------------------------------
// Each carry-out of v_mad_u64_u32 is consumed in the same asm statement, through VCC: no SGPR pair stays live
// (lane-mask carries held in SGPRs across statements spilled the kernel's scalar registers).
// d = a*b + c (64-bit); (hi:lo) += carry-out, returned in place
__device__ __forceinline__ uint64_t mad_kk(uint32_t a, uint32_t b, uint64_t c, uint32_t &lo, uint32_t &hi) {
    uint64_t d;
    asm("v_mad_u64_u32 %0, vcc, %3, %4, %5\n\t"
        "v_addc_co_u32 %1, vcc, %1, 0, vcc\n\t"
        "v_addc_co_u32 %2, vcc, %2, 0, vcc"
        : "=&v"(d), "+v"(lo), "+v"(hi) : "v"(a), "v"(b), "v"(c) : "vcc");
    return d;
}
// d = a*b + c (64-bit); x += carry-out
__device__ __forceinline__ uint64_t mad_k(uint32_t a, uint32_t b, uint64_t c, uint32_t &x) {
    uint64_t d;
    asm("v_mad_u64_u32 %0, vcc, %2, %3, %4\n\t"
        "v_addc_co_u32 %1, vcc, %1, 0, vcc"
        : "=&v"(d), "+v"(x) : "v"(a), "v"(b), "v"(c) : "vcc");
    return d;
}
// d = a*b + c (64-bit), carry-out dropped
__device__ __forceinline__ uint64_t mad_n(uint32_t a, uint32_t b, uint64_t c) {
    uint64_t d;
    asm("v_mad_u64_u32 %0, vcc, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "v"(c) : "vcc");
    return d;
}

// a*s + c (mod 2^128) on 32-bit limbs:
//   T  = a0 s0 + (c1:c0)                 -> r0; its carry (weight 2^64) goes into (c3:c2)
//   U  = a0 s1 + (c2:T.hi)                  carry (2^96) into c3
//   U2 = a1 s0 + U                       -> r1; carry (2^96) into c3
//   X  = a0 s2 + a1 s1 + a2 s0 + (c3:U2.hi) -> r2 (carries beyond 2^128 dropped)
//   r3 = X.hi + lo(a0 s3 + a1 s2 + a2 s1 + a3 s0)
__device__ __forceinline__ u128 mad128c(u128 a, u128 s, u128 c) {
    const uint32_t a0 = (uint32_t)a.lo, a1 = (uint32_t)(a.lo >> 32), a2 = (uint32_t)a.hi, a3 = (uint32_t)(a.hi >> 32);
    const uint32_t s0 = (uint32_t)s.lo, s1 = (uint32_t)(s.lo >> 32), s2 = (uint32_t)s.hi, s3 = (uint32_t)(s.hi >> 32);
    uint32_t c2 = (uint32_t)c.hi, c3 = (uint32_t)(c.hi >> 32);
    const uint64_t T = mad_kk(a0, s0, c.lo, c2, c3);
    const uint64_t U = mad_k(a0, s1, ((uint64_t)c2 << 32) | (T >> 32), c3);
    const uint64_t U2 = mad_k(a1, s0, U, c3);
    uint64_t X = mad_n(a0, s2, ((uint64_t)c3 << 32) | (U2 >> 32));
    X = mad_n(a1, s1, X);
    X = mad_n(a2, s0, X);
    const uint32_t r3 = (uint32_t)(X >> 32) + a0 * s3 + a1 * s2 + a2 * s1 + a3 * s0;
    return u128{((U2 & 0xFFFFFFFFull) << 32) | (T & 0xFFFFFFFFull), ((uint64_t)r3 << 32) | (X & 0xFFFFFFFFull)};
}
__device__ __forceinline__ u128 hot_apply(const SmallTab &sm, uint32_t i, u128 base) {
#if SV_ABLATE & 2
    return u128{base.lo ^ sm.A[i].lo, base.hi + sm.C[i].hi};
#else
    return mad128c(sm.A[i], base, sm.C[i]);
#endif
}

// NumPy random(): (x >> 11) * 2^-53, exactly: with m = x >> 11 = h 2^32 + l (h < 2^21),
// m 2^-53 = h 2^-21 + l 2^-53; l 2^-53 is exact, and the fma's sum is m 2^-53 (53 significant bits)
__device__ __forceinline__ double u53(uint64_t x) {
    // one 64-bit shift gives both halves of m = x >> 11 (h < 2^21, l < 2^32); h 2^-21 + l 2^-53 is exact
    const uint64_t m = x >> 11;
    return __builtin_fma((double)(uint32_t)(m >> 32), 0x1p-21, (double)(uint32_t)m * 0x1p-53);
}



// Per-sweep statistics are accumulated in NSTRIPE stripes (one 128-B line each) picked by workgroup:
// thousands of short waves adding into ONE address serialize in one L2 channel (measured: ~200 us
// per L=1024 colour pass).  fold_stripes sums them into the sweep's sv_stats in a fixed order.
static constexpr int NSTRIPE = 16;
struct StatStripe {
    unsigned long long acc;
    unsigned long long pw[3];  // the exact acceptance limbs (common.h)
    uint64_t pad[12];
};

#ifndef SV_WFLUSH_WG
#define SV_WFLUSH_WG 1  // 1: the workgroup's waves summed in LDS first, one stripe per workgroup (0: per wave, r5)
#endif
__device__ __forceinline__ void wflush(StatStripe *ss, int64_t acc, const AccFx &psum) {
    unsigned long long w[4];
    w[0] = (unsigned long long)acc;
    fx_limbs(psum, w[1], w[2], w[3]);
    for (int o = 32; o > 0; o >>= 1)
        for (int i = 0; i < 4; i++) w[i] += __shfl_xor(w[i], o);
#if SV_WFLUSH_WG
    __shared__ unsigned long long s_w[4][16];
    if ((threadIdx.x & 63) == 0)
        for (int i = 0; i < 4; i++) s_w[i][threadIdx.x >> 6] = w[i];
    __syncthreads();
    if (threadIdx.x < 4) {
        unsigned long long t = 0;
        for (int v = 0; v < (int)(blockDim.x >> 6); v++) t += s_w[threadIdx.x][v];
        StatStripe *st = ss + ((blockIdx.x + blockIdx.y * 7) & (NSTRIPE - 1));
        if (t) atomicAdd(threadIdx.x == 0 ? &st->acc : &st->pw[threadIdx.x - 1], t);
    }
    __syncthreads();
#else
    if ((threadIdx.x & 63) == 0) {
        StatStripe *st = ss + ((blockIdx.x + blockIdx.y * 7 + (threadIdx.x >> 6) * 3) & (NSTRIPE - 1));
        atomicAdd(&st->acc, w[0]);
        for (int i = 0; i < 3; i++) atomicAdd(&st->pw[i], w[1 + i]);
    }
#endif
}


// One site-update's draws in the fast kernels (villain_hot.hip, villain_block.hip)
struct HotDraws {
    double u, dphi;
    uint32_t w[4];  // the uint32 each choice block (f0, b0, f1, b1) draws for this site
};

// Edge strips: columns that wrap around the row draw from the second base set (at global column xw); every
// offset is < SMALL_LDS by construction; words unpaired (the wrap breaks the lane pairing).
// has4 / buf: each choice block's buffered-half flag and word.  SKIP (a sweep that replays known NumPy Lemire
// rejections): block j's draw d sits at stream position d + (the skips at or before it) -- skip_pos of the general
// kernel, with at most HOT_MAXSK positions per block read from LDS -- so its word is a half-word further on, still a
// small offset ahead of the row base (which sits at the unshifted position); spos returns the positions (reports).
static constexpr int HOT_MAXSK = 4;
// PB (the split replay, villain_sweep_hot_split): every choice block has its own buffered-half flag (a fwd/bwd pair
// may differ), so each block's word offset is computed from its own flag
template <bool SKIP = false, bool PB = false>
__device__ __forceinline__ HotDraws hot_draws_edge(const FArgs &A, int64_t gq, int32_t gx, int32_t xb, int32_t xw,
                                                   const u128 *bA, const u128 *bB, const SmallTab &sm,
                                                   const uint32_t *has4, const uint32_t *buf,
                                                   const uint32_t (*sk)[HOT_MAXSK] = nullptr, const int32_t *nsk = nullptr,
                                                   uint32_t *spos = nullptr) {
    const int64_t N = A.G.Nx;
    const bool wr = !(gx >= xb && gx < xb + SMALL_LDS);
    const int32_t xr = wr ? xw : xb;
    const int64_t lin = gq * N + gx, rank = lin >> 1, rb = (gq * N + xr) >> 1;
    // bA, bB point at the wave's two base sets in LDS: each lane reads the set it draws from (one base in
    // registers at a time, not both sets)
    const u128 *bs = wr ? bB : bA;
    HotDraws D;
    D.u = u53(xsl_rr(hot_apply(sm, (uint32_t)(gx - xr), bs[0])));
    D.dphi = A.P.lo_phi + A.P.range_phi * u53(xsl_rr(hot_apply(sm, (uint32_t)(rank - rb), bs[1])));
    if constexpr (PB) {
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const int64_t qq = rank - (int64_t)has4[j];
            const int64_t w0 = (rb - (int64_t)has4[j]) < 0 ? 0 : ((rb - (int64_t)has4[j]) >> 1);
            const uint32_t off = (uint32_t)((qq < 0 ? 0 : (qq >> 1)) - w0);
            const uint64_t X = xsl_rr(hot_apply(sm, off, bs[2 + j]));
            uint32_t word = (qq & 1) ? (uint32_t)(X >> 32) : (uint32_t)X;
            if (qq < 0) word = buf[j];
            D.w[j] = word;
        }
        return D;
    } else if constexpr (!SKIP) {
        // equal flags within each fwd/bwd pair: one word offset per direction
#pragma unroll
        for (int mu = 0; mu < 2; mu++) {
            const int64_t qq = rank - (int64_t)has4[2 * mu];
            const int64_t w0 = (rb - (int64_t)has4[2 * mu]) < 0 ? 0 : ((rb - (int64_t)has4[2 * mu]) >> 1);
            const uint32_t off = (uint32_t)((qq < 0 ? 0 : (qq >> 1)) - w0);
#pragma unroll
            for (int fb = 0; fb < 2; fb++) {
                const uint64_t X = xsl_rr(hot_apply(sm, off, bs[2 + 2 * mu + fb]));
                uint32_t word = (qq & 1) ? (uint32_t)(X >> 32) : (uint32_t)X;
                if (qq < 0) word = buf[2 * mu + fb];  // has && rank == 0: the block's buffered half-word
                D.w[2 * mu + fb] = word;
            }
        }
        return D;
    }
#pragma unroll
    for (int j = 0; j < 4; j++) {
        int64_t q = rank;
#pragma unroll
        for (int i = 0; i < HOT_MAXSK; i++)
            if (i < nsk[j] && (int64_t)sk[j][i] <= q) q++;
        spos[j] = (uint32_t)q;
        const int64_t qq = q - (int64_t)has4[j];
        const int64_t w0 = (rb - (int64_t)has4[j]) < 0 ? 0 : ((rb - (int64_t)has4[j]) >> 1);
        const uint32_t off = (uint32_t)((qq < 0 ? 0 : (qq >> 1)) - w0);
        const uint64_t X = xsl_rr(hot_apply(sm, off, bs[2 + j]));
        uint32_t word = (qq & 1) ? (uint32_t)(X >> 32) : (uint32_t)X;
        if (qq < 0) word = buf[j];  // has && position 0: the block's buffered half-word
        D.w[j] = word;
    }
    return D;
}

}  // namespace sv
