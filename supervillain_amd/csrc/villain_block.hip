// villain_block.hip -- multi-sweep launches of small periodic lattices by temporal blocking: K consecutive
// NeighborhoodUpdate sweeps (supervillain/generator/villain/neighborhood.py:59-137, one per call there) in one launch,
// with no workgroup ever waiting for another.
//
// Each workgroup owns a bs x bs block.  Sweep j of the launch decides the block extended by 2e rows / columns above
// and left and 3e below and right (e = K-1-j: domain.hip's deep-halo rule) and reads two more rows /
// columns around that; so the workgroup loads the frame of sweep 0 -- (bs + 5(K-1) + 5)^2 sites -- into LDS once, runs
// the K sweeps there, and after each sweep stores its own block into that sweep's output buffer (BlockArgs, villain.h).
// Every draw is addressed by its global stream position (the row bases of the frame's rows, in LDS, and the small-offset
// maps), so a halo site recomputed here receives exactly the update its owner gives it.  A later sweep's row bases are
// the earlier ones moved by one sweep's stream length (BlockArgs::step, checked by the host).
//
// Per site the arithmetic is villain_sweep_hot's (villain_hot.hip), operation for operation: the residuals of a
// colour-0 site from phi and n, the incremental r of neighborhood.py:129 handed to the colour-1 sites through LDS, the
// f64 exp of -dS and the comparison with the uniform, the unpaired choice words of the edge form.
#include "fused.h"

#ifndef SV_BLKTIME
#define SV_BLKTIME 0  // timing experiments: per-workgroup timestamps of the last launch (sv_debug_blocktime)
#endif

namespace sv {

#if SV_BLKTIME
// per workgroup: [0] entry, [1] frame loaded, [2] row bases ready, [3 + j] sweep j's stores issued, [15] exit
constexpr int BLT = 16;
__device__ uint64_t g_blktime[4096 * BLT];
#define BLK_T(i) do { if (threadIdx.x == 0 && blockIdx.x < 4096) g_blktime[blockIdx.x * BLT + (i)] = __builtin_amdgcn_s_memrealtime(); } while (0)
#else
#define BLK_T(i) do { } while (0)
#endif

// hot_draws_edge (fused.h) in 32-bit positions (N <= 512: every rank < 2^17): the frame's columns at or after xb draw
// from the row's set A, its wrapped columns (gx < xb) from set B at column 0; words unpaired, equal buffered-half flags
// within each fwd/bwd pair (hot_ok)
__device__ __forceinline__ HotDraws blk_draws(const VParams &P, int32_t N, int32_t gq, int32_t gx, int32_t xb,
                                             const u128 *bA, const u128 *bB, const SmallTab &sm, const uint32_t *has,
                                             const uint32_t *buf) {
    const bool wr = gx < xb;
    const int32_t xr = wr ? 0 : xb, row = gq * N;
    const int32_t rank = (row + gx) >> 1, rb = (row + xr) >> 1;
    const u128 *bs = wr ? bB : bA;
    HotDraws D;
    D.u = u53(xsl_rr(hot_apply(sm, (uint32_t)(gx - xr), bs[0])));
    D.dphi = P.lo_phi + P.range_phi * u53(xsl_rr(hot_apply(sm, (uint32_t)(rank - rb), bs[1])));
#pragma unroll
    for (int mu = 0; mu < 2; mu++) {
        const int32_t h = (int32_t)has[2 * mu], qq = rank - h, w0 = rb - h < 0 ? 0 : (rb - h) >> 1;
        const uint32_t off = (uint32_t)((qq < 0 ? 0 : qq >> 1) - w0);
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

template <int NWT>
__global__ __launch_bounds__(NWT * 64) void villain_sweep_block(FArgs A, BlockArgs B) {
    extern __shared__ __attribute__((aligned(16))) unsigned char blk_lds[];
    note_progress(A);
    if (sweep_cancelled(A.S, A.sweep)) return;  // (band batches' gate: a report in an earlier launch)
    BLK_T(0);
    constexpr int NT = NWT * 64;
    const int32_t N = A.G.Nx;
    const int64_t V = A.G.plane;
    const int K = B.K, E = K - 1, bs = B.bs;
    // (blocks dealt to the XCDs in contiguous runs measured level with round-robin, r4 profiles/r04_block_xcd_ab.txt)
    const int bl = (int)blockIdx.x;
    const int by = bl / B.nbx, bx = bl - by * B.nbx;
    const int32_t r0 = by * bs, c0 = bx * bs;
    const int F = block_frame(bs, K);
    const int32_t FR0 = r0 - 2 * E - 2, FC0 = c0 - 2 * E - 2;  // frame origin (lattice coordinates, may be < 0)

    SmallTab &s_small = *reinterpret_cast<SmallTab *>(blk_lds);
    u128 *s_base = reinterpret_cast<u128 *>(blk_lds + sizeof(SmallTab));  // [F][set][colour][6]
    double *s_phi = reinterpret_cast<double *>(s_base + (size_t)F * 24);
    double *s_r0 = s_phi + F * F;  // residual of link (0, q, x) at (q, x)
    double *s_r1 = s_r0 + F * F;   // residual of link (1, q, x) at (q, x)
    int32_t *s_n0 = reinterpret_cast<int32_t *>(s_r1 + F * F);
    int32_t *s_n1 = s_n0 + F * F;
    unsigned long long *s_acc = reinterpret_cast<unsigned long long *>(s_n1 + F * F);
    // per sweep j: s_acc[4 j + i], i = 0 accepted, 1..3 the exact acceptance limbs (common.h)
    int32_t *s_bad = reinterpret_cast<int32_t *>(s_acc + 64);

    int32_t *s_desc = s_bad + 4;  // [j][c][q]: choice block q of colour c in sweep j, {has, buf}
    if (threadIdx.x < 64) s_acc[threadIdx.x] = 0;
    if (threadIdx.x == 0) *s_bad = 0;

    // The prologue's loads are issued in the order they are consumed (the small-offset maps, the descriptors, the
    // frame's first round, the row bases' table entries), so that the workgroup waits about one memory round trip
    const int32_t xb = wrapN(FC0, N);
    const bool wraps = FC0 < 0 || FC0 + F > N;
    const int nset = wraps ? 2 : 1;
    for (int e = threadIdx.x; e < 2 * SMALL_LDS; e += NT) {
        if (e < SMALL_LDS) s_small.A[e] = A.T->small[e].A;
        else s_small.C[e - SMALL_LDS] = A.T->small[e - SMALL_LDS].C;
    }
    if ((int)threadIdx.x < 8 * K) {
        const int t = threadIdx.x, j = t >> 3, c = (t >> 2) & 1, q = t & 3;
        const Block &b = A.blocks[(int64_t)j * B.nb + 2 + 5 * c + q];
        s_desc[2 * t] = (int32_t)b.has;
        s_desc[2 * t + 1] = (int32_t)b.buf;
    }
    // the frame from the launch's input, wrapped onto the torus (F <= N: no site twice), FU sites per thread a round
    constexpr int FU = 4;
    uint32_t bad = 0;
    double fp[FU];
    int64_t fa[FU], fc[FU];
    auto frame_load = [&](int i0) {
#pragma unroll
        for (int u = 0; u < FU; u++) {
            const int idx = i0 + u * NT;
            if (idx < F * F) {
                const int i = idx / F, k = idx - i * F;
                const int32_t g = wrapN(FR0 + i, N) * N + wrapN(FC0 + k, N);
                fp[u] = B.phi[0][g];
                fa[u] = B.n[0][g];
                fc[u] = B.n[0][V + g];
            }
        }
    };
    auto frame_store = [&](int i0) {
#pragma unroll
        for (int u = 0; u < FU; u++) {
            const int idx = i0 + u * NT;
            if (idx < F * F) {
                // the +0.0 every site receives once per sweep (neighborhood.py:128), applied once: an accepted change
                // is added to the normalised value, which stays normalised (villain_hot.hip's commit)
                s_phi[idx] = fp[u] + 0.0;
                // the int32 image holds n exactly with room for K sweeps of changes (|W| interval_n <= 2^13)
                bad |= (uint32_t)((uint64_t)((fa[u] >> 30) + 1) > 1) | (uint32_t)((uint64_t)((fc[u] >> 30) + 1) > 1);
                s_n0[idx] = (int32_t)fa[u];
                s_n1[idx] = (int32_t)fc[u];
            }
        }
    };
    frame_load(threadIdx.x);
    // row bases of sweep 0 for frame rows 1 .. F-2 (the rows a colour pass decides): set 0 at column xb (the frame's
    // first column on the torus), set 1 at column 0 for the columns that wrap; per colour the six blocks in
    // hot_draws_edge's order (metropolis, dphi, the four choice blocks)
    for (int idx = threadIdx.x; idx < (F - 2) * nset * 12; idx += NT) {
        const int i = 1 + idx / (nset * 12), rem = idx % (nset * 12), s = rem / 12, slot = rem % 12;
        const int c = slot / 6, ty = slot % 6;
        const int blk = ty == 0 ? 0 : 1 + 5 * c + ty - 1;
        const uint32_t has = ty >= 2 ? A.blocks[blk].has : 0u;
        const uint32_t pos = (uint32_t)base_pos(ty, wrapN(FR0 + i, N), N, s ? 0 : xb, has);
        s_base[(i * 2 + s) * 12 + slot] =
            full_jump_flat(A.T, &A.blocks[blk], pos);
    }
    frame_store(threadIdx.x);
    for (int i0 = threadIdx.x + FU * NT; i0 < F * F; i0 += FU * NT) {  // (frames beyond FU sites per thread)
        frame_load(i0);
        frame_store(i0);
    }
    if (bad) *s_bad = 1;
#if SV_BLKTIME
    __syncthreads();
    BLK_T(1);
#endif

    const VParams P = A.P;
    const uint32_t kc = P.k, thr = P.thr;
    const int32_t Wn = (int32_t)P.W, nW = (int32_t)(P.W * P.interval_n);
    const double hk = P.half_kappa;

    for (int j = 0; j < K; j++) {
        const int e = E - j;
        const int32_t ra = r0 - 2 * e, rb = r0 + bs + 3 * e, ca = c0 - 2 * e, cb = c0 + bs + 3 * e;
        const uint32_t sweep_id = A.sweep + (uint32_t)j;
        __syncthreads();  // (the frame, the bases and the descriptors; the previous sweep's stores and advance)
        uint32_t has4[2][4], buf4[2][4];
#pragma unroll
        for (int c = 0; c < 2; c++)
#pragma unroll
            for (int q = 0; q < 4; q++) {
                has4[c][q] = (uint32_t)__builtin_amdgcn_readfirstlane(s_desc[2 * (8 * j + 4 * c + q)]);
                buf4[c][q] = (uint32_t)__builtin_amdgcn_readfirstlane(s_desc[2 * (8 * j + 4 * c + q) + 1]);
            }
        if (j == 0) BLK_T(2);
        int32_t acc_count = 0;
        AccFx psum;  // exact acceptance sum (common.h)

        // colour c on rows qlo..qhi and columns xlo..xhi (inclusive): villain_sweep_hot's ranges around the decided
        // region [ra, rb) x [ca, cb) -- colour 0 one row / column further on every side, colour 1 one further below
        // and right (the links stored at the region's last row / column).  The rows' colour-c sites are packed densely
        // onto the lanes (at most spr per row): idx -> (row, k) by an f32 reciprocal, exact here (idx + 1/2 sits at
        // least 1/(2 spr) from a multiple of spr; idx < 2^12)
        const int32_t qlo[2] = {ra - 1, ra}, qhi[2] = {rb + 1, rb}, xlo[2] = {ca - 1, ca}, xhi[2] = {cb + 1, cb};
        int nrows[2], spr[2];
        float inv[2];
#pragma unroll
        for (int c = 0; c < 2; c++) {
            nrows[c] = qhi[c] - qlo[c] + 1;
            spr[c] = (xhi[c] - xlo[c] + 2) >> 1;
            inv[c] = 1.0f / (float)spr[c];
        }
        auto site_of = [&](int c, int idx, int32_t &q, int32_t &x) {
            const int row = (int)(((float)idx + 0.5f) * inv[c]), k = idx - row * spr[c];
            q = qlo[c] + row;
            x = xlo[c] + ((q + xlo[c] + c) & 1) + 2 * k;  // colour c: q + x = c mod 2
            return row < nrows[c] && x <= xhi[c];
        };
        // the site's draws and the choice values W (index - interval_n) (neighborhood.py:105-107); a rejected word is
        // reported
        auto draw_site = [&](auto C, int32_t q, int32_t x, HotDraws &D, int32_t (&cn)[4]) {
            constexpr int c = decltype(C)::value;
            const int lq = q - FR0;
            const int32_t gq = wrapN(q, N), gx = wrapN(x, N);
            D = blk_draws(P, N, gq, gx, xb, &s_base[(lq * 2) * 12 + 6 * c], &s_base[(lq * 2 + 1) * 12 + 6 * c], s_small,
                          has4[c], buf4[c]);
            bool rej = false;
#pragma unroll
            for (int jj = 0; jj < 4; jj++) {
                const uint64_t m = (uint64_t)D.w[jj] * kc;
                rej |= (uint32_t)m < thr;
                cn[jj] = (int32_t)(m >> 32) * Wn - nW;
            }
            if (__builtin_expect(rej, 0)) {
                const uint32_t rank = (uint32_t)((gq * N + gx) >> 1);
#pragma unroll
                for (int jj = 0; jj < 4; jj++)
                    if ((uint32_t)((uint64_t)D.w[jj] * kc) < thr) report(A.S, sweep_id, (uint32_t)(1 + 5 * c + 1 + jj), rank);
            }
        };
        auto update = [&](auto C, int32_t q, int32_t x, const HotDraws &D, const int32_t (&cn)[4]) {
            constexpr int c = decltype(C)::value;
            const int s0 = (q - FR0) * F + (x - FC0);
            const bool own = q >= r0 && q < r0 + bs && x >= c0 && x < c0 + bs;
            const double mdp = 0.0 - D.dphi;  // d(change_phi) on a forward link, neighborhood.py:110
            if constexpr (c == 0) {
                const double ph = s_phi[s0];
                const int32_t n_f0 = s_n0[s0], n_b0 = s_n0[s0 - F], n_f1 = s_n1[s0], n_b1 = s_n1[s0 - 1];
                // r on the four links f0=(0,q,x), b0=(0,q-1,x), f1=(1,q,x), b1=(1,q,x-1) (neighborhood.py:91)
                double r[4];
                r[0] = (s_phi[s0 + F] - ph) - TWO_PI * (double)n_f0;
                r[1] = (ph - s_phi[s0 - F]) - TWO_PI * (double)n_b0;
                r[2] = (s_phi[s0 + 1] - ph) - TWO_PI * (double)n_f1;
                r[3] = (ph - s_phi[s0 - 1]) - TWO_PI * (double)n_b1;
                double tc[4], cr[4];
#pragma unroll
                for (int kk = 0; kk < 4; kk++) tc[kk] = TWO_PI * (double)cn[kk];
                cr[0] = mdp - tc[0];
                cr[1] = D.dphi - tc[1];
                cr[2] = mdp - tc[2];
                cr[3] = D.dphi - tc[3];
                double dS = (hk * cr[0]) * ((2.0 * r[0]) + cr[0]);
#pragma unroll
                for (int kk = 1; kk < 4; kk++) dS += (hk * cr[kk]) * ((2.0 * r[kk]) + cr[kk]);
                double p = sv_exp(-dS);
                p = p > 1.0 ? 1.0 : p;
                const bool acc = D.u < p;
                if (own) {
                    acc_count += acc;
                    fx_add(psum, p);
                }
                if (acc) {
                    // neighborhood.py:124-129: phi += change_phi, n += change_n, r += d(change_phi) - 2 pi change_n
                    s_phi[s0] = ph + D.dphi;
                    s_n0[s0] = n_f0 + cn[0];
                    s_n0[s0 - F] = n_b0 + cn[1];
                    s_n1[s0] = n_f1 + cn[2];
                    s_n1[s0 - 1] = n_b1 + cn[3];
                    r[0] = (r[0] + mdp) - tc[0];
                    r[1] = (r[1] + D.dphi) - tc[1];
                    r[2] = (r[2] + mdp) - tc[2];
                    r[3] = (r[3] + D.dphi) - tc[3];
                }
                s_r0[s0] = r[0];
                s_r0[s0 - F] = r[1];
                s_r1[s0] = r[2];
                s_r1[s0 - 1] = r[3];
            } else {
                double ri[4], cr[4];
                ri[0] = s_r0[s0];
                ri[1] = s_r0[s0 - F];
                ri[2] = s_r1[s0];
                ri[3] = s_r1[s0 - 1];
                cr[0] = mdp - TWO_PI * (double)cn[0];
                cr[1] = D.dphi - TWO_PI * (double)cn[1];
                cr[2] = mdp - TWO_PI * (double)cn[2];
                cr[3] = D.dphi - TWO_PI * (double)cn[3];
                double dS = (hk * cr[0]) * ((2.0 * ri[0]) + cr[0]);
#pragma unroll
                for (int kk = 1; kk < 4; kk++) dS += (hk * cr[kk]) * ((2.0 * ri[kk]) + cr[kk]);
                double p = sv_exp(-dS);
                p = p > 1.0 ? 1.0 : p;
                const bool acc = D.u < p;
                if (own) {
                    acc_count += acc;
                    fx_add(psum, p);
                }
                if (acc) {
                    s_phi[s0] = s_phi[s0] + D.dphi;
                    s_n0[s0] += cn[0];
                    s_n0[s0 - F] += cn[1];
                    s_n1[s0] += cn[2];
                    s_n1[s0 - 1] += cn[3];
                }
            }
        };
        const std::integral_constant<int, 0> C0{};
        const std::integral_constant<int, 1> C1{};
        // (8-wave workgroups only: the 16-wave form must stay within 128 VGPRs)
        // (the colour-1 draws made in the colour-0 pass: one round of lanes per colour)
        if (NWT == 8 && nrows[0] * spr[0] <= NT && nrows[1] * spr[1] <= NT) {
            // one round of lanes per colour: the colour-1 draws (independent of the state) are made in the colour-0
            // pass, beside its site-update, and held in registers across the barrier
            int32_t q1, x1;
            const bool a1 = site_of(1, threadIdx.x, q1, x1);
            HotDraws D1;
            int32_t cn1[4];
            if (a1) draw_site(C1, q1, x1, D1, cn1);
            int32_t q0, x0;
            if (site_of(0, threadIdx.x, q0, x0)) {
                HotDraws D0;
                int32_t cn0[4];
                draw_site(C0, q0, x0, D0, cn0);
                update(C0, q0, x0, D0, cn0);
            }
            __syncthreads();
            if (a1) update(C1, q1, x1, D1, cn1);
            __syncthreads();
        } else {
            for (int base = 0; base < nrows[0] * spr[0]; base += NT) {
                int32_t q, x;
                if (!site_of(0, base + threadIdx.x, q, x)) continue;
                HotDraws D;
                int32_t cn[4];
                draw_site(C0, q, x, D, cn);
                update(C0, q, x, D, cn);
            }
            __syncthreads();
            for (int base = 0; base < nrows[1] * spr[1]; base += NT) {
                int32_t q, x;
                if (!site_of(1, base + threadIdx.x, q, x)) continue;
                HotDraws D;
                int32_t cn[4];
                draw_site(C1, q, x, D, cn);
                update(C1, q, x, D, cn);
            }
            __syncthreads();
        }

        // the sweep's statistics (per wave into the workgroup's slot j; added to the sweep's sv_stats at the end)
        {
            unsigned long long w[4];
            w[0] = (unsigned long long)acc_count;
            fx_limbs(psum, w[1], w[2], w[3]);
            for (int o = 32; o > 0; o >>= 1)
                for (int i = 0; i < 4; i++) w[i] += __shfl_xor(w[i], o);
            if ((threadIdx.x & 63) == 0)
                for (int i = 0; i < 4; i++)
                    if (w[i]) atomicAdd(&s_acc[4 * j + i], w[i]);
        }
        // the own block into the sweep's output buffer
        {
            double *phi_out = B.phi[j + 1];
            int64_t *n_out = B.n[j + 1];
            for (int idx = threadIdx.x; idx < bs * bs; idx += NT) {
                const int i = idx / bs, k = idx - i * bs;
                const int s0 = (r0 + i - FR0) * F + (c0 + k - FC0);
                const int64_t g = (int64_t)(r0 + i) * N + (c0 + k);
                // write-through (global_store sc1): no dirty L2 lines for the launch's end to write back (L=256:
                // 7.72 -> 7.56 us per sweep, r5)
                __hip_atomic_store(&phi_out[g], s_phi[s0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(&n_out[g], (int64_t)s_n0[s0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(&n_out[V + g], (int64_t)s_n1[s0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        BLK_T(3 + j);
        // the next sweep's row bases: one sweep's stream length further on
        if (j + 1 < K) {
            for (int idx = threadIdx.x; idx < (F - 2) * nset * 12; idx += NT) {
                const int i = 1 + idx / (nset * 12), rem = idx % (nset * 12);
                u128 &b = s_base[(i * 2 + rem / 12) * 12 + rem % 12];
                b = apply(B.step, b);
            }
        }
    }
    __syncthreads();
    if (*s_bad && threadIdx.x == 0) report(A.S, A.sweep, OVERFLOW_BLOCK, 0);
    if ((int)threadIdx.x < 4 * K && s_acc[threadIdx.x])
        atomicAdd(stat_word(&A.stat[threadIdx.x >> 2], threadIdx.x & 3), s_acc[threadIdx.x]);
    BLK_T(15);
}
template __global__ void villain_sweep_block<8>(FArgs, BlockArgs);
template __global__ void villain_sweep_block<16>(FArgs, BlockArgs);

}  // namespace sv

#if SV_BLKTIME
extern "C" int sv_debug_blocktime(uint64_t *out, int32_t n) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(sv::g_blktime), (size_t)n * sv::BLT * sizeof(uint64_t)) == hipSuccess ? 0 : -2;
}
#endif

namespace svh {

void launch_block(const FArgs &A, const BlockArgs &B, hipStream_t stream) {
    const int F = block_frame(B.bs, B.K);
    const size_t lds = block_lds_bytes(F);
    static bool attr = [] {
        return hipFuncSetAttribute((const void *)villain_sweep_block<8>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                   160 * 1024) == hipSuccess &&
               hipFuncSetAttribute((const void *)villain_sweep_block<16>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                   160 * 1024) == hipSuccess;
    }();
    (void)attr;
    // 16 waves when the first colour pass has more sites than 8 waves have lanes (F - 2 rows of (F - 1) / 2)
    const bool w16 = (F - 2) * ((F - 1) / 2) > 8 * 64;
    if (w16) villain_sweep_block<16><<<B.nbx * B.nbx, 16 * 64, lds, stream>>>(A, B), SV_LAUNCHED("villain_sweep_block<16>", stream);
    else villain_sweep_block<8><<<B.nbx * B.nbx, 8 * 64, lds, stream>>>(A, B), SV_LAUNCHED("villain_sweep_block<8>", stream);
}

}  // namespace svh
