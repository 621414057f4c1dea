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
    const int by = (int)blockIdx.x / B.nbx, bx = (int)blockIdx.x - by * B.nbx;
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
    double *s_ps = reinterpret_cast<double *>(s_acc + 16);
    int32_t *s_bad = reinterpret_cast<int32_t *>(s_ps + 16);

    for (int e = threadIdx.x; e < SMALL_LDS; e += NT) {
        s_small.A[e] = A.T->small[e].A;
        s_small.C[e] = A.T->small[e].C;
    }
    if (threadIdx.x < 16) {
        s_acc[threadIdx.x] = 0;
        s_ps[threadIdx.x] = 0.0;
    }
    if (threadIdx.x == 0) *s_bad = 0;

    // the frame from the launch's input, wrapped onto the torus (F <= N: no site twice)
    {
        uint32_t bad = 0;
        for (int idx = threadIdx.x; idx < F * F; idx += NT) {
            const int i = idx / F, k = idx - i * F;
            const int64_t g = (int64_t)wrapN(FR0 + i, N) * N + wrapN(FC0 + k, N);
            // the +0.0 every site receives once per sweep (neighborhood.py:128), applied once: an accepted change is
            // added to the normalised value, which stays normalised (villain_hot.hip's commit)
            s_phi[idx] = B.phi[0][g] + 0.0;
            const int64_t a = B.n[0][g], c = B.n[0][V + g];
            // the int32 image holds n exactly with room for K sweeps of changes (|W| interval_n <= 2^13: hot_params_ok)
            bad |= (uint32_t)((uint64_t)((a >> 30) + 1) > 1) | (uint32_t)((uint64_t)((c >> 30) + 1) > 1);
            s_n0[idx] = (int32_t)a;
            s_n1[idx] = (int32_t)c;
        }
        if (bad) *s_bad = 1;
    }
#if SV_BLKTIME
    __syncthreads();
    BLK_T(1);
#endif

    // row bases of sweep 0 for frame rows 1 .. F-2 (the rows a colour pass decides): set 0 at column xb (the frame's
    // first column on the torus), set 1 at column 0 for the columns that wrap; per colour the six blocks in
    // hot_draws_edge's order (metropolis, dphi, the four choice blocks)
    const int32_t xb = wrapN(FC0, N);
    const bool wraps = FC0 < 0 || FC0 + F > N;
    const int nset = wraps ? 2 : 1;
    for (int idx = threadIdx.x; idx < (F - 2) * nset * 12; idx += NT) {
        const int i = 1 + idx / (nset * 12), rem = idx % (nset * 12), s = rem / 12, slot = rem % 12;
        const int c = slot / 6, ty = slot % 6;
        const int blk = ty == 0 ? 0 : 1 + 5 * c + ty - 1;
        const uint32_t has = ty >= 2 ? A.blocks[blk].has : 0u;
        s_base[(i * 2 + s) * 12 + slot] =
            full_jump(A.T, &A.blocks[blk], (uint32_t)base_pos(ty, wrapN(FR0 + i, N), N, s ? 0 : xb, has));
    }

    const VParams P = A.P;
    const uint32_t kc = P.k, thr = P.thr;
    const int32_t Wn = (int32_t)P.W, nW = (int32_t)(P.W * P.interval_n);
    const double hk = P.half_kappa;
    // lanes per frame row in a colour pass: a power of two >= the colour's sites in the widest row (F - 2 columns)
    int lg = 0;
    while ((1 << lg) < (F - 1) / 2) lg++;

    for (int j = 0; j < K; j++) {
        const int e = E - j;
        const int32_t ra = r0 - 2 * e, rb = r0 + bs + 3 * e, ca = c0 - 2 * e, cb = c0 + bs + 3 * e;
        const Block *blocks = A.blocks + (int64_t)j * B.nb;
        const uint32_t sweep_id = A.sweep + (uint32_t)j;
        uint32_t has4[2][4], buf4[2][4];
#pragma unroll
        for (int c = 0; c < 2; c++)
#pragma unroll
            for (int q = 0; q < 4; q++) {
                has4[c][q] = (uint32_t)__builtin_amdgcn_readfirstlane(blocks[2 + 5 * c + q].has);
                buf4[c][q] = (uint32_t)__builtin_amdgcn_readfirstlane(blocks[2 + 5 * c + q].buf);
            }
        __syncthreads();  // (the frame and the bases; the previous sweep's stores and advance)
        if (j == 0) BLK_T(2);
        int32_t acc_count = 0;
        double psum = 0.0;

        // colour c on rows qlo..qhi and columns xlo..xhi (inclusive): villain_sweep_hot's ranges around the decided
        // region [ra, rb) x [ca, cb) -- colour 0 one row / column further on every side, colour 1 one further below
        // and right (the links stored at the region's last row / column)
        auto pass = [&](auto C, int32_t qlo, int32_t qhi, int32_t xlo, int32_t xhi) {
            constexpr int c = decltype(C)::value;
            const int nrows = qhi - qlo + 1;
            for (int base = 0; base < (nrows << lg); base += NT) {
                const int idx = base + (int)threadIdx.x;
                const int row = idx >> lg, k = idx & ((1 << lg) - 1);
                const int32_t q = qlo + row;
                const int32_t x = xlo + ((q + xlo + c) & 1) + 2 * k;  // colour c: q + x = c mod 2
                if (row >= nrows || x > xhi) continue;
                const int lq = q - FR0, lx = x - FC0, s0 = lq * F + lx;
                const int32_t gq = wrapN(q, N), gx = wrapN(x, N);
                const HotDraws D = hot_draws_edge(A, gq, gx, xb, 0, &s_base[(lq * 2) * 12 + 6 * c],
                                                  &s_base[(lq * 2 + 1) * 12 + 6 * c], s_small, has4[c], buf4[c]);
                int32_t cn[4];
                bool rej = false;
#pragma unroll
                for (int jj = 0; jj < 4; jj++) {
                    const uint64_t m = (uint64_t)D.w[jj] * kc;
                    rej |= (uint32_t)m < thr;
                    cn[jj] = (int32_t)(m >> 32) * Wn - nW;  // W * (index - interval_n), neighborhood.py:105-107
                }
                if (__builtin_expect(rej, 0)) {
                    const uint32_t rank = (uint32_t)(((int64_t)gq * N + gx) >> 1);
#pragma unroll
                    for (int jj = 0; jj < 4; jj++)
                        if ((uint32_t)((uint64_t)D.w[jj] * kc) < thr) report(A.S, sweep_id, (uint32_t)(1 + 5 * c + 1 + jj), rank);
                }
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
                        psum += p;
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
                        psum += p;
                    }
                    if (acc) {
                        s_phi[s0] = s_phi[s0] + D.dphi;
                        s_n0[s0] += cn[0];
                        s_n0[s0 - F] += cn[1];
                        s_n1[s0] += cn[2];
                        s_n1[s0 - 1] += cn[3];
                    }
                }
            }
        };
        pass(std::integral_constant<int, 0>{}, ra - 1, rb + 1, ca - 1, cb + 1);
        __syncthreads();
        pass(std::integral_constant<int, 1>{}, ra, rb, ca, cb);
        __syncthreads();

        // the sweep's statistics (per wave into the workgroup's slot j; added to the sweep's sv_stats at the end)
        {
            unsigned long long a = (unsigned long long)acc_count;
            for (int o = 32; o > 0; o >>= 1) a += __shfl_xor(a, o);
            const double ps = wave_sum(psum);
            if ((threadIdx.x & 63) == 0 && (a || ps != 0.0)) {
                atomicAdd(&s_acc[j], a);
                atomicAdd(&s_ps[j], ps);
            }
        }
        // the own block into the sweep's output buffer
        {
            double *phi_out = B.phi[j + 1];
            int64_t *n_out = B.n[j + 1];
            for (int idx = threadIdx.x; idx < bs * bs; idx += NT) {
                const int i = idx / bs, k = idx - i * bs;
                const int s0 = (r0 + i - FR0) * F + (c0 + k - FC0);
                const int64_t g = (int64_t)(r0 + i) * N + (c0 + k);
                phi_out[g] = s_phi[s0];
                n_out[g] = (int64_t)s_n0[s0];
                n_out[V + g] = (int64_t)s_n1[s0];
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
    if ((int)threadIdx.x < K && (s_acc[threadIdx.x] || s_ps[threadIdx.x] != 0.0)) {
        atomicAdd((unsigned long long *)&A.stat[threadIdx.x].accepted, s_acc[threadIdx.x]);
        unsafeAtomicAdd(&A.stat[threadIdx.x].acceptance_sum, s_ps[threadIdx.x]);
    }
    BLK_T(15);
}
template __global__ void villain_sweep_block<8>(FArgs, BlockArgs);

}  // namespace sv

#if SV_BLKTIME
extern "C" int sv_debug_blocktime(uint64_t *out, int32_t n) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(sv::g_blktime), (size_t)n * sv::BLT * sizeof(uint64_t)) == hipSuccess ? 0 : -2;
}
#endif

namespace svh {

void launch_block(const FArgs &A, const BlockArgs &B, hipStream_t stream) {
    const size_t lds = block_lds_bytes(block_frame(B.bs, B.K));
    static bool attr = [] {
        return hipFuncSetAttribute((const void *)villain_sweep_block<8>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                   160 * 1024) == hipSuccess;
    }();
    (void)attr;
    villain_sweep_block<8><<<B.nbx * B.nbx, 8 * 64, lds, stream>>>(A, B);
}

}  // namespace svh
