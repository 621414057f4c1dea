// villain.hip -- NeighborhoodUpdate (supervillain/generator/villain/neighborhood.py:59-137) on gfx950.
//
// Two device paths, both bit-exact replays of the reference chain under a fixed NumPy seed:
//
//  * generic (any N, incl. odd N's four colours): one kernel per colour pass, the residual
//    r = d(phi) - 2 pi n kept in HBM and updated incrementally exactly as neighborhood.py:129 does.
//
//  * fused (even N): ONE kernel per sweep.  A workgroup owns a column strip of <=125 columns and
//    TH rows and streams down it with a ring of LDS rows: colour-0 decisions for rows t+2.., then
//    colour-1 decisions for rows t+1.. (reading the colour-0 results, including the incrementally
//    updated r, from LDS), then writes finished rows t.. .  Halo decisions (one row/column of
//    colour-1 and two of colour-0 beyond the strip) are recomputed redundantly -- every draw is
//    addressed by its global NumPy stream position, so neighbouring strips agree bit-for-bit.
//    HBM traffic is one read and one write of (phi, n) per sweep: 48 B/site instead of the
//    88 B/site of two colour passes.
//
// Floating point follows the reference op by op (compile with -ffp-contract=off):
//   d(phi) on link (mu,x):   0.0 + (phi[x+e] - phi[x])                 (lattice/reference.py:9-24)
//   change_r:               (0.0 + (cphi[x+e] - cphi[x])) - (2pi)*cn   (neighborhood.py:110)
//   dS_link:                ((kappa/2) * cr) * ((2*r) + cr)            (neighborhood.py:111)
//   face_sum:               (((0 + f0[x]) + f0[x-e0]) + f1[x]) + f1[x-e1]  (reference.py:48-64)
//   r update:               (r + d(cphi)) - (2pi)*cn                  (neighborhood.py:129)
#include <array>
#include <atomic>
#include <thread>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "fused.h"

namespace sv {

// ================================================================================================
// generic path
// ================================================================================================

// r = d(phi) - 2 pi n at sweep start (neighborhood.py:91); also phi <- phi + 0.0 (see DESIGN.md:
// every site receives `phi + change_phi` with change_phi = +0.0 in some colour pass).
__global__ void villain_r_init(int32_t N, double *phi, const int64_t *n, double *r, const int32_t *abort) {
    if (*(volatile const int32_t *)abort) return;
    int64_t V = (int64_t)N * N;
    for (int64_t s = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; s < V; s += (int64_t)gridDim.x * blockDim.x) {
        int64_t t = s / N, x = s - t * N;
        int64_t f0 = ((t + 1 == N) ? 0 : t + 1) * N + x;
        int64_t f1 = t * N + ((x + 1 == N) ? 0 : x + 1);
        double p = phi[s];
        r[s] = (0.0 + (phi[f0] - p)) - TWO_PI * (double)n[s];
        r[V + s] = (0.0 + (phi[f1] - p)) - TWO_PI * (double)n[V + s];
    }
}

__global__ void villain_phi_normalize(int32_t N, double *phi, const int32_t *abort) {
    if (*(volatile const int32_t *)abort) return;
    int64_t V = (int64_t)N * N;
    for (int64_t s = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; s < V; s += (int64_t)gridDim.x * blockDim.x)
        phi[s] = phi[s] + 0.0;
}

__global__ __launch_bounds__(256) void villain_pass_generic(VParams P, double *phi, int64_t *n, double *r,
                                                            const int32_t *sites, int64_t nc, int color,
                                                            const Block *blocks, const uint32_t *skips,
                                                            const JumpTables *T, sv_stats *stat, DevScratch S,
                                                            uint32_t sweep) {
    if (*(volatile const int32_t *)S.abort) return;
    const int64_t N = P.N, V = N * N;
    int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    int64_t acc_count = 0;
    AccFx psum;  // exact acceptance sum (common.h)
    if (i < nc) {
        const int64_t s = sites[i];
        const int64_t t = s / N, x = s - t * N;
        const int64_t b0s = ((t == 0) ? N - 1 : t - 1) * N + x;  // x - e0
        const int64_t b1s = t * N + ((x == 0) ? N - 1 : x - 1);  // x - e1
        const Block &BM = blocks[0];
        const int bb = 1 + 5 * color;
        const double u = 0.0 + 1.0 * to_double(xsl_rr(jump(T, block_base(BM), (uint32_t)s)));
        const double dphi = P.lo_phi + P.range_phi * to_double(xsl_rr(jump(T, block_base(blocks[bb]), (uint32_t)i)));
        int64_t cn[4] = {0, 0, 0, 0};  // f0, b0, f1, b1
        if (P.k > 1) {
#pragma unroll
            for (int q = 0; q < 4; q++)
                cn[q] = bounded_draw(T, blocks[bb + 1 + q], skips, (uint32_t)i, P, S, sweep, (uint32_t)(bb + 1 + q));
        }
        const int64_t L[4] = {s, b0s, V + s, V + b1s};
        double rr[4], cr[4];
#pragma unroll
        for (int q = 0; q < 4; q++) rr[q] = r[L[q]];
        cr[0] = (0.0 + (0.0 - dphi)) - TWO_PI * (double)cn[0];
        cr[1] = (0.0 + (dphi - 0.0)) - TWO_PI * (double)cn[1];
        cr[2] = (0.0 + (0.0 - dphi)) - TWO_PI * (double)cn[2];
        cr[3] = (0.0 + (dphi - 0.0)) - TWO_PI * (double)cn[3];
        double dS = 0.0;
#pragma unroll
        for (int q = 0; q < 4; q++) {
            double a = P.half_kappa * cr[q];
            double b = (2.0 * rr[q]) + cr[q];
            dS += a * b;
        }
        double p = exp(-dS);
        p = p < 0.0 ? 0.0 : p;
        p = p > 1.0 ? 1.0 : p;
        const int acc = u < p;
        acc_count = acc;
        fx_add(psum, p);
        const double cphi = dphi * (double)acc;
        phi[s] = phi[s] + cphi;
        const double dcp_f = 0.0 + (0.0 - cphi);
        const double dcp_b = 0.0 + (cphi - 0.0);
#pragma unroll
        for (int q = 0; q < 4; q++) {
            int64_t c = cn[q] * acc;
            n[L[q]] = n[L[q]] + c;
            r[L[q]] = (rr[q] + ((q & 1) ? dcp_b : dcp_f)) - TWO_PI * (double)c;
        }
    }
    flush_stats(stat, acc_count, psum);
}

// ================================================================================================
// fused path (even N)
// ================================================================================================



// FR (full rows, periodic lattices of Nx <= 128): one strip spans the whole row, its LDS columns ARE
// the lattice columns and neighbours wrap inside LDS -- no column halo, every lane busy at N = 128.
template <int NW, bool TILE, bool REPS, bool OBS, bool FR>
__device__ __forceinline__ void sweep_body(const FArgs &A) {
    static_assert(!(FR && TILE), "full-row strips are for periodic lattices");
    constexpr int R = FusedGeom<NW>::R;
    constexpr int nthreads = NW * 64;
    constexpr int PF = RW / 64;  // region columns per lane (each wave moves whole rows)
    __shared__ double s_phi[R][RW];
    __shared__ double s_r0[R][RW];
    __shared__ double s_r1[R][RW];
    __shared__ int32_t s_n0[R][RW];
    __shared__ int32_t s_n1[R][RW];
    __shared__ SmallTab s_small;
    __shared__ Affine s_adv[3];
    __shared__ u128 s_base[NW][32];  // per wave: [8c + ty] = block ty's base for the colour-c row; [16 + ..] at xw
    __shared__ int32_t s_bad;
    __shared__ unsigned long long s_obsw[5];  // OBS: the workgroup's exact observable words (common.h)
    __shared__ double s_obig;                 // OBS: its action terms t >= ACT_LIMIT
    __shared__ Block s_blk[11];  // this sweep's descriptors (LDS: no vector-memory waits in the loop)

    note_progress(A);
    if (sweep_cancelled(A.S, A.sweep)) return;

    const FGeom &Gm = A.G;
    const int32_t Nt = Gm.Nt, Nx = Gm.Nx;
    // the wave index is uniform: keep it (and all row / ring-slot arithmetic derived from it) scalar
    const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)), lane = threadIdx.x & 63;
    const int64_t V = Gm.plane;
    // global row of local row q; memory offset of local row q / local column c
    auto grow = [&](int32_t q) { return wrapN(Gm.T0 + q, Nt); };
    auto mrow = [&](int32_t q) -> int64_t { return TILE ? Gm.org + (int64_t)q * Gm.pitch : (int64_t)wrapN(q, Nt) * Nx; };
    auto mcol = [&](int32_t c) -> int32_t { return TILE ? c : wrapN(c, Nx); };
    const int32_t par0 = (Gm.T0 + Gm.X0) & 1;  // colour parity offset of local coordinates

    // XCD-aware tile order: blocks b, b+8, ... share an XCD; give each XCD a contiguous run of tiles
    const int G = gridDim.x;
    int b = blockIdx.x;
    {
        const int per = G / 8, rem = G % 8;
        const int xcd = b & 7, k = b >> 3;
        b = xcd * per + (xcd < rem ? xcd : rem) + k;
    }
    // domain tiles: the launch covers a subset of the strips (interior ones while the halos travel)
    // replica of this workgroup (replica batches; 0 otherwise)
    const int slot = REPS ? __builtin_amdgcn_readfirstlane(b / A.tiles_per_rep) : 0;  // uniform: keep it scalar
    if (REPS) b = __builtin_amdgcn_readfirstlane(b - slot * A.tiles_per_rep);
    const int rep = REPS && A.rep_map ? __builtin_amdgcn_readfirstlane(A.rep_map[slot]) : slot;
    const Rep RP{REPS ? A.blocks + (int64_t)rep * A.rep_blocks : A.blocks, REPS ? A.Trep[rep] : A.T, (uint32_t)rep};
    const double *phi_in = REPS ? A.phi_in + rep * A.rep_field : A.phi_in;
    const int64_t *n_in = REPS ? A.n_in + 2 * rep * A.rep_field : A.n_in;
    double *phi_out = REPS ? A.phi_out + rep * A.rep_field : A.phi_out;
    int64_t *n_out = REPS ? A.n_out + 2 * rep * A.rep_field : A.n_out;
    const int ix = b % A.nsx, iy = b / A.nsx;
    const int32_t x0 = (int32_t)((int64_t)ix * Gm.Wt / A.nsx), x1 = (int32_t)((int64_t)(ix + 1) * Gm.Wt / A.nsx);
    const int32_t w = x1 - x0;
    const int32_t t0 = iy * A.TH;
    const int32_t t1 = t0 + A.TH < Gm.Ht ? t0 + A.TH : Gm.Ht;
    const int32_t rbase = t0 - 2;  // local row 0
    const int32_t cols = FR ? w : w + 5;
    const int32_t cofs = FR ? 0 : x0 - 2;  // LDS column of local column x is x - cofs
    // LDS neighbour columns (full rows wrap inside the row)
    auto cxp = [&](int cx) { return FR ? (cx + 1 == w ? 0 : cx + 1) : cx + 1; };
    auto cxm = [&](int cx) { return FR ? (cx == 0 ? w - 1 : cx - 1) : cx - 1; };
    // global column origin of this strip (its first column wrapped onto the torus: deep-halo regions start
    // anywhere), and the sites it counts in the statistics (its own, within the launch's owned window)
    const int32_t X0s = TILE ? wrapN(Gm.X0 + x0, Nx) - x0 : Gm.X0;
    const int32_t q_lo = TILE && A.own_r0 > t0 ? A.own_r0 : t0, q_hi = TILE && A.own_r1 < t1 ? A.own_r1 : t1;
    const int32_t c_lo = TILE && A.own_c0 > x0 ? A.own_c0 : x0, c_hi = TILE && A.own_c1 < x1 ? A.own_c1 : x1;
    const int32_t gx0 = X0s + x0;                    // global column of the strip's first site
    const bool interior = !FR && gx0 >= 4 && gx0 + w + 2 < Nx;
    // row bases at the first non-wrapped region column (global); on rows of <= 128 sites at the row
    // start, so that every column -- wrapped halo columns included -- is a small-table offset away
    const int32_t xb = ((Nx <= SMALL_LDS && !interior) || gx0 - 2 < 0) ? 0 : gx0 - 2;
    // edge strips of longer rows: a second set of row bases at the first wrapped global column xw
    const bool edge = !(Nx <= SMALL_LDS && !interior) && (gx0 - 2 < 0 || gx0 + w + 2 >= Nx);
    const int32_t xw = gx0 - 2 < 0 ? Nx - 2 : 0;

    for (int e = threadIdx.x; e < SMALL_LDS; e += nthreads) {
        s_small.A[e] = RP.T->small[e].A;
        s_small.C[e] = RP.T->small[e].C;
    }
    if (threadIdx.x < 11) s_blk[threadIdx.x] = RP.blocks[threadIdx.x];
    const Rep RL{s_blk, RP.T, RP.id};  // the loop's view (valid after the prologue barrier)
    if (threadIdx.x < 3) s_adv[threadIdx.x] = REPS ? A.advrep[3 * rep + threadIdx.x] : A.adv[threadIdx.x];
    if (threadIdx.x == 0) s_bad = 0;
    if (OBS && threadIdx.x < 5) s_obsw[threadIdx.x] = 0;
    if (OBS && threadIdx.x == 5) s_obig = 0.0;

    // the buffered-half flags of the fwd choice blocks (mu = 0, 1) per colour, kept in SGPRs: reading
    // them from the descriptors inside the loop would put a vmcnt(0) wait behind the row prefetch
    const uint32_t has_c0[2] = {(uint32_t)__builtin_amdgcn_readfirstlane(RP.blocks[2].has),
                                (uint32_t)__builtin_amdgcn_readfirstlane(RP.blocks[4].has)};
    const uint32_t has_c1[2] = {(uint32_t)__builtin_amdgcn_readfirstlane(RP.blocks[7].has),
                                (uint32_t)__builtin_amdgcn_readfirstlane(RP.blocks[9].has)};
    // fast draws need, per colour, no skips and equal buffers within each fwd/bwd pair
    bool fast[2], fastfr[2];
#pragma unroll
    for (int c = 0; c < 2; c++) {
        const Block *B = &RP.blocks[2 + 5 * c];
        fast[c] = interior && B[0].nskip == 0 && B[1].nskip == 0 && B[2].nskip == 0 && B[3].nskip == 0 &&
                  B[0].has == B[1].has && B[2].has == B[3].has;
        // full-row strips (replica batches of N <= 128): every lane is busy, so the lane pairs that share a
        // choice word must not straddle the row -- true when the fwd/bwd blocks start on a whole word
        // (has == 0), which is the norm (each block draws an even V/2 half-words)
        fastfr[c] = FR && B[0].nskip == 0 && B[1].nskip == 0 && B[2].nskip == 0 && B[3].nskip == 0 &&
                    B[0].has == 0 && B[1].has == 0 && B[2].has == 0 && B[3].has == 0;
    }

    // ---- register prefetch of region rows [ra, ra+NW) (clipped to [t0-2, t1+2]): wave w moves row
    // ra + w, lane l columns l and l + 64 (row index math is uniform per wave)
    double pf_phi[PF];
    int64_t pf_n0[PF], pf_n1[PF];
    int pf_gx[PF];
#pragma unroll
    for (int k = 0; k < PF; k++) pf_gx[k] = FR ? lane + 64 * k : mcol(x0 - 2 + lane + 64 * k);
    auto prefetch = [&](int32_t ra) {
        const int32_t q = ra + wave;
        if (q >= t0 - 2 && q <= t1 + 2) {
            const int64_t g0 = mrow(q);
#pragma unroll
            for (int k = 0; k < PF; k++) {
                if (lane + 64 * k < cols) {
                    const int64_t g = g0 + pf_gx[k];
#if SV_ABLATE & 16
                    pf_phi[k] = (double)(g & 7);
                    pf_n0[k] = 0;
                    pf_n1[k] = 0;
#else
                    pf_phi[k] = phi_in[g];
                    pf_n0[k] = n_in[g];
                    pf_n1[k] = n_in[V + g];
#endif
                }
            }
        }
    };
    auto commit = [&](int32_t ra) {
        const int32_t q = ra + wave;
        if (q >= t0 - 2 && q <= t1 + 2) {
            const int slot = (q - rbase) % R;
#pragma unroll
            for (int k = 0; k < PF; k++) {
                const int cc = lane + 64 * k;
                if (cc < cols) {
                    s_phi[slot][cc] = pf_phi[k];
                    const int64_t a = pf_n0[k], c = pf_n1[k];
                    if (a > (1LL << 30) || a < -(1LL << 30) || c > (1LL << 30) || c < -(1LL << 30)) s_bad = 1;
                    s_n0[slot][cc] = (int32_t)a;
                    s_n1[slot][cc] = (int32_t)c;
                }
            }
        }
    };

    // ---- per-wave running row bases: lane 8c+ty holds block ty's base for this wave's colour-c row
    // (at column xb); lanes 16 + 8c + ty the same at column xw (edge strips only)
    const bool base_lane = (lane & 7) < 6 && (lane < 16 || (edge && lane < 32));
    const int bc = (lane >> 3) & 1, bty = lane & 7;
    const int32_t bx = lane >= 16 ? xw : xb;
    const int bblk = bty == 0 ? 0 : 1 + 5 * bc + bty - 1;
    const uint32_t bhas = (base_lane && bty >= 2) ? RP.blocks[bblk].has : 0u;
    const int32_t tfirst = t0 - 3;
    int32_t brow = tfirst + 2 - bc + wave;  // D0 row t+2+wave, D1 row t+1+wave
    u128 bases{0, 0};
    if (base_lane) bases = full_jump(RP.T, &RP.blocks[bblk], (uint32_t)base_pos(bty, grow(brow), Nx, bx, bhas));
    __builtin_amdgcn_s_waitcnt(0);
    if (base_lane) s_base[wave][lane] = bases;

    // fast-draw lane constants per colour (valid for every row of this wave, see fast_pack)
    uint32_t pk0 = 0, pk1 = 0;
    if (fast[0]) {
        const int32_t q = tfirst + 2 + wave;
        const int32_t xs = (x0 - 1) + ((par0 + q + x0 - 1) & 1);
        pk0 = fast_pack(has_c0, lane, (uint32_t)grow(q) * (uint32_t)Nx, (uint32_t)(X0s + xs),
                        (uint32_t)(X0s + xs + 2 * lane), (uint32_t)xb);
    }
    if (fast[1]) {
        const int32_t q = tfirst + 1 + wave;
        const int32_t xs = x0 + ((par0 + q + x0 + 1) & 1);
        pk1 = fast_pack(has_c1, lane, (uint32_t)grow(q) * (uint32_t)Nx, (uint32_t)(X0s + xs),
                        (uint32_t)(X0s + xs + 2 * lane), (uint32_t)xb);
    }

    int64_t acc_count = 0;
    AccFx psum;  // exact acceptance sum (common.h)

    // coalesced stores of finished rows [ra, ra+NW) (clipped to the tile) from the ring: wave w
    // stores row ra + w, lane l columns l and l + 64
    auto store_rows = [&](int32_t ra) {
        const int32_t q = ra + wave;
        unsigned long long o_act = 0, o_w2 = 0;  // OBS partials: exact action values (common.h), integer sums
        int64_t o_n0 = 0, o_n1 = 0;
        if (q >= t0 && q < t1) {
            const int slot = (q - rbase) % R;
            const int64_t g0 = mrow(q) + x0;  // tile sites never wrap
#pragma unroll
            for (int k = 0; k < PF; k++) {
                const int cc = lane + 64 * k;
                if (cc < w) {
                    const int cx = FR ? cc : cc + 2;
                    const int64_t g = g0 + cc;
#if !(SV_ABLATE & 8)
                    phi_out[g] = s_phi[slot][cx];
                    n_out[g] = (int64_t)s_n0[slot][cx];
                    n_out[V + g] = (int64_t)s_n1[slot][cx];
#endif
                    if (OBS) {
                        // rows <= q+1 and columns <= x+1 are final here (villain.py:51-66, winding.py:30-37,
                        // wrapping.py:17-25): link residuals, plaquette winding dn, holonomy sums
                        const int slot1 = (q + 1 - rbase) % R;
                        const double ph = s_phi[slot][cx];
                        const double l0 = (0.0 + (s_phi[slot1][cx] - ph)) - TWO_PI * (double)s_n0[slot][cx];
                        const double l1 = (0.0 + (s_phi[slot][cxp(cx)] - ph)) - TWO_PI * (double)s_n1[slot][cx];
                        const double t = l0 * l0 + l1 * l1;
                        if (t < ACT_LIMIT) o_act += act_fx(t);
                        else atomicAdd(&s_obig, t);
                        const int64_t dn = ((int64_t)s_n1[slot1][cx] - s_n1[slot][cx]) -
                                           ((int64_t)s_n0[slot][cxp(cx)] - s_n0[slot][cx]);
                        o_w2 += (unsigned long long)(dn * dn);
                        o_n0 += s_n0[slot][cx];
                        o_n1 += s_n1[slot][cx];
                    }
                }
            }
        }
        if (OBS) {
            // integer sums (a row's action values < 2^59): the same words in any order (common.h)
            unsigned long long w[4] = {o_act, o_w2, (unsigned long long)o_n0, (unsigned long long)o_n1};
            for (int o = 32; o > 0; o >>= 1)
                for (int i = 0; i < 4; i++) w[i] += __shfl_xor(w[i], o);
            if (lane == 0) {
                atomicAdd(&s_obsw[0], w[0] & 0xffffffffull);
                atomicAdd(&s_obsw[1], w[0] >> 32);
                atomicAdd(&s_obsw[2], w[1]);
                atomicAdd(&s_obsw[3], w[2]);
                atomicAdd(&s_obsw[4], w[3]);
            }
        }
    };

    for (int32_t ra = t0 - 2; ra < tfirst + 3 + NW; ra += NW) {
        prefetch(ra);
        commit(ra);
    }
    __syncthreads();

    for (int32_t t = tfirst; t < t1; t += NW) {
        prefetch(t + 3 + NW);  // rows for the next step; committed during phase C
        store_rows(t - NW);    // rows finished by the previous step (their slots are recycled in phase C)
        // ---------------- phase B: colour-0 decisions on row q = t+2+wave (+ stores of rows t-NW..t-1)
        {
            const int32_t q = t + 2 + wave;
            const bool row_ok = (q >= t0 - 1) && (q <= t1 + 1);
            const int32_t gq = grow(q);
            const int32_t xs = FR ? ((par0 + q) & 1) : (x0 - 1) + ((par0 + q + x0 - 1) & 1);  // global (t + x) even
            const int32_t x = xs + 2 * lane;
            const bool active = row_ok && (FR ? x < w : x <= x1 + 1);
            u128 bs[6];
#pragma unroll
            for (int k = 0; k < 6; k++) bs[k] = s_base[wave][k];
            Draws D;
            if (fast[0])
                D = draws_fastp(A, RL, 0, active, lane, pk0, ((uint32_t)gq * (uint32_t)Nx + (uint32_t)(X0s + x)) >> 1,
                                bs, s_small);
            else if (fastfr[0])
                D = draws_fast(A, RL, 0, has_c0, active, lane, (uint32_t)gq * (uint32_t)Nx, (uint32_t)xs, (uint32_t)x, 0u,
                               bs, s_small);
            else
                D = draws_general(A, RL, 0, active, gq, wrapN(X0s + x, Nx), xb, bs, s_small, edge, xw,
                                  &s_base[wave][16]);
            if (active) {
                const int lr = q - rbase;
                const int sm = (lr - 1) % R, s0 = lr % R, sp = (lr + 1) % R;
                const int cx = x - cofs, cp = cxp(cx), cm = cxm(cx);
                const double ph = s_phi[s0][cx];
                // r0 on the four links: f0=(0,q,x), b0=(0,q-1,x), f1=(1,q,x), b1=(1,q,x-1)
                const int32_t n_f0 = s_n0[s0][cx], n_b0 = s_n0[sm][cx], n_f1 = s_n1[s0][cx], n_b1 = s_n1[s0][cm];
                // r and change_r feed nothing but dS, and dS nothing but exp(-dS) (exp(+-0) = 1): the
                // reference's `0.0 +` of d() (lattice/reference.py:9-24) only normalizes a -0.0, so it is
                // dropped here; (0 - dphi) and dphi are never -0.0 (dphi = -pi + 2 pi u), so change_r is
                // bit-identical anyway
                double r0[4];
                r0[0] = (s_phi[sp][cx] - ph) - TWO_PI * (double)n_f0;
                r0[1] = (ph - s_phi[sm][cx]) - TWO_PI * (double)n_b0;
                r0[2] = (s_phi[s0][cp] - ph) - TWO_PI * (double)n_f1;
                r0[3] = (ph - s_phi[s0][cm]) - TWO_PI * (double)n_b1;
                double cr[4];
                cr[0] = (0.0 - D.dphi) - TWO_PI * (double)D.cn[0];
                cr[1] = D.dphi - TWO_PI * (double)D.cn[1];
                cr[2] = (0.0 - D.dphi) - TWO_PI * (double)D.cn[2];
                cr[3] = D.dphi - TWO_PI * (double)D.cn[3];
                double dS = 0.0;
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    const double a = A.P.half_kappa * cr[k];
                    const double bb2 = (2.0 * r0[k]) + cr[k];
                    dS += a * bb2;
                }
                double p = sv_exp(-dS);
                p = p < 0.0 ? 0.0 : p;
                p = p > 1.0 ? 1.0 : p;
                const int acc = D.u < p;
                const bool own = q >= q_lo && q < q_hi && (FR || (x >= c_lo && x < c_hi));
                if (own) {  // count each site once; colour-0 phi is final after this pass
                    acc_count += acc;
                    fx_add(psum, p);
                }
                const double cphi = D.dphi * (double)acc;
                s_phi[s0][cx] = (ph + cphi) + 0.0;  // final colour-0 phi (the colour-1 pass adds +0.0)
                const double dcp_f = 0.0 - cphi;  // d(change_phi) up to the sign of a zero (see above)
                const double dcp_b = cphi;
                const int32_t c0 = acc ? D.cn[0] : 0, c1 = acc ? D.cn[1] : 0;
                const int32_t c2 = acc ? D.cn[2] : 0, c3 = acc ? D.cn[3] : 0;
                s_n0[s0][cx] = n_f0 + c0;
                s_n0[sm][cx] = n_b0 + c1;
                s_n1[s0][cx] = n_f1 + c2;
                s_n1[s0][cm] = n_b1 + c3;
                s_r0[s0][cx] = (r0[0] + dcp_f) - TWO_PI * (double)c0;
                s_r0[sm][cx] = (r0[1] + dcp_b) - TWO_PI * (double)c1;
                s_r1[s0][cx] = (r0[2] + dcp_f) - TWO_PI * (double)c2;
                s_r1[s0][cm] = (r0[3] + dcp_b) - TWO_PI * (double)c3;
            }
        }
        __syncthreads();
        // ---------------- phase C: colour-1 decisions on row q = t+1+wave; rows t.. become final
        {
            const int32_t q = t + 1 + wave;
            const bool row_ok = (q >= t0) && (q <= t1);
            const int32_t gq = grow(q);
            const int32_t xs = FR ? ((par0 + q + 1) & 1) : x0 + ((par0 + q + x0 + 1) & 1);  // global (t + x) odd
            const int32_t x = xs + 2 * lane;
            const bool active = row_ok && (FR ? x < w : x <= x1);
            u128 bs[6];
#pragma unroll
            for (int k = 0; k < 6; k++) bs[k] = s_base[wave][8 + k];
            Draws D;
            if (fast[1])
                D = draws_fastp(A, RL, 1, active, lane, pk1, ((uint32_t)gq * (uint32_t)Nx + (uint32_t)(X0s + x)) >> 1,
                                bs, s_small);
            else if (fastfr[1])
                D = draws_fast(A, RL, 1, has_c1, active, lane, (uint32_t)gq * (uint32_t)Nx, (uint32_t)xs, (uint32_t)x, 0u,
                               bs, s_small);
            else
                D = draws_general(A, RL, 1, active, gq, wrapN(X0s + x, Nx), xb, bs, s_small, edge, xw,
                                  &s_base[wave][24]);
            if (active) {
                const int lr = q - rbase;
                const int sm = (lr - 1) % R, s0 = lr % R;
                const int cx = x - cofs, cm = cxm(cx);
                const double ph = s_phi[s0][cx];
                double ri[4];
                ri[0] = s_r0[s0][cx];
                ri[1] = s_r0[sm][cx];
                ri[2] = s_r1[s0][cx];
                ri[3] = s_r1[s0][cm];
                double cr[4];
                cr[0] = (0.0 - D.dphi) - TWO_PI * (double)D.cn[0];
                cr[1] = D.dphi - TWO_PI * (double)D.cn[1];
                cr[2] = (0.0 - D.dphi) - TWO_PI * (double)D.cn[2];
                cr[3] = D.dphi - TWO_PI * (double)D.cn[3];
                double dS = 0.0;
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    const double a = A.P.half_kappa * cr[k];
                    const double bb2 = (2.0 * ri[k]) + cr[k];
                    dS += a * bb2;
                }
                double p = sv_exp(-dS);
                p = p < 0.0 ? 0.0 : p;
                p = p > 1.0 ? 1.0 : p;
                const int acc = D.u < p;
                if (q >= q_lo && q < q_hi && (FR || (x >= c_lo && x < c_hi))) {
                    acc_count += acc;
                    fx_add(psum, p);
                }
                const double cphi = D.dphi * (double)acc;
                s_phi[s0][cx] = (ph + 0.0) + cphi;
                if (acc) {
                    s_n0[s0][cx] += D.cn[0];
                    s_n0[sm][cx] += D.cn[1];
                    s_n1[s0][cx] += D.cn[2];
                    s_n1[s0][cm] += D.cn[3];
                }
            }
        }
        commit(t + 3 + NW);  // slots of rows [t-NW, t): not read in phase C
        // advance the row bases by NW rows (one affine map; a full jump where the row wraps)
        if (base_lane) {
            const int64_t p_old = base_pos(bty, grow(brow), Nx, bx, bhas);
            const int64_t p_new = base_pos(bty, grow(brow + NW), Nx, bx, bhas);
            const int ai = bty == 0 ? 0 : (bty == 1 ? 1 : 2);
            const int64_t step = bty == 0 ? (int64_t)NW * Nx : (bty == 1 ? (int64_t)NW * Nx / 2 : (int64_t)NW * Nx / 4);
            if (p_new - p_old == step) bases = apply(s_adv[ai], bases);
            else bases = full_jump(RP.T, &s_blk[bblk], (uint32_t)p_new);
            brow += NW;
            s_base[wave][lane] = bases;  // read by this wave only, after the barrier below
        }
        __syncthreads();
    }
    {
        // the last step's rows; the loop ended with a barrier
        int32_t tl = tfirst;
        while (tl + NW < t1) tl += NW;
        store_rows(tl);
    }
    if (s_bad && threadIdx.x == 0) {
        // |n| too large for the int32 LDS image: the host falls back to the generic path
        report(A.S, A.sweep, OVERFLOW_BLOCK, 0, (uint32_t)rep);
    }
    flush_stats<NW>(REPS ? A.stat + (int64_t)rep * A.rep_stat : A.stat, acc_count, psum);
    if (OBS) {
        __syncthreads();
        unsigned long long *ow = A.obs + (int64_t)rep * A.rep_obs;
        if (threadIdx.x < 5 && s_obsw[threadIdx.x]) atomicAdd(&ow[threadIdx.x], s_obsw[threadIdx.x]);
        if (threadIdx.x == 5 && s_obig != 0.0) unsafeAtomicAdd((double *)&ow[5], s_obig);
    }
}

// 3 waves / SIMD (12 per CU, what the LDS ring allows): caps the kernel at 168 VGPRs
template <int NW, bool TILE, bool REPS, bool FR>
__global__ __launch_bounds__(NW * 64) __attribute__((amdgpu_waves_per_eu(3))) void villain_sweep_fused(FArgs A) {
    sweep_body<NW, TILE, REPS, false, FR>(A);
}
// replica batch with the inline observables fused into the row stores: held to 3 waves / SIMD
template <bool FR>
__global__ __launch_bounds__(4 * 64) __attribute__((amdgpu_waves_per_eu(3))) void villain_sweep_fused_obs(FArgs A) {
    sweep_body<4, false, true, true, FR>(A);
}

template __global__ void villain_sweep_fused<4, false, false, false>(FArgs);
template __global__ void villain_sweep_fused<4, true, false, false>(FArgs);
template __global__ void villain_sweep_fused<4, false, true, false>(FArgs);
template __global__ void villain_sweep_fused<4, false, true, true>(FArgs);
template __global__ void villain_sweep_fused_obs<false>(FArgs);
template __global__ void villain_sweep_fused_obs<true>(FArgs);

// ================================================================================================
// observables (fused reductions over the current state)
// ================================================================================================
__global__ void villain_observables_kernel(int32_t N, const double *phi, const int64_t *n, unsigned long long *out) {
    // the exact observable words of the state (common.h OBS_WORDS; the launch gives every thread <= 256 sites)
    const int64_t V = (int64_t)N * N;
    unsigned long long q = 0, w2 = 0;
    int64_t s_n0 = 0, s_n1 = 0;
    double big = 0.0;
    for (int64_t s = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; s < V; s += (int64_t)gridDim.x * blockDim.x) {
        int64_t t = s / N, x = s - t * N;
        int64_t f0 = ((t + 1 == N) ? 0 : t + 1) * N + x;
        int64_t f1 = t * N + ((x + 1 == N) ? 0 : x + 1);
        double p = phi[s];
        double l0 = (0.0 + (phi[f0] - p)) - TWO_PI * (double)n[s];
        double l1 = (0.0 + (phi[f1] - p)) - TWO_PI * (double)n[V + s];
        const double a = l0 * l0 + l1 * l1;
        if (a < ACT_LIMIT) q += act_fx(a);
        else big += a;
        // (dn)_01[x] = (n1[x+e0] - n1[x]) - (n0[x+e1] - n0[x])   (d on 1-forms, rows (0,1,0,+1),(0,0,1,-1))
        int64_t dn = (n[V + f0] - n[V + s]) - (n[f1] - n[s]);
        w2 += (unsigned long long)(dn * dn);
        s_n0 += n[s];
        s_n1 += n[V + s];
    }
    unsigned long long w[5] = {q & 0xffffffffull, q >> 32, w2, (unsigned long long)s_n0, (unsigned long long)s_n1};
    for (int o = 32; o > 0; o >>= 1)
        for (int i = 0; i < 5; i++) w[i] += __shfl_xor(w[i], o);
    if ((threadIdx.x & 63) == 0)
        for (int i = 0; i < 5; i++)
            if (w[i]) atomicAdd(&out[i], w[i]);
    if (big != 0.0) unsafeAtomicAdd((double *)&out[5], big);
}


// the exact acceptance limbs of each slot (its proposed, rejections and acceptance_sum words on the device, common.h)
// into its acceptance_sum; a finalized slot is marked (rejections = -1) and left alone by a second finalize
__global__ void stats_finalize(sv_stats *s, int64_t n) {
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    if (s[i].rejections == -1) return;  // (finalized already: limb 1 never reaches 2^63)
    const uint64_t w0 = stat_limb(s[i], 0), w1 = stat_limb(s[i], 1), w2 = stat_limb(s[i], 2);
    s[i].acceptance_sum = fx_value(w0, w1, w2);
    s[i].proposed = 0;
    s[i].rejections = -1;  // (every landing overwrites it on the host)
}

}  // namespace sv

// ==================================================================================================
// host drivers
// ==================================================================================================
namespace svh {

std::vector<BlockSpec> villain_specs(int64_t V, int ncol, const int64_t *count, bool has_bounded) {
    std::vector<BlockSpec> s;
    s.push_back({UNIFORM, (uint32_t)V});
    for (int c = 0; c < ncol; c++) {
        uint32_t nc = (uint32_t)count[c];
        s.push_back({UNIFORM, nc});
        for (int q = 0; q < 4; q++) s.push_back({BOUNDED, has_bounded ? nc : 0u});
    }
    return s;
}

std::vector<BlockSpec> villain_specs(const sv_villain *st, bool has_bounded) {
    return villain_specs((int64_t)st->N * st->N, st->ncol, st->count, has_bounded);
}

int64_t rejections_in(const SkipMap &skips, int sweep, int nblocks) {
    int64_t rj = 0;
    for (int bi = 0; bi < nblocks; bi++) {
        auto it = skips.find({sweep, bi});
        if (it != skips.end()) rj += (int64_t)it->second.size();
    }
    return rj;
}

void launch_fused_tile(const FArgs &A, int grid, hipStream_t stream, bool hot) {
    if (hot) launch_hot(A, grid, stream);
    else villain_sweep_fused<4, true, false, false><<<grid, 4 * 64, 0, stream>>>(A), SV_LAUNCHED("villain_sweep_fused<4, true, false, false>", stream);
}


void launch_fused_batch(const FArgs &A, int grid, bool obs, hipStream_t stream) {
    const bool fr = A.nsx == 1 && A.G.Nx <= RW;  // full-row strips
    if (obs && fr) villain_sweep_fused_obs<true><<<grid, 4 * 64, 0, stream>>>(A), SV_LAUNCHED("villain_sweep_fused_obs<true>", stream);
    else if (obs) villain_sweep_fused_obs<false><<<grid, 4 * 64, 0, stream>>>(A), SV_LAUNCHED("villain_sweep_fused_obs<false>", stream);
    else if (fr) villain_sweep_fused<4, false, true, true><<<grid, 4 * 64, 0, stream>>>(A), SV_LAUNCHED("villain_sweep_fused<4, false, true, true>", stream);
    else villain_sweep_fused<4, false, true, false><<<grid, 4 * 64, 0, stream>>>(A), SV_LAUNCHED("villain_sweep_fused<4, false, true, false>", stream);
}

void farg_single(FArgs &A, int nsx, int nsy) {
    A.tiles_per_rep = nsx * nsy;
    A.rep_blocks = 0;
    A.rep_field = 0;
    A.rep_stat = 0;
    A.rep_obs = 0;
    A.Trep = nullptr;
    A.advrep = nullptr;
    A.obs = nullptr;
    A.strips = nullptr;
    A.rep_map = nullptr;
}

// plan `count` sweeps starting at sweep `first`, writing descriptors to ctx host staging
void plan_sweeps(sv_ctx *ctx, Cursor &cur, u128 inc, const std::vector<BlockSpec> &specs, int first, int count,
                 const SkipMap &skips, std::vector<Block> &blocks, std::vector<uint32_t> &skipvec) {
    blocks.clear();
    skipvec.clear();
    static const std::vector<uint32_t> none;
    for (int sw = first; sw < first + count; sw++) {
        for (int bi = 0; bi < (int)specs.size(); bi++) {
            auto it = skips.find({sw, bi});
            const std::vector<uint32_t> &sk = it == skips.end() ? none : it->second;
            Block b = plan_block(cur, inc, specs[bi], sk, (int32_t)skipvec.size());
            skipvec.insert(skipvec.end(), sk.begin(), sk.end());
            blocks.push_back(b);
        }
    }
}

void upload_plan(sv_ctx *ctx, const std::vector<Block> &blocks, const std::vector<uint32_t> &skipvec) {
    ctx->upload_plan(blocks.data(), blocks.size(), skipvec.data(), skipvec.size());
}

VParams make_params(int32_t N, double kappa, int64_t W, double interval_phi, int64_t interval_n) {
    VParams P;
    P.N = N;
    P.half_kappa = kappa / 2.0;
    P.W = W;
    P.lo_phi = -interval_phi;
    P.range_phi = interval_phi - (-interval_phi);
    P.interval_n = interval_n;
    P.k = (uint32_t)(2 * interval_n + 1);
    P.thr = P.k > 1 ? (uint32_t)((0u - P.k) % P.k) : 0u;
    return P;
}

DevScratch scratch(sv_ctx *ctx) { return DevScratch{ctx->d_abort, ctx->d_nreport, ctx->d_reports}; }

AbortInfo read_abort(sv_ctx *ctx) {
    AbortInfo a;
    uint32_t nrep = 0;
    int32_t both[2];  // d_abort, d_nreport are adjacent (capi.hip)
    SV_HIP(hipMemcpyAsync(both, ctx->d_abort, sizeof(both), hipMemcpyDeviceToHost, ctx->stream));
    SV_HIP(hipStreamSynchronize(ctx->stream));
    a.abort = both[0];
    nrep = (uint32_t)both[1];
    if (nrep > (uint32_t)MAX_REPORTS) nrep = MAX_REPORTS;
    a.reports.resize(nrep);
    if (nrep) {
        SV_HIP(hipMemcpyAsync(a.reports.data(), ctx->d_reports, nrep * sizeof(Report), hipMemcpyDeviceToHost,
                              ctx->stream));
        SV_HIP(hipStreamSynchronize(ctx->stream));
    }
    return a;
}

// The batch tail in one synchronization: abort flag, report count, the first TAIL_REPORTS reports and the batch's
// statistics land in a pinned host block (DMA copies); the stats are copied to `stats` only when no rejection aborted
// the batch -- after an abort, `landed` points at them (the sweeps before the failing one are kept from there), and
// only a batch with more than TAIL_REPORTS reports needs a second copy
static constexpr size_t TAIL_HEAD = 16 + TAIL_REPORTS * sizeof(Report);  // 256 B
void finalize_stats(sv_stats *d, int64_t n, hipStream_t stream) {
    if (n <= 0) return;
    stats_finalize<<<(unsigned)((n + 255) / 256), 256, 0, stream>>>(d, n), SV_LAUNCHED("stats_finalize", stream);
}

AbortInfo read_abort_stats(sv_ctx *ctx, int count, sv_stats *stats, const sv_stats **landed = nullptr) {
    const size_t bytes = TAIL_HEAD + (size_t)count * sizeof(sv_stats);
    if (bytes > ctx->tail_cap) {
        SV_HIP(hipStreamSynchronize(ctx->stream));
        if (ctx->h_tail) SV_HIP(hipHostFree(ctx->h_tail));
        ctx->tail_cap = std::max<size_t>(bytes, TAIL_HEAD + 64 * sizeof(sv_stats));
        SV_HIP(hipHostMalloc((void **)&ctx->h_tail, ctx->tail_cap, hipHostMallocDefault));
    }
    int32_t *h_ab = (int32_t *)ctx->h_tail;
    uint32_t *h_nrep = (uint32_t *)(ctx->h_tail + 4);
    const Report *h_rep = (const Report *)(ctx->h_tail + 16);
    sv_stats *h_st = (sv_stats *)(ctx->h_tail + TAIL_HEAD);
    SV_HIP(hipMemcpyAsync(ctx->h_tail, ctx->d_abort, TAIL_HEAD, hipMemcpyDeviceToHost, ctx->stream));  // + d_nreport, reports
    finalize_stats(ctx->d_stats, count, ctx->stream);
    SV_HIP(hipMemcpyAsync(h_st, ctx->d_stats, count * sizeof(sv_stats), hipMemcpyDeviceToHost, ctx->stream));
    SV_HIP(hipStreamSynchronize(ctx->stream));
    AbortInfo a;
    a.abort = *h_ab;
    uint32_t nrep = *h_nrep;
    a.raw = nrep;
    if (landed) *landed = h_st;
    if (!a.abort) {
        std::memcpy(stats, h_st, count * sizeof(sv_stats));
        return a;
    }
    if (nrep > (uint32_t)MAX_REPORTS) nrep = MAX_REPORTS;
    a.reports.resize(nrep);
    if (nrep <= (uint32_t)TAIL_REPORTS) {
        std::memcpy(a.reports.data(), h_rep, nrep * sizeof(Report));
    } else {
        SV_HIP(hipMemcpyAsync(a.reports.data(), ctx->d_reports, nrep * sizeof(Report), hipMemcpyDeviceToHost,
                              ctx->stream));
        SV_HIP(hipStreamSynchronize(ctx->stream));
    }
    return a;
}

__global__ __launch_bounds__(256) void reset_batch_kernel(int32_t *abort, uint32_t *nreport, uint64_t *a, int64_t na,
                                                         uint64_t *b, int64_t nb, int32_t *gate) {
    const int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x, stride = (int64_t)gridDim.x * blockDim.x;
    if (t == 0) {
        *abort = 0;
        *nreport = 0;
        if (gate) *gate = INT32_MAX;
    }
    for (int64_t i = t; i < na; i += stride) a[i] = 0;
    for (int64_t i = t; i < nb; i += stride) b[i] = 0;
}

void reset_batch(sv_ctx *ctx, void *a, size_t a_bytes, void *b, size_t b_bytes, int32_t *gate) {
    if (a_bytes % 8 || b_bytes % 8) throw std::logic_error("reset_batch: sizes must be multiples of 8 bytes");
    const int64_t na = (int64_t)(a_bytes / 8), nb = (int64_t)(b_bytes / 8), n = std::max(na, nb);
    const int grid = (int)std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, 256));
    reset_batch_kernel<<<grid, 256, 0, ctx->stream>>>(ctx->d_abort, ctx->d_nreport, (uint64_t *)a, na, (uint64_t *)b, nb,
                                                      gate), SV_LAUNCHED("reset_batch_kernel", ctx->stream);
}

void clear_abort(sv_ctx *ctx) {
    SV_HIP(hipMemsetAsync(ctx->d_abort, 0, sizeof(int32_t), ctx->stream));
    SV_HIP(hipMemsetAsync(ctx->d_nreport, 0, sizeof(uint32_t), ctx->stream));
}

// Add the rejected positions of the earliest reported (sweep, block) to the skip map.
// Returns that sweep index (relative to the batch start).
// Skips of later choice blocks (of this sweep or a later one) were found against descriptors that did not yet know the
// skip just added: it moves every later block's start one half-word on, so their rejected words sit one position lower
// now.  They are dropped and found again, at their true positions, by the replay (r6: two rejections in one sweep whose
// later block's was found first -- the early stop left the earlier one unreported -- kept a stale skip and replayed the
// sweep wrong; tests/test_gpu_split.py two-rejection cases).  Skips within one block are positions in that block's own
// stream and stay valid.
void drop_later_skips(SkipMap &skips, const std::pair<int, int> &key) {
    skips.erase(skips.upper_bound(key), skips.end());
}

int absorb_reports(const AbortInfo &a, int first, SkipMap &skips) {
    if (a.reports.empty()) throw std::runtime_error("device aborted without a rejection report");
    std::pair<uint32_t, uint32_t> best{~0u, ~0u};
    for (const Report &r : a.reports)
        if (std::make_pair(r.sweep, r.block) < best) best = {r.sweep, r.block};
    const std::pair<int, int> key{first + (int)best.first, (int)best.second};
    auto &lst = skips[key];
    const size_t before = lst.size();
    for (const Report &r : a.reports)
        if (r.sweep == best.first && r.block == best.second) lst.push_back(r.pos);
    std::sort(lst.begin(), lst.end());
    lst.erase(std::unique(lst.begin(), lst.end()), lst.end());
    // a replay that meets only positions it already skips would repeat forever: a kernel drew a skipped word
    if (lst.size() == before) throw std::logic_error("rejection replay made no progress (a skipped word was drawn)");
    drop_later_skips(skips, key);
    return (int)best.first;
}

// rows per strip.  52 measured best at L=4096 (322 us vs 328 at 64, 324 at 48, 345 at 80; r73 sweep).
// Small lattices have few strips: there the strips are cut shorter (down to 4 rows, more halo rows
// recomputed) until the grid has `fill` = 512 workgroups, so that every CU has work (SURVEY.md 8(d)
// config 2; r203 sweep, us per sweep kernel: L=256 at 52 / 16 / 8 / 4 rows: 88.1 / 35.5 / 24.2 / 19.8;
// L=1024 at 52 / 32 / 24 / 16 / 12 / 8 rows: 90.8 / 67.3 / 54.6 / 47.9 / 55.7 / 59.5).
// Heights are 4k + 1: villain_sweep_hot covers a strip of TH rows in ceil((TH + 3) / NW) row steps of NW = 4 rows (the
// colour-1 pass runs one row and the colour-0 pass two rows ahead of the stores, the first step starting 3 rows
// above the strip), so 53 rows take the 14 steps 52 did (r3: L=1024 16 -> 17 rows, L=4096 52 -> 53).
int fused_th(int32_t N, int nsx) {
    const char *e = getenv("SV_FUSED_TH");
    if (e) {
        const int v = atoi(e);
        if (v >= 4) return v;
    }
    constexpr int fill = 512;
    int th = 53;
    while (th > 5 && (int64_t)nsx * ((N + th - 1) / th) < fill) th -= 4;
    return th;
}

bool fused_ok(int32_t N) { return N % 2 == 0 && N >= 4; }

void run_generic(sv_villain *st, const VParams &P, int32_t sweeps, Cursor &cur, u128 inc, sv_stats *stats) {
    sv_ctx *ctx = st->ctx;
    const JumpTables *T = ctx->jump_tables(inc.hi, inc.lo);
    const int64_t V = (int64_t)st->N * st->N;
    auto specs = villain_specs(st, P.k > 1);
    const int nb = (int)specs.size();
    SkipMap skips;
    std::vector<Block> blocks;
    std::vector<uint32_t> skipvec;
    ctx->ensure_stats(1);
    double *phi = st->phi[st->cur];
    int64_t *n = st->n[st->cur];
    for (int sw = 0; sw < sweeps; sw++) {
        SV_HIP(hipMemcpyAsync(st->snap_phi, phi, V * sizeof(double), hipMemcpyDeviceToDevice, ctx->stream));
        SV_HIP(hipMemcpyAsync(st->snap_n, n, 2 * V * sizeof(int64_t), hipMemcpyDeviceToDevice, ctx->stream));
        for (int attempt = 0;; attempt++) {
            if (attempt > 64) throw std::runtime_error("rejection replay did not converge");
            Cursor c = cur;
            plan_sweeps(ctx, c, inc, specs, sw, 1, skips, blocks, skipvec);
            upload_plan(ctx, blocks, skipvec);
            reset_batch(ctx, ctx->d_stats, sizeof(sv_stats));
            const int grid = (int)std::min<int64_t>((V + 255) / 256, 4096);
            villain_phi_normalize<<<grid, 256, 0, ctx->stream>>>(st->N, phi, ctx->d_abort), SV_LAUNCHED("villain_phi_normalize", ctx->stream);
            villain_r_init<<<grid, 256, 0, ctx->stream>>>(st->N, phi, n, st->r, ctx->d_abort), SV_LAUNCHED("villain_r_init", ctx->stream);
            ctx->sweeps_generic++;
            for (int col = 0; col < st->ncol; col++) {
                int64_t nc = st->count[col];
                if (!nc) continue;
                villain_pass_generic<<<(int)((nc + 255) / 256), 256, 0, ctx->stream>>>(
                    P, phi, n, st->r, st->sites + st->offset[col], nc, col, ctx->d_blocks, ctx->d_skips, T,
                    ctx->d_stats, scratch(ctx), 0u), SV_LAUNCHED("villain_pass_generic", ctx->stream);
            }
            SV_HIP(hipGetLastError());
            AbortInfo a = read_abort(ctx);
            if (!a.abort) {
                cur = c;
                break;
            }
            absorb_reports(a, sw, skips);
            SV_HIP(hipMemcpyAsync(phi, st->snap_phi, V * sizeof(double), hipMemcpyDeviceToDevice, ctx->stream));
            SV_HIP(hipMemcpyAsync(n, st->snap_n, 2 * V * sizeof(int64_t), hipMemcpyDeviceToDevice, ctx->stream));
        }
        finalize_stats(ctx->d_stats, 1, ctx->stream);
        SV_HIP(hipMemcpyAsync(&stats[sw], ctx->d_stats, sizeof(sv_stats), hipMemcpyDeviceToHost, ctx->stream));
        SV_HIP(hipStreamSynchronize(ctx->stream));
        stats[sw].proposed = V;
        // rejections actually met in this sweep
        int64_t rj = 0;
        for (int bi = 0; bi < nb; bi++) {
            auto it = skips.find({sw, bi});
            if (it != skips.end()) rj += (int64_t)it->second.size();
        }
        stats[sw].rejections = rj;
    }
}

// Strip schedule of villain_sweep_hot on a single lattice.  With uniform strips the last round of the chip's
// workgroup slots is partly empty while its strips finish (the WG timeline of an L=4096 sweep, r3: slots ~80% busy,
// a ~45 us tail of 240 us).  The lattice rows are cut into 8 bands, one per XCD (workgroup i runs on XCD i mod 8,
// and hot_body's logical order gives each XCD a contiguous range), and each band into segments whose heights (a
// descending list, e.g. "57x5,41x5,22": heights of 4k+1 rows) put the tall strips first and the short ones in the
// last rounds (band_strips builds the default; SV_STRIPS passes a list here).  Returns
// the table {ix, t0, t1} per logical strip, or an empty vector when the spec does not apply (then uniform TH).
std::vector<int32_t> strip_schedule(int32_t Nt, int nsx, const std::string &spec) {
    std::vector<int32_t> hs;
    size_t p = 0;
    while (p < spec.size()) {
        size_t q = spec.find(',', p);
        if (q == std::string::npos) q = spec.size();
        const std::string tok = spec.substr(p, q - p);
        const size_t x = tok.find('x');
        const int h = atoi(tok.substr(0, x).c_str()), m = x == std::string::npos ? 1 : atoi(tok.substr(x + 1).c_str());
        if (h < 4 || m < 1) return {};
        for (int i = 0; i < m; i++) hs.push_back(h);
        p = q + 1;
    }
    int32_t band = 0;
    for (int h : hs) band += h;
    if (hs.empty() || (int64_t)band * 8 != Nt) return {};
    std::vector<int32_t> tab;
    for (int xcd = 0; xcd < 8; xcd++) {
        int32_t t = xcd * band;
        for (int h : hs) {
            for (int ix = 0; ix < nsx; ix++) {
                tab.push_back(ix);
                tab.push_back(t);
                tab.push_back(t + h);
            }
            t += h;
        }
    }
    return tab;
}

// The default descending schedule for H rows (any H >= 64): 8 bands of H / 8 rows (one per XCD), each ~55% in
// 57-row strips, then 41-row strips, then the rest (heights 4k + 1, fused_th); a remainder under 5 rows joins the
// band's last strip.  L=4096: "57x5,41x5,22" per band.
std::vector<int32_t> band_strips(int32_t H, int nsx) {
    std::vector<int32_t> tab;
    for (int b = 0; b < 8; b++) {
        const int32_t r0 = (int32_t)((int64_t)b * H / 8), r1 = (int32_t)((int64_t)(b + 1) * H / 8), h = r1 - r0;
        std::vector<int32_t> hs;
        const int n57 = (int)(0.55 * h / 57 + 0.5), n41 = (h - 57 * n57) / 41;
        for (int i = 0; i < n57; i++) hs.push_back(57);
        for (int i = 0; i < n41; i++) hs.push_back(41);
        const int rest = h - 57 * n57 - 41 * n41;
        if (rest >= 5 || hs.empty()) hs.push_back(rest);
        else hs.back() += rest;
        int32_t t = r0;
        for (int hh : hs) {
            for (int ix = 0; ix < nsx; ix++) {
                tab.push_back(ix);
                tab.push_back(t);
                tab.push_back(t + hh);
            }
            t += hh;
        }
    }
    return tab;
}

// returns false if the fused path cannot represent the state (|n| too large): caller falls back
// set once a band launch has failed (BAND_FAIL_BLOCK): the process's small lattices then run one sweep per launch
static std::atomic<bool> band_broken{false};

bool run_fused(sv_villain *st, const VParams &P, int32_t sweeps, Cursor &cur, u128 inc, sv_stats *stats,
               int &done_sweeps) {
    sv_ctx *ctx = st->ctx;
    const JumpTables *T = ctx->jump_tables(inc.hi, inc.lo);
    const int32_t N = st->N;
    const int64_t V = (int64_t)N * N;
    auto specs = villain_specs(st, P.k > 1);
    const int nb = (int)specs.size();
    const int nsx = (N + FW_MAX - 1) / FW_MAX;
    constexpr int NWv = 4;  // (6-wave strips measured slower: 557-575 vs 320 us per sweep, round 1)
    // small lattices (strips cut to the 4-row minimum to fill the chip): 8-wave workgroups instead, over 5-row strips:
    // the kernel's row pipeline (colour 0 on rows t+2+w, colour 1 on t+1+w) then covers a strip in ONE row step, its
    // prologue rows included (8-row strips took two; L=256: 15.75 us per sweep at 4 rows / 4 waves, r369; 15.2 at
    // 8 rows / 8 waves; 13.5 at 5 rows, r3 -- 4 / 3 / 13 rows: 14.4 / 15.8 / 16.4)
    const bool small8 = !getenv("SV_FUSED_TH") && fused_th(N, nsx) <= 5 && NWv == 4;
    const int TH = small8 ? 5 : fused_th(N, nsx);
    const int nsy = (N + TH - 1) / TH;
    const int grid = nsx * nsy;
    // sweeps per host round trip (SV_BATCH overrides): 64 measured best at L=4096; small lattices amortize the ~80 us
    // batch boundary (statistics read back, the next batch's reset and plan upload) over 256 (L=256, r4: 8.4-8.6 vs
    // 9.1-9.7 us per sweep wall, profiles/r04_block_l256_batch.txt)
    const char *batch_env = getenv("SV_BATCH");
    const int BATCH = batch_env && atoi(batch_env) >= 1 ? atoi(batch_env) : (V <= (1 << 18) ? 256 : 64);
    // row-base advance maps for NW rows: NW*N metropolis draws, NW*N/2 ranks, NW*N/4 words
    if ((int64_t)NWv * N % 4) throw std::invalid_argument("fused path needs NW*N divisible by 4");
    const Affine adv[3] = {host_power(inc, (uint64_t)NWv * N), host_power(inc, (uint64_t)NWv * N / 2),
                           host_power(inc, (uint64_t)NWv * N / 4)};
    // villain_sweep_hot with 8 waves per workgroup (8 rows per step) when the strips allow it
    const int hot_nw = small8 ? 8 : 4;
    const Affine adv8[3] = {host_power(inc, 8 * (uint64_t)N), host_power(inc, 8 * (uint64_t)N / 2),
                            host_power(inc, 8 * (uint64_t)N / 4)};
    SkipMap skips;
    std::vector<Block> blocks;
    std::vector<uint32_t> skipvec;
    int sw = 0;
    const bool dbg = getenv("SV_DEBUG_TIMING") != nullptr;
    const bool use_hot = V < (int64_t(1) << 28);  // villain_sweep_hot's 32-bit row offsets
    // the hot kernel's strip schedule (SV_STRIPS overrides: "uniform" or "" = strips of TH rows).  Default on
    // lattices of >= 4096 rows: band_strips -- per XCD band, 57-row strips, then 41-row strips, then the rest (L=4096:
    // "57x5,41x5,22", heights 4k+1 so the last row step of a strip is full), so the last rounds of slots run shorter
    // strips (r3 A/B, 6 interleaved repetitions of 300 sweeps: uniform 230.6 -> 225.5 us per sweep)
    {
        const char *e = getenv("SV_STRIPS");
        const bool dflt = !e && N >= 4096;
        const std::string spec = dflt ? "band_strips" : (e ? (std::string(e) == "uniform" ? "" : e) : "");
        if (spec != st->strips_key || !st->d_strips) {
            const std::vector<int32_t> tab = hot_nw != 4 ? std::vector<int32_t>{}
                                             : (dflt ? band_strips(N, nsx) : strip_schedule(N, nsx, spec));
            if (st->d_strips) SV_HIP(hipFree(st->d_strips));
            st->d_strips = nullptr;
            st->h_strips = tab;
            st->n_strips = (int32_t)(tab.size() / 3);
            if (!tab.empty()) {
                SV_HIP(hipMalloc(&st->d_strips, tab.size() * sizeof(int32_t)));
                SV_HIP(hipMemcpy(st->d_strips, tab.data(), tab.size() * sizeof(int32_t), hipMemcpyHostToDevice));
            }
            st->strips_key = spec;
        }
    }
    // Small lattices: K sweeps per launch, one band of rows per XCD (villain_sweep_hot_band, BandArgs in villain.h).
    // K (odd, at most BAND_MAXK) is sv_ctx_set_multisweep's, else 3; the band's workgroups must all be resident on its XCD.
    const int nbands = 8;
    int bandK = 0, bandP = 0;
    // Temporal blocking (villain_sweep_block, BlockArgs in villain.h) is preferred where it applies: bs x bs blocks (bs =
    // N / 16, at least 4) whose frame of K sweeps fits the lattice and the small-offset maps.
    // sv_ctx_set_multisweep: 0 either (blocks first), 1 blocks only, 2 bands only, 3 neither, and K (else 3).
    int blockK = 0, blockBS = 0;
    Affine block_step{};
    const int mode = ctx->multisweep;
    {
        // one sweep's stream length in u64s (the buffered-half flags repeat from sweep to sweep when the bounded
        // words of a sweep are even in number; the launch checks every descriptor anyway)
        uint64_t S = 0, bounded = 0;
        for (const BlockSpec &b : specs) (b.kind == UNIFORM ? S : bounded) += b.count;
        if ((mode == 0 || mode == 1) && use_hot && hot_params_ok(P) && N % 2 == 0 && N <= 512 &&
            bounded % 2 == 0) {
            int bs = std::max(4, N / 16);
            while (bs > 2 && N % bs) bs--;
            int K = std::min(ctx->block_k > 0 ? ctx->block_k : 3, BAND_MAXK);
            if (K % 2 == 0) K--;
            if (N % bs == 0) {
                for (; K >= 3; K -= 2) {
                    const int F = block_frame(bs, K);
                    if (F <= N && F <= SMALL_LDS - 2 && block_lds_bytes(F) <= 160 * 1024) break;
                }
                if (K >= 3) {
                    blockK = K;
                    blockBS = bs;
                    block_step = host_power(inc, S + bounded / 2);
                }
            }
        }
    }
    {
        static const int cus = [] {
            int dev = 0, v = 0;
            if (hipGetDevice(&dev) != hipSuccess ||
                hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
                v = 0;
            return v;
        }();
        if (!blockK && (mode == 0 || mode == 2) && use_hot && small8 && hot_nw == 8 &&
            !band_broken.load() && N % nbands == 0 && N <= 512) {
            const int own = N / nbands, per_xcd = band_residency() * (cus / nbands);
            // (K = 3 measured best at L=256, r4: 11.8 / 12.7 / 13.7 us per sweep at K = 3 / 5 / 7, 13.7 one per launch)
            int K = std::min(ctx->block_k > 0 ? ctx->block_k : 3, BAND_MAXK);
            if (K % 2 == 0) K--;
            for (; K >= 3; K -= 2) {
                const int P = nsx * ((own + 5 * (K - 1) + TH - 1) / TH);
                if (P <= per_xcd && own + 5 * (K - 1) <= N) {
                    bandK = K;
                    bandP = P;
                    break;
                }
            }
        }
        if (blockK) bandK = blockK;  // (the band launches' buffers, gate and replay protocol)
        if (bandK) {
            while ((int)st->band_phi.size() < bandK - 1) {
                double *p = nullptr;
                int64_t *q = nullptr;
                SV_HIP(hipMalloc(&p, V * sizeof(double)));
                st->band_phi.push_back(p);
                SV_HIP(hipMalloc(&q, 2 * V * sizeof(int64_t)));
                st->band_n.push_back(q);
            }
            if (!st->band_ctrl) SV_HIP(hipMalloc(&st->band_ctrl, (nbands * BAND_CTRL + 64) * sizeof(uint32_t)));
        }
    }
    int32_t *band_gate = bandK ? (int32_t *)(st->band_ctrl + nbands * BAND_CTRL) : nullptr;  // (null: no gate)
    // |n| beyond villain_sweep_hot's int16 image: the failing sweep is replayed, and the rest of the call runs, on
    // villain_sweep_fused's int32 image; only an overflow of that one falls back to the per-colour int64 path
    bool hot_off = false;
    // The next batch is planned on the host while the device runs this one (a batch boundary otherwise leaves the
    // GPU idle for the plan of 64 sweeps, ~0.3 ms: 5 us per L=4096 sweep in the driver form); an abort discards it
    std::vector<Block> blocks_next;
    std::vector<uint32_t> skipvec_next;
    Cursor c_next{};
    int sw_next = -1;
    while (sw < sweeps) {
        const int count = std::min(BATCH, sweeps - sw);
        Cursor c = cur;
        // the batch reset first: the device clears the flags and statistics while the host plans
        ctx->ensure_stats(count);
        if (bandK)
            reset_batch(ctx, ctx->d_stats, count * sizeof(sv_stats), st->band_ctrl, nbands * BAND_CTRL * sizeof(uint32_t),
                        band_gate);
        else
            reset_batch(ctx, ctx->d_stats, count * sizeof(sv_stats));
        std::vector<int> band_starts;  // first sweeps of this batch's band launches
        auto tp0 = std::chrono::steady_clock::now();
        // A batch that is not pre-planned (a call's first) on a small lattice is planned in two parts: the first few
        // launches' sweeps, uploaded and launched, then the rest while the device runs them (the plan of a 200-sweep
        // L=256 batch is ~55 us, ~3% of the call, r4 profiles/r04b_l256_host_phases.log).  Only without known skips.

        int part = count;  // sweeps of the batch planned and uploaded
        if (sw_next == sw) {
            blocks.swap(blocks_next);
            skipvec.swap(skipvec_next);
            c = c_next;
        } else if ((skips.empty() || skips.rbegin()->first.first < sw + 3 * std::max(bandK, 1)) && V <= (1 << 18) &&
                   count >= 4 * 3 * std::max(bandK, 1)) {
            // (known skips only in the first part -- the replay after an abort starts the batch -- so the re-plan after
            // a rejection leaves the GPU idle for the first part's plan only, r6)
            part = 3 * std::max(bandK, 1);
            plan_sweeps(ctx, c, inc, specs, sw, part, skips, blocks, skipvec);
            ctx->ensure_blocks((size_t)count * nb);  // (the second part must not move d_blocks under the first launches)
        } else {
            plan_sweeps(ctx, c, inc, specs, sw, count, skips, blocks, skipvec);
        }
        sw_next = -1;
        auto tp1 = std::chrono::steady_clock::now();
        if (dbg) fprintf(stderr, "[sv] plan %d sweeps: %.1f us\n", count, std::chrono::duration<double, std::micro>(tp1 - tp0).count());
        // Sweeps with known rejections, at most one per choice block (the replay of a rejected sweep): the split replay
        // (villain_sweep_hot_split), ~one hot sweep; the descriptors after each switch go up with the batch's plan.  The
        // general int32 kernel takes the rest (~1.9 hot sweeps).  (r4 measured a skip-list form of the hot kernel on
        // every strip: slower than the general kernel)
        std::vector<std::pair<int, SplitArgs>> splits;
        std::vector<size_t> split_off;
        if (!skips.empty() && use_hot && !hot_off && NWv == 4 && hot_nw == 4 && nb == 11) {
            for (int k = 0; k < part; k++) {
                const Block *bk = &blocks[(size_t)k * nb];
                if (hot_ok(P, bk)) continue;
                SplitArgs SA;
                Block Bset[11];
                if (!split_plan(P, bk, skipvec.data(), inc, SA, Bset)) continue;
                split_order(SA, FGeom{N, N, 0, 0, N, N, N, V, 0}, nsx, TH, st->d_strips ? st->n_strips : grid,
                            st->d_strips ? st->h_strips.data() : nullptr);
                splits.push_back({k, SA});
                split_off.push_back(blocks.size());
                blocks.insert(blocks.end(), Bset, Bset + 11);
            }
        }
        upload_plan(ctx, blocks, skipvec);
        // sweep k of the batch reads buffer cur ^ (k & 1); after m sweeps the state is in cur ^ (m & 1)
        auto set_current = [&](int m) { st->cur ^= m & 1; };
        // Timing (sv_ctx_set_timing) measures villain_sweep_hot only: events around each run of consecutive hot
        // launches (mode 1) or around every hot launch (mode 2); the general kernel's replays are not counted
        hipEvent_t seg = nullptr;
        int seg_k0 = 0;
        const bool per_launch = ctx->timing_mode == 2;
        // Large lattices (>= 2^22 sites: a sweep takes >= 50 us) are enqueued two sweeps at a time behind the host-mapped
        // progress word (FArgs::progress): a NumPy Lemire rejection then leaves at most ~4 early-exit launches queued
        // (~5 us each) instead of the rest of the batch.  r5, scripts/perf/reject_window.py 4096 20 150, two runs each
        // (profiles/r05_chunk_ab.txt): extra per call that meets a rejection 0.270 / 0.274 ms whole, 0.225 / 0.228 ms in
        // chunks of 2, 0.241 / 0.254 in chunks of 4; clean calls level (4.38-4.40 ms).  Small lattices are enqueued whole
        // (their sweeps are a few us: the host would pace the GPU).  Host cost: the calling thread polls the progress word
        // for the length of the batch (std::this_thread::yield between polls, so other runnable threads get the core):
        // one host core per large-lattice call, the price of the ~5 us early exit.
        // Multi-sweep launches (temporal blocks, XCD bands) go out four launches (~90 us at L=256) at a time behind the
        // progress word too: a rejection then leaves at most ~8 early-exit launches queued instead of the rest of a
        // 256-sweep batch (r5: ~0.32 ms, ~41 sweeps, per rejection at L=256); four launches take the host ~20 us to
        // enqueue, well inside the chunk before them.
        const int CH = V >= (int64_t(1) << 22) ? 2 : (bandK ? 4 * bandK : count);
        int launched = count;
        *ctx->h_flag = 0;
        __atomic_store_n(ctx->h_prog, 0, __ATOMIC_RELEASE);  // (the previous batch's launches have all finished)
        int next_chunk = CH;
        for (int k = 0; k < count;) {
            if (part < count && k + std::max(bandK, 1) > part) {  // the two-part plan's second part
                std::vector<Block> b2;
                std::vector<uint32_t> s2;
                plan_sweeps(ctx, c, inc, specs, sw + part, count - part, skips, b2, s2);
                ctx->upload_plan(b2.data(), b2.size(), s2.data(), s2.size(), (size_t)part * nb);
                blocks.insert(blocks.end(), b2.begin(), b2.end());
                part = count;
            }
            // a band launch: the next K sweeps all pass hot_ok
            bool band_k = bandK && !hot_off && k + bandK <= count;
            for (int j = 0; band_k && j < bandK; j++) band_k = hot_ok(P, &blocks[(size_t)(k + j) * nb]);
            // a block launch: every descriptor of sweep j + 1 one sweep's stream length after sweep j's
            for (int j = 0; band_k && blockK && j + 1 < bandK; j++)
                for (int b = 0; band_k && b < nb; b++) {
                    const Block &x = blocks[(size_t)(k + j) * nb + b], &y = blocks[(size_t)(k + j + 1) * nb + b];
                    const u128 nx = apply(block_step, u128{x.base_lo, x.base_hi});
                    band_k = nx.lo == y.base_lo && nx.hi == y.base_hi && x.has == y.has;
                }
            const int step = band_k ? bandK : 1;
            const bool hot_k = band_k || (use_hot && !hot_off && NWv == 4 && hot_ok(P, &blocks[(size_t)k * nb]));
            int split_i = -1;  // this sweep's split replay
            if (!hot_k && !hot_off)
                for (size_t i = 0; i < splits.size(); i++)
                    if (splits[i].first == k) split_i = (int)i;
            const bool split_k = split_i >= 0;
            if (!hot_k && seg) {
                ctx->time_end(seg, k - seg_k0, seg_k0);
                seg = nullptr;
            }
            if (hot_k && !seg) {
                ctx->time_begin(&seg);
                seg_k0 = k;
            }
            FArgs A;
            A.P = P;
            A.G = FGeom{N, N, 0, 0, N, N, N, V, 0};
            A.phi_in = st->phi[st->cur ^ (k & 1)];
            A.n_in = st->n[st->cur ^ (k & 1)];
            A.phi_out = st->phi[st->cur ^ (k & 1) ^ 1];
            A.n_out = st->n[st->cur ^ (k & 1) ^ 1];
            A.nsx = nsx;
            A.TH = TH;
            A.nsy = nsy;
            A.blocks = ctx->d_blocks + (size_t)k * nb;
            A.skips = ctx->d_skips;
            A.T = T;
            A.adv[0] = adv[0];
            A.adv[1] = adv[1];
            A.adv[2] = adv[2];
            A.stat = ctx->d_stats + k;
            A.S = scratch(ctx);
            A.S.hflag = ctx->d_flag;
            A.progress = ctx->d_prog;
            A.sweep = (uint32_t)k;
            A.S.gate = band_gate;  // (band batches: a report gates the later launches by sweep)
            farg_single(A, nsx, nsy);
            if (band_k && blockK) {
                BlockArgs B;
                B.K = blockK;
                B.bs = blockBS;
                B.nbx = N / blockBS;
                B.nb = nb;
                B.step = block_step;
                B.phi[0] = st->phi[st->cur ^ (k & 1)];
                B.n[0] = st->n[st->cur ^ (k & 1)];
                for (int j = 1; j < blockK; j++) {
                    B.phi[j] = st->band_phi[j - 1];
                    B.n[j] = st->band_n[j - 1];
                }
                B.phi[blockK] = st->phi[st->cur ^ (k & 1) ^ 1];
                B.n[blockK] = st->n[st->cur ^ (k & 1) ^ 1];
                launch_block(A, B, ctx->stream);
                band_starts.push_back(k);
                ctx->sweeps_hot += blockK;
                ctx->sweeps_block += blockK;
                ctx->launches_block++;
            } else if (band_k) {
                A.hot_nw = 8;
                A.adv[0] = adv8[0];
                A.adv[1] = adv8[1];
                A.adv[2] = adv8[2];
                BandArgs B;
                B.K = bandK;
                B.P = bandP;
                B.own = N / nbands;
                B.TH = TH;
                B.gen = (int32_t)band_starts.size();
                B.nb = nb;
                B.nbands = nbands;
                B.ctrl = st->band_ctrl;
                B.phi[0] = st->phi[st->cur ^ (k & 1)];
                B.n[0] = st->n[st->cur ^ (k & 1)];
                for (int j = 1; j < bandK; j++) {
                    B.phi[j] = st->band_phi[j - 1];
                    B.n[j] = st->band_n[j - 1];
                }
                B.phi[bandK] = st->phi[st->cur ^ (k & 1) ^ 1];  // (K odd: the buffer k + K reads)
                B.n[bandK] = st->n[st->cur ^ (k & 1) ^ 1];
                launch_hot_band(A, B, ctx->stream);
                band_starts.push_back(k);
                ctx->sweeps_hot += bandK;
                ctx->sweeps_band += bandK;
                ctx->launches_band++;
            } else if (hot_k) {
                if (hot_nw == 8) {
                    A.hot_nw = 8;
                    A.adv[0] = adv8[0];
                    A.adv[1] = adv8[1];
                    A.adv[2] = adv8[2];
                }
                if (st->d_strips) A.strips = st->d_strips;
                launch_hot(A, st->d_strips ? st->n_strips : grid, ctx->stream);
                ctx->sweeps_hot++;
            } else if (split_k) {
                if (st->d_strips) A.strips = st->d_strips;
                SplitArgs &SA = splits[split_i].second;
                SA.blocksB = ctx->d_blocks + split_off[split_i];
                launch_hot_split(A, SA, st->d_strips ? st->n_strips : grid, ctx->stream);
                ctx->sweeps_split++;
            } else {
                ctx->sweeps_fused++;
                villain_sweep_fused<4, false, false, false><<<grid, 4 * 64, 0, ctx->stream>>>(A), SV_LAUNCHED("villain_sweep_fused<4, false, false, false>", ctx->stream);
            }
            if (per_launch && seg) {
                ctx->time_end(seg, step, k);
                seg = nullptr;
            }
            k += step;
            if (k >= next_chunk && k < count) {
                const int j = next_chunk / CH - 1;  // chunk j is enqueued
                next_chunk += CH;
                if (j >= 1) {
                    // chunk j - 1 has finished once the first launch of chunk j has started (FArgs::progress).  A
                    // stream event between the chunks did the same at ~6.5 us of idle GPU per event (its
                    // end-of-pipe release), 0.7% of a sweep; the host-mapped word costs the kernels one store.
                    // (no stream query while the chunk runs: a query between submissions left a ~6.5 us gap before
                    // the next chunk's first launch; only after ~20 ms, as a guard, is the stream asked)
                    const int32_t target = j * CH + 1;
                    const auto tw = std::chrono::steady_clock::now();
                    for (int spin = 0; __atomic_load_n(ctx->h_prog, __ATOMIC_ACQUIRE) < target; spin++) {
                        if (__atomic_load_n(ctx->h_flag, __ATOMIC_ACQUIRE)) break;
                        if ((spin & 1023) == 1023 && std::chrono::steady_clock::now() - tw > std::chrono::milliseconds(20) &&
                            hipStreamQuery(ctx->stream) == hipSuccess)
                            break;  // (drained: a launch that never stored its progress)
                        std::this_thread::yield();
                    }
                    if (__atomic_load_n(ctx->h_flag, __ATOMIC_ACQUIRE)) {
                        launched = k;  // the rest of the batch is not enqueued
                        break;
                    }
                }
            }
        }
        if (seg) ctx->time_end(seg, launched - seg_k0, seg_k0);
        SV_HIP(hipGetLastError());

        if (launched == count && sw + count < sweeps) {  // (the device runs this batch meanwhile)
            c_next = c;
            plan_sweeps(ctx, c_next, inc, specs, sw + count, std::min(BATCH, sweeps - sw - count), skips, blocks_next,
                        skipvec_next);
            sw_next = sw + count;
        }
        auto tp2 = std::chrono::steady_clock::now();
        const sv_stats *landed = nullptr;
        AbortInfo a = read_abort_stats(ctx, count, stats + sw, &landed);
        auto tp3 = std::chrono::steady_clock::now();
        if (dbg)
            fprintf(stderr, "[sv] launch %.1f us, wait %.1f us\n", std::chrono::duration<double, std::micro>(tp2 - tp1).count(),
                    std::chrono::duration<double, std::micro>(tp3 - tp2).count());
        // aborted launches exit early: only the timed segments that ended before the first failing sweep count
        if (a.abort) {
            uint32_t first = ~0u;
            for (const Report &r : a.reports) first = std::min(first, r.sweep);
            ctx->time_keep_before(first == ~0u ? 0 : first);
        }
        ctx->time_collect();
        if (!a.abort) {  // the stats already landed with the abort flag
            for (int k = 0; k < count; k++) {
                stats[sw + k].proposed = V;
                int64_t rj = 0;
                for (int bi = 0; bi < nb; bi++) {
                    auto it = skips.find({sw + k, bi});
                    if (it != skips.end()) rj += (int64_t)it->second.size();
                }
                stats[sw + k].rejections = rj;
            }
            cur = c;
            sw += count;
            set_current(count);
            continue;
        }
        // A failing sweep inside a band launch: the state before it is that launch's scratch output, not one of the
        // ping-pong pair -- copied to the buffer the replay reads (after set_current)
        auto restore_band = [&](int bad) {
            for (int k0 : band_starts) {
                if (bad > k0 && bad < k0 + bandK) {
                    const int j = bad - k0;
                    SV_HIP(hipMemcpyAsync(st->phi[st->cur], st->band_phi[j - 1], V * sizeof(double),
                                          hipMemcpyDeviceToDevice, ctx->stream));
                    SV_HIP(hipMemcpyAsync(st->n[st->cur], st->band_n[j - 1], 2 * V * sizeof(int64_t),
                                          hipMemcpyDeviceToDevice, ctx->stream));
                }
            }
        };
        sw_next = -1;  // (an abort changes the skips, or the kernel: the next batch is planned again)
        // earliest failing (sweep, block); an overflow tag sorts after every rejection of its sweep
        uint32_t first_bad = ~0u;
        bool overflow = false, band_fail = false;
        {
            std::pair<uint32_t, uint32_t> best{~0u, ~0u};
            for (const Report &r : a.reports)
                if (std::make_pair(r.sweep, r.block) < best) best = {r.sweep, r.block};
            first_bad = best.first;
            overflow = best.second == OVERFLOW_BLOCK;
            band_fail = best.second == BAND_FAIL_BLOCK;
        }
        // Multi-sweep launches report a rejected word once per workgroup that recomputes its site, from sweeps that run
        // concurrently; past MAX_REPORTS the reports are dropped in arrival order, so the earliest failing sweep (the
        // gate's atomic minimum) may have lost all of its reports.  Then the sweeps before the gate stand and the
        // rest of the call runs one sweep per launch, whose reports name the rejections anew.
        // (its own flag: a genuine BAND_FAIL_BLOCK report that arrives with more than MAX_REPORTS reports still takes the
        // process-wide band_broken path below)
        bool truncated = false;
        if (a.raw > (uint32_t)MAX_REPORTS && band_gate) {
            int32_t g = INT32_MAX;
            SV_HIP(hipMemcpy(&g, band_gate, sizeof(int32_t), hipMemcpyDeviceToHost));
            if (g >= 0 && (uint32_t)g < first_bad) {
                first_bad = (uint32_t)g;
                overflow = false;
                band_fail = false;
                truncated = true;  // (keep the sweeps before the gate, multi-sweep launches off for this call)
            }
        }
        if (truncated) {
            // (truncated reports, above: multi-sweep launches off for the rest of this call only)
            const int bad = (int)first_bad;
            if (bad > 0) {
                Cursor c2 = cur;
                std::vector<Block> b2;
                std::vector<uint32_t> s2;
                plan_sweeps(ctx, c2, inc, specs, sw, bad, skips, b2, s2);
                std::memcpy(stats + sw, landed, bad * sizeof(sv_stats));  // (landed with the batch's tail)
                for (int k = 0; k < bad; k++) {
                    stats[sw + k].proposed = V;
                    stats[sw + k].rejections = rejections_in(skips, sw + k, nb);
                }
                cur = c2;
            }
            set_current(bad);
            restore_band(bad);
            sw += bad;
            bandK = 0;
            band_gate = nullptr;
            continue;
        }
        if (band_fail) {
            // a band launch could not run as planned (tagged with its first sweep, whose input is intact): the
            // sweeps before it stand, and band launches are off for the rest of the process
            if (!band_broken.exchange(true))
                fprintf(stderr, "[sv] multi-sweep band launch failed (workgroups not spread over %d XCDs as planned, "
                                "or a band barrier timed out); single-sweep launches from here on\n", nbands);
            const int bad = (int)first_bad;
            if (bad > 0) {
                Cursor c2 = cur;
                std::vector<Block> b2;
                std::vector<uint32_t> s2;
                plan_sweeps(ctx, c2, inc, specs, sw, bad, skips, b2, s2);
                std::memcpy(stats + sw, landed, bad * sizeof(sv_stats));  // (landed with the batch's tail)
                for (int k = 0; k < bad; k++) {
                    stats[sw + k].proposed = V;
                    stats[sw + k].rejections = rejections_in(skips, sw + k, nb);
                }
                cur = c2;
            }
            set_current(bad);
            sw += bad;
            bandK = 0;
            band_gate = nullptr;
            continue;
        }
        if (overflow) {
            const int bad = (int)first_bad;
            const bool to_int32 = use_hot && !hot_off && NWv == 4;  // the failing sweep may have run on the int16 image
            if (bad > 0) {
                Cursor c2 = cur;
                std::vector<Block> b2;
                std::vector<uint32_t> s2;
                plan_sweeps(ctx, c2, inc, specs, sw, bad, skips, b2, s2);
                std::memcpy(stats + sw, landed, bad * sizeof(sv_stats));  // (landed with the batch's tail)
                for (int k = 0; k < bad; k++) {
                    stats[sw + k].proposed = V;
                    int64_t rj = 0;
                    for (int bi = 0; bi < nb; bi++) {
                        auto it = skips.find({sw + k, bi});
                        if (it != skips.end()) rj += (int64_t)it->second.size();
                    }
                    stats[sw + k].rejections = rj;
                }
                cur = c2;
            }
            set_current(bad);
            restore_band(bad);
            if (to_int32) {
                hot_off = true;
                sw += bad;
                continue;
            }
            done_sweeps = sw + bad;
            return false;
        }
        const int bad = absorb_reports(a, sw, skips);
        if (dbg) {
            fprintf(stderr, "[sv] abort at sweep %d of %d; reports:", bad, count);
            for (const Report &r : a.reports) fprintf(stderr, " (sweep %u block %u pos %u)", r.sweep, r.block, r.pos);
            fprintf(stderr, "\n");
        }
        // sweeps before `bad` in this batch are valid: keep them
        if (bad > 0) {
            Cursor c2 = cur;
            std::vector<Block> b2;
            std::vector<uint32_t> s2;
            plan_sweeps(ctx, c2, inc, specs, sw, bad, skips, b2, s2);
            std::memcpy(stats + sw, landed, bad * sizeof(sv_stats));  // (landed with the batch's tail)
            for (int k = 0; k < bad; k++) {
                stats[sw + k].proposed = V;
                int64_t rj = 0;
                for (int bi = 0; bi < nb; bi++) {
                    auto it = skips.find({sw + k, bi});
                    if (it != skips.end()) rj += (int64_t)it->second.size();
                }
                stats[sw + k].rejections = rj;
            }
            cur = c2;
        }
        set_current(bad);
        restore_band(bad);
        sw += bad;
    }
    done_sweeps = sweeps;
    return true;
}

}  // namespace svh

using namespace svh;

// ---------------------------------------------------------------------------- C-ABI (Villain)
extern "C" {

int sv_villain_create(sv_ctx *ctx, int32_t N, sv_villain **out) {
    try {
        if (!ctx || !out) return -1;
        if (N < 2) throw std::invalid_argument("N must be >= 2");
        SV_HIP(hipSetDevice(ctx->device));
        sv_villain *st = new sv_villain();
        st->ctx = ctx;
        st->N = N;
        const size_t V = (size_t)N * N;
        for (int i = 0; i < 2; i++) {
            SV_HIP(hipMalloc(&st->phi[i], V * sizeof(double)));
            SV_HIP(hipMalloc(&st->n[i], 2 * V * sizeof(int64_t)));
        }
        SV_HIP(hipMalloc(&st->r, 2 * V * sizeof(double)));
        SV_HIP(hipMalloc(&st->snap_phi, V * sizeof(double)));
        SV_HIP(hipMalloc(&st->snap_n, 2 * V * sizeof(int64_t)));
        std::vector<int32_t> sites;
        st->ncol = build_colors(N, sites, st->count, st->offset);
        SV_HIP(hipMalloc(&st->sites, sites.size() * sizeof(int32_t)));
        SV_HIP(hipMemcpy(st->sites, sites.data(), sites.size() * sizeof(int32_t), hipMemcpyHostToDevice));
        *out = st;
        return 0;
    } catch (const std::exception &e) {
        if (ctx) ctx->err = e.what();
        return -2;
    }
}

int sv_villain_destroy(sv_villain *st) {
    if (!st) return 0;
    int rc = sv_destroy_drain(st->ctx, "sv_villain_destroy");  // (no queued work may still use the buffers)
    for (int i = 0; i < 2; i++) {
        (void)hipFree(st->phi[i]);
        (void)hipFree(st->n[i]);
    }
    (void)hipFree(st->r);
    (void)hipFree(st->snap_phi);
    (void)hipFree(st->snap_n);
    (void)hipFree(st->sites);
    if (st->d_aux) (void)hipFree(st->d_aux);
    if (st->h_aux) (void)hipHostFree(st->h_aux);
    if (st->d_obs) (void)hipFree(st->d_obs);
    if (st->d_strips) (void)hipFree(st->d_strips);
    for (double *p : st->band_phi) (void)hipFree(p);
    for (int64_t *p : st->band_n) (void)hipFree(p);
    if (st->band_ctrl) (void)hipFree(st->band_ctrl);
    if (st->h_obs) (void)hipHostFree(st->h_obs);
    const hipError_t ee = st->emitter.release();
    if (ee != hipSuccess && !rc) {
        st->ctx->err = std::string("sv_villain_destroy: an emission copy failed: ") + hipGetErrorString(ee);
        rc = -2;
    }
    delete st;
    return rc;
}

int sv_villain_upload(sv_villain *st, const double *phi, const int64_t *n) {
    try {
        const size_t V = (size_t)st->N * st->N;
        SV_HIP(hipSetDevice(st->ctx->device));
        SV_HIP(hipMemcpyAsync(st->phi[st->cur], phi, V * sizeof(double), hipMemcpyHostToDevice, st->ctx->stream));
        SV_HIP(hipMemcpyAsync(st->n[st->cur], n, 2 * V * sizeof(int64_t), hipMemcpyHostToDevice, st->ctx->stream));
        SV_HIP(hipStreamSynchronize(st->ctx->stream));
        return 0;
    } catch (const std::exception &e) {
        st->ctx->err = e.what();
        return -2;
    }
}

int sv_villain_download(sv_villain *st, double *phi, int64_t *n) {
    try {
        const size_t V = (size_t)st->N * st->N;
        SV_HIP(hipSetDevice(st->ctx->device));
        SV_HIP(hipMemcpyAsync(phi, st->phi[st->cur], V * sizeof(double), hipMemcpyDeviceToHost, st->ctx->stream));
        SV_HIP(hipMemcpyAsync(n, st->n[st->cur], 2 * V * sizeof(int64_t), hipMemcpyDeviceToHost, st->ctx->stream));
        SV_HIP(hipStreamSynchronize(st->ctx->stream));
        return 0;
    } catch (const std::exception &e) {
        st->ctx->err = e.what();
        return -2;
    }
}

int sv_villain_run(sv_villain *st, double kappa, int64_t W, double interval_phi, int64_t interval_n, int32_t sweeps,
                   sv_rng *rng, sv_stats *stats, int32_t path) {
    if (!st || !rng || (sweeps > 0 && !stats)) return -1;
    sv_ctx *ctx = st->ctx;
    try {
        if (sweeps < 0) throw std::invalid_argument("sweeps must be >= 0");
        if (interval_n < 0) throw std::invalid_argument("interval_n must be >= 0");
        if (interval_n > (1 << 20)) throw std::invalid_argument("interval_n too large");
        SV_HIP(hipSetDevice(ctx->device));
        VParams P = make_params(st->N, kappa, W, interval_phi, interval_n);
        u128 inc{rng->inc_lo, rng->inc_hi};
        Cursor cur{u128{rng->state_lo, rng->state_hi}, (uint32_t)rng->has_uint32, rng->uinteger};
        const bool small_dn = (W < 0 ? -W : W) * interval_n < (1LL << 28);
        bool use_fused = path == 2 || (path == 0 && fused_ok(st->N) && small_dn);
        if (path == 2 && !fused_ok(st->N)) throw std::invalid_argument("fused path needs even N >= 4");
        int done = 0;
        if (use_fused && sweeps > 0) {
            // run as many sweeps as possible fused; on int32 overflow fall back for the rest
            bool all = run_fused(st, P, sweeps, cur, inc, stats, done);
            if (!all && path == 2) throw std::runtime_error("|n| exceeds the fused path's int32 LDS image (|n| < 2^30 required)");
        }
        if (done < sweeps) {
            // generic path works on phi[cur], n[cur] in place
            run_generic(st, P, sweeps - done, cur, inc, stats + done);
        }
        rng->state_hi = cur.s.hi;
        rng->state_lo = cur.s.lo;
        rng->has_uint32 = (int32_t)cur.has;
        rng->uinteger = cur.buf;
        return 0;
    } catch (const std::exception &e) {
        ctx->err = e.what();
        return -2;
    }
}

// The optional counter-based mode (SURVEY.md 8(b) sv_rng mode 1): the same fused sweep with Philox draws by
// (site, sweep, slot).  Nothing to plan and no NumPy Lemire rejection to replay (a rejected choice word is
// redrawn in place), so a batch of sweeps is launched back to back with one synchronization at its end.
int sv_villain_run_philox(sv_villain *st, double kappa, int64_t W, double interval_phi, int64_t interval_n,
                          int32_t sweeps, sv_philox *rng, sv_stats *stats) {
    if (!st || !rng || (sweeps > 0 && !stats)) return -1;
    sv_ctx *ctx = st->ctx;
    try {
        if (sweeps < 0) throw std::invalid_argument("sweeps must be >= 0");
        if (interval_n < 0 || interval_n > (1 << 20)) throw std::invalid_argument("interval_n out of range");
        const int32_t N = st->N;
        const int64_t V = (int64_t)N * N;
        if (!fused_ok(N)) throw std::invalid_argument("the counter-based mode needs an even N >= 4");
        if (V >= (int64_t(1) << 32)) throw std::invalid_argument("the counter-based mode addresses sites by 32 bits");
        VParams P = make_params(N, kappa, W, interval_phi, interval_n);
        if (rng->test_threshold) P.thr = rng->test_threshold;
        if (P.k < 2 || !hot_params_ok(P))
            throw std::invalid_argument("the counter-based mode needs interval_n >= 1, |W| <= 2^12 and |W| interval_n <= 2^13");
        SV_HIP(hipSetDevice(ctx->device));
        const int nsx = (N + FW_MAX - 1) / FW_MAX;
        const int TH = fused_th(N, nsx);
        const int nsy = (N + TH - 1) / TH;
        const int grid = nsx * nsy;
        const int BATCH = 64;
        for (int sw = 0; sw < sweeps;) {
            const int count = std::min(BATCH, sweeps - sw);
            ctx->ensure_stats(count);
            reset_batch(ctx, ctx->d_stats, count * sizeof(sv_stats));
            hipEvent_t ev;
            ctx->time_begin(&ev);
            for (int k = 0; k < count; k++) {
                FArgs A;
                A.P = P;
                A.G = FGeom{N, N, 0, 0, N, N, N, V, 0};
                A.phi_in = st->phi[st->cur];
                A.n_in = st->n[st->cur];
                A.phi_out = st->phi[st->cur ^ 1];
                A.n_out = st->n[st->cur ^ 1];
                A.nsx = nsx;
                A.TH = TH;
                A.nsy = nsy;
                A.blocks = nullptr;
                A.skips = nullptr;
                A.T = nullptr;
                A.stat = ctx->d_stats + k;
                A.S = scratch(ctx);
                A.sweep = (uint32_t)k;
                A.ph_key = rng->key;
                A.ph_sweep = rng->counter + (uint64_t)(sw + k);
                farg_single(A, nsx, nsy);
                launch_hot_ph(A, grid, ctx->stream);
                st->cur ^= 1;
            }
            ctx->time_end(ev, count);
            SV_HIP(hipGetLastError());
            AbortInfo a = read_abort_stats(ctx, count, stats + sw);
            ctx->time_collect();
            if (a.abort) {
                // the only report this kernel makes: |n| beyond its int16 image (|n| >= 2^14).  The ping-pong
                // buffers have been overwritten by the batch, so the fields are unspecified after this error
                // (re-upload before the next call); the counter is not advanced.
                throw std::runtime_error("|n| exceeds the counter-based mode's int16 image (|n| < 2^14 required); "
                                         "fields unspecified, re-upload");
            }
            for (int k = 0; k < count; k++) {
                stats[sw + k].proposed = V;
                stats[sw + k].rejections = 0;
            }
            sw += count;
        }
        rng->counter += (uint64_t)sweeps;
        return 0;
    } catch (const std::exception &e) {
        ctx->err = e.what();
        return -2;
    }
}

int sv_villain_neighborhood(sv_ctx *ctx, int32_t N, double kappa, int64_t W, double interval_phi, int64_t interval_n,
                            double *phi, int64_t *n, int32_t sweeps, sv_rng *rng, sv_stats *stats) {
    sv_villain *st = nullptr;
    int rc = sv_villain_create(ctx, N, &st);
    if (rc) return rc;
    rc = sv_villain_upload(st, phi, n);
    if (!rc) rc = sv_villain_run(st, kappa, W, interval_phi, interval_n, sweeps, rng, stats, 0);
    if (!rc) rc = sv_villain_download(st, phi, n);
    sv_villain_destroy(st);
    return rc;
}

int sv_villain_observables(sv_villain *st, double kappa, double *out) {
    try {
        sv_ctx *ctx = st->ctx;
        SV_HIP(hipSetDevice(ctx->device));
        // persistent device sums + pinned host image: a stream-ordered DMA, then a host copy after the sync
        // (a pooled hipMallocAsync buffer read back into pageable memory once returned zeros)
        if (!st->d_obs) {
            SV_HIP(hipMalloc((void **)&st->d_obs, OBS_WORDS * sizeof(unsigned long long)));
            SV_HIP(hipHostMalloc((void **)&st->h_obs, OBS_WORDS * sizeof(unsigned long long), hipHostMallocDefault));
        }
        unsigned long long *d = st->d_obs;
        SV_HIP(hipMemsetAsync(d, 0, OBS_WORDS * sizeof(unsigned long long), ctx->stream));
        const int64_t V = (int64_t)st->N * st->N;
        // <= 256 sites per thread (the exact action values of a thread stay below 2^60)
        const int grid = (int)std::max<int64_t>(std::min<int64_t>((V + 255) / 256, 2048), (V + 65535) / 65536);
        villain_observables_kernel<<<grid, 256, 0, ctx->stream>>>(st->N, st->phi[st->cur], st->n[st->cur], d),
            SV_LAUNCHED("villain_observables_kernel", ctx->stream);
        SV_HIP(hipGetLastError());
        SV_HIP(hipMemcpyAsync(st->h_obs, d, OBS_WORDS * sizeof(unsigned long long), hipMemcpyDeviceToHost, ctx->stream));
        SV_HIP(hipStreamSynchronize(ctx->stream));
        double raw[4];
        obs_raw(st->h_obs, raw);
        out[0] = kappa / 2.0 * raw[0];  // S = kappa / 2 sum (d phi - 2 pi n)^2 (villain.py:51-66)
        out[1] = raw[1];
        out[2] = raw[2];
        out[3] = raw[3];
        return 0;
    } catch (const std::exception &e) {
        st->ctx->err = e.what();
        return -2;
    }
}

}  // extern "C"
