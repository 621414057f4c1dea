// villain_local.hip -- the remaining local Villain updates of SURVEY.md 8(f) on gfx950, each a
// bit-exact replay of the reference chain under a fixed NumPy seed:
//
//   SiteUpdate        supervillain/generator/villain/site.py:43-120        phi only, checkerboard
//   LinkUpdate        supervillain/generator/villain/link.py:53-101        every link at once
//   ExactUpdate       supervillain/generator/villain/exact.py:50-129       n += d(z), checkerboard
//   CohomologyUpdate  supervillain/generator/villain/cohomology.py:64-117  one slice per direction
//
// Site/Exact/Link are colour (or whole-lattice) passes in which a lane owns one colour site (one
// link) per iteration of a grid-stride loop.  The grid stride S is chosen so that every draw a lane
// consumes sits at an arithmetic sequence of NumPy stream positions: the lane jumps once (4-level
// table) to its first draw of a block and then advances by ONE precomputed affine map per
// iteration (S, 2S or S/2 PCG64 steps).  Blocks holding known Lemire rejections (rare: only for
// interval counts that are not powers of two) take the per-element full-jump path instead.
//
// Floating point follows the reference op by op (-ffp-contract=off):
//   d(x) on link (mu,s):  0.0 + (x[s+e] - x[s])                            (lattice/reference.py:9-24)
//   Site dS_link:         ((kappa/2) * cd) * ((2 * (dphi - (2pi)*n)) + cd)  (site.py:94)
//   Site dphi update:     dphi + (0.0 + (cphi[s+e] - cphi[s]))             (site.py:111)
//   Exact/Link dS_link:   ((-2pi*kappa) * cn) * ((dphi - (2pi)*n) - pi*cn)  (exact.py:95-98, link.py:78-81)
//   face_sum:             (((0 + f0[x]) + f0[x-e0]) + f1[x]) + f1[x-e1]    (reference.py:48-64)
//   Cohomology dS:        NumPy pairwise float64 sum over the slice        (cohomology.py:97)
#include <cstdio>

#include "local.h"

namespace sv {

#define LTWO_PI 6.283185307179586  // 2 * np.pi
#define LPI 3.141592653589793      // np.pi

struct LParams {
    int32_t N;
    int64_t V;
    double half_kappa;   // Site: kappa / 2
    double m2pik;        // Exact/Link: -2 * np.pi * kappa
    double lo, range;    // Site: uniform(-interval_phi, +interval_phi) as low, high - low
    int64_t W;           // Link: change_n = W * choice(...)
    int64_t iv;          // Link/Exact: values (-iv .. -1, 1 .. iv)
    uint32_t k, thr;     // choice over 2 iv values: Lemire bound and threshold
};

using namespace loc;

// ------------------------------------------------------------------------------------------------
// d(phi) into D (2, N, N) at the start of a Site sweep (site.py:81) or an Exact call (exact.py:71);
// `normalize` also stores phi + 0.0 (every site receives phi + change_phi with change_phi = +0.0 in
// some colour pass of the reference, which maps -0.0 to +0.0).
__global__ void local_dphi_init(int32_t N, double *phi, double *D, int normalize, const int32_t *abort) {
    if (*(volatile const int32_t *)abort) return;
    const int64_t V = (int64_t)N * N;
    for (int64_t s = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; s < V; s += (int64_t)gridDim.x * blockDim.x) {
        int64_t t, x;
        divmod_site(s, N, t, x);
        const double p = phi[s];
        D[s] = 0.0 + (phi[((t + 1 == N) ? 0 : t + 1) * N + x] - p);
        D[V + s] = 0.0 + (phi[t * N + ((x + 1 == N) ? 0 : x + 1)] - p);
        if (normalize && p == 0.0 && __signbit(p)) phi[s] = p + 0.0;  // only -0.0 changes
    }
}

// One colour pass of SiteUpdate (site.py:83-111).  Blocks: [0] metropolis uniform(V), [1 + c] the
// colour's uniform(-interval_phi, interval_phi, n_c).  EVEN: colour sites computed from e, stride
// S = grid threads (a multiple of N, so metropolis positions advance by exactly 2S).
template <bool EVEN>
__global__ __launch_bounds__(256) void site_pass(LParams P, double *phi, const int64_t *n, double *D,
                                                 const int32_t *sites, int64_t nc, int color, const Block *blocks,
                                                 const JumpTables *T, Affine adv_m, Affine adv_e, sv_stats *stat,
                                                 const int32_t *abort) {
    if (*(volatile const int32_t *)abort) return;
    const int64_t N = P.N, V = P.V;
    const int64_t S = (int64_t)gridDim.x * blockDim.x;
    const Block BM = blocks[0], BD = blocks[1 + color];
    UniLane um{u128{0, 0}, false}, ud{u128{0, 0}, false};
    int64_t acc_count = 0;
    AccFx psum;  // exact acceptance sum (common.h)
    for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < nc; e += S) {
        const int64_t s = EVEN ? even_site(e, N, color) : sites[e];
        if (!EVEN) um.init = ud.init = false;
        const double u = 0.0 + 1.0 * to_double(um.next(T, BM, (uint32_t)s, adv_m));
        const double dph = P.lo + P.range * to_double(ud.next(T, BD, (uint32_t)e, adv_e));
        int64_t t, x;
        divmod_site(s, N, t, x);
        const int64_t L[4] = {s, ((t == 0) ? N - 1 : t - 1) * N + x, V + s, V + t * N + ((x == 0) ? N - 1 : x - 1)};
        const double cd_f = 0.0 + (0.0 - dph), cd_b = 0.0 + (dph - 0.0);
        double dv[4];
        int64_t nv[4];
#pragma unroll
        for (int q = 0; q < 4; q++) {
            dv[q] = D[L[q]];
            nv[q] = n[L[q]];
        }
        double dS = 0.0;
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const double cd = (q & 1) ? cd_b : cd_f;
            dS += (P.half_kappa * cd) * ((2.0 * (dv[q] - LTWO_PI * (double)nv[q])) + cd);
        }
        const double p = clip01(exp(-dS));
        const int acc = u < p;
        acc_count += acc;
        fx_add(psum, p);
        const double cphi = dph * (double)acc;
        phi[s] = phi[s] + cphi;
        const double dcf = 0.0 + (0.0 - cphi), dcb = 0.0 + (cphi - 0.0);
#pragma unroll
        for (int q = 0; q < 4; q++) D[L[q]] = dv[q] + ((q & 1) ? dcb : dcf);
    }
    lflush(stat, acc_count, psum);
}

// SiteUpdate for even N without a dphi array: pass 0 forms dphi = d(phi) from the sweep-start phi on the
// fly, decides colour 0 and keeps its accepted changes cphi0 (compact, colour index); pass 1 rebuilds the
// reference's incrementally updated dphi on its links as d(phi_start) + d(cphi0) (site.py:111) from the
// same sweep-start phi and cphi0.  phi is ping-ponged (phi_in stays the sweep-start field):
//   colour 0: (phi + cphi0) + 0.0,  colour 1: (phi + 0.0) + cphi1   (site.py:110, both colour passes)
template <int PASS>
__global__ __launch_bounds__(256) void site_pp(LParams P, const double *phi_in, double *phi_out, const int64_t *n,
                                               double *cbuf, const Block *blocks, const JumpTables *T, Affine adv_m,
                                               Affine adv_e, sv_stats *stat, const int32_t *abort) {
    if (*(volatile const int32_t *)abort) return;
    const int64_t N = P.N, V = P.V, nc = P.V >> 1;
    const int64_t S = (int64_t)gridDim.x * blockDim.x;
    const Block BM = blocks[0], BD = blocks[1 + PASS];
    UniLane um{u128{0, 0}, false}, ud{u128{0, 0}, false};
    int64_t acc_count = 0;
    AccFx psum;  // exact acceptance sum (common.h)
    for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < nc; e += S) {
        const int64_t s = even_site(e, N, PASS);
        const double u = 0.0 + 1.0 * to_double(um.next(T, BM, (uint32_t)s, adv_m));
        const double dph = P.lo + P.range * to_double(ud.next(T, BD, (uint32_t)e, adv_e));
        int64_t t, x;
        divmod_site(s, N, t, x);
        const int64_t f0 = ((t + 1 == N) ? 0 : t + 1) * N + x, b0 = ((t == 0) ? N - 1 : t - 1) * N + x;
        const int64_t f1 = t * N + ((x + 1 == N) ? 0 : x + 1), b1 = t * N + ((x == 0) ? N - 1 : x - 1);
        const double ps = phi_in[s];
        double D[4] = {0.0 + (phi_in[f0] - ps), 0.0 + (ps - phi_in[b0]), 0.0 + (phi_in[f1] - ps),
                       0.0 + (ps - phi_in[b1])};
        if (PASS == 1) {
            D[0] = D[0] + (0.0 + (cbuf[f0 >> 1] - 0.0));
            D[1] = D[1] + (0.0 + (0.0 - cbuf[b0 >> 1]));
            D[2] = D[2] + (0.0 + (cbuf[f1 >> 1] - 0.0));
            D[3] = D[3] + (0.0 + (0.0 - cbuf[b1 >> 1]));
        }
        const int64_t L[4] = {s, b0, V + s, V + b1};
        const double cd_f = 0.0 + (0.0 - dph), cd_b = 0.0 + (dph - 0.0);
        double dS = 0.0;
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const double cd = (q & 1) ? cd_b : cd_f;
            dS += (P.half_kappa * cd) * ((2.0 * (D[q] - LTWO_PI * (double)n[L[q]])) + cd);
        }
        const double p = clip01(exp(-dS));
        const int acc = u < p;
        acc_count += acc;
        fx_add(psum, p);
        const double cphi = dph * (double)acc;
        if (PASS == 0) {
            phi_out[s] = (ps + cphi) + 0.0;
            cbuf[e] = cphi;
        } else {
            phi_out[s] = (ps + 0.0) + cphi;
        }
    }
    lflush(stat, acc_count, psum);
}

// One colour pass of ExactUpdate (exact.py:85-115).  Blocks: [0] metropolis uniform(V), [1 + c] the
// colour's choice(zs, n_c).  dphi = d(phi) is fixed for the call, so it is formed on the fly from phi
// (bit-identical to the reference's array, and 16 B/site less traffic than keeping it in HBM).
template <bool EVEN>
__global__ __launch_bounds__(256) void exact_pass(LParams P, int64_t *n, const double *phi, const int32_t *sites,
                                                  int64_t nc, int color, const Block *blocks, const uint32_t *skips,
                                                  const JumpTables *T, Affine adv_m, Affine adv_half, sv_stats *stat,
                                                  DevScratch Sx, uint32_t sweep) {
    if (*(volatile const int32_t *)Sx.abort) return;
    const int64_t N = P.N, V = P.V;
    const int64_t S = (int64_t)gridDim.x * blockDim.x;
    const Block BM = blocks[0], BZ = blocks[1 + color];
    const bool slow = BZ.nskip > 0;
    UniLane um{u128{0, 0}, false};
    BndLane uz{u128{0, 0}, false};
    int64_t acc_count = 0;
    AccFx psum;  // exact acceptance sum (common.h)
    for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < nc; e += S) {
        const int64_t s = EVEN ? even_site(e, N, color) : sites[e];
        if (!EVEN) um.init = uz.init = false;
        const double u = 0.0 + 1.0 * to_double(um.next(T, BM, (uint32_t)s, adv_m));
        uint32_t q = (uint32_t)e, w;
        if (slow) w = bnd_word_slow(T, BZ, skips, (uint32_t)e, &q);
        else w = uz.next(T, BZ, (uint32_t)e, adv_half);
        bool rej;
        const uint32_t idx = lemire(w, P.k, P.thr, &rej);
        if (rej) lreport(Sx, sweep, 1u + (uint32_t)color, q);
        const int64_t z = nonzero_value(idx, P.iv);
        int64_t t, x;
        divmod_site(s, N, t, x);
        const int64_t L[4] = {s, ((t == 0) ? N - 1 : t - 1) * N + x, V + s, V + t * N + ((x == 0) ? N - 1 : x - 1)};
        const int64_t cn_f = 0 + (0 - z), cn_b = 0 + (z - 0);
        // d(phi) on the four links, exactly as d() forms it (phi is fixed during the update, exact.py:71)
        const double ps = phi[s];
        const double D[4] = {0.0 + (phi[((t + 1 == N) ? 0 : t + 1) * N + x] - ps), 0.0 + (ps - phi[L[1]]),
                             0.0 + (phi[t * N + ((x + 1 == N) ? 0 : x + 1)] - ps), 0.0 + (ps - phi[L[3] - V])};
        int64_t nv[4];
        double dS = 0.0;
#pragma unroll
        for (int q4 = 0; q4 < 4; q4++) {
            nv[q4] = n[L[q4]];
            const double cn = (double)((q4 & 1) ? cn_b : cn_f);
            dS += (P.m2pik * cn) * ((D[q4] - LTWO_PI * (double)nv[q4]) - LPI * cn);
        }
        const double p = clip01(exp(-dS));
        const int acc = u < p;
        acc_count += acc;
        fx_add(psum, p);
        if (acc) {
#pragma unroll
            for (int q4 = 0; q4 < 4; q4++) n[L[q4]] = nv[q4] + ((q4 & 1) ? cn_b : cn_f);
        }
    }
    lflush(stat, acc_count, psum);
}

// One LinkUpdate sweep (link.py:66-99).  Blocks: [0] choice(n_changes, (2,N,N)), [1] uniform(0,1,(2,N,N)).
// Link l = mu V + s; grid stride S is even, so bounded words advance by S/2 and uniforms by S.
__global__ __launch_bounds__(256) void link_sweep(LParams P, const double *phi, int64_t *n, const Block *blocks,
                                                  const uint32_t *skips, const JumpTables *T, Affine adv_u,
                                                  Affine adv_half, sv_stats *stat, DevScratch Sx, uint32_t sweep) {
    if (*(volatile const int32_t *)Sx.abort) return;
    const int64_t N = P.N, V = P.V;
    const int64_t S = (int64_t)gridDim.x * blockDim.x;
    const Block BC = blocks[0], BU = blocks[1];
    const bool slow = BC.nskip > 0;
    UniLane uu{u128{0, 0}, false};
    BndLane uc{u128{0, 0}, false};
    int64_t acc_count = 0;
    AccFx psum;  // exact acceptance sum (common.h)
    for (int64_t l = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; l < 2 * V; l += S) {
        uint32_t q = (uint32_t)l, w;
        if (slow) w = bnd_word_slow(T, BC, skips, (uint32_t)l, &q);
        else w = uc.next(T, BC, (uint32_t)l, adv_half);
        bool rej;
        const uint32_t idx = lemire(w, P.k, P.thr, &rej);
        if (rej) lreport(Sx, sweep, 0u, q);
        const int64_t cn = P.W * nonzero_value(idx, P.iv);
        const int mu = l >= V;
        const int64_t s = l - (mu ? V : 0);
        int64_t t, x;
        divmod_site(s, N, t, x);
        const int64_t f = mu ? t * N + ((x + 1 == N) ? 0 : x + 1) : ((t + 1 == N) ? 0 : t + 1) * N + x;
        const double dphi = 0.0 + (phi[f] - phi[s]);
        const int64_t nl = n[l];
        const double dS = (P.m2pik * (double)cn) * ((dphi - LTWO_PI * (double)nl) - LPI * (double)cn);
        const double p = clip01(exp(-dS));
        const double u = 0.0 + 1.0 * to_double(uu.next(T, BU, (uint32_t)l, adv_u));
        const int acc = u < p;
        acc_count += acc;
        fx_add(psum, p);
        if (acc) n[l] = nl + cn;
    }
    lflush(stat, acc_count, psum);
}

// ------------------------------------------------------------------------------------------------
// CohomologyUpdate (cohomology.py:79-117), every sweep of a call in one workgroup.  Per sweep and
// direction mu: h = choice(h) (one bounded uint32), dS = pairwise sum over the N links of the slice
// x_mu = 0 of ((kappa/2) change_r) (2 r + change_r), then one uniform(0,1); on acceptance n += h on
// the slice.  The few draws are made serially by thread 0 on the live PCG64 state.
struct CohoRng {
    uint64_t s_lo, s_hi, inc_lo, inc_hi;
    uint32_t has, buf;
};

// NumPy pairwise_sum plan for one length: leaves (start, len <= 128) in recursion order and a
// postfix program (0 = push next leaf, 1 = add the top two).
struct PairwisePlan {
    int32_t nleaf, nprog;
};
static constexpr int MAX_LEAVES = 2048;
// slices up to this length have all their terms formed at once by every thread into LDS (the loads of a mu = 1
// slice, one row apart each, then overlap); the leaves' sums then read LDS in NumPy's order
static constexpr int COHO_LDS_TERMS = 4096;

__device__ __forceinline__ uint64_t coho_u64(u128 &s, const u128 &inc) {
    s = add(mul(s, mult()), inc);
    return xsl_rr(s);
}

__global__ __launch_bounds__(256) void cohomology_run(int32_t N, double half_kappa, int64_t ih, uint32_t k,
                                                      uint32_t thr, const double *phi, int64_t *n,
                                                      int32_t sweeps, CohoRng *rng, sv_stats *stats,
                                                      const int32_t *leaves /* 2 per leaf */,
                                                      const uint8_t *prog, PairwisePlan plan) {
    __shared__ double leafv[MAX_LEAVES];
    __shared__ double s_terms[COHO_LDS_TERMS];
    __shared__ uint8_t s_prog[2 * MAX_LEAVES];
    __shared__ double s_stk[64];
    __shared__ double s_dS;
    __shared__ int64_t s_h;
    __shared__ int s_acc;
    const int64_t V = (int64_t)N * N;
    u128 st{rng->s_lo, rng->s_hi}, inc{rng->inc_lo, rng->inc_hi};
    uint32_t has = rng->has, buf = rng->buf;
    // the postfix program in LDS: thread 0 walks it once per direction and sweep (from global memory every step
    // of the walk waited on a load)
    for (int pc = threadIdx.x; pc < plan.nprog; pc += blockDim.x) s_prog[pc] = prog[pc];
    __syncthreads();
    for (int32_t sw = 0; sw < sweeps; sw++) {
        int64_t accepted = 0, rejections = 0;
        double psum = 0.0;
        for (int mu = 0; mu < 2; mu++) {
            if (threadIdx.x == 0) {
                uint32_t idx;
                for (;;) {  // buffered 32-bit Lemire (NumPy), rejections draw again
                    uint32_t x;
                    if (has) {
                        x = buf;
                        has = 0;
                    } else {
                        const uint64_t X = coho_u64(st, inc);
                        x = (uint32_t)X;
                        buf = (uint32_t)(X >> 32);
                        has = 1;
                    }
                    bool rej;
                    idx = lemire(x, k, thr, &rej);
                    if (!rej) break;
                    rejections++;
                }
                s_h = nonzero_value(idx, ih);
            }
            __syncthreads();
            const int64_t h = s_h;
            const double change_r = -LTWO_PI * (double)h;  // cohomology.py:94
            const double a = half_kappa * change_r;
            // leaves: slice x_mu = 0 is n[0, 0, i] (mu = 0) or n[1, i, 0] (mu = 1)
            auto term_at = [&](int64_t i) {
                const int64_t s = mu == 0 ? i : i * N;
                const int64_t fs = mu == 0 ? N + i : i * N + 1;  // s + e_mu (N >= 2: no wrap)
                const double r = (0.0 + (phi[fs] - phi[s])) - LTWO_PI * (double)n[(int64_t)mu * V + s];
                return a * ((2.0 * r) + change_r);
            };
            const bool in_lds = N <= COHO_LDS_TERMS;
            if (in_lds) {
#pragma unroll 8
                for (int64_t i = threadIdx.x; i < N; i += blockDim.x) s_terms[i] = term_at(i);
                __syncthreads();
            }
            for (int j = threadIdx.x; j < plan.nleaf; j += blockDim.x) {
                const int32_t i0 = leaves[2 * j], len = leaves[2 * j + 1];
                auto term = [&](int64_t i) { return in_lds ? s_terms[i] : term_at(i); };
                double res;
                if (len < 8) {
                    res = 0.0;
                    for (int i = 0; i < len; i++) res += term(i0 + i);
                } else {
                    double r8[8];
#pragma unroll
                    for (int q = 0; q < 8; q++) r8[q] = term(i0 + q);
                    int i = 8;
                    for (; i < len - (len % 8); i += 8)
#pragma unroll
                        for (int q = 0; q < 8; q++) r8[q] += term(i0 + i + q);
                    res = ((r8[0] + r8[1]) + (r8[2] + r8[3])) + ((r8[4] + r8[5]) + (r8[6] + r8[7]));
                    for (; i < len; i++) res += term(i0 + i);
                }
                leafv[j] = res;
            }
            __syncthreads();
            if (threadIdx.x == 0) {
                // (the stack in LDS: a private array indexed at run time lives in scratch memory)
                int top = 0, nl = 0;
                for (int pc = 0; pc < plan.nprog; pc++) {
                    if (s_prog[pc] == 0) s_stk[top++] = leafv[nl++];
                    else {
                        const double b = s_stk[--top];
                        s_stk[top - 1] = s_stk[top - 1] + b;
                    }
                }
                const double dS = s_stk[0];
                const double p = clip01(exp(-dS));
                const double u = 0.0 + 1.0 * to_double(coho_u64(st, inc));  // cohomology.py:100
                s_acc = u < p;
                s_dS = p;
            }
            __syncthreads();
            if (s_acc) {
                for (int64_t i = threadIdx.x; i < N; i += blockDim.x) {
                    const int64_t s = mu == 0 ? i : i * N;
                    n[(int64_t)mu * V + s] += h;
                }
            }
            accepted += s_acc;
            psum += s_dS;
            __syncthreads();
        }
        if (threadIdx.x == 0) {
            stats[sw].accepted = accepted;
            stats[sw].proposed = 2;
            stats[sw].acceptance_sum = psum;
            stats[sw].rejections = rejections;
        }
    }
    if (threadIdx.x == 0) {
        rng->s_lo = st.lo;
        rng->s_hi = st.hi;
        rng->has = has;
        rng->buf = buf;
    }
}

}  // namespace sv

// ==================================================================================================
// host drivers
// ==================================================================================================
namespace svh {

static LParams lparams(int32_t N) {
    LParams P{};
    P.N = N;
    P.V = (int64_t)N * N;
    return P;
}

static void set_bounded(LParams &P, int64_t iv) {
    if (iv < 1) throw std::invalid_argument("the interval must be >= 1");
    if (iv > (1 << 20)) throw std::invalid_argument("interval too large");
    P.iv = iv;
    P.k = (uint32_t)(2 * iv);
    P.thr = (uint32_t)((0u - P.k) % P.k);
}

using namespace loc;

// Villain state: the snapshot is (phi, n) as the update touches them
template <class LaunchSweep>
static void run_local(sv_villain *st, const std::vector<BlockSpec> &specs, int32_t sweeps, Cursor &cur, u128 inc,
                      sv_stats *stats, bool may_reject, bool touches_phi, bool touches_n, LaunchSweep launch_sweep) {
    sv_ctx *ctx = st->ctx;
    const int64_t V = (int64_t)st->N * st->N;
    double *phi = st->phi[st->cur];
    int64_t *n = st->n[st->cur];
    auto copy = [&](bool to_snap) {
        if (touches_phi)
            SV_HIP(hipMemcpyAsync(to_snap ? st->snap_phi : phi, to_snap ? phi : st->snap_phi, V * sizeof(double),
                                  hipMemcpyDeviceToDevice, ctx->stream));
        if (touches_n)
            SV_HIP(hipMemcpyAsync(to_snap ? st->snap_n : n, to_snap ? n : st->snap_n, 2 * V * sizeof(int64_t),
                                  hipMemcpyDeviceToDevice, ctx->stream));
    };
    run_batches(ctx, specs, sweeps, cur, inc, stats, may_reject, [&] { copy(true); }, [&] { copy(false); }, launch_sweep);
}

}  // namespace svh

using namespace svh;

extern "C" {

int sv_villain_site_run(sv_villain *st, double kappa, double interval_phi, int32_t sweeps, sv_rng *rng,
                        sv_stats *stats) {
    if (!st || !rng || (sweeps > 0 && !stats)) return -1;
    sv_ctx *ctx = st->ctx;
    try {
        if (sweeps < 0) throw std::invalid_argument("sweeps must be >= 0");
        SV_HIP(hipSetDevice(ctx->device));
        const int32_t N = st->N;
        const int64_t V = (int64_t)N * N;
        LParams P = lparams(N);
        P.half_kappa = kappa / 2.0;
        P.lo = -interval_phi;
        P.range = interval_phi - (-interval_phi);
        u128 inc{rng->inc_lo, rng->inc_hi};
        Cursor cur = cursor_of(rng);
        const JumpTables *T = ctx->jump_tables(inc.hi, inc.lo);
        std::vector<BlockSpec> specs{{UNIFORM, (uint32_t)V}};
        for (int c = 0; c < st->ncol; c++) specs.push_back({UNIFORM, (uint32_t)st->count[c]});
        const bool even = N % 2 == 0;
        const int grid = grid_for(V / 2 + 1, N);
        const int64_t Sl = (int64_t)grid * 256;
        const Affine adv_m = host_power(inc, 2 * Sl), adv_e = host_power(inc, Sl);
        const int gi = (int)std::min<int64_t>((V + 255) / 256, 4096);
        double *phi = st->phi[st->cur];
        const int64_t *n = st->n[st->cur];
        if (even) {
            // two launches per sweep; the new phi goes to the snapshot buffer, then the pointers swap
            // (SiteUpdate never replays: it makes no bounded draws)
            run_local(st, specs, sweeps, cur, inc, stats, false, false, false, [&](int k, const Block *B, sv_stats *ds) {
                (void)k;
                double *in = st->phi[st->cur], *out = st->snap_phi;
                site_pp<0><<<grid, 256, 0, ctx->stream>>>(P, in, out, n, st->r, B, T, adv_m, adv_e, ds, ctx->d_abort), SV_LAUNCHED("site_pp<0>", ctx->stream);
                site_pp<1><<<grid, 256, 0, ctx->stream>>>(P, in, out, n, st->r, B, T, adv_m, adv_e, ds, ctx->d_abort), SV_LAUNCHED("site_pp<1>", ctx->stream);
                std::swap(st->phi[st->cur], st->snap_phi);
            });
            for (int k = 0; k < sweeps; k++) stats[k].proposed = V;
            store_cursor(cur, rng);
            return 0;
        }
        run_local(st, specs, sweeps, cur, inc, stats, false, true, false, [&](int k, const Block *B, sv_stats *ds) {
            (void)k;
            local_dphi_init<<<gi, 256, 0, ctx->stream>>>(N, phi, st->r, 1, ctx->d_abort), SV_LAUNCHED("local_dphi_init", ctx->stream);
            for (int c = 0; c < st->ncol; c++) {
                const int64_t nc = st->count[c];
                if (!nc) continue;
                if (even)
                    site_pass<true><<<grid, 256, 0, ctx->stream>>>(P, phi, n, st->r, nullptr, nc, c, B, T, adv_m,
                                                                   adv_e, ds, ctx->d_abort), SV_LAUNCHED("site_pass<true>", ctx->stream);
                else
                    site_pass<false><<<(int)((nc + 255) / 256), 256, 0, ctx->stream>>>(
                        P, phi, n, st->r, st->sites + st->offset[c], nc, c, B, T, adv_m, adv_e, ds, ctx->d_abort), SV_LAUNCHED("site_pass<false>", ctx->stream);
            }
        });
        for (int k = 0; k < sweeps; k++) stats[k].proposed = V;
        store_cursor(cur, rng);
        return 0;
    } catch (const std::exception &e) {
        ctx->err = e.what();
        return -2;
    }
}

int sv_villain_exact_run(sv_villain *st, double kappa, int64_t interval_z, int32_t sweeps, sv_rng *rng,
                         sv_stats *stats) {
    if (!st || !rng || (sweeps > 0 && !stats)) return -1;
    sv_ctx *ctx = st->ctx;
    try {
        if (sweeps < 0) throw std::invalid_argument("sweeps must be >= 0");
        SV_HIP(hipSetDevice(ctx->device));
        const int32_t N = st->N;
        const int64_t V = (int64_t)N * N;
        LParams P = lparams(N);
        P.m2pik = -LTWO_PI * kappa;
        set_bounded(P, interval_z);
        u128 inc{rng->inc_lo, rng->inc_hi};
        Cursor cur = cursor_of(rng);
        const JumpTables *T = ctx->jump_tables(inc.hi, inc.lo);
        std::vector<BlockSpec> specs{{UNIFORM, (uint32_t)V}};
        for (int c = 0; c < st->ncol; c++) specs.push_back({BOUNDED, (uint32_t)st->count[c]});
        const bool even = N % 2 == 0;
        const int grid = grid_for(V / 2 + 1, N);
        const int64_t Sl = (int64_t)grid * 256;
        const Affine adv_m = host_power(inc, 2 * Sl), adv_half = host_power(inc, Sl / 2);
        double *phi = st->phi[st->cur];
        int64_t *n = st->n[st->cur];
        run_local(st, specs, sweeps, cur, inc, stats, P.thr != 0, false, true, [&](int k, const Block *B, sv_stats *ds) {
            for (int c = 0; c < st->ncol; c++) {
                const int64_t nc = st->count[c];
                if (!nc) continue;
                if (even)
                    exact_pass<true><<<grid, 256, 0, ctx->stream>>>(P, n, phi, nullptr, nc, c, B, ctx->d_skips, T,
                                                                    adv_m, adv_half, ds, scratch(ctx), (uint32_t)k), SV_LAUNCHED("exact_pass<true>", ctx->stream);
                else
                    exact_pass<false><<<(int)((nc + 255) / 256), 256, 0, ctx->stream>>>(
                        P, n, phi, st->sites + st->offset[c], nc, c, B, ctx->d_skips, T, adv_m, adv_half, ds,
                        scratch(ctx), (uint32_t)k), SV_LAUNCHED("exact_pass<false>", ctx->stream);
            }
        });
        for (int k = 0; k < sweeps; k++) stats[k].proposed = V;
        store_cursor(cur, rng);
        return 0;
    } catch (const std::exception &e) {
        ctx->err = e.what();
        return -2;
    }
}

int sv_villain_link_run(sv_villain *st, double kappa, int64_t W, int64_t interval_n, int32_t sweeps, sv_rng *rng,
                        sv_stats *stats) {
    if (!st || !rng || (sweeps > 0 && !stats)) return -1;
    sv_ctx *ctx = st->ctx;
    try {
        if (sweeps < 0) throw std::invalid_argument("sweeps must be >= 0");
        SV_HIP(hipSetDevice(ctx->device));
        const int32_t N = st->N;
        const int64_t V = (int64_t)N * N;
        LParams P = lparams(N);
        P.m2pik = -LTWO_PI * kappa;
        P.W = W;
        set_bounded(P, interval_n);
        u128 inc{rng->inc_lo, rng->inc_hi};
        Cursor cur = cursor_of(rng);
        const JumpTables *T = ctx->jump_tables(inc.hi, inc.lo);
        const std::vector<BlockSpec> specs{{BOUNDED, (uint32_t)(2 * V)}, {UNIFORM, (uint32_t)(2 * V)}};
        const int grid = grid_for(2 * V, 2);
        const int64_t Sl = (int64_t)grid * 256;
        const Affine adv_u = host_power(inc, Sl), adv_half = host_power(inc, Sl / 2);
        const double *phi = st->phi[st->cur];
        int64_t *n = st->n[st->cur];
        run_local(st, specs, sweeps, cur, inc, stats, P.thr != 0, false, true, [&](int k, const Block *B, sv_stats *ds) {
            link_sweep<<<grid, 256, 0, ctx->stream>>>(P, phi, n, B, ctx->d_skips, T, adv_u, adv_half, ds,
                                                      scratch(ctx), (uint32_t)k), SV_LAUNCHED("link_sweep", ctx->stream);
        });
        for (int k = 0; k < sweeps; k++) stats[k].proposed = 2 * V;
        store_cursor(cur, rng);
        return 0;
    } catch (const std::exception &e) {
        ctx->err = e.what();
        return -2;
    }
}

int sv_villain_cohomology_run(sv_villain *st, double kappa, int64_t interval_h, int32_t sweeps, sv_rng *rng,
                              sv_stats *stats) {
    if (!st || !rng || (sweeps > 0 && !stats)) return -1;
    sv_ctx *ctx = st->ctx;
    try {
        if (sweeps < 0) throw std::invalid_argument("sweeps must be >= 0");
        if (sweeps == 0) return 0;
        SV_HIP(hipSetDevice(ctx->device));
        LParams P = lparams(st->N);
        set_bounded(P, interval_h);
        std::vector<int32_t> leaves;
        std::vector<uint8_t> prog;
        pairwise_plan(0, st->N, leaves, prog);
        if ((int)leaves.size() / 2 > MAX_LEAVES) throw std::invalid_argument("lattice too large for the slice sum");
        // one device buffer (rng | stats | leaves | prog) and one pinned host image of it, kept by the
        // state: every transfer is a stream-ordered DMA on ctx->stream
        const size_t o_st = 64, o_lv = o_st + ((sizeof(sv_stats) * sweeps + 63) / 64) * 64;
        const size_t o_pg = o_lv + leaves.size() * sizeof(int32_t), total = o_pg + prog.size();
        if (total > st->aux_cap) {
            SV_HIP(hipStreamSynchronize(ctx->stream));
            if (st->d_aux) SV_HIP(hipFree(st->d_aux));
            if (st->h_aux) SV_HIP(hipHostFree(st->h_aux));
            st->d_aux = st->h_aux = nullptr;
            st->aux_cap = 0;
            SV_HIP(hipMalloc((void **)&st->d_aux, total));
            SV_HIP(hipHostMalloc((void **)&st->h_aux, total, hipHostMallocDefault));
            st->aux_cap = total;
        }
        char *hb = st->h_aux;
        CohoRng h{rng->state_lo, rng->state_hi, rng->inc_lo, rng->inc_hi, (uint32_t)rng->has_uint32, rng->uinteger};
        memcpy(hb, &h, sizeof(h));
        memcpy(hb + o_lv, leaves.data(), leaves.size() * sizeof(int32_t));
        memcpy(hb + o_pg, prog.data(), prog.size());
        char *d = st->d_aux;
        SV_HIP(hipMemcpyAsync(d, hb, total, hipMemcpyHostToDevice, ctx->stream));
        const PairwisePlan plan{(int32_t)(leaves.size() / 2), (int32_t)prog.size()};
        hipEvent_t ev;
        ctx->time_begin(&ev);
        cohomology_run<<<1, 256, 0, ctx->stream>>>(st->N, kappa / 2.0, P.iv, P.k, P.thr, st->phi[st->cur],
                                                   st->n[st->cur], sweeps, (CohoRng *)d, (sv_stats *)(d + o_st),
                                                   (const int32_t *)(d + o_lv), (const uint8_t *)(d + o_pg), plan), SV_LAUNCHED("cohomology_run", ctx->stream);
        ctx->time_end(ev, 1);
        SV_HIP(hipGetLastError());
        SV_HIP(hipMemcpyAsync(hb, d, o_lv, hipMemcpyDeviceToHost, ctx->stream));
        SV_HIP(hipStreamSynchronize(ctx->stream));
        ctx->time_collect();
        memcpy(&h, hb, sizeof(h));
        memcpy(stats, hb + o_st, sizeof(sv_stats) * sweeps);
        rng->state_lo = h.s_lo;
        rng->state_hi = h.s_hi;
        rng->has_uint32 = (int32_t)h.has;
        rng->uinteger = h.buf;
        return 0;
    } catch (const std::exception &e) {
        ctx->err = e.what();
        return -2;
    }
}

}  // extern "C"
