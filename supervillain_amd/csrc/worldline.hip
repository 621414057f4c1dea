// worldline.hip -- CoexactUpdate and PlaquetteUpdate on gfx950.
//
//  * CoexactUpdate (supervillain/generator/worldline/coexact.py:53-128): one kernel per colour pass,
//    m patched in place; delta(v)/W is formed on the fly from v (frozen for the sweep, coexact.py:80).
//    Bit-exact replay of the seeded reference chain.
//  * PlaquetteUpdate, reference order (plaquette.py:35-104): the visit order is the permutation the
//    reference draws from NumPy's global RandomState; the host hands it over.  Sequential semantics
//    are kept exactly by dependency LEVELS: level(p) = 1 + the highest level among the earlier-visited
//    plaquettes sharing a link with p.  Plaquettes of one level share no link and depend only on
//    lower levels, so one launch per level reproduces the sequential loop bit-for-bit (m, v and the
//    incrementally updated f = m - delta(v)/W).
//  * PlaquetteUpdate, checkerboard: this build's GPU-native chain: colour passes with f
//    evaluated fresh.  Oracle: oracle/sv_oracle.c sv_o_worldline_plaquette_cb.
#include <algorithm>
#include <cmath>
#include <exception>
#include <thread>

#include "local.h"
#include "fused.h"

namespace svh {
// worldline_fused.hip
bool wf_usable(int32_t N, bool v_is_float, double W_eff, int64_t it);
bool wf_fast(const sv::Block *blocks);
void launch_wf(const sv::FGeom &G, double kappa, double W_eff, int64_t it, const int64_t *m_in, const int64_t *v_in,
               int64_t *m_out, int64_t *v_out, const sv::Block *blocks, const sv::Block *hblocks, const uint32_t *skips, bool general,
               const sv::JumpTables *T, const sv::Affine adv[6], sv::u128 inc, void *pstat, void *cstat, sv::DevScratch S,
               uint32_t sweep, hipStream_t stream);
}  // namespace svh

namespace sv {

#define TWO_PI_W 6.283185307179586

__device__ __forceinline__ u128 wbase(const Block &b) { return u128{b.base_lo, b.base_hi}; }

__device__ __forceinline__ void wreport(const DevScratch &S, uint32_t sweep, uint32_t block, uint32_t pos) {
    uint32_t i = atomicAdd(S.nreport, 1u);
    if (i < (uint32_t)MAX_REPORTS) S.reports[i] = Report{sweep, block, pos, 0};
    __hip_atomic_store(S.abort, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ uint32_t wbounded(const JumpTables *T, const Block &b, const uint32_t *skips, uint32_t d,
                                             uint32_t k, uint32_t thr, const DevScratch &S, uint32_t sweep,
                                             uint32_t bidx) {
    uint32_t q = d;
    for (int i = 0; i < b.nskip; i++)
        if (skips[b.skip0 + i] <= q) q++;
    uint32_t word;
    if (b.has && q == 0) {
        word = b.buf;
    } else {
        uint32_t qq = q - b.has;
        uint64_t X = xsl_rr(jump(T, wbase(b), qq >> 1));
        word = (qq & 1) ? (uint32_t)(X >> 32) : (uint32_t)X;
    }
    bool rej;
    uint32_t idx = lemire(word, k, thr, &rej);
    if (rej) wreport(S, sweep, bidx, q);
    return idx;
}

__global__ void fold_stripes(const StatStripe *ss, sv_stats *out, int count) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= count) return;
    unsigned long long a = 0, w[3] = {0, 0, 0};
    for (int j = 0; j < NSTRIPE; j++) {
        a += ss[k * NSTRIPE + j].acc;
        for (int i = 0; i < 3; i++) w[i] += ss[k * NSTRIPE + j].pw[i];
    }
    // the exact acceptance limbs (common.h) in the slot's words, finalized before the slot lands
    *stat_word(&out[k], 0) = a;
    for (int i = 0; i < 3; i++) *stat_word(&out[k], 1 + i) = w[i];
}

// delta(v)/W on link (mu, s) of a D=2 two-form v, exactly as reference_delta + coexact.py:80:
//   dv0[s] = 0 - (-1)(v[s] - v[s-e1]),  dv1[s] = 0 - (+1)(v[s] - v[s-e0]);  then / W_eff
template <bool VF>
__device__ __forceinline__ double dvw_at(const void *v, int64_t N, int mu, int64_t s, int64_t t, int64_t x, double Weff) {
    const int64_t nb = mu == 0 ? t * N + (x == 0 ? N - 1 : x - 1) : (t == 0 ? N - 1 : t - 1) * N + x;
    double d;
    if (VF) {
        const double *vf = (const double *)v;
        double diff = vf[s] - vf[nb];
        d = mu == 0 ? 0.0 - (-diff) : 0.0 - diff;
    } else {
        const int64_t *vi = (const int64_t *)v;
        int64_t diff = vi[s] - vi[nb];
        d = mu == 0 ? (double)(0 - (-diff)) : (double)(0 - diff);
    }
    return d / Weff;
}
template <bool VF>
__device__ __forceinline__ double dvw_link(const void *v, int64_t N, int mu, int64_t s, double Weff) {
    int64_t t, x;
    divmod_site(s, N, t, x);
    return dvw_at<VF>(v, N, mu, s, t, x, Weff);
}

struct WParams {
    int32_t N;
    double kappa, Weff;
    double c;  // 0.5 / kappa
    int64_t it;
    uint32_t k, thr;
    double Winv;     // 1 / W when W is a power of two (x * Winv == x / W exactly)
    int32_t wpow2;
    int32_t grid;    // grid-stride colour passes (even N): workgroups, stride S = 256 grid
    Affine adv_m;    // metropolis positions advance by 2S per lane iteration
    Affine adv_half; // bounded-draw words advance by S/2
};

// delta(v)/W on link (mu, s) = (t, x), the division as dvw_at does it (exact reciprocal for power-of-two W)
template <bool VF>
__device__ __forceinline__ double dvw_p(const void *v, int64_t N, int mu, int64_t s, int64_t t, int64_t x,
                                        const WParams &P) {
    const int64_t nb = mu == 0 ? t * N + (x == 0 ? N - 1 : x - 1) : (t == 0 ? N - 1 : t - 1) * N + x;
    double d;
    if (VF) {
        const double *vf = (const double *)v;
        const double diff = vf[s] - vf[nb];
        d = mu == 0 ? 0.0 - (-diff) : 0.0 - diff;
    } else {
        const int64_t *vi = (const int64_t *)v;
        const int64_t diff = vi[s] - vi[nb];
        d = mu == 0 ? (double)(0 - (-diff)) : (double)(0 - diff);
    }
    return P.wpow2 ? d * P.Winv : d / P.Weff;
}

// ------------------------------------------------------------------------------------------------
// CoexactUpdate colour pass.  Blocks per sweep: [0] metropolis (uniform V), [1+c] t for colour c.
template <bool VF>
__global__ __launch_bounds__(256) void coexact_pass(WParams P, int64_t *m, const void *v, const int32_t *sites,
                                                    int64_t nc, int color, const Block *blocks, const uint32_t *skips,
                                                    const JumpTables *T, StatStripe *stat, DevScratch S,
                                                    uint32_t sweep) {
    if (*(volatile const int32_t *)S.abort) return;
    const int64_t N = P.N, V = N * N;
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    int64_t acc_count = 0;
    AccFx psum;  // exact acceptance sum (common.h)
    if (i < nc) {
        const int64_t x = sites[i];
        int64_t tt, xx;
        divmod_site(x, N, tt, xx);
        const int64_t xe0 = ((tt + 1 == N) ? 0 : tt + 1) * N + xx;
        const int64_t xe1 = tt * N + ((xx + 1 == N) ? 0 : xx + 1);
        const double u = 0.0 + 1.0 * to_double(xsl_rr(jump(T, wbase(blocks[0]), (uint32_t)x)));
        const uint32_t j = wbounded(T, blocks[1 + color], skips, (uint32_t)i, P.k, P.thr, S, sweep, 1 + color);
        const int64_t t = (int64_t)j < P.it ? (int64_t)j - P.it : (int64_t)j - P.it + 1;
        // coface_sum_at order ('coface_sum',1) rows (0,1,0,1),(0,0,1,1): l1[x], l1[x+e0], l0[x], l0[x+e1]
        const int mus[4] = {1, 1, 0, 0};
        const int64_t ss[4] = {x, xe0, x, xe1};
        const int64_t cm[4] = {-t, +t, +t, -t};
        double dS = 0.0;
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const int64_t l = mus[q] * V + ss[q];
            const double a = P.c * (double)cm[q];
            const double f = (double)m[l] - dvw_link<VF>(v, N, mus[q], ss[q], P.Weff);
            const double b = (2.0 * f) + (double)cm[q];
            dS += a * b;
        }
        double p = exp(-dS);
        p = p < 0.0 ? 0.0 : p;
        p = p > 1.0 ? 1.0 : p;
        const int acc = u < p;
        acc_count = acc;
        fx_add(psum, p);
        if (acc) {  // delta_sparse(..., t*accepted, out=m): m0[x]+=t, m0[x+e1]-=t, m1[x]-=t, m1[x+e0]+=t
            m[x] += t;
            m[xe1] -= t;
            m[V + x] -= t;
            m[V + xe0] += t;
        }
    }
    wflush(stat, acc_count, psum);
}

// ------------------------------------------------------------------------------------------------
// Checkerboard PlaquetteUpdate colour pass.  Blocks per sweep: [0] metropolis (uniform V),
// per colour c: [1+2c] change_m = choice([-1,1]), [2+2c] change_v = choice([-1,0,1]).
template <bool VF>
__global__ __launch_bounds__(256) void plaquette_cb_pass(WParams P, int64_t *m, void *v, const int32_t *sites,
                                                         int64_t nc, int color, const Block *blocks,
                                                         const uint32_t *skips, const JumpTables *T, StatStripe *stat,
                                                         DevScratch S, uint32_t sweep) {
    if (*(volatile const int32_t *)S.abort) return;
    const int64_t N = P.N, V = N * N;
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    int64_t acc_count = 0;
    AccFx psum;  // exact acceptance sum (common.h)
    if (i < nc) {
        const int64_t x = sites[i];
        int64_t tt, xx;
        divmod_site(x, N, tt, xx);
        const int64_t xm = ((tt + 1 == N) ? 0 : tt + 1) * N + xx;  // here + e_mu (mu = 0)
        const int64_t xn = tt * N + ((xx + 1 == N) ? 0 : xx + 1);  // here + e_nu (nu = 1)
        const double u = 0.0 + 1.0 * to_double(xsl_rr(jump(T, wbase(blocks[0]), (uint32_t)x)));
        const uint32_t jm = wbounded(T, blocks[1 + 2 * color], skips, (uint32_t)i, 2u, 0u, S, sweep, 1 + 2 * color);
        const uint32_t jv = wbounded(T, blocks[2 + 2 * color], skips, (uint32_t)i, 3u, 1u, S, sweep, 2 + 2 * color);
        const int64_t cm = jm ? 1 : -1, cv = (int64_t)jv - 1;
        const double f1 = (double)m[x] - dvw_link<VF>(v, N, 0, x, P.Weff);
        const double f2 = (double)m[V + xm] - dvw_link<VF>(v, N, 1, xm, P.Weff);
        const double f3 = (double)m[xn] - dvw_link<VF>(v, N, 0, xn, P.Weff);
        const double f4 = (double)m[V + x] - dvw_link<VF>(v, N, 1, x, P.Weff);
        const double df = (double)cm - (double)cv / P.Weff;
        const double dS = df / P.kappa * ((((f1 + f2) - f3) - f4) + 2.0 * df);
        double p = exp(-dS);
        p = p < 0.0 ? 0.0 : p;
        p = p > 1.0 ? 1.0 : p;
        const int acc = u < p;
        acc_count = acc;
        fx_add(psum, p);
        if (acc) {
            m[x] += cm;
            m[V + xm] += cm;
            m[xn] -= cm;
            m[V + x] -= cm;
            if (VF) ((double *)v)[x] += (double)cv;
            else ((int64_t *)v)[x] += cv;
        }
    }
    wflush(stat, acc_count, psum);
}

// ------------------------------------------------------------------------------------------------
// Grid-stride colour passes (even N; local.h stream addressing): a lane owns colour site e, e + S, ...;
// its metropolis and bounded-draw stream states advance by one precomputed affine map per iteration.
// CoexactUpdate, coexact.py:85-120: t = choice(ts) on the colour, m += delta(t accepted).
template <bool VF>
__global__ __launch_bounds__(256) void coexact_gs(WParams P, int64_t *m, const void *v, int color,
                                                  const Block *blocks, const uint32_t *skips, const JumpTables *T,
                                                  StatStripe *stat, DevScratch S, uint32_t sweep) {
    if (*(volatile const int32_t *)S.abort) return;
    const int64_t N = P.N, V = N * N, nc = V >> 1;
    const int64_t G = (int64_t)gridDim.x * blockDim.x;
    const Block BM = blocks[0], BT = blocks[1 + color];
    const bool slow = BT.nskip > 0;
    loc::UniLane um{u128{0, 0}, false};
    loc::BndLane bt{u128{0, 0}, false};
    int64_t acc_count = 0;
    AccFx psum;  // exact acceptance sum (common.h)
    for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < nc; e += G) {
        const int64_t x = loc::even_site(e, N, color);
        int64_t tt, xx;
        divmod_site(x, N, tt, xx);
        const double u = 0.0 + 1.0 * to_double(um.next(T, BM, (uint32_t)x, P.adv_m));
        uint32_t q = (uint32_t)e, w;
        if (slow) w = loc::bnd_word_slow(T, BT, skips, (uint32_t)e, &q);
        else w = bt.next(T, BT, (uint32_t)e, P.adv_half);
        bool rej;
        const uint32_t j = lemire(w, P.k, P.thr, &rej);
        if (rej) wreport(S, sweep, 1u + (uint32_t)color, q);
        const int64_t t = (int64_t)j < P.it ? (int64_t)j - P.it : (int64_t)j - P.it + 1;
        const int64_t tp = (tt + 1 == N) ? 0 : tt + 1, xp = (xx + 1 == N) ? 0 : xx + 1;
        const int64_t xe0 = tp * N + xx, xe1 = tt * N + xp;
        const int mus[4] = {1, 1, 0, 0};
        const int64_t ss[4] = {x, xe0, x, xe1};
        const int64_t st_[4] = {tt, tp, tt, tt}, sx_[4] = {xx, xx, xx, xp};
        const int64_t cm[4] = {-t, +t, +t, -t};
        double dS = 0.0;
#pragma unroll
        for (int q4 = 0; q4 < 4; q4++) {
            const int64_t l = mus[q4] * V + ss[q4];
            const double a = P.c * (double)cm[q4];
            const double f = (double)m[l] - dvw_p<VF>(v, N, mus[q4], ss[q4], st_[q4], sx_[q4], P);
            const double b = (2.0 * f) + (double)cm[q4];
            dS += a * b;
        }
        const double p = loc::clip01(exp(-dS));
        const int acc = u < p;
        acc_count += acc;
        fx_add(psum, p);
        if (acc) {
            m[x] += t;
            m[xe1] -= t;
            m[V + x] -= t;
            m[V + xe0] += t;
        }
    }
    wflush(stat, acc_count, psum);
}

// Checkerboard PlaquetteUpdate colour pass (the GPU-native chain): blocks [0] metropolis,
// [1 + 2c] change_m = choice((-1, 1)), [2 + 2c] change_v = choice((-1, 0, 1)) of colour c.
template <bool VF>
__global__ __launch_bounds__(256) void plaquette_cb_gs(WParams P, int64_t *m, void *v, int color, const Block *blocks,
                                                       const uint32_t *skips, const JumpTables *T, StatStripe *stat,
                                                       DevScratch S, uint32_t sweep) {
    if (*(volatile const int32_t *)S.abort) return;
    const int64_t N = P.N, V = N * N, nc = V >> 1;
    const int64_t G = (int64_t)gridDim.x * blockDim.x;
    const Block BM = blocks[0], BCM = blocks[1 + 2 * color], BCV = blocks[2 + 2 * color];
    const bool slow = BCM.nskip > 0 || BCV.nskip > 0;
    loc::UniLane um{u128{0, 0}, false};
    loc::BndLane bm{u128{0, 0}, false}, bv{u128{0, 0}, false};
    int64_t acc_count = 0;
    AccFx psum;  // exact acceptance sum (common.h)
    for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < nc; e += G) {
        const int64_t x = loc::even_site(e, N, color);
        int64_t tt, xx;
        divmod_site(x, N, tt, xx);
        const double u = 0.0 + 1.0 * to_double(um.next(T, BM, (uint32_t)x, P.adv_m));
        uint32_t qm = (uint32_t)e, qv = (uint32_t)e, wm, wv;
        if (slow) {
            wm = loc::bnd_word_slow(T, BCM, skips, (uint32_t)e, &qm);
            wv = loc::bnd_word_slow(T, BCV, skips, (uint32_t)e, &qv);
        } else {
            wm = bm.next(T, BCM, (uint32_t)e, P.adv_half);
            wv = bv.next(T, BCV, (uint32_t)e, P.adv_half);
        }
        bool rej;
        const uint32_t jm = lemire(wm, 2u, 0u, &rej);
        const uint32_t jv = lemire(wv, 3u, 1u, &rej);
        if (rej) wreport(S, sweep, 2u + 2u * (uint32_t)color, qv);
        const int64_t cm = jm ? 1 : -1, cv = (int64_t)jv - 1;
        const int64_t tp = (tt + 1 == N) ? 0 : tt + 1, xp = (xx + 1 == N) ? 0 : xx + 1;
        const int64_t xm = tp * N + xx, xn = tt * N + xp;
        const double f1 = (double)m[x] - dvw_p<VF>(v, N, 0, x, tt, xx, P);
        const double f2 = (double)m[V + xm] - dvw_p<VF>(v, N, 1, xm, tp, xx, P);
        const double f3 = (double)m[xn] - dvw_p<VF>(v, N, 0, xn, tt, xp, P);
        const double f4 = (double)m[V + x] - dvw_p<VF>(v, N, 1, x, tt, xx, P);
        const double df = (double)cm - (P.wpow2 ? (double)cv * P.Winv : (double)cv / P.Weff);
        const double dS = df / P.kappa * ((((f1 + f2) - f3) - f4) + 2.0 * df);
        const double p = loc::clip01(exp(-dS));
        const int acc = u < p;
        acc_count += acc;
        fx_add(psum, p);
        if (acc) {
            m[x] += cm;
            m[V + xm] += cm;
            m[xn] -= cm;
            m[V + x] -= cm;
            if (VF) ((double *)v)[x] += (double)cv;
            else ((int64_t *)v)[x] += cv;
        }
    }
    wflush(stat, acc_count, psum);
}

// ------------------------------------------------------------------------------------------------
// Reference-order PlaquetteUpdate: f = m - delta(v)/W once per sweep (plaquette.py:53), then one
// launch per dependency level.  Blocks: [0] change_m (k=2, V), [1] change_v (k=3, V),
// [2] metropolis (uniform V); the draw index of a plaquette is its visit position (plaquette.py:58-69).
template <bool VF>
__global__ void plaquette_f_init(WParams P, const int64_t *m, const void *v, double *f) {
    const int64_t N = P.N, V = N * N;
    for (int64_t s = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; s < V; s += (int64_t)gridDim.x * blockDim.x) {
        f[s] = (double)m[s] - dvw_link<VF>(v, N, 0, s, P.Weff);
        f[V + s] = (double)m[V + s] - dvw_link<VF>(v, N, 1, s, P.Weff);
    }
}

// One dependency level of the reference-order sweep: every plaquette in `list` has all of its
// earlier-visited link-sharing neighbours in lower levels, and no two share a link.
template <bool VF>
__global__ __launch_bounds__(256) void plaquette_level(WParams P, int64_t *m, void *v, double *f, const int32_t *list,
                                                       int32_t count, const int32_t *pos, const Block *blocks,
                                                       const uint32_t *skips, const JumpTables *T, StatStripe *stat,
                                                       DevScratch S) {
    if (*(volatile const int32_t *)S.abort) return;
    const int64_t N = P.N, V = N * N;
    const int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    int64_t acc_count = 0;
    AccFx psum;  // exact acceptance sum (common.h)
    if (i < count) {
        const int64_t x = list[i];
        int64_t tt, xx;
        divmod_site(x, N, tt, xx);
        const int64_t xm = ((tt + 1 == N) ? 0 : tt + 1) * N + xx;
        const int64_t xn = tt * N + ((xx + 1 == N) ? 0 : xx + 1);
        const uint32_t idx = (uint32_t)pos[x];
        const uint32_t jm = wbounded(T, blocks[0], skips, idx, 2u, 0u, S, 0, 0);
        const uint32_t jv = wbounded(T, blocks[1], skips, idx, 3u, 1u, S, 0, 1);
        const double met = 0.0 + 1.0 * to_double(xsl_rr(jump(T, wbase(blocks[2]), idx)));
        const int64_t cm = jm ? 1 : -1, cv = (int64_t)jv - 1;
        const double f1 = f[x], f2 = f[V + xm], f3 = f[xn], f4 = f[V + x];
        const double df = (double)cm - (double)cv / P.Weff;
        const double dS = df / P.kappa * ((((f1 + f2) - f3) - f4) + 2.0 * df);
        double p = exp(-dS);
        p = p < 0.0 ? 0.0 : p;
        p = p > 1.0 ? 1.0 : p;
        fx_add(psum, p);
        if (met < p) {
            m[x] += cm;
            m[V + xm] += cm;
            m[xn] += -cm;
            m[V + x] += -cm;
            if (VF) ((double *)v)[x] += (double)cv;
            else ((int64_t *)v)[x] += cv;
            f[x] += df;
            f[V + xm] += df;
            f[xn] -= df;
            f[V + x] -= df;
            acc_count = 1;
        }
    }
    wflush(stat, acc_count, psum);
}

// ------------------------------------------------------------------------------------------------
// The dependency levels of a reference-order sweep, on the device (the visit order of a 1024^2 lattice is 1M
// plaquettes; the O(V) host pass with its random accesses cost ~20 ms a sweep).  Level l(p) = 1 + max l(q) over the
// earlier-visited plaquettes q sharing a link with p (its four nearest neighbours); plaquettes of one level share no
// link and may run in any order.  A random permutation has ~15 levels at L = 1024 (any permutation is accepted:
// row-major order has 2N - 1).  Flags: [0] not a permutation, [1] max level, [2 + j] iteration j changed a level.
template <typename O>
__global__ void order_positions(const O *order, int64_t V, int32_t *pos, int32_t *flags) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < V; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t x = (int64_t)order[i];
        if (x < 0 || x >= V) {
            flags[0] = 1;
            continue;
        }
        if (atomicExch(&pos[x], (int32_t)i) != -1) flags[0] = 1;  // pos starts at -1: a repeated plaquette
    }
}

// one relaxation of l(p) = 1 + max over earlier neighbours, in place (values only rise toward the unique fixed point,
// so reading partly updated neighbours is safe); flags[2 + j] = 1 if any level changed
__global__ void order_levels(int64_t N, const int32_t *pos, int32_t *lev, int32_t *flags, int j) {
    const int64_t V = N * N;
    bool changed = false;
    for (int64_t x = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; x < V; x += (int64_t)gridDim.x * blockDim.x) {
        int64_t t, xx;
        divmod_site(x, N, t, xx);
        const int64_t nb[4] = {(t + 1 == N ? 0 : t + 1) * N + xx, (t == 0 ? N - 1 : t - 1) * N + xx,
                               t * N + (xx + 1 == N ? 0 : xx + 1), t * N + (xx == 0 ? N - 1 : xx - 1)};
        const int32_t px = pos[x];
        int32_t l = 0;
        for (int k = 0; k < 4; k++) {
            const int32_t ln = lev[nb[k]];
            if (pos[nb[k]] < px && ln > l) l = ln;
        }
        if (l + 1 != lev[x]) {
            lev[x] = l + 1;
            changed = true;
        }
    }
    if (__builtin_amdgcn_ballot_w64(changed) && (threadIdx.x & 63) == 0) flags[2 + j] = 1;
}

// per-level counts (levels below LB aggregated in LDS) and the maximum level
constexpr int LB = 256;
constexpr int LFLAGS = 2 + 8;  // flags of order_positions / order_levels: 8 relaxations per host check
__global__ __launch_bounds__(256) void order_level_counts(const int32_t *lev, int64_t V, int32_t *cnt, int32_t *flags) {
    __shared__ int32_t h[LB], wmax;
    for (int i = threadIdx.x; i < LB; i += blockDim.x) h[i] = 0;
    if (threadIdx.x == 0) wmax = 0;
    __syncthreads();
    int32_t mx = 0;
    for (int64_t x = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; x < V; x += (int64_t)gridDim.x * blockDim.x) {
        const int32_t l = lev[x];
        mx = l > mx ? l : mx;
        if (l < LB) atomicAdd(&h[l], 1);
        else atomicAdd(&cnt[l], 1);
    }
    __syncthreads();
    atomicMax(&wmax, mx);
    __syncthreads();
    for (int i = threadIdx.x; i < LB; i += blockDim.x)
        if (h[i]) atomicAdd(&cnt[i], h[i]);
    if (threadIdx.x == 0) atomicMax(&flags[1], wmax);  // one global atomic per workgroup (per thread: 190 us)
}

// the plaquettes grouped by level: fill[l] starts at the level's offset and hands out slots (within a level any order)
__global__ __launch_bounds__(256) void order_level_lists(const int32_t *lev, int64_t V, int32_t *fill, int32_t *list) {
    __shared__ int32_t h[LB], base[LB];
    for (int64_t x0 = blockIdx.x * (int64_t)blockDim.x; x0 < V; x0 += (int64_t)gridDim.x * blockDim.x) {
        for (int i = threadIdx.x; i < LB; i += blockDim.x) h[i] = 0;
        __syncthreads();
        const int64_t x = x0 + threadIdx.x;
        const int32_t l = x < V ? lev[x] : -1;
        int32_t slot = -1;
        if (l >= 0 && l < LB) slot = atomicAdd(&h[l], 1);
        __syncthreads();
        for (int i = threadIdx.x; i < LB; i += blockDim.x)
            if (h[i]) base[i] = atomicAdd(&fill[i], h[i]);
        __syncthreads();
        if (l >= LB) list[atomicAdd(&fill[l], 1)] = (int32_t)x;
        else if (l >= 0) list[base[l] + slot] = (int32_t)x;
        __syncthreads();
    }
}

}  // namespace sv

using namespace sv;

namespace {

using SkipMap = std::map<std::pair<int, int>, std::vector<uint32_t>>;

void wplan(Cursor &cur, u128 inc, const std::vector<BlockSpec> &specs, int first, int count, const SkipMap &skips,
           std::vector<Block> &blocks, std::vector<uint32_t> &skipvec) {
    blocks.clear();
    skipvec.clear();
    static const std::vector<uint32_t> none;
    for (int sw = first; sw < first + count; sw++)
        for (int bi = 0; bi < (int)specs.size(); bi++) {
            auto it = skips.find({sw, bi});
            const std::vector<uint32_t> &sk = it == skips.end() ? none : it->second;
            blocks.push_back(plan_block(cur, inc, specs[bi], sk, (int32_t)skipvec.size()));
            skipvec.insert(skipvec.end(), sk.begin(), sk.end());
        }
}

void wupload(sv_ctx *ctx, const std::vector<Block> &blocks, const std::vector<uint32_t> &skipvec) {
    ctx->upload_plan(blocks.data(), blocks.size(), skipvec.data(), skipvec.size());
}

bool wcheck(sv_ctx *ctx, std::vector<Report> &reps) {
    int32_t both[2];  // d_abort, d_nreport are adjacent (capi.hip)
    SV_HIP(hipMemcpyAsync(both, ctx->d_abort, sizeof(both), hipMemcpyDeviceToHost, ctx->stream));
    SV_HIP(hipStreamSynchronize(ctx->stream));
    const int32_t ab = both[0];
    uint32_t nrep = (uint32_t)both[1];
    reps.clear();
    if (!ab) return false;
    if (nrep > (uint32_t)MAX_REPORTS) nrep = MAX_REPORTS;
    reps.resize(nrep);
    if (nrep) {
        SV_HIP(hipMemcpyAsync(reps.data(), ctx->d_reports, nrep * sizeof(Report), hipMemcpyDeviceToHost, ctx->stream));
        SV_HIP(hipStreamSynchronize(ctx->stream));
    }
    if (reps.empty()) throw std::runtime_error("device aborted without a rejection report");
    return true;
}

int wabsorb(const std::vector<Report> &reps, int first, SkipMap &skips) {
    std::pair<uint32_t, uint32_t> best{~0u, ~0u};
    for (const Report &r : reps)
        if (std::make_pair(r.sweep, r.block) < best) best = {r.sweep, r.block};
    const std::pair<int, int> key{first + (int)best.first, (int)best.second};
    auto &lst = skips[key];
    for (const Report &r : reps)
        if (r.sweep == best.first && r.block == best.second) lst.push_back(r.pos);
    std::sort(lst.begin(), lst.end());
    lst.erase(std::unique(lst.begin(), lst.end()), lst.end());
    svh::drop_later_skips(skips, key);  // (later blocks' skips were found against the old block starts: stale)
    return (int)best.first;
}

WParams wparams(int32_t N, double kappa, double Weff, int64_t it, u128 inc) {
    WParams P{};
    P.N = N;
    P.kappa = kappa;
    P.Weff = Weff;
    P.c = 0.5 / kappa;
    P.it = it;
    P.k = (uint32_t)(2 * it);
    P.thr = (uint32_t)((0u - P.k) % P.k);
    int ex = 0;
    P.wpow2 = std::isfinite(Weff) && Weff > 0 && std::frexp(Weff, &ex) == 0.5;
    P.Winv = P.wpow2 ? 1.0 / Weff : 0.0;
    if (N % 2 == 0) {
        const int64_t V = (int64_t)N * N;
        P.grid = svh::loc::grid_for(V / 2 + 1, N);
        const int64_t G = (int64_t)P.grid * 256;
        P.adv_m = host_power(inc, 2 * G);
        P.adv_half = host_power(inc, G / 2);
    }
    return P;
}

DevScratch wscratch(sv_ctx *ctx) { return DevScratch{ctx->d_abort, ctx->d_nreport, ctx->d_reports}; }

// (m, v) copied in one launch: two hipMemcpyAsync device-to-device calls cost ~35 us of host time each at a batch
// boundary, the launch ~5 (16-B lanes; both sizes are multiples of 16 B)
__global__ void copy_pair(uint4 *__restrict__ d0, const uint4 *__restrict__ s0, int64_t n0, uint4 *__restrict__ d1,
                          const uint4 *__restrict__ s1, int64_t n1) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n0 + n1; i += stride) {
        if (i < n0) d0[i] = s0[i];
        else d1[i - n0] = s1[i - n0];
    }
}

void snapshot(sv_worldline *st, bool restore) {
    sv_ctx *ctx = st->ctx;
    const size_t V = (size_t)st->N * st->N;
    const size_t vb = V * (st->v_is_float ? sizeof(double) : sizeof(int64_t));
    const int64_t n0 = (int64_t)(2 * V * sizeof(int64_t) / 16), n1 = (int64_t)(vb / 16);
    const int grid = (int)std::min<int64_t>((n0 + n1 + 255) / 256, 4096);
    if (!restore) {
        st->m_at_snap = st->m;
        st->v_at_snap = st->v;
        if ((2 * V * sizeof(int64_t)) % 16 == 0 && vb % 16 == 0) {
            copy_pair<<<grid, 256, 0, ctx->stream>>>((uint4 *)st->snap_m, (const uint4 *)st->m, n0, (uint4 *)st->snap_v,
                                                     (const uint4 *)st->v, n1), SV_LAUNCHED("copy_pair", ctx->stream);
            SV_HIP(hipGetLastError());
        } else {
            SV_HIP(hipMemcpyAsync(st->snap_m, st->m, 2 * V * sizeof(int64_t), hipMemcpyDeviceToDevice, ctx->stream));
            SV_HIP(hipMemcpyAsync(st->snap_v, st->v, vb, hipMemcpyDeviceToDevice, ctx->stream));
        }
    } else {
        if (st->m_at_snap && st->m != st->m_at_snap) {  // fused steps swapped the buffer pairs since the snapshot
            std::swap(st->m, st->m_alt);
            std::swap(st->v, st->v_alt);
        }
        SV_HIP(hipMemcpyAsync(st->m, st->snap_m, 2 * V * sizeof(int64_t), hipMemcpyDeviceToDevice, ctx->stream));
        SV_HIP(hipMemcpyAsync(st->v, st->snap_v, vb, hipMemcpyDeviceToDevice, ctx->stream));
    }
}

// Batched colour-pass runner with snapshot + replay on a rejection.
// nstat statistics per sweep (a combined Plaquette + Coexact step has two); block b's rejections are
// counted in statistic stat_of[b].
template <typename Launch>
void run_colour_sweeps(sv_worldline *st, const std::vector<BlockSpec> &specs, int32_t sweeps, Cursor &cur, u128 inc,
                       sv_stats *stats, Launch launch, int nstat = 1, std::vector<int> stat_of = {},
                       bool may_reject = true) {
    sv_ctx *ctx = st->ctx;
    const int nb = (int)specs.size();
    if (stat_of.empty()) stat_of.assign(nb, 0);
    const int64_t V = (int64_t)st->N * st->N;
    const int BATCH = 64;  // (the striped statistics hold 64 sweeps)
    SkipMap skips;
    std::vector<Block> blocks;
    std::vector<uint32_t> skipvec;
    std::vector<Report> reps;
    // The next batch is planned on the host while this one runs on the device (the plan is most of a batch
    // boundary: ~160 us per 64 L=1024 steps); a replay in this batch (new skips) discards it
    std::vector<Block> blocks_next;
    std::vector<uint32_t> skipvec_next;
    Cursor c_next{};
    int sw_next = -1;
    int sw = 0;
    while (sw < sweeps) {
        const int count = std::min(BATCH, sweeps - sw);
        bool stats_landed = false;
        if (may_reject) snapshot(st, false);  // no bounded draw that can reject: nothing to replay
        for (int attempt = 0;; attempt++) {
            if (attempt > 256) throw std::runtime_error("rejection replay did not converge");
            Cursor c = cur;
            if (sw_next == sw && attempt == 0) {
                blocks.swap(blocks_next);
                skipvec.swap(skipvec_next);
                c = c_next;
            } else {
                wplan(c, inc, specs, sw, count, skips, blocks, skipvec);
            }
            sw_next = -1;
            wupload(ctx, blocks, skipvec);
            ctx->ensure_stats((size_t)count * nstat);
            StatStripe *ss = (StatStripe *)st->stripes;
            svh::reset_batch(ctx, ctx->d_stats, (size_t)count * nstat * sizeof(sv_stats), ss,
                        (size_t)count * nstat * NSTRIPE * sizeof(StatStripe));
            hipEvent_t ev;
            ctx->time_begin(&ev);
            for (int k = 0; k < count; k++)
                launch(ctx->d_blocks + (size_t)k * nb, ss + (size_t)k * nstat * NSTRIPE, (uint32_t)k,
                       blocks.data() + (size_t)k * nb, k + 1 < count ? blocks.data() + (size_t)(k + 1) * nb : nullptr);
            ctx->time_end(ev, count);
            fold_stripes<<<(count * nstat + 63) / 64, 64, 0, ctx->stream>>>(ss, ctx->d_stats, count * nstat), SV_LAUNCHED("fold_stripes", ctx->stream);
            SV_HIP(hipGetLastError());
            if (sw + count < sweeps) {  // (the device runs this batch meanwhile)
                c_next = c;
                wplan(c_next, inc, specs, sw + count, std::min(BATCH, sweeps - sw - count), skips, blocks_next,
                      skipvec_next);
                sw_next = sw + count;
            }
            if (!may_reject) {  // threshold 0: no rejection can occur, so the stats copy is the one sync
                cur = c;
                break;
            }
            // the batch's statistics travel with the abort check (one synchronization per batch, not two); an
            // aborted batch's copy is simply overwritten by its replay's
            svh::finalize_stats(ctx->d_stats, (int64_t)count * nstat, ctx->stream);
            SV_HIP(hipMemcpyAsync(stats + (size_t)sw * nstat, ctx->d_stats, (size_t)count * nstat * sizeof(sv_stats),
                                  hipMemcpyDeviceToHost, ctx->stream));
            if (!wcheck(ctx, reps)) {
                ctx->time_collect();
                cur = c;
                stats_landed = true;
                break;
            }
            ctx->time_discard();
            sw_next = -1;  // (the replay changes the skips: the next batch is planned again)
            if (std::any_of(reps.begin(), reps.end(), [](const Report &r) { return r.block == OVERFLOW_BLOCK; })) {
                st->wf_off = true;  // the fused kernel's int32 image cannot hold the state: replay on the pass kernels
            } else {
                wabsorb(reps, sw, skips);
            }
            snapshot(st, true);
        }
        const bool deferred = !may_reject && ctx->defer_stats(stats + (size_t)sw * nstat, (int64_t)count * nstat);
        if (!may_reject && !deferred) svh::loc::queue_abort_copy(ctx);
        if (!deferred && !stats_landed) {
            svh::finalize_stats(ctx->d_stats, (int64_t)count * nstat, ctx->stream);
            SV_HIP(hipMemcpyAsync(stats + (size_t)sw * nstat, ctx->d_stats, (size_t)count * nstat * sizeof(sv_stats),
                                  hipMemcpyDeviceToHost, ctx->stream));
            SV_HIP(hipStreamSynchronize(ctx->stream));
        }
        if (!may_reject && !deferred) {
            svh::loc::check_abort_copy(ctx);
            ctx->time_collect();
        }
        for (int k = 0; k < count; k++) {
            for (int j = 0; j < nstat; j++) {
                stats[(size_t)(sw + k) * nstat + j].proposed = V;
                stats[(size_t)(sw + k) * nstat + j].rejections = 0;
            }
            for (int bi = 0; bi < nb; bi++) {
                auto it = skips.find({sw + k, bi});
                if (it != skips.end()) stats[(size_t)(sw + k) * nstat + stat_of[bi]].rejections += (int64_t)it->second.size();
            }
        }
        sw += count;
    }
}

// one CoexactUpdate sweep's colour passes (blocks: [0] metropolis, [1 + c] t of colour c)
void launch_coexact(sv_worldline *st, const WParams &P, const Block *blocks, StatStripe *stat, uint32_t k,
                    const JumpTables *T) {
    sv_ctx *ctx = st->ctx;
    if (st->N % 2 == 0) {  // grid-stride colour passes
        for (int c = 0; c < 2; c++) {
            if (st->v_is_float)
                coexact_gs<true><<<P.grid, 256, 0, ctx->stream>>>(P, st->m, st->v, c, blocks, ctx->d_skips, T, stat,
                                                                  wscratch(ctx), k), SV_LAUNCHED("coexact_gs<true>", ctx->stream);
            else
                coexact_gs<false><<<P.grid, 256, 0, ctx->stream>>>(P, st->m, st->v, c, blocks, ctx->d_skips, T, stat,
                                                                   wscratch(ctx), k), SV_LAUNCHED("coexact_gs<false>", ctx->stream);
        }
        return;
    }
    for (int c = 0; c < st->ncol; c++) {
        const int64_t nc = st->count[c];
        if (!nc) continue;
        const int grid = (int)((nc + 255) / 256);
        if (st->v_is_float)
            coexact_pass<true><<<grid, 256, 0, ctx->stream>>>(P, st->m, st->v, st->sites + st->offset[c], nc, c, blocks,
                                                              ctx->d_skips, T, stat, wscratch(ctx), k), SV_LAUNCHED("coexact_pass<true>", ctx->stream);
        else
            coexact_pass<false><<<grid, 256, 0, ctx->stream>>>(P, st->m, st->v, st->sites + st->offset[c], nc, c, blocks,
                                                               ctx->d_skips, T, stat, wscratch(ctx), k), SV_LAUNCHED("coexact_pass<false>", ctx->stream);
    }
}

// one checkerboard PlaquetteUpdate sweep (blocks: [0] metropolis, [1 + 2c] change_m, [2 + 2c] change_v)
void launch_plaquette_cb(sv_worldline *st, const WParams &P, const Block *blocks, StatStripe *stat, uint32_t k,
                         const JumpTables *T) {
    sv_ctx *ctx = st->ctx;
    if (st->N % 2 == 0) {  // grid-stride colour passes
        for (int c = 0; c < 2; c++) {
            if (st->v_is_float)
                plaquette_cb_gs<true><<<P.grid, 256, 0, ctx->stream>>>(P, st->m, st->v, c, blocks, ctx->d_skips, T,
                                                                       stat, wscratch(ctx), k), SV_LAUNCHED("plaquette_cb_gs<true>", ctx->stream);
            else
                plaquette_cb_gs<false><<<P.grid, 256, 0, ctx->stream>>>(P, st->m, st->v, c, blocks, ctx->d_skips, T,
                                                                        stat, wscratch(ctx), k), SV_LAUNCHED("plaquette_cb_gs<false>", ctx->stream);
        }
        return;
    }
    for (int c = 0; c < st->ncol; c++) {
        const int64_t nc = st->count[c];
        if (!nc) continue;
        const int grid = (int)((nc + 255) / 256);
        if (st->v_is_float)
            plaquette_cb_pass<true><<<grid, 256, 0, ctx->stream>>>(P, st->m, st->v, st->sites + st->offset[c], nc, c,
                                                                   blocks, ctx->d_skips, T, stat, wscratch(ctx), k), SV_LAUNCHED("plaquette_cb_pass<true>", ctx->stream);
        else
            plaquette_cb_pass<false><<<grid, 256, 0, ctx->stream>>>(P, st->m, st->v, st->sites + st->offset[c], nc, c,
                                                                    blocks, ctx->d_skips, T, stat, wscratch(ctx), k), SV_LAUNCHED("plaquette_cb_pass<false>", ctx->stream);
    }
}

std::vector<BlockSpec> coexact_specs(const sv_worldline *st) {
    std::vector<BlockSpec> specs;
    specs.push_back({UNIFORM, (uint32_t)((int64_t)st->N * st->N)});
    for (int c = 0; c < st->ncol; c++) specs.push_back({BOUNDED, (uint32_t)st->count[c]});
    return specs;
}

std::vector<BlockSpec> plaquette_cb_specs(const sv_worldline *st) {
    std::vector<BlockSpec> specs;
    specs.push_back({UNIFORM, (uint32_t)((int64_t)st->N * st->N)});
    for (int c = 0; c < st->ncol; c++) {
        specs.push_back({BOUNDED, (uint32_t)st->count[c]});
        specs.push_back({BOUNDED, (uint32_t)st->count[c]});
    }
    return specs;
}

}  // namespace

extern "C" {

int sv_worldline_create(sv_ctx *ctx, int32_t N, int32_t v_is_float, sv_worldline **out) {
    try {
        if (!ctx || !out) return -1;
        if (N < 2) throw std::invalid_argument("N must be >= 2");
        SV_HIP(hipSetDevice(ctx->device));
        sv_worldline *st = new sv_worldline();
        st->ctx = ctx;
        st->N = N;
        st->v_is_float = v_is_float ? 1 : 0;
        const size_t V = (size_t)N * N;
        const size_t vb = V * (st->v_is_float ? sizeof(double) : sizeof(int64_t));
        SV_HIP(hipMalloc(&st->m, 2 * V * sizeof(int64_t)));
        SV_HIP(hipMalloc(&st->v, vb));
        SV_HIP(hipMalloc(&st->snap_m, 2 * V * sizeof(int64_t)));
        SV_HIP(hipMalloc(&st->stripes, (size_t)2 * 64 * NSTRIPE * sizeof(StatStripe)));  // batch x 2 stats
        SV_HIP(hipMalloc(&st->snap_v, vb));
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

int sv_worldline_destroy(sv_worldline *st) {
    if (!st) return 0;
    int rc = sv_destroy_drain(st->ctx, "sv_worldline_destroy");  // (no queued work may still use the buffers)
    (void)hipFree(st->m);
    (void)hipFree(st->v);
    (void)hipFree(st->snap_m);
    (void)hipFree(st->snap_v);
    (void)hipFree(st->m_alt);
    (void)hipFree(st->v_alt);
    (void)hipFree(st->stripes);
    (void)hipFree(st->sites);
    if (st->f) (void)hipFree(st->f);
    if (st->d_aux) (void)hipFree(st->d_aux);
    if (st->order) (void)hipFree(st->order);
    if (st->pos) (void)hipFree(st->pos);
    if (st->lev) (void)hipFree(st->lev);
    if (st->ord64) (void)hipFree(st->ord64);
    if (st->lcnt) (void)hipFree(st->lcnt);
    for (uint32_t *h : st->h_perm)
        if (h) (void)hipHostFree(h);
    const hipError_t ee = st->emitter.release();
    if (ee != hipSuccess && !rc) {
        st->ctx->err = std::string("sv_worldline_destroy: an emission copy failed: ") + hipGetErrorString(ee);
        rc = -2;
    }
    delete st;
    return rc;
}

int sv_worldline_upload(sv_worldline *st, const int64_t *m, const void *v) {
    try {
        const size_t V = (size_t)st->N * st->N;
        const size_t vb = V * (st->v_is_float ? sizeof(double) : sizeof(int64_t));
        SV_HIP(hipSetDevice(st->ctx->device));
        SV_HIP(hipMemcpyAsync(st->m, m, 2 * V * sizeof(int64_t), hipMemcpyHostToDevice, st->ctx->stream));
        SV_HIP(hipMemcpyAsync(st->v, v, vb, hipMemcpyHostToDevice, st->ctx->stream));
        SV_HIP(hipStreamSynchronize(st->ctx->stream));
        return 0;
    } catch (const std::exception &e) {
        st->ctx->err = e.what();
        return -2;
    }
}

int sv_worldline_download(sv_worldline *st, int64_t *m, void *v) {
    try {
        const size_t V = (size_t)st->N * st->N;
        const size_t vb = V * (st->v_is_float ? sizeof(double) : sizeof(int64_t));
        SV_HIP(hipSetDevice(st->ctx->device));
        SV_HIP(hipMemcpyAsync(m, st->m, 2 * V * sizeof(int64_t), hipMemcpyDeviceToHost, st->ctx->stream));
        if (v) SV_HIP(hipMemcpyAsync(v, st->v, vb, hipMemcpyDeviceToHost, st->ctx->stream));
        SV_HIP(hipStreamSynchronize(st->ctx->stream));
        return 0;
    } catch (const std::exception &e) {
        st->ctx->err = e.what();
        return -2;
    }
}

int sv_worldline_coexact_run(sv_worldline *st, double kappa, double W_eff, int64_t interval_t, int32_t sweeps,
                             sv_rng *rng, sv_stats *stats) {
    if (!st || !rng || (sweeps > 0 && !stats)) return -1;
    sv_ctx *ctx = st->ctx;
    try {
        if (interval_t < 1 || interval_t > (1 << 20)) throw std::invalid_argument("interval_t must be in [1, 2^20]");
        SV_HIP(hipSetDevice(ctx->device));
        WParams P = wparams(st->N, kappa, W_eff, interval_t, u128{rng->inc_lo, rng->inc_hi});
        u128 inc{rng->inc_lo, rng->inc_hi};
        Cursor cur{u128{rng->state_lo, rng->state_hi}, (uint32_t)rng->has_uint32, rng->uinteger};
        const JumpTables *T = ctx->jump_tables(inc.hi, inc.lo);
        run_colour_sweeps(
            st, coexact_specs(st), sweeps, cur, inc, stats,
            [&](const Block *blocks, StatStripe *stat, uint32_t k, const Block *, const Block *) {
                launch_coexact(st, P, blocks, stat, k, T);
            }, 1, {},
            P.thr != 0);
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

int sv_worldline_coexact(sv_ctx *ctx, int32_t N, double kappa, double W_eff, int64_t interval_t, int64_t *m,
                         const void *v, int32_t v_is_float, int32_t sweeps, sv_rng *rng, sv_stats *stats) {
    sv_worldline *st = nullptr;
    int rc = sv_worldline_create(ctx, N, v_is_float, &st);
    if (rc) return rc;
    rc = sv_worldline_upload(st, m, v);
    if (!rc) rc = sv_worldline_coexact_run(st, kappa, W_eff, interval_t, sweeps, rng, stats);
    if (!rc) rc = sv_worldline_download(st, m, nullptr);
    sv_worldline_destroy(st);
    return rc;
}

int sv_worldline_plaquette_checkerboard_run(sv_worldline *st, double kappa, double W_eff, int32_t sweeps, sv_rng *rng,
                                            sv_stats *stats) {
    if (!st || !rng || (sweeps > 0 && !stats)) return -1;
    sv_ctx *ctx = st->ctx;
    try {
        SV_HIP(hipSetDevice(ctx->device));
        WParams P = wparams(st->N, kappa, W_eff, 1, u128{rng->inc_lo, rng->inc_hi});
        u128 inc{rng->inc_lo, rng->inc_hi};
        Cursor cur{u128{rng->state_lo, rng->state_hi}, (uint32_t)rng->has_uint32, rng->uinteger};
        const JumpTables *T = ctx->jump_tables(inc.hi, inc.lo);
        run_colour_sweeps(st, plaquette_cb_specs(st), sweeps, cur, inc, stats,
                          [&](const Block *blocks, StatStripe *stat, uint32_t k, const Block *, const Block *) {
                              launch_plaquette_cb(st, P, blocks, stat, k, T);
                          });
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

// Sequentially(PlaquetteUpdate checkerboard, CoexactUpdate) for `sweeps` steps in one call, the two
// generators drawing from ONE Generator (G1.rng is G2.rng) in the order Sequentially.step
// (combining.py:38-40) calls them; stats[2 s] is the Plaquette sweep of step s, stats[2 s + 1] the
// Coexact sweep.
int sv_worldline_plaquette_coexact_run(sv_worldline *st, double kappa, double W_eff, int64_t interval_t, int32_t sweeps,
                                       sv_rng *rng, sv_stats *stats) {
    if (!st || !rng || (sweeps > 0 && !stats)) return -1;
    sv_ctx *ctx = st->ctx;
    try {
        if (interval_t < 1 || interval_t > (1 << 20)) throw std::invalid_argument("interval_t must be in [1, 2^20]");
        SV_HIP(hipSetDevice(ctx->device));
        const u128 inc0{rng->inc_lo, rng->inc_hi};
        const WParams Pp = wparams(st->N, kappa, W_eff, 1, inc0), Pc = wparams(st->N, kappa, W_eff, interval_t, inc0);
        u128 inc{rng->inc_lo, rng->inc_hi};
        Cursor cur{u128{rng->state_lo, rng->state_hi}, (uint32_t)rng->has_uint32, rng->uinteger};
        const JumpTables *T = ctx->jump_tables(inc.hi, inc.lo);
        std::vector<BlockSpec> specs = plaquette_cb_specs(st);
        const int np = (int)specs.size();
        for (const BlockSpec &b : coexact_specs(st)) specs.push_back(b);
        std::vector<int> stat_of(specs.size(), 0);
        for (size_t b = np; b < specs.size(); b++) stat_of[b] = 1;
        constexpr bool use_wf = true;  // (worldline_step_fused; the four pass kernels where it does not apply)
        const int64_t N = st->N;
        // row-base advance maps of worldline_step_fused for 4 and 8 waves (rows per step NW: NW N draws, NW N / 4 words)
        const Affine adv[6] = {host_power(inc, 4 * (uint64_t)N), host_power(inc, 2 * (uint64_t)N), host_power(inc, (uint64_t)N),
                               host_power(inc, 8 * (uint64_t)N), host_power(inc, 4 * (uint64_t)N), host_power(inc, 2 * (uint64_t)N)};
        if (use_wf && N % 2 == 0 && !st->v_is_float && !st->m_alt) {
            SV_HIP(hipMalloc(&st->m_alt, 2 * (size_t)N * N * sizeof(int64_t)));
            SV_HIP(hipMalloc(&st->v_alt, (size_t)N * N * sizeof(int64_t)));
        }
        run_colour_sweeps(
            st, specs, sweeps, cur, inc, stats,
            [&](const Block *blocks, StatStripe *stat, uint32_t k, const Block *hblocks, const Block *) {
                if (use_wf && !st->wf_off && svh::wf_usable(st->N, st->v_is_float, W_eff, interval_t) &&
                    N * N < (int64_t(1) << 28)) {  // (launch_wf's 32-bit row offsets)
                    // one launch for the whole step (worldline_fused.hip); it writes the other buffer pair
                    const int64_t V = N * N;
                    svh::launch_wf(FGeom{(int32_t)N, (int32_t)N, 0, 0, (int32_t)N, (int32_t)N, N, V, 0}, kappa, W_eff,
                                   interval_t, st->m, (const int64_t *)st->v, st->m_alt, (int64_t *)st->v_alt,
                                   blocks, hblocks, ctx->d_skips, !svh::wf_fast(hblocks), T, adv, inc, stat, stat + NSTRIPE,
                                   wscratch(ctx), k, ctx->stream);
                    std::swap(st->m, st->m_alt);
                    std::swap(st->v, st->v_alt);
                } else {
                    launch_plaquette_cb(st, Pp, blocks, stat, k, T);
                    launch_coexact(st, Pc, blocks + np, stat + NSTRIPE, k, T);
                }
            },
            2, stat_of);
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

namespace {

void ordered_alloc(sv_worldline *st) {
    const int64_t V = (int64_t)st->N * st->N;
    if (!st->f) {
        SV_HIP(hipMalloc(&st->f, 2 * V * sizeof(double)));
        SV_HIP(hipMalloc(&st->order, V * sizeof(int32_t)));
        SV_HIP(hipMalloc(&st->pos, V * sizeof(int32_t)));
        SV_HIP(hipMalloc(&st->lev, V * sizeof(int32_t)));
        SV_HIP(hipMalloc(&st->ord64, V * sizeof(int64_t)));
        SV_HIP(hipMalloc(&st->lcnt, (V + 2 + LFLAGS) * sizeof(int32_t)));
    }
}

// One reference-order Plaquette sweep in the visit order already at st->ord64 on the stream (int64 plaquette
// indices, or 32-bit ones when o32): dependency levels on the device, then one launch per level; rejection replays
// as the pass kernels.  Synchronizes the stream before returning.
void ordered_sweep(sv_worldline *st, double kappa, double W_eff, bool o32, u128 inc, Cursor &cur, sv_stats *stats) {
    sv_ctx *ctx = st->ctx;
    {
        const int64_t N = st->N, V = N * N;
        WParams P = wparams(st->N, kappa, W_eff, 1, inc);
        const JumpTables *T = ctx->jump_tables(inc.hi, inc.lo);
        // Dependency levels of the visit order, on the device (order_positions .. order_level_lists)
        int32_t *flags = st->lcnt + V + 2;
        const int lgrid = (int)std::min<int64_t>((V + 255) / 256, 4096);
        SV_HIP(hipMemsetAsync(st->pos, 0xFF, V * sizeof(int32_t), ctx->stream));
        SV_HIP(hipMemsetAsync(st->lev, 0, V * sizeof(int32_t), ctx->stream));
        SV_HIP(hipMemsetAsync(st->lcnt, 0, (V + 2 + LFLAGS) * sizeof(int32_t), ctx->stream));
        if (o32)
            order_positions<uint32_t><<<lgrid, 256, 0, ctx->stream>>>((const uint32_t *)st->ord64, V, st->pos, flags), SV_LAUNCHED("order_positions<uint32_t>", ctx->stream);
        else
            order_positions<int64_t><<<lgrid, 256, 0, ctx->stream>>>(st->ord64, V, st->pos, flags), SV_LAUNCHED("order_positions<int64_t>", ctx->stream);
        int32_t hf[LFLAGS];
        for (int it = 0;; it += LFLAGS - 2) {
            // relaxations in batches; a batch whose last relaxation changed nothing has converged
            if (it > 0) SV_HIP(hipMemsetAsync(flags + 2, 0, (LFLAGS - 2) * sizeof(int32_t), ctx->stream));
            for (int j = 0; j < LFLAGS - 2; j++) order_levels<<<lgrid, 256, 0, ctx->stream>>>(N, st->pos, st->lev, flags, j), SV_LAUNCHED("order_levels", ctx->stream);
            SV_HIP(hipMemcpyAsync(hf, flags, sizeof(hf), hipMemcpyDeviceToHost, ctx->stream));
            SV_HIP(hipStreamSynchronize(ctx->stream));
            if (hf[0]) throw std::invalid_argument("order is not a permutation");
            if (!hf[LFLAGS - 1]) break;
            if (it > 2 * V) throw std::logic_error("order levels did not converge");
        }
        order_level_counts<<<lgrid, 256, 0, ctx->stream>>>(st->lev, V, st->lcnt, flags), SV_LAUNCHED("order_level_counts", ctx->stream);
        int32_t nlev = 0;
        SV_HIP(hipMemcpyAsync(&nlev, flags + 1, sizeof(int32_t), hipMemcpyDeviceToHost, ctx->stream));
        SV_HIP(hipStreamSynchronize(ctx->stream));
        std::vector<int32_t> start(nlev + 2, 0);
        SV_HIP(hipMemcpyAsync(start.data() + 1, st->lcnt, (nlev + 1) * sizeof(int32_t), hipMemcpyDeviceToHost,
                              ctx->stream));
        SV_HIP(hipStreamSynchronize(ctx->stream));
        for (int l = 1; l <= nlev + 1; l++) start[l] += start[l - 1];  // start[l] = first slot of level l
        SV_HIP(hipMemcpyAsync(st->lcnt, start.data(), (nlev + 1) * sizeof(int32_t), hipMemcpyHostToDevice, ctx->stream));
        order_level_lists<<<lgrid, 256, 0, ctx->stream>>>(st->lev, V, st->lcnt, st->order), SV_LAUNCHED("order_level_lists", ctx->stream);
        std::vector<BlockSpec> specs = {{BOUNDED, (uint32_t)V}, {BOUNDED, (uint32_t)V}, {UNIFORM, (uint32_t)V}};
        SkipMap skips;
        std::vector<Block> blocks;
        std::vector<uint32_t> skipvec;
        std::vector<Report> reps;
        snapshot(st, false);
        ctx->ensure_stats(1);
        const int grid = (int)std::min<int64_t>((V + 255) / 256, 8192);
        for (int attempt = 0;; attempt++) {
            if (attempt > 256) throw std::runtime_error("rejection replay did not converge");
            Cursor c = cur;
            wplan(c, inc, specs, 0, 1, skips, blocks, skipvec);
            wupload(ctx, blocks, skipvec);
            StatStripe *ss = (StatStripe *)st->stripes;
            svh::reset_batch(ctx, ctx->d_stats, sizeof(sv_stats), ss, NSTRIPE * sizeof(StatStripe));
            if (st->v_is_float)
                plaquette_f_init<true><<<grid, 256, 0, ctx->stream>>>(P, st->m, st->v, st->f), SV_LAUNCHED("plaquette_f_init<true>", ctx->stream);
            else
                plaquette_f_init<false><<<grid, 256, 0, ctx->stream>>>(P, st->m, st->v, st->f), SV_LAUNCHED("plaquette_f_init<false>", ctx->stream);
            for (int l = 1; l <= nlev; l++) {
                const int32_t cnt = start[l + 1] - start[l];
                if (!cnt) continue;
                const int g = (cnt + 255) / 256;
                if (st->v_is_float)
                    plaquette_level<true><<<g, 256, 0, ctx->stream>>>(P, st->m, st->v, st->f, st->order + start[l], cnt,
                                                                      st->pos, ctx->d_blocks, ctx->d_skips, T,
                                                                      ss, wscratch(ctx)), SV_LAUNCHED("plaquette_level<true>", ctx->stream);
                else
                    plaquette_level<false><<<g, 256, 0, ctx->stream>>>(P, st->m, st->v, st->f, st->order + start[l],
                                                                       cnt, st->pos, ctx->d_blocks, ctx->d_skips, T,
                                                                       ss, wscratch(ctx)), SV_LAUNCHED("plaquette_level<false>", ctx->stream);
            }
            fold_stripes<<<1, 64, 0, ctx->stream>>>(ss, ctx->d_stats, 1), SV_LAUNCHED("fold_stripes", ctx->stream);
            SV_HIP(hipGetLastError());
            if (!wcheck(ctx, reps)) {
                cur = c;
                break;
            }
            wabsorb(reps, 0, skips);
            snapshot(st, true);
        }
        svh::finalize_stats(ctx->d_stats, 1, ctx->stream);
        SV_HIP(hipMemcpyAsync(stats, ctx->d_stats, sizeof(sv_stats), hipMemcpyDeviceToHost, ctx->stream));
        SV_HIP(hipStreamSynchronize(ctx->stream));
        stats->proposed = V;
        int64_t rj = 0;
        for (auto &kv : skips) rj += (int64_t)kv.second.size();
        stats->rejections = rj;
    }
}

void store_cursor_w(const Cursor &cur, sv_rng *rng) {
    rng->state_hi = cur.s.hi;
    rng->state_lo = cur.s.lo;
    rng->has_uint32 = (int32_t)cur.has;
    rng->uinteger = cur.buf;
}

}  // namespace

int sv_worldline_plaquette_ordered_run(sv_worldline *st, double kappa, double W_eff, const int64_t *order,
                                       sv_rng *rng, sv_stats *stats) {
    if (!st || !rng || !stats || !order) return -1;
    sv_ctx *ctx = st->ctx;
    try {
        SV_HIP(hipSetDevice(ctx->device));
        const int64_t V = (int64_t)st->N * st->N;
        u128 inc{rng->inc_lo, rng->inc_hi};
        Cursor cur{u128{rng->state_lo, rng->state_hi}, (uint32_t)rng->has_uint32, rng->uinteger};
        ordered_alloc(st);
        SV_HIP(hipMemcpyAsync(st->ord64, order, V * sizeof(int64_t), hipMemcpyHostToDevice, ctx->stream));
        ordered_sweep(st, kappa, W_eff, false, inc, cur, stats);
        store_cursor_w(cur, rng);
        return 0;
    } catch (const std::exception &e) {
        ctx->err = e.what();
        return -2;
    }
}

namespace {

// `sweeps` reference-order Plaquette sweeps, each followed by one CoexactUpdate sweep when interval_t > 0 (stats then
// [2 s], [2 s + 1]), all on the one PCG64 stream; the visit orders from the legacy MT19937 state *mt
int reference_steps(sv_worldline *st, double kappa, double W_eff, int64_t interval_t, int32_t sweeps, sv_mt19937 *mt,
                    sv_rng *rng, sv_stats *stats) {
    if (!st || !rng || !mt || (sweeps > 0 && !stats)) return -1;
    sv_ctx *ctx = st->ctx;
    const int nstat = interval_t > 0 ? 2 : 1;
    try {
        if (sweeps < 0) throw std::invalid_argument("sweeps must be >= 0");
        if (sweeps == 0) return 0;
        SV_HIP(hipSetDevice(ctx->device));
        const int64_t V = (int64_t)st->N * st->N;
        u128 inc{rng->inc_lo, rng->inc_hi};
        Cursor cur{u128{rng->state_lo, rng->state_hi}, (uint32_t)rng->has_uint32, rng->uinteger};
        ordered_alloc(st);
        for (int i = 0; i < 2; i++)
            if (!st->h_perm[i]) SV_HIP(hipHostMalloc((void **)&st->h_perm[i], V * sizeof(uint32_t), hipHostMallocDefault));
        // Three-stage pipeline over the sweeps: while the device runs sweep s (visit order h_perm[s & 1]), one host
        // thread draws sweep s + 2's intervals from the legacy MT19937 stream (serial) and another applies sweep
        // s + 1's swaps.  The legacy state advances in the drawing thread only; the caller's copy on success.
        sv_mt19937 m = *mt;
        std::vector<uint32_t> jb[3];
        for (auto &j : jb) j.resize((size_t)V);
        sv::legacy_intervals(m.key, m.pos, V, jb[0].data());
        sv::shuffle_from_intervals(jb[0].data(), V, st->h_perm[0]);
        if (sweeps > 1) sv::legacy_intervals(m.key, m.pos, V, jb[1].data());
        for (int s = 0; s < sweeps; s++) {
            std::exception_ptr e_draw, e_swap;
            std::thread t_draw, t_swap;
            struct Join {
                std::thread &a, &b;
                ~Join() {
                    if (a.joinable()) a.join();
                    if (b.joinable()) b.join();
                }
            } join{t_draw, t_swap};
            if (s + 2 < sweeps)
                t_draw = std::thread([&, s] {
                    try {
                        sv::legacy_intervals(m.key, m.pos, V, jb[(s + 2) % 3].data());
                    } catch (...) {
                        e_draw = std::current_exception();
                    }
                });
            // (h_perm[(s + 1) & 1] last fed sweep s - 1's copy, which completed inside that synchronized sweep)
            if (s + 1 < sweeps)
                t_swap = std::thread([&, s] { sv::shuffle_from_intervals(jb[(s + 1) % 3].data(), V, st->h_perm[(s + 1) & 1]); });
            SV_HIP(hipMemcpyAsync(st->ord64, st->h_perm[s & 1], V * sizeof(uint32_t), hipMemcpyHostToDevice, ctx->stream));
            ordered_sweep(st, kappa, W_eff, true, inc, cur, stats + (size_t)s * nstat);
            if (interval_t > 0) {  // Sequentially(PlaquetteUpdate, CoexactUpdate), combining.py:38-40
                sv_rng r{cur.s.hi, cur.s.lo, inc.hi, inc.lo, (int32_t)cur.has, cur.buf};
                if (sv_worldline_coexact_run(st, kappa, W_eff, interval_t, 1, &r, stats + (size_t)s * nstat + 1))
                    throw std::runtime_error(ctx->err);
                cur = Cursor{u128{r.state_lo, r.state_hi}, (uint32_t)r.has_uint32, r.uinteger};
            }
            if (t_draw.joinable()) t_draw.join();
            if (t_swap.joinable()) t_swap.join();
            if (e_draw) std::rethrow_exception(e_draw);
        }
        *mt = m;
        store_cursor_w(cur, rng);
        return 0;
    } catch (const std::exception &e) {
        ctx->err = e.what();
        return -2;
    }
}

}  // namespace

int sv_worldline_plaquette_reference_run(sv_worldline *st, double kappa, double W_eff, int32_t sweeps, sv_mt19937 *mt,
                                         sv_rng *rng, sv_stats *stats) {
    return reference_steps(st, kappa, W_eff, 0, sweeps, mt, rng, stats);
}

int sv_worldline_plaquette_reference_coexact_run(sv_worldline *st, double kappa, double W_eff, int64_t interval_t,
                                                 int32_t steps, sv_mt19937 *mt, sv_rng *rng, sv_stats *stats) {
    if (interval_t < 1) {
        if (st) st->ctx->err = "interval_t must be >= 1";
        return -2;
    }
    return reference_steps(st, kappa, W_eff, interval_t, steps, mt, rng, stats);
}

int sv_worldline_plaquette(sv_ctx *ctx, int32_t N, double kappa, double W_eff, int64_t *m, void *v,
                           int32_t v_is_float, const int64_t *order, sv_rng *rng, sv_stats *stats) {
    sv_worldline *st = nullptr;
    int rc = sv_worldline_create(ctx, N, v_is_float, &st);
    if (rc) return rc;
    rc = sv_worldline_upload(st, m, v);
    if (!rc) rc = sv_worldline_plaquette_ordered_run(st, kappa, W_eff, order, rng, stats);
    if (!rc) rc = sv_worldline_download(st, m, v);
    sv_worldline_destroy(st);
    return rc;
}

}  // extern "C"
