// worldline_local.hip -- the Worldline Hammer's VortexUpdate and WrappingUpdate
// on gfx950, bit-exact replays of the reference chain under a fixed NumPy seed:
//
//   VortexUpdate    supervillain/generator/worldline/vortex.py:51-136    v only, checkerboard
//   WrappingUpdate  supervillain/generator/worldline/wrapping.py:43-90   m on whole torus cycles
//
// Vortex: one grid-stride colour pass per colour (local.h stream addressing).  For integer v (finite
// W) delta(v) is exact, so the pass recomputes it from v on the fly (the reference's incremental
// delta_v, vortex.py:98/130, is bit-identical to that); for float v (W = inf) the incremental patches
// round differently, so delta_v lives in HBM, rebuilt at sweep start and patched like the reference.
//
// Wrapping: per sweep 2N cycle proposals.  The mu = 0 cycles (columns) are NumPy's axis-0 sum -- a
// sequential chain over t per column -- done by one wave per 16 columns while three waves stage the
// link terms through LDS; the mu = 1 cycles (rows) are NumPy's pairwise sum of a contiguous row, one
// workgroup per row (8 lanes per <=128-element leaf, one per pairwise accumulator).
#include <cmath>
#include <cstdio>

#include "local.h"

namespace sv {

#define WTWO_PI 6.283185307179586

// x / W.  For W a power of two (W = 1, 2, 4, ...) x * (1/W) is the same correctly rounded value and
// avoids the FP64 division sequence.
__device__ __forceinline__ double div_w(double x, double Weff, double Winv, int wpow2) {
    return wpow2 ? x * Winv : x / Weff;
}

struct VxParams {
    int32_t N;
    int64_t V;
    double hk;          // 0.5 / kappa
    double Weff;        // Worldline._W
    double Winv;        // 1 / W when W is a power of two
    int32_t wpow2;
    double lo, range;   // W = inf: uniform(-interval_v, +interval_v)
    int64_t iv;         // finite W: choice over (-iv .. -1, 1 .. iv)
    uint32_t k, thr;
};

using namespace loc;

__device__ __forceinline__ int64_t wl_site(int64_t e, int64_t N, int color) {
    const int64_t half = N >> 1;
    const int64_t t = e / half, j = e - t * half;
    return t * N + 2 * j + ((color + t) & 1);
}

// raw dense delta(v) (reference.py:27-45; rows ('delta',2) = (0,0,1,-1),(1,0,0,+1)) for float v
__global__ void vortex_dv_init(int32_t N, const double *v, double *dv, const int32_t *abort) {
    if (*(volatile const int32_t *)abort) return;
    const int64_t V = (int64_t)N * N;
    for (int64_t s = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; s < V; s += (int64_t)gridDim.x * blockDim.x) {
        int64_t t, x;
        divmod_site(s, N, t, x);
        const double vs = v[s];
        dv[s] = 0.0 - (-(vs - v[t * N + (x == 0 ? N - 1 : x - 1)]));
        dv[V + s] = 0.0 - (vs - v[(t == 0 ? N - 1 : t - 1) * N + x]);
    }
}

// One colour pass of VortexUpdate (vortex.py:100-131).  Blocks: [0] metropolis uniform(V), [1 + c] the
// colour's proposals (choice(vs) for finite W, uniform(-iv, iv) for W = inf).
template <bool EVEN, bool VF>
__global__ __launch_bounds__(256) void vortex_pass(VxParams P, const int64_t *m, void *vv, double *dv,
                                                   const int32_t *sites, int64_t nc, int color, const Block *blocks,
                                                   const uint32_t *skips, const JumpTables *T, Affine adv_m,
                                                   Affine adv_p, sv_stats *stat, DevScratch Sx, uint32_t sweep) {
    if (*(volatile const int32_t *)Sx.abort) return;
    const int64_t N = P.N, V = P.V;
    const int64_t S = (int64_t)gridDim.x * blockDim.x;
    const Block BM = blocks[0], BP = blocks[1 + color];
    const bool slow = !VF && BP.nskip > 0;
    UniLane um{u128{0, 0}, false}, up{u128{0, 0}, false};
    BndLane bp{u128{0, 0}, false};
    int64_t acc_count = 0;
    AccFx psum;  // exact acceptance sum (common.h)
    for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < nc; e += S) {
        const int64_t s = EVEN ? wl_site(e, N, color) : sites[e];
        if (!EVEN) um.init = up.init = bp.init = false;
        const double u = 0.0 + 1.0 * to_double(um.next(T, BM, (uint32_t)s, adv_m));
        int64_t t, x;
        divmod_site(s, N, t, x);
        const int64_t f0 = ((t + 1 == N) ? 0 : t + 1) * N + x, f1 = t * N + ((x + 1 == N) ? 0 : x + 1);
        const int64_t L0 = s, L0f = f1, L1 = V + s, L1f = V + f0;
        double a, c0, c0f, c1, c1f, d0, d0f, d1, d1f;
        int64_t ai = 0;
        if (VF) {
            a = P.lo + P.range * to_double(up.next(T, BP, (uint32_t)e, adv_p));
            c0 = div_w(0.0 - (-a), P.Weff, P.Winv, P.wpow2);
            c0f = div_w(0.0 + (-a), P.Weff, P.Winv, P.wpow2);
            c1 = div_w(0.0 - a, P.Weff, P.Winv, P.wpow2);
            c1f = div_w(0.0 + a, P.Weff, P.Winv, P.wpow2);
            d0 = dv[L0];
            d0f = dv[L0f];
            d1 = dv[L1];
            d1f = dv[L1f];
        } else {
            uint32_t q = (uint32_t)e, w;
            if (slow) w = bnd_word_slow(T, BP, skips, (uint32_t)e, &q);
            else w = bp.next(T, BP, (uint32_t)e, adv_p);
            bool rej;
            const uint32_t idx = lemire(w, P.k, P.thr, &rej);
            if (rej) lreport(Sx, sweep, 1u + (uint32_t)color, q);
            ai = nonzero_value(idx, P.iv);
            a = (double)ai;
            c0 = div_w((double)(0 - (-ai)), P.Weff, P.Winv, P.wpow2);
            c0f = div_w((double)(0 + (-ai)), P.Weff, P.Winv, P.wpow2);
            c1 = div_w((double)(0 - ai), P.Weff, P.Winv, P.wpow2);
            c1f = div_w((double)(0 + ai), P.Weff, P.Winv, P.wpow2);
            // delta(v) of the current integer v (exact; equals the reference's incremental delta_v)
            const int64_t *vi = (const int64_t *)vv;
            const int64_t vs = vi[s];
            d0 = (double)(0 - (-(vs - vi[t * N + ((x == 0) ? N - 1 : x - 1)])));
            d0f = (double)(0 - (-(vi[f1] - vs)));
            d1 = (double)(0 - (vs - vi[((t == 0) ? N - 1 : t - 1) * N + x]));
            d1f = (double)(0 - (vi[f0] - vs));
        }
        double dS = 0.0;  // coface_sum_at order: l1[x], l1[x+e0], l0[x], l0[x+e1]
        dS += (P.hk * (-c1)) * ((2.0 * ((double)m[L1] - div_w(d1, P.Weff, P.Winv, P.wpow2))) - c1);
        dS += (P.hk * (-c1f)) * ((2.0 * ((double)m[L1f] - div_w(d1f, P.Weff, P.Winv, P.wpow2))) - c1f);
        dS += (P.hk * (-c0)) * ((2.0 * ((double)m[L0] - div_w(d0, P.Weff, P.Winv, P.wpow2))) - c0);
        dS += (P.hk * (-c0f)) * ((2.0 * ((double)m[L0f] - div_w(d0f, P.Weff, P.Winv, P.wpow2))) - c0f);
        const double p = clip01(exp(-dS));
        const int acc = u < p;
        acc_count += acc;
        fx_add(psum, p);
        if (VF) {
            const double ap = a * (double)acc;
            double *vf = (double *)vv;
            vf[s] = vf[s] + ap;
            dv[L0] = d0 - (-ap);
            dv[L0f] = d0f + (-ap);
            dv[L1] = d1 - ap;
            dv[L1f] = d1f + ap;
        } else if (acc) {
            ((int64_t *)vv)[s] += ai;
        }
    }
    lflush(stat, acc_count, psum);
}

// ------------------------------------------------------------------------------------------------
// WrappingUpdate.  Blocks: [0] choice(w, 2N) (mu = 0 cycles x = 0..N-1, then mu = 1 cycles t = 0..N-1),
// [1] uniform(0, 1, 2N) in the same order (wrapping.py:62-80).
struct WrParams {
    int32_t N;
    int64_t V;
    double hk;    // 0.5 / kappa
    double Weff;
    double Winv;
    int32_t wpow2;
    int64_t iw;
    uint32_t k, thr;
};

// delta(v)/W on link (mu, t, x) (reference.py:27-45 then / _W, wrapping.py:69)
template <bool VF>
__device__ __forceinline__ double wr_dvw(const void *v, int64_t N, int mu, int64_t t, int64_t x, const WrParams &P) {
    const int64_t s = t * N + x;
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
    return div_w(d, P.Weff, P.Winv, P.wpow2);
}

// dS_link = ((0.5/kappa) * cm) * ((2 * (m - delta(v)/W)) + cm)   (wrapping.py:69)
template <bool VF>
__device__ __forceinline__ double wr_term(const WrParams &P, const int64_t *m, const void *v, int mu, int64_t t,
                                          int64_t x, int64_t c) {
    const double dvw = wr_dvw<VF>(v, P.N, mu, t, x, P);
    return (P.hk * (double)c) * ((2.0 * ((double)m[mu * P.V + t * P.N + x] - dvw)) + (double)c);
}

__global__ void wrap_draw(WrParams P, const Block *blocks, const uint32_t *skips, const JumpTables *T, int64_t *cprop,
                          DevScratch Sx, uint32_t sweep) {
    if (*(volatile const int32_t *)Sx.abort) return;
    const int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (j >= 2 * (int64_t)P.N) return;
    uint32_t q;
    const uint32_t w = bnd_word_slow(T, blocks[0], skips, (uint32_t)j, &q);
    bool rej;
    const uint32_t idx = lemire(w, P.k, P.thr, &rej);
    if (rej) lreport(Sx, sweep, 0u, q);
    cprop[j] = nonzero_value(idx, P.iw);
}

// mu = 0 cycles: dS[x] = sum over t of dS_link[0][t, x], sequentially from t = 0 (NumPy axis-0 reduce).
// Workgroup = 16 columns; waves 1..3 stage RC rows x 16 columns of link terms in LDS (double buffered),
// wave 0 lanes 0..15 add them in order.
static constexpr int WR_CW = 8, WR_RC = 192, WR_LOADERS = 192;
template <bool VF>
__global__ __launch_bounds__(256) void wrap_cols(WrParams P, const int64_t *m, const void *v, const int64_t *cprop,
                                                 double *dS, const int32_t *abort) {
    if (*(volatile const int32_t *)abort) return;
    __shared__ double tile[2][WR_RC][WR_CW + 1];
    const int64_t N = P.N;
    const int64_t x0 = (int64_t)blockIdx.x * WR_CW;
    const int tid = threadIdx.x;
    const int nch = (int)((N + WR_RC - 1) / WR_RC);
    // loader thread lt (waves 1..3) owns column lt % WR_CW and rows lt / WR_CW + 24 k of each chunk
    const int lt = tid - 64, col = lt & (WR_CW - 1), r0 = lt / WR_CW;
    const int64_t xl = x0 + col;
    const int64_t cl = (tid >= 64 && xl < N) ? cprop[xl] : 0;
    auto fill = [&](int ch) {
        if (xl >= N) return;
#pragma unroll
        for (int k = 0; k < WR_RC / (WR_LOADERS / WR_CW); k++) {
            const int r = r0 + k * (WR_LOADERS / WR_CW);
            const int64_t t = (int64_t)ch * WR_RC + r;
            if (t < N) tile[ch & 1][r][col] = wr_term<VF>(P, m, v, 0, t, xl, cl);
        }
    };
    if (tid >= 64) fill(0);
    __syncthreads();
    double acc = 0.0;
    for (int ch = 0; ch < nch; ch++) {
        if (tid >= 64) {
            if (ch + 1 < nch) fill(ch + 1);
        } else if (tid < WR_CW && x0 + tid < N) {
            const int64_t left = N - (int64_t)ch * WR_RC;
            const int rows = left < WR_RC ? (int)left : WR_RC;
            int r = 0;
            if (ch == 0) {
                acc = tile[0][0][tid];
                r = 1;
            }
            for (; r < rows; r++) acc = acc + tile[ch & 1][r][tid];
        }
        __syncthreads();
    }
    if (tid < WR_CW && x0 + tid < N) dS[x0 + tid] = acc;
}

// mu = 1 cycles: dS[N + t] = NumPy pairwise sum of the contiguous row dS_link[1][t, :].  One workgroup
// per row: leaf j (<= 128 elements) is summed by 8 lanes, lane a holding pairwise accumulator a.
static constexpr int WR_MAX_LEAVES = 2048;
template <bool VF>
__global__ __launch_bounds__(256) void wrap_rows(WrParams P, const int64_t *m, const void *v, const int64_t *cprop,
                                                 double *dS, const int32_t *leaves, const uint8_t *prog, int32_t nleaf,
                                                 int32_t nprog, const int32_t *abort) {
    if (*(volatile const int32_t *)abort) return;
    __shared__ double leafv[WR_MAX_LEAVES];
    const int64_t N = P.N, t = blockIdx.x;
    const int64_t c = cprop[N + t];
    const int tid = threadIdx.x, a = tid & 7;
    for (int j = tid >> 3; j < nleaf; j += 32) {
        const int64_t i0 = leaves[2 * j], len = leaves[2 * j + 1];
        double res = 0.0;
        if (len < 8) {
            if (a == 0)
                for (int64_t i = 0; i < len; i++) res += wr_term<VF>(P, m, v, 1, t, i0 + i, c);
        } else {
            const int64_t n8 = len - (len % 8);
            double r = wr_term<VF>(P, m, v, 1, t, i0 + a, c);
            for (int64_t i = 8; i < n8; i += 8) r += wr_term<VF>(P, m, v, 1, t, i0 + i + a, c);
            // ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7)) across the 8 lanes
            const double r1 = __shfl_xor(r, 1);
            const double p01 = (a & 1) ? r1 + r : r + r1;
            const double p23 = __shfl_xor(p01, 2);
            const double q = (a & 2) ? p23 + p01 : p01 + p23;
            const double q2 = __shfl_xor(q, 4);
            res = (a & 4) ? q2 + q : q + q2;
            if (a == 0)
                for (int64_t i = n8; i < len; i++) res += wr_term<VF>(P, m, v, 1, t, i0 + i, c);
        }
        if (a == 0) leafv[j] = res;
    }
    __syncthreads();
    if (tid == 0) {
        double stk[40];
        int top = 0, nl = 0;
        for (int pc = 0; pc < nprog; pc++) {
            if (prog[pc] == 0) stk[top++] = leafv[nl++];
            else {
                const double b = stk[--top];
                stk[top - 1] = stk[top - 1] + b;
            }
        }
        dS[N + t] = stk[0];
    }
}

// Metropolis on the 2N cycles (wrapping.py:71-84): accf[j] = uniform < clip(exp(-dS[j]))
__global__ __launch_bounds__(256) void wrap_metropolis(WrParams P, const Block *blocks, const JumpTables *T,
                                                       const double *dS, int32_t *accf, sv_stats *stat,
                                                       const int32_t *abort) {
    if (*(volatile const int32_t *)abort) return;
    const int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    int64_t acc_count = 0;
    AccFx psum;  // exact acceptance sum (common.h)
    if (j < 2 * (int64_t)P.N) {
        const double p = clip01(exp(-dS[j]));
        const double u = 0.0 + 1.0 * to_double(xsl_rr(jump(T, lbase(blocks[1]), (uint32_t)j)));
        const int acc = u < p;
        accf[j] = acc;
        acc_count = acc;
        fx_add(psum, p);
    }
    lflush(stat, acc_count, psum);
}

// m + change_m on the accepted cycles (wrapping.py:81, :90)
__global__ void wrap_apply(WrParams P, int64_t *m, const int64_t *cprop, const int32_t *accf, const int32_t *abort) {
    if (*(volatile const int32_t *)abort) return;
    const int64_t N = P.N, V = P.V;
    for (int64_t l = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; l < 2 * V; l += (int64_t)gridDim.x * blockDim.x) {
        const int mu = l >= V;
        const int64_t s = l - (mu ? V : 0);
        int64_t t, x;
        divmod_site(s, N, t, x);
        const int64_t j = mu ? N + t : x;
        if (accf[j]) m[l] += cprop[j];
    }
}

}  // namespace sv

// ==================================================================================================
// host drivers
// ==================================================================================================
namespace svh {
using namespace loc;

static void set_winv(double W, double &Winv, int32_t &pow2) {
    int e = 0;
    pow2 = std::isfinite(W) && W > 0 && std::frexp(W, &e) == 0.5;
    Winv = pow2 ? 1.0 / W : 0.0;
}

static void wl_bounded(int64_t iv, uint32_t &k, uint32_t &thr) {
    if (iv < 1) throw std::invalid_argument("the interval must be >= 1");
    if (iv > (1 << 20)) throw std::invalid_argument("interval too large");
    k = (uint32_t)(2 * iv);
    thr = (uint32_t)((0u - k) % k);
}

// snapshot / restore of the worldline fields an update changes
static void wl_copy(sv_worldline *st, bool to_snap, bool m_, bool v_) {
    sv_ctx *ctx = st->ctx;
    const size_t V = (size_t)st->N * st->N;
    const size_t vb = V * (st->v_is_float ? sizeof(double) : sizeof(int64_t));
    if (m_)
        SV_HIP(hipMemcpyAsync(to_snap ? st->snap_m : st->m, to_snap ? st->m : st->snap_m, 2 * V * sizeof(int64_t),
                              hipMemcpyDeviceToDevice, ctx->stream));
    if (v_)
        SV_HIP(hipMemcpyAsync(to_snap ? st->snap_v : st->v, to_snap ? st->v : st->snap_v, vb, hipMemcpyDeviceToDevice,
                              ctx->stream));
}

}  // namespace svh

using namespace svh;

extern "C" {

int sv_worldline_vortex_run(sv_worldline *st, double kappa, double W_eff, int64_t interval_v, int32_t sweeps,
                            sv_rng *rng, sv_stats *stats) {
    if (!st || !rng || (sweeps > 0 && !stats)) return -1;
    sv_ctx *ctx = st->ctx;
    try {
        if (sweeps < 0) throw std::invalid_argument("sweeps must be >= 0");
        SV_HIP(hipSetDevice(ctx->device));
        const int32_t N = st->N;
        const int64_t V = (int64_t)N * N;
        const bool vf = st->v_is_float;
        VxParams P{};
        P.N = N;
        P.V = V;
        P.hk = 0.5 / kappa;
        P.Weff = W_eff;
        set_winv(W_eff, P.Winv, P.wpow2);
        if (vf) {
            if (interval_v < 1) throw std::invalid_argument("the interval must be >= 1");
            P.lo = -(double)interval_v;
            P.range = (double)interval_v - (-(double)interval_v);
        } else {
            wl_bounded(interval_v, P.k, P.thr);
            P.iv = interval_v;
        }
        u128 inc{rng->inc_lo, rng->inc_hi};
        Cursor cur = cursor_of(rng);
        const JumpTables *T = ctx->jump_tables(inc.hi, inc.lo);
        std::vector<BlockSpec> specs{{UNIFORM, (uint32_t)V}};
        for (int c = 0; c < st->ncol; c++) specs.push_back({vf ? UNIFORM : BOUNDED, (uint32_t)st->count[c]});
        const bool even = N % 2 == 0;
        const int grid = grid_for(V / 2 + 1, N);
        const int64_t Sl = (int64_t)grid * 256;
        const Affine adv_m = host_power(inc, 2 * Sl), adv_p = host_power(inc, vf ? Sl : Sl / 2);
        if (vf && !st->f) SV_HIP(hipMalloc(&st->f, 2 * V * sizeof(double)));  // delta_v (vortex.py:98)
        const int gi = (int)std::min<int64_t>((V + 255) / 256, 4096);
        run_batches(
            ctx, specs, sweeps, cur, inc, stats, !vf && P.thr != 0, [&] { wl_copy(st, true, false, true); },
            [&] { wl_copy(st, false, false, true); },
            [&](int k, const Block *B, sv_stats *ds) {
                if (vf) vortex_dv_init<<<gi, 256, 0, ctx->stream>>>(N, (const double *)st->v, st->f, ctx->d_abort), SV_LAUNCHED("vortex_dv_init", ctx->stream);
                for (int c = 0; c < st->ncol; c++) {
                    const int64_t nc = st->count[c];
                    if (!nc) continue;
                    const int32_t *sites = st->sites + st->offset[c];
                    const int g = even ? grid : (int)((nc + 255) / 256);
                    if (even && vf)
                        vortex_pass<true, true><<<g, 256, 0, ctx->stream>>>(P, st->m, st->v, st->f, sites, nc, c, B,
                                                                          ctx->d_skips, T, adv_m, adv_p, ds,
                                                                          scratch(ctx), (uint32_t)k), SV_LAUNCHED("vortex_pass<true, true>", ctx->stream);
                    else if (even)
                        vortex_pass<true, false><<<g, 256, 0, ctx->stream>>>(P, st->m, st->v, st->f, sites, nc, c, B,
                                                                           ctx->d_skips, T, adv_m, adv_p, ds,
                                                                           scratch(ctx), (uint32_t)k), SV_LAUNCHED("vortex_pass<true, false>", ctx->stream);
                    else if (vf)
                        vortex_pass<false, true><<<g, 256, 0, ctx->stream>>>(P, st->m, st->v, st->f, sites, nc, c, B,
                                                                           ctx->d_skips, T, adv_m, adv_p, ds,
                                                                           scratch(ctx), (uint32_t)k), SV_LAUNCHED("vortex_pass<false, true>", ctx->stream);
                    else
                        vortex_pass<false, false><<<g, 256, 0, ctx->stream>>>(P, st->m, st->v, st->f, sites, nc, c,
                                                                            B, ctx->d_skips, T, adv_m, adv_p, ds,
                                                                            scratch(ctx), (uint32_t)k), SV_LAUNCHED("vortex_pass<false, false>", ctx->stream);
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

int sv_worldline_wrapping_run(sv_worldline *st, double kappa, double W_eff, int64_t interval_w, int32_t sweeps,
                              sv_rng *rng, sv_stats *stats) {
    if (!st || !rng || (sweeps > 0 && !stats)) return -1;
    sv_ctx *ctx = st->ctx;
    try {
        if (sweeps < 0) throw std::invalid_argument("sweeps must be >= 0");
        SV_HIP(hipSetDevice(ctx->device));
        const int32_t N = st->N;
        const int64_t V = (int64_t)N * N;
        WrParams P{};
        P.N = N;
        P.V = V;
        P.hk = 0.5 / kappa;
        P.Weff = W_eff;
        set_winv(W_eff, P.Winv, P.wpow2);
        P.iw = interval_w;
        wl_bounded(interval_w, P.k, P.thr);
        u128 inc{rng->inc_lo, rng->inc_hi};
        Cursor cur = cursor_of(rng);
        const JumpTables *T = ctx->jump_tables(inc.hi, inc.lo);
        const std::vector<BlockSpec> specs{{BOUNDED, (uint32_t)(2 * N)}, {UNIFORM, (uint32_t)(2 * N)}};
        std::vector<int32_t> leaves;
        std::vector<uint8_t> prog;
        pairwise_plan(0, N, leaves, prog);
        const int32_t nleaf = (int32_t)(leaves.size() / 2);
        if (nleaf > WR_MAX_LEAVES) throw std::invalid_argument("lattice too large for the row sums");
        // device scratch: cprop (2N i64) | dS (2N f64) | accf (2N i32) | leaves | prog
        const size_t o_ds = 16 * (size_t)N, o_acc = o_ds + 16 * (size_t)N, o_lv = o_acc + ((8 * (size_t)N + 63) / 64) * 64;
        const size_t o_pg = o_lv + leaves.size() * sizeof(int32_t), total = o_pg + prog.size();
        if (total > st->aux_cap) {
            SV_HIP(hipStreamSynchronize(ctx->stream));
            if (st->d_aux) SV_HIP(hipFree(st->d_aux));
            st->d_aux = nullptr;
            st->aux_cap = 0;
            SV_HIP(hipMalloc((void **)&st->d_aux, total));
            st->aux_cap = total;
        }
        char *d = st->d_aux;
        std::vector<char> plan(total - o_lv);
        memcpy(plan.data(), leaves.data(), leaves.size() * sizeof(int32_t));
        memcpy(plan.data() + (o_pg - o_lv), prog.data(), prog.size());
        SV_HIP(hipMemcpy(d + o_lv, plan.data(), plan.size(), hipMemcpyHostToDevice));  // synchronous (pageable)
        int64_t *cprop = (int64_t *)d;
        double *dS = (double *)(d + o_ds);
        int32_t *accf = (int32_t *)(d + o_acc);
        const int32_t *lv = (const int32_t *)(d + o_lv);
        const uint8_t *pg = (const uint8_t *)(d + o_pg);
        const bool vf = st->v_is_float;
        const int g2n = (int)((2 * (int64_t)N + 255) / 256);
        const int gcols = (int)((N + WR_CW - 1) / WR_CW);
        const int gapp = (int)std::min<int64_t>((2 * V + 255) / 256, 8192);
        run_batches(
            ctx, specs, sweeps, cur, inc, stats, P.thr != 0, [&] { wl_copy(st, true, true, false); },
            [&] { wl_copy(st, false, true, false); },
            [&](int k, const Block *B, sv_stats *ds) {
                wrap_draw<<<g2n, 256, 0, ctx->stream>>>(P, B, ctx->d_skips, T, cprop, scratch(ctx), (uint32_t)k), SV_LAUNCHED("wrap_draw", ctx->stream);
                if (vf) {
                    wrap_cols<true><<<gcols, 256, 0, ctx->stream>>>(P, st->m, st->v, cprop, dS, ctx->d_abort), SV_LAUNCHED("wrap_cols<true>", ctx->stream);
                    wrap_rows<true><<<N, 256, 0, ctx->stream>>>(P, st->m, st->v, cprop, dS, lv, pg, nleaf,
                                                                (int32_t)prog.size(), ctx->d_abort), SV_LAUNCHED("wrap_rows<true>", ctx->stream);
                } else {
                    wrap_cols<false><<<gcols, 256, 0, ctx->stream>>>(P, st->m, st->v, cprop, dS, ctx->d_abort), SV_LAUNCHED("wrap_cols<false>", ctx->stream);
                    wrap_rows<false><<<N, 256, 0, ctx->stream>>>(P, st->m, st->v, cprop, dS, lv, pg, nleaf,
                                                                 (int32_t)prog.size(), ctx->d_abort), SV_LAUNCHED("wrap_rows<false>", ctx->stream);
                }
                wrap_metropolis<<<g2n, 256, 0, ctx->stream>>>(P, B, T, dS, accf, ds, ctx->d_abort), SV_LAUNCHED("wrap_metropolis", ctx->stream);
                wrap_apply<<<gapp, 256, 0, ctx->stream>>>(P, st->m, cprop, accf, ctx->d_abort), SV_LAUNCHED("wrap_apply", ctx->stream);
            });
        for (int k = 0; k < sweeps; k++) stats[k].proposed = 2 * N;
        store_cursor(cur, rng);
        return 0;
    } catch (const std::exception &e) {
        ctx->err = e.what();
        return -2;
    }
}

}  // extern "C"
