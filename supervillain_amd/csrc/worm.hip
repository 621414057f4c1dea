// worm.hip -- the two ClassicWorms on batches of independent chains.
//
// A worm is a sequential random walk (supervillain/generator/villain/worm.py:133-183,
// supervillain/generator/worldline/worm.py:26-94): every move reads the link it would cross, draws
// from the chain's own NumPy stream and maybe moves.  Nothing inside one worm is parallel, so the
// GPU form runs ONE CHAIN PER LANE: lane r owns replica r's fields, its PCG64 state (stepped serially
// in registers, exactly NumPy's order of uniform / bounded draws) and its displacement histogram.
// This pays off only for batches (BASELINE config 5: 1024 replicas); a single lattice is a batch
// of one, correct but latency-bound.
//
// Memory per move: the crossed link's n (or m) and the two phi values of d(phi) on it (or v values of
// delta(v)/W), one conditional store of the link, one fire-and-forget histogram increment (a no-return
// global atomic on the lane's private histogram: no wait on its latency).  d(phi) and delta(v)/W are
// formed on the fly in the reference's operator order, so no derived arrays are kept.
#include <cstring>
#include <mutex>

#include "common.h"

namespace sv {
namespace {

static constexpr double TWO_PI = 6.283185307179586;  // Python's 2*np.pi

struct WormRng {
    uint64_t s_lo, s_hi, inc_lo, inc_hi;
    uint32_t has, buf;
};

// One chain's NumPy Generator(PCG64), stepped serially.
struct LaneRng {
    u128 s, inc;
    uint32_t has, buf;

    __device__ uint64_t next64() {
        s = add(mul(s, mult()), inc);  // advance first, then XSL-RR
        return xsl_rr(s);
    }
    __device__ double uniform01() { return to_double(next64()); }  // uniform(0, 1) = 0 + 1 * next_double
    __device__ uint32_t next32() {
        if (has) {
            has = 0;
            return buf;
        }
        const uint64_t x = next64();
        has = 1;
        buf = (uint32_t)(x >> 32);
        return (uint32_t)x;
    }
    // integers(0, k): NumPy's buffered 32-bit Lemire (rejection loop included)
    __device__ uint32_t bounded(uint32_t k) {
        const uint32_t thr = (0u - k) % k;
        uint64_t m = (uint64_t)next32() * k;
        uint32_t left = (uint32_t)m;
        if (left < k)
            while (left < thr) {
                m = (uint64_t)next32() * k;
                left = (uint32_t)m;
            }
        return (uint32_t)(m >> 32);
    }
    // integers(0, k) for a power-of-two k (threshold 0: never rejects)
    __device__ uint32_t bounded_pow2(uint32_t k) { return (uint32_t)(((uint64_t)next32() * k) >> 32); }
};

struct WormArgs {
    int32_t R, N;
    int64_t V;
    double kappa;
    int32_t w_is_one;    // Villain: W == 1 (open worms allowed, worm.py:123,143)
    double Weff;         // Worldline: S._W
    int32_t v_is_float;  // Worldline: v stored as float64 (W = infinity)
    const double *phi;   // Villain (R, N, N)
    int64_t *n;          // Villain (R, 2, N, N)
    int64_t *m;          // Worldline (R, 2, N, N)
    const void *v;       // Worldline (R, N, N)
    WormRng *rng;        // R
    unsigned long long *hist;  // R * V (zeroed; the last worm of the call is tallied) or nullptr
    int64_t *lengths;          // R * worms or nullptr
    int32_t worms;
    int64_t max_moves;
    int32_t *status;  // set to 1 when a worm exceeds max_moves
};

__device__ __forceinline__ int32_t wrapi(int32_t i, int32_t N) { return i < 0 ? i + N : (i >= N ? i - N : i); }

// Villain ClassicWorm, worm.py:110-131 (per-step draws) + worm_kernel :133-183.
__global__ __launch_bounds__(64) void villain_worm(WormArgs A) {
    const int32_t r = blockIdx.x * 64 + threadIdx.x;
    if (r >= A.R) return;
    const int32_t N = A.N;
    const int64_t V = A.V;
    const double *phi = A.phi + (int64_t)r * V;
    int64_t *n = A.n + (int64_t)r * 2 * V;
    unsigned long long *hist = A.hist ? A.hist + (int64_t)r * V : nullptr;
    WormRng g0 = A.rng[r];
    LaneRng g{u128{g0.s_lo, g0.s_hi}, u128{g0.inc_lo, g0.inc_hi}, g0.has, g0.buf};
    const double half_kappa = A.kappa / 2;
    for (int32_t w = 0; w < A.worms; w++) {
        const int64_t orientation = g.bounded_pow2(2) ? +1 : -1;       // choice([-1, +1])      :114
        const uint32_t ti = g.bounded((uint32_t)V);                       // choice(coordinates)   :119
        const int32_t tt = (int32_t)(ti / (uint32_t)N), tx = (int32_t)(ti % (uint32_t)N);
        int32_t ht = tt, hx = tx;
        if (A.w_is_one) {                                                 // :123
            const uint32_t hi = g.bounded((uint32_t)V);
            ht = (int32_t)(hi / (uint32_t)N), hx = (int32_t)(hi % (uint32_t)N);
        }
        const bool tally = hist && w == A.worms - 1;
        int64_t len = 0;
        for (;;) {
            // every candidate move's operands are loaded before the draws, so the memory round trip
            // overlaps the RNG arithmetic (the walk is latency-bound): phi on the plaquette's corners and
            // n on its four sides
            const int32_t tp = wrapi(ht + 1, N), xp = wrapi(hx + 1, N);
            const int64_t s00 = (int64_t)ht * N + hx, s10 = (int64_t)tp * N + hx, s01 = (int64_t)ht * N + xp;
            const int64_t s11 = (int64_t)tp * N + xp;
            const double p00 = phi[s00], p10 = phi[s10], p01 = phi[s01], p11 = phi[s11];
            const int64_t nE = n[s00], nN = n[V + s10], nWe = n[s01], nS = n[V + s00];
            if ((ht == tt && hx == tx) || A.w_is_one)                     // :143
                if (g.uniform01() >= 0.8) break;
            if (len >= A.max_moves) {
                atomicOr(A.status, 1);
                break;
            }
            const uint32_t c = g.bounded_pow2(4);                         // :148
            // neighbouring plaquette and crossed link (two_dimensional.py:255-300):
            // east (t, x-1) via (0, t, x); north (t+1, x) via (1, t+1, x); west (t, x+1) via (0, t, x+1);
            // south (t-1, x) via (1, t, x); d(phi) on link (mu, s) = 0 + (phi[s + e_mu] - phi[s]) (worm.py:104)
            int32_t nt = ht, nx = hx;
            int64_t l, nl;
            double dphi;
            if (c == 0) {
                nx = wrapi(hx - 1, N), l = s00, nl = nE, dphi = 0.0 + (p10 - p00);
            } else if (c == 1) {
                nt = tp, l = V + s10, nl = nN, dphi = 0.0 + (p11 - p10);
            } else if (c == 2) {
                nx = xp, l = s01, nl = nWe, dphi = 0.0 + (p11 - p01);
            } else {
                nt = wrapi(ht - 1, N), l = V + s00, nl = nS, dphi = 0.0 + (p01 - p00);
            }
            const double change_link = dphi - TWO_PI * (double)nl;         // :157
            const int64_t dn = (c < 2) ? orientation : -orientation;      // change_n[choice]
            const double dS = (half_kappa * ((-TWO_PI) * (double)dn)) * (2 * change_link - TWO_PI * (double)dn);
            double Ap = exp(-dS);                                         // :169
            Ap = Ap < 1.0 ? Ap : 1.0;
            if (g.uniform01() < Ap) {                                     // :172
                ht = nt, hx = nx;
                n[l] = nl + dn;
            }
            if (tally) atomicAdd(&hist[(int64_t)wrapi(ht - tt, N) * N + wrapi(hx - tx, N)], 1ull);  // :181-182
            len++;
        }
        if (A.lengths) A.lengths[(int64_t)r * A.worms + w] = len;
    }
    A.rng[r].s_lo = g.s.lo;
    A.rng[r].s_hi = g.s.hi;
    A.rng[r].has = g.has;
    A.rng[r].buf = g.buf;
}

// delta(v)/W on link (k, s) from v[s] and v[b], reference.py:27-45 with ('delta',2) rows (0,0,1,-1),(1,0,0,+1):
// k=0: (0 - (-(v[s] - v[s-e1]))) / W;  k=1: (0 - (v[s] - v[s-e0])) / W  (worldline/worm.py:164)
// (raw 64-bit loads: int64, or float64 when v_is_float)
__device__ __forceinline__ double dv_by_W_vals(uint64_t vs, uint64_t vb, int v_is_float, int k, double Weff) {
    double d;
    if (v_is_float) {
        const double a = __longlong_as_double((long long)vs) - __longlong_as_double((long long)vb);
        d = k == 0 ? 0.0 - (-a) : 0.0 - a;
    } else {
        const int64_t a = (int64_t)vs - (int64_t)vb;
        d = (double)(k == 0 ? 0 - (-a) : 0 - a);
    }
    return d / Weff;
}

// Worldline ClassicWorm, worldline/worm.py:146-193 (per-step draws) + worm_kernel :26-94.
__global__ __launch_bounds__(64) void worldline_worm(WormArgs A) {
    const int32_t r = blockIdx.x * 64 + threadIdx.x;
    if (r >= A.R) return;
    const int32_t N = A.N;
    const int64_t V = A.V;
    int64_t *m = A.m + (int64_t)r * 2 * V;
    const void *v = A.v_is_float ? (const void *)((const double *)A.v + (int64_t)r * V)
                                 : (const void *)((const int64_t *)A.v + (int64_t)r * V);
    unsigned long long *hist = A.hist ? A.hist + (int64_t)r * V : nullptr;
    WormRng g0 = A.rng[r];
    LaneRng g{u128{g0.s_lo, g0.s_hi}, u128{g0.inc_lo, g0.inc_hi}, g0.has, g0.buf};
    const double inv2k = 1.0 / (2.0 * A.kappa);
    for (int32_t w = 0; w < A.worms; w++) {
        const int64_t orientation = g.bounded_pow2(2) ? +1 : -1;       // :158
        const uint32_t ti = g.bounded((uint32_t)V);                       // :165
        const int32_t tt = (int32_t)(ti / (uint32_t)N), tx = (int32_t)(ti % (uint32_t)N);
        int32_t ht = tt, hx = tx;
        const bool tally = hist && w == A.worms - 1;
        int64_t len = 0;
        for (;;) {
            // operands of all four candidate moves first (latency overlaps the draws): m on the four links
            // at and behind the head, v on the four sites their delta(v) reads
            const int32_t tm = wrapi(ht - 1, N), xm = wrapi(hx - 1, N);
            const int64_t s00 = (int64_t)ht * N + hx, s0m = (int64_t)ht * N + xm, sm0 = (int64_t)tm * N + hx;
            const int64_t smm = (int64_t)tm * N + xm;
            const int64_t m0f = m[s00], m1f = m[V + s00], m0b = m[sm0], m1b = m[V + s0m];
            const uint64_t *vr = (const uint64_t *)v;
            const uint64_t v00 = vr[s00], v0m = vr[s0m], vm0 = vr[sm0], vmm = vr[smm];
            if (ht == tt && hx == tx)                                     // :49-50
                if (g.uniform01() < 1.0 / 5) break;
            if (len >= A.max_moves) {
                atomicOr(A.status, 1);
                break;
            }
            const uint32_t c = g.bounded_pow2(4);                         // :53
            const int k = c & 1;
            const bool forward = c < 2;
            // +e0 crosses (0, head), +e1 (1, head), -e0 (0, head - e0), -e1 (1, head - e1) (:70-73);
            // delta(v)/W on (k, s) reads v[s] and v[s - e1] (k = 0) or v[s - e0] (k = 1)
            int32_t nt = ht, nx = hx;
            int64_t l, ml;
            uint64_t va, vb;
            if (c == 0) {
                nt = wrapi(ht + 1, N), l = s00, ml = m0f, va = v00, vb = v0m;
            } else if (c == 1) {
                nx = wrapi(hx + 1, N), l = V + s00, ml = m1f, va = v00, vb = vm0;
            } else if (c == 2) {
                nt = tm, l = sm0, ml = m0b, va = vm0, vb = vmm;
            } else {
                nx = xm, l = V + s0m, ml = m1b, va = v0m, vb = vmm;
            }
            const double change_link = (double)ml - dv_by_W_vals(va, vb, A.v_is_float, k, A.Weff);  // :76
            const int64_t dm = forward ? orientation : -orientation;      // change_m[choice]
            const double dS = (inv2k * (double)dm) * (2.0 * change_link + (double)dm);
            double Ap = exp(-dS);                                         // :83
            Ap = 1.0 < Ap ? 1.0 : Ap;
            if (g.uniform01() < Ap) {                                     // :86
                ht = nt, hx = nx;
                m[l] = ml + dm;
            }
            if (tally) atomicAdd(&hist[(int64_t)wrapi(ht - tt, N) * N + wrapi(hx - tx, N)], 1ull);  // :93
            len++;
        }
        if (A.lengths) A.lengths[(int64_t)r * A.worms + w] = len;
    }
    A.rng[r].s_lo = g.s.lo;
    A.rng[r].s_hi = g.s.hi;
    A.rng[r].has = g.has;
    A.rng[r].buf = g.buf;
}

// Device scratch of one call: rng[R] | status | lengths[R*worms] | hist[R*V]; cached per context.
struct WormScratch {
    char *d = nullptr;
    size_t cap = 0;
};

std::map<sv_ctx *, WormScratch> g_scratch;
std::mutex g_scratch_mu;  // contexts live on different threads; the map is shared

char *worm_scratch(sv_ctx *ctx, size_t bytes) {
    std::lock_guard<std::mutex> lock(g_scratch_mu);
    WormScratch &w = g_scratch[ctx];
    if (bytes > w.cap) {
        SV_HIP(hipStreamSynchronize(ctx->stream));
        if (w.d) SV_HIP(hipFree(w.d));
        w.d = nullptr;
        w.cap = 0;
        SV_HIP(hipMalloc((void **)&w.d, bytes));
        w.cap = bytes;
    }
    return w.d;
}

size_t align256(size_t x) { return (x + 255) / 256 * 256; }

// Shared driver: copy the rngs in, launch, copy rngs / lengths / histograms back.  Synchronous.
void run_worms(sv_ctx *ctx, bool worldline, WormArgs A, sv_rng *rngs, int64_t *hist, int64_t *lengths) {
    if (A.R < 1 || A.N < 2) throw std::invalid_argument("need R >= 1 chains of N >= 2");
    if (A.worms < 0) throw std::invalid_argument("worms must be >= 0");
    if (A.V >= (1LL << 32)) throw std::invalid_argument("lattice too large for integers(0, V) on 32 bits");
    if (A.kappa <= 0) throw std::invalid_argument("kappa must be positive");
    if (A.worms == 0) return;
    const size_t R = (size_t)A.R;
    const size_t o_st = align256(R * sizeof(WormRng)), o_len = o_st + 256;
    const size_t o_hist = align256(o_len + R * A.worms * sizeof(int64_t));
    const size_t total = o_hist + (hist ? R * (size_t)A.V * sizeof(int64_t) : 0);
    char *d = worm_scratch(ctx, total);
    std::vector<WormRng> h(R);
    for (size_t r = 0; r < R; r++)
        h[r] = WormRng{rngs[r].state_lo, rngs[r].state_hi, rngs[r].inc_lo, rngs[r].inc_hi, (uint32_t)rngs[r].has_uint32,
                       rngs[r].uinteger};
    SV_HIP(hipMemcpyAsync(d, h.data(), R * sizeof(WormRng), hipMemcpyHostToDevice, ctx->stream));
    SV_HIP(hipMemsetAsync(d + o_st, 0, 256, ctx->stream));
    if (hist) SV_HIP(hipMemsetAsync(d + o_hist, 0, R * (size_t)A.V * sizeof(int64_t), ctx->stream));
    A.rng = (WormRng *)d;
    A.status = (int32_t *)(d + o_st);
    A.lengths = (int64_t *)(d + o_len);
    A.hist = hist ? (unsigned long long *)(d + o_hist) : nullptr;
    hipEvent_t ev;
    ctx->time_begin(&ev);
    const unsigned grid = (unsigned)((R + 63) / 64);
    if (worldline) worldline_worm<<<grid, 64, 0, ctx->stream>>>(A), SV_LAUNCHED("worldline_worm", ctx->stream);
    else villain_worm<<<grid, 64, 0, ctx->stream>>>(A), SV_LAUNCHED("villain_worm", ctx->stream);
    ctx->time_end(ev, 1);
    SV_HIP(hipGetLastError());
    int32_t status = 0;
    SV_HIP(hipMemcpyAsync(h.data(), d, R * sizeof(WormRng), hipMemcpyDeviceToHost, ctx->stream));
    SV_HIP(hipMemcpyAsync(&status, d + o_st, sizeof(int32_t), hipMemcpyDeviceToHost, ctx->stream));
    if (lengths)
        SV_HIP(hipMemcpyAsync(lengths, d + o_len, R * A.worms * sizeof(int64_t), hipMemcpyDeviceToHost, ctx->stream));
    if (hist) SV_HIP(hipMemcpyAsync(hist, d + o_hist, R * (size_t)A.V * sizeof(int64_t), hipMemcpyDeviceToHost, ctx->stream));
    SV_HIP(hipStreamSynchronize(ctx->stream));
    ctx->time_collect();
    for (size_t r = 0; r < R; r++) {
        rngs[r].state_lo = h[r].s_lo;
        rngs[r].state_hi = h[r].s_hi;
        rngs[r].has_uint32 = (int32_t)h[r].has;
        rngs[r].uinteger = h[r].buf;
    }
    if (status) throw std::runtime_error("a worm exceeded max_moves (fields and rng states are mid-worm)");
}

WormArgs base_args(int32_t R, int32_t N, double kappa, int32_t worms, int64_t max_moves) {
    WormArgs A{};
    A.R = R;
    A.N = N;
    A.V = (int64_t)N * N;
    A.kappa = kappa;
    A.worms = worms;
    A.max_moves = max_moves > 0 ? max_moves : INT64_MAX;
    return A;
}

}  // namespace

void worm_release(sv_ctx *ctx) {
    std::lock_guard<std::mutex> lock(g_scratch_mu);
    auto it = g_scratch.find(ctx);
    if (it == g_scratch.end()) return;
    if (it->second.d) (void)hipFree(it->second.d);
    g_scratch.erase(it);
}

// Villain worms over R chains stored as (R, N, N) phi and (R, 2, N, N) n on the device (replicas.hip).
void villain_worms_device(sv_ctx *ctx, int32_t R, int32_t N, const double *phi, int64_t *n, double kappa, int64_t W,
                          int32_t worms, int64_t max_moves, sv_rng *rngs, int64_t *hist, int64_t *lengths) {
    WormArgs A = base_args(R, N, kappa, worms, max_moves);
    A.w_is_one = W == 1;
    A.phi = phi;
    A.n = n;
    run_worms(ctx, false, A, rngs, hist, lengths);
}

}  // namespace sv

using namespace sv;

extern "C" {

int sv_villain_worm_run(sv_villain *st, double kappa, int64_t W, int32_t worms, int64_t max_moves, sv_rng *rng,
                        int64_t *hist, int64_t *lengths) {
    if (!st || !rng) return -1;
    sv_ctx *ctx = st->ctx;
    try {
        SV_HIP(hipSetDevice(ctx->device));
        villain_worms_device(ctx, 1, st->N, st->phi[st->cur], st->n[st->cur], kappa, W, worms, max_moves, rng, hist,
                             lengths);
        return 0;
    } catch (const std::exception &e) {
        ctx->err = e.what();
        return -2;
    }
}

int sv_worldline_worm_run(sv_worldline *st, double kappa, double W_eff, int32_t worms, int64_t max_moves, sv_rng *rng,
                          int64_t *hist, int64_t *lengths) {
    if (!st || !rng) return -1;
    sv_ctx *ctx = st->ctx;
    try {
        SV_HIP(hipSetDevice(ctx->device));
        WormArgs A = base_args(1, st->N, kappa, worms, max_moves);
        A.Weff = W_eff;
        A.v_is_float = st->v_is_float;
        A.m = st->m;
        A.v = st->v;
        run_worms(ctx, true, A, rng, hist, lengths);
        return 0;
    } catch (const std::exception &e) {
        ctx->err = e.what();
        return -2;
    }
}

int sv_worldline_worm_batch(sv_ctx *ctx, int32_t R, int32_t N, double kappa, double W_eff, int64_t *m, const void *v,
                            int32_t v_is_float, int32_t worms, int64_t max_moves, sv_rng *rngs, int64_t *hist,
                            int64_t *lengths) {
    if (!ctx || !m || !v || !rngs) return -1;
    int64_t *dm = nullptr;
    void *dv = nullptr;
    try {
        SV_HIP(hipSetDevice(ctx->device));
        if (R < 1 || N < 2) throw std::invalid_argument("need R >= 1 chains of N >= 2");
        const size_t V = (size_t)N * N;
        SV_HIP(hipMalloc((void **)&dm, 2 * R * V * sizeof(int64_t)));
        SV_HIP(hipMalloc(&dv, R * V * 8));
        SV_HIP(hipMemcpyAsync(dm, m, 2 * R * V * sizeof(int64_t), hipMemcpyHostToDevice, ctx->stream));
        SV_HIP(hipMemcpyAsync(dv, v, R * V * 8, hipMemcpyHostToDevice, ctx->stream));
        WormArgs A = base_args(R, N, kappa, worms, max_moves);
        A.Weff = W_eff;
        A.v_is_float = v_is_float;
        A.m = dm;
        A.v = dv;
        run_worms(ctx, true, A, rngs, hist, lengths);
        SV_HIP(hipMemcpy(m, dm, 2 * R * V * sizeof(int64_t), hipMemcpyDeviceToHost));
        SV_HIP(hipFree(dm));
        SV_HIP(hipFree(dv));
        return 0;
    } catch (const std::exception &e) {
        if (dm) (void)hipFree(dm);
        if (dv) (void)hipFree(dv);
        ctx->err = e.what();
        return -2;
    }
}

}  // extern "C"
