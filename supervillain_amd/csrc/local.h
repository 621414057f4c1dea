// local.h -- shared by the grid-stride "local update" passes (villain_local.hip: Site/Link/Exact/
// Cohomology; worldline_local.hip: Vortex/Wrapping).  Device: per-lane NumPy stream addressing for
// arithmetic position sequences, stats flush, small math.  Host: batch driver with rejection replay.
#pragma once
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <numeric>

#include "villain.h"

namespace sv {
namespace loc {

__device__ __forceinline__ u128 lbase(const Block &b) { return u128{b.base_lo, b.base_hi}; }

__device__ __forceinline__ void lreport(const DevScratch &S, uint32_t sweep, uint32_t block, uint32_t pos) {
    uint32_t i = atomicAdd(S.nreport, 1u);
    if (i < (uint32_t)MAX_REPORTS) S.reports[i] = Report{sweep, block, pos, 0};
    __hip_atomic_store(S.abort, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// stream position of bounded draw d, accounting for known rejected positions (sorted)
__device__ __forceinline__ uint32_t lskip_pos(const Block &b, const uint32_t *skips, uint32_t d) {
    uint32_t q = d;
    for (int i = 0; i < b.nskip; i++)
        if (skips[b.skip0 + i] <= q) q++;
    return q;
}

// value of choice index j among (-iv .. -1, 1 .. iv): link.py:43, exact.py:38, cohomology.py:60
__device__ __forceinline__ int64_t nonzero_value(uint32_t j, int64_t iv) {
    return (int64_t)j < iv ? (int64_t)j - iv : (int64_t)j - iv + 1;
}

// Uniform block draws at positions p0, p0 + stride, ...: one table jump, then one affine map each.
struct UniLane {
    u128 s;
    bool init;
    __device__ __forceinline__ uint64_t next(const JumpTables *T, const Block &b, uint32_t p, const Affine &adv) {
        s = init ? apply(adv, s) : jump(T, lbase(b), p);
        init = true;
        return xsl_rr(s);
    }
};

// Bounded block uint32 words at draw positions q0, q0 + stride, ... (stride even, no skips): NumPy's
// buffered half-word first, then the low and high halves of consecutive u64s.
struct BndLane {
    u128 s;
    bool init;
    __device__ __forceinline__ uint32_t next(const JumpTables *T, const Block &b, uint32_t q, const Affine &adv_half) {
        if (b.has && q == 0) return b.buf;
        const uint32_t qq = q - b.has;
        s = init ? apply(adv_half, s) : jump(T, lbase(b), qq >> 1);
        init = true;
        const uint64_t X = xsl_rr(s);
        return (qq & 1) ? (uint32_t)(X >> 32) : (uint32_t)X;
    }
};

// uint32 of bounded draw d by a full jump (blocks with known rejections)
__device__ __forceinline__ uint32_t bnd_word_slow(const JumpTables *T, const Block &b, const uint32_t *skips,
                                                  uint32_t d, uint32_t *qout) {
    const uint32_t q = lskip_pos(b, skips, d);
    *qout = q;
    if (b.has && q == 0) return b.buf;
    const uint32_t qq = q - b.has;
    const uint64_t X = xsl_rr(jump(T, lbase(b), qq >> 1));
    return (qq & 1) ? (uint32_t)(X >> 32) : (uint32_t)X;
}


// One atomic quadruple per workgroup (all threads call it); psum is the lane's exact acceptance sum (common.h).
__device__ __forceinline__ void lflush(sv_stats *st, int64_t acc, const AccFx &psum) {
    __shared__ unsigned long long s_w[4][16];
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

__device__ __forceinline__ double clip01(double p) {
    p = p < 0.0 ? 0.0 : p;
    return p > 1.0 ? 1.0 : p;
}

// colour-index e -> site (even N: row-major parity colouring, e = s >> 1)
__device__ __forceinline__ int64_t even_site(int64_t e, int64_t N, int color) {
    const int64_t half = N >> 1;
    const int64_t t = e / half, j = e - t * half;
    return t * N + 2 * j + ((color + t) & 1);
}


}  // namespace loc
}  // namespace sv

namespace svh {
namespace loc {

// Batches with no possible rejection skip the abort read: the flag is queued to pinned memory ahead of
// the stats copy and checked after that copy's synchronization.
static inline void queue_abort_copy(sv_ctx *ctx) {
    if (!ctx->h_abort) SV_HIP(hipHostMalloc((void **)&ctx->h_abort, sizeof(int32_t), hipHostMallocDefault));
    SV_HIP(hipMemcpyAsync(ctx->h_abort, ctx->d_abort, sizeof(int32_t), hipMemcpyDeviceToHost, ctx->stream));
}
static inline void check_abort_copy(sv_ctx *ctx) {
    if (*ctx->h_abort) throw std::runtime_error("unexpected NumPy Lemire rejection report");
}
using namespace sv;

static inline int gcd_i(int64_t a, int64_t b) { return (int)std::gcd(a, b); }

// Grid for a pass over `count` elements whose lanes advance by the whole grid: the stride is a
// multiple of `mult` (and of 256) so that per-lane stream positions stay arithmetic.  Lanes take
// about `iters` (default 2; measured flat from 1 to 16 at L=4096) elements each (one 4-level table jump amortized over them), the grid staying between
// 2^17 lanes (2 waves per SIMD) and 2^19.
static inline int grid_for(int64_t count, int64_t mult) {
    constexpr int64_t iters = 2;
    const int64_t target = std::min<int64_t>(1 << 19, std::max<int64_t>(1 << 17, count / iters));
    if (count <= target) return (int)std::max<int64_t>(1, (count + 255) / 256);
    const int64_t l = mult / gcd_i(mult, 256) * 256;  // lcm(mult, 256)
    int64_t S = std::max<int64_t>(1, target / l) * l;
    // at most 1024 grid-stride iterations per lane: a lane's exact acceptance sum must stay below 2^11 terms (common.h)
    S = std::max<int64_t>(S, (count + 1024 * l - 1) / (1024 * l) * l);
    return (int)(S / 256);
}

static inline Cursor cursor_of(const sv_rng *rng) {
    return Cursor{u128{rng->state_lo, rng->state_hi}, (uint32_t)rng->has_uint32, rng->uinteger};
}

static inline void store_cursor(const Cursor &c, sv_rng *rng) {
    rng->state_hi = c.s.hi;
    rng->state_lo = c.s.lo;
    rng->has_uint32 = (int32_t)c.has;
    rng->uinteger = c.buf;
}

// Pairwise-sum plan of NumPy's pairwise_sum (numpy/_core/src/umath/loops_utils.h.src) for length n.
static inline void pairwise_plan(int64_t i0, int64_t n, std::vector<int32_t> &leaves, std::vector<uint8_t> &prog) {
    if (n <= 128) {
        leaves.push_back((int32_t)i0);
        leaves.push_back((int32_t)n);
        prog.push_back(0);
        return;
    }
    int64_t n2 = n / 2;
    n2 -= n2 % 8;
    pairwise_plan(i0, n2, leaves, prog);
    pairwise_plan(i0 + n2, n - n2, leaves, prog);
    prog.push_back(1);
}

// Run `sweeps` sweeps of a local update in batches of up to 64: plan every draw block of the batch,
// launch every pass, then read the abort flag once.  A Lemire rejection (known only on the device)
// restores the batch-start snapshot and replays the batch with the rejected stream position skipped.
// snapshot()/restore() save and put back the fields the update changes; with may_reject == false (no
// bounded draws, or a Lemire threshold of 0: power-of-two choice counts never reject) no snapshot is taken.
template <class Snapshot, class Restore, class LaunchSweep>
static inline void run_batches(sv_ctx *ctx, const std::vector<BlockSpec> &specs, int32_t sweeps, Cursor &cur, u128 inc,
                        sv_stats *stats, bool may_reject, Snapshot snapshot, Restore restore,
                        LaunchSweep launch_sweep) {
    const int nb = (int)specs.size();
    SkipMap skips;
    std::vector<Block> blocks;
    std::vector<uint32_t> skipvec;
    const int BATCH = 64;
    for (int sw = 0; sw < sweeps;) {
        const int count = std::min(BATCH, sweeps - sw);
        if (may_reject) snapshot();
        for (int attempt = 0;; attempt++) {
            if (attempt > 256) throw std::runtime_error("rejection replay did not converge");
            Cursor c = cur;
            plan_sweeps(ctx, c, inc, specs, sw, count, skips, blocks, skipvec);
            upload_plan(ctx, blocks, skipvec);
            ctx->ensure_stats(count);
            reset_batch(ctx, ctx->d_stats, count * sizeof(sv_stats));
            hipEvent_t ev;
            ctx->time_begin(&ev);
            for (int k = 0; k < count; k++) launch_sweep(k, ctx->d_blocks + (size_t)k * nb, ctx->d_stats + k);
            ctx->time_end(ev, count);
            SV_HIP(hipGetLastError());
            if (!may_reject) {  // threshold 0: no rejection can occur, so the stats copy is the one sync
                cur = c;
                break;
            }
            AbortInfo a = read_abort(ctx);
            if (a.abort) ctx->time_discard();
            ctx->time_collect();
            if (!a.abort) {
                cur = c;
                break;
            }
            absorb_reports(a, sw, skips);
            restore();
        }
        if (!may_reject && ctx->defer_stats(stats + sw, count)) {  // landed by sv_ctx_sync
            sw += count;
            continue;
        }
        if (!may_reject) queue_abort_copy(ctx);
        finalize_stats(ctx->d_stats, count, ctx->stream);
        SV_HIP(hipMemcpyAsync(stats + sw, ctx->d_stats, count * sizeof(sv_stats), hipMemcpyDeviceToHost, ctx->stream));
        SV_HIP(hipStreamSynchronize(ctx->stream));
        if (!may_reject) {
            check_abort_copy(ctx);
            ctx->time_collect();
        }
        for (int k = 0; k < count; k++) stats[sw + k].rejections = rejections_in(skips, sw + k, nb);
        sw += count;
    }
}

}  // namespace loc
}  // namespace svh
