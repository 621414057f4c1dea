// replicas.hip -- a batch of independent Villain NeighborhoodUpdate chains (BASELINE config 5:
// 1024 replicas of L=128 at W=2 with inline observables; SURVEY.md 8e "replicas shard trivially").
//
// R replicas of one even N share every launch: one fused sweep kernel per sweep covers all of them
// (workgroup runs of tiles_per_rep serve one replica), each replica replaying its own NumPy PCG64
// stream.  Small lattices cannot fill 256 CUs on their own; batched they do.
//
// Planning.  Without rejections a sweep consumes exactly 4V u64 of a replica's stream (V metropolis,
// then per colour V/2 dphi and 4 x V/4 words of choices -- the buffered half-word parity `has` never
// changes because every choice block has an even number of draws), so every block descriptor is a
// closed-form jump from the replica's batch-start state: a device kernel writes all R x sweeps x 11
// descriptors at once.  A replica that met a NumPy Lemire rejection is planned on the host for the
// batches it affects (the shared skip machinery of villain.hip), and the batch is replayed from the
// failing sweep exactly like the single-lattice driver.
//
// Inline observables (ActionDensity, InternalEnergyDensity, WindingSquared, TorusWrapping) are summed
// by the sweep kernel while it writes the finished rows (0 extra HBM bytes).
#include <chrono>
#include <cstdio>
#include <algorithm>
#include <array>
#include <cstring>
#include <thread>

#include "villain.h"

namespace sv {

struct PlanIn {
    uint64_t s_lo, s_hi;  // cursor: state before the batch's first draw
    uint32_t has, buf;
};

static constexpr int REP_BATCH = 64;  // sweeps per batch (r4 A/B, profiles/r04_repbatch_ab.txt)
static constexpr int NB = 11;  // blocks per sweep (even N: 2 colours)

// u64 offset of block b inside a sweep (h = V/4 words per choice block)
__device__ __forceinline__ uint64_t block_off(int b, uint64_t V) {
    const uint64_t nc = V / 2, h = V / 4;
    if (b == 0) return 0;
    if (b == 1) return V;
    if (b <= 5) return V + nc + (uint64_t)(b - 2) * h;
    if (b == 6) return V + 3 * nc;
    return V + 4 * nc + (uint64_t)(b - 7) * h;
}

__global__ void plan_replicas(const PlanIn *in, const JumpTables *const *Trep, Block *out, int R, int count,
                              uint64_t V) {
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (i >= (int64_t)R * count * NB) return;
    const int b = (int)(i % NB);
    const int k = (int)((i / NB) % count);
    const int r = (int)(i / ((int64_t)NB * count));
    const PlanIn P = in[r];
    const JumpTables *T = Trep[r];
    const u128 s0{P.s_lo, P.s_hi};
    const uint64_t per = 4 * V;
    const u128 base = jump(T, s0, (uint32_t)(k * per + block_off(b, V) + 1));
    Block B;
    B.base_lo = base.lo;
    B.base_hi = base.hi;
    B.nskip = 0;
    B.skip0 = 0;
    const bool bounded = b != 0 && b != 1 && b != 6;
    if (!bounded) {
        B.has = 0;
        B.buf = 0;
    } else {
        B.has = P.has;
        if (k == 0 && b == 2) {
            B.buf = P.buf;
        } else {
            // high half of the last u64 of the previous choice block
            const int kp = b == 2 ? k - 1 : k;
            const int pb = b == 2 ? 10 : (b == 7 ? 5 : b - 1);
            const uint64_t last = kp * per + block_off(pb, V) + V / 4;  // steps to the state of that u64
            B.buf = (uint32_t)(xsl_rr(jump(T, s0, (uint32_t)last)) >> 32);
        }
    }
    out[i] = B;
}

}  // namespace sv

using namespace svh;

struct sv_replicas {
    sv_ctx *ctx = nullptr;
    int32_t R = 0, N = 0;
    int64_t V = 0;
    double *phi[2] = {nullptr, nullptr};
    int64_t *n[2] = {nullptr, nullptr};
    int cur = 0;
    std::map<std::pair<uint64_t, uint64_t>, JumpTables *> tables;  // device, per increment
    const JumpTables **d_Trep = nullptr;
    Affine *d_adv = nullptr;
    PlanIn *d_plan = nullptr;
    Block *d_blocks = nullptr;
    sv_stats *d_stats = nullptr;
    unsigned long long *d_obs = nullptr;  // per (replica, sweep): the OBS_WORDS exact observable words (common.h)
    std::vector<std::pair<uint64_t, uint64_t>> incs;  // current per-replica increments
    // pinned batch tail: abort flag, report count, then the batch's statistics and observables (one DMA each,
    // one synchronization)
    char *h_tail = nullptr;
    size_t tail_cap = 0;
    int32_t *d_map = nullptr;  // replica maps of the split launches of a batch (R * REP_BATCH slots)
    int32_t *d_gate = nullptr;  // the batch's first sweep with a report (DevScratch::gate)
    // Host-to-device uploads of a batch (cursors, host-planned descriptors, skips, replica maps) go through pinned
    // staging: an asynchronous copy from pageable memory waits for the stream, which would drain the GPU at every
    // batch boundary behind the batch before
    struct Stage {
        char *h[2] = {nullptr, nullptr};
        size_t cap[2] = {0, 0}, used = 0;
        int i = 0;
        hipEvent_t ev[2] = {nullptr, nullptr};
        void begin() {
            i ^= 1;
            used = 0;
            if (ev[i]) SV_HIP(hipEventSynchronize(ev[i]));  // (the slot's copies of two batches ago)
        }
        void put(hipStream_t s, void *dst, const void *src, size_t bytes) {
            if (!bytes) return;
            if (used + bytes > cap[i]) {
                SV_HIP(hipStreamSynchronize(s));  // (this slot's earlier copies have landed)
                if (h[i]) SV_HIP(hipHostFree(h[i]));
                cap[i] = std::max<size_t>(std::max<size_t>(2 * cap[i], bytes), 256 * 1024);
                SV_HIP(hipHostMalloc((void **)&h[i], cap[i], hipHostMallocDefault));
                used = 0;
            }
            std::memcpy(h[i] + used, src, bytes);
            SV_HIP(hipMemcpyAsync(dst, h[i] + used, bytes, hipMemcpyHostToDevice, s));
            used += (bytes + 255) & ~size_t(255);
        }
        void end(hipStream_t s) {
            if (!ev[i]) SV_HIP(hipEventCreateWithFlags(&ev[i], hipEventDisableTiming));
            SV_HIP(hipEventRecord(ev[i], s));
        }
        void release() {
            for (int k = 0; k < 2; k++) {
                if (h[k]) (void)hipHostFree(h[k]);
                if (ev[k]) (void)hipEventDestroy(ev[k]);
            }
        }
    } stage;
};

namespace {

const JumpTables *replica_tables(sv_replicas *b, u128 inc) {
    auto key = std::make_pair(inc.hi, inc.lo);
    auto it = b->tables.find(key);
    if (it != b->tables.end()) return it->second;
    JumpTables *h = new JumpTables(make_tables(inc));
    JumpTables *d = nullptr;
    SV_HIP(hipMalloc(&d, sizeof(JumpTables)));
    SV_HIP(hipMemcpy(d, h, sizeof(JumpTables), hipMemcpyHostToDevice));
    delete h;
    b->tables[key] = d;
    return d;
}

// (re)bind per-replica tables and row-advance maps when the increments change
void bind_increments(sv_replicas *b, const sv_rng *rngs) {
    std::vector<std::pair<uint64_t, uint64_t>> incs(b->R);
    for (int r = 0; r < b->R; r++) incs[r] = {rngs[r].inc_hi, rngs[r].inc_lo};
    if (incs == b->incs) return;
    std::vector<const JumpTables *> T(b->R);
    std::vector<Affine> adv(3 * (size_t)b->R);
    constexpr int NWv = 4;
    for (int r = 0; r < b->R; r++) {
        const u128 inc{incs[r].second, incs[r].first};
        T[r] = replica_tables(b, inc);
        adv[3 * r + 0] = host_power(inc, (uint64_t)NWv * b->N);
        adv[3 * r + 1] = host_power(inc, (uint64_t)NWv * b->N / 2);
        adv[3 * r + 2] = host_power(inc, (uint64_t)NWv * b->N / 4);
    }
    SV_HIP(hipMemcpy(b->d_Trep, T.data(), b->R * sizeof(JumpTables *), hipMemcpyHostToDevice));
    SV_HIP(hipMemcpy(b->d_adv, adv.data(), adv.size() * sizeof(Affine), hipMemcpyHostToDevice));
    b->incs = incs;
}

bool has_skips(const SkipMap &m, int first, int count) {
    auto it = m.lower_bound({first, -1});
    return it != m.end() && it->first.first < first + count;
}

// advance a no-skip replica's cursor by a whole number of sweeps (closed form, see the file header).  k PCG64
// steps map s to M^k s + inc (M^(k-1) + ... + 1): `unit` = the map of k steps with increment 1, (M^k, sum M^i), is
// shared by every replica, so each one costs two 128-bit products instead of its own power of its step map.
void advance_closed(Cursor &c, u128 inc, const Affine &unit) {
    c.s = add(mul(unit.A, c.s), mul(inc, unit.C));
    c.buf = (uint32_t)(xsl_rr(c.s) >> 32);
}

// One batch of sweeps in flight: what its enqueue planned and where its outcome lands.
struct RepBatch {
    int sw = 0, count = 0, cur0 = 0, slot = 0;
    std::vector<char> hosted;          // replicas planned on the host (known skips in the batch)
    std::vector<Cursor> end_host;      // their cursors after the whole batch
    std::vector<std::vector<Block>> hb;  // host-planned descriptors, alive until the batch's stream sync
    std::vector<uint32_t> hskip;
    std::vector<int32_t> hmap;
};

// The measured form of the inline observables (sv_replicas_run_measured): what VillainReplicas.run returns, written
// by the batch loop's copy-out (overlapped with the next batch) instead of by NumPy after the call
struct MeasOut {
    double *acceptance, *action, *energy, *w2;
    int64_t *tw;
    double kappa;
};

void run_replicas(sv_replicas *b, const VParams &P, int32_t sweeps, sv_rng *rngs, sv_stats *stats, double *obs,
                  const MeasOut *mo = nullptr) {
    sv_ctx *ctx = b->ctx;
    const bool inl = obs != nullptr || mo != nullptr;  // the inline observables are summed
    // sweep k of replica r: its 4 raw sums (action sum, w2 sum, n0 sum, n1 sum) into the caller's arrays -- as they are
    // (obs), or measured (mo: the operations of replicas.py's former NumPy post-processing, in its order)
    auto put_obs = [&](int r, int64_t k, const unsigned long long *words) {
        const size_t e = (size_t)r * sweeps + (size_t)k;
        double raw[4];
        obs_raw(words, raw);  // the exact words -> the 4 raw sums (common.h)
        if (obs) {
            std::memcpy(obs + e * 4, raw, 4 * sizeof(double));
            return;
        }
        const double Vd = (double)b->V;
        const double S = raw[0] * (mo->kappa / 2);
        mo->energy[e] = S / (Vd * mo->kappa);
        mo->action[e] = S / Vd;
        mo->w2[e] = raw[1] / Vd;
        mo->tw[2 * e] = (int64_t)raw[2];
        mo->tw[2 * e + 1] = (int64_t)raw[3];
    };
    const int R = b->R;
    const int64_t V = b->V;
    const int64_t counts[2] = {V / 2, V / 2};
    const auto specs = villain_specs(V, 2, counts, P.k > 1);
    if ((int)specs.size() != NB) throw std::logic_error("unexpected block count");
    bind_increments(b, rngs);
    std::vector<Cursor> cur(R);
    std::vector<u128> inc(R);
    for (int r = 0; r < R; r++) {
        cur[r] = Cursor{u128{rngs[r].state_lo, rngs[r].state_hi}, (uint32_t)rngs[r].has_uint32, rngs[r].uinteger};
        inc[r] = u128{rngs[r].inc_lo, rngs[r].inc_hi};
    }
    std::vector<SkipMap> skips(R);
    const int nsx = b->N <= RW ? 1 : (b->N + FW_MAX - 1) / FW_MAX;  // one full-row strip up to 128 columns
    // 64-row tiles, or 32 when that leaves the chip short of workgroups (measured: R=128, N=128)
    const int TH = getenv("SV_FUSED_TH") ? fused_th(b->N, nsx) : ((int64_t)R * nsx * ((b->N + 63) / 64) < 768 ? 32 : 64);
    const int nsy = (b->N + TH - 1) / TH;
    const int tiles = nsx * nsy;
    const bool fr_hot = hot_fr_ok(b->N) && nsx == 1 && hot_params_ok(P);
    // replicas whose |n| left villain_sweep_hot_fr's int16 image (|n| >= 2^14) in this call: from the failing sweep
    // on they run on the general fused kernel's int32 image, beside the others (the split launches below)
    std::vector<char> big(R, 0);
    // pinned batch tails, two slots: batch k+1 is enqueued before batch k's statistics are copied out
    const size_t slot_bytes = 64 + (size_t)R * REP_BATCH * (sizeof(sv_stats) + OBS_WORDS * sizeof(unsigned long long));
    if (b->tail_cap < 2 * slot_bytes) {
        SV_HIP(hipStreamSynchronize(ctx->stream));
        if (b->h_tail) SV_HIP(hipHostFree(b->h_tail));
        b->h_tail = nullptr;
        b->tail_cap = 0;
        SV_HIP(hipHostMalloc((void **)&b->h_tail, 2 * slot_bytes, hipHostMallocDefault));
        b->tail_cap = 2 * slot_bytes;
    }
    if (!b->d_map) SV_HIP(hipMalloc(&b->d_map, (size_t)R * REP_BATCH * sizeof(int32_t)));
    const bool dbg = getenv("SV_DEBUG_TIMING") != nullptr;
    using clk = std::chrono::steady_clock;
    auto us = [](clk::time_point a, clk::time_point b) { return std::chrono::duration<double, std::micro>(b - a).count(); };
    std::vector<PlanIn> pin(R);
    std::vector<uint32_t> sk;

    // --- enqueue the batch [sw, sw + count) from the cursors `cur`: plan (device closed form for every replica,
    // host planner for replicas with known skips), the sweeps, and the tail copies into pinned slot `slot`
    auto enqueue = [&](RepBatch &B, int sw, int count, int slot) {
        B.sw = sw;
        B.count = count;
        B.slot = slot;
        B.cur0 = b->cur;
        for (int r = 0; r < R; r++) pin[r] = PlanIn{cur[r].s.lo, cur[r].s.hi, cur[r].has, cur[r].buf};
        b->stage.begin();
        b->stage.put(ctx->stream, b->d_plan, pin.data(), R * sizeof(PlanIn));
        const int64_t nplan = (int64_t)R * count * NB;
        plan_replicas<<<(unsigned)((nplan + 255) / 256), 256, 0, ctx->stream>>>(b->d_plan, b->d_Trep, b->d_blocks, R,
                                                                                  count, (uint64_t)V), SV_LAUNCHED("plan_replicas", ctx->stream);
        B.hskip.clear();
        B.hb.clear();
        B.hmap.clear();
        B.end_host.assign(R, Cursor{});
        B.hosted.assign(R, 0);
        for (int r = 0; r < R; r++) {
            if (!has_skips(skips[r], sw, count)) continue;
            B.hosted[r] = 1;
            Cursor c = cur[r];
            B.hb.emplace_back();
            std::vector<Block> &blk = B.hb.back();
            plan_sweeps(ctx, c, inc[r], specs, sw, count, skips[r], blk, sk);
            for (Block &x : blk) x.skip0 += (int32_t)B.hskip.size();
            B.hskip.insert(B.hskip.end(), sk.begin(), sk.end());
            B.end_host[r] = c;
            b->stage.put(ctx->stream, b->d_blocks + (size_t)r * count * NB, blk.data(), blk.size() * sizeof(Block));
        }
        ctx->ensure_skips(B.hskip.size() + 1);
        b->stage.put(ctx->stream, ctx->d_skips, B.hskip.data(), B.hskip.size() * sizeof(uint32_t));
        reset_batch(ctx, b->d_stats, (size_t)R * count * sizeof(sv_stats), inl ? b->d_obs : nullptr,
                    inl ? (size_t)R * count * OBS_WORDS * sizeof(unsigned long long) : 0);
        // A sweep runs on the fast-draw kernel (villain_sweep_hot_fr) when no replica's choice blocks of that sweep
        // carry a skip (the closed-form replicas have none; the host-planned ones are checked), else on the general
        // fused kernel.  Within a skip-free sweep a replica's four choice blocks start on the same half-word parity
        // (they draw V/2, an even count), which is all the fast kernel's two draw forms need.
        std::vector<char> hot_k(count, fr_hot);
        std::vector<std::vector<int32_t>> skipped(count);  // per sweep: replicas on the general kernel (ascending)
        if (fr_hot) {
            // only the replicas on the int32 image or with host-planned descriptors can leave the fast kernel: the scan
            // walks those (a scan of every replica and sweep, 65536 steps at config 5, cost ~0.1 ms of idle GPU per
            // batch boundary, r5 profiles/r05_rep_idle*.txt)
            std::vector<std::pair<int, const std::vector<Block> *>> special;
            size_t hi = 0;
            for (int r = 0; r < R; r++) {
                const std::vector<Block> *h = B.hosted[r] ? &B.hb[hi++] : nullptr;
                if (big[r] || h) special.push_back({r, h});
            }
            for (int k = 0; k < count; k++)
                for (const auto &sp : special) {
                    bool gen = big[sp.first] != 0;
                    if (sp.second)
                        for (int bi = 2; bi < NB; bi++) gen |= bi != 6 && (*sp.second)[(size_t)k * NB + bi].nskip != 0;
                    if (gen) {
                        hot_k[k] = 0;
                        skipped[k].push_back(sp.first);
                    }
                }
        }
        // a sweep with skips in a few replicas runs as two launches over replica maps: the fast kernel for the
        // others, the general kernel for those (so a NumPy Lemire rejection slows one replica's replay, not all)
        std::vector<std::array<int64_t, 4>> split(count, {0, 0, 0, 0});  // hot offset, hot count, general offset, count
        for (int k = 0; k < count; k++) {
            if (!fr_hot || hot_k[k]) continue;
            split[k][0] = (int64_t)B.hmap.size();
            size_t j = 0;
            for (int r = 0; r < R; r++) {
                if (j < skipped[k].size() && skipped[k][j] == r) {
                    j++;
                    continue;
                }
                B.hmap.push_back(r);
            }
            split[k][1] = (int64_t)B.hmap.size() - split[k][0];
            split[k][2] = (int64_t)B.hmap.size();
            B.hmap.insert(B.hmap.end(), skipped[k].begin(), skipped[k].end());
            split[k][3] = (int64_t)skipped[k].size();
        }
        b->stage.put(ctx->stream, b->d_map, B.hmap.data(), B.hmap.size() * sizeof(int32_t));
        b->stage.end(ctx->stream);
        // The batch goes out in chunks of CH sweeps: after chunk j is enqueued the host waits for chunk j - 1 (the
        // progress word the first launch of chunk j stores) and reads the host-mapped abort flag, so that a NumPy
        // Lemire rejection leaves at most ~2 CH launches queued behind it (each an early exit over every workgroup)
        // instead of the rest of the batch (r3: 220 early-exit launches, 1.1 ms, in a 200-sweep config-5 window)
        const char *ch_env = getenv("SV_REP_CHUNK");  // overrides the chunk (0: the whole batch)
        const int CH_set = ch_env ? atoi(ch_env) : 8;
        const int CH = CH_set > 0 ? CH_set : count;
        *ctx->h_flag = 0;
        __atomic_store_n(ctx->h_prog, 0, __ATOMIC_RELEASE);  // (the previous batch has finished)
        int64_t launches = 0;  // kernel launches enqueued (a split sweep makes two): the timing's per-launch average
        SV_HIP(hipMemsetAsync(b->d_gate, 0x7f, sizeof(int32_t), ctx->stream));  // no report yet (0x7f7f7f7f)
        hipEvent_t ev;
        ctx->time_begin(&ev);
        for (int k = 0; k < count; k++) {
            FArgs A;
            A.P = P;
            A.G = FGeom{b->N, b->N, 0, 0, b->N, b->N, b->N, V, 0};
            A.phi_in = b->phi[b->cur];
            A.n_in = b->n[b->cur];
            A.phi_out = b->phi[b->cur ^ 1];
            A.n_out = b->n[b->cur ^ 1];
            A.nsx = nsx;
            A.TH = TH;
            A.nsy = nsy;
            A.blocks = b->d_blocks + (size_t)k * NB;
            A.skips = ctx->d_skips;
            A.T = nullptr;
            A.stat = b->d_stats + k;
            A.S = DevScratch{ctx->d_abort, ctx->d_nreport, ctx->d_reports, ctx->d_flag, b->d_gate};
            A.progress = ctx->d_prog;
            A.sweep = (uint32_t)k;
            A.tiles_per_rep = tiles;
            A.rep_blocks = count * NB;
            A.rep_field = V;
            A.rep_stat = count;
            A.rep_obs = OBS_WORDS * count;
            A.Trep = b->d_Trep;
            A.advrep = b->d_adv;
            A.obs = inl ? b->d_obs + OBS_WORDS * k : nullptr;
            if (hot_k[k]) {
                launch_hot_fr(A, R * tiles, inl, ctx->stream);
                ctx->sweeps_hot++;
                launches++;
            } else if (split[k][3] > 0) {
                FArgs Ah = A, Ag = A;
                Ah.rep_map = b->d_map + split[k][0];
                Ag.rep_map = b->d_map + split[k][2];
                // the few replaying replicas: 8-row strips, so that their launch is not one long strip per
                // workgroup serialized behind the fast launch
                Ag.TH = 8;
                Ag.nsy = (b->N + 7) / 8;
                Ag.tiles_per_rep = nsx * Ag.nsy;
                if (split[k][1] > 0) launch_hot_fr(Ah, (int)split[k][1] * tiles, inl, ctx->stream);
                launch_fused_batch(Ag, (int)split[k][3] * Ag.tiles_per_rep, inl, ctx->stream);
                ctx->sweeps_hot += split[k][1] > 0;
                ctx->sweeps_fused++;
                launches += 1 + (split[k][1] > 0);
            } else {
                launch_fused_batch(A, R * tiles, inl, ctx->stream);
                ctx->sweeps_fused++;
                launches++;
            }
            b->cur ^= 1;
            if ((k + 1) % CH == 0 && k + 1 < count && k + 1 >= 2 * CH) {
                // chunk j = (k + 1) / CH - 1 is enqueued: wait until chunk j - 1 has finished (the first launch of
                // chunk j has started), or a rejection was reported, or (guard) the stream has drained
                const int32_t target = (int32_t)(k + 1 - CH) + 1;
                const auto tw = clk::now();
                for (int spin = 0; __atomic_load_n(ctx->h_prog, __ATOMIC_ACQUIRE) < target; spin++) {
                    if (__atomic_load_n(ctx->h_flag, __ATOMIC_ACQUIRE)) break;
                    if ((spin & 1023) == 1023 && clk::now() - tw > std::chrono::milliseconds(20) &&
                        hipStreamQuery(ctx->stream) == hipSuccess)
                        break;  // (drained: e.g. a sweep with no launch that stores its progress)
                    std::this_thread::yield();
                }
                if (__atomic_load_n(ctx->h_flag, __ATOMIC_ACQUIRE)) break;  // the rest of the batch is not enqueued
            }
        }
        ctx->time_end(ev, launches);
        SV_HIP(hipGetLastError());
        // outcome: abort flag, report count, statistics and observables land in the pinned slot
        char *tail = b->h_tail + slot * slot_bytes;
        const size_t st_bytes = (size_t)R * count * sizeof(sv_stats);
        SV_HIP(hipMemcpyAsync(tail, ctx->d_abort, 2 * sizeof(int32_t), hipMemcpyDeviceToHost, ctx->stream));  // + d_nreport
        finalize_stats(b->d_stats, (int64_t)R * count, ctx->stream);
        SV_HIP(hipMemcpyAsync(tail + 64, b->d_stats, st_bytes, hipMemcpyDeviceToHost, ctx->stream));
        if (inl)
            SV_HIP(hipMemcpyAsync(tail + 64 + st_bytes, b->d_obs, (size_t)R * count * OBS_WORDS * sizeof(unsigned long long),
                                  hipMemcpyDeviceToHost, ctx->stream));
    };
    // --- keep sweeps [B.sw, B.sw + good) of a finished batch: statistics and observables into the caller's arrays
    // (fail: after an abort at sweep `good`, the replicas that did not report in it keep that sweep too)
    auto keep = [&](const RepBatch &B, int good, const std::vector<char> *fail = nullptr) {
        const char *tail = b->h_tail + B.slot * slot_bytes;
        const sv_stats *h_st = (const sv_stats *)(tail + 64);
        const unsigned long long *h_ob = (const unsigned long long *)(tail + 64 + (size_t)R * B.count * sizeof(sv_stats));
        for (int r = 0; r < R; r++) {
            const bool none = skips[r].empty();
            sv_stats *dst = stats + (size_t)r * sweeps + B.sw;
            const sv_stats *src = h_st + (size_t)r * B.count;
            const int upto = good + (fail && !(*fail)[r] && good < B.count ? 1 : 0);
            for (int k = 0; k < upto; k++) {
                dst[k] = src[k];
                dst[k].proposed = V;
                dst[k].rejections = none ? 0 : rejections_in(skips[r], B.sw + k, NB);
                if (mo) mo->acceptance[(size_t)r * sweeps + B.sw + k] = src[k].acceptance_sum / (double)V;
            }
            if (inl)
                for (int k = 0; k < upto; k++) put_obs(r, B.sw + k, h_ob + ((size_t)r * B.count + k) * OBS_WORDS);
        }
    };

    // Sweep k of batch B again for the replicas F that reported in it (their cursors in `cur` are at sweep k), on the
    // general kernel with the absorbed skip lists, until it completes without a new report; their statistics and
    // observables of that sweep go straight to the caller's arrays and their cursors move past it
    auto replay_failed = [&](const RepBatch &B, int k, const std::vector<int32_t> &F) {
        if (F.empty()) return;
        const int count = B.count;
        for (int attempt = 0;; attempt++) {
            if (attempt > 64) throw std::runtime_error("rejection replay did not converge");
            std::vector<Cursor> cf(F.size());
            std::vector<Block> fb((size_t)F.size() * NB);
            std::vector<uint32_t> allsk;
            for (size_t i = 0; i < F.size(); i++) {
                const int r = F[i];
                Cursor c = cur[r];
                std::vector<Block> blk;
                plan_sweeps(ctx, c, inc[r], specs, B.sw + k, 1, skips[r], blk, sk);
                for (int j = 0; j < NB; j++) {
                    fb[i * NB + j] = blk[j];
                    fb[i * NB + j].skip0 += (int32_t)allsk.size();
                }
                allsk.insert(allsk.end(), sk.begin(), sk.end());
                cf[i] = c;
            }
            ctx->ensure_skips(allsk.size() + 1);
            b->stage.begin();
            for (size_t i = 0; i < F.size(); i++) {
                const size_t e = (size_t)F[i] * count + k;
                b->stage.put(ctx->stream, b->d_blocks + e * NB, &fb[i * NB], NB * sizeof(Block));
                SV_HIP(hipMemsetAsync(b->d_stats + e, 0, sizeof(sv_stats), ctx->stream));
                if (inl) SV_HIP(hipMemsetAsync(b->d_obs + OBS_WORDS * e, 0, OBS_WORDS * sizeof(unsigned long long), ctx->stream));
            }
            b->stage.put(ctx->stream, ctx->d_skips, allsk.data(), allsk.size() * sizeof(uint32_t));
            b->stage.put(ctx->stream, b->d_map, F.data(), F.size() * sizeof(int32_t));
            b->stage.end(ctx->stream);
            clear_abort(ctx);
            SV_HIP(hipMemsetAsync(b->d_gate, 0x7f, sizeof(int32_t), ctx->stream));
            FArgs A;
            A.P = P;
            A.G = FGeom{b->N, b->N, 0, 0, b->N, b->N, b->N, V, 0};
            A.phi_in = b->phi[B.cur0 ^ (k & 1)];
            A.n_in = b->n[B.cur0 ^ (k & 1)];
            A.phi_out = b->phi[B.cur0 ^ (k & 1) ^ 1];
            A.n_out = b->n[B.cur0 ^ (k & 1) ^ 1];
            A.nsx = nsx;
            A.TH = 8;  // short strips: the few replaying replicas fill more of the chip
            A.nsy = (b->N + 7) / 8;
            A.blocks = b->d_blocks + (size_t)k * NB;
            A.skips = ctx->d_skips;
            A.T = nullptr;
            A.stat = b->d_stats + k;
            A.S = DevScratch{ctx->d_abort, ctx->d_nreport, ctx->d_reports, nullptr, b->d_gate};
            A.sweep = (uint32_t)k;
            A.tiles_per_rep = nsx * A.nsy;
            A.rep_blocks = count * NB;
            A.rep_field = V;
            A.rep_stat = count;
            A.rep_obs = OBS_WORDS * count;
            A.Trep = b->d_Trep;
            A.advrep = b->d_adv;
            A.obs = inl ? b->d_obs + OBS_WORDS * k : nullptr;
            A.rep_map = b->d_map;
            launch_fused_batch(A, (int)F.size() * A.tiles_per_rep, inl, ctx->stream);
            ctx->sweeps_fused++;
            SV_HIP(hipGetLastError());
            AbortInfo a = read_abort(ctx);  // (synchronizes)
            if (!a.abort) {
                for (size_t i = 0; i < F.size(); i++) {
                    const int r = F[i];
                    const size_t e = (size_t)r * count + k;
                    sv_stats *dst = stats + (size_t)r * sweeps + B.sw + k;
                    finalize_stats(b->d_stats + e, 1, ctx->stream);
                    SV_HIP(hipMemcpyAsync(dst, b->d_stats + e, sizeof(sv_stats), hipMemcpyDeviceToHost, ctx->stream));
                    SV_HIP(hipStreamSynchronize(ctx->stream));
                    dst->proposed = V;
                    dst->rejections = rejections_in(skips[r], B.sw + k, NB);
                    if (mo) mo->acceptance[(size_t)r * sweeps + B.sw + k] = dst->acceptance_sum / (double)V;
                    if (inl) {
                        unsigned long long words[OBS_WORDS];
                        SV_HIP(hipMemcpy(words, b->d_obs + OBS_WORDS * e, sizeof words, hipMemcpyDeviceToHost));
                        put_obs(r, B.sw + k, words);
                    }
                    cur[r] = cf[i];
                }
                return;
            }
            for (const Report &x : a.reports)
                if (x.block == OVERFLOW_BLOCK)
                    throw std::runtime_error("|n| exceeds the general fused kernel's int32 LDS image (|n| < 2^30 required)");
            for (int r : F) {
                AbortInfo ar{1, {}};
                for (const Report &x : a.reports)
                    if ((int)x.pad == r) ar.reports.push_back(x);
                if (!ar.reports.empty()) absorb_reports(ar, B.sw, skips[r]);
            }
        }
    };

    RepBatch batch[2];
    int cb = 0;  // batch[cb] is in flight
    int sw = 0;
    if (sweeps > 0) enqueue(batch[cb], 0, std::min(REP_BATCH, sweeps), 0);
    while (sw < sweeps) {
        RepBatch &B = batch[cb];
        const auto t_a = clk::now();
        SV_HIP(hipStreamSynchronize(ctx->stream));
        const auto t_b = clk::now();
        const char *tail = b->h_tail + B.slot * slot_bytes;
        const int32_t ab = *(const int32_t *)tail;
        if (ab) {
            // a NumPy Lemire rejection (or |n| overflow): keep the sweeps before the failing one, absorb the
            // rejected positions into the failing replicas' skip lists, replay from there
            ctx->time_discard();
            uint32_t nrep = std::min<uint32_t>(*(const uint32_t *)(tail + 4), MAX_REPORTS);
            std::vector<Report> reps(nrep);
            if (nrep) SV_HIP(hipMemcpy(reps.data(), ctx->d_reports, nrep * sizeof(Report), hipMemcpyDeviceToHost));
            if (reps.empty()) throw std::runtime_error("device aborted without a rejection report");
            uint32_t bad = ~0u;
            for (const Report &x : reps) bad = std::min(bad, x.sweep);
            for (const Report &x : reps)
                if (x.block == OVERFLOW_BLOCK && x.sweep == bad) {
                    // int16 image of the fast kernel: replay this replica on the general kernel's int32 image
                    if (!fr_hot || big[x.pad]) throw std::runtime_error("|n| exceeds the general fused kernel's int32 LDS image (|n| < 2^30 required)");
                    big[x.pad] = 1;
                }
            for (int r = 0; r < R; r++) {
                AbortInfo a{1, {}};
                for (const Report &x : reps)
                    if ((int)x.pad == r && x.sweep == bad && x.block != OVERFLOW_BLOCK) a.reports.push_back(x);
                if (!a.reports.empty()) absorb_reports(a, B.sw, skips[r]);
            }
            const int good = (int)bad;
            // the gate (DevScratch::gate) let the failing sweep complete: only the replicas that reported in it
            // replay it; every other replica keeps its result
            std::vector<char> fail(R, 0);
            for (const Report &x : reps)
                if (x.sweep == bad) fail[x.pad] = 1;
            const Affine unit = good > 0 ? host_power(u128{1, 0}, (uint64_t)good * 4 * V) : Affine{};
            for (int r = 0; r < R; r++) {
                if (has_skips(skips[r], B.sw, good)) {
                    Cursor c = cur[r];
                    std::vector<Block> blk;
                    plan_sweeps(ctx, c, inc[r], specs, B.sw, good, skips[r], blk, sk);
                    cur[r] = c;
                } else if (good > 0) {
                    advance_closed(cur[r], inc[r], unit);
                }
            }
            const Affine unit1 = host_power(u128{1, 0}, (uint64_t)4 * V);
            std::vector<int32_t> F;
            for (int r = 0; r < R; r++) {
                if (fail[r]) {
                    F.push_back(r);
                } else if (has_skips(skips[r], B.sw + good, 1)) {
                    Cursor c = cur[r];
                    std::vector<Block> blk;
                    plan_sweeps(ctx, c, inc[r], specs, B.sw + good, 1, skips[r], blk, sk);
                    cur[r] = c;
                } else {
                    advance_closed(cur[r], inc[r], unit1);
                }
            }
            const auto t_c = clk::now();
            replay_failed(B, good, F);
            b->cur = B.cur0 ^ ((good + 1) & 1);
            sw = B.sw + good + 1;
            const auto t_d = clk::now();
            // the next batch goes out first (into the other slot), the kept sweeps are copied out while it runs
            if (sw < sweeps) enqueue(batch[cb ^ 1], sw, std::min(REP_BATCH, sweeps - sw), B.slot ^ 1);
            keep(B, good, &fail);
            if (dbg)
                fprintf(stderr, "[sv replicas] wait %.1f us, abort at %d/%d (%zu replicas replay it), replan %.1f us, "
                        "replay %.1f us, enqueue + keep %.1f us\n", us(t_a, t_b), good, B.count, F.size(),
                        us(t_b, t_c), us(t_c, t_d), us(t_d, clk::now()));
            cb ^= 1;
            continue;
        }
        ctx->time_collect();
        // clean batch: advance the cursors past it, enqueue the next batch, and copy this one's statistics out
        // while the next one runs
        const Affine unit = host_power(u128{1, 0}, (uint64_t)B.count * 4 * V);
        for (int r = 0; r < R; r++) {
            if (B.hosted[r])
                cur[r] = B.end_host[r];
            else
                advance_closed(cur[r], inc[r], unit);
        }
        sw = B.sw + B.count;
        const auto t_c = clk::now();
        if (sw < sweeps) enqueue(batch[cb ^ 1], sw, std::min(REP_BATCH, sweeps - sw), B.slot ^ 1);
        const auto t_d = clk::now();
        keep(B, B.count);
        if (dbg)
            fprintf(stderr, "[sv replicas] wait %.1f us, advance %.1f us, enqueue next %.1f us, keep %.1f us, %d sweeps\n",
                    us(t_a, t_b), us(t_b, t_c), us(t_c, t_d), us(t_d, clk::now()), B.count);
        cb ^= 1;
    }
    for (int r = 0; r < R; r++) {
        rngs[r].state_hi = cur[r].s.hi;
        rngs[r].state_lo = cur[r].s.lo;
        rngs[r].has_uint32 = (int32_t)cur[r].has;
        rngs[r].uinteger = cur[r].buf;
    }
}


int replicas_run(sv_replicas *b, double kappa, int64_t W, double interval_phi, int64_t interval_n,
                            int32_t sweeps, sv_rng *rngs, sv_stats *stats, double *obs, const MeasOut *mo) {
    if (!b || !rngs || (sweeps > 0 && !stats)) return -1;
    sv_ctx *ctx = b->ctx;
    try {
        if (sweeps < 0) throw std::invalid_argument("sweeps must be >= 0");
        if (interval_n < 0 || interval_n > (1 << 20)) throw std::invalid_argument("interval_n out of range");
        if ((W < 0 ? -W : W) * interval_n >= (1LL << 28)) throw std::invalid_argument("|W * interval_n| too large");
        SV_HIP(hipSetDevice(ctx->device));
        const VParams P = make_params(b->N, kappa, W, interval_phi, interval_n);
        run_replicas(b, P, sweeps, rngs, stats, obs, mo);
        return 0;
    } catch (const std::exception &e) {
        ctx->err = e.what();
        return -2;
    }
}

}  // namespace

extern "C" {

int sv_replicas_create(sv_ctx *ctx, int32_t R, int32_t N, sv_replicas **out) {
    if (!ctx || !out) return -1;
    *out = nullptr;
    sv_replicas *b = new sv_replicas();
    try {
        if (R < 1) throw std::invalid_argument("need at least one replica");
        if (N < 4 || N % 2) throw std::invalid_argument("replica batches need an even N >= 4");
        if ((int64_t)REP_BATCH * 4 * (int64_t)N * N >= (1LL << 32))
            throw std::invalid_argument("N too large for replica batches (use sv_villain_* per lattice)");
        SV_HIP(hipSetDevice(ctx->device));
        b->ctx = ctx;
        b->R = R;
        b->N = N;
        b->V = (int64_t)N * N;
        const size_t V = (size_t)b->V;
        for (int i = 0; i < 2; i++) {
            SV_HIP(hipMalloc(&b->phi[i], R * V * sizeof(double)));
            SV_HIP(hipMalloc(&b->n[i], 2 * R * V * sizeof(int64_t)));
        }
        SV_HIP(hipMalloc(&b->d_Trep, R * sizeof(JumpTables *)));
        SV_HIP(hipMalloc(&b->d_adv, 3 * R * sizeof(Affine)));
        SV_HIP(hipMalloc(&b->d_plan, R * sizeof(PlanIn)));
        SV_HIP(hipMalloc(&b->d_blocks, (size_t)R * REP_BATCH * NB * sizeof(Block)));
        SV_HIP(hipMalloc(&b->d_stats, (size_t)R * REP_BATCH * sizeof(sv_stats)));
        SV_HIP(hipMalloc(&b->d_obs, (size_t)R * REP_BATCH * OBS_WORDS * sizeof(unsigned long long)));
        SV_HIP(hipMalloc(&b->d_gate, sizeof(int32_t)));
        *out = b;
        return 0;
    } catch (const std::exception &e) {
        ctx->err = e.what();
        sv_replicas_destroy(b);
        return -2;
    }
}

int sv_replicas_destroy(sv_replicas *b) {
    if (!b) return 0;
    const int rc = sv_destroy_drain(b->ctx, "sv_replicas_destroy");
    for (int i = 0; i < 2; i++) {
        (void)hipFree(b->phi[i]);
        (void)hipFree(b->n[i]);
    }
    for (auto &kv : b->tables) (void)hipFree(kv.second);
    (void)hipFree(b->d_Trep);
    (void)hipFree(b->d_adv);
    (void)hipFree(b->d_plan);
    (void)hipFree(b->d_gate);
    (void)hipFree(b->d_blocks);
    (void)hipFree(b->d_stats);
    (void)hipFree(b->d_obs);
    if (b->h_tail) (void)hipHostFree(b->h_tail);
    if (b->d_map) (void)hipFree(b->d_map);
    b->stage.release();
    delete b;
    return rc;
}

int sv_replicas_upload(sv_replicas *b, const double *phi, const int64_t *n) {
    if (!b) return -1;
    sv_ctx *ctx = b->ctx;
    try {
        SV_HIP(hipSetDevice(ctx->device));
        const size_t V = (size_t)b->V, R = (size_t)b->R;
        if (!phi || !n) {
            SV_HIP(hipMemsetAsync(b->phi[b->cur], 0, R * V * sizeof(double), ctx->stream));
            SV_HIP(hipMemsetAsync(b->n[b->cur], 0, 2 * R * V * sizeof(int64_t), ctx->stream));
        } else {
            SV_HIP(hipMemcpyAsync(b->phi[b->cur], phi, R * V * sizeof(double), hipMemcpyHostToDevice, ctx->stream));
            SV_HIP(hipMemcpyAsync(b->n[b->cur], n, 2 * R * V * sizeof(int64_t), hipMemcpyHostToDevice, ctx->stream));
        }
        SV_HIP(hipStreamSynchronize(ctx->stream));
        return 0;
    } catch (const std::exception &e) {
        ctx->err = e.what();
        return -2;
    }
}

int sv_replicas_download(sv_replicas *b, double *phi, int64_t *n) {
    if (!b || !phi || !n) return -1;
    sv_ctx *ctx = b->ctx;
    try {
        SV_HIP(hipSetDevice(ctx->device));
        const size_t V = (size_t)b->V, R = (size_t)b->R;
        SV_HIP(hipMemcpyAsync(phi, b->phi[b->cur], R * V * sizeof(double), hipMemcpyDeviceToHost, ctx->stream));
        SV_HIP(hipMemcpyAsync(n, b->n[b->cur], 2 * R * V * sizeof(int64_t), hipMemcpyDeviceToHost, ctx->stream));
        SV_HIP(hipStreamSynchronize(ctx->stream));
        return 0;
    } catch (const std::exception &e) {
        ctx->err = e.what();
        return -2;
    }
}

int sv_replicas_run(sv_replicas *b, double kappa, int64_t W, double interval_phi, int64_t interval_n, int32_t sweeps,
                    sv_rng *rngs, sv_stats *stats, double *obs) {
    return replicas_run(b, kappa, W, interval_phi, interval_n, sweeps, rngs, stats, obs, nullptr);
}

int sv_replicas_run_measured(sv_replicas *b, double kappa, int64_t W, double interval_phi, int64_t interval_n,
                             int32_t sweeps, sv_rng *rngs, sv_stats *stats, double *acceptance, double *action_density,
                             double *energy_density, double *winding_squared, int64_t *torus_wrapping) {
    if (sweeps > 0 && (!acceptance || !action_density || !energy_density || !winding_squared || !torus_wrapping)) return -1;
    const MeasOut mo{acceptance, action_density, energy_density, winding_squared, torus_wrapping, kappa};
    return replicas_run(b, kappa, W, interval_phi, interval_n, sweeps, rngs, stats, nullptr, &mo);
}

int sv_replicas_worm_run(sv_replicas *b, double kappa, int64_t W, int32_t worms, int64_t max_moves, sv_rng *rngs,
                         int64_t *hist, int64_t *lengths) {
    if (!b || !rngs) return -1;
    sv_ctx *ctx = b->ctx;
    try {
        SV_HIP(hipSetDevice(ctx->device));
        villain_worms_device(ctx, b->R, b->N, b->phi[b->cur], b->n[b->cur], kappa, W, worms, max_moves, rngs, hist,
                             lengths);
        return 0;
    } catch (const std::exception &e) {
        ctx->err = e.what();
        return -2;
    }
}

// One-shot form over host arrays (SURVEY.md 8(b)'s sv_replicas_villain): create, upload, run, download.
int sv_replicas_villain(sv_ctx *ctx, int32_t R, int32_t N, double kappa, int64_t W, double interval_phi,
                        int64_t interval_n, double *phi, int64_t *n, int32_t sweeps, sv_rng *rngs, sv_stats *stats,
                        double *inline_out) {
    if (!ctx || !phi || !n || !rngs) return -1;
    sv_replicas *b = nullptr;
    int rc = sv_replicas_create(ctx, R, N, &b);
    if (!rc) rc = sv_replicas_upload(b, phi, n);
    if (!rc) rc = sv_replicas_run(b, kappa, W, interval_phi, interval_n, sweeps, rngs, stats, inline_out);
    if (!rc) rc = sv_replicas_download(b, phi, n);
    if (b) sv_replicas_destroy(b);
    return rc;
}

}  // extern "C"
