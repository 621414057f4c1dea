// capi.hip -- context management of libsvhip.so (see include/supervillain_amd.h).
#include <cstring>

#include "common.h"

static bool alloc_log() { return getenv("SV_ALLOC_LOG") != nullptr; }  // (read per call: tests set it in-process)

hipError_t sv_log_malloc(void **p, size_t bytes, const char *site) {
    const hipError_t e = (hipMalloc)(p, bytes);
    if (alloc_log()) fprintf(stderr, "[sv alloc] malloc %p +%zu %s rc=%d\n", *p, bytes, site, (int)e);
    return e;
}

hipError_t sv_log_free(void *p, const char *site) {
    if (alloc_log() && p) fprintf(stderr, "[sv alloc] free %p %s\n", p, site);
    return (hipFree)(p);
}

hipError_t sv_log_host_malloc(void **p, size_t bytes, unsigned flags, const char *site) {
    const hipError_t e = (hipHostMalloc)(p, bytes, flags);
    if (alloc_log()) fprintf(stderr, "[sv alloc] hostmalloc %p +%zu %s rc=%d\n", *p, bytes, site, (int)e);
    return e;
}

hipError_t sv_log_host_free(void *p, const char *site) {
    if (alloc_log() && p) fprintf(stderr, "[sv alloc] hostfree %p %s\n", p, site);
    return (hipHostFree)(p);
}

const sv::JumpTables *sv_ctx::jump_tables(uint64_t inc_hi, uint64_t inc_lo) {
    auto key = std::make_pair(inc_hi, inc_lo);
    auto it = tables.find(key);
    if (it != tables.end()) return it->second;

    if (tables.size() >= (table_cap ? table_cap : MAX_TABLES)) {
        if (alloc_log()) fprintf(stderr, "[sv alloc] jump-table cache purge #%lld (%zu tables)\n", (long long)table_purges + 1,
                                 tables.size());
        // a long-lived context seeing many generators drops its cache.  Launches already enqueued on ANY stream of
        // the device (the context stream, deferred pipeline members, a domain's scan stream, emission copies) may
        // hold one of these tables, so the whole device drains first -- explicitly, not through hipFree's own
        // implicit synchronization -- and a failure there is reported, not swallowed.  No caller keeps a table
        // pointer across calls: every entry point fetches its table on entry.
        // (the drain covers every stream of the device: an error it meets may come from work this context did not
        // enqueue, and is reported as such)
        const hipError_t de = hipDeviceSynchronize();
        if (de != hipSuccess)
            throw std::runtime_error(std::string("jump-table purge: draining the device (every stream, this context's and "
                                                 "any other's) failed: ") + hipGetErrorString(de));
        for (auto &kv : tables) SV_HIP(hipFree(kv.second));
        tables.clear();
        table_purges++;
    }
    sv::JumpTables *h = new sv::JumpTables(sv::make_tables(sv::u128{inc_lo, inc_hi}));
    sv::JumpTables *d = nullptr;
    try {
        SV_HIP(hipMalloc(&d, sizeof(sv::JumpTables)));
        SV_HIP(hipMemcpy(d, h, sizeof(sv::JumpTables), hipMemcpyHostToDevice));
    } catch (...) {
        delete h;
        throw;
    }
    delete h;
    tables[key] = d;
    return d;
}

void sv_ctx::ensure_blocks(size_t n) {
    if (n <= blocks_cap) return;
    SV_HIP(hipStreamSynchronize(stream));
    if (d_blocks) SV_HIP(hipFree(d_blocks));
    blocks_cap = std::max(n, 2 * blocks_cap);
    SV_HIP(hipMalloc(&d_blocks, blocks_cap * sizeof(sv::Block)));
}

void sv_ctx::upload_plan(const sv::Block *blocks, size_t nblocks, const uint32_t *skips, size_t nskips, size_t offset) {
    if (offset && offset + nblocks > blocks_cap) throw std::logic_error("upload_plan: a second part beyond the capacity");
    ensure_blocks(offset + nblocks);
    ensure_skips(nskips + 1);
    const size_t bb = nblocks * sizeof(sv::Block), sb = nskips * sizeof(uint32_t);
    const int i = h_plan_i;
    h_plan_i ^= 1;
    if (!ev_plan[i]) SV_HIP(hipEventCreateWithFlags(&ev_plan[i], hipEventDisableTiming));
    else SV_HIP(hipEventSynchronize(ev_plan[i]));  // (its last copies have long run, unless runs are deferred)
    if (bb + sb > h_plan_cap[i]) {
        SV_HIP(hipStreamSynchronize(stream));  // (the buffer may still feed an earlier copy)
        if (h_plan[i]) SV_HIP(hipHostFree(h_plan[i]));
        h_plan_cap[i] = std::max<size_t>(2 * (bb + sb), 64 * 1024);
        SV_HIP(hipHostMalloc((void **)&h_plan[i], h_plan_cap[i], hipHostMallocDefault));
    }
    std::memcpy(h_plan[i], blocks, bb);
    if (sb) std::memcpy(h_plan[i] + bb, skips, sb);
    SV_HIP(hipMemcpyAsync(d_blocks + offset, h_plan[i], bb, hipMemcpyHostToDevice, stream));
    if (sb) SV_HIP(hipMemcpyAsync(d_skips, h_plan[i] + bb, sb, hipMemcpyHostToDevice, stream));
    SV_HIP(hipEventRecord(ev_plan[i], stream));
}

void sv_ctx::ensure_skips(size_t n) {
    if (n <= skips_cap) return;
    SV_HIP(hipStreamSynchronize(stream));
    if (d_skips) SV_HIP(hipFree(d_skips));
    skips_cap = std::max<size_t>(std::max(n, 2 * skips_cap), 64);
    SV_HIP(hipMalloc(&d_skips, skips_cap * sizeof(uint32_t)));
}

void sv_ctx::ensure_stats(size_t n) {
    if (n <= stats_cap) return;
    SV_HIP(hipStreamSynchronize(stream));
    if (d_stats) SV_HIP(hipFree(d_stats));
    stats_cap = std::max(n, 2 * stats_cap);
    SV_HIP(hipMalloc(&d_stats, stats_cap * sizeof(sv_stats)));
}

bool sv_ctx::defer_stats(sv_stats *dst, int64_t count) {
    if (!deferred) return false;
    if (stage_used + (size_t)count > stage_cap || abort_used + 1 > abort_cap) {
        SV_HIP(hipStreamSynchronize(stream));
        land();
        if (h_stage) SV_HIP(hipHostFree(h_stage));
        if (h_stage_abort) SV_HIP(hipHostFree(h_stage_abort));
        stage_cap = std::max<size_t>(std::max<size_t>(2 * stage_cap, (size_t)count), 1024);
        abort_cap = std::max<size_t>(2 * abort_cap, 256);
        SV_HIP(hipHostMalloc((void **)&h_stage, stage_cap * sizeof(sv_stats), hipHostMallocDefault));
        SV_HIP(hipHostMalloc((void **)&h_stage_abort, abort_cap * sizeof(int32_t), hipHostMallocDefault));
    }
    svh::finalize_stats(d_stats, count, stream);
    SV_HIP(hipMemcpyAsync(h_stage + stage_used, d_stats, count * sizeof(sv_stats), hipMemcpyDeviceToHost, stream));
    SV_HIP(hipMemcpyAsync(h_stage_abort + abort_used, d_abort, sizeof(int32_t), hipMemcpyDeviceToHost, stream));
    landings.push_back(Landing{dst, stage_used, count, abort_used});
    stage_used += count;
    abort_used += 1;
    return true;
}

void sv_ctx::land() {
    bool bad = false;
    for (const Landing &L : landings) {
        for (int64_t i = 0; i < L.count; i++) {
            L.dst[i].accepted = h_stage[L.off + i].accepted;
            L.dst[i].acceptance_sum = h_stage[L.off + i].acceptance_sum;
            L.dst[i].rejections = 0;  // deferred runs cannot meet a rejection
        }
        bad |= h_stage_abort[L.abort_slot] != 0;
    }
    landings.clear();
    stage_used = abort_used = 0;
    // deferred runs draw only power-of-two ranges, so NumPy's Lemire sampler cannot reject there: an abort is a
    // kernel's OVERFLOW report (a field beyond the kernel's LDS image).  The statistics above landed; the device
    // state of the aborting run is past its failing sweep and unspecified.
    if (bad)
        throw std::runtime_error("a deferred run aborted on the device (a field beyond a kernel's LDS image: OVERFLOW; "
                                 "deferred runs cannot meet NumPy Lemire rejections); the device state is unspecified: "
                                 "re-upload the configuration");
}

void sv::Emitter::emit(hipStream_t compute, const void *a, size_t bytes0, const void *b, size_t bytes1, void *ha,
                       void *hb) {
    SV_HIP(hipGetDevice(&device));
    if (!copy) {
        SV_HIP(hipStreamCreateWithFlags(&copy, hipStreamNonBlocking));
        for (int i = 0; i < 2; i++) {
            SV_HIP(hipEventCreateWithFlags(&snap[i], hipEventDisableTiming));
            SV_HIP(hipEventCreateWithFlags(&done[i], hipEventDisableTiming));
        }
    }
    if (bytes[0] != bytes0 || bytes[1] != bytes1) {
        wait();
        for (int i = 0; i < 2; i++)
            for (int f = 0; f < 2; f++) {
                if (buf[i][f]) SV_HIP(hipFree(buf[i][f]));
                buf[i][f] = nullptr;
                const size_t nb = f == 0 ? bytes0 : bytes1;
                if (nb) SV_HIP(hipMalloc(&buf[i][f], nb));
            }
        bytes[0] = bytes0;
        bytes[1] = bytes1;
    }
    const int i = k;
    k ^= 1;
    if (busy[i]) SV_HIP(hipStreamWaitEvent(compute, done[i], 0));  // the buffer's previous copy has left
    const void *src[2] = {a, b};
    void *dst[2] = {ha, hb};
    for (int f = 0; f < 2; f++)
        if (src[f] && dst[f] && bytes[f]) SV_HIP(hipMemcpyAsync(buf[i][f], src[f], bytes[f], hipMemcpyDeviceToDevice, compute));
    SV_HIP(hipEventRecord(snap[i], compute));
    SV_HIP(hipStreamWaitEvent(copy, snap[i], 0));
    for (int f = 0; f < 2; f++)
        if (src[f] && dst[f] && bytes[f]) SV_HIP(hipMemcpyAsync(dst[f], buf[i][f], bytes[f], hipMemcpyDeviceToHost, copy));
    SV_HIP(hipEventRecord(done[i], copy));
    busy[i] = true;
}

void sv::Emitter::wait() {
    if (!copy) return;
    SV_HIP(hipStreamSynchronize(copy));
    busy[0] = busy[1] = false;
}

hipError_t sv::Emitter::release() {
    if (!copy) return hipSuccess;
    (void)hipSetDevice(device);
    const hipError_t e = hipStreamSynchronize(copy);
    for (int i = 0; i < 2; i++) {
        for (int f = 0; f < 2; f++)
            if (buf[i][f]) (void)hipFree(buf[i][f]);
        (void)hipEventDestroy(snap[i]);
        (void)hipEventDestroy(done[i]);
    }
    (void)hipStreamDestroy(copy);
    *this = Emitter();
    return e;
}

static hipEvent_t take_event(std::vector<hipEvent_t> &pool) {
    if (!pool.empty()) {
        hipEvent_t e = pool.back();
        pool.pop_back();
        return e;
    }
    hipEvent_t e;
    SV_HIP(hipEventCreate(&e));
    return e;
}

void sv_ctx::time_begin(hipEvent_t *a) {
    *a = nullptr;
    if (!timing) return;
    *a = take_event(ev_pool);
    SV_HIP(hipEventRecord(*a, stream));
}

void sv_ctx::time_end(hipEvent_t a, int64_t launches, int64_t first) {
    if (!timing || !a) return;
    hipEvent_t b = take_event(ev_pool);
    SV_HIP(hipEventRecord(b, stream));
    ev_pending.push_back({a, b});
    ev_launches.push_back(launches);
    ev_first.push_back(first);
}

void sv_ctx::time_collect() {
    for (size_t i = 0; i < ev_pending.size(); i++) {
        auto &p = ev_pending[i];
        float ms = 0.f;
        SV_HIP(hipEventSynchronize(p.second));
        SV_HIP(hipEventElapsedTime(&ms, p.first, p.second));
        timed_ms += ms;
        timed_launches += ev_launches[i];
        ev_pool.push_back(p.first);
        ev_pool.push_back(p.second);
    }
    ev_pending.clear();
    ev_launches.clear();
    ev_first.clear();
}

void sv_ctx::time_discard() {
    for (auto &p : ev_pending) {
        ev_pool.push_back(p.first);
        ev_pool.push_back(p.second);
    }
    ev_pending.clear();
    ev_launches.clear();
    ev_first.clear();
}

void sv_ctx::time_keep_before(int64_t bad) {
    size_t j = 0;
    for (size_t i = 0; i < ev_pending.size(); i++) {
        if (ev_first[i] + ev_launches[i] <= bad) {
            ev_pending[j] = ev_pending[i];
            ev_launches[j] = ev_launches[i];
            ev_first[j] = ev_first[i];
            j++;
        } else {
            ev_pool.push_back(ev_pending[i].first);
            ev_pool.push_back(ev_pending[i].second);
        }
    }
    ev_pending.resize(j);
    ev_launches.resize(j);
    ev_first.resize(j);
}

// Streaming copy b[i] = a[i] with W-byte lanes (16: dwordx4, 8: dwordx2): the measured HBM ceiling the
// roofline fraction is also reported against, and the known byte count that calibrates
// the PMC FETCH_SIZE / WRITE_SIZE counters for this repo's access widths (MI355X_MICROARCH.md, HBM).
template <typename T, int U>
__global__ __launch_bounds__(256) void hbm_copy(const T *__restrict__ a, T *__restrict__ b, int64_t n) {
    // U loads in flight per lane before the stores; each workgroup copies one contiguous chunk of 256 U
    // vectors (sv_hbm_copy reports the fastest U: one load per lane in a grid-stride loop measured 4.9 TB/s)
    const int64_t base = (int64_t)blockIdx.x * (256 * U) + threadIdx.x;
    T v[U];
#pragma unroll
    for (int k = 0; k < U; k++)
        if (base + 256 * k < n) v[k] = a[base + 256 * k];
#pragma unroll
    for (int k = 0; k < U; k++)
        if (base + 256 * k < n) b[base + 256 * k] = v[k];
}

extern "C" {

int sv_ctx_set_timing(sv_ctx *ctx, int32_t enable) {
    if (!ctx) return -1;
    ctx->timing = enable != 0;
    ctx->timing_mode = enable;
    try {  // the first timed batch should not pay for creating its events
        SV_HIP(hipSetDevice(ctx->device));
        while (enable && ctx->ev_pool.size() < 4) {
            hipEvent_t e;
            SV_HIP(hipEventCreate(&e));
            ctx->ev_pool.push_back(e);
        }
    } catch (const std::exception &e) {
        ctx->err = e.what();
        return -2;
    }
    ctx->timed_ms = 0.0;
    ctx->timed_launches = 0;
    return 0;
}

int sv_ctx_sweep_counts(sv_ctx *ctx, int64_t *hot, int64_t *fused, int64_t *generic) {
    if (!ctx) return -1;
    if (hot) *hot = ctx->sweeps_hot;
    if (fused) *fused = ctx->sweeps_fused;
    if (generic) *generic = ctx->sweeps_generic;
    ctx->sweeps_hot = ctx->sweeps_fused = ctx->sweeps_generic = 0;
    return 0;
}

int sv_ctx_split_counts(sv_ctx *ctx, int64_t *sweeps) {
    if (!ctx) return -1;
    if (sweeps) *sweeps = ctx->sweeps_split;
    ctx->sweeps_split = 0;
    return 0;
}

int sv_ctx_set_table_cap(sv_ctx *ctx, int32_t cap) {
    if (!ctx || cap < 0) return -1;
    ctx->table_cap = (size_t)cap;
    return 0;
}

int sv_ctx_table_purges(sv_ctx *ctx, int64_t *purges) {
    if (!ctx || !purges) return -1;
    *purges = ctx->table_purges;
    return 0;
}

int sv_ctx_band_counts(sv_ctx *ctx, int64_t *sweeps, int64_t *launches) {
    if (!ctx) return -1;
    if (sweeps) *sweeps = ctx->sweeps_band;
    if (launches) *launches = ctx->launches_band;
    ctx->sweeps_band = ctx->launches_band = 0;
    return 0;
}

int sv_ctx_block_counts(sv_ctx *ctx, int64_t *sweeps, int64_t *launches) {
    if (!ctx) return -1;
    if (sweeps) *sweeps = ctx->sweeps_block;
    if (launches) *launches = ctx->launches_block;
    ctx->sweeps_block = ctx->launches_block = 0;
    return 0;
}

int sv_ctx_set_multisweep(sv_ctx *ctx, int32_t mode, int32_t K) {
    // (K = 1, 2 would leave no odd K >= 3: rejected rather than silently running the default; BAND_MAXK = 15)
    if (!ctx || mode < 0 || mode > 3 || K < 0 || K == 1 || K == 2 || K > 15) return -1;
    ctx->multisweep = mode;
    ctx->block_k = K;
    return 0;
}

int sv_ctx_kernel_time(sv_ctx *ctx, double *ms_total, int64_t *launches) {
    if (!ctx) return -1;
    try {
        ctx->time_collect();
    } catch (const std::exception &e) {
        ctx->err = e.what();
        return -2;
    }
    if (ms_total) *ms_total = ctx->timed_ms;
    if (launches) *launches = ctx->timed_launches;
    return 0;
}

int sv_hbm_copy(sv_ctx *ctx, int64_t bytes, int32_t width, int32_t iters, double *GBps) {
    if (!ctx || bytes < 4096 || iters < 1 || (width != 8 && width != 16)) return -1;
    void *a = nullptr, *b = nullptr;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    int rc = 0;
    try {
        SV_HIP(hipSetDevice(ctx->device));
        bytes &= ~(int64_t)4095;
        SV_HIP(hipMalloc(&a, bytes));
        SV_HIP(hipMalloc(&b, bytes));
        SV_HIP(hipMemsetAsync(a, 1, bytes, ctx->stream));
        SV_HIP(hipMemsetAsync(b, 0, bytes, ctx->stream));
        SV_HIP(hipEventCreate(&e0));
        SV_HIP(hipEventCreate(&e1));
        const int64_t nvec = bytes / width;
        double best_ms = 1e30;
        for (int u : {1, 2, 4, 8}) {
            const int grid = (int)((nvec + 256 * u - 1) / (256 * u));
            auto launch = [&]() {
#define SV_COPY(T, UU) hbm_copy<T, UU><<<grid, 256, 0, ctx->stream>>>((const T *)a, (T *)b, nvec), SV_LAUNCHED("hbm_copy", ctx->stream)
                if (width == 16) {
                    if (u == 1) SV_COPY(uint4, 1); else if (u == 2) SV_COPY(uint4, 2); else if (u == 4) SV_COPY(uint4, 4); else SV_COPY(uint4, 8);
                } else {
                    if (u == 1) SV_COPY(uint2, 1); else if (u == 2) SV_COPY(uint2, 2); else if (u == 4) SV_COPY(uint2, 4); else SV_COPY(uint2, 8);
                }
#undef SV_COPY
            };
            launch();  // warm: page mappings, clocks
            SV_HIP(hipEventRecord(e0, ctx->stream));
            for (int i = 0; i < iters; i++) launch();
            SV_HIP(hipEventRecord(e1, ctx->stream));
            SV_HIP(hipEventSynchronize(e1));
            SV_HIP(hipGetLastError());
            float ms = 0.f;
            SV_HIP(hipEventElapsedTime(&ms, e0, e1));
            best_ms = std::min(best_ms, (double)ms);
        }
        const double ms = best_ms;
        if (GBps) *GBps = 2.0 * (double)bytes * iters / (ms * 1e-3) / 1e9;
    } catch (const std::exception &e) {
        ctx->err = e.what();
        rc = -2;
    }
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
    (void)hipFree(a);
    (void)hipFree(b);
    return rc;
}

int sv_ctx_set_deferred(sv_ctx *ctx, int32_t on) {
    if (!ctx) return -1;
    try {
        SV_HIP(hipSetDevice(ctx->device));
        if (!on && ctx->deferred) {
            ctx->deferred = false;
            SV_HIP(hipStreamSynchronize(ctx->stream));
            ctx->land();
            ctx->time_collect();
        }
        ctx->deferred = on != 0;
        return 0;
    } catch (const std::exception &e) {
        ctx->err = e.what();
        return -2;
    }
}

int sv_ctx_sync(sv_ctx *ctx) {
    if (!ctx) return -1;
    try {
        SV_HIP(hipSetDevice(ctx->device));
        SV_HIP(hipStreamSynchronize(ctx->stream));
        ctx->land();
        ctx->time_collect();
        return 0;
    } catch (const std::exception &e) {
        ctx->err = e.what();
        return -2;
    }
}

int sv_host_alloc(size_t bytes, void **out) {
    if (!out) return -1;
    *out = nullptr;
    if (!bytes) return -1;
    void *p = nullptr;
    if (hipHostMalloc(&p, bytes, hipHostMallocDefault) != hipSuccess) return -2;
    *out = p;
    return 0;
}

int sv_host_free(void *p) {
    if (!p) return -1;
    return hipHostFree(p) == hipSuccess ? 0 : -2;
}

int sv_villain_emit(sv_villain *st, double *phi, int64_t *n) {
    if (!st || (!phi && !n)) return -1;
    try {
        SV_HIP(hipSetDevice(st->ctx->device));
        const size_t V = (size_t)st->N * st->N;
        st->emitter.emit(st->ctx->stream, st->phi[st->cur], V * sizeof(double), st->n[st->cur], 2 * V * sizeof(int64_t),
                         phi, n);
        return 0;
    } catch (const std::exception &e) {
        st->ctx->err = e.what();
        return -2;
    }
}

int sv_villain_emit_wait(sv_villain *st) {
    if (!st) return -1;
    try {
        SV_HIP(hipSetDevice(st->ctx->device));
        st->emitter.wait();
        return 0;
    } catch (const std::exception &e) {
        st->ctx->err = e.what();
        return -2;
    }
}

int sv_worldline_emit(sv_worldline *st, int64_t *m, void *v) {
    if (!st || (!m && !v)) return -1;
    try {
        SV_HIP(hipSetDevice(st->ctx->device));
        const size_t V = (size_t)st->N * st->N;
        st->emitter.emit(st->ctx->stream, st->m, 2 * V * sizeof(int64_t), st->v,
                         V * (st->v_is_float ? sizeof(double) : sizeof(int64_t)), m, v);
        return 0;
    } catch (const std::exception &e) {
        st->ctx->err = e.what();
        return -2;
    }
}

int sv_worldline_emit_wait(sv_worldline *st) {
    if (!st) return -1;
    try {
        SV_HIP(hipSetDevice(st->ctx->device));
        st->emitter.wait();
        return 0;
    } catch (const std::exception &e) {
        st->ctx->err = e.what();
        return -2;
    }
}

int sv_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

const char *sv_build_info(void) {
    return "libsvhip gfx950 (PCG64 stream replay; fused Villain sweep; Coexact/Plaquette colour passes)";
}

int sv_ctx_create(int device, sv_ctx **out) {
    if (!out) return -1;
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) return -3;  // no such HIP device
    sv_ctx *ctx = new sv_ctx();
    try {
        ctx->device = device;
        SV_HIP(hipSetDevice(device));
        SV_HIP(hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking));
        // abort flag, report count and the reports in one allocation: a batch tail reads the flag, the count and the
        // first TAIL_REPORTS reports with one copy
        SV_HIP(hipMalloc(&ctx->d_abort, 16 + sv::MAX_REPORTS * sizeof(sv::Report)));
        ctx->d_nreport = reinterpret_cast<uint32_t *>(ctx->d_abort + 1);
        ctx->d_reports = reinterpret_cast<sv::Report *>(reinterpret_cast<char *>(ctx->d_abort) + 16);
        SV_HIP(hipMemset(ctx->d_abort, 0, sizeof(int32_t)));
        SV_HIP(hipMemset(ctx->d_nreport, 0, sizeof(uint32_t)));
        SV_HIP(hipHostMalloc((void **)&ctx->h_flag, 2 * sizeof(int32_t), hipHostMallocMapped | hipHostMallocCoherent));
        SV_HIP(hipHostGetDevicePointer((void **)&ctx->d_flag, ctx->h_flag, 0));
        ctx->h_prog = ctx->h_flag + 1;
        ctx->d_prog = ctx->d_flag + 1;
        ctx->h_flag[0] = ctx->h_flag[1] = 0;
        ctx->ensure_blocks(64);
        ctx->ensure_skips(64);
        ctx->ensure_stats(64);
        *out = ctx;
        return 0;
    } catch (const std::exception &e) {
        static thread_local std::string last;
        last = e.what();
        delete ctx;
        return -2;
    }
}

int sv_ctx_destroy(sv_ctx *ctx) {
    if (!ctx) return 0;
    (void)hipSetDevice(ctx->device);
    const hipError_t e = hipDeviceSynchronize();  // every stream: no queued launch may still hold a table or scratch
    for (auto &kv : ctx->tables) (void)hipFree(kv.second);
    for (auto &p : ctx->ev_pending) {
        (void)hipEventDestroy(p.first);
        (void)hipEventDestroy(p.second);
    }
    for (auto e : ctx->ev_pool) (void)hipEventDestroy(e);
    (void)hipFree(ctx->d_abort);
    if (ctx->h_abort) (void)hipHostFree(ctx->h_abort);
    if (ctx->h_flag) (void)hipHostFree(ctx->h_flag);
    for (char *h : ctx->h_plan)
        if (h) (void)hipHostFree(h);
    for (hipEvent_t e : ctx->ev_plan)
        if (e) (void)hipEventDestroy(e);
    if (ctx->h_stage) (void)hipHostFree(ctx->h_stage);
    if (ctx->h_tail) (void)hipHostFree(ctx->h_tail);
    if (ctx->h_stage_abort) (void)hipHostFree(ctx->h_stage_abort);
    (void)hipFree(ctx->d_blocks);
    (void)hipFree(ctx->d_skips);
    (void)hipFree(ctx->d_stats);
    sv::worm_release(ctx);
    (void)hipStreamDestroy(ctx->stream);
    delete ctx;
    return e == hipSuccess ? 0 : -2;  // (the context is gone: the caller learns only that its last work failed)
}

extern "C++" {
namespace sv {
void launch_failed(const char *kernel, const char *stage, hipError_t e) {
    const std::string m = std::string("SV_SYNC_CHECK: kernel ") + kernel + " failed at " + stage + ": " + hipGetErrorString(e);
    fprintf(stderr, "[sv] %s\n", m.c_str());
    throw std::runtime_error(m);
}
}  // namespace sv
}

const char *sv_last_error(sv_ctx *ctx) { return ctx ? ctx->err.c_str() : "no context"; }

// NumPy's pcg64_state (numpy/random/src/pcg64/pcg64.h) with a native 128-bit pcg128_t: the Python side
// checks this layout against the public state dict before it passes any address here.
struct np_pcg64_state {
    uint64_t *pcg;  // {state lo, state hi, inc lo, inc hi}
    int has_uint32;
    uint32_t uinteger;
};

int sv_rng_gather(void *const *pcg64_states, int32_t R, sv_rng *out) {
    if (!pcg64_states || !out || R < 0) return -1;
    for (int32_t r = 0; r < R; r++) {
        const np_pcg64_state *st = (const np_pcg64_state *)pcg64_states[r];
        if (!st || !st->pcg) return -1;
        out[r] = sv_rng{st->pcg[1], st->pcg[0], st->pcg[3], st->pcg[2], st->has_uint32, st->uinteger};
    }
    return 0;
}

int sv_rng_scatter(const sv_rng *in, int32_t R, void *const *pcg64_states) {
    if (!pcg64_states || !in || R < 0) return -1;
    for (int32_t r = 0; r < R; r++) {
        np_pcg64_state *st = (np_pcg64_state *)pcg64_states[r];
        if (!st || !st->pcg) return -1;
        st->pcg[0] = in[r].state_lo;
        st->pcg[1] = in[r].state_hi;
        st->pcg[2] = in[r].inc_lo;
        st->pcg[3] = in[r].inc_hi;
        st->has_uint32 = in[r].has_uint32;
        st->uinteger = in[r].uinteger;
    }
    return 0;
}

}  // extern "C"
