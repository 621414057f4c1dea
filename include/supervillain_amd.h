/*
 * supervillain_amd.h -- C-ABI of libsvhip.so, the MI355X (gfx950) Metropolis sweep engine behind the
 * supervillain generator plugin API.
 *
 * The reference (evanberkowitz/supervillain, pure Python/NumPy) has no native boundary of its own:
 * its generators are duck-typed Python objects called as `generator.step(cfg) -> cfg`
 * (supervillain/generator/generator.py:5-17) from Ensemble.generate (supervillain/ensemble.py:89-92),
 * Sequentially.step (generator/combining.py:38-40) and KeepEvery.step (combining.py:100-104).
 * This header is the boundary a binding of that protocol needs: plain pointers and sizes, no torch
 * types.  the supervillain_amd.generator classes bind it with ctypes (INTEGRATION.md shows the binding).
 *
 * Conventions
 *   - Every function returns 0 on success and a negative code on failure; sv_last_error(ctx) then
 *     holds the message.  Calls are synchronous on return (except sv_*_emit, which says so).
 *   - Host arrays are borrowed, C-contiguous, row-major (component axis first, then (t, x)), exactly
 *     the reference's Form layout (supervillain/lattice/compact.py:244-261): phi (1,N,N) float64,
 *     n and m (2,N,N) int64, v (1,N,N) int64 (float64 when W is infinite, worldline.py:110-112).
 *   - Randomness: the generator's NumPy Generator(PCG64) state crosses as sv_rng and is advanced
 *     exactly as the reference's NumPy calls would advance it, so a seeded device chain equals the
 *     seeded reference chain (integers bit-exact, floats bit-exact up to exp() rounding).
 *   - A context (sv_ctx) owns one HIP device and stream; it is not thread-safe.
 */
#ifndef SUPERVILLAIN_AMD_H
#define SUPERVILLAIN_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct sv_ctx sv_ctx;
typedef struct sv_villain sv_villain;
typedef struct sv_worldline sv_worldline;

/* NumPy PCG64 bit-generator state: bit_generator.state['state'] = {state, inc} as 128-bit halves,
 * plus the half-word buffer ('has_uint32', 'uinteger') NumPy's bounded sampler keeps there. */
typedef struct sv_rng {
    uint64_t state_hi, state_lo, inc_hi, inc_lo;
    int32_t has_uint32;
    uint32_t uinteger;
} sv_rng;

/* Per-sweep counters.  The generators fold these exactly like the reference does, e.g.
 * neighborhood.py:131-135: proposed += V, accepted += accepted, acceptance += acceptance_sum / V. */
typedef struct sv_stats {
    int64_t accepted;
    int64_t proposed;
    double acceptance_sum;
    int64_t rejections; /* NumPy Lemire rejections met (diagnostic; they shift the stream) */
} sv_stats;

/* ---- context ------------------------------------------------------------------------------ */
int sv_ctx_create(int device, sv_ctx **out);
int sv_ctx_destroy(sv_ctx *ctx);
const char *sv_last_error(sv_ctx *ctx);
int sv_device_count(void);
/* Measurement hooks: enable = 1 brackets each batch of back-to-back sweep-kernel launches with
 * hipEvents on the context's stream, enable = 2 brackets every single-lattice fused launch;
 * sv_ctx_kernel_time returns the summed device time and the number of launches since enable
 * (batches that hit a Lemire rejection are not counted). */
int sv_ctx_set_timing(sv_ctx *ctx, int32_t enable);
int sv_ctx_kernel_time(sv_ctx *ctx, double *ms_total, int64_t *launches);
/* Diagnostic: Villain NeighborhoodUpdate sweep launches since the last call (then reset), by kernel -- hot: the
 * fast-draw kernel (int16 n image, no skip lists); fused: the general fused kernel (int32 n image, skip lists,
 * replays); generic: the per-colour int64 path.  A domain counts one launch per tile, a replica batch one per
 * launch.  Lets tests prove which kernel ran (e.g. the int32 fallback after |n| >= 2^14). */
int sv_ctx_sweep_counts(sv_ctx *ctx, int64_t *hot, int64_t *fused, int64_t *generic);
/* Diagnostic: of the hot sweeps since the last call (then reset), those run K at a time by the multi-sweep band
 * launches of small periodic lattices (villain_sweep_hot_band), and the number of such launches. */
int sv_ctx_band_counts(sv_ctx *ctx, int64_t *sweeps, int64_t *launches);
/* Diagnostic: the same for the temporal-blocking launches (villain_sweep_block: K sweeps per launch, each workgroup
 * on its own block and deep-halo frame in LDS). */
int sv_ctx_block_counts(sv_ctx *ctx, int64_t *sweeps, int64_t *launches);
/* Diagnostic: single-lattice sweeps replayed since the last call (then reset) on the split replay
 * (villain_sweep_hot_split): the re-run of a sweep that met NumPy Lemire rejections -- at most one per choice block --
 * drawing each row from the block segment it lies in (the reference draws again, neighborhood.py:105-107). */
int sv_ctx_split_counts(sv_ctx *ctx, int64_t *sweeps);
/* Which multi-sweep launches small periodic lattices may use: 0 temporal blocks or else bands (default), 1 blocks
 * only, 2 bands only, 3 one sweep per launch; K: sweeps per multi-sweep launch, blocks or bands (0: the default, 3; an
 * even K runs as K - 1, and K shrinks until the launch's frame fits; one sweep per launch is mode 3).  Returns -1 for another
 * mode or K outside {0, 3..15}. */
int sv_ctx_set_multisweep(sv_ctx *ctx, int32_t mode, int32_t K);
/* Diagnostic (tests): the context's PCG64 jump-table cache holds at most `cap` increments (0: the default,
 * 1024); a full cache drains the device and is dropped.  sv_ctx_table_purges reports how often it was. */
int sv_ctx_set_table_cap(sv_ctx *ctx, int32_t cap);
int sv_ctx_table_purges(sv_ctx *ctx, int64_t *purges);
/* Host-only: copy R NumPy PCG64 bit-generator states into (gather) or out of (scatter) sv_rng records, given
 * each generator's `bit_generator.ctypes.state_address` (NumPy's pcg64_state, numpy/random/src/pcg64/pcg64.h,
 * native 128-bit layout; the Python wrapper verifies it against the public state dict first).  Lets a
 * batch of R chains cross the boundary without R Python state-dict round trips. */
int sv_rng_gather(void *const *pcg64_states, int32_t R, sv_rng *out);
int sv_rng_scatter(const sv_rng *in, int32_t R, void *const *pcg64_states);
const char *sv_build_info(void);
/* Measurement only: a streaming device copy of `bytes` (two buffers, well above the 256 MB Infinity Cache
 * for a ceiling) with `width`-byte lanes (16 or 8), `iters` timed launches after one warm-up; *GBps = read +
 * write bytes / time.  The roofline is reported against this measured ceiling beside the 8 TB/s spec
 * (SURVEY.md 8(d)); under rocprofv3 --pmc its known byte count calibrates FETCH_SIZE / WRITE_SIZE. */
int sv_hbm_copy(sv_ctx *ctx, int64_t bytes, int32_t width, int32_t iters, double *GBps);

/* ---- Villain (phi, n): NeighborhoodUpdate ------------------------------------------------- */
/* Replaces NeighborhoodUpdate.step, supervillain/generator/villain/neighborhood.py:59-137
 * (constructor arguments kappa, W from the Villain action villain.py:41-45; interval_phi,
 * interval_n from neighborhood.py:38).  Runs `sweeps` consecutive steps; stats has `sweeps`
 * entries.  phi/n are read, updated and written back in place. */
int sv_villain_neighborhood(sv_ctx *ctx, int32_t N, double kappa, int64_t W, double interval_phi, int64_t interval_n,
                            double *phi, int64_t *n, int32_t sweeps, sv_rng *rng, sv_stats *stats);

/* Device-resident form of the same (what a KeepEvery stride or a benchmark folds into one call). */
int sv_villain_create(sv_ctx *ctx, int32_t N, sv_villain **out);
int sv_villain_destroy(sv_villain *st);
int sv_villain_upload(sv_villain *st, const double *phi, const int64_t *n);
int sv_villain_download(sv_villain *st, double *phi, int64_t *n);
/* The optional counter-based mode (sv_rng mode 1, "Philox fast").  The same NeighborhoodUpdate
 * sweep (neighborhood.py:59-137, operation order and acceptance as above) with every draw from Philox4x32-10:
 * site s of sweep number c (rng->counter counts the sweeps done) draws u and dphi from call (s, c, 0) and its four
 * choice words from call (s, c, 1) under key rng->key; a word NumPy's bounded Lemire sampler would reject is
 * redrawn in place (call (s, c, 2 + j + 4 t)).  A different Markov chain from the reference's (NumPy PCG64),
 * statistically equivalent; no replays.  Even N, |W| <= 2^12, |n| < 2^14.  test_threshold (tests
 * only, 0 = Lemire's) replaces the rejection threshold to exercise the redraws.  Returns -2 with the fields
 * unspecified if |n| outgrows the int16 image (re-upload); rng->counter then is not advanced. */
typedef struct sv_philox {
    uint64_t key, counter;
    uint32_t test_threshold;
} sv_philox;
int sv_villain_run_philox(sv_villain *st, double kappa, int64_t W, double interval_phi, int64_t interval_n,
                          int32_t sweeps, sv_philox *rng, sv_stats *stats);

/* Asynchronous emission of the resident configuration into host storage (the D2H of
 * Ensemble.generate's kept configurations, ensemble.py:89-92, overlapped with the sweeps that follow).
 * sv_villain_emit returns at once: the state as of every sweep queued so far is snapshotted on the device
 * (two alternating emission buffers) and copied to phi / n on a copy stream.  The host arrays must stay
 * valid and unread until sv_villain_emit_wait returns; allocate them with sv_host_alloc for a true DMA. */
int sv_villain_emit(sv_villain *st, double *phi, int64_t *n);
int sv_villain_emit_wait(sv_villain *st);
/* Deferred statistics: with on = 1, runs whose sweeps cannot meet a NumPy Lemire rejection (every bounded draw
 * of the update has a power-of-two range) return without synchronizing; their sv_stats arrays are filled
 * (and an unexpected device abort reported) by the next sv_ctx_sync, or by sv_ctx_set_deferred(ctx, 0).  Other
 * calls synchronize as usual.  The stats arrays must stay valid until then. */
int sv_ctx_set_deferred(sv_ctx *ctx, int32_t on);
int sv_ctx_sync(sv_ctx *ctx);
/* Page-locked host memory owned by the library (hipHostMalloc): emission targets whose copies overlap the sweeps.
 * The library never registers caller memory (page-locking arrays that share pages with other objects is unsafe). */
int sv_host_alloc(size_t bytes, void **out);
int sv_host_free(void *p);
/* path: 0 = auto (fused two-colour sweep kernel for even N, per-colour kernels otherwise),
 *       1 = per-colour kernels (any N), 2 = fused (even N only). */
int sv_villain_run(sv_villain *st, double kappa, int64_t W, double interval_phi, int64_t interval_n, int32_t sweeps,
                   sv_rng *rng, sv_stats *stats, int32_t path);
/* Inline observables of the current state (observable/action.py:25-31, energy.py:25-30,
 * winding.py:30-37, wrapping.py:17-25): out[0]=S (villain.py:51-66), out[1]=sum (dn)^2, out[2..3]=sum n_mu */
int sv_villain_observables(sv_villain *st, double kappa, double *out);

/* ---- Villain (phi, n): the other local updates of the Villain Hammer ----------- */
/* Each runs `sweeps` consecutive steps of one generator on the device-resident state of
 * sv_villain_create (upload/download as above), advancing rng exactly as the reference's NumPy calls
 * would; stats has `sweeps` entries, folded by the caller like the reference generator does. */
/* Replaces SiteUpdate.step, supervillain/generator/villain/site.py:43-120 (interval_phi: site.py:23).
 * stats.proposed = V; acceptance_sum = sum of the V Metropolis probabilities. */
int sv_villain_site_run(sv_villain *st, double kappa, double interval_phi, int32_t sweeps, sv_rng *rng,
                        sv_stats *stats);
/* Replaces LinkUpdate.step, supervillain/generator/villain/link.py:53-101 (interval_n: link.py:32; W from
 * the Villain action).  stats.proposed = 2 V; acceptance_sum = sum of the 2 V probabilities (the
 * reference adds their mean, link.py:94). */
int sv_villain_link_run(sv_villain *st, double kappa, int64_t W, int64_t interval_n, int32_t sweeps, sv_rng *rng,
                        sv_stats *stats);
/* Replaces ExactUpdate.step, supervillain/generator/villain/exact.py:50-129 (interval_z: exact.py:29).
 * stats.proposed = V. */
int sv_villain_exact_run(sv_villain *st, double kappa, int64_t interval_z, int32_t sweeps, sv_rng *rng,
                         sv_stats *stats);
/* Replaces CohomologyUpdate.step, supervillain/generator/villain/cohomology.py:64-117 (interval_h:
 * cohomology.py:45).  stats.proposed = D = 2; accepted counts accepted directions. */
int sv_villain_cohomology_run(sv_villain *st, double kappa, int64_t interval_h, int32_t sweeps, sv_rng *rng,
                              sv_stats *stats);

/* ---- Worldline (m, v): CoexactUpdate, PlaquetteUpdate ------------------------------------- */
/* W_eff is Worldline._W (worldline.py:49): W, or 2*pi when W is infinite; v_is_float selects the
 * float64 v layout used at W = infinity. */
int sv_worldline_create(sv_ctx *ctx, int32_t N, int32_t v_is_float, sv_worldline **out);
int sv_worldline_destroy(sv_worldline *st);
int sv_worldline_upload(sv_worldline *st, const int64_t *m, const void *v);
int sv_worldline_download(sv_worldline *st, int64_t *m, void *v);
/* As sv_villain_emit / sv_villain_emit_wait, for (m, v). */
int sv_worldline_emit(sv_worldline *st, int64_t *m, void *v);
int sv_worldline_emit_wait(sv_worldline *st);

/* Replaces CoexactUpdate.step, supervillain/generator/worldline/coexact.py:53-128 (interval_t from
 * coexact.py:32).  v is read only. */
int sv_worldline_coexact_run(sv_worldline *st, double kappa, double W_eff, int64_t interval_t, int32_t sweeps,
                             sv_rng *rng, sv_stats *stats);
int sv_worldline_coexact(sv_ctx *ctx, int32_t N, double kappa, double W_eff, int64_t interval_t, int64_t *m,
                         const void *v, int32_t v_is_float, int32_t sweeps, sv_rng *rng, sv_stats *stats);

/* Replaces PlaquetteUpdate.step, supervillain/generator/worldline/plaquette.py:35-104, in the
 * reference's own visit order: `order` (N*N row-major site indices) is the row-major image of the
 * permutation the reference draws from NumPy's global RandomState (plaquette.py:63).  One sweep. */
int sv_worldline_plaquette_ordered_run(sv_worldline *st, double kappa, double W_eff, const int64_t *order,
                                       sv_rng *rng, sv_stats *stats);
/* NumPy's legacy global RandomState (MT19937) as np.random.get_state() reports it: the 624-word key and the
 * position of the next word (0..624).  has_gauss / gauss are untouched by permutations (the caller keeps them). */
typedef struct {
    uint32_t key[624];
    int32_t pos;
} sv_mt19937;
/* np.random.permutation(n) of that state (numpy/random/mtrand.pyx permutation -> shuffle -> _shuffle_raw with
 * distributions.c random_interval), advancing *mt exactly as NumPy does; the image of plaquette.py:63's
 * np.random.permutation(L.coordinates) in row-major site indices.  Host only (no device work). */
int sv_mt19937_permutation(sv_mt19937 *mt, int64_t n, int64_t *out);
/* `sweeps` reference-order PlaquetteUpdate sweeps (plaquette.py:35-104), each in the visit order NumPy's legacy
 * global RandomState draws (plaquette.py:63), drawn natively from *mt (advanced as NumPy would) -- the next sweep's
 * permutation on a host thread while the device runs the current one; stats has `sweeps` entries. */
int sv_worldline_plaquette_reference_run(sv_worldline *st, double kappa, double W_eff, int32_t sweeps, sv_mt19937 *mt,
                                         sv_rng *rng, sv_stats *stats);
/* Sequentially(PlaquetteUpdate [reference order], CoexactUpdate) (combining.py:38-40) for `steps` steps, both
 * generators on one Generator (G1.rng is G2.rng), the visit orders from *mt as above; stats[2 s] the Plaquette sweep
 * of step s, stats[2 s + 1] its Coexact sweep (interval_t: coexact.py:32). */
int sv_worldline_plaquette_reference_coexact_run(sv_worldline *st, double kappa, double W_eff, int64_t interval_t,
                                                 int32_t steps, sv_mt19937 *mt, sv_rng *rng, sv_stats *stats);
/* Checkerboard variant (a different, equally valid chain): colour passes instead of the
 * random sequential order.  `sweeps` consecutive sweeps. */
int sv_worldline_plaquette_checkerboard_run(sv_worldline *st, double kappa, double W_eff, int32_t sweeps, sv_rng *rng,
                                            sv_stats *stats);
/* Sequentially(PlaquetteUpdate [checkerboard], CoexactUpdate) (combining.py:38-40) for `sweeps` steps in one
 * call, both generators drawing from the same Generator (G1.rng is G2.rng); stats has 2 * sweeps entries:
 * [2 s] the Plaquette sweep of step s, [2 s + 1] its Coexact sweep. */
int sv_worldline_plaquette_coexact_run(sv_worldline *st, double kappa, double W_eff, int64_t interval_t, int32_t sweeps,
                                       sv_rng *rng, sv_stats *stats);
int sv_worldline_plaquette(sv_ctx *ctx, int32_t N, double kappa, double W_eff, int64_t *m, void *v,
                           int32_t v_is_float, const int64_t *order, sv_rng *rng, sv_stats *stats);

/* ---- Worldline (m, v): the other updates of the Worldline Hammer -------------- */
/* Replaces VortexUpdate.step, supervillain/generator/worldline/vortex.py:51-136 (interval_v: vortex.py:33):
 * checkerboard Metropolis on v alone, m read only.  stats.proposed = V. */
int sv_worldline_vortex_run(sv_worldline *st, double kappa, double W_eff, int64_t interval_v, int32_t sweeps,
                            sv_rng *rng, sv_stats *stats);
/* Replaces WrappingUpdate.step, supervillain/generator/worldline/wrapping.py:43-90 (interval_w: wrapping.py:26):
 * 2N torus-cycle proposals on m, v read only.  stats.proposed = 2N. */
int sv_worldline_wrapping_run(sv_worldline *st, double kappa, double W_eff, int64_t interval_w, int32_t sweeps,
                              sv_rng *rng, sv_stats *stats);


/* ---- Villain on a domain-decomposed lattice (multi-GPU; SURVEY.md 8e, BASELINE config 4) -------- */
/* The same chain as sv_villain_* (NeighborhoodUpdate, neighborhood.py:59-137) on an Nt x Nx lattice
 * (Nt = Nx = N for the reference's square Lattice2D) cut into tiles_t x tiles_x tiles, one halo
 * exchange per sweep.  nranks == 1: every tile lives on this context's GPU (bit-exact emulation of any
 * tile grid).  nranks > 1: one tile per rank (rank = tile index, row-major), halos over RCCL; all
 * ranks must make the same calls with the same arguments (collective), and rank 0's
 * sv_domain_unique_id bytes must reach every rank (e.g. a torch.distributed broadcast).
 * Tiles must be even and at least 4 x 4; stats are global (summed over tiles, identical on every rank).
 * nranks == 1 with a unique id and a 1 x 1 grid: the tile's halos go through RCCL to itself (a one-GPU
 * check of the RCCL path). */
typedef struct sv_domain sv_domain;
#define SV_UNIQUE_ID_BYTES 128
int sv_domain_unique_id(uint8_t *id /* SV_UNIQUE_ID_BYTES */);
int sv_domain_create(sv_ctx *ctx, int32_t Nt, int32_t Nx, int32_t tiles_t, int32_t tiles_x, int32_t nranks,
                     int32_t rank, const uint8_t *unique_id, sv_domain **out);
int sv_domain_destroy(sv_domain *d);
/* The same multi-rank domain with its two collectives carried by the caller instead of RCCL (an engine extension:
 * the reference runs one process).  Per halo exchange the library copies this rank's packed messages to host
 * memory and calls xfer(user, nsend, sends, sendbuf, nrecv, recvs, recvbuf): sends / recvs are {peer, offset,
 * words} triples (offsets and sizes in uint64 words of sendbuf / recvbuf, the sv_domain_message_layout grouping),
 * and xfer returns 0 once every message has been sent and received.  Per batch it calls gather(user, local, all,
 * bytes): `all` receives every rank's `bytes`-byte batch summary in rank order (an all-gather).  Both must be called
 * collectively on every rank (e.g. torch.distributed over gloo); a non-zero return fails the run.  model: 0
 * Villain (then sv_domain_run), 1 Worldline (sv_domain_run_worldline).  For checking the multi-rank protocol where
 * RCCL cannot run (two ranks on one GPU), not for speed. */
typedef int (*sv_xfer_fn)(void *user, int32_t nsend, const int64_t *sends, const uint64_t *sendbuf, int32_t nrecv,
                          const int64_t *recvs, uint64_t *recvbuf);
typedef int (*sv_gather_fn)(void *user, const void *local, void *all, int64_t bytes);
int sv_domain_create_hosted(sv_ctx *ctx, int32_t model, int32_t Nt, int32_t Nx, int32_t tiles_t, int32_t tiles_x,
                            int32_t nranks, int32_t rank, sv_xfer_fn xfer, sv_gather_fn gather, void *user,
                            sv_domain **out);
/* Global (Nt, Nx) row-major host arrays; each rank copies its own tiles.  phi == NULL: cold start. */
int sv_domain_upload(sv_domain *d, const double *phi, const int64_t *n);
int sv_domain_download(sv_domain *d, double *phi, int64_t *n);
int sv_domain_run(sv_domain *d, double kappa, int64_t W, double interval_phi, int64_t interval_n, int32_t sweeps,
                  sv_rng *rng, sv_stats *stats);
/* Host-only geometry query (no GPU needed): for each of the 8 halo messages s (in send order) of tile
 * `rank`: out[10 s ..] = {dy, dx, send_to, src_row0, src_col0, rows, cols, recv_from, dst_row0, dst_col0}
 * -- the message of direction (dy, dx) is the interior block [src_row0, +rows) x [src_col0, +cols),
 * and the message of direction s received from `recv_from` fills the ghost block at (dst_row0, dst_col0)
 * (tile-local coordinates; ghosts are negative or >= the tile extent). */
int sv_domain_exchange_plan(int32_t Nt, int32_t Nx, int32_t tiles_t, int32_t tiles_x, int32_t rank, int64_t *out);
/* Host-only: the RCCL message layout of `rank` when every tile is its own rank (messages grouped per
 * remote peer, one ncclSend / ncclRecv each).  out (>= 2 + 3*16 + 8 + 8 + 8 + 1 int64) = {nsend, nrecv,
 * nsend x {peer, offset, words}, nrecv x {peer, offset, words}, soff[8], roff[8], words[8], msg_words}. */
int sv_domain_message_layout(int32_t Nt, int32_t Nx, int32_t tiles_t, int32_t tiles_x, int32_t rank, int64_t *out);

/* ---- Worldline on a domain-decomposed lattice ("Worldline (config 3) decomposes the same way")
 * One step = the checkerboard PlaquetteUpdate sweep + the CoexactUpdate sweep of
 * sv_worldline_plaquette_coexact_run (plaquette.py:35-104 in its GPU-native colour order, coexact.py:53-128),
 * the same chain bit for bit, on an even Nt x Nx lattice cut into tiles (one halo exchange of (v, m) per step,
 * a 5/4-wide ghost frame).  Same rank / RCCL conventions as sv_domain_*.  Integer v, W_eff a power of two.
 * Arrays: m (2, Nt, Nx) int64, v (Nt, Nx) int64; m == NULL: cold start.  stats: 2 per step
 * ({Plaquette, Coexact}, summed over tiles). */
int sv_domain_create_worldline(sv_ctx *ctx, int32_t Nt, int32_t Nx, int32_t tiles_t, int32_t tiles_x, int32_t nranks,
                               int32_t rank, const uint8_t *unique_id, sv_domain **out);
int sv_domain_upload_worldline(sv_domain *d, const int64_t *m, const int64_t *v);
int sv_domain_download_worldline(sv_domain *d, int64_t *m, int64_t *v);
int sv_domain_run_worldline(sv_domain *d, double kappa, double W_eff, int64_t interval_t, int32_t steps, sv_rng *rng,
                            sv_stats *stats);
/* Host-only geometry queries of a Worldline decomposition (as sv_domain_exchange_plan / _message_layout). */
int sv_domain_exchange_plan_worldline(int32_t Nt, int32_t Nx, int32_t tiles_t, int32_t tiles_x, int32_t rank,
                                      int64_t *out);
int sv_domain_message_layout_worldline(int32_t Nt, int32_t Nx, int32_t tiles_t, int32_t tiles_x, int32_t rank,
                                       int64_t *out);


/* ---- Villain replica batches (BASELINE config 5; SURVEY.md 8e: replicas need no collectives) ------- */
/* R independent NeighborhoodUpdate chains of one even N >= 4 advanced together (one launch per sweep
 * for all replicas); replica r follows rngs[r] exactly as a single sv_villain_run with that state
 * would.  Arrays are (R, N, N) phi and (R, 2, N, N) n; phi == NULL uploads a cold start.  stats has
 * R * sweeps entries ([r][sweep]); obs (optional, R * sweeps * 4 doubles) receives per sweep the
 * sums over the new configuration of (d phi - 2 pi n)^2 (the Villain action is kappa/2 times it,
 * villain.py:51-66), (dn)^2 (winding.py:30-37) and n_0, n_1 (wrapping.py:17-25), computed by the
 * sweep kernel itself (observable/observable.py:50-54 "inline" measurement). */
typedef struct sv_replicas sv_replicas;
int sv_replicas_create(sv_ctx *ctx, int32_t R, int32_t N, sv_replicas **out);
int sv_replicas_destroy(sv_replicas *b);
int sv_replicas_upload(sv_replicas *b, const double *phi, const int64_t *n);
int sv_replicas_download(sv_replicas *b, double *phi, int64_t *n);
int sv_replicas_run(sv_replicas *b, double kappa, int64_t W, double interval_phi, int64_t interval_n, int32_t sweeps,
                    sv_rng *rngs, sv_stats *stats, double *obs);
/* The same with the inline observables measured as the reference's observables report them, each (R, sweeps)
 * row-major (torus_wrapping (R, sweeps, 2)): acceptance = acceptance_sum / V (G.acceptance's per-sweep increment),
 * ActionDensity S / V and InternalEnergyDensity S / (V kappa) with S = kappa / 2 times the first sum (action.py:25-31,
 * energy.py:25-30), WindingSquared the second sum / V (winding.py:30-37), TorusWrapping the n sums (wrapping.py:17-25).
 * Written by the batch loop's copy-out, which overlaps the next batch's sweeps. */
int sv_replicas_run_measured(sv_replicas *b, double kappa, int64_t W, double interval_phi, int64_t interval_n,
                             int32_t sweeps, sv_rng *rngs, sv_stats *stats, double *acceptance, double *action_density,
                             double *energy_density, double *winding_squared, int64_t *torus_wrapping);
/* One-shot form over host arrays: phi (R, N, N) f64 and n (R, 2, N, N) int64 in/out, rngs[R] in/out,
 * stats[R * sweeps], inline_out (R * sweeps * 4, may be NULL) as sv_replicas_run's obs. */
int sv_replicas_villain(sv_ctx *ctx, int32_t R, int32_t N, double kappa, int64_t W, double interval_phi,
                        int64_t interval_n, double *phi, int64_t *n, int32_t sweeps, sv_rng *rngs, sv_stats *stats,
                        double *inline_out);

/* ---- ClassicWorm ---------------------------------------------------------
 * `worms` consecutive worm steps of every chain, one GPU lane per chain (a worm is sequential).
 *   Villain:   replaces ClassicWorm.step, supervillain/generator/villain/worm.py:85-131 + worm_kernel
 *              :133-183 (W: the action's W; only W == 1 changes the algorithm, pass 0 for infinity).
 *   Worldline: replaces ClassicWorm.step, supervillain/generator/worldline/worm.py:137-193 + worm_kernel
 *              :26-94 (W_eff = Worldline._W).
 * rng / rngs: one NumPy PCG64 state per chain, in/out.  hist (may be NULL): per chain the N*N int64
 * displacement histogram of the LAST worm (Vortex_Vortex / Spin_Spin).  lengths (may be NULL): per
 * chain `worms` int64 Worm_Length values.  max_moves (<= 0: unbounded) caps one worm; exceeding it is
 * an error that leaves the chain mid-worm.  The fields are the state's device-resident ones. */
int sv_villain_worm_run(sv_villain *st, double kappa, int64_t W, int32_t worms, int64_t max_moves, sv_rng *rng,
                        int64_t *hist, int64_t *lengths);
int sv_replicas_worm_run(sv_replicas *b, double kappa, int64_t W, int32_t worms, int64_t max_moves, sv_rng *rngs,
                         int64_t *hist, int64_t *lengths);
int sv_worldline_worm_run(sv_worldline *st, double kappa, double W_eff, int32_t worms, int64_t max_moves, sv_rng *rng,
                          int64_t *hist, int64_t *lengths);
/* R independent Worldline chains from host arrays: m (R, 2, N, N) int64 in/out, v (R, N, N) int64 or
 * float64 (v_is_float), rngs[R]. */
int sv_worldline_worm_batch(sv_ctx *ctx, int32_t R, int32_t N, double kappa, double W_eff, int64_t *m, const void *v,
                            int32_t v_is_float, int32_t worms, int64_t max_moves, sv_rng *rngs, int64_t *hist,
                            int64_t *lengths);

#ifdef __cplusplus
}
#endif
#endif
