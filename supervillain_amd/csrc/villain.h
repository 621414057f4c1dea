// villain.h -- declarations shared by villain.hip (single-lattice drivers) and domain.hip
// (domain decomposition): the fused sweep kernel's arguments and the host planning helpers.
#pragma once
#include "common.h"

namespace sv {

struct VParams {
    int32_t N;
    double half_kappa;
    int64_t W;
    double lo_phi, range_phi;  // uniform(-interval_phi, +interval_phi): low, high - low
    int64_t interval_n;
    uint32_t k, thr;           // choice over 2*interval_n+1 values; Lemire threshold
};

static constexpr uint32_t OVERFLOW_BLOCK = 0xFFFFu;  // report tag: state not representable on this path
// report tag: a multi-sweep band launch (villain_sweep_hot_band) could not run as planned (its workgroups were not
// spread over the XCDs as expected, or a band barrier timed out); the launch's first sweep is replayed without it
static constexpr uint32_t BAND_FAIL_BLOCK = 0xFFFEu;

// (t, x) = (s / N, s mod N) for a site index s of a lattice of fewer than 2^32 sites (every device path addresses
// stream positions with 32 bits): one 32-bit unsigned division instead of the 64-bit one (a long emulated
// sequence on the GPU) the grid-stride kernels paid per element
__device__ __forceinline__ void divmod_site(int64_t s, int64_t N, int64_t &t, int64_t &x) {
    const uint32_t q = (uint32_t)s / (uint32_t)N;
    t = q;
    x = s - (int64_t)q * N;
}
static constexpr int FW_MAX = 123;     // colour-0 sites per region row <= 63, so lane 63 is always spare
static constexpr int RW = FW_MAX + 5;  // 128 region columns: x0-2 .. x1+2
static constexpr int SMALL_LDS = 128;  // small-offset maps cached in LDS (in-row offsets are <= w+4)

// Geometry of one fused launch.  Periodic mode (TILE=false): the whole N x N lattice, rows and
// columns wrap in memory.  Tile mode (TILE=true, domain decomposition): an Ht x Wt tile at global
// origin (T0, X0) of an Nt x Nx lattice, stored with a ghost frame (rows -2..Ht+2, columns
// -2..Wt+2 filled by the halo exchange) so memory never wraps; only the RNG addressing and the
// colouring use global coordinates.
struct FGeom {
    int32_t Nt, Nx;   // global lattice
    int32_t T0, X0;   // tile origin (0, 0 in periodic mode)
    int32_t Ht, Wt;   // tile extent (Nt, Nx in periodic mode)
    int64_t pitch;    // row pitch of phi/n buffers (elements)
    int64_t plane;    // n component stride (elements)
    int64_t org;      // element offset of tile site (0, 0)
};

struct FArgs {
    VParams P;
    FGeom G;
    const double *phi_in;
    const int64_t *n_in;
    double *phi_out;
    int64_t *n_out;
    int32_t nsx, TH, nsy;  // column strips, rows per strip tile, row tiles
    const Block *blocks;   // this sweep's 11 descriptors
    const uint32_t *skips;
    const JumpTables *T;
    Affine adv[3];  // advance a row base by NW rows: [0] NW*Nx draws, [1] NW*Nx/2, [2] NW*Nx/4
    sv_stats *stat;
    DevScratch S;
    uint32_t sweep;
    uint64_t ph_key = 0, ph_sweep = 0;  // counter-based mode: Philox key, this launch's global sweep number
    // replica batch (periodic mode): consecutive runs of tiles_per_rep workgroups serve one replica
    int32_t tiles_per_rep;          // nsx * nsy
    int32_t rep_blocks;             // descriptors per replica (0: shared)
    int64_t rep_field;              // phi elements per replica (n: twice that)
    int32_t rep_stat;               // stats entries per replica
    int32_t rep_obs;                // obs entries per replica
    const JumpTables *const *Trep;  // per-replica tables, or nullptr (all use T)
    const Affine *advrep;           // per-replica adv[3], or nullptr (all use adv)
    unsigned long long *obs;        // OBS kernels: per replica the OBS_WORDS exact observable words (common.h)
    // villain_sweep_hot: per strip (in the XCD-aware logical order) its column strip and rows {ix, t0, t1}, or null
    // (uniform strips of TH rows); lets the strips of the last rounds of slots be shorter (strip_schedule)
    const int32_t *strips = nullptr;
    const int32_t *rep_map = nullptr;    // replica batches: launch's replica slot -> replica (a subset launch), or identity
    // TILE: the window of the launch's region whose sites are counted in the statistics, [r0, r1) x [c0, c1) in
    // region coordinates (domain.hip's deep halos run sweeps over a tile extended by a ring it does not own)
    int32_t own_r0 = -(1 << 30), own_r1 = 1 << 30, own_c0 = -(1 << 30), own_c1 = 1 << 30;
    // villain_sweep_hot: waves (rows per step) of a workgroup, 4 or 8 (adv must then advance 8 rows)
    int32_t hot_nw = 4;
    // single-lattice batches: workgroup 0 of the launch of batch sweep k stores k + 1 here (host-mapped) as it starts,
    // i.e. once every earlier launch of the stream has finished; the host bounds its queue by it (run_fused)
    int32_t *progress = nullptr;
};

// Multi-sweep launches of small periodic lattices (villain_sweep_hot_band): the lattice rows are cut
// into one band per XCD; the band's workgroups (all on that XCD, found by its XCC_ID) run K consecutive sweeps, sweep j
// deciding the band extended by 2(K-1-j) rows above and 3(K-1-j) below (the deep-halo rule of domain.hip: every
// draw is addressed by its global stream position, so a recomputed halo row equals its owner's), with an XCD-local
// barrier (atomics and data in that XCD's L2) between sweeps.  Sweep j reads buffer j and writes buffer j + 1:
// [0] is the launch's input, [K] its output, the rest scratch, so bands never wait on each other.
static constexpr int BAND_MAXK = 15;
static constexpr int BAND_CTRL = 64;  // uint32 words per XCD in BandArgs::ctrl: [0] tickets, [32] barrier arrivals
struct BandArgs {
    int32_t K;       // sweeps per launch (odd: the output lands in the other buffer of the ping-pong pair)
    int32_t P;       // workgroups per band
    int32_t own;     // rows owned by a band (Nt / nbands)
    int32_t TH;      // strip rows
    int32_t gen;     // band launches before this one in the batch (ticket and barrier targets)
    int32_t nb;      // descriptors per sweep
    int32_t nbands;  // bands = XCDs
    uint32_t *ctrl;  // nbands * BAND_CTRL counters, zeroed per batch
    double *phi[BAND_MAXK + 1];
    int64_t *n[BAND_MAXK + 1];
};

// Multi-sweep launches by temporal blocking (villain_sweep_block, villain_block.hip): each workgroup
// owns a bs x bs block and keeps the block's deep-halo frame for the whole launch in LDS (sweep j decides the block
// extended by 2(K-1-j) rows / columns above and left and 3(K-1-j) below and right, and reads two more around that), so
// no workgroup waits for another.  Buffers as BandArgs: sweep j's own blocks go to buffer j + 1.  The launch's later
// sweeps move their row bases by `step` (the map of one sweep's stream length: the host checks that every descriptor of
// sweep j + 1 is `step` of sweep j's, with equal buffered-half flags).
struct BlockArgs {
    int32_t K;     // sweeps per launch (odd, as BandArgs)
    int32_t bs;    // block side
    int32_t nbx;   // blocks per row of blocks (N / bs)
    int32_t nb;    // descriptors per sweep
    Affine step;
    double *phi[BAND_MAXK + 1];
    int64_t *n[BAND_MAXK + 1];
};
// The replay of a sweep that met NumPy Lemire rejections, at most one per choice block (villain_sweep_hot_split,
// DESIGN.md 5.0): block j of colour c (blocks[2 + 5 c + j]) draws its sites of rank >= s[4 c + j] from the stream one
// half-word further on -- the rejected word is skipped, neighborhood.py:105-107 drawing again -- which is the block
// descriptor blocksB[2 + 5 c + j] (s = UINT32_MAX: no switch; blocksB is the sweep's 11 descriptors with those
// replaced).  Each row draws from the descriptors of its side of every switch: a strip whose rows all lie on one side
// with one descriptor per block, a strip whose rows contain a switch's row (or wrap around the torus) per row, and the
// few strips whose columns straddle a switch's site in its row on the skip-list body (~2.5x slower: they are dispatched
// first on their XCDs, swap[]).
static constexpr int SPLIT_SWAPS = 32;
struct SplitArgs {
    uint32_t s[8];
    const Block *blocksB;
    int32_t nswap;
    int32_t swap[SPLIT_SWAPS][2];  // (logical slot, strip it runs) where the two differ (split_order)
};
// whether strip [t0, t1) x [x0, x1) of an Nt x Nx periodic lattice draws on both sides of the switch at site rank s
// within one row (sites of rank >= s: linear index >= 2 s, one site of each colour per pair of sites): the switch's
// row lies among the rows it draws in (halo and base rows included) and its site among the columns (lane 63's word and
// the lane pairs included), or the strip's columns wrap around the torus; the switch's row qs, and whether the strip's
// columns lie after its site
__host__ __device__ inline bool split_straddles(uint32_t s, int32_t Nt, int32_t Nx, int32_t t0, int32_t t1, int32_t x0,
                                                int32_t x1, int32_t *qs_out, bool *after) {
    const uint32_t lin = 2u * s;
    const int32_t qs = (int32_t)(lin / (uint32_t)Nx), xs = (int32_t)(lin % (uint32_t)Nx);
    const int32_t ra = t0 - 3, rb = t1 + 3, ca = x0 - 4, cb = x0 + 127;
    *qs_out = qs;
    *after = ca >= xs;
    int32_t d = (qs - ra) % Nt;
    if (d < 0) d += Nt;
    if (!(rb - ra + 1 >= Nt || d <= rb - ra)) return false;
    const bool interior = x0 >= 4 && x1 + 2 < Nx;
    return !interior || (ca < xs && xs <= cb);
}

// strip b of a launch (strip table `tab` or uniform strips of TH rows, nsx column strips over the region's Wt columns)
// in global coordinates: rows [tg0, tg1) (tg0 may be negative or tg1 beyond Nt: they wrap), columns [xg0, xg1), xg0
// the strip's first column wrapped onto the torus (as villain_sweep_hot's X0s + x0)
__host__ __device__ inline void split_strip(const FGeom &G, int nsx, int TH, const int32_t *tab, int b, int32_t &tg0,
                                            int32_t &tg1, int32_t &xg0, int32_t &xg1) {
    const int ix = tab ? tab[3 * b] : b % nsx;
    const int32_t t0 = tab ? tab[3 * b + 1] : (b / nsx) * TH;
    const int32_t t1 = tab ? tab[3 * b + 2] : (t0 + TH < G.Ht ? t0 + TH : G.Ht);
    const int32_t x0 = (int32_t)((int64_t)ix * G.Wt / nsx), x1 = (int32_t)((int64_t)(ix + 1) * G.Wt / nsx);
    tg0 = G.T0 + t0;
    tg1 = G.T0 + t1;
    int32_t g = (G.X0 + x0) % G.Nx;
    if (g < 0) g += G.Nx;
    xg0 = g;
    xg1 = g + (x1 - x0);
}

// whether strip [t0, t1)'s rows (halo and base rows included) contain row qs or wrap around the torus: its rows then lie
// on both sides of a switch in row qs, and the descriptors are chosen per row
__host__ __device__ inline bool split_rows(int32_t qs, int32_t Nt, int32_t t0, int32_t t1) {
    const int32_t ra = t0 - 3, rb = t1 + 3;
    return ra < 0 || rb >= Nt || (ra <= qs && qs <= rb);
}

// the frame's side (rows = columns) and the launch's dynamic LDS bytes
__host__ __device__ inline int32_t block_frame(int32_t bs, int32_t K) { return bs + 5 * (K - 1) + 5; }
__host__ __device__ inline size_t block_lds_bytes(int32_t F) {
    // small-offset maps, row bases [F][2 sets][2 colours][6], phi / r0 / r1 (f64) and n0 / n1 (int32) per frame
    // site, per-sweep statistics (16 x 4 words: count, exact acceptance limbs), the overflow flag and the choice-block
    // descriptors (16 sweeps x 8)
    return 2 * 16 * (size_t)SMALL_LDS + (size_t)F * 24 * 16 + (size_t)F * F * 32 + 512 + 16 + 16 * 8 * 8;
}

// (FArgs::progress) the launch has started: every earlier launch of its stream has finished
__device__ __forceinline__ void note_progress(const FArgs &A) {
    if (A.progress && blockIdx.x == 0 && threadIdx.x == 0)
        __hip_atomic_store(A.progress, (int32_t)A.sweep + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

}  // namespace sv

namespace svh {
using namespace sv;

// Skip lists keyed by (sweep index within the call, block index)
using SkipMap = std::map<std::pair<int, int>, std::vector<uint32_t>>;

struct AbortInfo {
    int32_t abort;
    std::vector<Report> reports;
    uint32_t raw = 0;  // the device's report count (reports past MAX_REPORTS were dropped, in arrival order)
};

// One sweep's block sequence: metropolis uniform(V), then per colour
// [dphi uniform(n_c)][4 bounded choice(n_c)].
std::vector<BlockSpec> villain_specs(int64_t V, int ncol, const int64_t *count, bool has_bounded);
void plan_sweeps(sv_ctx *ctx, Cursor &cur, u128 inc, const std::vector<BlockSpec> &specs, int first, int count,
                 const SkipMap &skips, std::vector<Block> &blocks, std::vector<uint32_t> &skipvec);
void upload_plan(sv_ctx *ctx, const std::vector<Block> &blocks, const std::vector<uint32_t> &skipvec);
VParams make_params(int32_t N, double kappa, int64_t W, double interval_phi, int64_t interval_n);
int absorb_reports(const AbortInfo &a, int first, SkipMap &skips);
void drop_later_skips(SkipMap &skips, const std::pair<int, int> &key);  // (skips after key: stale)
DevScratch scratch(sv_ctx *ctx);
AbortInfo read_abort(sv_ctx *ctx);  // synchronizes the stream

void clear_abort(sv_ctx *ctx);
// Before a batch, in ONE launch: the abort flag and report count, and up to two arrays (multiples of 8 bytes) zeroed
// -- each small hipMemsetAsync is a blit of its own on the queue (~4.5 us of GPU time apiece in the Hammer traces)
// (and, given one, a gate word set to INT32_MAX: no sweep has reported)
void reset_batch(sv_ctx *ctx, void *a, size_t a_bytes, void *b = nullptr, size_t b_bytes = 0, int32_t *gate = nullptr);
int64_t rejections_in(const SkipMap &skips, int sweep, int nblocks);
int fused_th(int32_t N, int nsx);  // rows per strip (SV_FUSED_TH overrides)
// launch one tile-mode sweep with `grid` workgroups: villain_sweep_hot when `hot` (the sweep passes hot_ok),
// villain_sweep_fused<4, true> otherwise
void launch_fused_tile(const FArgs &A, int grid, hipStream_t stream, bool hot);
// launch villain_sweep_fused<4, false, obs> over a replica batch (grid = replicas * tiles_per_rep)
void launch_fused_batch(const FArgs &A, int grid, bool obs, hipStream_t stream);
// villain_hot.hip: whether the fast-draw kernel covers the sweep whose 11 descriptors start at `blocks`,
// and its launch (periodic single lattice or a domain tile, from the geometry)
bool hot_ok(const VParams &P, const Block *blocks);
// the split replay (villain_sweep_hot_split, single lattices and domain tiles, 4 waves): whether it covers the sweep whose
// descriptors start at `blocks` (<= 1 known rejected position per choice block), filling its SplitArgs; its launch
// descriptors start at `blocks` (<= 1 known rejected position per choice block), filling S.s and the sweep's 11
// descriptors after the switches (Bset)
bool split_plan(const VParams &P, const Block *blocks, const uint32_t *skips, u128 inc, SplitArgs &S, Block *Bset);
void launch_hot_split(const FArgs &A, const SplitArgs &S, int grid, hipStream_t stream);
// fill S.nswap / S.swap: the skip-list strips of a launch over region G (strip table `tab` of `grid` entries, or uniform
// strips of TH rows) moved to the start of their XCD's range
void split_order(SplitArgs &S, const FGeom &G, int nsx, int TH, int grid, const int32_t *tab);
// villain_sweep_hot's default descending strip table for H rows and nsx column strips ({ix, t0, t1} per strip)
std::vector<int32_t> band_strips(int32_t H, int nsx);
void launch_hot(const FArgs &A, int grid, hipStream_t stream);
// the band launch (8-wave strips of B.TH rows); band_residency: how many of its workgroups one CU holds at once
void launch_hot_band(const FArgs &A, const BandArgs &B, hipStream_t stream);
int band_residency();
// the temporal-blocking launch (nbx * nbx workgroups of 8 waves)
void launch_block(const FArgs &A, const BlockArgs &B, hipStream_t stream);
// full-row replica batches (config 5) on the fast-draw kernel: whether N qualifies, and the launch (the sweep must
// pass hot_ok for every replica: no skips, no buffered half-word, choice values in range)
bool hot_fr_ok(int32_t N);
bool hot_params_ok(const VParams &P);  // the parameter part of hot_ok
void launch_hot_ph(const FArgs &A, int grid, hipStream_t stream);  // counter-based (Philox) mode
void launch_hot_fr(const FArgs &A, int grid, bool obs, hipStream_t stream);
// plain single-lattice FArgs defaults (one replica, no observables)
void farg_single(FArgs &A, int nsx, int nsy);

}  // namespace svh
