// villain_hot.hip -- the headline sweep kernel: one NeighborhoodUpdate sweep
// (supervillain/generator/villain/neighborhood.py:59-137), both colours, in one launch.
//
// Same decomposition and exact arithmetic as villain.hip's villain_sweep_fused (column strips streamed
// through an LDS ring of rows), specialised to the sweeps that make up all but a few percent
// of a chain -- no NumPy Lemire rejection known in the sweep's choice blocks, and equal buffered-half flags
// within each forward/backward block pair -- so that the instruction stream carries nothing else:
//
//  * every strip draws from LDS-cached small-offset maps: interior strips with the paired choice words
//    (4 PCG64 compositions per site-update), edge strips with a second row-base set at the first wrapped
//    column and unpaired words (6 compositions, ~6% of the waves at L=4096);
//  * the 128-bit affine step is written out with the carries of v_mad_u64_u32 (6 v_mad_u64_u32,
//    4 v_mul_lo_u32, 4 v_addc: the compiler's form of the same product spends ~12 moves and 7 64-bit adds);
//  * a rejected choice word is detected with one compare per word and reported on a rare branch;
//  * what a rejected proposal leaves unchanged is not recomputed: phi is normalised (+0.0) once when a row
//    enters LDS, and n, phi and the incremental r of neighborhood.py:129 are rewritten only by lanes whose
//    proposal was accepted (0.7% of them at kappa = 0.5), behind a wave-uniform ballot.
//
// Exactness: every value that reaches phi or n is computed in the reference's operation order.
// The residual r and dS reach nothing but exp(-dS); the `0.0 +` the reference's d() and face_sum() put in
// front of them changes at most the sign of a zero, and exp(+-0) = 1.
// 4 waves per SIMD: LDS <= 40 KB (6-row residual ring, int16 n image), <= 128 VGPRs
#ifndef SV_EXP_SCOEF
#define SV_EXP_SCOEF 1  // exp coefficients as SGPR operands (18 VGPRs fewer)
#endif
#include "fused.h"
#include "philox.h"

// Measured and kept (r3-r4 A/Bs): row loads / stores by 32-bit byte offsets from the SGPR bases; row bases
// advanced by precomputed maps behind a wave-uniform test; the next row step's loads issued right after the commit,
// before the step's barrier; n read from LDS with sign-extending loads; each lane of a paired draw reading the one base
// it composes with (r4: the last three with u53's one-shift form 221.8 / 225.3 -> 218.7 / 221.2 us per L=4096 sweep).
// The counter-based kernel (29.5 KB of LDS, 81 VGPRs) runs at 4 waves per SIMD: 4, 5 and 6 measured flat (r336).

#ifndef SV_WGTIME
#define SV_WGTIME 0  // timing experiments: per-workgroup timestamps (sv_debug_wgtime)
#endif

namespace sv {

#if SV_WGTIME
// per launch slot: [wg][0..3] = entry, loop start, loop end, exit (s_memrealtime, 100 MHz), [4] = HW_ID,
// [5] = row bases ready (prologue split)
constexpr int WGT = 6;
__device__ uint64_t g_wgtime[65536 * WGT];
// band launches: per (band slot, sweep) entry, row bases, loop start, loop end, exit, barrier passed, HW_ID, XCC_ID
constexpr int BT = 8, BT_SW = 16;
__device__ uint64_t g_bandtime[8 * 128 * BT_SW * BT];
__device__ __forceinline__ uint64_t rt_now() { return __builtin_amdgcn_s_memrealtime(); }
#endif

// Interior strips: the fwd/bwd blocks of a direction read the two halves of one u64 for two adjacent lanes (draws_fastp
// in fused.h explains the packing of pk); each lane reads the one word base of each direction it composes with (bw:
// the wave's colour set in LDS), a per-lane LDS address instead of two broadcast reads and four selects per direction
__device__ __forceinline__ HotDraws hot_draws_paired_sel(const FArgs &A, int32_t lane, uint32_t pk, const u128 *bw,
                                                         const SmallTab &sm) {
    HotDraws D;
    D.u = u53(xsl_rr(hot_apply(sm, pk & (SMALL_LDS - 1), bw[0])));
    D.dphi = A.P.lo_phi + A.P.range_phi * u53(xsl_rr(hot_apply(sm, (pk >> 7) & (SMALL_LDS - 1), bw[1])));
#pragma unroll
    for (int mu = 0; mu < 2; mu++) {
        const uint32_t half = (pk >> (28 + mu)) & 1u;
        const uint64_t X = xsl_rr(hot_apply(sm, (pk >> (14 + 7 * mu)) & (SMALL_LDS - 1), bw[2 + 2 * mu + half]));
        const uint32_t send = half ? (uint32_t)X : (uint32_t)(X >> 32);
        const uint32_t got = pair_exchange(send, half, lane);
        D.w[2 * mu] = half ? got : (uint32_t)X;
        D.w[2 * mu + 1] = half ? (uint32_t)(X >> 32) : got;
    }
    return D;
}

// The split replay's paired draws (fast_pack_g): a matched direction as hot_draws_paired_sel; a mismatched one (bit mu
// of the wave-uniform `mism`) keeps the low half of the word it computed and passes the high half to lane + 1
__device__ __forceinline__ HotDraws hot_draws_paired_g(const FArgs &A, int32_t lane, uint32_t pk, uint32_t mism,
                                                       const u128 *bw, const SmallTab &sm) {
    HotDraws D;
    D.u = u53(xsl_rr(hot_apply(sm, pk & (SMALL_LDS - 1), bw[0])));
    D.dphi = A.P.lo_phi + A.P.range_phi * u53(xsl_rr(hot_apply(sm, (pk >> 7) & (SMALL_LDS - 1), bw[1])));
#pragma unroll
    for (int mu = 0; mu < 2; mu++) {
        const uint32_t sel = (pk >> (28 + mu)) & 1u;
        const uint64_t X = xsl_rr(hot_apply(sm, (pk >> (14 + 7 * mu)) & (SMALL_LDS - 1), bw[2 + 2 * mu + sel]));
        const uint32_t mm = (mism >> mu) & 1u;
        const uint32_t oh = mm ? 0u : sel;  // the half of X this lane draws itself: 1 high, 0 low
        const uint32_t send = oh ? (uint32_t)X : (uint32_t)(X >> 32);
        const uint32_t got = pair_exchange(send, mm | sel, lane);  // (mm | sel): from lane - 1, else lane + 1
        const uint32_t own = oh ? (uint32_t)(X >> 32) : (uint32_t)X;
        D.w[2 * mu] = sel ? got : own;
        D.w[2 * mu + 1] = sel ? own : got;
    }
    return D;
}

// The split replay's switches as one workgroup sees them (at most two; villain_sweep_hot_split): switch k changes
// block blk[k] (4 c + j) at global row qs[k] -- rows after it draw from blocksB, rows before from blocks, and row qs[k]
// itself by `after` (the strip's columns all lie after the switch's site, or all before: strips whose columns straddle
// it run the skip-list body)
struct SplitSw {
    int32_t qs[2];       // INT32_MAX: no switch
    uint32_t blk[2];     // 4 c + j
    uint32_t after;      // bit k
    __device__ __forceinline__ uint32_t mask(int c, int32_t gq) const {
        uint32_t m = 0;
#pragma unroll
        for (int k = 0; k < 2; k++) {
            const bool on = gq > qs[k] || (gq == qs[k] && ((after >> k) & 1u));
            m |= (on && (blk[k] >> 2) == (uint32_t)c) ? 1u << (blk[k] & 3u) : 0u;
        }
        return m;
    }
    // a switch row within [g - 1, g + span]
    __device__ __forceinline__ bool near(int32_t g, int32_t span) const {
        return (qs[0] >= g - 1 && qs[0] <= g + span) || (qs[1] >= g - 1 && qs[1] <= g + span);
    }
};

// The workgroup's LDS (one allocation shared by the two bodies below)
struct HotEmpty {};
// PH (counter-based mode) keeps no small-offset maps, row-advance maps or row bases: its LDS is 6 KB smaller, which
// lets a fifth workgroup onto a CU
// OBSL (replica batches with inline observables): each lane's running sums over the strip live in LDS, added to by
// no-return LDS atomics at every row store -- a wave reduction per row step cost ~25% of the sweep (r352), and the
// same sums held in registers spilled (r353); full-row strips never need the second set of row bases, which makes
// the room.  n0 and n1 sums share one 64-bit word (n0 + 2^32 n1, two's complement).
struct ObsLane {
    unsigned long long act[256];  // exact action values round(t 2^40) (common.h)
    unsigned long long w2[256];
    unsigned long long npk[256];
};
template <bool PH, bool OBSL = false, int NWL = 4>
struct HotLDST {
    static constexpr int R = FusedGeom<NWL>::R;
    // the residuals r live from the colour-0 pass of step t (rows t+1..t+5) to the colour-1 pass of step t+4
    // (which reads row t+4 again): NW + 2 rows
    static constexpr int RR = NWL + 2;
    using nint = int16_t;  // hot_ok / commit bound |n|
    double phi[R][RW];
    double r0[RR][RW];
    double r1[RR][RW];
    nint n0[R][RW];
    nint n1[R][RW];
    std::conditional_t<PH, HotEmpty, SmallTab> small;
    std::conditional_t<PH, HotEmpty, Affine[3]> adv;
    // per wave: [8c + ty] block ty's base for the colour-c row at xb; [16 + ..] at xw (edge strips of rows > SMALL_LDS)
    std::conditional_t<PH, HotEmpty, std::conditional_t<OBSL, u128[NWL][16], u128[NWL][32]>> base;
    int32_t bad;
    int32_t stop;  // POLL: a rejection was reported by some workgroup: leave the (discarded) sweep
    // SKIP: per colour and choice block, its known rejected stream positions (not in the replica-observables layout,
    // which needs every byte for its fourth workgroup per CU)
    std::conditional_t<OBSL, HotEmpty, uint32_t[2][4][HOT_MAXSK]> sk;
    unsigned long long obsw[5];  // OBS: the workgroup's exact observable words (common.h OBS_WORDS, but the big term)
    double obig;                 // OBS: the workgroup's action terms t >= ACT_LIMIT (common.h)
    std::conditional_t<OBSL, ObsLane, HotEmpty> ol;
    // band launches (8-wave workgroups): the workgroup's statistics per sweep of the launch, flushed once at its end
    struct BandStats {
        unsigned long long w[16][4];  // per sweep: accepted, the exact acceptance limbs (common.h)
    };
    std::conditional_t<NWL == 8, BandStats, HotEmpty> bst;
};
using HotLDS = HotLDST<false>;

// EDGE: the strip's region wraps around the lattice rows (or sits within 4 columns of an edge); a
// template parameter so that the two draw forms are two code paths, not one if-converted stream.
// FR: replica batches of full-row lattices (Nx <= 128, Nx % 4 == 0): consecutive runs of
// tiles_per_rep workgroups serve one replica (its fields, descriptors, tables and statistics), one strip spans
// the whole row, its LDS columns ARE the lattice columns and neighbours wrap inside LDS; the paired draws hold
// because a row's first rank N/2 q is even -- unless the replica's choice blocks start on a buffered half-word
// (after an odd number of NumPy Lemire rejections in its chain): then the pairs would straddle rows and the
// replica draws unpaired (the EDGE form).  OBS: the inline observables fused into the row stores.
// PH: the optional counter-based mode (SURVEY.md 8(b) sv_rng mode 1): every draw is Philox4x32-10 of (global site,
// sweep, slot) -- no stream positions, row bases, jump tables or replays
// the launch's logical workgroup index: workgroups are dealt round-robin over the 8 XCDs, so each XCD gets a
// contiguous range of logical indices (neighbouring strips share an L2)
__device__ __forceinline__ int logical_block() {
    const int b = blockIdx.x, G = gridDim.x, per = G / 8, rem = G % 8;
    const int xcd = b & 7, k = b >> 3;
    return xcd * per + (xcd < rem ? xcd : rem) + k;
}

// BAND (villain_sweep_hot_band): one sweep of a multi-sweep launch -- the strip and the counted rows come from the
// caller, the LDS tables are filled only by the launch's first sweep, and no progress / cancellation checks
struct HotBand {
    int32_t ix, t0, t1;   // column strip and rows (lattice rows, may lie outside [0, Nt): they wrap)
    int32_t q_lo, q_hi;   // rows counted in the statistics (the band's own)
    bool first;           // the launch's first sweep: fill the LDS tables
    // the sweep's own descriptors, buffers, statistics slot and number (FArgs holds the launch's first sweep)
    const Block *blocks;
    const double *phi_in;
    const int64_t *n_in;
    double *phi_out;
    int64_t *n_out;
    sv_stats *stat;
    uint32_t sweep;
    int32_t j;            // the sweep's index within the launch (its statistics slot in LDS)
    int32_t tslot;        // SV_WGTIME: the (slot, sweep) record of g_bandtime
    // the workgroup's strip in the launch's next sweep (next_t0 < next_t1), or none: its row bases are jumped to at the
    // end of this sweep, so that the jumps' latency overlaps the last stores and the barrier
    int32_t next_t0, next_t1;
    const Block *next_blocks;
};

// SPLIT (villain_sweep_hot_split): the replay of a sweep that met NumPy Lemire rejections (at most one per choice block,
// two in all): a row of colour c draws choice block j from blocksB[2 + 5 c + j] (the descriptor after the block's
// switch) when the row lies after the switch (SplitSw::mask), else from blocks; the flags are per block (a fwd/bwd pair
// may sit at opposite pairing parities: fast_pack_g, hot_draws_edge<false, true>)
// ROWM (SPLIT): the strip's rows lie on both sides of a switch (the switch's row is among them, or they wrap around the
// torus): the mask is re-evaluated per row; otherwise it is the strip's constant.
template <bool TILE, bool EDGE, bool FR = false, bool OBS = false, bool PH = false, int NWT = 4, bool SKIP = false,
          bool BAND = false, bool SPLIT = false, bool ROWM = false>
__device__ __forceinline__ void hot_body(const FArgs &A, HotLDST<PH, FR && OBS, NWT> &Ls, int bl,
                                         const HotBand *hb = nullptr, const Block *blocksB = nullptr,
                                         const SplitSw *sw = nullptr) {
    static_assert(!SPLIT || (!FR && !PH && !SKIP && !BAND && NWT == 4), "split replays: single lattices and tiles");
    static_assert(!(FR && TILE), "full-row replica strips are periodic");
    static_assert(!SKIP || (EDGE && !FR && !PH), "skip lists: the unpaired (edge) draws of single lattices and tiles");
    static_assert(NWT == 4 || (NWT == 8 && !FR && !PH), "8-wave strips: single lattices and tiles");
    static_assert(!BAND || (!TILE && !FR && !PH && !SKIP), "band sweeps: periodic single lattices");
    constexpr int NW = NWT;
    constexpr int R = HotLDST<PH, FR && OBS, NWT>::R, RR = HotLDST<PH, FR && OBS, NWT>::RR;
    // rows move by 32-bit byte offsets from the uniform bases: the hosts keep every offset below 2^32 on this kernel
    // (run_fused: 16 V < 2^32; domain tiles: 16 plane < 2^32; replica batches address within one replica of N <= 128)
    constexpr bool OFF32 = !PH && !(SV_ABLATE & (16 | 256 | 512 | 8));
    constexpr int PF = RW / 64;
    auto &s_phi = Ls.phi;
    auto &s_r0 = Ls.r0;
    auto &s_r1 = Ls.r1;
    auto &s_n0 = Ls.n0;
    auto &s_n1 = Ls.n1;
    auto &s_small = Ls.small;
    auto &s_adv = Ls.adv;
    auto &s_base = Ls.base;
    int32_t &s_bad = Ls.bad;

    if constexpr (!PH && !BAND) note_progress(A);  // (FArgs::progress: the chunked enqueues of single lattices and replica batches)
    if (!BAND && sweep_cancelled(A.S, A.sweep)) return;
#if SV_WGTIME
    const uint64_t wg_t0 = rt_now();
#endif

    const FGeom &Gm = A.G;
    const int32_t Nt = Gm.Nt, Nx = Gm.Nx;
    const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)), lane = threadIdx.x & 63;
    const int64_t V = Gm.plane;
    auto grow = [&](int32_t q) { return wrapN(Gm.T0 + q, Nt); };
    auto mrow = [&](int32_t q) -> int64_t { return TILE ? Gm.org + (int64_t)q * Gm.pitch : (int64_t)wrapN(q, Nt) * Nx; };
    auto mcol = [&](int32_t c) -> int32_t { return TILE ? c : wrapN(c, Nx); };
    const int32_t par0 = (Gm.T0 + Gm.X0) & 1;

    int b = bl;
    const int slot = FR ? __builtin_amdgcn_readfirstlane(b / A.tiles_per_rep) : 0;  // uniform: keep it scalar
    if (FR) b = __builtin_amdgcn_readfirstlane(b - slot * A.tiles_per_rep);
    const int rep = FR && A.rep_map ? __builtin_amdgcn_readfirstlane(A.rep_map[slot]) : slot;
    const Block *blocks = BAND ? hb->blocks : (FR ? A.blocks + (int64_t)rep * A.rep_blocks : A.blocks);
    const JumpTables *Tb = FR ? A.Trep[rep] : A.T;
    const double *phi_in = BAND ? hb->phi_in : (FR ? A.phi_in + rep * A.rep_field : A.phi_in);
    const int64_t *n_in = BAND ? hb->n_in : (FR ? A.n_in + 2 * rep * A.rep_field : A.n_in);
    double *phi_out = BAND ? hb->phi_out : (FR ? A.phi_out + rep * A.rep_field : A.phi_out);
    int64_t *n_out = BAND ? hb->n_out : (FR ? A.n_out + 2 * rep * A.rep_field : A.n_out);
    const uint32_t sweep_id = BAND ? hb->sweep : A.sweep;
    int ix, t0s, t1s;
    if (BAND) {
        ix = hb->ix;
        t0s = hb->t0;
        t1s = hb->t1;
    } else if (!FR && A.strips) {
        ix = __builtin_amdgcn_readfirstlane(A.strips[3 * b]);
        t0s = __builtin_amdgcn_readfirstlane(A.strips[3 * b + 1]);
        t1s = __builtin_amdgcn_readfirstlane(A.strips[3 * b + 2]);
    } else {
        ix = b % A.nsx;
        t0s = (b / A.nsx) * A.TH;
        t1s = t0s + A.TH < Gm.Ht ? t0s + A.TH : Gm.Ht;
    }
    const int32_t x0 = (int32_t)((int64_t)ix * Gm.Wt / A.nsx), x1 = (int32_t)((int64_t)(ix + 1) * Gm.Wt / A.nsx);
    const int32_t w = x1 - x0;
    const int32_t t0 = t0s, t1 = t1s;
    // the sites this strip counts in the statistics (its own, within the launch's owned window)
    const int32_t q_lo = BAND ? (hb->q_lo > t0 ? hb->q_lo : t0) : (TILE && A.own_r0 > t0 ? A.own_r0 : t0);
    const int32_t q_hi = BAND ? (hb->q_hi < t1 ? hb->q_hi : t1) : (TILE && A.own_r1 < t1 ? A.own_r1 : t1);
    const int32_t c_lo = TILE && A.own_c0 > x0 ? A.own_c0 : x0, c_hi = TILE && A.own_c1 < x1 ? A.own_c1 : x1;
    // global column origin of this strip: its first column wrapped onto the torus, so that X0s + x stays within
    // [-2, Nx + 126) on the strip wherever the launch's region starts (deep-halo regions start anywhere)
    const int32_t X0s = TILE ? wrapN(Gm.X0 + x0, Nx) - x0 : Gm.X0;
    const int32_t rbase = t0 - 2;  // local row 0
    const int32_t cols = FR ? w : w + 5;
    const int32_t cofs = FR ? 0 : x0 - 2;   // LDS column of local column x is x - cofs
    // LDS neighbour columns (full rows wrap inside the row)
    auto cxp = [&](int cx) { return FR ? (cx + 1 == w ? 0 : cx + 1) : cx + 1; };
    auto cxm = [&](int cx) { return FR ? (cx == 0 ? w - 1 : cx - 1) : cx - 1; };
    const int32_t gx0 = X0s + x0;
    const bool interior = gx0 >= 4 && gx0 + w + 2 < Nx;
    const int32_t xb = (FR || (Nx <= SMALL_LDS && !interior) || gx0 - 2 < 0) ? 0 : gx0 - 2;
    constexpr bool edge = EDGE;
    (void)interior;
    const bool two_sets = edge && Nx > SMALL_LDS;   // wrapped columns need the second base set
    const int32_t xw = gx0 - 2 < 0 ? Nx - 2 : 0;

    if constexpr (!PH) {
        if (!BAND || hb->first) {
            for (int e = threadIdx.x; e < SMALL_LDS; e += NW * 64) {
                s_small.A[e] = Tb->small[e].A;
                s_small.C[e] = Tb->small[e].C;
            }
            if (threadIdx.x < 3) s_adv[threadIdx.x] = FR ? A.advrep[3 * rep + threadIdx.x] : A.adv[threadIdx.x];
        }
    }
    // POLL (single lattices): the abort flag is polled by wave 0 at the start and once per row step (an agent-scope
    // load: the reporting workgroup may sit on another XCD, whose L2 the plain loads do not see), and a workgroup leaves
    // the sweep as soon as it is set -- a sweep that met a rejection is discarded and replayed, so its remaining work
    // is waste.  The poll is issued just before the next rows' prefetch and read after their commit, so it adds no wait.
    constexpr bool POLL = !TILE && !FR && !BAND && !PH;
    int32_t pv = 0;
    if constexpr (POLL) {
        if (wave == 0) pv = __hip_atomic_load(A.S.abort, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (threadIdx.x == 0) s_bad = 0;
    if (POLL && threadIdx.x == 0) Ls.stop = 0;
    if (OBS && threadIdx.x < 5) Ls.obsw[threadIdx.x] = 0;
    if (OBS && threadIdx.x == 5) Ls.obig = 0.0;
    if constexpr (FR && OBS) {  // this lane's running sums (only this lane touches its slots)
        Ls.ol.act[threadIdx.x] = 0;
        Ls.ol.w2[threadIdx.x] = 0;
        Ls.ol.npk[threadIdx.x] = 0;
    }

    // per colour: the buffered-half flags and words of the choice blocks (equal within each fwd/bwd pair on
    // this kernel unless SKIP), uniform
    // (non-SKIP edge draws read has4[c][2 mu], the pair's common flag)
    uint32_t has_c[2][2], buf_c[2][4], has4[2][4];
    int32_t nsk[2][4];
#pragma unroll
    for (int c = 0; c < 2; c++) {
#pragma unroll
        for (int mu = 0; mu < 2; mu++)
            has_c[c][mu] = PH ? 0u : (uint32_t)__builtin_amdgcn_readfirstlane(blocks[2 + 5 * c + 2 * mu].has);
#pragma unroll
        for (int j = 0; j < 4; j++) {
            if constexpr (SKIP) {
                has4[c][j] = (uint32_t)__builtin_amdgcn_readfirstlane(blocks[2 + 5 * c + j].has);
                nsk[c][j] = __builtin_amdgcn_readfirstlane(blocks[2 + 5 * c + j].nskip);
            } else {
                has4[c][j] = has_c[c][j >> 1];
                nsk[c][j] = 0;
            }
        }
        if (edge) {
#pragma unroll
            for (int j = 0; j < 4; j++) buf_c[c][j] = (uint32_t)__builtin_amdgcn_readfirstlane(blocks[2 + 5 * c + j].buf);
        }
    }
    // SPLIT: each colour's current row mask (bit j: block j draws from blocksB) and those descriptors' flags
    uint32_t cur_m[2] = {0u, 0u};
    auto seg_load = [&](int c, uint32_t m) {
        cur_m[c] = m;
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const Block &Bd = ((m >> j) & 1u) ? blocksB[2 + 5 * c + j] : blocks[2 + 5 * c + j];
            has4[c][j] = (uint32_t)__builtin_amdgcn_readfirstlane(Bd.has);
            buf_c[c][j] = (uint32_t)__builtin_amdgcn_readfirstlane(Bd.buf);
        }
    };
    if constexpr (SPLIT) {
        seg_load(0, sw->mask(0, grow(t0s - 3 + 2 + wave)));
        seg_load(1, sw->mask(1, grow(t0s - 3 + 1 + wave)));
    }
    if constexpr (SKIP) {  // the skip lists into LDS (the host bounds them by HOT_MAXSK per block)
        if (threadIdx.x < 2 * 4 * HOT_MAXSK) {
            const int c = threadIdx.x / (4 * HOT_MAXSK), j = (threadIdx.x / HOT_MAXSK) & 3, i = threadIdx.x % HOT_MAXSK;
            const Block &B = blocks[2 + 5 * c + j];
            if constexpr (!(FR && OBS)) Ls.sk[c][j][i] = i < B.nskip ? A.skips[B.skip0 + i] : 0xFFFFFFFFu;
        }
    }
    const VParams P = A.P;
    const uint32_t kc = P.k, thr = P.thr;
    const int32_t Wn = (int32_t)P.W, nW = (int32_t)(P.W * P.interval_n);

    // ---- register prefetch of region rows [ra, ra+NW): wave w moves row ra + w, lane l columns l, l + 64
    double pf_phi[PF];
    int64_t pf_n0[PF], pf_n1[PF];
    int pf_gx[PF];
#pragma unroll
    for (int k = 0; k < PF; k++) pf_gx[k] = FR ? lane + 64 * k : mcol(x0 - 2 + lane + 64 * k);
    if (SV_ABLATE & 16) {
#pragma unroll
        for (int k = 0; k < PF; k++) pf_phi[k] = 0.0, pf_n0[k] = pf_n1[k] = 0;
    }
    auto prefetch = [&](int32_t ra) {
        if (SV_ABLATE & 16) return;
        const int32_t q = ra + wave;
        if (q >= t0 - 2 && q <= t1 + 2) {
            const int64_t g0 = mrow(q);
#pragma unroll
            for (int k = 0; k < PF; k++) {
                if (lane + 64 * k < cols) {
                    const int64_t g = g0 + pf_gx[k];
                    if (OFF32) {  // 32-bit byte offsets from the uniform bases (global_load's SGPR-base form)
                        const uint32_t o = ((uint32_t)g0 + (uint32_t)pf_gx[k]) * 8u;
                        pf_phi[k] = *(const double *)((const char *)phi_in + o);
                        pf_n0[k] = *(const int64_t *)((const char *)n_in + o);
                        pf_n1[k] = *(const int64_t *)((const char *)n_in + (o + (uint32_t)V * 8u));
                        continue;
                    }
                    pf_phi[k] = phi_in[g];
                    if (SV_ABLATE & 256) {  // timing experiment: a compact int32 n layout (cold start only)
                        pf_n0[k] = ((const int32_t *)n_in)[g];
                        pf_n1[k] = ((const int32_t *)n_in)[V + g];
                    } else if (SV_ABLATE & 512) {  // the same with int16
                        pf_n0[k] = ((const int16_t *)n_in)[g];
                        pf_n1[k] = ((const int16_t *)n_in)[V + g];
                    } else {
                        pf_n0[k] = n_in[g];
                        pf_n1[k] = n_in[V + g];
                    }
                }
            }
        }
    };
    auto commit = [&](int32_t ra) {
        const int32_t q = ra + wave;
        if (q >= t0 - 2 && q <= t1 + 2) {
            const int slot = (q - rbase) % R;
            uint32_t bad = 0;
#pragma unroll
            for (int k = 0; k < PF; k++) {
                const int cc = lane + 64 * k;
                if (cc < cols) {
                    // the +0.0 every site receives in one of the two colour passes (neighborhood.py:128),
                    // applied up front: the accepted change is added to the normalised value
                    s_phi[slot][cc] = pf_phi[k] + 0.0;
                    const int32_t a = (int32_t)pf_n0[k], c = (int32_t)pf_n1[k];
                    // the int32 image must hold n exactly, with headroom for one sweep's changes
                    constexpr int NB = 14;  // |n| < 2^NB, headroom for one sweep's 2|W| <= 2^13
                    bad |= (uint32_t)((uint64_t)((pf_n0[k] >> NB) + 1) > 1) | (uint32_t)((uint64_t)((pf_n1[k] >> NB) + 1) > 1);
                    s_n0[slot][cc] = a;
                    s_n1[slot][cc] = c;
                }
            }
            if (bad) s_bad = 1;
        }
    };

    // ---- per-wave running row bases: lane 8c+ty holds block ty's base for this wave's colour-c row
    // (at column xb); lanes 16 + 8c + ty the same at column xw (edge strips of rows longer than SMALL_LDS)
    const bool base_lane = !PH && (lane & 7) < 6 && (lane < 16 || (two_sets && lane < 32));
    const int bc = (lane >> 3) & 1, bty = lane & 7;
    const int32_t bx = lane >= 16 ? xw : xb;
    const int bblk = bty == 0 ? 0 : 1 + 5 * bc + bty - 1;
    const uint32_t bhas = (!PH && base_lane && bty >= 2) ? blocks[bblk].has : 0u;
    // SPLIT: this base lane's descriptor (blocks or blocksB) for a row
    auto bdsc = [&](int32_t row) -> const Block * {
        if constexpr (SPLIT) {
            const uint32_t m = ROWM ? (bc ? sw->mask(1, grow(row)) : sw->mask(0, grow(row))) : (bc ? cur_m[1] : cur_m[0]);
            if (bty >= 2 && ((m >> (bty - 2)) & 1u)) return &blocksB[bblk];
        }
        return &blocks[bblk];
    };
    const int32_t tfirst = t0 - 3;
    int32_t brow = tfirst + 2 - bc + wave;  // colour 0 row t+2+wave, colour 1 row t+1+wave
    int32_t brow1 = tfirst + 1 + wave;      // the colour-1 row, wave-uniform
    if constexpr (!PH) {  // (the running bases live in LDS only: the advance reads them back)
        if (!BAND || hb->first) {  // (a band sweep after the first: its predecessor jumped to them)
            u128 bases{0, 0};
            // (flat table loads: not in the replica kernels, whose registers they would push into scratch)
            if (SPLIT && base_lane) {
                const Block *d = bdsc(brow);
                bases = full_jump_flat(Tb, d, (uint32_t)base_pos(bty, grow(brow), Nx, bx, bty >= 2 ? d->has : 0u));
            } else if (base_lane)
                bases = FR ? full_jump(Tb, &blocks[bblk], (uint32_t)base_pos(bty, grow(brow), Nx, bx, bhas))
                           : full_jump_flat(Tb, &blocks[bblk], (uint32_t)base_pos(bty, grow(brow), Nx, bx, bhas));
            __builtin_amdgcn_s_waitcnt(0);
            if (base_lane) s_base[wave][lane] = bases;
        }
    }
#if SV_WGTIME
    const uint64_t wg_tb = rt_now();
#endif

    // paired-draw lane constants per colour (interior strips; valid for every row of this wave)
    uint32_t pk0 = 0, pk1 = 0;
    uint32_t mism0 = 0, mism1 = 0;  // SPLIT: mismatched directions (fast_pack_g)
    // SPLIT: the paired-draw constants of colour c for its row q (the row's flags)
    auto pack_g = [&](int c, int32_t q) {
        const int32_t xs = c == 0 ? (x0 - 1) + ((par0 + q + x0 - 1) & 1) : x0 + ((par0 + q + x0 + 1) & 1);
        uint32_t mm = 0;
        const uint32_t pk = fast_pack_g(has4[c], lane, (uint32_t)grow(q) * (uint32_t)Nx, (uint32_t)(X0s + xs),
                                        (uint32_t)(X0s + xs + 2 * lane), (uint32_t)xb, mm);
        if (c == 0) pk0 = pk, mism0 = mm;
        else pk1 = pk, mism1 = mm;
    };
    if constexpr (SPLIT && !edge) {
        pack_g(0, tfirst + 2 + wave);
        pack_g(1, tfirst + 1 + wave);
    } else if constexpr (!edge && !PH) {
        {
            const int32_t q = tfirst + 2 + wave;
            const int32_t xs = FR ? ((par0 + q) & 1) : (x0 - 1) + ((par0 + q + x0 - 1) & 1);
            pk0 = fast_pack(has_c[0], lane, (uint32_t)grow(q) * (uint32_t)Nx, (uint32_t)(X0s + xs),
                            (uint32_t)(X0s + xs + 2 * lane), (uint32_t)xb);
        }
        {
            const int32_t q = tfirst + 1 + wave;
            const int32_t xs = FR ? ((par0 + q + 1) & 1) : x0 + ((par0 + q + x0 + 1) & 1);
            pk1 = fast_pack(has_c[1], lane, (uint32_t)grow(q) * (uint32_t)Nx, (uint32_t)(X0s + xs),
                            (uint32_t)(X0s + xs + 2 * lane), (uint32_t)xb);
        }
    }

    int64_t acc_count = 0;
    AccFx psum;  // exact acceptance sum (common.h)

    auto store_rows = [&](int32_t ra) {
        if (SV_ABLATE & 8) return;
        const int32_t q = ra + wave;
        unsigned long long o_act = 0;  // OBS partials of this row step (exact action values, common.h)
        int64_t o_w2 = 0;
        int32_t o_n0 = 0, o_n1 = 0;
        if (q >= t0 && q < t1) {
            const int slot = (q - rbase) % R;
            const int64_t g0 = mrow(q) + x0;
#pragma unroll
            for (int k = 0; k < PF; k++) {
                const int cc = lane + 64 * k;
                if (cc < w) {
                    const int cx = FR ? cc : cc + 2;
                    const int64_t g = g0 + cc;
                    if (OFF32 && TILE && !BAND) {
                        // a domain tile (one short launch per sweep): write-through row stores (global_store sc1) leave
                        // no dirty L2 lines for the launch's end to write back (2048 x 1024 depth 4: 49.2 -> 47.8 us
                        // per sweep, r5); on the whole lattice (many rounds of strips) they measured slower, and level
                        // for only its last 256-1024 workgroups and for the replica batches (r5)
                        const uint32_t o = ((uint32_t)g0 + (uint32_t)cc) * 8u;
                        __hip_atomic_store((double *)((char *)phi_out + o), s_phi[slot][cx], __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
                        __hip_atomic_store((int64_t *)((char *)n_out + o), (int64_t)s_n0[slot][cx], __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
                        __hip_atomic_store((int64_t *)((char *)n_out + (o + (uint32_t)V * 8u)), (int64_t)s_n1[slot][cx],
                                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    } else if (OFF32) {
                        const uint32_t o = ((uint32_t)g0 + (uint32_t)cc) * 8u;
                        *(double *)((char *)phi_out + o) = s_phi[slot][cx];
                        *(int64_t *)((char *)n_out + o) = (int64_t)s_n0[slot][cx];
                        *(int64_t *)((char *)n_out + (o + (uint32_t)V * 8u)) = (int64_t)s_n1[slot][cx];
                    } else {
                    phi_out[g] = s_phi[slot][cx];
                    if (SV_ABLATE & 256) {
                        ((int32_t *)n_out)[g] = s_n0[slot][cx];
                        ((int32_t *)n_out)[V + g] = s_n1[slot][cx];
                    } else if (SV_ABLATE & 512) {
                        ((int16_t *)n_out)[g] = s_n0[slot][cx];
                        ((int16_t *)n_out)[V + g] = s_n1[slot][cx];
                    } else {
                        n_out[g] = (int64_t)s_n0[slot][cx];
                        n_out[V + g] = (int64_t)s_n1[slot][cx];
                    }
                    }
                    if (OBS) {
                        // rows <= q+1 and columns <= x+1 are final here (villain.py:51-66, winding.py:30-37,
                        // wrapping.py:17-25): link residuals, plaquette winding dn, holonomy sums
                        const int slot1 = (q + 1 - rbase) % R;
                        const double ph = s_phi[slot][cx];
                        const double l0 = (0.0 + (s_phi[slot1][cx] - ph)) - TWO_PI * (double)s_n0[slot][cx];
                        const double l1 = (0.0 + (s_phi[slot][cxp(cx)] - ph)) - TWO_PI * (double)s_n1[slot][cx];
                        const double t = l0 * l0 + l1 * l1;
                        if (__builtin_expect(t < ACT_LIMIT, 1)) o_act += act_fx(t);
                        else atomicAdd(&Ls.obig, t);
                        // |n| <= 2^15 on the int16 image, so |dn| < 2^17 fits int32 and dn^2 needs 64 bits
                        const int32_t dn = ((int32_t)s_n1[slot1][cx] - s_n1[slot][cx]) - ((int32_t)s_n0[slot][cxp(cx)] - s_n0[slot][cx]);
                        o_w2 += (int64_t)dn * dn;
                        o_n0 += s_n0[slot][cx];
                        o_n1 += s_n1[slot][cx];
                    }
                }
            }
        }
        if (OBS) {
            // this lane's running sums over the strip (LDS, no-return atomics; reduced once at the strip's end)
            if constexpr (FR && OBS) {
                atomicAdd(&Ls.ol.act[threadIdx.x], o_act);
                atomicAdd(&Ls.ol.w2[threadIdx.x], (unsigned long long)o_w2);
                atomicAdd(&Ls.ol.npk[threadIdx.x],
                          (unsigned long long)((int64_t)o_n0 + (int64_t)((uint64_t)(int64_t)o_n1 << 32)));
            }
        }
    };

    // draws of colour c for global row gq, local column x; the 4 choice values; a rejected word is reported
    auto draw = [&](int c, int32_t q, int32_t x, bool active, HotDraws &D, int32_t cn[4]) {
        const int32_t gq = grow(q);
        uint32_t spos[4] = {0, 0, 0, 0};  // SKIP: the choice draws' stream positions
        if constexpr (PH) {
            // site s of sweep `ph_sweep`: call (s, sweep, 0) -> u, dphi; call (s, sweep, 1) -> the four choice words; a
            // word Lemire rejects is replaced in place by word 0 of call (s, sweep, 2 + j + 4 t) (sv_oracle.c, philox)
            const uint32_t site = (uint32_t)gq * (uint32_t)Nx + (uint32_t)wrapN(X0s + x, Nx);
            const uint32_t s0 = (uint32_t)A.ph_sweep, s1 = (uint32_t)(A.ph_sweep >> 32);
            const uint32_t k0 = (uint32_t)A.ph_key, k1 = (uint32_t)(A.ph_key >> 32);
            const P4 a = philox4x32_10(P4{{site, s0, s1, 0u}}, k0, k1);
            const P4 b = philox4x32_10(P4{{site, s0, s1, 1u}}, k0, k1);
            D.u = u53(((uint64_t)a.v[1] << 32) | a.v[0]);
            D.dphi = A.P.lo_phi + A.P.range_phi * u53(((uint64_t)a.v[3] << 32) | a.v[2]);
#pragma unroll
            for (int j = 0; j < 4; j++) {
                uint64_t m = (uint64_t)b.v[j] * kc;
                for (uint32_t t = 0; __builtin_expect((uint32_t)m < thr, 0) && t < 64; t++)
                    m = (uint64_t)philox4x32_10(P4{{site, s0, s1, 2u + (uint32_t)j + 4u * t}}, k0, k1).v[0] * kc;
                cn[j] = (int32_t)(m >> 32) * Wn - nW;
            }
            (void)active;
            return;
        } else if constexpr (SPLIT) {
            if constexpr (ROWM) {
                const uint32_t m = sw->mask(c, gq);  // (wave-uniform)
                if (m != cur_m[c]) {                // the row crossed a switch: its descriptors and flags
                    seg_load(c, m);
                    if constexpr (!edge) pack_g(c, q);
                }
            }
            if constexpr (!edge)
                D = hot_draws_paired_g(A, lane, c == 0 ? pk0 : pk1, c == 0 ? mism0 : mism1, &s_base[wave][8 * c], s_small);
            else
                D = hot_draws_edge<false, true>(A, gq, wrapN(X0s + x, Nx), xb, two_sets ? xw : xb, &s_base[wave][8 * c],
                                                &s_base[wave][(two_sets ? 16 : 0) + 8 * c], s_small, has4[c], buf_c[c]);
        } else if constexpr (!edge) {
            D = hot_draws_paired_sel(A, lane, c == 0 ? pk0 : pk1, &s_base[wave][8 * c], s_small);
        } else {
            const uint32_t(*skl)[HOT_MAXSK] = nullptr;
            if constexpr (SKIP) skl = Ls.sk[c];
            D = hot_draws_edge<SKIP>(A, gq, wrapN(X0s + x, Nx), xb, two_sets ? xw : xb, &s_base[wave][8 * c],
                                     &s_base[wave][(two_sets ? 16 : 0) + 8 * c], s_small, has4[c], buf_c[c], skl,
                                     nsk[c], spos);
        }
        bool rej = false;
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const uint64_t m = (uint64_t)D.w[j] * kc;
            rej |= (uint32_t)m < thr;
            // W * (index - interval_n), neighborhood.py:105-107: one v_mad_i32_i24 (hot_ok bounds |W|, k < 2^20)
            cn[j] = (int32_t)(m >> 32) * Wn - nW;
        }
        if (__builtin_expect(rej && active && !(SV_ABLATE & 2), 0)) {
            const uint32_t rank = (uint32_t)(((int64_t)gq * Nx + wrapN(X0s + x, Nx)) >> 1);
#pragma unroll
            for (int j = 0; j < 4; j++)
                if ((uint32_t)((uint64_t)D.w[j] * kc) < thr)
                    report(A.S, sweep_id, (uint32_t)(1 + 5 * c + 1 + j), SKIP ? spos[j] : rank + (SPLIT ? ((cur_m[c] >> j) & 1u) : 0u),
                           (uint32_t)rep);
        }
    };

    for (int32_t ra = t0 - 2; ra < tfirst + 3 + NW; ra += NW) {
        prefetch(ra);
        commit(ra);
    }
    if constexpr (POLL) {
        if (wave == 0 && lane == 0 && pv) Ls.stop = 1;
    }
    __syncthreads();
    if constexpr (POLL) {
        if (Ls.stop) return;
    }
#if SV_WGTIME
    const uint64_t wg_t1 = rt_now();
#endif

    const double hk = P.half_kappa;
    prefetch(tfirst + 3 + NW);
    for (int32_t t = tfirst; t < t1; t += NW) {
        if constexpr (POLL) {
            if (Ls.stop) return;
        }
        store_rows(t - NW);
        // ---------------- colour 0 on row q = t+2+wave
        {
            const int32_t q = t + 2 + wave;
            const bool row_ok = (q >= t0 - 1) && (q <= t1 + 1);
            const int32_t xs = FR ? ((par0 + q) & 1) : (x0 - 1) + ((par0 + q + x0 - 1) & 1);
            const int32_t x = xs + 2 * lane;
            const bool active = row_ok && (FR ? x < w : x <= x1 + 1);
            HotDraws D;
            int32_t cn[4];
            draw(0, q, x, active, D, cn);
            if (active) {
                const int lr = q - rbase;
                const int sm = (lr - 1) % R, s0 = lr % R, sp = (lr + 1) % R;
                const int cx = x - cofs, cp = cxp(cx), cm = cxm(cx);
                const double ph = s_phi[s0][cx];
                int32_t n_f0 = s_n0[s0][cx], n_b0 = s_n0[sm][cx], n_f1 = s_n1[s0][cx], n_b1 = s_n1[s0][cm];
                // every later use takes the sign-extended value: ds_read_i16, no v_bfe_i32
                asm volatile("" : "+v"(n_f0), "+v"(n_b0), "+v"(n_f1), "+v"(n_b1));
                // r on the four links f0=(0,q,x), b0=(0,q-1,x), f1=(1,q,x), b1=(1,q,x-1) (neighborhood.py:91)
                double r0[4];
                r0[0] = (s_phi[sp][cx] - ph) - TWO_PI * (double)n_f0;
                r0[1] = (ph - s_phi[sm][cx]) - TWO_PI * (double)n_b0;
                r0[2] = (s_phi[s0][cp] - ph) - TWO_PI * (double)n_f1;
                r0[3] = (ph - s_phi[s0][cm]) - TWO_PI * (double)n_b1;
                double tc[4], cr[4];
#pragma unroll
                for (int k = 0; k < 4; k++) tc[k] = TWO_PI * (double)cn[k];
                const double mdp = 0.0 - D.dphi;  // d(change_phi) on a forward link, neighborhood.py:110
                cr[0] = mdp - tc[0];
                cr[1] = D.dphi - tc[1];
                cr[2] = mdp - tc[2];
                cr[3] = D.dphi - tc[3];
                double dS = (hk * cr[0]) * ((2.0 * r0[0]) + cr[0]);
#pragma unroll
                for (int k = 1; k < 4; k++) dS += (hk * cr[k]) * ((2.0 * r0[k]) + cr[k]);
                double p = sv_exp(-dS);
                p = p > 1.0 ? 1.0 : p;
                const bool acc = D.u < p;
                if (q >= q_lo && q < q_hi && (FR || (x >= c_lo && x < c_hi))) {
                    acc_count += acc;
                    fx_add(psum, p);
                }
                double wr[4] = {r0[0], r0[1], r0[2], r0[3]};
                if (__builtin_amdgcn_ballot_w64(acc)) {
                    if (acc) {
                        // neighborhood.py:124-129: phi += change_phi, n += change_n, r += d(change_phi) - 2 pi change_n
                        s_phi[s0][cx] = ph + D.dphi;
                        s_n0[s0][cx] = n_f0 + cn[0];
                        s_n0[sm][cx] = n_b0 + cn[1];
                        s_n1[s0][cx] = n_f1 + cn[2];
                        s_n1[s0][cm] = n_b1 + cn[3];
                        wr[0] = (r0[0] + mdp) - tc[0];
                        wr[1] = (r0[1] + D.dphi) - tc[1];
                        wr[2] = (r0[2] + mdp) - tc[2];
                        wr[3] = (r0[3] + D.dphi) - tc[3];
                    }
                }
                const int r0s = lr % RR, rms = (lr - 1) % RR;
                s_r0[r0s][cx] = wr[0];
                s_r0[rms][cx] = wr[1];
                s_r1[r0s][cx] = wr[2];
                s_r1[r0s][cm] = wr[3];
            }
        }
        if (!(SV_ABLATE & 32)) __syncthreads();
        // ---------------- colour 1 on row q = t+1+wave; rows t.. become final
        {
            const int32_t q = t + 1 + wave;
            const bool row_ok = (q >= t0) && (q <= t1);
            const int32_t xs = FR ? ((par0 + q + 1) & 1) : x0 + ((par0 + q + x0 + 1) & 1);
            const int32_t x = xs + 2 * lane;
            const bool active = row_ok && (FR ? x < w : x <= x1);
            HotDraws D;
            int32_t cn[4];
            draw(1, q, x, active, D, cn);
            if (active) {
                const int lr = q - rbase;
                const int sm = (lr - 1) % R, s0 = lr % R;
                const int cx = x - cofs, cm = cxm(cx);
                double ri[4];
                const int r0s = lr % RR, rms = (lr - 1) % RR;
                ri[0] = s_r0[r0s][cx];
                ri[1] = s_r0[rms][cx];
                ri[2] = s_r1[r0s][cx];
                ri[3] = s_r1[r0s][cm];
                double cr[4];
                const double mdp = 0.0 - D.dphi;
                cr[0] = mdp - TWO_PI * (double)cn[0];
                cr[1] = D.dphi - TWO_PI * (double)cn[1];
                cr[2] = mdp - TWO_PI * (double)cn[2];
                cr[3] = D.dphi - TWO_PI * (double)cn[3];
                double dS = (hk * cr[0]) * ((2.0 * ri[0]) + cr[0]);
#pragma unroll
                for (int k = 1; k < 4; k++) dS += (hk * cr[k]) * ((2.0 * ri[k]) + cr[k]);
                double p = sv_exp(-dS);
                p = p > 1.0 ? 1.0 : p;
                const bool acc = D.u < p;
                if (q >= q_lo && q < q_hi && (FR || (x >= c_lo && x < c_hi))) {
                    acc_count += acc;
                    fx_add(psum, p);
                }
                if (__builtin_amdgcn_ballot_w64(acc)) {
                    if (acc) {
                        s_phi[s0][cx] = s_phi[s0][cx] + D.dphi;
                        s_n0[s0][cx] += cn[0];
                        s_n0[sm][cx] += cn[1];
                        s_n1[s0][cx] += cn[2];
                        s_n1[s0][cm] += cn[3];
                    }
                }
            }
        }
        commit(t + 3 + NW);
        if constexpr (POLL) {
            if (wave == 0 && lane == 0 && pv) Ls.stop = 1;
            if (wave == 0) pv = __hip_atomic_load(A.S.abort, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (t + NW < t1) prefetch(t + 3 + 2 * NW);
        // The bases of the wave's two rows (brow1, brow1 + 1) move NW rows down.  Unless a row wraps around the
        // lattice or sits on global row 0 (where a buffered half-word clamps the word index), every block's
        // position moves by exactly its stride, so each base lane applies its precomputed advance map; the
        // wave-uniform test keeps the position arithmetic (64-bit, on every lane) off the common path.
        const int32_t glo = grow(brow1);
        brow1 += NW;
        if constexpr (PH) {
            // no row bases
        } else if (glo >= 1 && glo + NW + 1 < Nt && !(ROWM && sw->near(glo, NW + 2))) {
            if (base_lane) {
                const int ai = bty == 0 ? 0 : (bty == 1 ? 1 : 2);
                s_base[wave][lane] = mad128c(s_adv[ai].A, s_base[wave][lane], s_adv[ai].C);
            }
            brow += NW;
        } else if (base_lane) {
            // (SPLIT: a row that crosses a switch takes the other descriptor: a full jump)
            const Block *d_old = bdsc(brow), *d_new = bdsc(brow + NW);
            const uint32_t h_old = SPLIT ? (bty >= 2 ? d_old->has : 0u) : bhas, h_new = SPLIT ? (bty >= 2 ? d_new->has : 0u) : bhas;
            const int64_t p_old = base_pos(bty, grow(brow), Nx, bx, h_old);
            const int64_t p_new = base_pos(bty, grow(brow + NW), Nx, bx, h_new);
            const int ai = bty == 0 ? 0 : (bty == 1 ? 1 : 2);
            const int64_t step = bty == 0 ? (int64_t)NW * Nx : (bty == 1 ? (int64_t)NW * Nx / 2 : (int64_t)NW * Nx / 4);
            u128 bases = s_base[wave][lane];
            if (p_new - p_old == step && d_old == d_new) bases = apply(s_adv[ai], bases);
            else bases = full_jump(Tb, d_new, (uint32_t)p_new);
            brow += NW;
            s_base[wave][lane] = bases;
        } else {
            brow += NW;
        }
        if (!(SV_ABLATE & 32)) __syncthreads();
    }
#if SV_WGTIME
    const uint64_t wg_t2 = rt_now();
#endif
    {
        int32_t tl = tfirst;
        while (tl + NW < t1) tl += NW;
        store_rows(tl);
    }
    if constexpr (BAND) {
        // the next sweep's row bases (this wave's own LDS entries, free once its last row step is done)
        if (hb->next_t0 < hb->next_t1) {
            const int32_t nbrow = hb->next_t0 - 3 + 2 - bc + wave;
            const uint32_t nhas = (base_lane && bty >= 2) ? hb->next_blocks[bblk].has : 0u;
            u128 bases{0, 0};
            if (base_lane)
                bases = full_jump(Tb, &hb->next_blocks[bblk], (uint32_t)base_pos(bty, grow(nbrow), Nx, bx, nhas));
            if (base_lane) s_base[wave][lane] = bases;
        }
    }
    if (s_bad && threadIdx.x == 0) report(A.S, sweep_id, OVERFLOW_BLOCK, 0, (uint32_t)rep);
    if constexpr (BAND) {
        // into the workgroup's per-sweep slots (LDS); band_sweeps adds them to the sweeps' statistics at the end
        unsigned long long w[4];
        w[0] = (unsigned long long)acc_count;
        fx_limbs(psum, w[1], w[2], w[3]);
        for (int o = 32; o > 0; o >>= 1)
            for (int i = 0; i < 4; i++) w[i] += __shfl_xor(w[i], o);
        if (lane == 0)
            for (int i = 0; i < 4; i++) atomicAdd(&Ls.bst.w[hb->j][i], w[i]);
    } else {
        flush_stats<NWT>(FR ? A.stat + (int64_t)rep * A.rep_stat : A.stat, acc_count, psum);
    }
#if SV_WGTIME
    __builtin_amdgcn_s_waitcnt(0);
    if (BAND && threadIdx.x == 0 && hb->tslot >= 0 && hb->tslot < 8 * 128 * BT_SW) {
        uint64_t *o = g_bandtime + BT * (size_t)hb->tslot;
        o[0] = wg_t0;
        o[1] = wg_tb;
        o[2] = wg_t1;
        o[3] = wg_t2;
        o[4] = rt_now();
        o[6] = (uint64_t)(uint32_t)__builtin_amdgcn_s_getreg(4 | (31 << 11));
        o[7] = (uint64_t)(uint32_t)__builtin_amdgcn_s_getreg(20 | (31 << 11));
    } else if (!BAND && threadIdx.x == 0 && blockIdx.x < 65536) {
        uint64_t *o = g_wgtime + WGT * (size_t)blockIdx.x;
        o[0] = wg_t0;
        o[1] = wg_t1;
        o[2] = wg_t2;
        o[3] = rt_now();
        o[5] = wg_tb;
        // HW_ID (hwreg 4: wave, SIMD, CU, SH, SE) and XCC_ID (hwreg 20)
        o[4] = (uint64_t)(uint32_t)__builtin_amdgcn_s_getreg(4 | (31 << 11)) |
               ((uint64_t)(uint32_t)__builtin_amdgcn_s_getreg(20 | (31 << 11)) << 32);
    }
#endif
    if constexpr (FR && OBS) {
        // |sum n0|, |sum n1| <= 2 sites x 2^14 x strip rows < 2^31: the packed halves decode exactly
        const uint64_t pk = Ls.ol.npk[threadIdx.x];
        const int32_t a_n0 = (int32_t)(uint32_t)pk;
        const int64_t a_n1 = (int64_t)(pk - (uint64_t)(int64_t)a_n0) >> 32;
        const uint64_t q = Ls.ol.act[threadIdx.x];  // < 2^60: 2 sites x 128 rows of round(t 2^40) < 2^52
        // integer sums over the workgroup: the same words in any order (common.h)
        unsigned long long w[5] = {q & 0xffffffffull, q >> 32, Ls.ol.w2[threadIdx.x], (uint64_t)(int64_t)a_n0,
                                   (uint64_t)a_n1};
#pragma unroll
        for (int o = 32; o > 0; o >>= 1)
#pragma unroll
            for (int i = 0; i < 5; i++) w[i] += __shfl_xor(w[i], o);
        if (lane == 0)
#pragma unroll
            for (int i = 0; i < 5; i++) atomicAdd(&Ls.obsw[i], w[i]);
        __syncthreads();
        unsigned long long *ow = A.obs + (int64_t)rep * A.rep_obs;
        if (threadIdx.x < 5 && Ls.obsw[threadIdx.x]) atomicAdd(&ow[threadIdx.x], Ls.obsw[threadIdx.x]);
        if (threadIdx.x == 5 && Ls.obig != 0.0) unsafeAtomicAdd((double *)&ow[5], Ls.obig);
    }
}

template <bool TILE, int NWT>
__global__ __launch_bounds__(NWT * 64) __attribute__((amdgpu_waves_per_eu(4))) void villain_sweep_hot(FArgs A) {
    __shared__ HotLDST<false, false, NWT> Ls;
    // the strip this workgroup owns (the same mapping hot_body makes), to pick the body
    int b = blockIdx.x;
    {
        const int G = gridDim.x, per = G / 8, rem = G % 8;
        const int xcd = b & 7, k = b >> 3;
        b = xcd * per + (xcd < rem ? xcd : rem) + k;
    }
    const int ix = A.strips ? A.strips[3 * b] : b % A.nsx;
    const int bl = b;
    const int32_t x0 = (int32_t)((int64_t)ix * A.G.Wt / A.nsx), x1 = (int32_t)((int64_t)(ix + 1) * A.G.Wt / A.nsx);
    const int32_t gx0 = wrapN(A.G.X0 + x0, A.G.Nx);
    const bool interior = gx0 >= 4 && gx0 + (x1 - x0) + 2 < A.G.Nx;
    if (__builtin_amdgcn_readfirstlane((int)interior)) hot_body<TILE, false, false, false, false, NWT>(A, Ls, bl);
    else hot_body<TILE, true, false, false, false, NWT>(A, Ls, bl);
}


// The replay of a sweep that met NumPy Lemire rejections, at most one per choice block and two in all (single lattices
// and domain tiles): a strip whose rows all lie on one side of each block's switch runs the hot kernel's draws with one
// descriptor per block (paired on interior strips, a fwd/bwd pair at opposite pairing parities included), a strip
// whose rows contain a switch's row or wrap around the torus picks them per row, and the few strips whose columns
// straddle a switch's site run the skip-list body, moved to the head of their XCD's range.  A replay thus costs about
// one hot sweep instead of a general-kernel sweep (~1.9x).
template <bool TILE>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) void villain_sweep_hot_split(
    FArgs A, SplitArgs S) {
    __shared__ HotLDST<false, false, 4> Ls;
    // the skip-list strips run in their XCD's first-dispatched slots (SplitArgs::swap: slot -> strip where they differ)
    const int lb = logical_block();
    int b = lb;
    for (int i = 0; i < S.nswap; i++)
        if (lb == S.swap[i][0]) b = S.swap[i][1];
    int32_t tg0, tg1, xg0, xg1;  // the strip in global rows / columns
    split_strip(A.G, A.nsx, A.TH, A.strips, b, tg0, tg1, xg0, xg1);
    const bool interior = xg0 >= 4 && xg1 + 2 < A.G.Nx;
    bool straddle = false, rows = false;
    SplitSw sw;
    sw.qs[0] = sw.qs[1] = INT32_MAX;
    sw.blk[0] = sw.blk[1] = 0;
    sw.after = 0;
    int k = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        if (S.s[i] == 0xFFFFFFFFu || k >= 2) continue;
        bool after = false;
        straddle |= split_straddles(S.s[i], A.G.Nt, A.G.Nx, tg0, tg1, xg0, xg1, &sw.qs[k], &after);
        rows |= split_rows(sw.qs[k], A.G.Nt, tg0, tg1);
        sw.blk[k] = (uint32_t)i;
        sw.after |= (uint32_t)after << k;
        k++;
    }
    if (__builtin_amdgcn_readfirstlane((int)straddle))
        hot_body<TILE, true, false, false, false, 4, true>(A, Ls, b);
    else if (__builtin_amdgcn_readfirstlane((int)rows))
        hot_body<TILE, true, false, false, false, 4, false, false, true, true>(A, Ls, b, nullptr, S.blocksB, &sw);
    else if (__builtin_amdgcn_readfirstlane((int)interior))
        hot_body<TILE, false, false, false, false, 4, false, false, true>(A, Ls, b, nullptr, S.blocksB, &sw);
    else
        hot_body<TILE, true, false, false, false, 4, false, false, true>(A, Ls, b, nullptr, S.blocksB, &sw);
}
template __global__ void villain_sweep_hot_split<false>(FArgs, SplitArgs);
template __global__ void villain_sweep_hot_split<true>(FArgs, SplitArgs);

// ---- multi-sweep band launches of small periodic lattices (BandArgs, villain.h)
// The XCD-local barrier between two sweeps of a band: every wave's stores acknowledged by the L2, one arrival per
// workgroup, then a spin until the band's P workgroups have arrived.  Workgroup-scope atomics stay in the XCD's own L2,
// which every member of the band shares; nothing here crosses XCDs (the cross-XCD barrier of round 2 paid an L2
// write-back per workgroup and cost more than the launch it saved).  The next sweep's rows come from the L2 because
// no CU has them in its L1: sweep j reads buffer j, which this launch reads in no other sweep, and a launch starts with
// its L1s invalidated.  (The `buffer_inv sc0` below is a workgroup-scope invalidate and does NOT drop L1 lines
// -- measured, profiles/r06_xcd_barrier.txt: a re-read of a line after the first is stale; an L1-bypassing re-read
// costs nothing extra, `buffer_inv sc1` 1.7 us per barrier.)  1.0 us per barrier with 32 workgroups per XCD against
// 12.8 for the device-wide form (r6).  A barrier that has waited 20 ms (the band's workgroups not all resident)
// gives up.
__device__ __forceinline__ bool band_barrier(uint32_t *cnt, uint32_t target) {
    __shared__ int32_t s_ok;
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    if (threadIdx.x == 0) {
        __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        int ok = 1;
        for (;;) {
            // an agent-scope load misses the L1 and reads the L2 line the arrivals update; unlike a read-modify-write
            // it does not queue behind the other pollers in the L2's atomic unit (r4: CAS polling spread the barrier
            // passes of one band over ~4 us)
            const uint32_t v = __hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (v >= target) break;
            if (__builtin_amdgcn_s_memrealtime() - t0 > 2000000u) {  // 20 ms at 100 MHz
                ok = 0;
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
        asm volatile("buffer_inv sc0" ::: "memory");
        s_ok = ok;
    }
    __syncthreads();
    return s_ok != 0;
}

// workgroup i of a band: column strip i % nsx, row strip i / nsx of each sweep's region (the band's rows extended by
// 2e above and 3e below, e = K-1-j, cut into ceil(rows / TH) strips of at most TH rows; a row strip the shrinking
// region no longer has leaves the workgroup idle at the barriers)
template <bool EDGE, int NWT>
__device__ __forceinline__ void band_sweeps(const FArgs &A, const BandArgs &B, HotLDST<false, false, NWT> &Ls, int band,
                                            int i) {
    const int ix = i % A.nsx, r = i / A.nsx;
    uint32_t *bar = B.ctrl + BAND_CTRL * band + 32;
    // this workgroup's row strip of sweep j (empty when the shrinking region has no row strip r)
    auto strip = [&](int j, int32_t &t0, int32_t &t1) {
        const int32_t e = B.K - 1 - j, R0 = band * B.own - 2 * e, H = B.own + 5 * e, nr = (H + B.TH - 1) / B.TH;
        t0 = r < nr ? R0 + r * H / nr : 0;
        t1 = r < nr ? R0 + (r + 1) * H / nr : 0;
    };
    if (threadIdx.x < 16) {
        for (int i = 0; i < 4; i++) Ls.bst.w[threadIdx.x][i] = 0;
    }
    for (int j = 0; j < B.K; j++) {
        int32_t t0, t1, n0 = 0, n1 = 0;
        strip(j, t0, t1);
        if (j + 1 < B.K) strip(j + 1, n0, n1);
        if (t0 < t1) {
            const HotBand hb{ix, t0, t1, band * B.own, (band + 1) * B.own, j == 0,
                             A.blocks + (int64_t)j * B.nb, B.phi[j], B.n[j], B.phi[j + 1], B.n[j + 1], A.stat + j,
                             A.sweep + (uint32_t)j, j, (band * B.P + i) * 16 + j, n0, n1, A.blocks + (int64_t)(j + 1) * B.nb};
            hot_body<false, EDGE, false, false, false, NWT, false, true>(A, Ls, 0, &hb);
        }
        if (j + 1 < B.K && !band_barrier(bar, (uint32_t)((B.gen * (B.K - 1) + j + 1) * B.P))) {
            if (threadIdx.x == 0) report(A.S, A.sweep, BAND_FAIL_BLOCK, 0);
            return;
        }
#if SV_WGTIME
        if (threadIdx.x == 0 && (band * B.P + i) < 8 * 128) g_bandtime[BT * (size_t)((band * B.P + i) * BT_SW + j) + 5] = rt_now();
#endif
    }
    // the launch's statistics: one lane per sweep (integer sums: order-free, the acceptance words too)
    __syncthreads();
    if (threadIdx.x < 4 * B.K && Ls.bst.w[threadIdx.x >> 2][threadIdx.x & 3])
        atomicAdd(stat_word(&A.stat[threadIdx.x >> 2], threadIdx.x & 3), Ls.bst.w[threadIdx.x >> 2][threadIdx.x & 3]);
}

template <int NWT>
__global__ __launch_bounds__(NWT * 64) __attribute__((amdgpu_waves_per_eu(4))) void villain_sweep_hot_band(
    FArgs A, BandArgs B) {
    __shared__ HotLDST<false, false, NWT> Ls;
    __shared__ int32_t s_slot;
    note_progress(A);
    // run_fused gives band batches a gate: a launch skips only behind a sweep that reported, which this launch's own
    // reports (sweeps >= A.sweep) never are -- so every workgroup of the launch decides alike
    if (sweep_cancelled(A.S, A.sweep)) return;
    if (threadIdx.x == 0) {
        // the band is this workgroup's XCD; its place in the band, a ticket from that XCD's counter
        const uint32_t xcc = (uint32_t)__builtin_amdgcn_s_getreg(20 | (31 << 11)) & 0xFu;  // HW_REG_XCC_ID
        int32_t slot = -1;
        if ((int32_t)xcc < B.nbands) {
            const int32_t t = (int32_t)__hip_atomic_fetch_add(B.ctrl + BAND_CTRL * xcc, 1u, __ATOMIC_RELAXED,
                                                              __HIP_MEMORY_SCOPE_WORKGROUP) - B.gen * B.P;
            if (t >= 0 && t < B.P) slot = (int32_t)xcc * B.P + t;
        }
        s_slot = slot;
    }
    __syncthreads();
    const int slot = s_slot;
    if (slot < 0) {  // more workgroups on this XCD than the plan has places: some band stays short
        if (threadIdx.x == 0) report(A.S, A.sweep, BAND_FAIL_BLOCK, 0);
        return;
    }
    const int band = slot / B.P, i = slot % B.P, ix = i % A.nsx;
    const int32_t x0 = (int32_t)((int64_t)ix * A.G.Wt / A.nsx), x1 = (int32_t)((int64_t)(ix + 1) * A.G.Wt / A.nsx);
    const bool interior = x0 >= 4 && x1 + 2 < A.G.Nx;
    if (__builtin_amdgcn_readfirstlane((int)interior)) band_sweeps<false, NWT>(A, B, Ls, band, i);
    else band_sweeps<true, NWT>(A, B, Ls, band, i);
}
template __global__ void villain_sweep_hot_band<8>(FArgs, BandArgs);

template __global__ void villain_sweep_hot<false, 4>(FArgs);
template __global__ void villain_sweep_hot<true, 4>(FArgs);
template __global__ void villain_sweep_hot<false, 8>(FArgs);
template __global__ void villain_sweep_hot<true, 8>(FArgs);

// replica batches of full-row lattices (config 5), with or without the inline observables
template <bool OBS>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) void villain_sweep_hot_fr(FArgs A) {
    __shared__ HotLDST<false, OBS> Ls;
    // the replica this workgroup serves (the mapping hot_body makes), to pick the draw form
    int b = blockIdx.x;
    {
        const int G = gridDim.x, per = G / 8, rem = G % 8;
        const int xcd = b & 7, k = b >> 3;
        b = xcd * per + (xcd < rem ? xcd : rem) + k;
    }
    const int slot = b / A.tiles_per_rep;
    const Block *blk = A.blocks + (int64_t)(A.rep_map ? A.rep_map[slot] : slot) * A.rep_blocks;
    if (__builtin_amdgcn_readfirstlane((int)(blk[2].has | blk[4].has | blk[7].has | blk[9].has)))
        hot_body<false, true, true, OBS>(A, Ls, b);
    else
        hot_body<false, false, true, OBS>(A, Ls, b);
}
template __global__ void villain_sweep_hot_fr<false>(FArgs);
template __global__ void villain_sweep_hot_fr<true>(FArgs);

// the counter-based mode on a periodic single lattice (every strip draws the same way)
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) void villain_sweep_hot_ph(FArgs A) {
    __shared__ HotLDST<true> Ls;
    hot_body<false, false, false, false, true>(A, Ls, logical_block());
}

}  // namespace sv

#if SV_WGTIME
extern "C" int sv_debug_wgtime(uint64_t *out, int32_t n) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(sv::g_wgtime), (size_t)n * sv::WGT * sizeof(uint64_t)) == hipSuccess ? 0 : -2;
}
// g_bandtime: [slot][sweep < 16][8] (slot = band * P + i)
extern "C" int sv_debug_bandtime(uint64_t *out, int32_t slots) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(sv::g_bandtime), (size_t)slots * sv::BT_SW * sv::BT * sizeof(uint64_t)) == hipSuccess ? 0 : -2;
}
#endif

namespace svh {

// The hot kernel covers a sweep when its choice blocks carry no skip list and each fwd/bwd pair has equal
// buffered-half flags, and the choice values W (index - interval_n) fit int32
bool hot_params_ok(const VParams &P) {
    const int64_t aw = P.W < 0 ? -P.W : P.W;
    if (P.k <= 1 || P.k > (1u << 20) || aw > (1 << 20) || aw * (int64_t)P.k >= (1 << 28)) return false;  // int32 values
    // the int16 n image: a row enters LDS with |n| < 2^14 (else OVERFLOW is reported) and each link changes at most
    // twice per sweep (once per colour) by |W (index - interval_n)| <= |W| interval_n, so |W| interval_n <= 2^13 keeps
    // every value within int16
    if ((aw > (1 << 12) || aw * P.interval_n > (1 << 13))) return false;
    return true;
}

bool hot_ok(const VParams &P, const Block *blocks) {
    if (!hot_params_ok(P)) return false;
    for (int c = 0; c < 2; c++) {
        const Block *B = blocks + 2 + 5 * c;
        if (B[0].nskip || B[1].nskip || B[2].nskip || B[3].nskip) return false;
        if (B[0].has != B[1].has || B[2].has != B[3].has) return false;
    }
    return true;
}

// The split replay covers a sweep of the hot kernel's parameters whose choice blocks hold at most one known rejected
// position each; `S` receives each switch and the descriptor after it: a rejected half-word at stream position p moves
// every later draw of the block one half-word on, which for a block starting on a buffered half (has = 1) is the same
// words with has = 0, and otherwise the next word's stream with has = 1 and word 0's high half buffered
bool split_plan(const VParams &P, const Block *blocks, const uint32_t *skips, u128 inc, SplitArgs &S, Block *Bset) {
    if (!hot_params_ok(P)) return false;
    int nsw = 0;
    for (int i = 0; i < 11; i++) Bset[i] = blocks[i];
    for (int c = 0; c < 2; c++)
        for (int j = 0; j < 4; j++) {
            const Block &b = blocks[2 + 5 * c + j];
            Block &B = Bset[2 + 5 * c + j];
            B.nskip = 0;
            S.s[4 * c + j] = 0xFFFFFFFFu;
            if (b.nskip > 1) return false;
            if (b.nskip == 0) continue;
            if (++nsw > 2) return false;  // (SplitSw: at most two switches)
            S.s[4 * c + j] = skips[b.skip0];
            const u128 base{b.base_lo, b.base_hi};
            if (b.has) {
                B.has = 0;
            } else {
                const u128 nb = host_jump(base, inc, 1);
                B.base_lo = nb.lo;
                B.base_hi = nb.hi;
                B.has = 1;
                B.buf = (uint32_t)(xsl_rr(base) >> 32);
            }
        }
    return true;
}

void split_order(SplitArgs &S, const FGeom &G, int nsx, int TH, int grid, const int32_t *tab) {
    // logical blocks are dealt to the XCDs in contiguous ranges (logical_block), dispatched from the range's start; the
    // skip-list strips take the first slots of their own XCD's range and the strips there move to the slots they left,
    // so that the XCD's set of strips (its share of the work) is unchanged.  The result is a permutation of the slots,
    // sent as its non-identity entries (slot -> strip); a straddler already sitting in a head slot that another one is
    // sent to is moved along with it (r5: an earlier pairwise-swap form ran one strip twice and another not at all then).
    S.nswap = 0;
    const int per = grid / 8, rem = grid % 8;
    std::vector<int32_t> perm(grid), where(grid);  // slot -> strip, strip -> slot
    for (int b = 0; b < grid; b++) perm[b] = where[b] = b;
    int used[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int b = 0; b < grid; b++) {
        int32_t tg0, tg1, xg0, xg1;
        split_strip(G, nsx, TH, tab, b, tg0, tg1, xg0, xg1);
        bool st = false, after;
        int32_t qs;
        for (int i = 0; i < 8 && !st; i++)
            st = S.s[i] != 0xFFFFFFFFu && split_straddles(S.s[i], G.Nt, G.Nx, tg0, tg1, xg0, xg1, &qs, &after);
        if (!st) continue;
        int x = 0;
        while (x < 7 && b >= (x + 1) * per + std::min(x + 1, rem)) x++;
        const int a = x * per + std::min(x, rem) + used[x]++;  // the XCD's next head slot
        const int pb = where[b];                               // where strip b sits now
        if (pb == a) continue;
        const int sa = perm[a];
        perm[a] = b;
        where[b] = a;
        perm[pb] = sa;
        where[sa] = pb;
    }
    for (int s = 0; s < grid; s++) {
        if (perm[s] == s) continue;
        if (S.nswap == SPLIT_SWAPS) {  // (more than the table holds: the identity, the order only costs time)
            S.nswap = 0;
            return;
        }
        S.swap[S.nswap][0] = s;
        S.swap[S.nswap][1] = perm[s];
        S.nswap++;
    }
}

void launch_hot_split(const FArgs &A, const SplitArgs &S, int grid, hipStream_t stream) {
    const bool periodic =
        A.G.org == 0 && A.G.pitch == A.G.Nx && A.G.T0 == 0 && A.G.X0 == 0 && A.G.Ht == A.G.Nt && A.G.Wt == A.G.Nx;
    if (periodic) villain_sweep_hot_split<false><<<grid, 4 * 64, 0, stream>>>(A, S), SV_LAUNCHED("villain_sweep_hot_split<false>", stream);
    else villain_sweep_hot_split<true><<<grid, 4 * 64, 0, stream>>>(A, S), SV_LAUNCHED("villain_sweep_hot_split<true>", stream);
}

// replica batch of full-row lattices: N <= 128 columns (one strip), N % 4 == 0 (row ranks start on whole words)
bool hot_fr_ok(int32_t N) { return N <= RW && N % 4 == 0 && N >= 8; }

void launch_hot_fr(const FArgs &A, int grid, bool obs, hipStream_t stream) {
    if (obs) villain_sweep_hot_fr<true><<<grid, 4 * 64, 0, stream>>>(A), SV_LAUNCHED("villain_sweep_hot_fr<true>", stream);
    else villain_sweep_hot_fr<false><<<grid, 4 * 64, 0, stream>>>(A), SV_LAUNCHED("villain_sweep_hot_fr<false>", stream);
}

void launch_hot_ph(const FArgs &A, int grid, hipStream_t stream) { villain_sweep_hot_ph<<<grid, 4 * 64, 0, stream>>>(A), SV_LAUNCHED("villain_sweep_hot_ph", stream); }

void launch_hot_band(const FArgs &A, const BandArgs &B, hipStream_t stream) {
    villain_sweep_hot_band<8><<<B.nbands * B.P, 8 * 64, 0, stream>>>(A, B), SV_LAUNCHED("villain_sweep_hot_band<8>", stream);
}

int band_residency() {
    static const int n = [] {
        int v = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&v, villain_sweep_hot_band<8>, 8 * 64, 0) != hipSuccess) v = 0;
        return v;
    }();
    return n;
}

void launch_hot(const FArgs &A, int grid, hipStream_t stream) {
    const bool periodic =
        A.G.org == 0 && A.G.pitch == A.G.Nx && A.G.T0 == 0 && A.G.X0 == 0 && A.G.Ht == A.G.Nt && A.G.Wt == A.G.Nx;
    if (A.hot_nw == 8) {
        if (periodic) villain_sweep_hot<false, 8><<<grid, 8 * 64, 0, stream>>>(A), SV_LAUNCHED("villain_sweep_hot<false, 8>", stream);
        else villain_sweep_hot<true, 8><<<grid, 8 * 64, 0, stream>>>(A), SV_LAUNCHED("villain_sweep_hot<true, 8>", stream);
    } else if (periodic) {
        villain_sweep_hot<false, 4><<<grid, 4 * 64, 0, stream>>>(A), SV_LAUNCHED("villain_sweep_hot<false, 4>", stream);
    } else {
        villain_sweep_hot<true, 4><<<grid, 4 * 64, 0, stream>>>(A), SV_LAUNCHED("villain_sweep_hot<true, 4>", stream);
    }
}

}  // namespace svh
