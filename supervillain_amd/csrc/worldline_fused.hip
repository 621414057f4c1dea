// worldline_fused.hip -- BASELINE config 3's step in one launch: a checkerboard PlaquetteUpdate sweep (both
// colours, the GPU-native chain of worldline.hip: plaquette_cb_gs) followed by a CoexactUpdate sweep (both
// colours, coexact.py:53-128: coexact_gs), i.e. exactly what sv_worldline_plaquette_coexact_run launches as
// four colour passes, with the same per-plaquette arithmetic (bit-identical results).
//
// The four passes are plaquette-local checkerboard updates whose stencil reaches one row / column: a
// plaquette (t, x) reads and writes its four boundary links m0[t][x], m0[t][x+1], m1[t][x], m1[t+1][x] and
// reads v on (t, x) and its four neighbours (f = m - delta(v)/W).  So, as in villain_sweep_hot, a workgroup
// owns a column strip of <= 119 columns and streams down its rows with an LDS ring, each pass one row behind
// the one before it:  P0 on row t+3+w, P1 on t+2+w, C0 on t+1+w, C1 on t+w (wave w), a barrier between
// passes.  A strip stores the links of its own sites, which the plaquettes one row above and one column to
// the left also change, so C1 covers those halo plaquettes too and every earlier pass one more ring (P0 4
// rows/columns above/left of the strip and 3 below/right); every draw is addressed by its NumPy stream
// position, so neighbouring strips agree bit for bit.  The fields are read once and written once per step (m 16 B + v 8 B each way per
// plaquette) instead of four read-modify-write passes.
//
// Covered steps: even N, integer v, W a power of two (f and df exact as the pass kernels form them), no
// Lemire rejection known in the step's blocks and equal buffered-half flags in each colour's change_m /
// change_v pair; the host keeps the four pass kernels for the rest (worldline.hip).
#include "fused.h"

#ifndef SV_WFTIME
#define SV_WFTIME 0  // timing experiments: per-workgroup timestamps of worldline_step_fused (sv_debug_wftime)
#endif
namespace sv {

#if SV_WFTIME
// per launch slot: [wg][0..3] = entry, loop start, loop end, exit (s_memrealtime, 100 MHz), [4] = HW_ID | XCC_ID << 32,
// [5] = row bases ready (the layout of villain_hot.hip's g_wgtime)
__device__ uint64_t g_wftime[65536 * 6];
#endif

static constexpr int WF_W = 119;          // output columns per strip: region = WF_W + 9 <= RW
// NW waves = NW rows per step.  Ring rows: during step t the passes read rows t-1..t+NW+3 (C1 reads v[t-1], P0
// up to v[t+NW+3]) and the rows t+NW+4..t+2NW+3 that step t+NW's P0 needs are committed at its end, after C1,
// with no barrier between: 2 NW + 5 slots (NW = 4: the ring holds rows t-5..t+7, the next rows t+8..t+11 go
// into the slots of t-5..t-2, stored at the start of steps t-4 and t)
template <int NW>
struct WFGeom {
    static constexpr int R = 2 * NW + 5;
    static constexpr int AHEAD = NW + 4;  // step t prefetches (and commits) rows t + AHEAD ..
};

struct WFArgs {
    FGeom G;  // the periodic Nt x Nx lattice, or one domain tile with its ghost frame (villain.h)
    int32_t nsx, TH, nsy;
    // periodic lattices (16 waves): the column strips turned left by rot columns, so that strip 0 alone holds the
    // torus's column seam, in nsy_s row strips of ths rows (2 row steps: the seam strip's MODE 1 draws cost ~10% more
    // a row step); ths = 0: the plain layout (strip 0 at column 0, the last strip's region wrapping as well)
    int32_t rot, ths, nsy_s;
    // with the turned layout: the last interior row strip (fewer rows, and measured slowest) cut in two strips of
    // tail rows (2 row steps each); 0: not cut
    int32_t tail;
    const int64_t *m_in;
    const int64_t *v_in;
    int64_t *m_out;
    int64_t *v_out;
    const Block *blocks;  // 5 plaquette blocks ([0] metropolis, [1+2c] change_m, [2+2c] change_v), then 3 coexact
    Block blk[8];         // the same descriptors by value: the prologue's row-base jumps start one load earlier
    const uint32_t *skips;  // known rejected stream positions (GENERAL mode)
    const JumpTables *T;  // ([5] metropolis, [6+c] t)
    Affine adv[5];        // advance a row base by NW rows: [0] NW N draws, [2] NW N / 4 words; [3], [4]: the same
                          // across the torus's row seam (NW N - V draws, (NW N - V) / 4 words: inverse maps)
    StatStripe *pstat, *cstat;
    DevScratch S;
    uint32_t sweep;
    double Winv;  // 1 / W (W a power of two: x * Winv == x / W exactly)
    double c;     // 0.5 / kappa (coexact)
    double df[6], dfk[6];  // plaquette: df = cm - cv / W and df / kappa for index 3 jm + jv
    // plaquette acceptance table (WF_KP): Sigma = ((f1 + f2) - f3) - f4 = S unit with the integer
    // S = (m1 + m2 - m3 - m4) << sa + (vl + vu + vr + vd - 4 vc) << sb (unit = min(1, 1 / W)); ptab = 0: no table
    double unit;
    int32_t sa, sb, ptab;
    int32_t it;            // coexact: t in -it..-1, 1..it
    uint32_t kt, thrt;     // its choice count 2 it and Lemire threshold
    int32_t general;       // MODE 2 for every strip (wf_body)
};

// Column strip boundaries: uniform widths (narrower seam strips measured level, r4), turned left by rot (r5: the
// seam strip column then runs in short row strips instead)
__device__ __forceinline__ int32_t wf_xb(const WFArgs &A, int ix) {
    return (int32_t)((int64_t)ix * A.G.Wt / A.nsx) - A.rot;
}
// launch slot -> strip (column ix, rows [t0, t1)); slots are dealt to the XCDs in contiguous runs
__device__ __forceinline__ void wf_strip(const WFArgs &A, int &ix, int32_t &t0, int32_t &t1) {
    int b = blockIdx.x;
    {
        const int G = gridDim.x, per = G / 8, rem = G % 8;
        const int xcd = b & 7, k = b >> 3;
        b = xcd * per + (xcd < rem ? xcd : rem) + k;
    }
    int32_t th;
    if (A.ths) {
        const int ni = A.nsx - 1, ny = A.tail ? A.nsy - 1 : A.nsy;
        if (b < ni * ny) {
            ix = 1 + b % ni, th = A.TH, t0 = (b / ni) * th;
        } else if (b < ni * (ny + 2) && A.tail) {
            const int k = b - ni * ny;
            ix = 1 + k % ni, th = A.tail, t0 = ny * A.TH + (k / ni) * th;
        } else {
            ix = 0, th = A.ths, t0 = (b - ni * (A.tail ? ny + 2 : ny)) * th;
        }
    } else {
        ix = b % A.nsx, th = A.TH, t0 = (b / A.nsx) * th;
    }
    t1 = t0 + th < A.G.Ht ? t0 + th : A.G.Ht;
}

// The plaquette pass's acceptance min(1, exp(-dS)), dS = dfk ((((f1 + f2) - f3) - f4) + 2 df) (plaquette.py via
// plaquette_cb_gs), depends on the choice pair and on Sigma = ((f1 + f2) - f3) - f4 only, and Sigma is a small multiple
// of unit = min(1, 1 / W) held exactly (f = m - dv / W, W a power of two): for |S| <= WF_KP it is read from a table
// the prologue fills with the same expression (bit-identical), otherwise computed as before
static constexpr int WF_KP = 63, WF_PT = 2 * WF_KP + 1;

template <int NW>
struct WFLDS {
    static constexpr int R = WFGeom<NW>::R;
    double ptab[6 * WF_PT];
    int32_t m0[R][RW];
    int32_t m1[R][RW];
    int32_t v[R][RW];
    SmallTab small;
    Affine adv[5];
    u128 base[NW][64];  // per wave: lane 8p + ty = block ty's base for pass p's row at xb; 32 + .. at xw
    double df[6], dfk[6];
    int32_t bad;
};

// row-base stream position: uniform blocks by site, bounded blocks by u64 word of the colour rank
__device__ __forceinline__ int64_t wf_base_pos(bool bounded, int64_t gq, int64_t N, int64_t xb, uint32_t has) {
    const int64_t lin = gq * N + xb;
    if (!bounded) return lin;
    const int64_t p = (lin >> 1) - (int64_t)has;
    return p < 0 ? 0 : (p >> 1);
}

// delta(v)/W on a link from the two v values its difference takes (worldline.hip dvw_p): mu = 0:
// (double)(0 - (-diff)) / W, mu = 1: (double)(0 - diff) / W, with diff = v[s] - v[s - e_nu]
__device__ __forceinline__ double wf_dv0(int32_t vs, int32_t vn, double Winv) { return (double)(vs - vn) * Winv; }
__device__ __forceinline__ double wf_dv1(int32_t vs, int32_t vn, double Winv) { return (double)(-(vs - vn)) * Winv; }

// MODE 0: interior strip, paired plaquette words; 1: edge strip (rows wrap), unpaired words from two base sets;
// 2: GENERAL, a step with known Lemire rejections (skip lists) or unequal buffered-half flags: bounded words by
// a full table jump at their skip-adjusted stream position (the rare replay of a rejected step)
template <bool TILE, int MODE, int NW>
__device__ __forceinline__ void wf_body(const WFArgs &A, WFLDS<NW> &Ls) {
    constexpr bool EDGE = MODE != 0;
    constexpr int R = WFGeom<NW>::R, AH = WFGeom<NW>::AHEAD, PF = RW / 64;
    auto &s_m0 = Ls.m0;
    auto &s_m1 = Ls.m1;
    auto &s_v = Ls.v;
    auto &s_small = Ls.small;
    if (*(volatile const int32_t *)A.S.abort) return;
#if SV_WFTIME
    const uint64_t wf_t0 = __builtin_amdgcn_s_memrealtime();
#endif

    const FGeom &Gm = A.G;
    const int32_t N = Gm.Nx, Nt = Gm.Nt;  // global row length (stream layout) and row count
    const int64_t V = Gm.plane;
    const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)), lane = threadIdx.x & 63;
    int ix;
    int32_t t0, t1;
    wf_strip(A, ix, t0, t1);
    const int32_t x0 = wf_xb(A, ix), x1 = wf_xb(A, ix + 1);
    const int32_t w = x1 - x0;
    const int32_t rbase = t0 - 5;  // local row 0
    const int32_t cols = w + 9;
    const int32_t cofs = x0 - 5;   // LDS column of lattice column x is x - cofs
    auto grow = [&](int32_t q) { return wrapN(Gm.T0 + q, Nt); };   // global row of local row q
    auto gcol = [&](int32_t x) { return wrapN(Gm.X0 + x, N); };     // global column of local column x
    auto mrow = [&](int32_t q) -> int64_t { return TILE ? Gm.org + (int64_t)q * Gm.pitch : (int64_t)wrapN(q, Nt) * N; };
    auto mcol = [&](int32_t c) -> int32_t { return TILE ? c : wrapN(c, N); };
    // row bases at the strip's first region column (global), or at column 0 and at the first wrapped column
    const int32_t gx0 = Gm.X0 + x0;
    const int32_t xb = (N <= SMALL_LDS || gx0 - 5 < 0) ? 0 : gx0 - 5;
    const bool two_sets = EDGE && N > SMALL_LDS;
    const int32_t xw = gx0 - 5 < 0 ? N + gx0 - 5 : 0;  // (gx0 >= -N / 2)

    for (int e = threadIdx.x; e < SMALL_LDS; e += NW * 64) {
        s_small.A[e] = A.T->small[e].A;
        s_small.C[e] = A.T->small[e].C;
    }
    if (threadIdx.x < 5) Ls.adv[threadIdx.x] = A.adv[threadIdx.x];
    if (threadIdx.x < 6) {
        Ls.df[threadIdx.x] = A.df[threadIdx.x];
        Ls.dfk[threadIdx.x] = A.dfk[threadIdx.x];
    }
    if (threadIdx.x == 0) Ls.bad = 0;
    for (int e = threadIdx.x; e < 6 * WF_PT; e += NW * 64) {
        const int di = e / WF_PT, s = e % WF_PT - WF_KP;
        double df = A.df[0], dfk = A.dfk[0];  // (selects: no dynamically indexed kernel argument)
#pragma unroll
        for (int k = 1; k < 6; k++) {
            df = di == k ? A.df[k] : df;
            dfk = di == k ? A.dfk[k] : dfk;
        }
        const double dS = dfk * (((double)s * A.unit) + 2.0 * df);
        const double pr = sv_exp(-dS);
        Ls.ptab[e] = pr > 1.0 ? 1.0 : pr;
    }
    const double Winv = A.Winv, cc = A.c;
    const int32_t it = A.it;
    const uint32_t kt = A.kt, thrt = A.thrt;
    // buffered-half flags (uniform): plaquette colour c's change_m / change_v pair, coexact colour c's t block
    uint32_t hasp[2], bufp[2][2], hast[2], buft[2];
#pragma unroll
    for (int c = 0; c < 2; c++) {
        hasp[c] = A.blk[1 + 2 * c].has;
        bufp[c][0] = A.blk[1 + 2 * c].buf;
        bufp[c][1] = A.blk[2 + 2 * c].buf;
        hast[c] = A.blk[6 + c].has;
        buft[c] = A.blk[6 + c].buf;
    }

    // ---- register prefetch of region rows [ra, ra+NW): wave w moves row ra + w, lane l columns l, l + 64
    int64_t pf_m0[PF], pf_m1[PF], pf_v[PF];
    int pf_gx[PF];
#pragma unroll
    for (int k = 0; k < PF; k++) pf_gx[k] = mcol(x0 - 5 + lane + 64 * k);
    auto prefetch_to = [&](int32_t ra, int64_t(&pf_m0)[PF], int64_t(&pf_m1)[PF], int64_t(&pf_v)[PF]) {
        const int32_t q = ra + wave;
        if (SV_ABLATE & 16) {  // timing experiments only (fused.h SV_ABLATE): no HBM loads
#pragma unroll
            for (int k = 0; k < PF; k++) pf_m0[k] = pf_m1[k] = pf_v[k] = 0;
            return;
        }
        if (q >= t0 - 5 && q < t1 + 4) {
            const int64_t g0 = mrow(q);
#pragma unroll
            for (int k = 0; k < PF; k++) {
                if (lane + 64 * k < cols) {
                    // 32-bit byte offsets from the uniform bases (global_load's SGPR-base form; launch_wf keeps
                    // 16 plane < 2^32)
                    const uint32_t o = ((uint32_t)g0 + (uint32_t)pf_gx[k]) * 8u;
                    pf_m0[k] = *(const int64_t *)((const char *)A.m_in + o);
                    pf_m1[k] = *(const int64_t *)((const char *)A.m_in + (o + (uint32_t)V * 8u));
                    pf_v[k] = *(const int64_t *)((const char *)A.v_in + o);
                }
            }
        }
    };
    auto prefetch = [&](int32_t ra) { prefetch_to(ra, pf_m0, pf_m1, pf_v); };
    auto commit_from = [&](int32_t ra, const int64_t(&pf_m0)[PF], const int64_t(&pf_m1)[PF], const int64_t(&pf_v)[PF]) {
        const int32_t q = ra + wave;
        if (q >= t0 - 5 && q < t1 + 4) {
            const int slot = (q - rbase) % R;
            uint32_t bad = 0;
#pragma unroll
            for (int k = 0; k < PF; k++) {
                const int cx = lane + 64 * k;
                if (cx < cols) {
                    // the int32 image must hold the fields exactly, with headroom for one step's changes: -2^30 <= x
                    // < 2^30, as one 64-bit add and one unsigned compare
                    constexpr uint64_t H = uint64_t(1) << 30;
                    bad |= (uint32_t)((uint64_t)pf_m0[k] + H >= 2 * H) | (uint32_t)((uint64_t)pf_m1[k] + H >= 2 * H) |
                           (uint32_t)((uint64_t)pf_v[k] + H >= 2 * H);
                    s_m0[slot][cx] = (int32_t)pf_m0[k];
                    s_m1[slot][cx] = (int32_t)pf_m1[k];
                    s_v[slot][cx] = (int32_t)pf_v[k];
                }
            }
            if (bad) Ls.bad = 1;
        }
    };
    auto commit = [&](int32_t ra) { commit_from(ra, pf_m0, pf_m1, pf_v); };
    auto store_rows = [&](int32_t ra) {
        const int32_t q = ra + wave;
        if (SV_ABLATE & 8) return;  // timing experiments only: no HBM stores
        if (q >= t0 && q < t1) {
            const int slot = (q - rbase) % R;
            // own sites wrap only in the turned layout's seam strip (x0 < 0): column x0 + cc2 is the load column
            // pf_gx[k] five on, wrapped (periodic lattices; a tile's own columns never wrap)
            const int64_t g0 = TILE ? mrow(q) + x0 : mrow(q);
#pragma unroll
            for (int k = 0; k < PF; k++) {
                const int cc2 = lane + 64 * k;
                if (cc2 < w) {
                    if constexpr (!TILE) {
                        const uint32_t c = (uint32_t)pf_gx[k] + 5u, cw = c >= (uint32_t)N ? c - (uint32_t)N : c;
                        const uint32_t o = ((uint32_t)g0 + cw) * 8u;
                        // write-through (global_store sc1: agent-scope relaxed atomic stores): no dirty lines left
                        // in the XCD's L2 for the kernel's end to write back (-2.1 us a step at L=1024, r5)
                        __hip_atomic_store((int64_t *)((char *)A.m_out + o), (int64_t)s_m0[slot][cc2 + 5], __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
                        __hip_atomic_store((int64_t *)((char *)A.m_out + (o + (uint32_t)V * 8u)), (int64_t)s_m1[slot][cc2 + 5],
                                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        __hip_atomic_store((int64_t *)((char *)A.v_out + o), (int64_t)s_v[slot][cc2 + 5], __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
                        continue;
                    }
                    const uint32_t o = ((uint32_t)g0 + (uint32_t)cc2) * 8u;  // (a tile: write-through as well)
                    __hip_atomic_store((int64_t *)((char *)A.m_out + o), (int64_t)s_m0[slot][cc2 + 5], __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
                    __hip_atomic_store((int64_t *)((char *)A.m_out + (o + (uint32_t)V * 8u)), (int64_t)s_m1[slot][cc2 + 5],
                                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    __hip_atomic_store((int64_t *)((char *)A.v_out + o), (int64_t)s_v[slot][cc2 + 5], __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
                }
            }
        }
    };

    // ---- per-wave running row bases.  Pass p (0: plaquette colour 0, 1: plaquette colour 1, 2: coexact
    // colour 0, 3: coexact colour 1) works on row t + 3 - p + wave; block types ty: plaquette 0 metropolis,
    // 1 change_m, 2 change_v; coexact 0 metropolis, 1 t.
    const int bp = (lane >> 3) & 3, bty = lane & 7;
    const bool base_lane = bty < (bp < 2 ? 3 : 2) && (lane < 32 || (two_sets && lane < 64));
    const int32_t bx = lane >= 32 ? xw : xb;
    const int bblk = bp < 2 ? (bty == 0 ? 0 : bty + 2 * bp) : (bty == 0 ? 5 : 6 + (bp - 2));
    const bool bbnd = bty != 0;
    Block kb;  // this lane's descriptor (selects: no dynamically indexed kernel argument)
    {
        uint64_t lo = A.blk[0].base_lo, hi = A.blk[0].base_hi;
        uint32_t h = A.blk[0].has;
#pragma unroll
        for (int k = 1; k < 8; k++) {
            lo = bblk == k ? A.blk[k].base_lo : lo;
            hi = bblk == k ? A.blk[k].base_hi : hi;
            h = bblk == k ? A.blk[k].has : h;
        }
        kb.base_lo = lo, kb.base_hi = hi, kb.has = h, kb.buf = 0, kb.nskip = 0, kb.skip0 = 0;
    }
    const uint32_t bhas = (base_lane && bbnd) ? kb.has : 0u;
    const int32_t tfirst = t0 - 7;
    int32_t brow = tfirst + 3 - bp + wave;
    u128 bases{0, 0};
    prefetch(t0 - 5);  // the first region rows in flight while the row bases are jumped to
    if (base_lane) bases = full_jump_flat(A.T, &kb, (uint32_t)wf_base_pos(bbnd, grow(brow), N, bx, bhas));
    __builtin_amdgcn_s_waitcnt(0);
    if (base_lane) Ls.base[wave][lane] = bases;
#if SV_WFTIME
    const uint64_t wf_tb = __builtin_amdgcn_s_memrealtime();
#endif

    // the first column of pass p's colour on row q: pass p covers rows [t0 - 4 + p, t1 + 3 - p) and columns
    // [x0 - 4 + p, x1 + 3 - p): the links a strip stores are also changed by the plaquettes one row above and
    // one column left of it, so even the last pass (C1) covers those, and each earlier pass one more ring
    auto first_col = [&](int p, int32_t q) {
        const int32_t lo = x0 - (4 - p);
        const int c = p & 1;
        return lo + ((grow(q) + gcol(lo) + c) & 1);  // global (t + x) % 2 == c (N even)
    };
    // interior strips: per-lane constants of the paired plaquette draws (metropolis offset, change_m/change_v
    // word offset, half), the same for every row of the wave (rows advance 4 at a time)
    uint32_t pk[2] = {0, 0};
    if constexpr (!EDGE) {
#pragma unroll
        for (int p = 0; p < 2; p++) {
            const int32_t q = tfirst + 3 - p + wave;
            const uint32_t rowlin = (uint32_t)grow(q) * (uint32_t)N;
            const int32_t xs = first_col(p, q);
            const uint32_t gx = (uint32_t)(Gm.X0 + xs + 2 * lane);
            const uint32_t rank = (rowlin + gx) >> 1, R0 = (rowlin + (uint32_t)(Gm.X0 + xs)) >> 1;
            const uint32_t h = hasp[p], PR = (rowlin + (uint32_t)xb) >> 1;
            const uint32_t P = (R0 - h) & 1u, PW = (PR - h) >> 1;
            uint32_t qq = rank - h;
            if (lane == 63 && P) qq = R0 - h;  // lane 63 serves lane 0's word
            const uint32_t half = (lane == 63 && P) ? 0u : (qq & 1u);
            pk[p] = ((gx - (uint32_t)xb) & (SMALL_LDS - 1)) | ((((qq >> 1) - PW) & (SMALL_LDS - 1)) << 7) | (half << 14);
        }
    }

    int32_t pacc = 0, cacc = 0;  // (a lane's counts stay below 2^11)
    AccFx ppsum, cpsum;          // exact acceptance sums (common.h)

    // uniform draw and bounded word at stream offsets of row q's base (set A or, for wrapped columns, set B)
    auto draw_u = [&](const u128 &base, uint32_t off) { return u53(xsl_rr(hot_apply(s_small, off & (SMALL_LDS - 1), base))); };
    // (32-bit positions: launch_wf keeps V < 2^31, so ranks and word indices fit int32)
    auto word_at = [&](const u128 &base, int32_t rank, uint32_t has, uint32_t buf, int32_t rb) {
        const int32_t qq = rank - (int32_t)has;
        const int32_t w0 = (rb - (int32_t)has) < 0 ? 0 : ((rb - (int32_t)has) >> 1);
        const uint64_t X = xsl_rr(hot_apply(s_small, (uint32_t)((qq < 0 ? 0 : (qq >> 1)) - w0) & (SMALL_LDS - 1), base));
        uint32_t word = (qq & 1) ? (uint32_t)(X >> 32) : (uint32_t)X;
        return qq < 0 ? buf : word;
    };

    // ---------------- plaquette pass (colour c = p) on row q
    auto plaquette = [&](int p, int32_t q) {
        const int c = p;
        const bool row_ok = q >= t0 - (4 - p) && q < t1 + (3 - p);
        const int32_t x = first_col(p, q) + 2 * lane;
        const bool active = row_ok && x < x1 + (3 - p);
        const int32_t gq = grow(q), gx = gcol(x);
        const u128 *bs = &Ls.base[wave][8 * p];
        double u;
        uint32_t wm, wv;
        uint32_t qm = ((uint32_t)gq * (uint32_t)N + (uint32_t)gx) >> 1, qv = qm;  // stream positions (skip-adjusted)
        (void)qm;
        if constexpr (!EDGE) {
            u = draw_u(bs[0], pk[p]);
            const uint32_t half = (pk[p] >> 14) & 1u;
            const uint64_t X = xsl_rr(hot_apply(s_small, (pk[p] >> 7) & (SMALL_LDS - 1), half ? bs[2] : bs[1]));
            // lo lanes computed the change_m word (send its high half), hi lanes the change_v word
            const uint32_t send = half ? (uint32_t)X : (uint32_t)(X >> 32);
            const uint32_t got = pair_exchange(send, half, lane);
            wm = half ? got : (uint32_t)X;
            wv = half ? (uint32_t)(X >> 32) : got;
        } else {
            const bool wr = two_sets && !(gx >= xb && gx < xb + SMALL_LDS);
            const int32_t xr = wr ? xw : xb;
            const u128 *bb = wr ? &Ls.base[wave][32 + 8 * p] : bs;
            const int32_t rank = (int32_t)(((uint32_t)gq * (uint32_t)N + (uint32_t)gx) >> 1);
            const int32_t rb = (int32_t)(((uint32_t)gq * (uint32_t)N + (uint32_t)xr) >> 1);
            u = draw_u(bb[0], (uint32_t)(gx - xr));
            if constexpr (MODE == 2) {
                qm = skip_pos(A.blocks[1 + 2 * c], A.skips, (uint32_t)rank);
                qv = skip_pos(A.blocks[2 + 2 * c], A.skips, (uint32_t)rank);
                wm = bounded_word(A.T, A.blocks[1 + 2 * c], qm);
                wv = bounded_word(A.T, A.blocks[2 + 2 * c], qv);
            } else {
                wm = word_at(bb[1], rank, hasp[c], bufp[c][0], rb);
                wv = word_at(bb[2], rank, hasp[c], bufp[c][1], rb);
            }
        }
        const uint32_t jm = (uint32_t)(((uint64_t)wm * 2u) >> 32);       // choice((-1, 1)): threshold 0
        const uint64_t mv = (uint64_t)wv * 3u;                           // choice((-1, 0, 1)): threshold 1
        const uint32_t jv = (uint32_t)(mv >> 32);
        if (__builtin_expect((uint32_t)mv == 0u && active, 0)) report(A.S, A.sweep, (uint32_t)(2 + 2 * c), qv);
        if (active) {
            const int lr = q - rbase;
            const int sm = (lr - 1) % R, s0 = lr % R, sp = (lr + 1) % R;
            const int cx = x - cofs;
            const int32_t vc = s_v[s0][cx];
            // plaquette_cb_gs: f1 (0,q,x), f2 (1,q+1,x), f3 (0,q,x+1), f4 (1,q,x)
            const int32_t m_1 = s_m0[s0][cx], m_2 = s_m1[sp][cx], m_3 = s_m0[s0][cx + 1], m_4 = s_m1[s0][cx];
            const int32_t vl = s_v[s0][cx - 1], vu = s_v[sp][cx], vr = s_v[s0][cx + 1], vd = s_v[sm][cx];
            const int di = 3 * (int)jm + (int)jv;
            // (the int32 image bounds |m|, |v| < 2^30: the pair sums fit int32, the rest is 64-bit)
            const int64_t S = (((int64_t)(m_1 + m_2) - (int64_t)(m_3 + m_4)) << A.sa) +
                              (((int64_t)(vl + vu) + (int64_t)(vr + vd) - 4 * (int64_t)vc) << A.sb);
            double pr;
            if (A.ptab && (uint64_t)(S + WF_KP) < (uint64_t)WF_PT) {
                pr = Ls.ptab[di * WF_PT + (int)S + WF_KP];
            } else {
                const double f1 = (double)m_1 - wf_dv0(vc, vl, Winv);
                const double f2 = (double)m_2 - wf_dv1(vu, vc, Winv);
                const double f3 = (double)m_3 - wf_dv0(vr, vc, Winv);
                const double f4 = (double)m_4 - wf_dv1(vc, vd, Winv);
                const double df = Ls.df[di], dfk = Ls.dfk[di];
                const double dS = dfk * ((((f1 + f2) - f3) - f4) + 2.0 * df);
                pr = sv_exp(-dS);
                pr = pr > 1.0 ? 1.0 : pr;
            }
            const bool acc = u < pr;
            if (q >= t0 && q < t1 && x >= x0 && x < x1) {
                pacc += acc;
                fx_add(ppsum, pr);
            }
            if (__builtin_amdgcn_ballot_w64(acc)) {
                if (acc) {
                    const int32_t cm = jm ? 1 : -1, cv = (int32_t)jv - 1;
                    s_m0[s0][cx] = m_1 + cm;
                    s_m1[sp][cx] = m_2 + cm;
                    s_m0[s0][cx + 1] = m_3 - cm;
                    s_m1[s0][cx] = m_4 - cm;
                    s_v[s0][cx] = vc + cv;
                }
            }
        }
    };

    // ---------------- coexact pass (colour c = p - 2) on row q
    auto coexact = [&](int p, int32_t q) {
        const int c = p - 2;
        const bool row_ok = q >= t0 - (4 - p) && q < t1 + (3 - p);
        const int32_t x = first_col(p, q) + 2 * lane;
        const bool active = row_ok && x < x1 + (3 - p);
        const int32_t gq = grow(q), gx = gcol(x);
        const bool wr = two_sets && !(gx >= xb && gx < xb + SMALL_LDS);
        const int32_t xr = wr ? xw : xb;
        const u128 *bb = wr ? &Ls.base[wave][32 + 8 * p] : &Ls.base[wave][8 * p];
        const int32_t rank = (int32_t)(((uint32_t)gq * (uint32_t)N + (uint32_t)gx) >> 1);
        const int32_t rb = (int32_t)(((uint32_t)gq * (uint32_t)N + (uint32_t)xr) >> 1);
        const double u = draw_u(bb[0], (uint32_t)(gx - xr));
        uint32_t qt = (uint32_t)rank, wt;
        if constexpr (MODE == 2) {
            qt = skip_pos(A.blocks[6 + c], A.skips, (uint32_t)rank);
            wt = bounded_word(A.T, A.blocks[6 + c], qt);
        } else {
            wt = word_at(bb[1], rank, hast[c], buft[c], rb);
        }
        const uint64_t mt = (uint64_t)wt * kt;
        const int32_t j = (int32_t)(mt >> 32);
        if (__builtin_expect((uint32_t)mt < thrt && active, 0)) report(A.S, A.sweep, (uint32_t)(6 + c), qt);
        if (active) {
            const int32_t t = j < it ? j - it : j - it + 1;
            const int lr = q - rbase;
            const int sm = (lr - 1) % R, s0 = lr % R, sp = (lr + 1) % R;
            const int cx = x - cofs;
            const int32_t vc = s_v[s0][cx];
            // coexact_gs, coface_sum_at order: (1,q,x) -t, (1,q+1,x) +t, (0,q,x) +t, (0,q,x+1) -t
            const int32_t m_a = s_m1[s0][cx], m_b = s_m1[sp][cx], m_c = s_m0[s0][cx], m_d = s_m0[s0][cx + 1];
            const double fa = (double)m_a - wf_dv1(vc, s_v[sm][cx], Winv);
            const double fb = (double)m_b - wf_dv1(s_v[sp][cx], vc, Winv);
            const double fc = (double)m_c - wf_dv0(vc, s_v[s0][cx - 1], Winv);
            const double fd = (double)m_d - wf_dv0(s_v[s0][cx + 1], vc, Winv);
            const double tp = (double)t, tm = (double)(-t);
            double dS = (cc * tm) * ((2.0 * fa) + tm);
            dS += (cc * tp) * ((2.0 * fb) + tp);
            dS += (cc * tp) * ((2.0 * fc) + tp);
            dS += (cc * tm) * ((2.0 * fd) + tm);
            double pr = sv_exp(-dS);
            pr = pr > 1.0 ? 1.0 : pr;
            const bool acc = u < pr;
            if (q >= t0 && q < t1 && x >= x0 && x < x1) {
                cacc += acc;
                fx_add(cpsum, pr);
            }
            if (__builtin_amdgcn_ballot_w64(acc)) {
                if (acc) {  // delta_sparse(t accepted): m0[x] += t, m0[x+e1] -= t, m1[x] -= t, m1[x+e0] += t
                    s_m0[s0][cx] = m_c + t;
                    s_m0[s0][cx + 1] = m_d - t;
                    s_m1[s0][cx] = m_a - t;
                    s_m1[sp][cx] = m_b + t;
                }
            }
        }
    };

    for (int32_t ra = t0 - 5; ra < tfirst + AH; ra += NW) {
        if (ra != t0 - 5) prefetch(ra);
        commit(ra);
    }
    __syncthreads();
#if SV_WFTIME
    const uint64_t wf_t1 = __builtin_amdgcn_s_memrealtime();
#endif

    for (int32_t t = tfirst; t < t1; t += NW) {
        prefetch(t + AH);
        store_rows(t - NW);
        plaquette(0, t + 3 + wave);
        __syncthreads();
        plaquette(1, t + 2 + wave);
        __syncthreads();
        coexact(2, t + 1 + wave);
        __syncthreads();
        coexact(3, t + wave);
        commit(t + AH);
        // The wave's four rows (t + wave .. t + 3 + wave) move NW rows down.  Unless one of them wraps around the
        // lattice or sits on global row 0 (where a buffered half-word clamps the word index), every block's position
        // moves by exactly its stride: one precomputed map per base lane (as villain_hot.hip's), the
        // position arithmetic kept off the common path by a wave-uniform test.
        const int32_t glo = grow(t + wave);
        if (glo >= 1 && glo + NW + 3 < Nt) {
            if (base_lane) {
                const Affine &ad = Ls.adv[bbnd ? 2 : 0];
                bases = mad128c(ad.A, bases, ad.C);
                brow += NW;
                Ls.base[wave][lane] = bases;
            }
        } else if (base_lane) {
            const int64_t p_old = wf_base_pos(bbnd, grow(brow), N, bx, bhas);
            const int64_t p_new = wf_base_pos(bbnd, grow(brow + NW), N, bx, bhas);
            const int64_t step = bbnd ? (int64_t)NW * N / 4 : (int64_t)NW * N;
            if (p_new - p_old == step) bases = apply(Ls.adv[bbnd ? 2 : 0], bases);
            else if (p_new - p_old == step - (bbnd ? (int64_t)Nt * N / 4 : (int64_t)Nt * N))
                bases = apply(Ls.adv[bbnd ? 4 : 3], bases);  // the wave's rows wrapped around the torus
            else bases = full_jump(A.T, &A.blocks[bblk], (uint32_t)p_new);
            brow += NW;
            Ls.base[wave][lane] = bases;
        }
        __syncthreads();
    }
#if SV_WFTIME
    const uint64_t wf_t2 = __builtin_amdgcn_s_memrealtime();
#endif
    {
        int32_t tl = tfirst;
        while (tl + NW < t1) tl += NW;
        store_rows(tl);
    }
    if (Ls.bad && threadIdx.x == 0) report(A.S, A.sweep, OVERFLOW_BLOCK, 0, 0);
    wflush(A.pstat, pacc, ppsum);
    wflush(A.cstat, cacc, cpsum);
#if SV_WFTIME
    __builtin_amdgcn_s_waitcnt(0);
    if (threadIdx.x == 0 && blockIdx.x < 65536) {
        uint64_t *o = g_wftime + 6 * (size_t)blockIdx.x;
        o[0] = wf_t0;
        o[1] = wf_t1;
        o[2] = wf_t2;
        o[3] = __builtin_amdgcn_s_memrealtime();
        o[5] = wf_tb;
        o[4] = (uint64_t)(uint32_t)__builtin_amdgcn_s_getreg(4 | (31 << 11)) |
               ((uint64_t)(uint32_t)__builtin_amdgcn_s_getreg(20 | (31 << 11)) << 32);
    }
#endif
}

// the 8-wave kernel is compiled for 2 waves per SIMD (one workgroup per CU; two at <= 128 VGPRs measured slower, r386)
constexpr int WF_OCC8 = 2;
template <bool TILE, int NW>
__global__ __launch_bounds__(NW * 64) __attribute__((amdgpu_waves_per_eu(NW == 8 ? WF_OCC8 : 1))) void worldline_step_fused(WFArgs A) {
    __shared__ WFLDS<NW> Ls;
    int ix;
    int32_t t0, t1;
    wf_strip(A, ix, t0, t1);
    const int32_t x0 = wf_xb(A, ix), x1 = wf_xb(A, ix + 1);
    const int32_t gx0 = A.G.X0 + x0;
    const bool interior = gx0 - 5 >= 0 && gx0 + (x1 - x0) + 4 <= A.G.Nx && A.G.Nx > SMALL_LDS;
    if (A.general) wf_body<TILE, 2, NW>(A, Ls);
    else if (__builtin_amdgcn_readfirstlane((int)interior)) wf_body<TILE, 0, NW>(A, Ls);
    else wf_body<TILE, 1, NW>(A, Ls);
}
template __global__ void worldline_step_fused<false, 4>(WFArgs);
template __global__ void worldline_step_fused<true, 4>(WFArgs);
template __global__ void worldline_step_fused<false, 8>(WFArgs);
template __global__ void worldline_step_fused<true, 8>(WFArgs);
template __global__ void worldline_step_fused<false, 16>(WFArgs);
template __global__ void worldline_step_fused<true, 16>(WFArgs);

}  // namespace sv

namespace svh {
using namespace sv;

static int wf_th(int32_t N, int nsx, int nw);

// waves per workgroup (SV_WF_NW = 4 or 8 overrides).  8-wave workgroups recompute the 7 halo rows a strip's passes
// need for more rows each, at one workgroup per CU (r386 at L=1024: 46.0 -> 43.4 us per step, 8 x 40-row strips; with
// two 8-wave workgroups per CU at <= 128 VGPRs 44.1 us over 24-row strips, 51 us over 16 or 32); used when one round
// of them covers at least 3/4 of the CUs, else 4 waves
// 16-wave workgroups (r3): 41-row strips take ceil((41 + 7) / 16) = 3 row steps at 4 waves per SIMD, one workgroup
// per CU, where 8 waves took 6 steps over 40 rows at 2 (L=1024: 43.8 -> 40.1 us per step; 16 waves over 25 / 33 / 57
// rows: 57.0 / 68.0 / 47.8 us, two rounds or fewer CUs); used when one round of them covers at least 3/4 of the CUs
static int wf_nw(int32_t Ht, int nsx) {
    const int64_t g16 = (int64_t)nsx * ((Ht + 40) / 41);
    if (g16 >= 192 && g16 <= 256) return 16;
    const int th = wf_th(Ht, nsx, 8);
    return (int64_t)nsx * ((Ht + th - 1) / th) >= 192 ? 8 : 4;
}

// rows per strip (SV_WF_TH overrides).  4 waves: as fused_th, cut down until the grid has `fill` workgroups.  448: at
// L=1024 (9 column strips) that stops at 20 rows, 468 workgroups for the 768 slots of 3 per CU (r381: 16 / 20 / 24 /
// 28 rows 47.9 / 46.1 / 51.3 / 56.5 us per step; 512 stopped at 16).  8 waves: the fewest row steps per strip with
// at most one workgroup per CU (L=1024: 40 rows; r386: 32 / 40 / 48 rows 68.7 / 43.4 / 49.1 us, 32 needing two rounds)
static int wf_th(int32_t N, int nsx, int nw) {
    const char *e = getenv("SV_WF_TH");
    if (e) {
        const int v = atoi(e);
        if (v >= 4) return v;
    }
    if (nw == 16) return 41;  // (16 k - 7 rows fill the last row step: the passes reach 7 rows past the strip)
    if (nw == 8) {
        const int slots = 256 * (WF_OCC8 >= 4 ? 2 : 1);
        int th = 8;
        while (th < N && (int64_t)nsx * ((N + th - 1) / th) > slots) th += 8;
        return th;
    }
    constexpr int fill = 448;
    int th = 64;
    while (th > 4 && (int64_t)nsx * ((N + th - 1) / th) < fill) th -= 4;
    return th;
}

// Whether worldline_step_fused can run these parameters at all (even N, integer v, W a power of two: f and df
// exact as the pass kernels form them)
bool wf_usable(int32_t N, bool v_is_float, double W_eff, int64_t it) {
    int ex = 0;
    return !(N % 2 || N < 4 || v_is_float || !(W_eff > 0) || std::frexp(W_eff, &ex) != 0.5 || it < 1 || it > (1 << 20));
}
// Whether one step (5 plaquette blocks then 3 coexact blocks) runs in the fast modes (no skip list, equal
// buffered-half flags in each change_m / change_v pair); otherwise it runs in the GENERAL mode
bool wf_fast(const Block *blocks) {
    for (int c = 0; c < 2; c++) {
        if (blocks[1 + 2 * c].nskip || blocks[2 + 2 * c].nskip || blocks[6 + c].nskip) return false;
        if (blocks[1 + 2 * c].has != blocks[2 + 2 * c].has) return false;
    }
    return true;
}

// compute units of the current device (the turned layout runs its strips in one round)
static int cu_count() {
    static const int n = [] {
        int dev = 0, c = 0;
        if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
            return 0;
        return c;
    }();
    return n;
}
// SV_WF_TURN=0: the plain layout (A/B and tests), read per call
static bool turn_off() {
    const char *e = std::getenv("SV_WF_TURN");
    return e && e[0] == '0';
}

// SV_WF_TAIL=0: the last row strip not cut (A/B), read per call
static bool tail_off() {
    const char *e = std::getenv("SV_WF_TAIL");
    return e && e[0] == '0';
}

// the inverse of s -> A s + C mod 2^128 (A odd): s -> A^-1 s - A^-1 C; A^-1 by Newton's iteration, each step doubling
// the bits that are right (A A = 1 mod 8 to start)
static Affine inverse(const Affine &f) {
    u128 x = f.A;
    for (int i = 0; i < 6; i++) {
        const u128 ax = mul(f.A, x);
        const u128 two_minus = add(u128{~ax.lo, ~ax.hi}, u128{3, 0});  // 2 - ax = ~ax + 1 + 2
        x = mul(x, two_minus);
    }
    const u128 xc = mul(x, f.C);
    return Affine{x, add(u128{~xc.lo, ~xc.hi}, u128{1, 0})};
}

void launch_wf(const FGeom &G, double kappa, double W_eff, int64_t it, const int64_t *m_in, const int64_t *v_in,
               int64_t *m_out, int64_t *v_out, const Block *blocks, const Block *hblocks, const uint32_t *skips, bool general,
               const JumpTables *T, const Affine adv[6], u128 inc, void *pstat, void *cstat, DevScratch S, uint32_t sweep,
               hipStream_t stream) {
    if ((int64_t)G.Nt * G.Nx >= (int64_t(1) << 31))
        throw std::invalid_argument("worldline_step_fused addresses stream positions with 31 bits (V < 2^31)");
    if (G.plane >= (int64_t(1) << 28))
        throw std::invalid_argument("worldline_step_fused moves rows by 32-bit byte offsets (plane < 2^28)");
    WFArgs A{};
    A.skips = skips;
    A.general = general ? 1 : 0;
    A.G = G;
    A.nsx = (G.Wt + WF_W - 1) / WF_W;
    const int nw = wf_nw(G.Ht, A.nsx);
    A.TH = wf_th(G.Ht, A.nsx, nw);
    A.nsy = (G.Ht + A.TH - 1) / A.TH;
    A.rot = A.ths = A.nsy_s = A.tail = 0;
    const bool tile = !(G.T0 == 0 && G.X0 == 0 && G.Ht == G.Nt && G.Wt == G.Nx && G.pitch == G.Nx && G.org == 0);
    if (!tile && nw == 16 && G.Nx > SMALL_LDS && A.nsx >= 3 && !turn_off()) {
        // the turned layout: strip 0 = [-rot, W - rot) holds the column seam (W = Nx / nsx); the other strips' regions
        // stay within [0, Nx) (rot >= 5 and W - rot >= 5)
        const int32_t W0 = G.Nx / A.nsx, rot = W0 / 2;
        const int32_t ths = 25, nsy_s = (G.Ht + ths - 1) / ths;
        if (rot >= 5 && W0 - rot >= 5 && (int64_t)(A.nsx - 1) * A.nsy + nsy_s <= cu_count()) {
            A.rot = rot;
            A.ths = ths;
            A.nsy_s = nsy_s;
            const int32_t rest = G.Ht - (A.nsy - 1) * A.TH, tail = (rest + 1) / 2;
            if (A.nsy >= 2 && tail + 7 <= 32 && (int64_t)(A.nsx - 1) * (A.nsy + 1) + nsy_s <= cu_count() && !tail_off())
                A.tail = tail;
        }
    }
    const int grid = A.ths ? (A.nsx - 1) * (A.tail ? A.nsy + 1 : A.nsy) + A.nsy_s : A.nsx * A.nsy;
    A.m_in = m_in;
    A.v_in = v_in;
    A.m_out = m_out;
    A.v_out = v_out;
    A.blocks = blocks;
    for (int i = 0; i < 8; i++) A.blk[i] = hblocks[i];
    A.T = T;
    for (int i = 0; i < 3; i++) A.adv[i] = nw == 16 ? compose(adv[3 + i], adv[3 + i]) : adv[(nw == 8 ? 3 : 0) + i];
    {
        // NW rows on across the row seam moves a row's stream position back by V - NW N draws ((V - NW N) / 4 words;
        // N even, so both are whole): the inverse of the forward maps
        const uint64_t V = (uint64_t)G.Nt * (uint64_t)G.Nx, fw = (uint64_t)nw * (uint64_t)G.Nx;
        A.adv[3] = V > fw ? inverse(host_power(inc, V - fw)) : Affine{{1, 0}, {0, 0}};
        A.adv[4] = V > fw ? inverse(host_power(inc, (V - fw) / 4)) : Affine{{1, 0}, {0, 0}};
    }
    A.pstat = (StatStripe *)pstat;
    A.cstat = (StatStripe *)cstat;
    A.S = S;
    A.sweep = sweep;
    A.Winv = 1.0 / W_eff;
    A.c = 0.5 / kappa;
    for (int jm = 0; jm < 2; jm++)
        for (int jv = 0; jv < 3; jv++) {  // plaquette_cb_gs: df = cm - cv * Winv, dS = df / kappa * (...)
            const double cm = jm ? 1.0 : -1.0, cv = (double)(jv - 1);
            const double df = cm - cv * A.Winv;
            A.df[3 * jm + jv] = df;
            A.dfk[3 * jm + jv] = df / kappa;
        }
    {
        int ex = 0;
        std::frexp(W_eff, &ex);  // W_eff = 2^(ex - 1)
        const int lw = ex - 1;
        A.sa = lw > 0 ? lw : 0;
        A.sb = lw < 0 ? -lw : 0;
        A.unit = lw > 0 ? A.Winv : 1.0;
        A.ptab = lw >= -20 && lw <= 20;  // (shifts that keep S exact in 64 bits)
    }
    A.it = (int32_t)it;
    A.kt = (uint32_t)(2 * it);
    A.thrt = (uint32_t)((0u - A.kt) % A.kt);
    if (nw == 16) {
        if (tile) worldline_step_fused<true, 16><<<grid, 16 * 64, 0, stream>>>(A), SV_LAUNCHED("worldline_step_fused<true, 16>", stream);
        else worldline_step_fused<false, 16><<<grid, 16 * 64, 0, stream>>>(A), SV_LAUNCHED("worldline_step_fused<false, 16>", stream);
    } else if (nw == 8) {
        if (tile) worldline_step_fused<true, 8><<<grid, 8 * 64, 0, stream>>>(A), SV_LAUNCHED("worldline_step_fused<true, 8>", stream);
        else worldline_step_fused<false, 8><<<grid, 8 * 64, 0, stream>>>(A), SV_LAUNCHED("worldline_step_fused<false, 8>", stream);
    } else {
        if (tile) worldline_step_fused<true, 4><<<grid, 4 * 64, 0, stream>>>(A), SV_LAUNCHED("worldline_step_fused<true, 4>", stream);
        else worldline_step_fused<false, 4><<<grid, 4 * 64, 0, stream>>>(A), SV_LAUNCHED("worldline_step_fused<false, 4>", stream);
    }
}

}  // namespace svh

#if SV_WFTIME
extern "C" int sv_debug_wftime(uint64_t *out, int32_t n) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(sv::g_wftime), (size_t)n * 6 * sizeof(uint64_t)) == hipSuccess ? 0 : -2;
}
#endif
