// domain.hip -- NeighborhoodUpdate on a domain-decomposed lattice (BASELINE config 4).
//
// The Nt x Nx lattice is cut into tiles_t x tiles_x tiles of Ht x Wt sites.  Each tile lives in HBM
// with a ghost frame (2 rows above, 3 below, 2 columns left, 3 right: exactly what the fused sweep
// kernel reads around a tile, villain.hip) and one sweep is
//
//     pack (8 halo messages) -> exchange -> unpack into the ghost frame -> fused sweep kernel.
//
// Because both colours are decided inside one launch there is ONE exchange per sweep -- or one per K sweeps with
// deep halos (villain_depth: a K-times deeper frame, each sweep of a group deciding the tile plus the ring its
// successor reads).  Every draw is addressed by its global NumPy stream position and the colouring by global
// coordinates, so the decomposed chain is bit-identical to the single-lattice chain (and to the reference's).
//
// Transport: tiles in the same process (one GPU emulating any tile grid -- the parity tests -- or a
// tile grid dimension of 1) read each other's send buffers directly; tiles on other ranks exchange
// through RCCL point-to-point (ncclSend/ncclRecv in one group, over xGMI), on the context's stream.
//
// Rejections (NumPy's Lemire sampler rejecting a uint32, which shifts the rest of its block) are
// found by whichever tile draws the position.  Each halo message carries its sender's abort flag,
// so an abort spreads one tile-hop per exchange and every tile stops within D K sweeps (D = tile-torus
// radius); the tile states are kept in a ring of R = D K + 2 buffers so the input of the failing sweep
// survives everywhere.  With several ranks the rejections are mostly predicted (scan_rejections) and no abort happens.  After each batch the ranks all-gather their reports (one collective per
// batch) and take the same replay decision as the single-lattice driver.
#include <rccl/rccl.h>

#include <algorithm>
#include <array>
#include <cmath>
#include <cstring>

#include "fused.h"
#include "villain.h"

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

// Ghost frames (rows above / below, columns left / right of a tile) = what one sweep's kernel reads around
// the tile: villain_sweep_hot / _fused 2, 3, 2, 3; worldline_step_fused (four passes, each one ring wider)
// 5, 4, 5, 4.  The three 8-byte planes a tile holds are (phi, n0, n1) for Villain and (v, m0, m1) for
// Worldline: the halo code moves them as bits.
struct Ghost {
    int32_t top, bottom, left, right;
};
static constexpr Ghost VILLAIN_GHOST{2, 3, 2, 3}, WORLDLINE_GHOST{5, 4, 5, 4};
static constexpr int LEFT_PAD = 16;  // interior starts 128 B-aligned
static constexpr int DOMAIN_BATCH = 64;
static constexpr int NDIR = 8;

// direction s = 0..7 <-> (dy, dx) in {-1,0,1}^2 \ {(0,0)}, row-major
__host__ __device__ inline void dir_of(int s, int &dy, int &dx) {
    const int k = s < 4 ? s : s + 1;
    dy = k / 3 - 1;
    dx = k % 3 - 1;
}
inline int opp(int s) { return NDIR - 1 - s; }  // (-dy, -dx)

// Message of direction s (toward the tile at (dy, dx)): the sender's interior rectangle the
// receiver needs for its ghost block on the opposite side.
struct Rect {
    int32_t r0, c0, rows, cols;
};
inline Rect send_rect(int s, int32_t Ht, int32_t Wt, const Ghost &g) {
    int dy, dx;
    dir_of(s, dy, dx);
    Rect R;
    R.r0 = dy > 0 ? Ht - g.top : 0;
    R.rows = dy == 0 ? Ht : (dy > 0 ? g.top : g.bottom);
    R.c0 = dx > 0 ? Wt - g.left : 0;
    R.cols = dx == 0 ? Wt : (dx > 0 ? g.left : g.right);
    return R;
}
// Ghost block filled by the message of direction s (it arrives from the tile at (-dy, -dx)).
inline Rect recv_rect(int s, int32_t Ht, int32_t Wt, const Ghost &g) {
    int dy, dx;
    dir_of(s, dy, dx);
    Rect R = send_rect(s, Ht, Wt, g);
    R.r0 = dy > 0 ? -g.top : (dy == 0 ? 0 : Ht);
    R.c0 = dx > 0 ? -g.left : (dx == 0 ? 0 : Wt);
    return R;
}

struct HaloTable {
    Rect rect[NDIR];
    int64_t off[NDIR];  // u64 words; message = [flag, pad, phi[cnt], n0[cnt], n1[cnt]]
};
struct HaloSrc {
    const uint64_t *msg[NDIR];  // message of direction s for this tile's ghost block s
};

__global__ void halo_pack(const double *phi, const int64_t *n, int64_t pitch, int64_t plane, int64_t org,
                          HaloTable H, uint64_t *send, const int32_t *abort) {
    const int s = blockIdx.y;
    const Rect R = H.rect[s];
    const int64_t cnt = (int64_t)R.rows * R.cols;
    uint64_t *m = send + H.off[s];
    const int32_t ab = *(volatile const int32_t *)abort;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        m[0] = (uint64_t)ab;
        m[1] = 0;
    }
    if (ab) return;
    for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < cnt; e += (int64_t)gridDim.x * blockDim.x) {
        const int32_t r = (int32_t)(e / R.cols), c = (int32_t)(e - (int64_t)r * R.cols);
        const int64_t g = org + (int64_t)(R.r0 + r) * pitch + R.c0 + c;
        m[2 + e] = __double_as_longlong(phi[g]);
        m[2 + cnt + e] = (uint64_t)n[g];
        m[2 + 2 * cnt + e] = (uint64_t)n[plane + g];
    }
}

__global__ void halo_unpack(double *phi, int64_t *n, int64_t pitch, int64_t plane, int64_t org, HaloTable H,
                            HaloSrc src, int32_t *abort) {
    const int s = blockIdx.y;
    const uint64_t *m = src.msg[s];
    if (*(volatile const uint64_t *)m) {  // the sender has aborted: stop here too
        if (blockIdx.x == 0 && threadIdx.x == 0) __hip_atomic_store(abort, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return;
    }
    if (*(volatile const int32_t *)abort) return;
    const Rect R = H.rect[s];
    const int64_t cnt = (int64_t)R.rows * R.cols;
    for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < cnt; e += (int64_t)gridDim.x * blockDim.x) {
        const int32_t r = (int32_t)(e / R.cols), c = (int32_t)(e - (int64_t)r * R.cols);
        const int64_t g = org + (int64_t)(R.r0 + r) * pitch + R.c0 + c;
        phi[g] = __longlong_as_double((long long)m[2 + e]);
        n[g] = (int64_t)m[2 + cnt + e];
        n[plane + g] = (int64_t)m[2 + 2 * cnt + e];
    }
}

// Per-tile batch summary, contiguous so that ranks can all-gather it in one collective.
static constexpr int MAX_CAND = 64;
struct Summary {
    int32_t abort;
    uint32_t nreport;
    uint32_t ncand;      // rejection prediction: words of the NEXT batch NumPy's Lemire sampler would reject
    uint32_t pad;
    Report reports[MAX_REPORTS];
    sv_stats stats[2 * DOMAIN_BATCH];  // Villain: one per sweep; Worldline: (Plaquette, Coexact) per step
    uint64_t cand[MAX_CAND];           // half-word indices (2 u64 + high) counted from the next batch's start state
};

// Rejection prediction.  A NumPy Lemire rejection aborts a decomposed batch from its sweep on, and with small tiles
// (the strong-scaled config 4) the drained sweeps and the host round trip of the replay cost several sweep times;
// so the batch size was kept short, and with it every batch pays an all-gather and a synchronization.  Whether a
// word is rejected depends only on the stream, not on the lattice, so the words the NEXT batch's choice blocks will
// draw can be tested while this batch runs: sweep k of a batch draws its bounded words from u64 [1.5V, 2.5V) and
// [3V, 4V) after its nominal start (4V u64 per sweep; skips shift that by a few half-words, covered by a margin of
// SCAN_MARGIN u64 on each side).  The ranks split the scan, and the words found travel in the batch summaries the
// ranks all-gather anyway; the host turns them into skip lists before planning the batch (add_predicted).  The
// abort / replay protocol stays as the safety net (a word outside the scanned ranges, the first batch of a call).
static constexpr uint64_t SCAN_MARGIN = 32;
static constexpr int SCAN_CHUNK = 64;  // u64 per lane: one table jump, then single steps

struct ScanArgs {
    const u128 *s_k;      // per sweep of the scanned batch: the state after k 4V steps from the batch start
    const JumpTables *T;
    uint64_t V, lo, hi;   // this rank's slice [lo, hi) of the batch's scan index space (2 (V + 2 M) per sweep)
    uint32_t k, thr;      // bounded draws over k values; NumPy's rejection threshold
    uint32_t *ncand;
    uint64_t *cand;
};

__global__ __launch_bounds__(256) void scan_rejections(ScanArgs a) {
    const uint64_t seg = a.V + 2 * SCAN_MARGIN, per = 2 * seg;
    uint64_t v = a.lo + (blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) * SCAN_CHUNK;
    if (v >= a.hi) return;
    const uint64_t v1 = v + SCAN_CHUNK < a.hi ? v + SCAN_CHUNK : a.hi;
    uint32_t k = (uint32_t)(v / per);
    uint64_t r = v - (uint64_t)k * per;
    const Affine one = a.T->small[1];
    while (v < v1) {
        // a run of consecutive u64 within sweep k: the colour-0 choice run or the colour-1 one (with margins)
        const bool first = r < seg;
        uint64_t j = first ? a.V + a.V / 2 - SCAN_MARGIN + r : 3 * a.V - SCAN_MARGIN + (r - seg);
        const uint64_t left = (first ? seg - r : per - r), n = left < v1 - v ? left : v1 - v;
        u128 st = jump(a.T, a.s_k[k], (uint32_t)(j + 1));  // the state whose output is u64 j
        for (uint64_t e = 0; e < n; e++, j++) {
            const uint64_t x = xsl_rr(st);
            const bool rl = (uint32_t)((uint64_t)(uint32_t)x * a.k) < a.thr;
            const bool rh = (uint32_t)((uint64_t)(uint32_t)(x >> 32) * a.k) < a.thr;
            if (__builtin_expect(rl | rh, 0)) {
                const uint64_t h = 2 * ((uint64_t)k * 4 * a.V + j);
                for (int half = 0; half < 2; half++)
                    if (half ? rh : rl) {
                        const uint32_t i = atomicAdd(a.ncand, 1u);
                        if (i < MAX_CAND) a.cand[i] = h + half;
                    }
            }
            st = mad128c(one.A, st, one.C);
        }
        v += n;
        r += n;
        if (r == per) {
            r = 0;
            k++;
        }
    }
}

// Worldline tiles: the per-step StatStripes of worldline_step_fused folded into the tile's Summary
__global__ void wd_fold(const StatStripe *ss, sv_stats *out, int count) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= count) return;
    unsigned long long a = 0, w[3] = {0, 0, 0};
    for (int j = 0; j < NSTRIPE; j++) {
        a += ss[k * NSTRIPE + j].acc;
        for (int i = 0; i < 3; i++) w[i] += ss[k * NSTRIPE + j].pw[i];
    }
    // the exact acceptance limbs (common.h) in the slot's words: summed over tiles on the host
    *stat_word(&out[k], 0) = a;
    for (int i = 0; i < 3; i++) *stat_word(&out[k], 1 + i) = w[i];
}

}  // namespace sv

using namespace svh;

struct sv_domain_tile {
    int32_t iy = 0, ix = 0, T0 = 0, X0 = 0;
    int nbr[NDIR] = {0};            // global tile index of the neighbour in direction s
    std::vector<double *> phi;      // ring of R buffers, ghost layout
    std::vector<int64_t *> n;
    uint64_t *send = nullptr, *recv = nullptr;
    Summary *sum = nullptr;         // device
    StatStripe *stripes = nullptr;  // Worldline: DOMAIN_BATCH x 2 x NSTRIPE
    // message layout: the messages bound for (or coming from) one remote peer are contiguous, so one
    // ncclSend / ncclRecv per distinct peer carries them all (e.g. 4 peers instead of 8 for 2 x 4 tiles)
    int64_t soff[NDIR] = {0}, roff[NDIR] = {0};
    std::vector<std::array<int64_t, 3>> sends, recvs;  // {peer, offset, words}
};

struct sv_domain {
    sv_ctx *ctx = nullptr;
    int model = 0;                  // 0 Villain (phi, n), 1 Worldline (v, m)
    Ghost ghost = VILLAIN_GHOST;
    int32_t Nt = 0, Nx = 0, ty = 1, tx = 1, Ht = 0, Wt = 0;
    int nranks = 1, rank = 0;
    int64_t pitch = 0, plane = 0, org = 0;
    int R = 2, cur = 0;
    int depth = 1;                  // Villain: sweeps per halo exchange (deep halos, see villain_depth)
    u128 *d_scan = nullptr;         // rejection prediction: per-sweep start states of the scanned batch
    hipStream_t scan_stream = nullptr;  // lowest priority: the scan fills the slots the sweeps leave free
    hipEvent_t ev_sum = nullptr, ev_scan = nullptr;
    struct Pred {                   // the scanned words of the batch starting at cursor c (kept across calls)
        bool valid = false;
        int sw = 0, count = 0;
        Cursor c{};
        u128 inc{0, 0};
        uint32_t k = 0, thr = 0;    // the bounded draws the words were tested for (from interval_n)
        std::vector<uint64_t> cand;
    } pred;
    HaloTable H{};
    int64_t msg_words = 0;
    std::vector<sv_domain_tile> tiles;  // local tiles (all tiles when nranks == 1)
    std::vector<int> local_of;          // global tile index -> local index, or -1
    ncclComm_t comm = nullptr;
    bool loopback = false;              // 1 rank, 1 tile, halos through RCCL to itself (tests the RCCL path)
    Summary *gathered = nullptr;        // device, nranks summaries (RCCL mode)
    // hosted transport (sv_domain_create_hosted): the caller's callbacks carry the messages and the all-gather
    sv_xfer_fn xfer = nullptr;
    sv_gather_fn gatherfn = nullptr;
    void *user = nullptr;
    uint64_t *h_send = nullptr, *h_recv = nullptr;  // page-locked message staging
    Summary *h_local = nullptr;                      // page-locked: this rank's summary
    std::vector<Summary> host_sum;
};

namespace {

void check_nccl(ncclResult_t r, const char *what) {
    if (r != ncclSuccess) throw std::runtime_error(std::string(what) + " failed: " + ncclGetErrorString(r));
}

int tile_index(const sv_domain *d, int iy, int ix) {
    iy = ((iy % d->ty) + d->ty) % d->ty;
    ix = ((ix % d->tx) + d->tx) % d->tx;
    return iy * d->tx + ix;
}

// Deep halos (Villain).  One sweep reads a 2/3/2/3 ring around the sites it decides, so K sweeps can run between two
// halo exchanges when the ghost frame is K times as deep (2K above, 3K below, 2K left, 3K right) and sweep j of a
// group of K decides the tile extended by 2(K-1-j) rows / columns above and left and 3(K-1-j) below and right: each
// sweep recomputes, bit for bit, the ring its successor reads (every draw is addressed by its global stream
// position), counts only the tile's own sites, and the group's last sweep decides exactly the tile.  The
// redundant ring costs ~5(K-1)/2 rows and columns per sweep (0.6% of a 2048 x 1024 tile at K = 4) and saves K-1
// of every K exchanges -- on the strong-scaled config 4 the RCCL exchange is a large part of a tile sweep.  The
// frame must come from the adjacent tiles only (3K <= tile extents) and the extended rows must stay within the
// kernels' single wrap of the torus (5K - 2 <= lattice extents).  SV_DOMAIN_DEPTH sets K (default 4, at most 8:
// the interior's 16-column left pad).
int villain_depth(int32_t Ht, int32_t Wt, int32_t Nt, int32_t Nx) {
    const char *e = getenv("SV_DOMAIN_DEPTH");
    int K = e ? atoi(e) : 4;
    K = std::max(1, std::min(8, K));
    while (K > 1 && (3 * K > std::min(Ht, Wt) || 5 * K - 2 > std::min(Nt, Nx))) K--;
    return K;
}

void geometry(sv_domain *d) {
    if (d->Nt % d->ty || d->Nx % d->tx) throw std::invalid_argument("the lattice must divide evenly into tiles");
    d->Ht = d->Nt / d->ty;
    d->Wt = d->Nx / d->tx;
    if (d->Ht % 2 || d->Wt % 2 || d->Ht < 4 || d->Wt < 4)
        throw std::invalid_argument("tiles must be at least 4 x 4 with even extents");
    if (d->model == 0) {
        d->depth = villain_depth(d->Ht, d->Wt, d->Nt, d->Nx);
        const int K = d->depth;
        d->ghost = Ghost{VILLAIN_GHOST.top * K, VILLAIN_GHOST.bottom * K, VILLAIN_GHOST.left * K, VILLAIN_GHOST.right * K};
    }
    if ((int64_t)d->Nt * d->Nx >= (1LL << 32)) throw std::invalid_argument("lattice too large for 32-bit stream positions");
    const Ghost &g = d->ghost;
    if (d->Ht < std::max(g.top, g.bottom) || d->Wt < std::max(g.left, g.right))
        throw std::invalid_argument("tiles must be at least as large as their ghost frame");
    d->pitch = ((LEFT_PAD + d->Wt + g.right + 15) / 16) * 16;
    d->plane = (int64_t)(d->Ht + g.top + g.bottom) * d->pitch;
    d->org = (int64_t)g.top * d->pitch + LEFT_PAD;
    // ring depth: an abort travels one tile-hop (8-neighbour torus) per exchange, i.e. per K sweeps, so a tile
    // D hops away runs at most D K sweeps past the failing one
    const int D = std::max(d->ty / 2, d->tx / 2);
    d->R = std::max(2, D * d->depth + 2);
    int64_t off = 0;
    for (int s = 0; s < NDIR; s++) {
        d->H.rect[s] = send_rect(s, d->Ht, d->Wt, d->ghost);
        d->H.off[s] = off;
        off += 2 + 3 * (int64_t)d->H.rect[s].rows * d->H.rect[s].cols;
    }
    d->msg_words = off;
}

HaloTable recv_table(const sv_domain *d) {
    HaloTable h = d->H;
    for (int s = 0; s < NDIR; s++) h.rect[s] = recv_rect(s, d->Ht, d->Wt, d->ghost);
    return h;
}

// Per-tile message offsets grouped by remote peer (see sv_domain_tile).  Sender and receiver order a
// peer's messages by direction s: the sender's {s : nbr[s] == B} equals the receiver's
// {s : nbr[opp(s)] == A}, so the concatenations line up word for word.
void halo_layout(sv_domain *d) {
    auto words = [&](int s) { return 2 + 3 * (int64_t)d->H.rect[s].rows * d->H.rect[s].cols; };
    for (auto &T : d->tiles) {
        auto remote = [&](int peer) { return d->loopback || d->local_of[peer] < 0; };
        for (int side = 0; side < 2; side++) {
            int64_t *off = side == 0 ? T.soff : T.roff;
            auto &lst = side == 0 ? T.sends : T.recvs;
            lst.clear();
            int64_t o = 0;
            std::vector<int> peers;
            for (int s = 0; s < NDIR; s++) {
                const int peer = side == 0 ? T.nbr[s] : T.nbr[opp(s)];
                if (remote(peer) && std::find(peers.begin(), peers.end(), peer) == peers.end()) peers.push_back(peer);
            }
            for (int peer : peers) {
                const int64_t o0 = o;
                for (int s = 0; s < NDIR; s++)
                    if ((side == 0 ? T.nbr[s] : T.nbr[opp(s)]) == peer) {
                        off[s] = o;
                        o += words(s);
                    }
                lst.push_back({peer, o0, o - o0});
            }
            for (int s = 0; s < NDIR; s++)
                if (!remote(side == 0 ? T.nbr[s] : T.nbr[opp(s)])) {
                    off[s] = o;
                    o += words(s);
                }
        }
    }
}

// The local tiles (all of them with one rank, else the rank's own) and their neighbour tables.
void build_tiles(sv_domain *d) {
    const int ntiles = d->ty * d->tx;
    d->local_of.assign(ntiles, -1);
    d->tiles.clear();
    for (int t = 0; t < ntiles; t++) {
        if (d->nranks > 1 && t != d->rank) continue;
        sv_domain_tile T;
        T.iy = t / d->tx;
        T.ix = t % d->tx;
        T.T0 = T.iy * d->Ht;
        T.X0 = T.ix * d->Wt;
        for (int s = 0; s < NDIR; s++) {
            int dy, dx;
            dir_of(s, dy, dx);
            T.nbr[s] = tile_index(d, T.iy + dy, T.ix + dx);
        }
        d->local_of[t] = (int)d->tiles.size();
        d->tiles.push_back(T);
    }
}

void exchange(sv_domain *d, hipStream_t stream) {
    sv_ctx *ctx = d->ctx;
    (void)ctx;
    const int slot = d->cur;
    const int threads = 256;
    // pack every local tile
    for (auto &T : d->tiles) {
        int64_t mx = 0;
        for (int s = 0; s < NDIR; s++) mx = std::max<int64_t>(mx, (int64_t)d->H.rect[s].rows * d->H.rect[s].cols);
        dim3 grid((unsigned)std::min<int64_t>((mx + threads - 1) / threads, 1024), NDIR);
        HaloTable HS = d->H;
        for (int s = 0; s < NDIR; s++) HS.off[s] = T.soff[s];
        halo_pack<<<grid, threads, 0, stream>>>(T.phi[slot], T.n[slot], d->pitch, d->plane, d->org, HS, T.send,
                                                     &T.sum->abort), SV_LAUNCHED("halo_pack", stream);
    }
    // remote messages (one tile per rank in RCCL mode)
    if (d->xfer) {
        // hosted transport: this rank's packed messages through host memory and the caller's callback
        sv_domain_tile &T = d->tiles[0];
        SV_HIP(hipMemcpyAsync(d->h_send, T.send, d->msg_words * sizeof(uint64_t), hipMemcpyDeviceToHost, stream));
        SV_HIP(hipStreamSynchronize(stream));
        std::vector<int64_t> sd, rv;
        for (const auto &m : T.sends) sd.insert(sd.end(), {m[0], m[1], m[2]});
        for (const auto &m : T.recvs) rv.insert(rv.end(), {m[0], m[1], m[2]});
        if (d->xfer(d->user, (int32_t)T.sends.size(), sd.data(), d->h_send, (int32_t)T.recvs.size(), rv.data(),
                    d->h_recv) != 0)
            throw std::runtime_error("the hosted halo exchange failed (sv_xfer_fn returned non-zero)");
        SV_HIP(hipMemcpyAsync(T.recv, d->h_recv, d->msg_words * sizeof(uint64_t), hipMemcpyHostToDevice, stream));
    } else if (d->comm) {
        sv_domain_tile &T = d->tiles[0];
        check_nccl(ncclGroupStart(), "ncclGroupStart");
        for (const auto &m : T.sends)
            check_nccl(ncclSend(T.send + m[1], (size_t)m[2], ncclUint64, (int)m[0], d->comm, stream), "ncclSend");
        for (const auto &m : T.recvs)
            check_nccl(ncclRecv(T.recv + m[1], (size_t)m[2], ncclUint64, (int)m[0], d->comm, stream), "ncclRecv");
        check_nccl(ncclGroupEnd(), "ncclGroupEnd");
    }
    // unpack: ghost block s takes the message of direction s from the neighbour at -s
    const HaloTable HR = recv_table(d);
    for (auto &T : d->tiles) {
        HaloSrc src;
        int64_t mx = 0;
        for (int s = 0; s < NDIR; s++) {
            const int peer = T.nbr[opp(s)];
            const int li = d->local_of[peer];
            src.msg[s] = (li >= 0 && !d->loopback) ? d->tiles[li].send + d->tiles[li].soff[s] : T.recv + T.roff[s];
            mx = std::max<int64_t>(mx, (int64_t)HR.rect[s].rows * HR.rect[s].cols);
        }
        dim3 grid((unsigned)std::min<int64_t>((mx + threads - 1) / threads, 1024), NDIR);
        halo_unpack<<<grid, threads, 0, stream>>>(T.phi[slot], T.n[slot], d->pitch, d->plane, d->org, HR, src,
                                                       &T.sum->abort), SV_LAUNCHED("halo_unpack", stream);
    }
}

// Gather every tile's batch summary (local tiles, then all ranks), in global tile order.
void gather(sv_domain *d) {
    sv_ctx *ctx = d->ctx;
    const int ntiles = d->ty * d->tx;
    d->host_sum.resize(ntiles);
    if (d->gatherfn) {
        SV_HIP(hipMemcpyAsync(d->h_local, d->tiles[0].sum, sizeof(Summary), hipMemcpyDeviceToHost, ctx->stream));
        SV_HIP(hipStreamSynchronize(ctx->stream));
        if (d->gatherfn(d->user, d->h_local, d->host_sum.data(), (int64_t)sizeof(Summary)) != 0)
            throw std::runtime_error("the hosted all-gather failed (sv_gather_fn returned non-zero)");
        return;
    }
    if (d->comm) {
        check_nccl(ncclAllGather(d->tiles[0].sum, d->gathered, sizeof(Summary), ncclChar, d->comm, ctx->stream),
                   "ncclAllGather");
        SV_HIP(hipMemcpyAsync(d->host_sum.data(), d->gathered, ntiles * sizeof(Summary), hipMemcpyDeviceToHost,
                              ctx->stream));
    } else {
        for (int t = 0; t < ntiles; t++)
            SV_HIP(hipMemcpyAsync(&d->host_sum[t], d->tiles[d->local_of[t]].sum, sizeof(Summary),
                                  hipMemcpyDeviceToHost, ctx->stream));
    }
    SV_HIP(hipStreamSynchronize(ctx->stream));
}

// Skip lists of the batch [sw, sw + count) from cursor c0 given the rejected words found by the scan (half-word
// indices from c0's state, sorted): walk the blocks as plan_block does, mapping each bounded block's draw positions
// to half-word indices -- position 0 is the buffered half (from the last u64 of an earlier bounded block) when
// `has`, then the halves of the block's own u64s in order.
void add_predicted(SkipMap &skips, const Cursor &c0, const std::vector<BlockSpec> &specs, int sw, int count,
                   const std::vector<uint64_t> &cand) {
    int64_t j = 0, buf = -1;  // u64 drawn so far; half-word index of the buffered word (-1: before the batch)
    uint32_t has = c0.has;
    const int nb = (int)specs.size();
    for (int k = 0; k < count; k++)
        for (int b = 0; b < nb; b++) {
            const BlockSpec &sp = specs[b];
            if (sp.kind == UNIFORM) {
                j += sp.count;
                continue;
            }
            if (sp.count == 0) continue;
            const auto key = std::make_pair(sw + k, b);
            auto it = skips.find(key);
            std::vector<uint32_t> S = it == skips.end() ? std::vector<uint32_t>{} : it->second;
            std::vector<uint32_t> Pd;
            for (uint64_t c : cand) {
                int64_t p = -1;
                if (has && (int64_t)c == buf) p = 0;
                else if ((int64_t)c >= 2 * j) p = (int64_t)c - 2 * j + has;
                if (p >= 0 && p < (int64_t)sp.count + 2 * MAX_CAND) Pd.push_back((uint32_t)p);
            }
            std::vector<uint32_t> all = S;
            all.insert(all.end(), Pd.begin(), Pd.end());
            std::sort(all.begin(), all.end());
            all.erase(std::unique(all.begin(), all.end()), all.end());
            uint64_t u = sp.count;
            for (;;) {  // words consumed: the draws plus every rejected position met on the way
                const uint64_t z = (uint64_t)std::count_if(all.begin(), all.end(), [&](uint32_t p) { return p < u; });
                if (sp.count + z == u) break;
                u = sp.count + z;
            }
            all.erase(std::remove_if(all.begin(), all.end(), [&](uint32_t p) { return p >= u; }), all.end());
            if (all.size() != S.size()) skips[key] = all;
            const uint64_t rest = u - (has ? 1 : 0), words = (rest + 1) / 2;
            if (rest & 1) buf = 2 * (j + (int64_t)words - 1) + 1;
            j += (int64_t)words;
            has = (uint32_t)(rest & 1);
        }
}

void fill_stats(const sv_domain *d, const SkipMap &skips, int nb, int sw, int count, sv_stats *stats) {
    const int64_t V = (int64_t)d->Nt * d->Nx;
    for (int k = 0; k < count; k++) {
        sv_stats s{0, V, 0.0, 0};
        uint64_t w[3] = {0, 0, 0};  // the tiles' exact acceptance limbs (common.h): the single lattice's statistic
        for (const Summary &S : d->host_sum) {  // global tile order: identical on every rank
            s.accepted += S.stats[k].accepted;
            for (int i = 0; i < 3; i++) w[i] += stat_limb(S.stats[k], i);
        }
        s.acceptance_sum = fx_value(w[0], w[1], w[2]);
        s.rejections = rejections_in(skips, sw + k, nb);
        stats[sw + k] = s;
    }
}

// Sweeps per batch.  A NumPy Lemire rejection anywhere in the (whole, decomposed) lattice aborts the
// batch from its sweep on, and every sweep still queued behind it costs an exchange (RCCL pairs must
// match on every rank, so the ranks cannot stop early) plus three early-exit launches; a batch costs
// one all-gather and a host round trip.  With q rejections expected per sweep (4 V bounded draws of
// threshold thr / 2^32), an aborted sweep costing r sweeps and a batch o sweeps, the overhead per sweep
// is o / B + q (1 + r B / 2), least at B = sqrt(2 o / (q r)): the weak-scaled 2 x 4 lattice
// (8192 x 16384, q = 12.5%) runs batches of ~5 sweeps, one L=4096 tile (q = 1.6%) the full 64.
// SV_DOMAIN_BATCH overrides.
int domain_batch_q(const sv_domain *d, double q) {
    if (const char *e = getenv("SV_DOMAIN_BATCH")) return std::max(1, std::min(DOMAIN_BATCH, atoi(e)));
    if (q <= 0) return DOMAIN_BATCH;
    const double o = 0.3, r = d->nranks > 1 || d->comm ? 0.17 : 0.05;  // measured: RCCL exchange ~50 us, batch ~100 us, sweep 330 us
    const int B = (int)std::lround(std::sqrt(2.0 * o / (q * r)));
    return std::max(4, std::min(DOMAIN_BATCH, B));
}
// Rows per strip of a Villain tile.  A tile of a strong-scaled lattice is small for one GPU (2048 x 1024 per GPU at
// L=4096 on 8): with 52-row strips its 9 x 40 workgroups fill a third of the chip's 1024 slots (4 per CU) and the
// sweep takes one strip's time.  When 52-row strips need at most two rounds of the slots, the strips are cut to
// the shortest height (>= 20 rows, a multiple of 4) that keeps the same number of rounds.  Measured (r343, one
// MI355X, one periodic tile): 2048 x 1024 at 52 / 36 (the single-lattice rule) / 20 rows 72.2 / 65.0 / 55.9 us per
// sweep; 4096 x 2048 at 52 / 36 152.8 / 144.9 us; 4096^2 (three rounds) keeps 52.  SV_FUSED_TH overrides.
//
// 8-wave strips.  When even 52-row strips leave the tile short of one round and 40-row strips of 8 waves (8 rows per
// step, 2 workgroups per CU) fill at most one round of those slots, the tile runs villain_sweep_hot with 8 waves and
// 40-row strips: half the halo rows per row decided.  Measured (r365, one periodic tile): 2048 x 1024 (the per-GPU
// tile at N = 8) 56.0 us with 4 waves x 20 rows, 52.7-52.9 us with 8 waves x 40 rows; 2048 x 2048 75.9 us with 4
// waves x 36 rows, 78.1-99.6 us with 8 waves (kept at 4); the L=4096 single lattice 240 us with 4 waves, 260-279 us
// with 8 (r364).  *nw8 is set when the 8-wave form is chosen.
int domain_th(const sv_domain *d, int nsx, int *nw8 = nullptr) {
    if (nw8) *nw8 = 0;
    if (getenv("SV_FUSED_TH")) return fused_th(d->Ht, nsx);
    static const int slots = [] {
        int dev = 0;
        hipDeviceProp_t prop;
        if (hipGetDevice(&dev) != hipSuccess || hipGetDeviceProperties(&prop, dev) != hipSuccess) return 1024;
        return 4 * prop.multiProcessorCount;
    }();
    auto wgs = [&](int th) { return (int64_t)nsx * ((d->Ht + th - 1) / th); };
    const int64_t rounds = (wgs(52) + slots - 1) / slots;
    // (heights 8k - 3 / 4k + 1: a strip of TH rows takes ceil((TH + 3) / NW) row steps, fused_th; 37 rows of 8 waves
    // take the 5 steps 35 would, 40 took 6)
    constexpr int th8 = 37;
    if (nw8 && rounds == 1 && wgs(th8) <= slots / 2) {
        *nw8 = 1;
        return th8;
    }
    if (rounds > 2) return fused_th(d->Ht, nsx);
    int th = 53;
    while (th > 21 && wgs(th - 4) <= rounds * slots) th -= 4;
    return th;
}

int domain_batch(const sv_domain *d, const VParams &P) {
    const double V = (double)d->Nt * d->Nx;
    const int B = domain_batch_q(d, P.k > 1 ? 4.0 * V * (double)P.thr / 4294967296.0 : 0.0);
    if (getenv("SV_DOMAIN_BATCH")) return B;  // as given (tests: batches shorter than a group)
    const int K = d->depth;  // whole groups of K sweeps per exchange where the batch allows
    return std::min(DOMAIN_BATCH, std::max(K, (B + K / 2) / K * K));
}

void run_domain(sv_domain *d, const VParams &P, int32_t sweeps, Cursor &cur, u128 inc, sv_stats *stats) {
    sv_ctx *ctx = d->ctx;
    const JumpTables *T = ctx->jump_tables(inc.hi, inc.lo);
    const int64_t V = (int64_t)d->Nt * d->Nx;
    const int64_t counts[2] = {V / 2, V / 2};
    const auto specs = villain_specs(V, 2, counts, P.k > 1);
    const int nb = (int)specs.size();
    constexpr int NWv = 4;
    const int nsx = (d->Wt + FW_MAX - 1) / FW_MAX;
    int nw8 = 0;
    const int TH = domain_th(d, nsx, &nw8);
    const int nsy = (d->Ht + TH - 1) / TH;
    const Affine adv[3] = {host_power(inc, (uint64_t)NWv * d->Nx), host_power(inc, (uint64_t)NWv * d->Nx / 2),
                           host_power(inc, (uint64_t)NWv * d->Nx / 4)};
    const int hot_nw = nw8 ? 8 : 4;  // villain_sweep_hot with 8 rows per step (domain_th)
    const Affine adv8[3] = {host_power(inc, 8 * (uint64_t)d->Nx), host_power(inc, 8 * (uint64_t)d->Nx / 2),
                            host_power(inc, 8 * (uint64_t)d->Nx / 4)};
    SkipMap skips;
    std::vector<Block> blocks;
    std::vector<uint32_t> skipvec;
    // rejection prediction (see scan_rejections): the scan of batch b+1 runs behind batch b's sweeps
    // On by default where the ranks split the scan (several RCCL ranks: each scans 1/N of the batch's words, ~3 us
    // per sweep and rank at L=4096 on 8 GPUs, against all-gathers every ~16 sweeps and aborts that drain the rest
    // of a batch); one process scanning a whole lattice pays ~20 us per L=4096 sweep (r348), more than the ~3% the
    // rejections cost there.  SV_DOMAIN_PREDICT=1 / 0 forces it on / off.
    const char *np_env = getenv("SV_DOMAIN_PREDICT");
    const bool predict = P.k > 1 && P.thr > 0 && V >= 256 &&
                         (np_env ? np_env[0] == '1' : d->nranks > 1);
    // unpredicted batches stay short (an abort drains the rest of the batch); predicted ones run the full 64
    const int batch = domain_batch(d, P), full = predict && !getenv("SV_DOMAIN_BATCH") ? DOMAIN_BATCH : batch;
    auto &pred = d->pred;
    sv_domain::Pred next;
    if (pred.valid && pred.sw != 0) pred.valid = false;  // a scan is for the batch a call starts with, or its own
    const Affine per_sweep = host_power(inc, 4 * (uint64_t)V);
    if (predict && !d->d_scan) {
        SV_HIP(hipMalloc(&d->d_scan, DOMAIN_BATCH * sizeof(u128)));
        int least = 0, greatest = 0;
        SV_HIP(hipDeviceGetStreamPriorityRange(&least, &greatest));
        SV_HIP(hipStreamCreateWithPriority(&d->scan_stream, hipStreamNonBlocking, least));
        SV_HIP(hipEventCreateWithFlags(&d->ev_sum, hipEventDisableTiming));
        SV_HIP(hipEventCreateWithFlags(&d->ev_scan, hipEventDisableTiming));
    }
    std::vector<u128> h_scan(DOMAIN_BATCH);
    // scan the choice words of n sweeps from cursor `from` on `stream`: the scan is split into one part per tile --
    // each rank scans its own share into its summary (the words found travel in the summaries the ranks all-gather),
    // and one process emulating a tile grid runs every tile's share into that tile's summary: the same partition
    // and merge as several ranks
    auto launch_scan = [&](const Cursor &from, int n, hipStream_t stream) {
        u128 sk = from.s;
        for (int k = 0; k < n; k++) {
            h_scan[k] = sk;
            sk = apply(per_sweep, sk);
        }
        SV_HIP(hipMemcpyAsync(d->d_scan, h_scan.data(), n * sizeof(u128), hipMemcpyHostToDevice, stream));
        const uint64_t total = (uint64_t)n * 2 * ((uint64_t)V + 2 * SCAN_MARGIN);
        const int parts = d->nranks > 1 ? d->nranks : (int)d->tiles.size();
        for (size_t li = 0; li < d->tiles.size(); li++) {
            const int me = d->nranks > 1 ? d->rank : (int)li;
            ScanArgs a;
            a.s_k = d->d_scan;
            a.T = T;
            a.V = (uint64_t)V;
            a.lo = total * me / parts;
            a.hi = total * (me + 1) / parts;
            a.k = P.k;
            a.thr = P.thr;
            a.ncand = &d->tiles[li].sum->ncand;
            a.cand = d->tiles[li].sum->cand;
            const uint64_t lanes = (a.hi - a.lo + SCAN_CHUNK - 1) / SCAN_CHUNK;
            if (lanes) scan_rejections<<<(unsigned)((lanes + 255) / 256), 256, 0, stream>>>(a), SV_LAUNCHED("scan_rejections", stream);
        }
    };
    // the finds of every part (gathered summaries, global tile order), sorted; false if a part overflowed
    auto merge_cand = [&](std::vector<uint64_t> &cand) {
        cand.clear();
        bool over = false;
        for (const Summary &S : d->host_sum) {
            over |= S.ncand > (uint32_t)MAX_CAND;
            cand.insert(cand.end(), S.cand, S.cand + std::min<uint32_t>(S.ncand, MAX_CAND));
        }
        std::sort(cand.begin(), cand.end());
        cand.erase(std::unique(cand.begin(), cand.end()), cand.end());
        return !over;
    };
    int predicted_batches = 0, prescanned = 0, aborts = 0, predicted_aborts = 0;
    // |n| beyond villain_sweep_hot's int16 image (|n| >= 2^14): the failing sweep is replayed, and the rest of the
    // call runs, on villain_sweep_fused's int32 image -- the single-lattice driver's fallback (run_fused)
    bool no_hot = false;
    int sw = 0;
    while (sw < sweeps) {
        int count = std::min(batch, sweeps - sw);
        bool predicted = false;
        if (pred.valid && pred.sw == sw && pred.c.s.lo == cur.s.lo && pred.c.s.hi == cur.s.hi && pred.c.has == cur.has &&
            pred.inc.lo == inc.lo && pred.inc.hi == inc.hi && pred.k == P.k && pred.thr == P.thr) {
            count = std::min(sweeps - sw, pred.count);
            add_predicted(skips, cur, specs, sw, count, pred.cand);
            predicted_batches++;
            predicted = true;
        } else if (predict) {
            // no scan ran ahead of this batch (a call's first batch, or the replay after an abort): scan it now, in
            // front of it (one more scan and all-gather), so that it runs predicted and full-length too
            const int n = std::min(full, sweeps - sw);
            for (auto &Tl : d->tiles) SV_HIP(hipMemsetAsync(Tl.sum, 0, sizeof(Summary), ctx->stream));
            launch_scan(cur, n, ctx->stream);
            SV_HIP(hipGetLastError());
            gather(d);
            std::vector<uint64_t> cand;
            if (merge_cand(cand)) {
                count = n;
                add_predicted(skips, cur, specs, sw, count, cand);
                predicted_batches++;
                prescanned++;
                predicted = true;
            }
        }
        pred.valid = false;
        Cursor c = cur;
        plan_sweeps(ctx, c, inc, specs, sw, count, skips, blocks, skipvec);
        std::vector<char> hot(count);
        // (villain_sweep_hot's 32-bit row offsets: 16 plane < 2^32)
        for (int k = 0; k < count; k++)
            hot[k] = !no_hot && d->plane < (int64_t(1) << 28) && hot_ok(P, &blocks[(size_t)k * nb]);
        // sweeps with known (predicted or reported) rejections, at most one per choice block: the split replay
        // (villain_sweep_hot_split in tile mode), its descriptors after the switches uploaded with the batch's plan
        std::vector<int> split_i(count, -1);
        std::vector<SplitArgs> splits;
        std::vector<size_t> split_off;
        for (int k = 0; k < count; k++) {
            if (hot[k] || no_hot || d->plane >= (int64_t(1) << 28) || nb != 11) continue;
            SplitArgs SA;
            Block Bset[11];
            if (!split_plan(P, &blocks[(size_t)k * nb], skipvec.data(), inc, SA, Bset)) continue;
            split_i[k] = (int)splits.size();
            splits.push_back(SA);
            split_off.push_back(blocks.size());
            blocks.insert(blocks.end(), Bset, Bset + 11);
        }
        upload_plan(ctx, blocks, skipvec);
        for (auto &Tl : d->tiles) SV_HIP(hipMemsetAsync(Tl.sum, 0, sizeof(Summary), ctx->stream));
        if (predict) SV_HIP(hipEventRecord(d->ev_sum, ctx->stream));
        const int cur0 = d->cur;
        auto fargs = [&](sv_domain_tile &Tl, int k, int in, int out) {
            FArgs A;
            A.P = P;
            A.G = FGeom{d->Nt, d->Nx, Tl.T0, Tl.X0, d->Ht, d->Wt, d->pitch, d->plane, d->org};
            A.phi_in = Tl.phi[in];
            A.n_in = Tl.n[in];
            A.phi_out = Tl.phi[out];
            A.n_out = Tl.n[out];
            A.nsx = nsx;
            A.TH = TH;
            A.nsy = nsy;
            A.blocks = ctx->d_blocks + (size_t)k * nb;
            A.skips = ctx->d_skips;
            A.T = T;
            A.adv[0] = adv[0];
            A.adv[1] = adv[1];
            A.adv[2] = adv[2];
            A.stat = &Tl.sum->stats[k];
            A.S = DevScratch{&Tl.sum->abort, &Tl.sum->nreport, Tl.sum->reports};
            A.sweep = (uint32_t)k;
            farg_single(A, nsx, nsy);
            if (hot[k] && hot_nw == 8) {
                A.hot_nw = 8;
                A.adv[0] = adv8[0];
                A.adv[1] = adv8[1];
                A.adv[2] = adv8[2];
            }
            return A;
        };
        hipEvent_t ev;
        ctx->time_begin(&ev);
        for (int k = 0; k < count; k++) {
            const int in = d->cur, out = (d->cur + 1) % d->R;
            // deep halos: one exchange per group of K sweeps; sweep j of a group of g decides the tile extended
            // by e = g-1-j rings of (2 above, 3 below, 2 left, 3 right), counting only the tile's own sites
            const int K = d->depth, g0 = k - k % K, e = std::min(K, count - g0) - 1 - (k - g0);
            if (k == g0) exchange(d, ctx->stream);
            for (auto &Tl : d->tiles) {
                FArgs A = fargs(Tl, k, in, out);
                if (e > 0) {
                    const int32_t up = 2 * e, left = 2 * e;
                    A.G.T0 = (Tl.T0 - up + d->Nt) % d->Nt;
                    A.G.X0 = (Tl.X0 - left + d->Nx) % d->Nx;
                    A.G.Ht = d->Ht + 5 * e;
                    A.G.Wt = d->Wt + 5 * e;
                    A.G.org = d->org - (int64_t)up * d->pitch - left;
                    A.nsx = (A.G.Wt + FW_MAX - 1) / FW_MAX;
                    A.nsy = (A.G.Ht + TH - 1) / TH;
                    A.tiles_per_rep = A.nsx * A.nsy;
                    A.own_r0 = up;
                    A.own_r1 = up + d->Ht;
                    A.own_c0 = left;
                    A.own_c1 = left + d->Wt;
                }
                int grid = A.nsx * A.nsy;
                // (two waves of strips, taller for the workgroups dispatched first, measured slower than uniform strips:
                // 50.8 / 50.9 vs 49.5 / 49.6 us per 2048 x 1024 tile sweep, r4 profiles/r04_tile_ab.txt)
                if (split_i[k] >= 0) {
                    SplitArgs SA = splits[split_i[k]];
                    SA.blocksB = ctx->d_blocks + split_off[split_i[k]];
                    // (tiles run uniform strips: no strip table -- split_order reads one on the host, never A.strips,
                    // which is a device pointer)
                    split_order(SA, A.G, A.nsx, A.TH, grid, nullptr);
                    launch_hot_split(A, SA, grid, ctx->stream);
                    ctx->sweeps_split++;
                } else {
                    launch_fused_tile(A, grid, ctx->stream, hot[k]);
                    (hot[k] ? ctx->sweeps_hot : ctx->sweeps_fused)++;
                }
            }
            d->cur = out;
        }
        ctx->time_end(ev, count);
        // scan the words of the next batch (from this batch's end cursor c) for NumPy rejections; this rank's share
        // (past the end of the call: as many sweeps as this batch, for the batch the next call starts with)
        next.valid = false;
        const int ncount = sweeps - sw - count > 0 ? std::min(full, sweeps - sw - count) : std::min(full, count);
        if (predict && ncount > 0) {
            // on the low-priority stream, after this batch's summary was cleared; the gather waits for it
            SV_HIP(hipStreamWaitEvent(d->scan_stream, d->ev_sum, 0));
            launch_scan(c, ncount, d->scan_stream);
            SV_HIP(hipEventRecord(d->ev_scan, d->scan_stream));
            SV_HIP(hipStreamWaitEvent(ctx->stream, d->ev_scan, 0));
            next.valid = true;
            next.sw = sw + count < sweeps ? sw + count : 0;
            next.count = ncount;
            next.c = c;
            next.inc = inc;
            next.k = P.k;
            next.thr = P.thr;
        }
        SV_HIP(hipGetLastError());
        gather(d);
        AbortInfo a{0, {}};
        for (const Summary &S : d->host_sum) {
            a.abort |= S.abort;
            const uint32_t nr = std::min<uint32_t>(S.nreport, MAX_REPORTS);
            a.reports.insert(a.reports.end(), S.reports, S.reports + nr);
        }
        if (a.abort) ctx->time_discard();
        ctx->time_collect();
        if (!a.abort) {
            fill_stats(d, skips, nb, sw, count, stats);
            cur = c;
            sw += count;
            if (next.valid && merge_cand(next.cand)) pred = next;  // (an overflowing scan: abort protocol)
            continue;
        }
        aborts++;
        predicted_aborts += predicted;
        // an overflow report: the sweeps before it stand, the failing one is replayed on the int32 kernel (a
        // rejection report of an earlier sweep, or of the same sweep, is absorbed first as usual)
        uint32_t ovf = ~0u;
        for (const Report &r : a.reports)
            if (r.block == OVERFLOW_BLOCK) ovf = std::min(ovf, r.sweep);
        if (ovf != ~0u) {
            if (no_hot) throw std::runtime_error("|n| exceeds villain_sweep_fused's int32 LDS image (|n| < 2^30 required)");
            no_hot = true;
            a.reports.erase(std::remove_if(a.reports.begin(), a.reports.end(),
                                           [&](const Report &r) { return r.block == OVERFLOW_BLOCK || r.sweep > ovf; }),
                            a.reports.end());
        }
        const int bad = a.reports.empty() ? (int)ovf : absorb_reports(a, sw, skips);
        if (bad > 0) {
            Cursor c2 = cur;
            std::vector<Block> b2;
            std::vector<uint32_t> s2;
            plan_sweeps(ctx, c2, inc, specs, sw, bad, skips, b2, s2);
            fill_stats(d, skips, nb, sw, bad, stats);
            cur = c2;
        }
        d->cur = (cur0 + bad) % d->R;
        sw += bad;
    }
    if (getenv("SV_DEBUG_TIMING"))
        fprintf(stderr, "[sv domain] %d sweeps, batch %d, depth %d, predicted batches %d (%d pre-scanned), aborts %d (%d in "
                "predicted batches)\n", sweeps, batch, d->depth, predicted_batches, prescanned, aborts, predicted_aborts);
}

// Worldline (config 3 decomposed): one step = checkerboard PlaquetteUpdate sweep + CoexactUpdate
// sweep, run per tile by worldline_step_fused in tile mode after one halo exchange of (v, m0, m1) with the
// 5/4-wide ghost frame.  Same batch / abort / replay protocol as run_domain; two statistics per step.
void run_wdomain(sv_domain *d, double kappa, double W_eff, int64_t it, int32_t steps, Cursor &cur, u128 inc,
                 sv_stats *stats) {
    sv_ctx *ctx = d->ctx;
    const JumpTables *T = ctx->jump_tables(inc.hi, inc.lo);
    const int64_t V = (int64_t)d->Nt * d->Nx;
    const uint32_t half = (uint32_t)(V / 2);
    // worldline.hip plaquette_cb_specs + coexact_specs (even lattices: two colours of V/2 plaquettes)
    const std::vector<BlockSpec> specs = {{UNIFORM, (uint32_t)V}, {BOUNDED, half}, {BOUNDED, half}, {BOUNDED, half},
                                          {BOUNDED, half}, {UNIFORM, (uint32_t)V}, {BOUNDED, half}, {BOUNDED, half}};
    const int nb = (int)specs.size();
    const Affine adv[6] = {host_power(inc, 4 * (uint64_t)d->Nx), host_power(inc, 2 * (uint64_t)d->Nx),
                           host_power(inc, (uint64_t)d->Nx), host_power(inc, 8 * (uint64_t)d->Nx),
                           host_power(inc, 4 * (uint64_t)d->Nx), host_power(inc, 2 * (uint64_t)d->Nx)};
    // rejections possible in the change_v blocks (threshold 1) and, for interval_t > 2, the t blocks
    const uint32_t kt = (uint32_t)(2 * it), thrt = (0u - kt) % kt;
    const double q = (double)V * (1.0 + (double)thrt) / 4294967296.0;
    const int batch = domain_batch_q(d, q);
    SkipMap skips;
    std::vector<Block> blocks;
    std::vector<uint32_t> skipvec;
    auto fill = [&](int sw, int count) {
        for (int k = 0; k < count; k++)
            for (int j = 0; j < 2; j++) {
                sv_stats st{0, V, 0.0, 0};
                uint64_t w[3] = {0, 0, 0};  // exact acceptance limbs (common.h)
                for (const Summary &S : d->host_sum) {
                    st.accepted += S.stats[2 * k + j].accepted;
                    for (int i = 0; i < 3; i++) w[i] += stat_limb(S.stats[2 * k + j], i);
                }
                st.acceptance_sum = fx_value(w[0], w[1], w[2]);
                for (int bi = j == 0 ? 0 : 5; bi < (j == 0 ? 5 : nb); bi++) {
                    auto itk = skips.find({sw + k, bi});
                    if (itk != skips.end()) st.rejections += (int64_t)itk->second.size();
                }
                stats[2 * (sw + k) + j] = st;
            }
    };
    int sw = 0;
    while (sw < steps) {
        const int count = std::min(batch, steps - sw);
        Cursor c = cur;
        plan_sweeps(ctx, c, inc, specs, sw, count, skips, blocks, skipvec);
        upload_plan(ctx, blocks, skipvec);
        for (auto &Tl : d->tiles) {
            SV_HIP(hipMemsetAsync(Tl.sum, 0, sizeof(Summary), ctx->stream));
            SV_HIP(hipMemsetAsync(Tl.stripes, 0, (size_t)count * 2 * NSTRIPE * sizeof(StatStripe), ctx->stream));
        }
        const int cur0 = d->cur;
        hipEvent_t ev;
        ctx->time_begin(&ev);
        for (int k = 0; k < count; k++) {
            const int in = d->cur, out = (d->cur + 1) % d->R;
            exchange(d, ctx->stream);
            const bool general = !wf_fast(&blocks[(size_t)k * nb]);
            for (auto &Tl : d->tiles)
                launch_wf(FGeom{d->Nt, d->Nx, Tl.T0, Tl.X0, d->Ht, d->Wt, d->pitch, d->plane, d->org}, kappa, W_eff, it,
                          Tl.n[in], (const int64_t *)Tl.phi[in], Tl.n[out], (int64_t *)Tl.phi[out],
                          ctx->d_blocks + (size_t)k * nb, &blocks[(size_t)k * nb], ctx->d_skips, general, T, adv, inc,
                          Tl.stripes + (size_t)k * 2 * NSTRIPE, Tl.stripes + (size_t)k * 2 * NSTRIPE + NSTRIPE,
                          DevScratch{&Tl.sum->abort, &Tl.sum->nreport, Tl.sum->reports}, (uint32_t)k, ctx->stream);
            d->cur = out;
        }
        for (auto &Tl : d->tiles) wd_fold<<<(2 * count + 63) / 64, 64, 0, ctx->stream>>>(Tl.stripes, Tl.sum->stats, 2 * count), SV_LAUNCHED("wd_fold", ctx->stream);
        ctx->time_end(ev, count);
        SV_HIP(hipGetLastError());
        gather(d);
        AbortInfo a{0, {}};
        for (const Summary &S : d->host_sum) {
            a.abort |= S.abort;
            const uint32_t nr = std::min<uint32_t>(S.nreport, MAX_REPORTS);
            a.reports.insert(a.reports.end(), S.reports, S.reports + nr);
        }
        if (a.abort) ctx->time_discard();
        ctx->time_collect();
        if (!a.abort) {
            fill(sw, count);
            cur = c;
            sw += count;
            continue;
        }
        for (const Report &r : a.reports)
            if (r.block == OVERFLOW_BLOCK)
                throw std::runtime_error("|m| or |v| exceeds worldline_step_fused's int32 LDS image (domain mode has no fallback)");
        const int bad = absorb_reports(a, sw, skips);
        if (bad > 0) {
            Cursor c2 = cur;
            std::vector<Block> b2;
            std::vector<uint32_t> s2;
            plan_sweeps(ctx, c2, inc, specs, sw, bad, skips, b2, s2);
            fill(sw, bad);
            cur = c2;
        }
        d->cur = (cur0 + bad) % d->R;
        sw += bad;
    }
}

}  // namespace

// ---------------------------------------------------------------------------------------- C-ABI
extern "C" {

int sv_domain_unique_id(uint8_t *id) {
    if (!id) return -1;
    ncclUniqueId u;
    if (ncclGetUniqueId(&u) != ncclSuccess) return -2;
    std::memcpy(id, u.internal, NCCL_UNIQUE_ID_BYTES);
    return 0;
}

static int exchange_plan_impl(int model, int32_t Nt, int32_t Nx, int32_t tiles_t, int32_t tiles_x, int32_t rank,
                              int64_t *out) {
    try {
        if (!out || tiles_t < 1 || tiles_x < 1 || rank < 0 || rank >= tiles_t * tiles_x) return -1;
        sv_domain d;
        d.model = model;
        d.ghost = model == 1 ? WORLDLINE_GHOST : VILLAIN_GHOST;
        d.Nt = Nt;
        d.Nx = Nx;
        d.ty = tiles_t;
        d.tx = tiles_x;
        geometry(&d);
        const int iy = rank / tiles_x, ix = rank % tiles_x;
        for (int s = 0; s < NDIR; s++) {
            int dy, dx;
            dir_of(s, dy, dx);
            const Rect S = send_rect(s, d.Ht, d.Wt, d.ghost), Rr = recv_rect(s, d.Ht, d.Wt, d.ghost);
            int64_t *o = out + 10 * s;
            o[0] = dy;
            o[1] = dx;
            o[2] = tile_index(&d, iy + dy, ix + dx);  // send to
            o[3] = S.r0;
            o[4] = S.c0;
            o[5] = S.rows;
            o[6] = S.cols;
            o[7] = tile_index(&d, iy - dy, ix - dx);  // receive the message of direction s from
            o[8] = Rr.r0;
            o[9] = Rr.c0;
        }
        return 0;
    } catch (const std::exception &) {
        return -2;
    }
}

static int message_layout_impl(int model, int32_t Nt, int32_t Nx, int32_t tiles_t, int32_t tiles_x, int32_t rank,
                               int64_t *out) {
    try {
        if (!out || tiles_t < 1 || tiles_x < 1 || rank < 0 || rank >= tiles_t * tiles_x) return -1;
        sv_domain d;
        d.model = model;
        d.ghost = model == 1 ? WORLDLINE_GHOST : VILLAIN_GHOST;
        d.Nt = Nt;
        d.Nx = Nx;
        d.ty = tiles_t;
        d.tx = tiles_x;
        d.nranks = tiles_t * tiles_x;
        d.rank = rank;
        geometry(&d);
        build_tiles(&d);
        halo_layout(&d);
        const sv_domain_tile &T = d.tiles[0];
        int64_t *o = out;
        *o++ = (int64_t)T.sends.size();
        *o++ = (int64_t)T.recvs.size();
        for (const auto &m : T.sends) o = std::copy(m.begin(), m.end(), o);
        for (const auto &m : T.recvs) o = std::copy(m.begin(), m.end(), o);
        o = std::copy(T.soff, T.soff + NDIR, o);
        o = std::copy(T.roff, T.roff + NDIR, o);
        for (int s = 0; s < NDIR; s++) *o++ = 2 + 3 * (int64_t)d.H.rect[s].rows * d.H.rect[s].cols;
        *o++ = d.msg_words;
        return 0;
    } catch (const std::exception &) {
        return -2;
    }
}

int sv_domain_exchange_plan(int32_t Nt, int32_t Nx, int32_t tiles_t, int32_t tiles_x, int32_t rank, int64_t *out) {
    return exchange_plan_impl(0, Nt, Nx, tiles_t, tiles_x, rank, out);
}
int sv_domain_exchange_plan_worldline(int32_t Nt, int32_t Nx, int32_t tiles_t, int32_t tiles_x, int32_t rank,
                                      int64_t *out) {
    return exchange_plan_impl(1, Nt, Nx, tiles_t, tiles_x, rank, out);
}
int sv_domain_message_layout(int32_t Nt, int32_t Nx, int32_t tiles_t, int32_t tiles_x, int32_t rank, int64_t *out) {
    return message_layout_impl(0, Nt, Nx, tiles_t, tiles_x, rank, out);
}
int sv_domain_message_layout_worldline(int32_t Nt, int32_t Nx, int32_t tiles_t, int32_t tiles_x, int32_t rank,
                                       int64_t *out) {
    return message_layout_impl(1, Nt, Nx, tiles_t, tiles_x, rank, out);
}

static int domain_create(sv_ctx *ctx, int model, int32_t Nt, int32_t Nx, int32_t tiles_t, int32_t tiles_x,
                         int32_t nranks, int32_t rank, const uint8_t *unique_id, sv_domain **out,
                         sv_xfer_fn xfer = nullptr, sv_gather_fn gatherfn = nullptr, void *user = nullptr) {
    if (!ctx || !out) return -1;
    *out = nullptr;
    sv_domain *d = new sv_domain();
    try {
        SV_HIP(hipSetDevice(ctx->device));
        d->ctx = ctx;
        d->model = model;
        d->xfer = xfer;
        d->gatherfn = gatherfn;
        d->user = user;
        d->ghost = model == 1 ? WORLDLINE_GHOST : VILLAIN_GHOST;
        d->Nt = Nt;
        d->Nx = Nx;
        d->ty = tiles_t;
        d->tx = tiles_x;
        d->nranks = nranks;
        d->rank = rank;
        if (tiles_t < 1 || tiles_x < 1) throw std::invalid_argument("tile grid must be at least 1 x 1");
        if (nranks < 1 || rank < 0 || rank >= nranks) throw std::invalid_argument("bad rank / nranks");
        if (nranks > 1 && nranks != tiles_t * tiles_x)
            throw std::invalid_argument("with several ranks, each rank owns exactly one tile (nranks == tiles_t * tiles_x)");
        if ((xfer == nullptr) != (gatherfn == nullptr)) throw std::invalid_argument("a hosted transport needs both callbacks");
        if (xfer && unique_id) throw std::invalid_argument("a hosted transport takes no RCCL unique id");
        if (nranks > 1 && !unique_id && !xfer)
            throw std::invalid_argument("a unique id (sv_domain_unique_id on rank 0) is required");
        d->loopback = nranks == 1 && unique_id != nullptr;
        if (d->loopback && tiles_t * tiles_x != 1) throw std::invalid_argument("RCCL loopback mode needs a 1 x 1 tile grid");
        geometry(d);
        build_tiles(d);
        halo_layout(d);
        for (auto &T : d->tiles) {
            T.phi.assign(d->R, nullptr);
            T.n.assign(d->R, nullptr);
            for (int i = 0; i < d->R; i++) {
                SV_HIP(hipMalloc(&T.phi[i], d->plane * sizeof(double)));
                SV_HIP(hipMalloc(&T.n[i], 2 * d->plane * sizeof(int64_t)));
                SV_HIP(hipMemset(T.phi[i], 0, d->plane * sizeof(double)));
                SV_HIP(hipMemset(T.n[i], 0, 2 * d->plane * sizeof(int64_t)));
            }
            SV_HIP(hipMalloc(&T.send, d->msg_words * sizeof(uint64_t)));
            SV_HIP(hipMalloc(&T.recv, d->msg_words * sizeof(uint64_t)));
            SV_HIP(hipMemset(T.recv, 0, d->msg_words * sizeof(uint64_t)));
            SV_HIP(hipMalloc(&T.sum, sizeof(Summary)));
            SV_HIP(hipMemset(T.sum, 0, sizeof(Summary)));
            if (model == 1) SV_HIP(hipMalloc(&T.stripes, (size_t)DOMAIN_BATCH * 2 * NSTRIPE * sizeof(StatStripe)));
        }
        if (xfer) {
            SV_HIP(hipHostMalloc((void **)&d->h_send, std::max<int64_t>(d->msg_words, 1) * sizeof(uint64_t),
                                 hipHostMallocDefault));
            SV_HIP(hipHostMalloc((void **)&d->h_recv, std::max<int64_t>(d->msg_words, 1) * sizeof(uint64_t),
                                 hipHostMallocDefault));
            SV_HIP(hipHostMalloc((void **)&d->h_local, sizeof(Summary), hipHostMallocDefault));
            std::memset(d->h_recv, 0, std::max<int64_t>(d->msg_words, 1) * sizeof(uint64_t));
        } else if (nranks > 1 || d->loopback) {
            ncclUniqueId u;
            std::memcpy(u.internal, unique_id, NCCL_UNIQUE_ID_BYTES);
            check_nccl(ncclCommInitRank(&d->comm, nranks, u, rank), "ncclCommInitRank");
            SV_HIP(hipMalloc(&d->gathered, (size_t)nranks * sizeof(Summary)));
        }
        SV_HIP(hipDeviceSynchronize());
        *out = d;
        return 0;
    } catch (const std::exception &e) {
        ctx->err = e.what();
        sv_domain_destroy(d);
        return -2;
    }
}

int sv_domain_create(sv_ctx *ctx, int32_t Nt, int32_t Nx, int32_t tiles_t, int32_t tiles_x, int32_t nranks,
                     int32_t rank, const uint8_t *unique_id, sv_domain **out) {
    return domain_create(ctx, 0, Nt, Nx, tiles_t, tiles_x, nranks, rank, unique_id, out);
}

static int worldline_limits(sv_ctx *ctx, int32_t Nt, int32_t Nx);
static int worldline_tile_limit(sv_ctx *ctx, int rc, sv_domain **out);

int sv_domain_create_hosted(sv_ctx *ctx, int32_t model, int32_t Nt, int32_t Nx, int32_t tiles_t, int32_t tiles_x,
                            int32_t nranks, int32_t rank, sv_xfer_fn xfer, sv_gather_fn gather, void *user,
                            sv_domain **out) {
    if (!xfer || !gather || (model != 0 && model != 1)) {
        if (ctx) ctx->err = "sv_domain_create_hosted: model 0 or 1 and both callbacks are required";
        return -2;
    }
    if (model == 1 && worldline_limits(ctx, Nt, Nx) != 0) return -2;
    const int rc = domain_create(ctx, model, Nt, Nx, tiles_t, tiles_x, nranks, rank, nullptr, out, xfer, gather, user);
    return model == 1 ? worldline_tile_limit(ctx, rc, out) : rc;
}

static int worldline_limits(sv_ctx *ctx, int32_t Nt, int32_t Nx) {
    if (Nt % 2 || Nx % 2) {
        if (ctx) ctx->err = "the Worldline decomposition needs even lattice extents";
        return -2;
    }
    // worldline_step_fused (the decomposition's only kernel) addresses stream positions with 31 bits and moves rows by
    // 32-bit byte offsets: refuse here, before any exchange is enqueued, what its first launch would
    if ((int64_t)Nt * Nx >= (int64_t(1) << 31)) {
        if (ctx) ctx->err = "the Worldline decomposition needs Nt * Nx < 2^31 (worldline_step_fused's 31-bit positions)";
        return -2;
    }
    return 0;
}

// (a Worldline domain whose tiles exceed worldline_step_fused's 32-bit row offsets is refused after its geometry is known)
static int worldline_tile_limit(sv_ctx *ctx, int rc, sv_domain **out) {
    if (rc == 0 && (*out)->plane >= (int64_t(1) << 28)) {
        (void)sv_domain_destroy(*out);
        *out = nullptr;
        ctx->err = "the Worldline decomposition needs tiles of < 2^28 sites with their ghost frames (worldline_step_fused's "
                   "32-bit row offsets): use more tiles";
        return -2;
    }
    return rc;
}

int sv_domain_create_worldline(sv_ctx *ctx, int32_t Nt, int32_t Nx, int32_t tiles_t, int32_t tiles_x, int32_t nranks,
                               int32_t rank, const uint8_t *unique_id, sv_domain **out) {
    if (worldline_limits(ctx, Nt, Nx) != 0) return -2;
    return worldline_tile_limit(ctx, domain_create(ctx, 1, Nt, Nx, tiles_t, tiles_x, nranks, rank, unique_id, out), out);
}

int sv_domain_destroy(sv_domain *d) {
    if (!d) return 0;
    // both streams drain BEFORE anything is freed: a rejection scan running behind the last batch on scan_stream
    // writes its tile's Summary (T.sum) and reads d_scan
    const int rc = sv_destroy_drain(d->ctx, "sv_domain_destroy", d->scan_stream);
    for (auto &T : d->tiles) {
        for (auto p : T.phi) (void)hipFree(p);
        for (auto p : T.n) (void)hipFree(p);
        (void)hipFree(T.send);
        (void)hipFree(T.recv);
        (void)hipFree(T.sum);
        (void)hipFree(T.stripes);
    }
    if (d->comm) (void)ncclCommDestroy(d->comm);
    if (d->h_send) (void)hipHostFree(d->h_send);
    if (d->h_recv) (void)hipHostFree(d->h_recv);
    if (d->h_local) (void)hipHostFree(d->h_local);
    (void)hipFree(d->gathered);
    (void)hipFree(d->d_scan);
    if (d->scan_stream) (void)hipStreamDestroy(d->scan_stream);
    if (d->ev_sum) (void)hipEventDestroy(d->ev_sum);
    if (d->ev_scan) (void)hipEventDestroy(d->ev_scan);
    delete d;
    return rc;
}

int sv_domain_upload(sv_domain *d, const double *phi, const int64_t *n) {
    if (!d) return -1;
    sv_ctx *ctx = d->ctx;
    try {
        SV_HIP(hipSetDevice(ctx->device));
        const int64_t V = (int64_t)d->Nt * d->Nx;
        for (auto &T : d->tiles) {
            if (!phi || !n) {
                SV_HIP(hipMemsetAsync(T.phi[d->cur], 0, d->plane * sizeof(double), ctx->stream));
                SV_HIP(hipMemsetAsync(T.n[d->cur], 0, 2 * d->plane * sizeof(int64_t), ctx->stream));
                continue;
            }
            const int64_t g0 = (int64_t)T.T0 * d->Nx + T.X0;
            SV_HIP(hipMemcpy2DAsync(T.phi[d->cur] + d->org, d->pitch * sizeof(double), phi + g0, d->Nx * sizeof(double),
                                    d->Wt * sizeof(double), d->Ht, hipMemcpyHostToDevice, ctx->stream));
            for (int c = 0; c < 2; c++)
                SV_HIP(hipMemcpy2DAsync(T.n[d->cur] + c * d->plane + d->org, d->pitch * sizeof(int64_t), n + c * V + g0,
                                        d->Nx * sizeof(int64_t), d->Wt * sizeof(int64_t), d->Ht, hipMemcpyHostToDevice,
                                        ctx->stream));
        }
        SV_HIP(hipStreamSynchronize(ctx->stream));
        return 0;
    } catch (const std::exception &e) {
        ctx->err = e.what();
        return -2;
    }
}

int sv_domain_download(sv_domain *d, double *phi, int64_t *n) {
    if (!d || !phi || !n) return -1;
    sv_ctx *ctx = d->ctx;
    try {
        SV_HIP(hipSetDevice(ctx->device));
        const int64_t V = (int64_t)d->Nt * d->Nx;
        for (auto &T : d->tiles) {
            const int64_t g0 = (int64_t)T.T0 * d->Nx + T.X0;
            SV_HIP(hipMemcpy2DAsync(phi + g0, d->Nx * sizeof(double), T.phi[d->cur] + d->org, d->pitch * sizeof(double),
                                    d->Wt * sizeof(double), d->Ht, hipMemcpyDeviceToHost, ctx->stream));
            for (int c = 0; c < 2; c++)
                SV_HIP(hipMemcpy2DAsync(n + c * V + g0, d->Nx * sizeof(int64_t), T.n[d->cur] + c * d->plane + d->org,
                                        d->pitch * sizeof(int64_t), d->Wt * sizeof(int64_t), d->Ht,
                                        hipMemcpyDeviceToHost, ctx->stream));
        }
        SV_HIP(hipStreamSynchronize(ctx->stream));
        return 0;
    } catch (const std::exception &e) {
        ctx->err = e.what();
        return -2;
    }
}

int sv_domain_run(sv_domain *d, double kappa, int64_t W, double interval_phi, int64_t interval_n, int32_t sweeps,
                  sv_rng *rng, sv_stats *stats) {
    if (!d || !rng || (sweeps > 0 && !stats)) return -1;
    sv_ctx *ctx = d->ctx;
    try {
        if (d->model != 0) throw std::invalid_argument("sv_domain_run runs a Villain domain (sv_domain_create)");
        if (sweeps < 0) throw std::invalid_argument("sweeps must be >= 0");
        if (interval_n < 0 || interval_n > (1 << 20)) throw std::invalid_argument("interval_n out of range");
        if ((W < 0 ? -W : W) * interval_n >= (1LL << 28)) throw std::invalid_argument("|W * interval_n| too large");
        SV_HIP(hipSetDevice(ctx->device));
        VParams P = make_params(d->Nx, kappa, W, interval_phi, interval_n);
        u128 inc{rng->inc_lo, rng->inc_hi};
        Cursor cur{u128{rng->state_lo, rng->state_hi}, (uint32_t)rng->has_uint32, rng->uinteger};
        run_domain(d, P, sweeps, cur, inc, stats);
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

int sv_domain_upload_worldline(sv_domain *d, const int64_t *m, const int64_t *v) {
    if (!d) return -1;
    if (d->model != 1) {
        d->ctx->err = "not a Worldline domain";
        return -2;
    }
    return sv_domain_upload(d, (const double *)v, m);  // the 8-byte planes are moved as bits
}

int sv_domain_download_worldline(sv_domain *d, int64_t *m, int64_t *v) {
    if (!d) return -1;
    if (d->model != 1) {
        d->ctx->err = "not a Worldline domain";
        return -2;
    }
    return sv_domain_download(d, (double *)v, m);
}

int sv_domain_run_worldline(sv_domain *d, double kappa, double W_eff, int64_t interval_t, int32_t steps, sv_rng *rng,
                            sv_stats *stats) {
    if (!d || !rng || (steps > 0 && !stats)) return -1;
    sv_ctx *ctx = d->ctx;
    try {
        if (d->model != 1) throw std::invalid_argument("sv_domain_run_worldline runs a Worldline domain");
        if (steps < 0) throw std::invalid_argument("steps must be >= 0");
        if (!wf_usable(d->Nx, false, W_eff, interval_t) || d->Nt % 2)
            throw std::invalid_argument("the decomposed Worldline step needs W a power of two and 1 <= interval_t <= 2^20");
        SV_HIP(hipSetDevice(ctx->device));
        u128 inc{rng->inc_lo, rng->inc_hi};
        Cursor cur{u128{rng->state_lo, rng->state_hi}, (uint32_t)rng->has_uint32, rng->uinteger};
        run_wdomain(d, kappa, W_eff, interval_t, steps, cur, inc, stats);
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

}  // extern "C"
