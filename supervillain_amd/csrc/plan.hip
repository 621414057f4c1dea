// plan.hip -- host side of the stream replay: PCG64 jumps, block planning, jump tables, colourings.
#include <algorithm>
#include <unordered_map>

#include "common.h"

namespace sv {

static Affine power(Affine f, uint64_t k) {
    Affine r = identity();
    while (k) {
        if (k & 1) r = compose(f, r);
        f = compose(f, f);
        k >>= 1;
    }
    return r;
}

// The planner jumps by the same few distances over and over (a block's draws, its words, one step): the maps
// are cached per thread by (increment, distance), so a planned block costs three 128-bit affine applications
// instead of three binary powers (L=4096: 64 sweeps 66 -> ~10 us)
static const Affine &cached_power(u128 inc, uint64_t steps) {
    struct Key {
        uint64_t lo, hi, k;
        bool operator==(const Key &o) const { return lo == o.lo && hi == o.hi && k == o.k; }
    };
    struct Hash {
        size_t operator()(const Key &x) const { return (size_t)(x.lo * 0x9E3779B97F4A7C15ULL ^ x.hi ^ (x.k * 0xC2B2AE3D27D4EB4FULL)); }
    };
    thread_local std::unordered_map<Key, Affine, Hash> cache;
    const Key key{inc.lo, inc.hi, steps};
    auto it = cache.find(key);
    if (it != cache.end()) return it->second;
    if (cache.size() >= 4096) cache.clear();  // (bounded: many increments or distances)
    return cache.emplace(key, power(step_map(inc), steps)).first->second;
}

u128 host_jump(u128 s, u128 inc, uint64_t steps) { return apply(cached_power(inc, steps), s); }

Affine host_power(u128 inc, uint64_t steps) { return cached_power(inc, steps); }

uint64_t host_output_at(u128 s, u128 inc, uint64_t pos) { return xsl_rr(host_jump(s, inc, pos + 1)); }

Block plan_block(Cursor &cur, u128 inc, const BlockSpec &spec, const std::vector<uint32_t> &skips, int32_t skip0) {
    Block b{};
    u128 base = host_jump(cur.s, inc, 1);
    b.base_lo = base.lo;
    b.base_hi = base.hi;
    b.nskip = 0;
    b.skip0 = skip0;
    if (spec.kind == UNIFORM) {
        b.has = 0;
        b.buf = 0;
        cur.s = host_jump(cur.s, inc, spec.count);
        return b;
    }
    b.has = cur.has;
    b.buf = cur.buf;
    b.nskip = (int32_t)skips.size();
    if (spec.count == 0) return b;
    // stream positions consumed: count draws plus every rejected position met on the way
    uint64_t u = spec.count;
    for (;;) {
        uint64_t z = (uint64_t)std::count_if(skips.begin(), skips.end(), [&](uint32_t p) { return p < u + 0; });
        // positions < u that are skipped push the end out; iterate to the fixed point
        uint64_t nu = spec.count + z;
        if (nu == u) break;
        u = nu;
    }
    // u64s consumed from the stream.  NumPy keeps the LAST buffered high half in `uinteger` even
    // after the buffer is used (has_uint32 = 0), so `buf` changes only when a u64 is drawn.
    uint64_t rest = u - (cur.has ? 1 : 0);
    uint64_t words = (rest + 1) / 2;
    if (words > 0) cur.buf = (uint32_t)(host_output_at(cur.s, inc, words - 1) >> 32);
    cur.has = (rest & 1) ? 1 : 0;
    cur.s = host_jump(cur.s, inc, words);
    return b;
}

JumpTables make_tables(u128 inc) {
    JumpTables T;
    Affine P = step_map(inc);
    for (int l = 0; l < JUMP_LEVELS; l++) {
        T.level[l][0] = identity();
        for (int d = 1; d < JUMP_DIGITS; d++) T.level[l][d] = compose(P, T.level[l][d - 1]);
        P = compose(P, T.level[l][JUMP_DIGITS - 1]);  // P^(256)
    }
    T.small[0] = identity();
    Affine s = step_map(inc);
    for (int k = 1; k < SMALL; k++) T.small[k] = compose(s, T.small[k - 1]);
    return T;
}

static inline int64_t fftc(int64_t i, int64_t N) { return i <= N / 2 ? i : i - N; }

int build_colors(int32_t N, std::vector<int32_t> &sites, int64_t count[4], int64_t offset[4]) {
    const int ncol = (N % 2 == 0) ? 2 : 4;
    std::vector<std::vector<int32_t>> lists(4);
    for (int64_t t = 0; t < N; t++)
        for (int64_t x = 0; x < N; x++) {
            int64_t c0 = fftc(t, N), c1 = fftc(x, N);
            int par = (int)((((c0 + c1) % 2) + 2) % 2);
            int col = par;
            if (N % 2) {
                bool b0 = (c0 >= 0 && c1 >= 0) || (c0 < 0 && c1 < 0);
                col = 2 * (b0 ? 0 : 1) + par;
            }
            lists[col].push_back((int32_t)(t * N + x));
        }
    sites.clear();
    for (int c = 0; c < 4; c++) {
        offset[c] = (int64_t)sites.size();
        count[c] = (int64_t)lists[c].size();
        sites.insert(sites.end(), lists[c].begin(), lists[c].end());
    }
    return ncol;
}

}  // namespace sv
