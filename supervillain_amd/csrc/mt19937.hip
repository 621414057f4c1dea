// mt19937.hip -- NumPy's legacy global RandomState permutation, natively (host code).
//
// The reference-order PlaquetteUpdate visits the plaquettes in np.random.permutation(L.coordinates) order
// (supervillain/generator/worldline/plaquette.py:63), drawn from NumPy's legacy global RandomState (MT19937), not
// from the generator's own PCG64.  For an (n, D) array, RandomState.permutation shuffles an index array
// arange(n) (numpy/random/mtrand.pyx: permutation -> shuffle -> _shuffle_raw) with
//
//     for i = n - 1 .. 1:  j = random_interval(i);  swap(a[i], a[j])
//
// where random_interval (numpy/random/src/distributions/distributions.c) masks 32-bit MT19937 outputs to the
// smallest all-ones mask >= i and rejects values above i.  L.coordinates lists the sites row-major, so the visit
// order of plaquette indices IS that shuffled index array.  Done by NumPy on the host this costs ~7.6 ms per
// L=1024 sweep (89% of the bit-exact reference-order step); here the MT19937 stream is generated a
// 624-word block at a time (the twist loops vectorise), the masking/rejection scan is branch-free, the shuffle runs
// on 32-bit indices, and sv_worldline_plaquette_reference_run draws the next sweep's permutation on a host thread
// while the device runs the current sweep.
#include <cstring>

#include "common.h"

namespace sv {
namespace mt {

static constexpr int NK = 624, MK = 397;
static constexpr uint32_t MATRIX_A = 0x9908b0dfu, UPPER = 0x80000000u, LOWER = 0x7fffffffu;

// mt19937_gen (numpy/random/src/mt19937/mt19937.c): the next 624 words of the state, in place
#if defined(__x86_64__)
__attribute__((target("avx2")))
#endif
static void twist(uint32_t *k) {
    int i;
    for (i = 0; i < NK - MK; i++) {
        const uint32_t y = (k[i] & UPPER) | (k[i + 1] & LOWER);
        k[i] = k[i + MK] ^ (y >> 1) ^ (-(y & 1u) & MATRIX_A);
    }
    for (; i < NK - 1; i++) {
        const uint32_t y = (k[i] & UPPER) | (k[i + 1] & LOWER);
        k[i] = k[i + (MK - NK)] ^ (y >> 1) ^ (-(y & 1u) & MATRIX_A);
    }
    const uint32_t y = (k[NK - 1] & UPPER) | (k[0] & LOWER);
    k[NK - 1] = k[MK - 1] ^ (y >> 1) ^ (-(y & 1u) & MATRIX_A);
}

// mt19937_next32's tempering of words [from, NK) of the state into o
#if defined(__x86_64__)
__attribute__((target("avx2")))
#endif
static void temper(const uint32_t *k, int from, uint32_t *o) {
    for (int i = from; i < NK; i++) {
        uint32_t y = k[i];
        y ^= y >> 11;
        y ^= (y << 7) & 0x9d2c5680u;
        y ^= (y << 15) & 0xefc60000u;
        y ^= y >> 18;
        o[i] = y;
    }
}

// The shuffle's draws j[i] = random_interval(i) for i = n - 1 .. 1 (j[0] unused), advancing (key, pos).
// random_interval(max): mask = smallest 2^b - 1 >= max; draw 32-bit words until (word & mask) <= max.
static void intervals(uint32_t *key, int32_t &pos, int64_t n, uint32_t *j) {
    uint32_t tw[NK];
    int64_t i = n - 1;
    int p = pos;
    if (p < NK) temper(key, p, tw);
    while (i >= 1) {
        if (p >= NK) {
            twist(key);
            p = 0;
            temper(key, 0, tw);
        }
        uint32_t mask = (uint32_t)i;
        mask |= mask >> 1;
        mask |= mask >> 2;
        mask |= mask >> 4;
        mask |= mask >> 8;
        mask |= mask >> 16;
        const int64_t lo = (int64_t)(mask >> 1);  // i > lo keeps this mask
        // branch-free: every word is written to j[i]; i moves on only when the word is accepted
        while (p < NK && i > lo) {
            const uint32_t v = tw[p++] & mask;
            j[i] = v;
            i -= (int64_t)(v <= (uint32_t)i);
        }
    }
    pos = p;
}

}  // namespace mt

// The shuffle's draws j[1 .. n-1] (the MT19937 part, serial), advancing (key, pos)
void legacy_intervals(uint32_t *key, int32_t &pos, int64_t n, uint32_t *j) {
    if (pos < 0 || pos > mt::NK) throw std::invalid_argument("MT19937 position must be in [0, 624]");
    if (n >= (int64_t(1) << 32)) throw std::invalid_argument("permutation too long for 32-bit indices");
    if (n > 1) mt::intervals(key, pos, n, j);
}

// The shuffle itself: arange(n) with a[i] <-> a[j[i]] for i = n-1 .. 1 (mtrand.pyx _shuffle_raw)
void shuffle_from_intervals(const uint32_t *j, int64_t n, uint32_t *out) {
    for (int64_t i = 0; i < n; i++) out[i] = (uint32_t)i;
    for (int64_t i = n - 1; i >= 1; i--) {
        const uint32_t a = out[j[i]];
        out[j[i]] = out[i];
        out[i] = a;
    }
}

// np.random.permutation(n) of the legacy global RandomState, as 32-bit indices; advances (key, pos)
void legacy_permutation32(uint32_t *key, int32_t &pos, int64_t n, uint32_t *out) {
    if (n <= 0) return;
    std::vector<uint32_t> j((size_t)n);
    legacy_intervals(key, pos, n, j.data());
    shuffle_from_intervals(j.data(), n, out);
}

}  // namespace sv

extern "C" {

int sv_mt19937_permutation(sv_mt19937 *mt, int64_t n, int64_t *out) {
    if (!mt || n < 0 || (n > 0 && !out)) return -1;
    try {
        std::vector<uint32_t> p((size_t)n);
        sv::legacy_permutation32(mt->key, mt->pos, n, p.data());
        for (int64_t i = 0; i < n; i++) out[i] = (int64_t)p[i];
        return 0;
    } catch (const std::exception &) {
        return -2;
    }
}

}  // extern "C"
