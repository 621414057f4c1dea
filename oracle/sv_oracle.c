/*
 * sv_oracle.c -- CPU restatement of the reference hot path.  TEST INFRASTRUCTURE ONLY.
 *
 * This file is the parity checker for the HIP product path, never part of it: only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load liboracle.so.  It is pinned
 * against golden vectors captured from the reference itself (tests/golden/, made by
 * tools/make_golden.py through tools/refshim.py in the survey container).
 *
 * What it restates (all citations are /root/reference paths):
 *   - NumPy's Generator(PCG64) draw semantics used by the generators (third-party, NumPy 2.2.6 in
 *     this image): PCG64 XSL-RR 128/64 step-then-output, uniform() as
 *     low + range*((u64>>11)*2^-53), choice(seq,k) == seq[integers(0,len)] via the buffered 32-bit
 *     Lemire rejection sampler whose half-word buffer lives in the bit generator state.
 *   - NeighborhoodUpdate.step     supervillain/generator/villain/neighborhood.py:59-137
 *   - CoexactUpdate.step          supervillain/generator/worldline/coexact.py:53-128
 *   - PlaquetteUpdate.step        supervillain/generator/worldline/plaquette.py:35-104 (visit order
 *     supplied by the caller, since the reference draws it from NumPy's global MT19937)
 *   - the D=2 operators d/delta/face_sum/coface_sum in the reference's summation order
 *     supervillain/lattice/reference.py:9-81, _operator_tables compact.py:143-174,
 *     coface_sum_at compact.py:1185-1247, delta_sparse compact.py:1042-1116
 *   - Lattice.checkerboarding     supervillain/lattice/compact.py:191-239 (odd N: 4 colours built
 *     from FFT-convention coordinates, lattice/__init__.py:4-9, compact.py:36-53)
 * plus one chain the reference does not have: the checkerboard PlaquetteUpdate variant the GPU
 * runs in mode="checkerboard" (defined in DESIGN.md); here it is the bit-exact oracle for that mode.
 *
 * Build: oracle/Makefile (gcc -O2 -ffp-contract=off, no fast-math: the op order IS the spec).
 */
#include <math.h>
#ifdef _OPENMP
#include <omp.h>
#endif
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef unsigned __int128 u128;

typedef struct {
    uint64_t state_hi, state_lo, inc_hi, inc_lo;
    int32_t has_uint32;
    uint32_t uinteger;
} sv_rng;

typedef struct {
    int64_t accepted;
    int64_t proposed;
    double acceptance_sum; /* sum of per-proposal Metropolis probabilities in this sweep */
    int64_t rejections;    /* Lemire rejections met in this sweep (diagnostic) */
} sv_stats;

/* ---------------------------------------------------------------- exact acceptance sums
 * The sweep statistic acceptance_sum sums the per-proposal Metropolis probabilities (neighborhood.py:118,
 * coexact.py:117, plaquette.py:88; the reference adds NumPy pairwise sums per colour).  It is kept here as the
 * exact sum of the probabilities rounded to 2^-103, T(p) = round(p 2^51) 2^52 + round(r 2^103) with r = p - (p
 * rounded to 2^-51), accumulated as three 38-bit limb sums and turned into a double by the same function as
 * libsvhip.so (supervillain_amd/csrc/common.h fx_value): within ~2 ulp of the exact sum of the p, so within rounding
 * of the reference's pairwise sums.  The device keeps only the first level, round(p 2^51) per proposal (one integer
 * add, common.h fx_add), so device and oracle agree within 2^-52 per proposal (the GPU tests: 1e-12 relative), and
 * the device's value is the same for every launch geometry.  The running sum of the sv_stats being filled lives
 * beside it (thread-local); a cleared or different sv_stats restarts it. */
#define FX_LIMB ((UINT64_C(1) << 38) - 1)
static _Thread_local const sv_stats *fx_owner;
static _Thread_local uint64_t fx_w[3];
static _Thread_local double fx_last;
static double fx_value(uint64_t w0, uint64_t w1, uint64_t w2) {
    w1 += w0 >> 38;
    w0 &= FX_LIMB;
    w2 += w1 >> 38;
    w1 &= FX_LIMB;
    return ((double)w2 * 0x1p76 + (double)w1 * 0x1p38 + (double)w0) * 0x1p-103;
}
/* T(p) for p in [0, 1] as three limbs (added to w) */
static void fx_term_limbs(double p, uint64_t w[3]) {
    const double x = p + 2.0;
    uint64_t bx;
    memcpy(&bx, &x, sizeof bx);
    const uint64_t a = bx - UINT64_C(0x4000000000000000); /* round(p 2^51) */
    const double r = p - (x - 2.0);                       /* exact, |r| <= 2^-52 */
    const double y = fma(r, 0x1p103, 0x1.8p52);
    int64_t by;
    memcpy(&by, &y, sizeof by);
    const int64_t b = by - INT64_C(0x4338000000000000); /* round(r 2^103) */
    const u128 T = ((u128)a << 52) + (u128)(__int128)b;
    w[0] += (uint64_t)T & FX_LIMB;
    w[1] += (uint64_t)(T >> 38) & FX_LIMB;
    w[2] += (uint64_t)(T >> 76);
}
static double exact_acceptance_add_w(const sv_stats *st, const uint64_t add[3]) {
    if (fx_owner != st || st->acceptance_sum != fx_last) {
        fx_owner = st;
        fx_w[0] = fx_w[1] = fx_w[2] = 0;
    }
    for (int i = 0; i < 3; i++) fx_w[i] += add[i];
    fx_last = fx_value(fx_w[0], fx_w[1], fx_w[2]);
    return fx_last;
}
static double exact_acceptance_add(const sv_stats *st, double p) {
    uint64_t w[3] = {0, 0, 0};
    fx_term_limbs(p, w);
    return exact_acceptance_add_w(st, w);
}

/* ---------------------------------------------------------------- PCG64 (NumPy) */
static const u128 PCG_MULT = (((u128)0x2360ED051FC65DA4ULL) << 64) | (u128)0x4385DF649FCCF645ULL;

typedef struct {
    u128 s, inc;
    int has;
    uint32_t buf;
} pcg;

static pcg pcg_load(const sv_rng *r) {
    pcg g;
    g.s = (((u128)r->state_hi) << 64) | r->state_lo;
    g.inc = (((u128)r->inc_hi) << 64) | r->inc_lo;
    g.has = r->has_uint32;
    g.buf = r->uinteger;
    return g;
}

static void pcg_store(const pcg *g, sv_rng *r) {
    r->state_hi = (uint64_t)(g->s >> 64);
    r->state_lo = (uint64_t)g->s;
    r->has_uint32 = g->has;
    r->uinteger = g->buf;
}

static inline uint64_t pcg_u64(pcg *g) {
    g->s = g->s * PCG_MULT + g->inc; /* advance first ... */
    uint64_t x = (uint64_t)(g->s >> 64) ^ (uint64_t)g->s;
    unsigned rot = (unsigned)(g->s >> 122);
    return (x >> rot) | (x << ((64u - rot) & 63u)); /* ... then XSL-RR output */
}

static inline double pcg_double(pcg *g) { return (double)(pcg_u64(g) >> 11) * (1.0 / 9007199254740992.0); }

static inline double pcg_uniform(pcg *g, double low, double range) {
    double d = pcg_double(g);
    double t = range * d;
    return low + t;
}

static inline uint32_t pcg_u32(pcg *g) {
    if (g->has) {
        g->has = 0;
        return g->buf;
    }
    uint64_t x = pcg_u64(g);
    g->has = 1;
    g->buf = (uint32_t)(x >> 32);
    return (uint32_t)x;
}

/* integers(0, k) for 1 <= k <= 2^32 via NumPy's buffered bounded Lemire (32-bit path).
 * k == 1 consumes nothing (NumPy returns `off` when rng == 0). */
static inline uint32_t pcg_bounded(pcg *g, uint32_t k, int64_t *rejections) {
    if (k <= 1) return 0;
    uint32_t thr = (uint32_t)((0u - k) % k); /* (2^32 - k) mod k */
    uint64_t m = (uint64_t)pcg_u32(g) * (uint64_t)k;
    uint32_t left = (uint32_t)m;
    if (left < k) {
        while (left < thr) {
            if (rejections) (*rejections)++;
            m = (uint64_t)pcg_u32(g) * (uint64_t)k;
            left = (uint32_t)m;
        }
    }
    return (uint32_t)(m >> 32);
}

/* ---------------------------------------------------------------- KAT helpers */
int sv_o_raw(sv_rng *r, int64_t count, uint64_t *out) {
    pcg g = pcg_load(r);
    for (int64_t i = 0; i < count; i++) out[i] = pcg_u64(&g);
    pcg_store(&g, r);
    return 0;
}

int sv_o_uniform(sv_rng *r, double low, double high, int64_t count, double *out) {
    pcg g = pcg_load(r);
    double range = high - low;
    for (int64_t i = 0; i < count; i++) out[i] = pcg_uniform(&g, low, range);
    pcg_store(&g, r);
    return 0;
}

int sv_o_integers(sv_rng *r, uint32_t k, int64_t count, int64_t *out) {
    pcg g = pcg_load(r);
    for (int64_t i = 0; i < count; i++) out[i] = pcg_bounded(&g, k, NULL);
    pcg_store(&g, r);
    return 0;
}

/* ---------------------------------------------------------------- lattice (D=2) */
static inline int64_t wrap(int64_t i, int64_t N) { return ((i % N) + N) % N; }

/* FFT-convention coordinate, lattice/__init__.py:4-9: [0..N//2] then [-N//2+1 .. -1]. */
static inline int64_t fftc(int64_t i, int64_t N) { return i <= N / 2 ? i : i - N; }

/* Colour of every site and the colour count, compact.py:191-239 for D=2.
 * Even N: parity of the coordinate sum.  Odd N: 4 colours ordered (b,c) =
 * (0,0),(0,1),(1,0),(1,1) with b the hyperoctant pair and c the parity. */
int sv_o_colors(int32_t N, int32_t *color_of_site) {
    int64_t V = (int64_t)N * N;
    for (int64_t t = 0; t < N; t++)
        for (int64_t x = 0; x < N; x++) {
            int64_t c0 = fftc(t, N), c1 = fftc(x, N);
            int par = (int)((((c0 + c1) % 2) + 2) % 2);
            int col;
            if (N % 2 == 0) {
                col = par;
            } else {
                int b0 = (c0 >= 0 && c1 >= 0) || (c0 < 0 && c1 < 0);
                int b = b0 ? 0 : 1;
                col = 2 * b + par;
            }
            color_of_site[t * N + x] = col;
        }
    (void)V;
    return N % 2 == 0 ? 2 : 4;
}

/* Colour site lists in np.where (row-major) order. */
typedef struct {
    int ncol;
    int64_t count[4];
    int64_t *sites[4];
} colors_t;

static colors_t colors_make(int32_t N) {
    colors_t C;
    int64_t V = (int64_t)N * N;
    int32_t *col = (int32_t *)malloc(sizeof(int32_t) * V);
    C.ncol = sv_o_colors(N, col);
    for (int c = 0; c < 4; c++) {
        C.count[c] = 0;
        C.sites[c] = (int64_t *)malloc(sizeof(int64_t) * (V + 1));
    }
    for (int64_t s = 0; s < V; s++) {
        int c = col[s];
        C.sites[c][C.count[c]++] = s;
    }
    free(col);
    return C;
}

static void colors_free(colors_t *C) {
    for (int c = 0; c < 4; c++) free(C->sites[c]);
}

/* Even Nt x Nx rectangle (the domain-decomposition extension; the reference's Lattice2D is square):
 * colours are the parity of t + x, row-major, as compact.py:191-239 gives for even square N. */
static colors_t colors_make_rect(int32_t Nt, int32_t Nx) {
    colors_t C;
    int64_t V = (int64_t)Nt * Nx;
    C.ncol = 2;
    for (int c = 0; c < 4; c++) {
        C.count[c] = 0;
        C.sites[c] = (int64_t *)malloc(sizeof(int64_t) * (V + 1));
    }
    for (int64_t s = 0; s < V; s++) {
        int c = (int)(((s / Nx) + (s % Nx)) & 1);
        C.sites[c][C.count[c]++] = s;
    }
    return C;
}

/* neighbours on an Nt x Nx torus: e0 moves t (axis 0, rows), e1 moves x (axis 1, columns) */
static inline int64_t fwd2(int64_t s, int mu, int64_t Nt, int64_t Nx) {
    int64_t t = s / Nx, x = s % Nx;
    if (mu == 0) t = (t + 1) % Nt; else x = (x + 1) % Nx;
    return t * Nx + x;
}
static inline int64_t bwd2(int64_t s, int mu, int64_t Nt, int64_t Nx) {
    int64_t t = s / Nx, x = s % Nx;
    if (mu == 0) t = (t + Nt - 1) % Nt; else x = (x + Nx - 1) % Nx;
    return t * Nx + x;
}
static inline int64_t fwd(int64_t s, int mu, int64_t N) { return fwd2(s, mu, N, N); }
static inline int64_t bwd(int64_t s, int mu, int64_t N) { return bwd2(s, mu, N, N); }

#define TWO_PI 6.283185307179586 /* Python's 2*np.pi, rounded once */

/* ---------------------------------------------------------------- Villain NeighborhoodUpdate */
/* One sweep of neighborhood.py:59-137 on D=2.  phi: (N,N) f64, n: (2,N,N) i64, in place. */
static void villain_sweep(int64_t Nt, int64_t Nx, double kappa, int64_t W, double interval_phi, int64_t interval_n,
                          double *phi, int64_t *n, pcg *g, const colors_t *C, sv_stats *st, double *work) {
    int64_t V = Nt * Nx;
    double *metro = work;          /* V */
    double *r = metro + V;         /* 2V */
    double *cphi = r + 2 * V;      /* V */
    double *dSl = cphi + V;        /* 2V */
    int64_t *cn = (int64_t *)(dSl + 2 * V); /* 2V */
    int64_t *acc = cn + 2 * V;     /* V (per-site accepted flag for the current colour) */
    const double half_kappa = kappa / 2.0;
    const uint32_t k = (uint32_t)(2 * interval_n + 1);
    const double range_phi = interval_phi - (-interval_phi);

    memset(st, 0, sizeof(*st));
    for (int64_t s = 0; s < V; s++) metro[s] = pcg_uniform(g, 0.0, 1.0); /* :87 */
    for (int mu = 0; mu < 2; mu++)                                         /* :91 */
        for (int64_t s = 0; s < V; s++)
            r[mu * V + s] = (0.0 + (phi[fwd2(s, mu, Nt, Nx)] - phi[s])) - TWO_PI * (double)n[mu * V + s];

    for (int c = 0; c < C->ncol; c++) { /* :93 */
        const int64_t nc = C->count[c];
        const int64_t *sites = C->sites[c];
        for (int64_t s = 0; s < V; s++) cphi[s] = 0.0;
        for (int64_t l = 0; l < 2 * V; l++) cn[l] = 0;
        for (int64_t i = 0; i < nc; i++) cphi[sites[i]] = pcg_uniform(g, -interval_phi, range_phi); /* :98 */
        for (int mu = 0; mu < 2; mu++) { /* :104-107 */
            for (int64_t i = 0; i < nc; i++)
                cn[mu * V + sites[i]] = W * ((int64_t)pcg_bounded(g, k, &st->rejections) - interval_n);
            for (int64_t i = 0; i < nc; i++)
                cn[mu * V + bwd2(sites[i], mu, Nt, Nx)] = W * ((int64_t)pcg_bounded(g, k, &st->rejections) - interval_n);
        }
        /* :110-112  change_r = d(change_phi) - 2 pi change_n ; dS_link ; face_sum */
        for (int mu = 0; mu < 2; mu++)
            for (int64_t s = 0; s < V; s++) {
                double cr = (0.0 + (cphi[fwd2(s, mu, Nt, Nx)] - cphi[s])) - TWO_PI * (double)cn[mu * V + s];
                double a = half_kappa * cr;
                double b = (2.0 * r[mu * V + s]) + cr;
                dSl[mu * V + s] = a * b;
            }
        for (int64_t i = 0; i < nc; i++) { /* :115-118 */
            int64_t s = sites[i];
            double dS = 0.0;
            dS += dSl[0 * V + s];
            dS += dSl[0 * V + bwd2(s, 0, Nt, Nx)];
            dS += dSl[1 * V + s];
            dS += dSl[1 * V + bwd2(s, 1, Nt, Nx)];
            double p = exp(-dS);
            p = p < 0.0 ? 0.0 : p;
            p = p > 1.0 ? 1.0 : p;
            int a = metro[s] < p;
            acc[s] = a;
            st->accepted += a;
            st->acceptance_sum = exact_acceptance_add(st, p);
        }
        for (int64_t i = 0; i < nc; i++) { /* :121-125 */
            int64_t s = sites[i];
            double a = (double)acc[s];
            cphi[s] = cphi[s] * a;
            for (int mu = 0; mu < 2; mu++) {
                cn[mu * V + s] *= acc[s];
                cn[mu * V + bwd2(s, mu, Nt, Nx)] *= acc[s];
            }
        }
        for (int64_t s = 0; s < V; s++) phi[s] = phi[s] + cphi[s]; /* :127 */
        for (int64_t l = 0; l < 2 * V; l++) n[l] = n[l] + cn[l];    /* :128 */
        for (int mu = 0; mu < 2; mu++)                              /* :129 */
            for (int64_t s = 0; s < V; s++) {
                double dcp = 0.0 + (cphi[fwd2(s, mu, Nt, Nx)] - cphi[s]);
                r[mu * V + s] = (r[mu * V + s] + dcp) - TWO_PI * (double)cn[mu * V + s];
            }
    }
    st->proposed = V;
}

int sv_o_villain_neighborhood(int32_t N, double kappa, int64_t W, double interval_phi, int64_t interval_n,
                              double *phi, int64_t *n, int32_t sweeps, sv_rng *rng, sv_stats *stats) {
    if (N < 2 || sweeps < 0) return -1;
    int64_t V = (int64_t)N * N;
    colors_t C = colors_make(N);
    double *work = (double *)malloc(sizeof(double) * 6 * V + sizeof(int64_t) * 3 * V);
    pcg g = pcg_load(rng);
    for (int32_t s = 0; s < sweeps; s++)
        villain_sweep(N, N, kappa, W, interval_phi, interval_n, phi, n, &g, &C, &stats[s], work);
    pcg_store(&g, rng);
    free(work);
    colors_free(&C);
    return 0;
}

/* The same chain on an even Nt x Nx torus (stream layout unchanged: V = Nt Nx metropolis draws, then
 * per colour V/2 dphi and 4 x V/2 choices).  Checks the decomposed GPU engine on rectangles. */
int sv_o_villain_neighborhood_rect(int32_t Nt, int32_t Nx, double kappa, int64_t W, double interval_phi,
                                   int64_t interval_n, double *phi, int64_t *n, int32_t sweeps, sv_rng *rng,
                                   sv_stats *stats) {
    if (Nt < 2 || Nx < 2 || (Nt % 2) || (Nx % 2) || sweeps < 0) return -1;
    int64_t V = (int64_t)Nt * Nx;
    colors_t C = colors_make_rect(Nt, Nx);
    double *work = (double *)malloc(sizeof(double) * 6 * V + sizeof(int64_t) * 3 * V);
    pcg g = pcg_load(rng);
    for (int32_t s = 0; s < sweeps; s++)
        villain_sweep(Nt, Nx, kappa, W, interval_phi, interval_n, phi, n, &g, &C, &stats[s], work);
    pcg_store(&g, rng);
    free(work);
    colors_free(&C);
    return 0;
}

/* ---------------------------------------------------------------- optional counter-based mode (Philox) */
/* SURVEY.md 8(b) sv_rng mode 1: the same NeighborhoodUpdate sweep (neighborhood.py:59-137, the operation order of
 * villain_sweep above) with its draws from Philox4x32-10 by counter instead of NumPy's PCG64 stream.  For colour
 * site s (row-major index) in sweep number `sweep` (a 64-bit count kept by the caller):
 *   call (s, sweep_lo, sweep_hi, 0) -> words w0..w3: metropolis u = next_double(w1:w0), dphi = uniform(w3:w2);
 *   call (s, sweep_lo, sweep_hi, 1) -> the 4 choice words: [2 mu] the forward link (mu, s), [2 mu + 1] the
 *   backward link (mu, s - e_mu);
 *   choice j is Lemire's bounded draw on its word; a rejected word is replaced by word 0 of call
 *   (s, sweep_lo, sweep_hi, 2 + j + 4 t) at retry t (in place: nothing else shifts).
 * Every site draws u (the reference draws it for all sites, :87), only colour sites use it.  `thr_override`
 * (tests only) replaces Lemire's threshold to exercise the retry path. */
static inline void philox4x32_10(uint32_t c[4], uint32_t k0, uint32_t k1) {
    for (int i = 0; i < 10; i++) {
        if (i) {
            k0 += 0x9E3779B9u;
            k1 += 0xBB67AE85u;
        }
        uint64_t p0 = (uint64_t)0xD2511F53u * c[0], p1 = (uint64_t)0xCD9E8D57u * c[2];
        uint32_t n0 = (uint32_t)(p1 >> 32) ^ c[1] ^ k0, n1 = (uint32_t)p1, n2 = (uint32_t)(p0 >> 32) ^ c[3] ^ k1,
                 n3 = (uint32_t)p0;
        c[0] = n0;
        c[1] = n1;
        c[2] = n2;
        c[3] = n3;
    }
}

int sv_o_philox4x32_10(const uint32_t *ctr, const uint32_t *key, uint32_t *out) {
    uint32_t c[4] = {ctr[0], ctr[1], ctr[2], ctr[3]};
    philox4x32_10(c, key[0], key[1]);
    for (int i = 0; i < 4; i++) out[i] = c[i];
    return 0;
}

static inline double u53_of(uint32_t lo, uint32_t hi) {
    return (double)((((uint64_t)hi << 32) | lo) >> 11) * (1.0 / 9007199254740992.0);
}

static uint32_t philox_choice(uint32_t s, uint64_t sweep, uint64_t key, uint32_t word, int j, uint32_t k, uint32_t thr,
                              int64_t *retries) {
    uint64_t m = (uint64_t)word * k;
    for (uint32_t t = 0; (uint32_t)m < thr; t++) {
        uint32_t c[4] = {s, (uint32_t)sweep, (uint32_t)(sweep >> 32), 2u + (uint32_t)j + 4u * t};
        philox4x32_10(c, (uint32_t)key, (uint32_t)(key >> 32));
        m = (uint64_t)c[0] * k;
        if (retries) (*retries)++;
    }
    return (uint32_t)(m >> 32);
}

int sv_o_villain_neighborhood_philox(int32_t N, double kappa, int64_t W, double interval_phi, int64_t interval_n,
                                     double *phi, int64_t *n, int32_t sweeps, uint64_t key, uint64_t counter,
                                     uint32_t thr_override, sv_stats *stats) {
    if (N < 2 || (N % 2) || sweeps < 0) return -1;
    const int64_t Nt = N, Nx = N, V = (int64_t)N * N;
    colors_t C = colors_make(N);
    double *metro = (double *)malloc(sizeof(double) * 6 * V + sizeof(int64_t) * 3 * V);
    double *r = metro + V, *cphi = r + 2 * V, *dSl = cphi + V;
    int64_t *cn = (int64_t *)(dSl + 2 * V), *acc = cn + 2 * V;
    const double half_kappa = kappa / 2.0, range_phi = interval_phi - (-interval_phi);
    const uint32_t k = (uint32_t)(2 * interval_n + 1);
    const uint32_t thr = thr_override ? thr_override : (k > 1 ? (uint32_t)((0u - k) % k) : 0u);
    for (int32_t sw = 0; sw < sweeps; sw++) {
        const uint64_t sweep = counter + (uint64_t)sw;
        sv_stats *st = &stats[sw];
        memset(st, 0, sizeof(*st));
        double *dphi_all = dSl; /* scratch: the dphi of every site (used by colour sites only) */
        for (int64_t s = 0; s < V; s++) {
            uint32_t c[4] = {(uint32_t)s, (uint32_t)sweep, (uint32_t)(sweep >> 32), 0u};
            philox4x32_10(c, (uint32_t)key, (uint32_t)(key >> 32));
            metro[s] = 0.0 + 1.0 * u53_of(c[0], c[1]);
            dphi_all[s] = -interval_phi + range_phi * u53_of(c[2], c[3]);
        }
        for (int mu = 0; mu < 2; mu++)
            for (int64_t s = 0; s < V; s++)
                r[mu * V + s] = (0.0 + (phi[fwd2(s, mu, Nt, Nx)] - phi[s])) - TWO_PI * (double)n[mu * V + s];
        for (int col = 0; col < C.ncol; col++) {
            const int64_t nc = C.count[col];
            const int64_t *sites = C.sites[col];
            for (int64_t s = 0; s < V; s++) cphi[s] = 0.0;
            for (int64_t l = 0; l < 2 * V; l++) cn[l] = 0;
            for (int64_t i = 0; i < nc; i++) {
                const int64_t s = sites[i];
                cphi[s] = dphi_all[s];
                uint32_t c[4] = {(uint32_t)s, (uint32_t)sweep, (uint32_t)(sweep >> 32), 1u};
                philox4x32_10(c, (uint32_t)key, (uint32_t)(key >> 32));
                for (int mu = 0; mu < 2; mu++) {
                    uint32_t f = philox_choice((uint32_t)s, sweep, key, c[2 * mu], 2 * mu, k, thr, &st->rejections);
                    uint32_t b = philox_choice((uint32_t)s, sweep, key, c[2 * mu + 1], 2 * mu + 1, k, thr, &st->rejections);
                    cn[mu * V + s] = W * ((int64_t)f - interval_n);
                    cn[mu * V + bwd2(s, mu, Nt, Nx)] = W * ((int64_t)b - interval_n);
                }
            }
            /* from here on exactly villain_sweep's :110-129 */
            double *dS_l = (double *)malloc(sizeof(double) * 2 * V);
            for (int mu = 0; mu < 2; mu++)
                for (int64_t s = 0; s < V; s++) {
                    double cr = (0.0 + (cphi[fwd2(s, mu, Nt, Nx)] - cphi[s])) - TWO_PI * (double)cn[mu * V + s];
                    double a = half_kappa * cr;
                    double b = (2.0 * r[mu * V + s]) + cr;
                    dS_l[mu * V + s] = a * b;
                }
            for (int64_t i = 0; i < nc; i++) {
                int64_t s = sites[i];
                double dS = 0.0;
                dS += dS_l[0 * V + s];
                dS += dS_l[0 * V + bwd2(s, 0, Nt, Nx)];
                dS += dS_l[1 * V + s];
                dS += dS_l[1 * V + bwd2(s, 1, Nt, Nx)];
                double p = exp(-dS);
                p = p < 0.0 ? 0.0 : p;
                p = p > 1.0 ? 1.0 : p;
                int a = metro[s] < p;
                acc[s] = a;
                st->accepted += a;
                st->acceptance_sum = exact_acceptance_add(st, p);
            }
            free(dS_l);
            for (int64_t i = 0; i < nc; i++) {
                int64_t s = sites[i];
                double a = (double)acc[s];
                cphi[s] = cphi[s] * a;
                for (int mu = 0; mu < 2; mu++) {
                    cn[mu * V + s] *= acc[s];
                    cn[mu * V + bwd2(s, mu, Nt, Nx)] *= acc[s];
                }
            }
            for (int64_t s = 0; s < V; s++) phi[s] = phi[s] + cphi[s];
            for (int64_t l = 0; l < 2 * V; l++) n[l] = n[l] + cn[l];
            for (int mu = 0; mu < 2; mu++)
                for (int64_t s = 0; s < V; s++) {
                    double dcp = 0.0 + (cphi[fwd2(s, mu, Nt, Nx)] - cphi[s]);
                    r[mu * V + s] = (r[mu * V + s] + dcp) - TWO_PI * (double)cn[mu * V + s];
                }
        }
        st->proposed = V;
    }
    free(metro);
    colors_free(&C);
    return 0;
}

/* Villain action, villain.py:51-66 (sequential sum; the reference uses NumPy pairwise). */
double sv_o_villain_action(int32_t N, double kappa, const double *phi, const int64_t *n) {
    int64_t V = (int64_t)N * N;
    double S = 0.0;
    for (int mu = 0; mu < 2; mu++)
        for (int64_t s = 0; s < V; s++) {
            double l = (0.0 + (phi[fwd(s, mu, N)] - phi[s])) - TWO_PI * (double)n[mu * V + s];
            S += l * l;
        }
    return (kappa / 2.0) * S;
}

/* ---------------------------------------------------------------- Worldline helpers */
/* delta(v)/_W for a D=2 two-form v (comp (0,1)), reference.py:27-45 with table rows
 * ('delta',2) = (0,0,1,-1),(1,0,0,+1): dv0[x] = 0 - (-1)(v[x]-v[x-e1]), dv1[x] = 0 - (+1)(v[x]-v[x-e0]).
 * coexact.py:80 / plaquette.py:53 then divide by _W (worldline.py:49). */
static void delta_v_by_W(int64_t N, const void *v, int v_is_float, double Weff, double *dvw) {
    int64_t V = N * N;
    for (int64_t s = 0; s < V; s++) {
        int64_t b1 = bwd(s, 1, N), b0 = bwd(s, 0, N);
        double d0, d1;
        if (v_is_float) {
            const double *vf = (const double *)v;
            double a = vf[s] - vf[b1];
            double b = vf[s] - vf[b0];
            d0 = 0.0 - (-a);
            d1 = 0.0 - b;
        } else {
            const int64_t *vi = (const int64_t *)v;
            d0 = (double)(0 - (-(vi[s] - vi[b1])));
            d1 = (double)(0 - (vi[s] - vi[b0]));
        }
        dvw[s] = d0 / Weff;
        dvw[V + s] = d1 / Weff;
    }
}

/* ---------------------------------------------------------------- Worldline CoexactUpdate */
/* coexact.py:53-128 on D=2 (one 2-form component).  ts = (-it..-1, 1..it).
 * Plaquette at x with value t changes  m0[x] += t, m0[x+e1] -= t, m1[x] -= t, m1[x+e0] += t
 * (delta_sparse with ('delta',2) rows), and dS sums dS_link in coface_sum_at row order
 * ('coface_sum',1) = (0,1,0,1),(0,0,1,1):  dl1[x], dl1[x+e0], dl0[x], dl0[x+e1]. */
int sv_o_worldline_coexact(int32_t N_, double kappa, double Weff, int64_t interval_t, int64_t *m, const void *v,
                           int32_t v_is_float, int32_t sweeps, sv_rng *rng, sv_stats *stats) {
    int64_t N = N_, V = N * N;
    if (N < 2 || interval_t < 1) return -1;
    colors_t C = colors_make(N_);
    double *dvw = (double *)malloc(sizeof(double) * 2 * V);
    double *metro = (double *)malloc(sizeof(double) * V);
    int64_t *tv = (int64_t *)malloc(sizeof(int64_t) * V);
    delta_v_by_W(N, v, v_is_float, Weff, dvw);
    const double c = 0.5 / kappa;
    const uint32_t k = (uint32_t)(2 * interval_t);
    pcg g = pcg_load(rng);
    for (int32_t sw = 0; sw < sweeps; sw++) {
        sv_stats *st = &stats[sw];
        memset(st, 0, sizeof(*st));
        for (int64_t s = 0; s < V; s++) metro[s] = pcg_uniform(&g, 0.0, 1.0); /* :89 */
        for (int col = 0; col < C.ncol; col++) {
            const int64_t nc = C.count[col];
            const int64_t *sites = C.sites[col];
            for (int64_t i = 0; i < nc; i++) { /* :99 choice(ts) */
                int64_t j = (int64_t)pcg_bounded(&g, k, &st->rejections);
                tv[i] = j < interval_t ? j - interval_t : j - interval_t + 1;
            }
            for (int64_t i = 0; i < nc; i++) {
                int64_t x = sites[i], t = tv[i];
                int64_t xe0 = fwd(x, 0, N), xe1 = fwd(x, 1, N);
                /* links and their cm, in coface order */
                int64_t L[4] = {V + x, V + xe0, x, xe1};
                int64_t cm[4] = {-t, +t, +t, -t};
                double dS = 0.0;
                for (int q = 0; q < 4; q++) {
                    double a = c * (double)cm[q];
                    double f = (double)m[L[q]] - dvw[L[q]];
                    double b = (2.0 * f) + (double)cm[q];
                    dS += a * b;
                }
                double p = exp(-dS);
                p = p < 0.0 ? 0.0 : p;
                p = p > 1.0 ? 1.0 : p;
                int a = metro[x] < p;
                st->accepted += a;
                st->acceptance_sum = exact_acceptance_add(st, p);
                if (a) { /* :120 (links of same-colour plaquettes are disjoint) */
                    m[x] += t;
                    m[xe1] -= t;
                    m[V + x] -= t;
                    m[V + xe0] += t;
                }
            }
        }
        st->proposed = V;
    }
    pcg_store(&g, rng);
    free(dvw);
    free(metro);
    free(tv);
    colors_free(&C);
    return 0;
}

/* ---------------------------------------------------------------- Worldline PlaquetteUpdate */
/* plaquette.py:35-104 on D=2 with the visit order supplied (order[i] = row-major site of the i-th
 * entry of np.random.permutation(L.coordinates)).  One sweep. */
int sv_o_worldline_plaquette_seq(int32_t N_, double kappa, double Weff, int64_t *m, void *v, int32_t v_is_float,
                                 const int64_t *order, sv_rng *rng, sv_stats *st) {
    int64_t N = N_, V = N * N;
    if (N < 2) return -1;
    double *f = (double *)malloc(sizeof(double) * 2 * V);
    int64_t *cm = (int64_t *)malloc(sizeof(int64_t) * V);
    int64_t *cv = (int64_t *)malloc(sizeof(int64_t) * V);
    double *met = (double *)malloc(sizeof(double) * V);
    memset(st, 0, sizeof(*st));
    delta_v_by_W(N, v, v_is_float, Weff, f);
    for (int64_t l = 0; l < 2 * V; l++) f[l] = (double)m[l] - f[l]; /* :53 */
    pcg g = pcg_load(rng);
    for (int64_t i = 0; i < V; i++) cm[i] = pcg_bounded(&g, 2, &st->rejections) ? 1 : -1;          /* :58 */
    for (int64_t i = 0; i < V; i++) cv[i] = (int64_t)pcg_bounded(&g, 3, &st->rejections) - 1;       /* :59 */
    for (int64_t i = 0; i < V; i++) met[i] = pcg_uniform(&g, 0.0, 1.0);                           /* :60 */
    pcg_store(&g, rng);
    for (int64_t i = 0; i < V; i++) { /* :63-101 */
        int64_t x = order[i];
        int64_t xm = fwd(x, 0, N), xn = fwd(x, 1, N);
        double df = (double)cm[i] - (double)cv[i] / Weff;
        double dS = df / kappa * ((((f[x] + f[V + xm]) - f[xn]) - f[V + x]) + 2.0 * df);
        double p = exp(-dS);
        p = p < 0.0 ? 0.0 : p;
        p = p > 1.0 ? 1.0 : p;
        st->acceptance_sum = exact_acceptance_add(st, p);
        if (met[i] < p) {
            m[x] += cm[i];
            m[V + xm] += cm[i];
            m[xn] += -cm[i];
            m[V + x] += -cm[i];
            if (v_is_float) ((double *)v)[x] += (double)cv[i];
            else ((int64_t *)v)[x] += cv[i];
            f[x] += df;
            f[V + xm] += df;
            f[xn] -= df;
            f[V + x] -= df;
            st->accepted++;
        }
    }
    st->proposed = V;
    free(f);
    free(cm);
    free(cv);
    free(met);
    return 0;
}

/* Checkerboard PlaquetteUpdate (this build's GPU-native chain, DESIGN.md "Plaquette modes").
 * Per sweep: metropolis = uniform(0,1,V) in row-major order; then per colour c (compact.py
 * checkerboarding): cm = choice([-1,1], n_c), cv = choice([-1,0,1], n_c).  Each colour pass
 * evaluates f = m - delta(v)/W FRESH from the current fields (same expression and order as
 * plaquette.py:53,84-85), accepts with metropolis[x] < clip(exp(-dS),0,1), and applies the
 * plaquette.py:91-96 field changes.  Same-colour plaquettes share no link, so the pass is
 * order-independent. */
int sv_o_worldline_plaquette_cb(int32_t N_, double kappa, double Weff, int64_t *m, void *v, int32_t v_is_float,
                                int32_t sweeps, sv_rng *rng, sv_stats *stats) {
    int64_t N = N_, V = N * N;
    if (N < 2) return -1;
    colors_t C = colors_make(N_);
    double *metro = (double *)malloc(sizeof(double) * V);
    int64_t *cm = (int64_t *)malloc(sizeof(int64_t) * V);
    int64_t *cv = (int64_t *)malloc(sizeof(int64_t) * V);
    pcg g = pcg_load(rng);
    for (int32_t sw = 0; sw < sweeps; sw++) {
        sv_stats *st = &stats[sw];
        memset(st, 0, sizeof(*st));
        for (int64_t s = 0; s < V; s++) metro[s] = pcg_uniform(&g, 0.0, 1.0);
        for (int col = 0; col < C.ncol; col++) {
            const int64_t nc = C.count[col];
            const int64_t *sites = C.sites[col];
            for (int64_t i = 0; i < nc; i++) cm[i] = pcg_bounded(&g, 2, &st->rejections) ? 1 : -1;
            for (int64_t i = 0; i < nc; i++) cv[i] = (int64_t)pcg_bounded(&g, 3, &st->rejections) - 1;
            for (int64_t i = 0; i < nc; i++) {
                int64_t x = sites[i];
                int64_t xm = fwd(x, 0, N), xn = fwd(x, 1, N);
                /* f on the four boundary links, fresh: f_l = m_l - dvw_l */
                int64_t links[4] = {x, V + xm, xn, V + x};
                double fl[4];
                for (int q = 0; q < 4; q++) {
                    int64_t l = links[q];
                    int64_t s = l % V;
                    int mu = (int)(l / V);
                    double dv;
                    if (mu == 0) {
                        int64_t b1 = bwd(s, 1, N);
                        if (v_is_float) {
                            const double *vf = (const double *)v;
                            dv = 0.0 - (-(vf[s] - vf[b1]));
                        } else {
                            const int64_t *vi = (const int64_t *)v;
                            dv = (double)(vi[s] - vi[b1]);
                        }
                    } else {
                        int64_t b0 = bwd(s, 0, N);
                        if (v_is_float) {
                            const double *vf = (const double *)v;
                            dv = 0.0 - (vf[s] - vf[b0]);
                        } else {
                            const int64_t *vi = (const int64_t *)v;
                            dv = (double)(0 - (vi[s] - vi[b0]));
                        }
                    }
                    fl[q] = (double)m[l] - dv / Weff;
                }
                double df = (double)cm[i] - (double)cv[i] / Weff;
                double dS = df / kappa * ((((fl[0] + fl[1]) - fl[2]) - fl[3]) + 2.0 * df);
                double p = exp(-dS);
                p = p < 0.0 ? 0.0 : p;
                p = p > 1.0 ? 1.0 : p;
                st->acceptance_sum = exact_acceptance_add(st, p);
                if (metro[x] < p) {
                    m[x] += cm[i];
                    m[V + xm] += cm[i];
                    m[xn] -= cm[i];
                    m[V + x] -= cm[i];
                    if (v_is_float) ((double *)v)[x] += (double)cv[i];
                    else ((int64_t *)v)[x] += cv[i];
                    st->accepted++;
                }
            }
        }
        st->proposed = V;
    }
    pcg_store(&g, rng);
    free(metro);
    free(cm);
    free(cv);
    colors_free(&C);
    return 0;
}

/* ================================================================ SURVEY.md 8(f) Villain generators */
#define PI_D 3.141592653589793 /* np.pi */

/* NumPy's float64 pairwise sum of a contiguous array (np.sum of a 1-D array; checked against
 * numpy 2.2 for n = 1..299, 513, 1000, 4096 by tools/make_golden.py's author). */
static double np_pairwise_sum(const double *a, int64_t n) {
    if (n < 8) {
        double res = 0.0;
        for (int64_t i = 0; i < n; i++) res += a[i];
        return res;
    } else if (n <= 128) {
        double r[8];
        for (int j = 0; j < 8; j++) r[j] = a[j];
        int64_t i;
        for (i = 8; i < n - (n % 8); i += 8)
            for (int j = 0; j < 8; j++) r[j] += a[i + j];
        double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
        for (; i < n; i++) res += a[i];
        return res;
    } else {
        int64_t n2 = n / 2;
        n2 -= n2 % 8;
        return np_pairwise_sum(a, n2) + np_pairwise_sum(a + n2, n - n2);
    }
}

/* value of choice index j among (-iv..-1, 1..iv): link.py:44, exact.py:38, cohomology.py:60 */
static inline int64_t nonzero_value(uint32_t j, int64_t iv) { return (int64_t)j < iv ? (int64_t)j - iv : (int64_t)j - iv + 1; }

/* SiteUpdate.step, site.py:43-118: NeighborhoodUpdate's phi proposal, n untouched; d(phi) kept and
 * updated incrementally between the colours. */
int sv_o_villain_site(int32_t N, double kappa, double interval_phi, double *phi, const int64_t *n, int32_t sweeps,
                      sv_rng *rng, sv_stats *stats) {
    if (N < 2 || sweeps < 0) return -1;
    const int64_t V = (int64_t)N * N;
    colors_t C = colors_make(N);
    double *metro = (double *)malloc(sizeof(double) * V), *dphi = (double *)malloc(sizeof(double) * 2 * V);
    double *cphi = (double *)malloc(sizeof(double) * V), *dSl = (double *)malloc(sizeof(double) * 2 * V);
    int64_t *acc = (int64_t *)malloc(sizeof(int64_t) * V);
    const double range = interval_phi - (-interval_phi);
    pcg g = pcg_load(rng);
    for (int32_t sw = 0; sw < sweeps; sw++) {
        sv_stats *st = &stats[sw];
        memset(st, 0, sizeof(*st));
        for (int64_t s = 0; s < V; s++) metro[s] = pcg_uniform(&g, 0.0, 1.0);                      /* :72 */
        for (int mu = 0; mu < 2; mu++)                                                              /* :84 */
            for (int64_t s = 0; s < V; s++) dphi[mu * V + s] = 0.0 + (phi[fwd(s, mu, N)] - phi[s]);
        for (int c = 0; c < C.ncol; c++) {
            const int64_t nc = C.count[c];
            const int64_t *sites = C.sites[c];
            for (int64_t s = 0; s < V; s++) cphi[s] = 0.0;
            for (int64_t i = 0; i < nc; i++) cphi[sites[i]] = pcg_uniform(&g, -interval_phi, range);   /* :92 */
            for (int mu = 0; mu < 2; mu++)                                                          /* :96-97 */
                for (int64_t s = 0; s < V; s++) {
                    const double cd = 0.0 + (cphi[fwd(s, mu, N)] - cphi[s]);
                    dSl[mu * V + s] = ((kappa / 2) * cd) * ((2 * (dphi[mu * V + s] - TWO_PI * (double)n[mu * V + s])) + cd);
                }
            for (int64_t i = 0; i < nc; i++) {                                                      /* :101-108 */
                const int64_t s = sites[i];
                double dS = 0.0;
                dS += dSl[s];
                dS += dSl[bwd(s, 0, N)];
                dS += dSl[V + s];
                dS += dSl[V + bwd(s, 1, N)];
                double p = exp(-dS);
                p = p < 0.0 ? 0.0 : p;
                p = p > 1.0 ? 1.0 : p;
                acc[s] = metro[s] < p;
                st->accepted += acc[s];
                st->acceptance_sum = exact_acceptance_add(st, p);
            }
            for (int64_t i = 0; i < nc; i++) cphi[sites[i]] *= (double)acc[sites[i]];             /* :111 */
            for (int64_t s = 0; s < V; s++) phi[s] = phi[s] + cphi[s];                              /* :112 */
            for (int mu = 0; mu < 2; mu++)                                                          /* :113 */
                for (int64_t s = 0; s < V; s++) dphi[mu * V + s] = dphi[mu * V + s] + (0.0 + (cphi[fwd(s, mu, N)] - cphi[s]));
        }
        st->proposed = V;
    }
    pcg_store(&g, rng);
    free(metro), free(dphi), free(cphi), free(dSl), free(acc);
    colors_free(&C);
    return 0;
}

/* LinkUpdate.step, link.py:53-99: every link at once; change_n = W * choice(n_changes, (2,N,N)) is drawn
 * BEFORE the metropolis uniforms.  stats.acceptance_sum = sum of the 2V probabilities. */
int sv_o_villain_link(int32_t N, double kappa, int64_t W, int64_t interval_n, const double *phi, int64_t *n,
                      int32_t sweeps, sv_rng *rng, sv_stats *stats) {
    if (N < 2 || sweeps < 0 || interval_n < 1) return -1;
    const int64_t V = (int64_t)N * N;
    int64_t *cn = (int64_t *)malloc(sizeof(int64_t) * 2 * V);
    double *p = (double *)malloc(sizeof(double) * 2 * V);
    const uint32_t k = (uint32_t)(2 * interval_n);
    pcg g = pcg_load(rng);
    for (int32_t sw = 0; sw < sweeps; sw++) {
        sv_stats *st = &stats[sw];
        memset(st, 0, sizeof(*st));
        for (int64_t l = 0; l < 2 * V; l++) cn[l] = W * nonzero_value(pcg_bounded(&g, k, &st->rejections), interval_n); /* :76 */
        for (int mu = 0; mu < 2; mu++)
            for (int64_t s = 0; s < V; s++) {                                                       /* :78-81 */
                const int64_t l = mu * V + s;
                const double dphi = 0.0 + (phi[fwd(s, mu, N)] - phi[s]);
                const double dS = ((-TWO_PI * kappa) * (double)cn[l]) * ((dphi - TWO_PI * (double)n[l]) - PI_D * (double)cn[l]);
                double q = exp(-dS);
                q = q < 0.0 ? 0.0 : q;
                p[l] = q > 1.0 ? 1.0 : q;
            }
        for (int64_t l = 0; l < 2 * V; l++) {                                                       /* :83-91 */
            const double u = pcg_uniform(&g, 0.0, 1.0);
            const int a = u < p[l];
            st->accepted += a;
            st->acceptance_sum = exact_acceptance_add(st, p[l]);
            if (a) n[l] += cn[l];
        }
        st->proposed = 2 * V;
    }
    pcg_store(&g, rng);
    free(cn), free(p);
    return 0;
}

/* ExactUpdate.step, exact.py:50-129: n += d(z) for a colour's worth of integer zero-forms z. */
int sv_o_villain_exact(int32_t N, double kappa, int64_t interval_z, const double *phi, int64_t *n, int32_t sweeps,
                       sv_rng *rng, sv_stats *stats) {
    if (N < 2 || sweeps < 0 || interval_z < 1) return -1;
    const int64_t V = (int64_t)N * N;
    colors_t C = colors_make(N);
    double *metro = (double *)malloc(sizeof(double) * V), *dphi = (double *)malloc(sizeof(double) * 2 * V);
    double *dSl = (double *)malloc(sizeof(double) * 2 * V);
    int64_t *z = (int64_t *)malloc(sizeof(int64_t) * V), *acc = (int64_t *)malloc(sizeof(int64_t) * V);
    const uint32_t k = (uint32_t)(2 * interval_z);
    pcg g = pcg_load(rng);
    for (int mu = 0; mu < 2; mu++)
        for (int64_t s = 0; s < V; s++) dphi[mu * V + s] = 0.0 + (phi[fwd(s, mu, N)] - phi[s]);      /* :71 */
    for (int32_t sw = 0; sw < sweeps; sw++) {
        sv_stats *st = &stats[sw];
        memset(st, 0, sizeof(*st));
        for (int64_t s = 0; s < V; s++) metro[s] = pcg_uniform(&g, 0.0, 1.0);                      /* :73 */
        for (int c = 0; c < C.ncol; c++) {
            const int64_t nc = C.count[c];
            const int64_t *sites = C.sites[c];
            for (int64_t s = 0; s < V; s++) z[s] = 0;
            for (int64_t i = 0; i < nc; i++) z[sites[i]] = nonzero_value(pcg_bounded(&g, k, &st->rejections), interval_z); /* :91 */
            for (int mu = 0; mu < 2; mu++)                                                          /* :94-99 */
                for (int64_t s = 0; s < V; s++) {
                    const int64_t l = mu * V + s;
                    const int64_t cnl = 0 + (z[fwd(s, mu, N)] - z[s]);
                    dSl[l] = ((-TWO_PI * kappa) * (double)cnl) * ((dphi[l] - TWO_PI * (double)n[l]) - PI_D * (double)cnl);
                }
            for (int64_t i = 0; i < nc; i++) {                                                      /* :103-111 */
                const int64_t s = sites[i];
                double dS = 0.0;
                dS += dSl[s];
                dS += dSl[bwd(s, 0, N)];
                dS += dSl[V + s];
                dS += dSl[V + bwd(s, 1, N)];
                double p = exp(-dS);
                p = p < 0.0 ? 0.0 : p;
                p = p > 1.0 ? 1.0 : p;
                acc[s] = metro[s] < p;
                st->accepted += acc[s];
                st->acceptance_sum = exact_acceptance_add(st, p);
            }
            for (int64_t i = 0; i < nc; i++) z[sites[i]] *= acc[sites[i]];                         /* :114 */
            for (int mu = 0; mu < 2; mu++)                                                          /* :115 */
                for (int64_t s = 0; s < V; s++) n[mu * V + s] += 0 + (z[fwd(s, mu, N)] - z[s]);
        }
        st->proposed = V;
    }
    pcg_store(&g, rng);
    free(metro), free(dphi), free(dSl), free(z), free(acc);
    colors_free(&C);
    return 0;
}

/* CohomologyUpdate.step, cohomology.py:64-117: per direction one h (choice) then one uniform; the
 * change in action on the slice x_mu = 0 is a NumPy float64 sum (pairwise).  stats.accepted counts
 * accepted directions, acceptance_sum sums the D probabilities, proposed = D = 2. */
int sv_o_villain_cohomology(int32_t N, double kappa, int64_t interval_h, const double *phi, int64_t *n, int32_t sweeps,
                            sv_rng *rng, sv_stats *stats) {
    if (N < 2 || sweeps < 0 || interval_h < 1) return -1;
    const int64_t V = (int64_t)N * N;
    double *terms = (double *)malloc(sizeof(double) * N);
    const uint32_t k = (uint32_t)(2 * interval_h);
    pcg g = pcg_load(rng);
    for (int32_t sw = 0; sw < sweeps; sw++) {
        sv_stats *st = &stats[sw];
        memset(st, 0, sizeof(*st));
        for (int mu = 0; mu < 2; mu++) {
            const int64_t h = nonzero_value(pcg_bounded(&g, k, &st->rejections), interval_h);       /* :89 */
            const double change_r = -TWO_PI * (double)h;                                            /* :94 */
            for (int64_t i = 0; i < N; i++) {
                const int64_t s = mu == 0 ? i : i * N;  /* slice x_mu = 0: (0, 0, i) or (1, i, 0) */
                const int64_t l = mu * V + s;
                /* r = d(phi) - 2 pi n, fresh each step (:82); D = 2 slices are disjoint links */
                const double r = (0.0 + (phi[fwd(s, mu, N)] - phi[s])) - TWO_PI * (double)n[l];
                terms[i] = ((kappa / 2) * change_r) * ((2 * r) + change_r);                           /* :97 */
            }
            const double dS = np_pairwise_sum(terms, N);
            double p = exp(-dS);
            p = p < 0.0 ? 0.0 : p;
            p = p > 1.0 ? 1.0 : p;
            const double u = pcg_uniform(&g, 0.0, 1.0);                                            /* :100 */
            if (u < p) {
                for (int64_t i = 0; i < N; i++) n[mu * V + (mu == 0 ? i : i * N)] += h;
                st->accepted += 1;
            }
            st->acceptance_sum += p;  /* (two terms, added in order as the device does) */
        }
        st->proposed = 2;
    }
    pcg_store(&g, rng);
    free(terms);
    return 0;
}

/* ================================================================ SURVEY.md 8(f) Worldline generators */
/* raw dense delta(v) for a D=2 two-form (reference.py:27-45, rows ('delta',2) = (0,0,1,-1),(1,0,0,+1)):
 * dv0[x] = 0 - (-1)(v[x] - v[x-e1]), dv1[x] = 0 - (+1)(v[x] - v[x-e0]); float64 for either v dtype. */
static void delta_v_raw(int64_t N, const void *v, int v_is_float, double *dv) {
    const int64_t V = N * N;
    for (int64_t s = 0; s < V; s++) {
        const int64_t b1 = bwd(s, 1, N), b0 = bwd(s, 0, N);
        if (v_is_float) {
            const double *vf = (const double *)v;
            dv[s] = 0.0 - (-(vf[s] - vf[b1]));
            dv[V + s] = 0.0 - (vf[s] - vf[b0]);
        } else {
            const int64_t *vi = (const int64_t *)v;
            dv[s] = (double)(0 - (-(vi[s] - vi[b1])));
            dv[V + s] = (double)(0 - (vi[s] - vi[b0]));
        }
    }
}

/* VortexUpdate.step, vortex.py:51-136 (D=2: one 2-form component).  metropolis = uniform(V) first (:92);
 * per colour the proposals (choice(vs) for finite W, uniform(-iv, iv) at W = inf, :105-108); delta_v kept
 * incrementally (:98, :130) -- for integer v it stays exact, for float v the patch order is the spec.
 * dS_link = ((0.5/kappa) * (-cdv/W)) * ((2 * (m - delta_v/W)) - cdv/W)   (:112-115)
 * dS      = (((0 + dSl1[x]) + dSl1[x+e0]) + dSl0[x]) + dSl0[x+e1]   (coface_sum_at, compact.py:1185-1247) */
int sv_o_worldline_vortex(int32_t N, double kappa, double Weff, int64_t interval_v, const int64_t *m, void *v,
                          int32_t v_is_float, int32_t sweeps, sv_rng *rng, sv_stats *stats) {
    if (N < 2 || sweeps < 0 || interval_v < 1) return -1;
    const int64_t V = (int64_t)N * N;
    colors_t C = colors_make(N);
    double *metro = (double *)malloc(sizeof(double) * V), *dv = (double *)malloc(sizeof(double) * 2 * V);
    double *vals = (double *)malloc(sizeof(double) * V);
    const uint32_t k = (uint32_t)(2 * interval_v);
    const double lo = -(double)interval_v, range = (double)interval_v - (-(double)interval_v);
    pcg g = pcg_load(rng);
    for (int32_t sw = 0; sw < sweeps; sw++) {
        sv_stats *st = &stats[sw];
        memset(st, 0, sizeof(*st));
        for (int64_t s = 0; s < V; s++) metro[s] = pcg_uniform(&g, 0.0, 1.0);
        delta_v_raw(N, v, v_is_float, dv);                                                      /* :98 */
        for (int c = 0; c < C.ncol; c++) {
            const int64_t nc = C.count[c];
            const int64_t *sites = C.sites[c];
            for (int64_t i = 0; i < nc; i++)
                vals[i] = v_is_float ? pcg_uniform(&g, lo, range)
                                     : (double)nonzero_value(pcg_bounded(&g, k, &st->rejections), interval_v);
            for (int64_t i = 0; i < nc; i++) {
                const int64_t s = sites[i];
                const int64_t L0 = s, L0f = fwd(s, 1, N), L1 = V + s, L1f = V + fwd(s, 0, N);
                const double a = vals[i];
                /* cdv / W on the four boundary links (delta_sparse, compact.py:1042-1116) */
                const double c0 = v_is_float ? (0.0 - (-a)) / Weff : (double)(0 - (-(int64_t)a)) / Weff;
                const double c0f = v_is_float ? (0.0 + (-a)) / Weff : (double)(0 + (-(int64_t)a)) / Weff;
                const double c1 = v_is_float ? (0.0 - a) / Weff : (double)(0 - (int64_t)a) / Weff;
                const double c1f = v_is_float ? (0.0 + a) / Weff : (double)(0 + (int64_t)a) / Weff;
                const double hk = 0.5 / kappa;
#define DSL(L, c) ((hk * (-(c))) * ((2 * ((double)m[L] - dv[L] / Weff)) - (c)))
                double dS = 0.0;
                dS += DSL(L1, c1);
                dS += DSL(L1f, c1f);
                dS += DSL(L0, c0);
                dS += DSL(L0f, c0f);
#undef DSL
                double p = exp(-dS);
                p = p < 0.0 ? 0.0 : p;
                p = p > 1.0 ? 1.0 : p;
                const int acc = metro[s] < p;
                st->accepted += acc;
                st->acceptance_sum = exact_acceptance_add(st, p);
                /* v[x] += vals * accepted; delta_v patched with the same sparse delta (:129-131) */
                if (v_is_float) {
                    const double ap = a * (double)acc;
                    ((double *)v)[s] = ((double *)v)[s] + ap;
                    dv[L0] = dv[L0] - (-ap);
                    dv[L0f] = dv[L0f] + (-ap);
                    dv[L1] = dv[L1] - ap;
                    dv[L1f] = dv[L1f] + ap;
                } else {
                    const int64_t ap = (int64_t)a * acc;
                    ((int64_t *)v)[s] += ap;
                    dv[L0] = (double)((int64_t)dv[L0] + ap);
                    dv[L0f] = (double)((int64_t)dv[L0f] - ap);
                    dv[L1] = (double)((int64_t)dv[L1] - ap);
                    dv[L1f] = (double)((int64_t)dv[L1f] + ap);
                }
            }
        }
        st->proposed = V;
    }
    pcg_store(&g, rng);
    free(metro), free(dv), free(vals);
    colors_free(&C);
    return 0;
}

/* WrappingUpdate.step, wrapping.py:43-90 (D=2).  Draws: choice(w, N) for the mu = 0 cycles (one per x,
 * constant along t), choice(w, N) for mu = 1 (one per t), then per mu uniform(0, 1, N) (:76).
 * dS_link = ((0.5/kappa) * cm) * ((2 * (m - delta(v)/W)) + cm)           (:69)
 * mu = 0: dS[x] = dS_link[0].sum(axis=0) -- NumPy reduces the outer axis sequentially from row 0;
 * mu = 1: dS[t] = dS_link[1].sum(axis=1) -- NumPy pairwise sum of each contiguous row. */
int sv_o_worldline_wrapping(int32_t N, double kappa, double Weff, int64_t interval_w, int64_t *m, const void *v,
                            int32_t v_is_float, int32_t sweeps, sv_rng *rng, sv_stats *stats) {
    if (N < 2 || sweeps < 0 || interval_w < 1) return -1;
    const int64_t V = (int64_t)N * N;
    double *dvw = (double *)malloc(sizeof(double) * 2 * V), *row = (double *)malloc(sizeof(double) * N);
    double *prob = (double *)malloc(sizeof(double) * 2 * N);
    int64_t *cm = (int64_t *)malloc(sizeof(int64_t) * 2 * N);
    const uint32_t k = (uint32_t)(2 * interval_w);
    const double hk = 0.5 / kappa;
    delta_v_by_W(N, v, v_is_float, Weff, dvw);
    pcg g = pcg_load(rng);
    for (int32_t sw = 0; sw < sweeps; sw++) {
        sv_stats *st = &stats[sw];
        memset(st, 0, sizeof(*st));
        for (int64_t i = 0; i < 2 * N; i++) cm[i] = nonzero_value(pcg_bounded(&g, k, &st->rejections), interval_w);
#define DSL(mu, t, x, c) \
    ((hk * (double)(c)) * ((2 * ((double)m[(mu) * V + (t) * N + (x)] - dvw[(mu) * V + (t) * N + (x)])) + (double)(c)))
        for (int mu = 0; mu < 2; mu++)
            for (int64_t j = 0; j < N; j++) { /* cycle j: column x = j (mu = 0) or row t = j (mu = 1) */
                const int64_t c = cm[mu * N + j];
                double dS;
                if (mu == 0) {
                    dS = DSL(0, 0, j, c);
                    for (int64_t t = 1; t < N; t++) dS = dS + DSL(0, t, j, c);
                } else {
                    for (int64_t x = 0; x < N; x++) row[x] = DSL(1, j, x, c);
                    dS = np_pairwise_sum(row, N);
                }
                double p = exp(-dS);
                p = p < 0.0 ? 0.0 : p;
                prob[mu * N + j] = p > 1.0 ? 1.0 : p;
            }
#undef DSL
        for (int mu = 0; mu < 2; mu++)
            for (int64_t j = 0; j < N; j++) {
                const double u = pcg_uniform(&g, 0.0, 1.0);
                const double p = prob[mu * N + j];
                const int acc = u < p;
                st->accepted += acc;
                st->acceptance_sum = exact_acceptance_add(st, p);
                if (acc) {
                    const int64_t c = cm[mu * N + j];
                    if (mu == 0)
                        for (int64_t t = 0; t < N; t++) m[t * N + j] += c;
                    else
                        for (int64_t x = 0; x < N; x++) m[V + j * N + x] += c;
                }
            }
        st->proposed = 2 * N;
    }
    pcg_store(&g, rng);
    free(dvw), free(row), free(prob), free(cm);
    return 0;
}

/* ---------------------------------------------------------------- worms */
/* Villain ClassicWorm.step, supervillain/generator/villain/worm.py:96-131 (per-worm draws) and
 * worm_kernel :133-183, D=2, `worms` consecutive steps on one (phi, n).  Coordinates are kept mod N:
 * the reference's FFT-convention values (lattice/two_dimensional.py:221-249) only ever index arrays,
 * where NumPy's negative indexing makes them equal to their value mod N.
 *   orientation = choice([-1,+1])                 :114  -> integers(0, 2)
 *   tail = choice(L.coordinates)                  :119  -> row integers(0, V) of the 'ij' meshgrid
 *   head = tail if W != 1 else choice(coordinates) :123
 *   loop: exit test (head==tail or W==1) and uniform >= 0.8      :143
 *         choice = integers(0, 4)                                 :148
 *         next plaquette / crossed link (two_dimensional.py:255-300): east (t,x-1) via link (0,t,x),
 *         north (t+1,x) via (1,t+1,x), west (t,x+1) via (0,t,x+1), south (t-1,x) via (1,t,x)
 *         dS = ((kappa/2)(-2 pi dn))(2 (dphi - 2 pi n) - 2 pi dn), accept on uniform < min(1, e^-dS)
 *         histogram of head - tail after every move                :181-182
 * hist (N*N, may be NULL): the LAST worm's Vortex_Vortex; lengths[w] = that worm's Worm_Length. */
int sv_o_villain_worm(int32_t N_, double kappa, int64_t W, const double *phi, int64_t *n, int32_t worms, sv_rng *rng,
                      int64_t *hist, int64_t *lengths) {
    const int64_t N = N_, V = N * N;
    if (N < 2 || worms < 0) return -1;
    double *dphi = (double *)malloc(sizeof(double) * 2 * V);
    int64_t *h = (int64_t *)malloc(sizeof(int64_t) * V);
    for (int mu = 0; mu < 2; mu++) /* d(phi), worm.py:104 */
        for (int64_t s = 0; s < V; s++) dphi[mu * V + s] = 0.0 + (phi[fwd(s, mu, N)] - phi[s]);
    static const int64_t plaq[4] = {+1, +1, -1, -1}; /* east, north, west, south, worm.py:68 */
    pcg g = pcg_load(rng);
    for (int32_t w = 0; w < worms; w++) {
        const int64_t orientation = pcg_bounded(&g, 2, NULL) ? +1 : -1;
        const int64_t ti = pcg_bounded(&g, (uint32_t)V, NULL);
        const int64_t tt = ti / N, tx = ti % N;
        int64_t ht = tt, hx = tx;
        if (W == 1) {
            const int64_t hi = pcg_bounded(&g, (uint32_t)V, NULL);
            ht = hi / N, hx = hi % N;
        }
        memset(h, 0, sizeof(int64_t) * V);
        int64_t len = 0;
        for (;;) {
            if ((ht == tt && hx == tx) || W == 1)
                if (pcg_uniform(&g, 0.0, 1.0) >= 0.8) break;
            const uint32_t c = pcg_bounded(&g, 4, NULL);
            int64_t nt = ht, nx = hx, lmu, lt = ht, lx = hx;
            switch (c) {
                case 0: nx = wrap(hx - 1, N); lmu = 0; break;                 /* east */
                case 1: nt = wrap(ht + 1, N); lmu = 1; lt = nt; break;        /* north */
                case 2: nx = wrap(hx + 1, N); lmu = 0; lx = nx; break;        /* west */
                default: nt = wrap(ht - 1, N); lmu = 1; break;                /* south */
            }
            const int64_t l = lmu * V + lt * N + lx;
            const double change_link = dphi[l] - TWO_PI * (double)n[l];
            const int64_t dn = orientation * plaq[c];
            const double dS = ((kappa / 2) * ((-TWO_PI) * (double)dn)) * (2 * change_link - TWO_PI * (double)dn);
            double A = exp(-dS);
            A = A < 1.0 ? A : 1.0;
            if (pcg_uniform(&g, 0.0, 1.0) < A) {
                ht = nt, hx = nx;
                n[l] += dn;
            }
            h[wrap(ht - tt, N) * N + wrap(hx - tx, N)] += 1;
            len++;
        }
        if (lengths) lengths[w] = len;
    }
    if (hist) memcpy(hist, h, sizeof(int64_t) * V);
    pcg_store(&g, rng);
    free(dphi), free(h);
    return 0;
}

/* Worldline ClassicWorm.step, supervillain/generator/worldline/worm.py:146-193 (draws) and worm_kernel
 * :26-94, D=2.  change_m = orientation * (+1,+1,-1,-1); moves +e0,+e1,-e0,-e1 (choice % 2 = axis,
 * choice < 2 = forward); forward crosses the link at head, backward the link at next_head;
 * dS = ((1/(2 kappa)) dm)(2 (m - delta(v)/W) + dm); exit when head == tail and uniform < 1/5.
 * hist: the last worm's Spin_Spin histogram; lengths[w] = Worm_Length. */
int sv_o_worldline_worm(int32_t N_, double kappa, double Weff, int64_t *m, const void *v, int32_t v_is_float,
                        int32_t worms, sv_rng *rng, int64_t *hist, int64_t *lengths) {
    const int64_t N = N_, V = N * N;
    if (N < 2 || worms < 0) return -1;
    double *dvw = (double *)malloc(sizeof(double) * 2 * V);
    int64_t *h = (int64_t *)malloc(sizeof(int64_t) * V);
    delta_v_by_W(N, v, v_is_float, Weff, dvw); /* worm.py:164 */
    static const int64_t div[4] = {+1, +1, -1, -1};
    pcg g = pcg_load(rng);
    for (int32_t w = 0; w < worms; w++) {
        const int64_t orientation = pcg_bounded(&g, 2, NULL) ? +1 : -1;
        const int64_t ti = pcg_bounded(&g, (uint32_t)V, NULL);
        const int64_t tail[2] = {ti / N, ti % N};
        int64_t head[2] = {tail[0], tail[1]};
        memset(h, 0, sizeof(int64_t) * V);
        int64_t len = 0;
        for (;;) {
            if (head[0] == tail[0] && head[1] == tail[1])
                if (pcg_uniform(&g, 0.0, 1.0) < 1.0 / 5) break;
            const uint32_t c = pcg_bounded(&g, 4, NULL);
            const int k = (int)(c % 2);
            const int forward = c < 2;
            int64_t next[2] = {head[0], head[1]};
            next[k] = wrap(head[k] + (forward ? 1 : -1), N);
            const int64_t *at = forward ? head : next;
            const int64_t l = k * V + at[0] * N + at[1];
            const double change_link = (double)m[l] - dvw[l];
            const int64_t dm = orientation * div[c];
            const double dS = ((1.0 / (2.0 * kappa)) * (double)dm) * (2.0 * change_link + (double)dm);
            double A = exp(-dS);
            A = 1.0 < A ? 1.0 : A;
            if (pcg_uniform(&g, 0.0, 1.0) < A) {
                head[0] = next[0], head[1] = next[1];
                m[l] += dm;
            }
            h[wrap(head[0] - tail[0], N) * N + wrap(head[1] - tail[1], N)] += 1;
            len++;
        }
        if (lengths) lengths[w] = len;
    }
    if (hist) memcpy(hist, h, sizeof(int64_t) * V);
    pcg_store(&g, rng);
    free(dvw), free(h);
    return 0;
}

/* ---------------------------------------------------------------- multi-core CPU baseline */
/* The same NeighborhoodUpdate chain with the sweep's draws generated in parallel by jumping the PCG64
 * stream (s_p = A^p s_0 + C_p, square-and-multiply) and the per-site arithmetic split over OpenMP
 * threads.  Used only as bench.py's multi-core CPU baseline ("run once on all cores and
 * once on 1 core"); tests check it equals the sequential restatement above.  Parallel sweeps need an even
 * N and no buffered half-word at the sweep start (the draws then fall on whole u64s: 4V per sweep); any
 * NumPy Lemire rejection met in a sweep makes that sweep rerun sequentially. */
static void pcg_jump(u128 *s, u128 inc, uint64_t steps) {
    u128 A = 1, C = 0, M = PCG_MULT, Ci = inc;
    while (steps) {
        if (steps & 1) {
            A = A * M;
            C = C * M + Ci;
        }
        Ci = Ci * (M + 1);
        M = M * M;
        steps >>= 1;
    }
    *s = A * *s + C;
}

static inline uint64_t xslrr(u128 s) {
    uint64_t x = (uint64_t)(s >> 64) ^ (uint64_t)s;
    unsigned rot = (unsigned)(s >> 122);
    return (x >> rot) | (x << ((64u - rot) & 63u));
}

int sv_o_villain_neighborhood_mt(int32_t N_, double kappa, int64_t W, double interval_phi, int64_t interval_n,
                                 double *phi, int64_t *n, int32_t sweeps, sv_rng *rng, sv_stats *stats,
                                 int32_t threads) {
    const int64_t N = N_, V = N * N;
    if (N < 2 || sweeps < 0 || threads < 1) return -1;
    colors_t C = colors_make(N);
    double *work = (double *)malloc(sizeof(double) * 6 * V + sizeof(int64_t) * 3 * V);
    uint64_t *raw = (uint64_t *)malloc(sizeof(uint64_t) * 4 * V);
    double *r = (double *)malloc(sizeof(double) * 2 * V), *cphi = (double *)malloc(sizeof(double) * V);
    double *dSl = (double *)malloc(sizeof(double) * 2 * V);
    int64_t *cn = (int64_t *)malloc(sizeof(int64_t) * 2 * V);
    unsigned char *acc = (unsigned char *)malloc(V);
    const uint32_t k = (uint32_t)(2 * interval_n + 1), thr = (uint32_t)((0u - k) % k);
    const double half_kappa = kappa / 2.0, range_phi = interval_phi - (-interval_phi);
    pcg g = pcg_load(rng);
    for (int32_t sw = 0; sw < sweeps; sw++) {
        sv_stats *st = &stats[sw];
        if ((N % 2) || g.has || C.ncol != 2 || k < 2) { /* general case: the sequential sweep */
            villain_sweep(N, N, kappa, W, interval_phi, interval_n, phi, n, &g, &C, st, work);
            continue;
        }
        /* 1. the sweep's 4V raw outputs, chunked over threads by stream position */
        int rejected = 0;
#pragma omp parallel num_threads(threads)
        {
            int T = 1, t = 0;
#ifdef _OPENMP
            T = omp_get_num_threads(), t = omp_get_thread_num();
#endif
            const int64_t total = 4 * V, a = total * t / T, b = total * (t + 1) / T;
            u128 s = g.s;
            pcg_jump(&s, g.inc, (uint64_t)a);
            for (int64_t p = a; p < b; p++) {
                s = s * PCG_MULT + g.inc;
                raw[p] = xslrr(s);
            }
        }
        /* positions: metro [0, V); colour c at o_c = V + c 3V/2: dphi [o_c, o_c + V/2), choice blocks of V/4 u64 */
        {
#pragma omp parallel for num_threads(threads) reduction(| : rejected)
            for (int64_t q = 0; q < 2 * V; q++) { /* the 2 x 4 blocks hold 2V uint32 draws in 8 runs of V/4 u64 */
                const int c = (int)(q / V), j = (int)((q % V) / (V / 4));
                const int64_t p = V + c * (3 * V / 2) + V / 2 + j * (V / 4) + (q % (V / 4));
                const uint64_t x = raw[p];
                const uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
                if ((uint32_t)((uint64_t)lo * k) < thr || (uint32_t)((uint64_t)hi * k) < thr) rejected = 1;
            }
        }
        if (rejected) { /* a Lemire rejection shifts its block: redo this sweep in order */
            villain_sweep(N, N, kappa, W, interval_phi, interval_n, phi, n, &g, &C, st, work);
            continue;
        }
        memset(st, 0, sizeof(*st));
        /* 2. the sweep, neighborhood.py:87-135, elementwise loops in parallel */
#pragma omp parallel for num_threads(threads)
        for (int64_t s = 0; s < V; s++)
            for (int mu = 0; mu < 2; mu++)
                r[mu * V + s] = (0.0 + (phi[fwd(s, mu, N)] - phi[s])) - TWO_PI * (double)n[mu * V + s];
        for (int c = 0; c < 2; c++) {
            const int64_t nc = C.count[c], *sites = C.sites[c], o = V + c * (3 * V / 2);
#pragma omp parallel for num_threads(threads)
            for (int64_t s = 0; s < V; s++) {
                cphi[s] = 0.0;
                cn[s] = 0;
                cn[V + s] = 0;
            }
#pragma omp parallel for num_threads(threads)
            for (int64_t i = 0; i < nc; i++) {
                const int64_t s = sites[i];
                cphi[s] = -interval_phi + range_phi * ((double)(raw[o + i] >> 11) * (1.0 / 9007199254740992.0));
                for (int mu = 0; mu < 2; mu++) {
                    const uint64_t xf = raw[o + nc + (2 * mu) * (nc / 2) + i / 2];
                    const uint64_t xb = raw[o + nc + (2 * mu + 1) * (nc / 2) + i / 2];
                    const uint32_t uf = (i & 1) ? (uint32_t)(xf >> 32) : (uint32_t)xf;
                    const uint32_t ub = (i & 1) ? (uint32_t)(xb >> 32) : (uint32_t)xb;
                    cn[mu * V + s] = W * ((int64_t)(((uint64_t)uf * k) >> 32) - interval_n);
                    cn[mu * V + bwd(s, mu, N)] = W * ((int64_t)(((uint64_t)ub * k) >> 32) - interval_n);
                }
            }
#pragma omp parallel for num_threads(threads)
            for (int64_t s = 0; s < V; s++)
                for (int mu = 0; mu < 2; mu++) {
                    const double cr = (0.0 + (cphi[fwd(s, mu, N)] - cphi[s])) - TWO_PI * (double)cn[mu * V + s];
                    dSl[mu * V + s] = (half_kappa * cr) * ((2.0 * r[mu * V + s]) + cr);
                }
            int64_t accepted = 0;
            uint64_t fx0 = 0, fx1 = 0, fx2 = 0; /* the exact acceptance limb sums (order-free) */
#pragma omp parallel for num_threads(threads) reduction(+ : accepted, fx0, fx1, fx2)
            for (int64_t i = 0; i < nc; i++) {
                const int64_t s = sites[i];
                double dS = 0.0;
                dS += dSl[s];
                dS += dSl[bwd(s, 0, N)];
                dS += dSl[V + s];
                dS += dSl[V + bwd(s, 1, N)];
                double p = exp(-dS);
                p = p < 0.0 ? 0.0 : p;
                p = p > 1.0 ? 1.0 : p;
                const double u = (double)(raw[s] >> 11) * (1.0 / 9007199254740992.0);
                acc[s] = u < p;
                accepted += acc[s];
                uint64_t w[3] = {0, 0, 0};
                fx_term_limbs(p, w);
                fx0 += w[0];
                fx1 += w[1];
                fx2 += w[2];
            }
            st->accepted += accepted;
            const uint64_t add[3] = {fx0, fx1, fx2};
            st->acceptance_sum = exact_acceptance_add_w(st, add);
#pragma omp parallel for num_threads(threads)
            for (int64_t i = 0; i < nc; i++) {
                const int64_t s = sites[i];
                const int64_t a = acc[s];
                cphi[s] = cphi[s] * (double)a;
                for (int mu = 0; mu < 2; mu++) {
                    cn[mu * V + s] *= a;
                    cn[mu * V + bwd(s, mu, N)] *= a;
                }
            }
#pragma omp parallel for num_threads(threads)
            for (int64_t s = 0; s < V; s++) {
                phi[s] = phi[s] + cphi[s];
                n[s] = n[s] + cn[s];
                n[V + s] = n[V + s] + cn[V + s];
            }
#pragma omp parallel for num_threads(threads)
            for (int64_t s = 0; s < V; s++)
                for (int mu = 0; mu < 2; mu++) {
                    const double dcp = 0.0 + (cphi[fwd(s, mu, N)] - cphi[s]);
                    r[mu * V + s] = (r[mu * V + s] + dcp) - TWO_PI * (double)cn[mu * V + s];
                }
        }
        st->proposed = V;
        pcg_jump(&g.s, g.inc, (uint64_t)(4 * V)); /* whole words only: the buffer stays empty, */
        g.buf = (uint32_t)(raw[4 * V - 1] >> 32);  /* holding (stale) the last word's high half, as NumPy's does */
    }
    pcg_store(&g, rng);
    free(work), free(raw), free(r), free(cphi), free(dSl), free(cn), free(acc);
    colors_free(&C);
    return 0;
}
