/*
 * pgmg_oracle.c — CPU restatement of the reference's `mg_cpu_exec` multigrid.
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the parity checker for the MI355X
 * HIP path.  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
 * leg may load it.  The product library (libpgmg.so) never links or calls it.
 *
 * Pinned: tests/golden/ holds vectors produced by the reference's own C++
 * (/root/reference/2_part_MG/MultiGrid.hpp driven by oracle/ref_harness.cpp,
 * built by oracle/Makefile into oracle/_ref/).  tests/test_oracle_golden.py
 * checks this restatement against them bit for bit.
 *
 * Semantics restated (reference file:line):
 *   - grid: N x N vertex-centred, row-major idx = y*W + x, h = a/(N-1)
 *     (2_part_MG/MultiGridTestRunner.hpp:130-131, DynamicGridUtils.hpp:52)
 *   - Jacobi smoother: num_iter+1 sweeps, out-of-place, copy back, then the
 *     residual norm over the whole array (boundary 0) and `norm < eps` early
 *     exit after EVERY sweep (Smoother.hpp:38-116)
 *   - residual (DynamicGridUtils.hpp:59-69), norm (:21-27), rhs (:111-124),
 *     exact solution (:97-108)
 *   - v_cycle / w_cycle / f_cycle / compute_coarsest_grid
 *     (2_part_MG/MultiGrid.hpp:28-183), restriction (:187-205),
 *     prolongation incl. the skipped fine row/col 1 (:208-226)
 *   - the GPU path's symmetric prolongation, prolungator_kernel
 *     (3_part_parallel/Parallel_Method.cu:79-138)
 * Floating point: compiled with -ffp-contract=off so every expression rounds
 * exactly as the reference's plain C++ does (no FMA contraction).
 *
 * Element type: `real` = double (liboracle.so, the pinned restatement) or, with
 * -DORC_REAL=float, float (liboracle_f32.so): the same algorithm with every grid
 * value and every arithmetic operation in fp32, h*h and 1/(h*h) rounded once from
 * fp64, the RHS computed in fp64 and rounded, squares of the norms accumulated in
 * fp64.  That is the checker of the library's PGMG_PRECISION_FP32 variant (SURVEY
 * §8 f3; the reference itself is fp64-only).  For real = double every expression
 * below is the one the reference evaluates.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#ifndef M_PI
#define M_PI 3.14159265358979323846
#endif

#ifndef ORC_REAL
#define ORC_REAL double
#endif
typedef ORC_REAL real;

int orc_real_size(void) { return (int)sizeof(real); }

typedef struct orc_ctx {
    double eps;        /* smoother tolerance (MultiGridTestRunner.hpp:144 -> 1e-7) */
    int n_coarse;      /* recursion floor N_coarse (MultiGrid.hpp:19 -> 5)        */
    int v1, v2;        /* pre/post smoothing num_iter (MultiGrid.hpp:15-16)       */
    int coarse_iter;   /* num_iter on the coarsest grid (MultiGrid.hpp:61 -> 10)  */
    int alpha;         /* W-cycle recursions (main.cpp:15 -> 3)                   */
    double a, p, q;    /* problem constants (globals.cpp:2-4)                     */
    /* statistics */
    long long sweeps;
    long long early_exits;
    long long smooth_calls;
} orc_ctx;

void orc_ctx_init(orc_ctx *c)
{
    c->eps = 1e-7;
    c->n_coarse = 5;
    c->v1 = 1;
    c->v2 = 1;
    c->coarse_iter = 10;
    c->alpha = 3;
    c->a = 1.0;
    c->p = 1.0;
    c->q = 1.0;
    c->sweeps = 0;
    c->early_exits = 0;
    c->smooth_calls = 0;
}

int orc_ctx_size(void) { return (int)sizeof(orc_ctx); }

/* ---- grid utilities (DynamicGridUtils.hpp) ---------------------------- */

void orc_zero(real *x, long long n)
{
    for (long long i = 0; i < n; ++i)
        x[i] = 0;
}

/* DynamicGridUtils.hpp:21-27 — sequential sum of squares over l entries */
double orc_norm(const real *v, long long l)
{
    double s = 0.0;
    for (long long i = 0; i < l; ++i)
        s += (double)v[i] * (double)v[i];
    return sqrt(s);
}

/* DynamicGridUtils.hpp:59-69 — interior only; boundary of r untouched */
void orc_residual(real *r, const real *x, const real *f, int W, int H, double h)
{
    const real ih = (real)(1.0 / (h * h));
    for (int y = 1; y < H - 1; ++y) {
        for (int xi = 1; xi < W - 1; ++xi) {
            long long k = (long long)y * W + xi;
            r[k] = f[k] - ih * (4 * x[k] - x[k - 1] - x[k + 1] - x[k - W] - x[k + W]);
        }
    }
}

/* DynamicGridUtils.hpp:111-124 */
void orc_rhs(const orc_ctx *c, real *f, int W, int H, double h)
{
    double factor = (M_PI * M_PI / (c->a * c->a)) * (c->p * c->p + c->q * c->q);
    for (int j = 0; j < H; ++j) {
        for (int i = 0; i < W; ++i) {
            double xx = i * h;
            double yy = j * h;
            f[(long long)j * W + i] = (real)(factor * sin(c->p * M_PI * xx / c->a) *
                                             sin(c->q * M_PI * yy / c->a));
        }
    }
}

/* DynamicGridUtils.hpp:97-108 */
void orc_exact(const orc_ctx *c, double *u, double h, int W, int H)
{
    for (int j = 0; j < H; ++j) {
        for (int i = 0; i < W; ++i) {
            double xx = i * h;
            double yy = j * h;
            u[(long long)j * W + i] = sin(c->p * M_PI * xx / c->a) * sin(c->q * M_PI * yy / c->a);
        }
    }
}

/* ||r(x)|| of Smoother.hpp:75-76 without the residual buffer: the same r values
 * (orc_residual's expression, rounded to `real`), squared and summed in the same
 * sequential index order as orc_norm over the whole array — the boundary entries of the
 * reference's buffer are 0 and adding +0.0 leaves the sum unchanged — so the result is
 * bitwise orc_norm(r, L).  Saves one grid of host memory (N = 32769 goldens). */
static double orc_residual_norm_seq(const real *x, const real *f, int W, int H, double h)
{
    const real ih = (real)(1.0 / (h * h));
    double s = 0.0;
    for (int y = 1; y < H - 1; ++y) {
        for (int xi = 1; xi < W - 1; ++xi) {
            long long k = (long long)y * W + xi;
            const real r = f[k] - ih * (4 * x[k] - x[k - 1] - x[k + 1] - x[k - W] - x[k + W]);
            s += (double)r * (double)r;
        }
    }
    return sqrt(s);
}

/* ---- Jacobi smoother (Smoother.hpp:38-116) ------------------------------
 * Returns the number of sweeps performed.  `work` must hold W*H elements.
 */
int orc_jacobi_smooth(orc_ctx *c, real *x, const real *f, int W, int H, double h,
                      int num_iter, real *work)
{
    long long L = (long long)W * H;
    real *out = work;       /* Smoother.hpp:46-47: seeded with x */
    const real hh = (real)(h * h);
    memcpy(out, x, sizeof(real) * L);
    int done = 0;
    c->smooth_calls++;
    for (int it = 0; it <= num_iter; ++it) {
        for (int y = 1; y < H - 1; ++y) {
            for (int xi = 1; xi < W - 1; ++xi) {
                long long k = (long long)y * W + xi;
                out[k] = (real)0.25 * ((hh * f[k]) + x[k - 1] + x[k + 1] + x[k - W] + x[k + W]);
            }
        }
        memcpy(x, out, sizeof(real) * L);
        ++done;
        c->sweeps++;
        double nr = orc_residual_norm_seq(x, f, W, H, h);
        if (nr < c->eps) {
            c->early_exits++;
            break;
        }
    }
    return done;
}

/* ---- transfer operators (MultiGrid.hpp:187-226) ------------------------ */

void orc_restrict(const real *F, real *C, int Nf, int Nc)
{
    for (int jc = 1; jc < Nc - 1; ++jc) {
        for (int ic = 1; ic < Nc - 1; ++ic) {
            long long c = (long long)jc * Nc + ic;
            long long k = (long long)(2 * jc) * Nf + 2 * ic;
            C[c] = (real)0.25 * F[k] +
                   (real)0.125 * (F[k + 1] + F[k - 1] + F[k + Nf] + F[k - Nf]) +
                   (real)0.0625 * (F[k - Nf - 1] + F[k - Nf + 1] + F[k + Nf - 1] + F[k + Nf + 1]);
        }
    }
}

/* fine += P * coarse; the loop bounds never touch fine row/col 1 (MultiGrid.hpp:210-225) */
void orc_prolong(real *F, const real *C, int Nf, int Nc)
{
    for (int jc = 1; jc < Nc - 1; ++jc) {
        for (int ic = 1; ic < Nc - 1; ++ic) {
            long long c = (long long)jc * Nc + ic;
            long long J = 2 * jc, I = 2 * ic;
            F[J * Nf + I] += C[c];
            F[(J + 1) * Nf + I] += (real)0.5 * (C[c] + C[c + Nc]);
            F[J * Nf + I + 1] += (real)0.5 * (C[c] + C[c + 1]);
            F[(J + 1) * Nf + I + 1] += (real)0.25 * (C[c] + C[c + 1] + C[c + Nc] + C[c + Nc + 1]);
        }
    }
}

/* fine += P_sym * coarse over the thread grid [0, ext_y) x [0, ext_x) of the reference's
 * GPU prolongation `prolungator_kernel` (3_part_parallel/Parallel_Method.cu:79-138), launched
 * by Parallel::ComputeProlungator (:188-199) with max(1, fine_N / num_thread) blocks of
 * num_thread^2 threads per axis.  Unlike MultiGrid.hpp:208-226 it is symmetric: every
 * interior fine point is corrected (row/col 1 included), and the boundary points the grid
 * covers are set to 0 (:88-93).  Per case (:100-135): even/even injection; odd/odd the
 * 4-corner average 0.25*(c + c_e + c_s + c_se) if cx+1 < Wc and cy+1 < Hc, else 0;
 * odd column 0.5*(c + c_e) if cx+1 < Wc; odd row 0.5*(c + c_s) if cy+1 < Hc.  Points
 * outside the thread grid are untouched (for fine_N = 2^k+1 > num_thread the grid is
 * fine_N-1 wide, so the last boundary row/column keep their values). */
void orc_prolong_sym(real *F, const real *C, int Hc, int Wc, int Hf, int Wf, int ext_y, int ext_x)
{
    for (int y = 0; y < ext_y && y < Hf; ++y) {
        for (int x = 0; x < ext_x && x < Wf; ++x) {
            long long k = (long long)y * Wf + x;
            if (y == 0 || y == Hf - 1 || x == 0 || x == Wf - 1) {
                F[k] = 0;
                continue;
            }
            real v = 0;
            int cx = x / 2, cy = y / 2;
            long long c = (long long)cy * Wc + cx;
            if (x % 2 == 0 && y % 2 == 0) {
                v = C[c];
            } else if (x % 2 == 1 && y % 2 == 1) {
                if (cx + 1 < Wc && cy + 1 < Hc)
                    v = (real)0.25 * (C[c] + C[c + 1] + C[c + Wc] + C[c + Wc + 1]);
            } else if (x % 2 == 1 && y % 2 == 0) {
                if (cx + 1 < Wc) v = (real)0.5 * (C[c] + C[c + 1]);
            } else {
                if (cy + 1 < Hc) v = (real)0.5 * (C[c] + C[c + Wc]);
            }
            F[k] += v;
        }
    }
}

/* ---- cycles ------------------------------------------------------------- */

static real *orc_alloc(long long n) { return (real *)calloc((size_t)n, sizeof(real)); }

/* one smoother call with its own scratch grid (allocated only while it runs) */
static void orc_smooth_alloc(orc_ctx *c, real *x, const real *f, int N, double h, int num_iter)
{
    real *work = orc_alloc((long long)N * N);
    orc_jacobi_smooth(c, x, f, N, N, h, num_iter, work);
    free(work);
}

/* MultiGrid.hpp:57-94 */
void orc_v_cycle(orc_ctx *c, real *phi, const real *f, int N, double h)
{
    long long L = (long long)N * N;
    if (N <= c->n_coarse) {
        orc_smooth_alloc(c, phi, f, N, h, c->coarse_iter);
        return;
    }
    orc_smooth_alloc(c, phi, f, N, h, c->v1);
    real *res = orc_alloc(L);
    orc_residual(res, phi, f, N, N, h);
    int Nc = (N - 1) / 2 + 1;
    long long Lc = (long long)Nc * Nc;
    real *rc = orc_alloc(Lc);
    orc_restrict(res, rc, N, Nc);
    free(res);   /* dead from here (host memory at N = 32769) */
    real *ec = orc_alloc(Lc);
    orc_v_cycle(c, ec, rc, Nc, 2 * h);
    orc_prolong(phi, ec, N, Nc);
    orc_smooth_alloc(c, phi, f, N, h, c->v2);
    free(rc);
    free(ec);
}

/* MultiGrid.hpp:96-136 */
void orc_w_cycle(orc_ctx *c, real *phi, const real *f, int N, double h)
{
    long long L = (long long)N * N;
    if (N <= c->n_coarse) {
        orc_smooth_alloc(c, phi, f, N, h, c->coarse_iter);
        return;
    }
    orc_smooth_alloc(c, phi, f, N, h, c->v1);
    real *res = orc_alloc(L);
    orc_residual(res, phi, f, N, N, h);
    int Nc = (N - 1) / 2 + 1;
    long long Lc = (long long)Nc * Nc;
    real *rc = orc_alloc(Lc);
    orc_restrict(res, rc, N, Nc);
    free(res);   /* dead from here (host memory at N = 32769) */
    real *ec = orc_alloc(Lc);
    for (int i = 0; i < c->alpha; ++i)
        orc_w_cycle(c, ec, rc, Nc, 2.0 * h);
    orc_prolong(phi, ec, N, Nc);
    orc_smooth_alloc(c, phi, f, N, h, c->v2);
    free(rc);
    free(ec);
}

/* MultiGrid.hpp:28-55 — restrict `fine` repeatedly down to N_coarsest.
 * Writes the coarsest grid into `out` (N_coarsest^2 doubles). */
void orc_coarsest_grid(const real *fine, real *out, int N_fine, int N_coarsest)
{
    int Nc = N_fine;
    real *cur = orc_alloc((long long)Nc * Nc);
    memcpy(cur, fine, sizeof(real) * (size_t)((long long)Nc * Nc));
    while (Nc > N_coarsest) {
        int Nn = (Nc - 1) / 2 + 1;
        real *nx = orc_alloc((long long)Nn * Nn);
        orc_restrict(cur, nx, Nc, Nn);
        free(cur);
        cur = nx;
        Nc = Nn;
    }
    memcpy(out, cur, sizeof(real) * (size_t)((long long)Nc * Nc));
    free(cur);
}

/* MultiGrid.hpp:138-183 — full multigrid from N_init up to N_final; the
 * result (N_final^2) goes to `final_solution`.  The finer RHS is regenerated
 * analytically on every level (MultiGrid.hpp:162). */
void orc_f_cycle(orc_ctx *c, const real *phi, const real *f, int N_init, double h_init,
                 int N_final, real *final_solution)
{
    int N = N_init;
    double h = h_init;
    long long L = (long long)N * N;
    real *phic = orc_alloc(L);
    real *fc = orc_alloc(L);
    memcpy(phic, phi, sizeof(real) * (size_t)L);
    memcpy(fc, f, sizeof(real) * (size_t)L);
    while (N < N_final) {
        orc_smooth_alloc(c, phic, fc, N, h, 3);
        int Nf = 2 * N - 1;
        long long Lf = (long long)Nf * Nf;
        real *phif = orc_alloc(Lf);
        real *ff = orc_alloc(Lf);
        orc_rhs(c, ff, Nf, Nf, h / 2);
        orc_prolong(phif, phic, Nf, N);
        orc_v_cycle(c, phif, ff, Nf, h / 2);
        free(phic);
        free(fc);
        phic = phif;
        fc = ff;
        N = Nf;
        h /= 2;
    }
    memcpy(final_solution, phic, sizeof(real) * (size_t)((long long)N * N));
    free(phic);
    free(fc);
}

/* One outer iteration of MultiGridTestRunner::run_cycle("F-cycle")
 * (MultiGridTestRunner.hpp:192-205): restrict phi to N_coarse, run f_cycle
 * from there with the analytic coarse RHS, copy the result into phi. */
void orc_f_cycle_outer(orc_ctx *c, real *phi, int N)
{
    int n0 = c->n_coarse;
    double h0 = 1.0 / (n0 - 1);
    real *f0 = orc_alloc((long long)n0 * n0);
    real *p0 = orc_alloc((long long)n0 * n0);
    orc_rhs(c, f0, n0, n0, h0);
    orc_coarsest_grid(phi, p0, N, n0);
    orc_f_cycle(c, p0, f0, n0, h0, N, phi);
    free(f0);
    free(p0);
}

/* ---- harness helpers ---------------------------------------------------- */

/* ||phi - u|| / ||u|| as printed by MultiGridTestRunner.hpp:252-255 */
double orc_rel_error(const orc_ctx *c, const real *phi, int N)
{
    /* sequential sums in fp64 over the exact solution of orc_exact (fp32: phi widened) */
    double h = c->a / (N - 1);
    double se = 0.0, su = 0.0;
    for (int j = 0; j < N; ++j) {
        for (int i = 0; i < N; ++i) {
            double xx = i * h;
            double yy = j * h;
            double u = sin(c->p * M_PI * xx / c->a) * sin(c->q * M_PI * yy / c->a);
            double e = (double)phi[(long long)j * N + i] - u;
            se += e * e;
            su += u * u;
        }
    }
    return sqrt(se) / sqrt(su);
}

/* sqrt(sum_interior r^2) of the current iterate */
double orc_residual_norm(const real *phi, const real *f, int N, double h)
{
    long long L = (long long)N * N;
    real *r = orc_alloc(L);
    orc_residual(r, phi, f, N, N, h);
    double n = orc_norm(r, L);
    free(r);
    return n;
}

/* FNV-style 64-bit hash over the IEEE words */
uint64_t orc_hash(const real *v, long long n)
{
    uint64_t hsh = 1469598103934665603ULL;
    for (long long i = 0; i < n; ++i) {
        uint64_t w = 0;
        memcpy(&w, &v[i], sizeof(real));
        hsh = (hsh ^ w) * 1099511628211ULL;
    }
    return hsh;
}

/* The robustness right-hand side of SURVEY §8(d): uniform values in [-1, 1) from
 * std::mt19937_64 seeded with `seed`, drawn for every point in row-major order
 * (boundary points included, then set to 0), each as libstdc++'s
 * std::uniform_real_distribution<double>(-1, 1) computes it:
 * u = generate_canonical<double, 53> = (double)x / 2^64 (k = 1 draw of 64 bits; u >= 1
 * becomes nextafter(1, 0)), value = u * (b - a) + a.  The engine is the standard's
 * mt19937_64 (w 64, n 312, m 156, r 31; its required 10000th output of the default
 * seed is checked by tests/test_oracle_mt_rhs.py), and tests/golden/mt_rhs.json
 * (tests/golden/make_mt_rhs.cpp, libstdc++ itself) pins the values. */
typedef struct {
    uint64_t mt[312];
    int i;
} orc_mt64;

static void orc_mt64_seed(orc_mt64 *g, uint64_t seed)
{
    g->mt[0] = seed;
    for (int i = 1; i < 312; ++i)
        g->mt[i] = 6364136223846793005ULL * (g->mt[i - 1] ^ (g->mt[i - 1] >> 62)) + (uint64_t)i;
    g->i = 312;
}

static uint64_t orc_mt64_next(orc_mt64 *g)
{
    const uint64_t up = ~((1ULL << 31) - 1), lo = (1ULL << 31) - 1;
    if (g->i >= 312) {
        for (int k = 0; k < 312; ++k) {
            const uint64_t x = (g->mt[k] & up) | (g->mt[(k + 1) % 312] & lo);
            uint64_t xa = x >> 1;
            if (x & 1ULL) xa ^= 0xB5026F5AA96619E9ULL;
            g->mt[k] = g->mt[(k + 156) % 312] ^ xa;
        }
        g->i = 0;
    }
    uint64_t y = g->mt[g->i++];
    y ^= (y >> 29) & 0x5555555555555555ULL;
    y ^= (y << 17) & 0x71D67FFFEDA60000ULL;
    y ^= (y << 37) & 0xFFF7EEE000000000ULL;
    y ^= y >> 43;
    return y;
}

/* the n-th output (1-based) of mt19937_64 seeded with `seed` */
uint64_t orc_mt64_nth(uint64_t seed, long long n)
{
    orc_mt64 g;
    orc_mt64_seed(&g, seed);
    uint64_t y = 0;
    for (long long k = 0; k < n; ++k) y = orc_mt64_next(&g);
    return y;
}

void orc_rhs_mt64(real *f, int N, uint64_t seed)
{
    orc_mt64 g;
    orc_mt64_seed(&g, seed);
    const double two64 = 18446744073709551616.0;
    for (int j = 0; j < N; ++j)
        for (int i = 0; i < N; ++i) {
            double u = (double)orc_mt64_next(&g) / two64;
            if (u >= 1.0) u = nextafter(1.0, 0.0);
            const double v = u * (1.0 - -1.0) + -1.0;
            const int b = j == 0 || i == 0 || j == N - 1 || i == N - 1;
            f[(long long)j * N + i] = b ? (real)0 : (real)v;
        }
}
