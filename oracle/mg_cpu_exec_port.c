/*
 * mg_cpu_exec_port.c — CLI over oracle/pgmg_oracle.c (TEST INFRASTRUCTURE).
 *
 * Same output lines as oracle/ref_harness.cpp plus per-cycle wall time, so the
 * restatement can be diffed against the reference and timed as bench.py's
 * cpu_baseline ("port") on the GPU box, where /root/reference does not exist.
 *
 * Usage: mg_cpu_exec_port <V|W|F|G> <N> <cycles> <eps> [phi_out.bin]
 *   G = FMG start + W-cycles (BASELINE config 5): cycle 1 is an F-cycle, later ones W
 */
#define _POSIX_C_SOURCE 200809L
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <time.h>

typedef struct orc_ctx {
    double eps;
    int n_coarse, v1, v2, coarse_iter, alpha;
    double a, p, q;
    long long sweeps, early_exits, smooth_calls;
} orc_ctx;

void orc_ctx_init(orc_ctx *c);
void orc_rhs(const orc_ctx *c, double *f, int W, int H, double h);
void orc_v_cycle(orc_ctx *c, double *phi, const double *f, int N, double h);
void orc_w_cycle(orc_ctx *c, double *phi, const double *f, int N, double h);
void orc_f_cycle_outer(orc_ctx *c, double *phi, int N);
double orc_rel_error(const orc_ctx *c, const double *phi, int N);
double orc_residual_norm(const double *phi, const double *f, int N, double h);
uint64_t orc_hash(const double *v, long long n);

static double now_s(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + 1e-9 * ts.tv_nsec;
}

int main(int argc, char **argv)
{
    if (argc < 5) {
        fprintf(stderr, "usage: %s <V|W|F|G> <N> <cycles> <eps> [phi_out.bin]\n", argv[0]);
        return 2;
    }
    char kind = argv[1][0];
    int N = atoi(argv[2]);
    int cycles = atoi(argv[3]);
    orc_ctx c;
    orc_ctx_init(&c);
    c.eps = atof(argv[4]);
    long long L = (long long)N * N;
    double h = c.a / (N - 1);
    double *phi = calloc((size_t)L, sizeof(double));
    double *f = calloc((size_t)L, sizeof(double));
    if (!phi || !f) return 4;
    orc_rhs(&c, f, N, N, h);
    for (int k = 1; k <= cycles; ++k) {
        double t0 = now_s();
        if (kind == 'V')
            orc_v_cycle(&c, phi, f, N, h);
        else if (kind == 'W' || (kind == 'G' && k > 1))
            orc_w_cycle(&c, phi, f, N, h);
        else
            orc_f_cycle_outer(&c, phi, N);
        double t1 = now_s();
        printf("cycle %d relerr %.17g res %.17g center %.17g hash %016llx sweeps %lld exits %lld"
               " seconds %.6f\n",
               k, orc_rel_error(&c, phi, N), orc_residual_norm(phi, f, N, h),
               phi[(long long)(N / 2) * N + N / 2], (unsigned long long)orc_hash(phi, L), c.sweeps,
               c.early_exits, t1 - t0);
        fflush(stdout);
    }
    if (argc > 5) {
        FILE *fp = fopen(argv[5], "wb");
        if (!fp) return 3;
        fwrite(phi, sizeof(double), (size_t)L, fp);
        fclose(fp);
    }
    free(phi);
    free(f);
    return 0;
}
