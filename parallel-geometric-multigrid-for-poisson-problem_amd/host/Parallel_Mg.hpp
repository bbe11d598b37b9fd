// Parallel_Mg.hpp — the reference's ParallelMultiGridSolver
// (3_part_parallel/Parallel_Mg.cu:3-103), same constructor and cycle signatures.
//
// v_cycle / w_cycle take the caller's HOST arrays phi (in/out) and f, N x N
// row-major (the reference takes managed memory usable from both sides).  Each call
// runs one cycle on the MI355X context with the numerics of the CPU MultigridSolver
// (2_part_MG/MultiGrid.hpp:57-136: 2+2 Jacobi sweeps with the per-sweep early exit,
// recursion to N = 5) — bit-identical to mg_cpu_exec, unlike the reference GPU path
// (in-place racy Jacobi, symmetric prolongation, CPU tail for N <= 17).
// The context (level pyramid in HBM) is created on first use for a given (N, h, epsilon)
// and kept; h is the caller's finest mesh width, doubled per level as the reference does.
#pragma once
#include <memory>
#include <stdexcept>

#include "pgmg.hpp"

class ParallelMultiGridSolver {
  public:
    int N_cpu = 17;         // kept for interface parity; the whole hierarchy runs on the GPU
    double epsilon = 1e-7;  // smoother early-exit tolerance (Parallel_Mg.cu:14)

    explicit ParallelMultiGridSolver(int alpha_) : alpha(alpha_) {}

    void v_cycle(double *phi, double *f, int N, double h) { cycle(phi, f, N, h, false); }
    void w_cycle(double *phi, double *f, int N, double h) { cycle(phi, f, N, h, true); }

    // device time of the last cycle (hipEvents), ms
    double last_device_ms() const
    {
        double ms = 0.0;
        if (ctx) pgmg_host::check(pgmg_last_elapsed_ms(ctx->get(), &ms), "pgmg_last_elapsed_ms");
        return ms;
    }

  private:
    int alpha;
    int ctx_N = 0;
    double ctx_eps = 0.0, ctx_h = 0.0;
    std::unique_ptr<pgmg_host::Context> ctx;

    void cycle(double *phi, double *f, int N, double h, bool w)
    {
        if (!(h > 0.0)) throw std::invalid_argument("ParallelMultiGridSolver: h must be > 0");
        if (!ctx || ctx_N != N || ctx_eps != epsilon || ctx_h != h) {
            ctx.reset(new pgmg_host::Context(N, alpha, epsilon, h));
            ctx_N = N;
            ctx_eps = epsilon;
            ctx_h = h;
        }
        pgmg_ctx *c = ctx->get();
        pgmg_host::check(pgmg_set_problem(c, phi, f), "pgmg_set_problem");
        pgmg_host::check(w ? pgmg_wcycle(c, 1) : pgmg_vcycle(c, 1), w ? "pgmg_wcycle" : "pgmg_vcycle");
        pgmg_host::check(pgmg_get_solution(c, phi), "pgmg_get_solution");
    }
};
