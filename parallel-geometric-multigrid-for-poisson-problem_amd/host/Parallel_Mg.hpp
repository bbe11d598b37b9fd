// Parallel_Mg.hpp — the reference's ParallelMultiGridSolver
// (3_part_parallel/Parallel_Mg.cu:3-103), same constructor and cycle signatures.
//
// v_cycle / w_cycle(phi, f, N, h) run one cycle on the MI355X context with the numerics of
// the CPU MultigridSolver (2_part_MG/MultiGrid.hpp:57-136: 2+2 Jacobi sweeps with the
// per-sweep early exit, recursion to N = 5) — bit-identical to mg_cpu_exec, unlike the
// reference GPU path (in-place racy Jacobi, symmetric prolongation, CPU tail for N <= 17).
//
// Memory contract, as the reference's (Parallel_Mg.cu:21-60 mutates the caller's
// cudaMallocManaged arrays in place, ParallelTestRunner.cu:162-163):
//   * phi and f DEVICE arrays (pgmg_host::DeviceGrid, or any device pointer), N x N
//     row-major: bound to the context once (pgmg_set_problem_device) and updated in place
//     on the device; nothing crosses PCIe per call.  With phi from DeviceGrid the context's
//     finest-level passes read and write it where it lies.  When f holds the analytic RHS
//     (rhs_is_analytic(f), as ParallelTestRunner's f does) the context regenerates it
//     in-kernel instead of reading it.  The binding (and with it the statistics and the
//     early-exit speculation history) lasts while the caller passes the same pointers.
//   * phi and f HOST arrays: uploaded and downloaded around every call (the general
//     fallback for callers whose arrays are not on the device).
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

    // f (a device array) holds compute_rhs's values (DynamicGridUtils.hpp:111-124) for this
    // problem's a, p, q and h: calls with that f regenerate it instead of reading it
    void rhs_is_analytic(const double *f) { analytic_f = f; }

    // device time of the last cycle (hipEvents), ms
    double last_device_ms() const
    {
        double ms = 0.0;
        if (ctx) pgmg_host::check(pgmg_last_elapsed_ms(ctx->get(), &ms), "pgmg_last_elapsed_ms");
        return ms;
    }

    // 1 when the last device call ran in place on the caller's phi, 0 when staged, -1 host
    int device_mode() const
    {
        if (!ctx || !bound_phi) return -1;
        int b = 0, inplace = 0;
        pgmg_host::check(pgmg_problem_device_info(ctx->get(), &b, &inplace), "pgmg_problem_device_info");
        return inplace;
    }

  private:
    int alpha;
    int ctx_N = 0;
    double ctx_eps = 0.0, ctx_h = 0.0;
    std::unique_ptr<pgmg_host::Context> ctx;
    const double *analytic_f = nullptr;
    const double *bound_phi = nullptr, *bound_f = nullptr;

    void cycle(double *phi, double *f, int N, double h, bool w)
    {
        if (!(h > 0.0)) throw std::invalid_argument("ParallelMultiGridSolver: h must be > 0");
        if (!ctx || ctx_N != N || ctx_eps != epsilon || ctx_h != h) {
            ctx.reset(new pgmg_host::Context(N, alpha, epsilon, h));
            ctx_N = N;
            ctx_eps = epsilon;
            ctx_h = h;
            bound_phi = bound_f = nullptr;
        }
        pgmg_ctx *c = ctx->get();
        const char *what = w ? "pgmg_wcycle" : "pgmg_vcycle";
        if (pgmg_host::is_device_pointer(phi)) {
            if (bound_phi != phi || bound_f != f) {
                pgmg_host::check(pgmg_set_problem_device(c, phi, f == analytic_f ? nullptr : f),
                                 "pgmg_set_problem_device");
                bound_phi = phi;
                bound_f = f;
            }
            pgmg_host::check(w ? pgmg_wcycle(c, 1) : pgmg_vcycle(c, 1), what);
            return;
        }
        bound_phi = bound_f = nullptr;
        pgmg_host::check(pgmg_set_problem(c, phi, f), "pgmg_set_problem");
        pgmg_host::check(w ? pgmg_wcycle(c, 1) : pgmg_vcycle(c, 1), what);
        pgmg_host::check(pgmg_get_solution(c, phi), "pgmg_get_solution");
    }
};
