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
//   * mixed: a device phi with a host f binds phi and a device copy of f (uploaded at every
//     call); a host phi with a device f reads f back and takes the host path.
// The context (level pyramid in HBM) is created on first use for a given (N, h, epsilon)
// and kept; h is the caller's finest mesh width, doubled per level as the reference does.
#pragma once
#include <memory>
#include <stdexcept>
#include <vector>

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

    // forget the device binding: the next call binds (phi, f) afresh (statistics and the
    // early-exit speculation history restart).  Calls rebind by themselves when the pointers
    // change or a pgmg_alloc_grid phi / f was freed and re-allocated at the same address.
    void rebind() { bound_phi = bound_f = nullptr; }

  private:
    int alpha;
    int ctx_N = 0;
    double ctx_eps = 0.0, ctx_h = 0.0;
    std::unique_ptr<pgmg_host::Context> ctx;
    const double *analytic_f = nullptr;
    const double *bound_phi = nullptr, *bound_f = nullptr;
    unsigned long long bound_phi_serial = 0, bound_f_serial = 0;
    // f staged on the device when phi is a device array and f a host one
    std::unique_ptr<pgmg_host::DeviceArray> f_dev;

    static unsigned long long serial_of(const double *p)
    {
        unsigned long long s = 0;
        pgmg_host::check(pgmg_grid_serial(p, &s), "pgmg_grid_serial");
        return s;
    }

    void cycle(double *phi, double *f, int N, double h, bool w)
    {
        if (!(h > 0.0)) throw std::invalid_argument("ParallelMultiGridSolver: h must be > 0");
        if (!ctx || ctx_N != N || ctx_eps != epsilon || ctx_h != h) {
            ctx.reset(new pgmg_host::Context(N, alpha, epsilon, h));
            ctx_N = N;
            ctx_eps = epsilon;
            ctx_h = h;
            rebind();
        }
        pgmg_ctx *c = ctx->get();
        const char *what = w ? "pgmg_wcycle" : "pgmg_vcycle";
        const bool phi_dev = pgmg_host::is_device_pointer(phi);
        const bool f_dev_ptr = f != nullptr && pgmg_host::is_device_pointer(f);
        if (phi_dev) {
            // f for the device binding: the analytic RHS (regenerated), the caller's device f,
            // or a host f copied into a device array of our own at every call
            const double *fb = f == analytic_f ? nullptr : f;
            if (fb && !f_dev_ptr) {
                const size_t n = (size_t)N * N;
                if (!f_dev || f_dev->size() != n) f_dev.reset(new pgmg_host::DeviceArray(n));
                f_dev->upload(f);
                fb = f_dev->get();
            }
            const unsigned long long ps = serial_of(phi), fs = fb ? serial_of(fb) : 0;
            if (bound_phi != phi || bound_f != fb || bound_phi_serial != ps || bound_f_serial != fs) {
                pgmg_host::check(pgmg_set_problem_device(c, phi, fb), "pgmg_set_problem_device");
                bound_phi = phi;
                bound_f = fb;
                bound_phi_serial = ps;
                bound_f_serial = fs;
            }
            pgmg_host::check(w ? pgmg_wcycle(c, 1) : pgmg_vcycle(c, 1), what);
            return;
        }
        rebind();
        // host phi: upload / download around the call (a device f is read back first)
        std::vector<double> fh;
        const double *fp = f;
        if (f_dev_ptr) {
            fh.resize((size_t)N * N);
            pgmg_host::check(pgmg_memcpy_d2h(fh.data(), f, fh.size() * sizeof(double)), "f to host");
            fp = fh.data();
        }
        pgmg_host::check(pgmg_set_problem(c, phi, fp), "pgmg_set_problem");
        pgmg_host::check(w ? pgmg_wcycle(c, 1) : pgmg_vcycle(c, 1), what);
        pgmg_host::check(pgmg_get_solution(c, phi), "pgmg_get_solution");
    }
};
