// SequentialOps.hpp — the CPU half of the reference's per-op timing study
// (3_part_parallel/ParallelTestRunner.cu:231-468, plotTimeSequentialVsParallel).
//
// The reference times each GPU op beside its sequential CPU counterpart for N < 4096
// and writes both to OUTPUT_RESULT/timings_<op>_{cpu,gpu}.txt, which
// python_plot/plot_timings_SeqVsParall.py reads.  These are those CPU counterparts,
// single-threaded, with the reference's loop structure:
//   jacobi       JacobiSmoother::smooth (Smoother.hpp:38-116): num_iter+1 out-of-place
//                sweeps, copy back, residual norm over the whole array, exit < eps
//   residual     DynamicGridUtils::compute_residual (DynamicGridUtils.hpp:59-69)
//   restriction  restrict_full_weighting_2 (ParallelTestRunner.cu:10-36)
//   prolongation prolongation_2 (ParallelTestRunner.cu:38-67)
// They exist only to be timed against the MI355X ops; no solver path calls them.
#pragma once
#include <algorithm>
#include <cmath>
#include <vector>

namespace pgmg_seq {

inline void residual(double *r, const double *x, const double *f, int W, int H, double h)
{
    for (int y = 1; y < H - 1; ++y)
        for (int i = 1; i < W - 1; ++i) {
            const int k = y * W + i;
            r[k] = f[k] - (1.0 / (h * h)) * (4 * x[k] - x[k - 1] - x[k + 1] - x[k - W] - x[k + W]);
        }
}

inline double norm(const double *v, size_t n)
{
    double s = 0.0;
    for (size_t k = 0; k < n; ++k) s += v[k] * v[k];
    return std::sqrt(s);
}

// returns the sweeps performed
inline int jacobi(double *x, const double *f, int W, int H, double h, int num_iter, double eps)
{
    const size_t L = (size_t)W * H;
    std::vector<double> out(x, x + L), r(L, 0.0);
    for (int it = 0; it <= num_iter; ++it) {
        for (int y = 1; y < H - 1; ++y)
            for (int i = 1; i < W - 1; ++i) {
                const int k = y * W + i;
                out[k] = 0.25 * ((h * h * f[k]) + x[k - 1] + x[k + 1] + x[k - W] + x[k + W]);
            }
        std::copy(out.begin(), out.end(), x);
        residual(r.data(), x, f, W, H, h);
        if (norm(r.data(), L) < eps) return it + 1;
    }
    return num_iter + 1;
}

inline void restrict_full_weighting(const double *fine, double *coarse, int Nf, int Nc)
{
    for (int i = 0; i < Nc; ++i) {
        coarse[i] = 0.0;
        coarse[(size_t)(Nc - 1) * Nc + i] = 0.0;
        coarse[(size_t)i * Nc] = 0.0;
        coarse[(size_t)i * Nc + Nc - 1] = 0.0;
    }
    for (int jc = 1; jc < Nc - 1; ++jc)
        for (int ic = 1; ic < Nc - 1; ++ic) {
            const size_t c = (size_t)jc * Nc + ic, k = (size_t)(2 * jc) * Nf + 2 * ic;
            coarse[c] = 0.25 * fine[k] +
                        0.125 * (fine[k + 1] + fine[k - 1] + fine[k + Nf] + fine[k - Nf]) +
                        0.0625 * (fine[k - Nf - 1] + fine[k - Nf + 1] + fine[k + Nf - 1] +
                                  fine[k + Nf + 1]);
        }
}

inline void prolongation(double *fine, const double *coarse, int Nf, int Nc)
{
    for (int jc = 1; jc < Nc - 1; ++jc)
        for (int ic = 1; ic < Nc - 1; ++ic) {
            const size_t c = (size_t)jc * Nc + ic, J = 2 * jc, I = 2 * ic;
            fine[J * Nf + I] += coarse[c];
            fine[(J + 1) * Nf + I] += 0.5 * (coarse[c] + coarse[c + Nc]);
            fine[J * Nf + I + 1] += 0.5 * (coarse[c] + coarse[c + 1]);
            fine[(J + 1) * Nf + I + 1] +=
                0.25 * (coarse[c] + coarse[c + 1] + coarse[c + Nc] + coarse[c + Nc + 1]);
        }
    for (int j = 0; j < Nf; ++j)
        for (int i = 0; i < Nf; ++i)
            if (i == 0 || i == Nf - 1 || j == 0 || j == Nf - 1) fine[(size_t)j * Nf + i] = 0.0;
}

}  // namespace pgmg_seq
