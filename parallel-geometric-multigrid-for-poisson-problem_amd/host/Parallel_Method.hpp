// Parallel_Method.hpp — the reference's `class Parallel` op launchers
// (3_part_parallel/Parallel_Method.cu:140-200), same names and arguments, now on
// the MI355X kernels through the C ABI.
//
// Arguments are device pointers (the reference passes cudaMallocManaged memory;
// allocate with pgmg_host::DeviceArray / pgmg_device_alloc).  Differences kept on
// purpose:
//   * ComputeJacobi is out-of-place (ping-pong) instead of the reference's racy
//     in-place kernel; it still performs v+1 sweeps and, like the
//     reference GPU op, no early exit.
//   * errors throw std::runtime_error (the reference checks nothing).
#pragma once
#include "pgmg.hpp"

class Parallel {
  public:
    // the CUDA block edge of the reference's launches (globals.cpp:6, rewritten by
    // plotTimeSequentialVsParallel, ParallelTestRunner.cu:102); ComputeProlungator's thread
    // grid depends on it (a class member here: the reference's global `num_thread` lives in
    // its globals.cpp, which a program may link beside this header)
    static inline int num_thread = 32;

    // Parallel_Method.cu:144-160: v+1 Jacobi sweeps of d_x with right-hand side d_f
    static void ComputeJacobi(double *d_x, double *d_f, int height, int weight, double h_act, int v)
    {
        pgmg_host::check(pgmg_jacobi(d_x, nullptr, d_f, height, weight, h_act, v, -1.0, nullptr,
                                     nullptr),
                         "ComputeJacobi");
        pgmg_host::check(pgmg_device_sync(), "ComputeJacobi sync");
    }

    // Parallel_Method.cu:162-173: d_r = f - A x on the interior
    static void ComputeResidual(double *d_r, double *d_x, double *d_f, int height, int width,
                                double h_act)
    {
        pgmg_host::check(pgmg_residual(d_r, d_x, d_f, height, width, h_act, nullptr),
                         "ComputeResidual");
        pgmg_host::check(pgmg_device_sync(), "ComputeResidual sync");
    }

    // Parallel_Method.cu:175-186: full-weighting restriction fine -> coarse
    static void ComputeRestriction(double *fine, double *coarse, int fine_N, int coarse_N)
    {
        pgmg_host::check(pgmg_restrict(fine, coarse, fine_N, coarse_N, nullptr),
                         "ComputeRestriction");
        pgmg_host::check(pgmg_device_sync(), "ComputeRestriction sync");
    }

    // Parallel_Method.cu:188-199: fine += P coarse, the GPU reference's symmetric
    // bilinear prolongation with the fine boundary set to 0, over the reference's thread
    // grid (max(1, fine_N / num_thread) blocks of num_thread per side: for fine_N = 2^k + 1
    // the last row and column are left as they are)
    static void ComputeProlungator(double *coarse, double *fine, int coarse_N, int fine_N)
    {
        pgmg_host::check(pgmg_prolong_grid(coarse, fine, coarse_N, fine_N, PGMG_PROLONG_SYMMETRIC,
                                           num_thread, nullptr),
                         "ComputeProlungator");
        pgmg_host::check(pgmg_device_sync(), "ComputeProlungator sync");
    }
};
