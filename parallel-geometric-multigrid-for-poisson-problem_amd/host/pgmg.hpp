// pgmg.hpp — thin C++17 helpers over the C ABI (include/pgmg.h).
// The reference-named classes (Parallel_Method.hpp, Parallel_Mg.hpp,
// ParallelTestRunner.hpp) are built on these; nothing here includes HIP headers.
#pragma once
#include <stdexcept>
#include <string>

#include "pgmg.h"

namespace pgmg_host {

inline void check(int rc, const char *what)
{
    if (rc != PGMG_OK)
        throw std::runtime_error(std::string(what) + " failed (" + std::to_string(rc) +
                                 "): " + pgmg_last_error());
}

// RAII device buffer of doubles (reference: cudaMallocManaged buffers)
class DeviceArray {
  public:
    DeviceArray() = default;
    explicit DeviceArray(size_t n) : n_(n)
    {
        void *p = nullptr;
        check(pgmg_device_alloc(&p, n * sizeof(double)), "pgmg_device_alloc");
        p_ = static_cast<double *>(p);
    }
    ~DeviceArray()
    {
        if (p_) pgmg_device_free(p_);
    }
    DeviceArray(const DeviceArray &) = delete;
    DeviceArray &operator=(const DeviceArray &) = delete;
    DeviceArray(DeviceArray &&o) noexcept : p_(o.p_), n_(o.n_) { o.p_ = nullptr; }
    double *get() const { return p_; }
    size_t size() const { return n_; }
    void upload(const double *h) { check(pgmg_memcpy_h2d(p_, h, n_ * sizeof(double)), "h2d"); }
    void download(double *h) const { check(pgmg_memcpy_d2h(h, p_, n_ * sizeof(double)), "d2h"); }

  private:
    double *p_ = nullptr;
    size_t n_ = 0;
};

// RAII N x N device grid in the reference layout (pitch N) with guard rows
// (pgmg_alloc_grid): the stand-in for the reference's cudaMallocManaged phi and f
// (ParallelTestRunner.cu:162-163).  The library's finest-level passes read and write such a
// phi in place (pgmg_set_problem_device); the host reaches it through upload / download.
class DeviceGrid {
  public:
    explicit DeviceGrid(int N) : N_(N)
    {
        check(pgmg_alloc_grid(&p_, N), "pgmg_alloc_grid");
    }
    ~DeviceGrid()
    {
        if (p_) pgmg_free_grid(p_);
    }
    DeviceGrid(const DeviceGrid &) = delete;
    DeviceGrid &operator=(const DeviceGrid &) = delete;
    double *get() const { return p_; }
    size_t size() const { return (size_t)N_ * N_; }
    void upload(const double *h) { check(pgmg_memcpy_h2d(p_, h, size() * sizeof(double)), "h2d"); }
    void download(double *h) const { check(pgmg_memcpy_d2h(h, p_, size() * sizeof(double)), "d2h"); }

  private:
    double *p_ = nullptr;
    int N_ = 0;
};

inline bool is_device_pointer(const void *p)
{
    int d = 0;
    check(pgmg_pointer_is_device(p, &d), "pgmg_pointer_is_device");
    return d != 0;
}

// RAII multigrid context
class Context {
  public:
    // h <= 0: the context's own a / (N - 1)
    Context(int N, int alpha, double eps, double h = 0.0)
    {
        pgmg_config cfg;
        check(pgmg_config_default(&cfg, N), "pgmg_config_default");
        cfg.alpha = alpha;
        cfg.eps = eps;
        if (h > 0.0) cfg.h0 = h;
        check(pgmg_create(&c_, &cfg), "pgmg_create");
    }
    ~Context()
    {
        if (c_) pgmg_destroy(c_);
    }
    Context(const Context &) = delete;
    Context &operator=(const Context &) = delete;
    pgmg_ctx *get() const { return c_; }

  private:
    pgmg_ctx *c_ = nullptr;
};

}  // namespace pgmg_host
