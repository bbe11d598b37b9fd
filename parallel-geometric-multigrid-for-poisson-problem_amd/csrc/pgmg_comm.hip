// pgmg_comm.hip — row-strip domain decomposition of the level pyramid over ranks.
//
// One process per GPU (BASELINE north star: "partitioned across the 8 GPUs ... halo
// exchange as RCCL point-to-point ... the coarsest levels collapsing to rank 0").
// The reference has no multi-GPU path; this is new.
//
//  * Split points s_r of the finest level are multiples of 2^Ld, so level l < Ld
//    splits at s_r >> l and the coarse row jc sits on the rank owning fine row 2jc.
//    Rank r owns rows [s_r, s_{r+1}) (rank 0 also row 0, the last rank row N-1).
//  * Every kernel is pointwise with a bounded neighbourhood, so halo rows make the
//    strip computation bit-identical to one GPU.  Halo depths (rows): k_pre reads
//    x0/f 4 rows past its strip (two sweeps + residual + restriction), k_post reads
//    phi 2 rows and the coarse correction 1-2 rows.
//  * The smoother's early-exit norm is a global sum: a local partial sum, then one
//    allreduce of a single double (all ranks take the same decision).
//  * Levels with N <= gather_n (or strips thinner than kMinRows) are "gathered" and
//    replicated: every rank sends its rows of the coarse right-hand side to every other
//    rank (one grouped exchange), then every rank runs the remaining cycle (bulk kernels
//    + LDS tail) on its full copy — identical work and results on every rank, so no
//    scatter of the correction is needed (one collective step instead of two).
//  * Transport: RCCL grouped ncclSend/ncclRecv + ncclAllReduce on the context's
//    stream (RCCL over xGMI on MI355X).  Tests use an in-process loopback
//    transport (ranks = host threads sharing one GPU; RCCL refuses two ranks per
//    device) that gives the same message semantics.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <map>
#include <mutex>
#include <thread>
#include <tuple>
#include <vector>

#include "pgmg_ctx.h"

namespace pgmg {

namespace {

constexpr int kMinRows = 16;  // thinnest strip a distributed level may have

#define NCCLC(expr)                                                                        \
    do {                                                                                   \
        ncclResult_t r_ = (expr);                                                          \
        if (r_ != ncclSuccess)                                                             \
            return set_err(PGMG_ERR_COMM, std::string(#expr) + ": " + ncclGetErrorString(r_)); \
    } while (0)

// ---------------------------------------------------------------------------
// transports
// ---------------------------------------------------------------------------
class Transport {
  public:
    // what the next group / allreduce is (StripComm sets it): named by a stall message
    std::string label;
    long long ngroups = 0;       // groups and allreduces enqueued (the stall message's index)
    virtual ~Transport() {}
    virtual int ranks(int *n) { return *n = -1, PGMG_OK; }
    virtual int group_start() = 0;
    virtual int send(const void *buf, size_t bytes, int peer, hipStream_t s) = 0;
    virtual int recv(void *buf, size_t bytes, int peer, hipStream_t s) = 0;
    virtual int group_end(hipStream_t s) = 0;
    virtual int allreduce_sum(double *d, int n, hipStream_t s) = 0;
    virtual int allreduce_min_u32(unsigned *d, int n, hipStream_t s) = 0;
    virtual int wait(hipStream_t s)
    {
        PGMG_HIPC(hipStreamSynchronize(s));
        return PGMG_OK;
    }
};

class RcclTransport : public Transport {
  public:
    ncclComm_t comm = nullptr;
    double timeout_s = 600.0;
    // one event recorded after every enqueued group / allreduce (a ring): wait() counts a
    // completed one as progress, so comm_timeout_s bounds the time WITHOUT progress, not
    // the time behind a long queue of healthy work
    static constexpr int kRing = 64;
    hipEvent_t ring[kRing] = {};
    std::string ring_label[kRing];
    long long rec = 0, done = 0;
    ~RcclTransport() override
    {
        for (hipEvent_t e : ring)
            if (e) (void)hipEventDestroy(e);
        if (comm) ncclCommDestroy(comm);
    }
    int abort_with(const std::string &why)
    {
        if (comm) ncclCommAbort(comm);
        comm = nullptr;
        return set_err(PGMG_ERR_COMM, why);
    }
    int mark(hipStream_t s)
    {
        if (!ring[0])
            for (hipEvent_t &e : ring) PGMG_HIPC(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        PGMG_HIPC(hipEventRecord(ring[rec % kRing], s));
        ring_label[rec % kRing] = "group #" + std::to_string(ngroups) + ": " + label;
        ++rec;
        if (rec - done > kRing) done = rec - kRing;   // older marks were overwritten
        return PGMG_OK;
    }
    // Poll the stream instead of blocking in hipStreamSynchronize: a peer that died or
    // stopped posting its sends would otherwise hang this rank forever.
    int wait(hipStream_t s) override
    {
        if (!comm) return set_err(PGMG_ERR_COMM, "communicator aborted by an earlier error");
        auto t0 = std::chrono::steady_clock::now();
        for (int spin = 0;; ++spin) {
            const hipError_t q = hipStreamQuery(s);
            if (q == hipSuccess) {
                done = rec;
                return PGMG_OK;
            }
            if (q != hipErrorNotReady)
                return abort_with(std::string("stream error while waiting: ") + hipGetErrorString(q));
            ncclResult_t ae = ncclSuccess;
            if (ncclCommGetAsyncError(comm, &ae) == ncclSuccess && ae != ncclSuccess &&
                ae != ncclInProgress)
                return abort_with(std::string("RCCL asynchronous error: ") + ncclGetErrorString(ae));
            bool progressed = false;
            while (done < rec && hipEventQuery(ring[done % kRing]) == hipSuccess) {
                ++done;
                progressed = true;
            }
            if (progressed) t0 = std::chrono::steady_clock::now();
            const double dt =
                std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
            if (dt > timeout_s)   // name the first group that has not completed
                return abort_with("RCCL wait: no progress for pgmg_config.comm_timeout_s (" +
                                  std::to_string(timeout_s) + " s); stalled at " +
                                  (done < rec ? ring_label[done % kRing] : std::string("the stream's tail")));
            if (spin > 64) std::this_thread::sleep_for(std::chrono::microseconds(20));
        }
    }
    int init(const void *uid, int world, int rank)
    {
        ncclUniqueId id;
        std::memcpy(&id, uid, sizeof(id));
        NCCLC(ncclCommInitRank(&comm, world, id, rank));
        return PGMG_OK;
    }
    int group_start() override
    {
        if (!comm) return set_err(PGMG_ERR_COMM, "communicator aborted by an earlier error");
        NCCLC(ncclGroupStart());
        return PGMG_OK;
    }
    int ranks(int *n) override
    {
        if (!comm) return set_err(PGMG_ERR_COMM, "communicator aborted by an earlier error");
        NCCLC(ncclCommCount(comm, n));
        return PGMG_OK;
    }
    int send(const void *buf, size_t bytes, int peer, hipStream_t s) override
    {
        NCCLC(ncclSend(buf, bytes, ncclChar, peer, comm, s));
        return PGMG_OK;
    }
    int recv(void *buf, size_t bytes, int peer, hipStream_t s) override
    {
        NCCLC(ncclRecv(buf, bytes, ncclChar, peer, comm, s));
        return PGMG_OK;
    }
    int group_end(hipStream_t s) override
    {
        NCCLC(ncclGroupEnd());
        return mark(s);
    }
    int allreduce_sum(double *d, int n, hipStream_t s) override
    {
        if (!comm) return set_err(PGMG_ERR_COMM, "communicator aborted by an earlier error");
        NCCLC(ncclAllReduce(d, d, n, ncclDouble, ncclSum, comm, s));
        return mark(s);
    }
    int allreduce_min_u32(unsigned *d, int n, hipStream_t s) override
    {
        if (!comm) return set_err(PGMG_ERR_COMM, "communicator aborted by an earlier error");
        NCCLC(ncclAllReduce(d, d, n, ncclUint32, ncclMin, comm, s));
        return mark(s);
    }
};

}  // namespace

// In-process hub for the loopback transport (test infrastructure for the strip
// decomposition on a single GPU).  Message matching by (src, dst, sequence).
struct LoopbackHub {
    int world = 0;
    std::mutex m;
    std::condition_variable cv;
    struct Msg {
        const void *src = nullptr;
        size_t bytes = 0;
        hipEvent_t ready = nullptr;  // recorded on the sender's stream
        hipEvent_t done = nullptr;   // recorded on the receiver's stream after the copy
        bool posted = false, copied = false;
    };
    std::map<std::tuple<int, int, long long>, Msg> box;
    std::map<std::pair<int, int>, long long> seq_send, seq_recv;
    // test hook (pgmg_loopback_fail): group_end of rank r fails at its fail_at[r]-th call
    // (1-based; 0 = never) with PGMG_ERR_COMM, before posting anything; every rank runs the
    // same sequence of groups, so failing all ranks at the same count hangs none of them
    long long groups[64] = {0}, fail_at[64] = {0};
    // allreduce rendezvous
    long long ar_round[64] = {0};
    std::map<long long, std::vector<double>> ar_vals;
    std::map<long long, int> ar_count, ar_taken;
};

namespace {

class LoopbackTransport : public Transport {
  public:
    LoopbackHub *hub;
    int me;
    struct Pend {
        bool is_send;
        void *buf;
        size_t bytes;
        int peer;
    };
    std::vector<Pend> pend;
    LoopbackTransport(LoopbackHub *h, int rank) : hub(h), me(rank) {}
    int group_start() override
    {
        pend.clear();
        return PGMG_OK;
    }
    int send(const void *buf, size_t bytes, int peer, hipStream_t) override
    {
        pend.push_back({true, const_cast<void *>(buf), bytes, peer});
        return PGMG_OK;
    }
    int recv(void *buf, size_t bytes, int peer, hipStream_t) override
    {
        pend.push_back({false, buf, bytes, peer});
        return PGMG_OK;
    }
    int group_end(hipStream_t s) override
    {
        {
            std::lock_guard<std::mutex> g(hub->m);
            if (++hub->groups[me] == hub->fail_at[me]) {
                pend.clear();
                return set_err(PGMG_ERR_COMM, "loopback: injected transport failure");
            }
        }
        std::vector<std::tuple<int, int, long long>> my_sends;
        // 1. post sends (data ready when the sender's stream reaches this point)
        for (auto &p : pend) {
            if (!p.is_send) continue;
            hipEvent_t ready, done;
            PGMG_HIPC(hipEventCreateWithFlags(&ready, hipEventDisableTiming));
            PGMG_HIPC(hipEventCreateWithFlags(&done, hipEventDisableTiming));
            PGMG_HIPC(hipEventRecord(ready, s));
            std::lock_guard<std::mutex> g(hub->m);
            const long long q = hub->seq_send[{me, p.peer}]++;
            auto key = std::make_tuple(me, p.peer, q);
            auto &msg = hub->box[key];
            msg.src = p.buf;
            msg.bytes = p.bytes;
            msg.ready = ready;
            msg.done = done;
            msg.posted = true;
            my_sends.push_back(key);
            hub->cv.notify_all();
        }
        // 2. receive: wait for the matching send, copy on this stream
        for (auto &p : pend) {
            if (p.is_send) continue;
            std::unique_lock<std::mutex> g(hub->m);
            const long long q = hub->seq_recv[{p.peer, me}]++;
            auto key = std::make_tuple(p.peer, me, q);
            hub->cv.wait(g, [&] { return hub->box.count(key) && hub->box[key].posted; });
            auto msg = hub->box[key];
            g.unlock();
            if (msg.bytes != p.bytes) return set_err(PGMG_ERR_COMM, "loopback size mismatch");
            PGMG_HIPC(hipStreamWaitEvent(s, msg.ready, 0));
            PGMG_HIPC(hipMemcpyAsync(p.buf, msg.src, p.bytes, hipMemcpyDeviceToDevice, s));
            PGMG_HIPC(hipEventRecord(msg.done, s));
            g.lock();
            hub->box[key].copied = true;
            hub->cv.notify_all();
        }
        // 3. the sender may not overwrite its buffer before the receiver copied it
        for (auto &key : my_sends) {
            std::unique_lock<std::mutex> g(hub->m);
            hub->cv.wait(g, [&] { return hub->box[key].copied; });
            auto msg = hub->box[key];
            hub->box.erase(key);
            g.unlock();
            PGMG_HIPC(hipStreamWaitEvent(s, msg.done, 0));
            (void)hipEventDestroy(msg.ready);
            // `done` is destroyed lazily: the wait above holds a reference
            (void)hipEventDestroy(msg.done);
        }
        pend.clear();
        return PGMG_OK;
    }
    int allreduce_min_u32(unsigned *d, int n, hipStream_t s) override
    {
        // through the double rendezvous: values 0/1 (exact in double), min = -sum(-x)...
        // simplest exact form: each rank contributes x, the minimum of 0/1 flags over the
        // world is 1 iff their sum equals the world size
        std::vector<unsigned> u(n);
        PGMG_HIPC(hipMemcpyAsync(u.data(), d, n * sizeof(unsigned), hipMemcpyDeviceToHost, s));
        PGMG_HIPC(hipStreamSynchronize(s));
        double *tmp = nullptr;
        PGMG_HIPC(hipMalloc((void **)&tmp, n * sizeof(double)));
        std::vector<double> v(u.begin(), u.end());
        for (auto &x : v) x = x ? 1.0 : 0.0;
        PGMG_HIPC(hipMemcpy(tmp, v.data(), n * sizeof(double), hipMemcpyHostToDevice));
        int e = allreduce_sum(tmp, n, s);
        if (!e) {
            PGMG_HIPC(hipMemcpy(v.data(), tmp, n * sizeof(double), hipMemcpyDeviceToHost));
            for (int i = 0; i < n; ++i) u[i] = v[i] == (double)hub->world ? 1u : 0u;
            PGMG_HIPC(hipMemcpy(d, u.data(), n * sizeof(unsigned), hipMemcpyHostToDevice));
        }
        (void)hipFree(tmp);
        return e;
    }
    int allreduce_sum(double *d, int n, hipStream_t s) override
    {
        std::vector<double> v(n);
        PGMG_HIPC(hipMemcpyAsync(v.data(), d, n * sizeof(double), hipMemcpyDeviceToHost, s));
        PGMG_HIPC(hipStreamSynchronize(s));
        std::vector<double> tot;
        {
            std::unique_lock<std::mutex> g(hub->m);
            const long long r = hub->ar_round[me]++;
            auto &vals = hub->ar_vals[r];
            if (vals.empty()) vals.assign((size_t)hub->world * n, 0.0);
            std::copy(v.begin(), v.end(), vals.begin() + (size_t)me * n);
            hub->ar_count[r]++;
            hub->cv.notify_all();
            hub->cv.wait(g, [&] { return hub->ar_count[r] == hub->world; });
            tot.assign(n, 0.0);
            for (int k = 0; k < hub->world; ++k)  // rank order: deterministic
                for (int i = 0; i < n; ++i) tot[i] += vals[(size_t)k * n + i];
            if (++hub->ar_taken[r] == hub->world) {
                hub->ar_vals.erase(r);
                hub->ar_count.erase(r);
                hub->ar_taken.erase(r);
            }
        }
        PGMG_HIPC(hipMemcpyAsync(d, tot.data(), n * sizeof(double), hipMemcpyHostToDevice, s));
        PGMG_HIPC(hipStreamSynchronize(s));
        return PGMG_OK;
    }
};

// Host-staged transport (PGMG_FLAG_HOST_TRANSPORT): the caller's functions move the
// messages (MPI, torch.distributed/gloo, ...), so ranks in separate processes can run the
// strip decomposition without RCCL — several of them on one GPU, which RCCL refuses.  Each
// group waits for the stream, copies the send buffers to host, calls exchange(), copies the
// received bytes back; the reductions likewise.  A correctness path, not a fast one.
class HostTransport : public Transport {
  public:
    const pgmg_host_transport *ht;
    struct Pend {
        bool is_send;
        void *buf;
        size_t bytes;
        int peer;
    };
    std::vector<Pend> pend;
    std::vector<std::vector<unsigned char>> stage;
    explicit HostTransport(const pgmg_host_transport *h) : ht(h) {}
    int group_start() override
    {
        pend.clear();
        return PGMG_OK;
    }
    int send(const void *buf, size_t bytes, int peer, hipStream_t) override
    {
        pend.push_back({true, const_cast<void *>(buf), bytes, peer});
        return PGMG_OK;
    }
    int recv(void *buf, size_t bytes, int peer, hipStream_t) override
    {
        pend.push_back({false, buf, bytes, peer});
        return PGMG_OK;
    }
    int group_end(hipStream_t s) override
    {
        std::vector<Pend> p;
        p.swap(pend);
        PGMG_HIPC(hipStreamSynchronize(s));   // the send buffers are final on the stream
        stage.resize(p.size());
        std::vector<int> speer, rpeer;
        std::vector<const void *> sbuf;
        std::vector<void *> rbuf;
        std::vector<unsigned long long> sbytes, rbytes;
        for (size_t i = 0; i < p.size(); ++i) {
            stage[i].resize(p[i].bytes);
            if (p[i].is_send) {
                if (p[i].bytes)
                    PGMG_HIPC(hipMemcpy(stage[i].data(), p[i].buf, p[i].bytes, hipMemcpyDeviceToHost));
                speer.push_back(p[i].peer);
                sbuf.push_back(stage[i].data());
                sbytes.push_back(p[i].bytes);
            } else {
                rpeer.push_back(p[i].peer);
                rbuf.push_back(stage[i].data());
                rbytes.push_back(p[i].bytes);
            }
        }
        if (ht->exchange(ht->user, (int)speer.size(), speer.data(), sbuf.data(), sbytes.data(),
                         (int)rpeer.size(), rpeer.data(), rbuf.data(), rbytes.data()) != 0)
            return set_err(PGMG_ERR_COMM, "host transport: exchange failed");
        for (size_t i = 0; i < p.size(); ++i)
            if (!p[i].is_send && p[i].bytes)
                PGMG_HIPC(hipMemcpy(p[i].buf, stage[i].data(), p[i].bytes, hipMemcpyHostToDevice));
        return PGMG_OK;
    }
    int allreduce_sum(double *d, int n, hipStream_t s) override
    {
        std::vector<double> v(n);
        PGMG_HIPC(hipMemcpyAsync(v.data(), d, n * sizeof(double), hipMemcpyDeviceToHost, s));
        PGMG_HIPC(hipStreamSynchronize(s));
        if (ht->allreduce_sum_f64(ht->user, v.data(), n) != 0)
            return set_err(PGMG_ERR_COMM, "host transport: allreduce_sum_f64 failed");
        PGMG_HIPC(hipMemcpy(d, v.data(), n * sizeof(double), hipMemcpyHostToDevice));
        return PGMG_OK;
    }
    int allreduce_min_u32(unsigned *d, int n, hipStream_t s) override
    {
        std::vector<unsigned> v(n);
        PGMG_HIPC(hipMemcpyAsync(v.data(), d, n * sizeof(unsigned), hipMemcpyDeviceToHost, s));
        PGMG_HIPC(hipStreamSynchronize(s));
        if (ht->allreduce_min_u32(ht->user, v.data(), n) != 0)
            return set_err(PGMG_ERR_COMM, "host transport: allreduce_min_u32 failed");
        PGMG_HIPC(hipMemcpy(d, v.data(), n * sizeof(unsigned), hipMemcpyHostToDevice));
        return PGMG_OK;
    }
};

// Null transport (PGMG_FLAG_SOLO, measurement only): no messages, allreduces return the
// local values.  One rank of a world-W decomposition runs alone on one GPU, so its
// compute time per cycle can be measured without W GPUs.
class NullTransport : public Transport {
  public:
    int group_start() override { return PGMG_OK; }
    int send(const void *, size_t, int, hipStream_t) override { return PGMG_OK; }
    int recv(void *, size_t, int, hipStream_t) override { return PGMG_OK; }
    int group_end(hipStream_t) override { return PGMG_OK; }
    int allreduce_sum(double *, int, hipStream_t) override { return PGMG_OK; }
    int allreduce_min_u32(unsigned *, int, hipStream_t) override { return PGMG_OK; }
};

// ---------------------------------------------------------------------------
// strip decomposition
// ---------------------------------------------------------------------------
class StripComm : public Comm {
  public:
    Transport *t = nullptr;
    int me = 0, world = 1;
    int Ld = 0;                  // levels 0..Ld-1 distributed; Ld = first gathered level
    std::vector<int> split;      // finest-level split points s_0 .. s_world
    // halo_begin's exchange, not yet posted: it joins the next grouped exchange of the
    // stream (or is posted alone by halo_end / before an allreduce)
    bool pending = false;
    Grid pend_g;
    Level pend_L;
    int pend_depth = 0;

    // PGMG_FLAG_TIME_COMM: events around every collective group on the stream (comm_stats)
    bool timing = false;
    std::vector<hipEvent_t> tev;   // start / end pairs
    int tused = 0;
    long long groups = 0;

    ~StripComm() override
    {
        for (hipEvent_t e : tev)
            if (e) (void)hipEventDestroy(e);
        delete t;
    }
    // every collective of the strips goes through here: labelled (a stall message names it),
    // counted and, when timing, bracketed by events
    template <class F>
    int collective(hipStream_t s, const std::string &what, F &&f)
    {
        t->label = what;
        int i0 = -1;
        if (timing) {
            if (tev.empty()) {
                tev.assign(2 * 4096, nullptr);
                for (hipEvent_t &e : tev) PGMG_HIPC(hipEventCreate(&e));
            }
            if (tused + 2 <= (int)tev.size()) {
                i0 = tused;
                PGMG_HIPC(hipEventRecord(tev[i0], s));
            }
        }
        const int e = f();
        if (i0 >= 0) {
            PGMG_HIPC(hipEventRecord(tev[i0 + 1], s));
            tused = i0 + 2;
        }
        ++groups;
        ++t->ngroups;
        return e;
    }
    int comm_stats(hipStream_t s, long long *ng, double *ms) override
    {
        const int e = t->wait(s);
        if (e) return e;
        double tot = 0.0;
        for (int i = 0; i + 1 < tused; i += 2) {
            float f = 0.f;
            PGMG_HIPC(hipEventElapsedTime(&f, tev[i], tev[i + 1]));
            tot += f;
        }
        if (ng) *ng = groups;
        if (ms) *ms = timing ? tot : -1.0;
        groups = 0;
        tused = 0;
        return PGMG_OK;
    }
    int comm_ranks(int *n) override
    {
        int r = -1;
        const int e = t->ranks(&r);
        *n = r > 0 ? r : world;
        return e;
    }
    int gathered_level() const override { return Ld; }
    int rank() const override { return me; }

    int strip_lo(int r, int l) const { return split[r] >> l; }
    int strip_hi(int r, int l, int N) const { return r == world - 1 ? N : (split[r + 1] >> l); }

    int plan(pgmg_ctx *c) override
    {
        const int N0 = c->lv[0].N;
        const int G = N0 - 1;
        const int gather_n = std::max(c->cfg.gather_n, c->lv[c->nb].N);
        // distributed levels: N_l > gather_n and every strip at least kMinRows rows
        Ld = 0;
        for (int l = 0; l < c->nb; ++l) {
            const int Nl = c->lv[l].N;
            if (Nl <= gather_n || (Nl - 1) / world < kMinRows) break;
            Ld = l + 1;
        }
        if (Ld == 0) return 1;  // too small to split: every rank runs its own replica
        const int align = 1 << Ld;
        split.assign(world + 1, 0);
        for (int r = 1; r < world; ++r)
            split[r] = (int)(((long long)r * G / world) / align * align);
        split[world] = N0;
        for (int r = 0; r < world; ++r)
            if (split[r + 1] - split[r] < kMinRows * (1 << (Ld - 1)) && r + 1 < world)
                return set_err(PGMG_ERR_ARG, "grid too small for this many ranks");
        for (int l = 0; l < (int)c->lv.size(); ++l) {
            Level &L = c->lv[l];
            if (l < Ld) {
                L.lo = strip_lo(me, l);
                L.hi = strip_hi(me, l, L.N);
                L.on_this_rank = true;
                L.gathered = false;
            } else {
                L.lo = 0;
                L.hi = L.N;
                L.gathered = true;
                L.on_this_rank = true;  // the coarse levels are replicated on every rank
            }
            L.u0 = std::max(L.lo, 1);
            L.u1 = std::min(L.hi, L.N - 1);
        }
        return PGMG_OK;
    }

    int setup(pgmg_ctx *) override { return PGMG_OK; }

    // The finest level's halo rows are final a whole coarse hierarchy before the next
    // finest pass reads them.  Instead of a second communicator on a side stream (two
    // communicators' kernels running concurrently on one device can deadlock), the exchange
    // is held back and posted INSIDE the next grouped exchange of the same stream: the
    // coarse level's right-hand-side halos, or the all-to-all of the first gathered level.
    // One RCCL group per cycle instead of two, on one communicator, in stream order.
    int halo_begin(const Grid &g, const Level &L, int depth, hipStream_t s) override
    {
        if (pending) {
            const int e = flush(s);
            if (e) return e;
        }
        pend_g = g;
        pend_L = L;
        pend_depth = depth;
        pending = true;
        return PGMG_OK;
    }

    int flush(hipStream_t s)
    {
        if (!pending) return PGMG_OK;
        pending = false;
        const HaloReq r{&pend_g, &pend_L, pend_depth};
        return halos_on(t, &r, 1, s);
    }

    int halo_end(hipStream_t s) override { return flush(s); }

    int halos(const HaloReq *reqs, int n, hipStream_t s) override
    {
        if (!pending) return halos_on(t, reqs, n, s);
        std::vector<HaloReq> all;
        all.reserve(n + 1);
        all.push_back(HaloReq{&pend_g, &pend_L, pend_depth});
        all.insert(all.end(), reqs, reqs + n);
        pending = false;
        return halos_on(t, all.data(), n + 1, s);
    }

    // one array's halo send/recv pairs inside an open group
    int post_halo(Transport *tp, const HaloReq &q, hipStream_t s)
    {
        const Grid &g = *q.g;
        const Level &L = *q.L;
        const int depth = q.depth;
        const size_t row = (size_t)L.P * L.es;
        int e = PGMG_OK;
        if (me > 0) {
            e = tp->send(row_ptr(g, L.lo, L.P, L.es), depth * row, me - 1, s);
            if (!e) e = tp->recv(row_ptr(g, L.lo - depth, L.P, L.es), depth * row, me - 1, s);
        }
        if (!e && me < world - 1) {
            e = tp->send(row_ptr(g, L.hi - depth, L.P, L.es), depth * row, me + 1, s);
            if (!e) e = tp->recv(row_ptr(g, L.hi, L.P, L.es), depth * row, me + 1, s);
        }
        return e;
    }

    int halos_on(Transport *tp, const HaloReq *reqs, int n, hipStream_t s)
    {
        std::string what = "halo exchange";
        for (int k = 0; k < n; ++k)
            what += (k ? ", " : " of ") + std::string("level N=") + std::to_string(reqs[k].L->N) +
                    " (" + std::to_string(reqs[k].depth) + " rows)";
        return collective(s, what, [&]() {
            int e = tp->group_start();
            if (e) return e;
            for (int k = 0; k < n && !e; ++k) e = post_halo(tp, reqs[k], s);
            const int e2 = tp->group_end(s);   // the group is closed even after a failed call
            return e ? e : e2;
        });
    }

    int allreduce_sum(double *d, int n, hipStream_t s) override
    {
        const int e = flush(s);
        return e ? e : collective(s, "allreduce(sum) of " + std::to_string(n) + " doubles",
                                  [&]() { return t->allreduce_sum(d, n, s); });
    }
    int wait(hipStream_t s) override
    {
        const int e = flush(s);
        return e ? e : t->wait(s);
    }
    int allreduce_min_u32(unsigned *d, int n, hipStream_t s) override
    {
        const int e = flush(s);
        return e ? e : collective(s, "allreduce(min) of " + std::to_string(n) + " u32",
                                  [&]() { return t->allreduce_min_u32(d, n, s); });
    }

    int allgather_rows(pgmg_ctx *c, int l, const Grid &g) override
    {
        return collective(c->s, "all-to-all rows of gathered level N=" + std::to_string(c->lv[l].N) +
                                    (pending ? " (+ the finest level's halo)" : ""),
                          [&]() { return allgather_rows_group(c, l, g); });
    }
    int allgather_rows_group(pgmg_ctx *c, int l, const Grid &g)
    {
        Level &L = c->lv[l];
        const size_t row = (size_t)L.P * L.es;
        int e = t->group_start();
        if (e) return e;
        if (pending) {   // the finest level's held-back halo rides in this group
            pending = false;
            e = post_halo(t, HaloReq{&pend_g, &pend_L, pend_depth}, c->s);
        }
        for (int r = 0; r < world && !e; ++r) {
            const int a = std::max(strip_lo(r, l), 1), b = std::min(strip_hi(r, l, L.N), L.N - 1);
            if (b <= a) continue;
            if (r == me) {
                for (int q = 0; q < world && !e; ++q)
                    if (q != me) e = t->send(row_ptr(g, a, L.P, L.es), (b - a) * row, q, c->s);
            } else {
                e = t->recv(row_ptr(g, a, L.P, L.es), (b - a) * row, r, c->s);
            }
        }
        const int e2 = t->group_end(c->s);   // the group is closed even after a failed call
        return e ? e : e2;
    }

    int run_gathered(pgmg_ctx *c, int l, int gamma, int repeats) override
    {
        // 1. every rank's rows of the coarse right-hand side -> every rank (one group)
        int e = allgather_rows(c, l, c->lv[l].F);
        if (e) return e;
        // 2. every rank runs the rest of the hierarchy on its full copy: identical inputs,
        //    identical (pointwise, deterministic) results, so the parent's prolongation reads
        //    the correction from its own copy and no scatter is needed
        for (int i = 0; i < repeats; ++i)
            if ((e = enqueue_cycle(c, l, gamma, i == 0))) return e;
        return PGMG_OK;
    }

    int gather_solution(pgmg_ctx *c, double *phi, int root) override
    {
        Level &L = c->lv[0];
        const int N = L.N;
        const size_t row = (size_t)L.P * L.es;
        const bool want = root < 0 || root == me;
        if (const int ef = flush(c->s)) return ef;
        Grid full;
        if (want) {
            PGMG_HIPC(hipMalloc(&full.base, (size_t)N * row));
            full.o = full.base;
            PGMG_HIPC(hipMemcpyAsync(row_ptr(full, L.lo, L.P, L.es), row_ptr(L.A, L.lo, L.P, L.es),
                                     (L.hi - L.lo) * row, hipMemcpyDeviceToDevice, c->s));
        }
        int e = t->group_start();
        for (int r = 0; r < world && !e; ++r) {
            if (r == me) continue;
            if (root < 0 || root == r)
                e = t->send(row_ptr(L.A, L.lo, L.P, L.es), (L.hi - L.lo) * row, r, c->s);
            if (!e && want) {
                const int a = strip_lo(r, 0), b = strip_hi(r, 0, N);
                e = t->recv(row_ptr(full, a, L.P, L.es), (b - a) * row, r, c->s);
            }
        }
        const int e2 = t->group_end(c->s);   // closed even after a failed send/recv
        if (!e) e = e2;
        if (!e && want) e = download_grid(c, full.o, L.P, N, phi);
        if (!e) e = t->wait(c->s);
        else (void)hipStreamSynchronize(c->s);
        if (want) (void)hipFree(full.base);
        return e;
    }
};

}  // namespace

Comm *Comm::create(pgmg_ctx *c, int *rc)
{
    *rc = PGMG_OK;
    const pgmg_config &cfg = c->cfg;
    if (cfg.flags & PGMG_FLAG_SOLO) {
        auto *sc = new StripComm();
        sc->me = cfg.rank;
        sc->world = cfg.world;
        sc->timing = (cfg.flags & PGMG_FLAG_TIME_COMM) != 0;
        sc->t = new NullTransport();
        return sc;
    }
    if (!cfg.nccl_unique_id) {
        *rc = set_err(PGMG_ERR_ARG,
                      "world > 1 needs nccl_unique_id (or a loopback hub / host transport)");
        return nullptr;
    }
    if ((cfg.flags & PGMG_FLAG_LOOPBACK) && (cfg.flags & PGMG_FLAG_HOST_TRANSPORT)) {
        *rc = set_err(PGMG_ERR_ARG, "PGMG_FLAG_LOOPBACK and PGMG_FLAG_HOST_TRANSPORT exclude each other");
        return nullptr;
    }
    auto *sc = new StripComm();
    sc->me = cfg.rank;
    sc->world = cfg.world;
    sc->timing = (cfg.flags & PGMG_FLAG_TIME_COMM) != 0;
    if (cfg.flags & PGMG_FLAG_HOST_TRANSPORT) {
        auto *ht = (const pgmg_host_transport *)cfg.nccl_unique_id;
        if (!ht->exchange || !ht->allreduce_sum_f64 || !ht->allreduce_min_u32) {
            *rc = set_err(PGMG_ERR_ARG, "pgmg_host_transport: null function");
            delete sc;
            return nullptr;
        }
        sc->t = new HostTransport(ht);
    } else if (cfg.flags & PGMG_FLAG_LOOPBACK) {
        auto *hub = (LoopbackHub *)cfg.nccl_unique_id;
        if (hub->world != cfg.world) {
            *rc = set_err(PGMG_ERR_ARG, "loopback hub world mismatch");
            delete sc;
            return nullptr;
        }
        sc->t = new LoopbackTransport(hub, cfg.rank);
    } else {
        auto *rt = new RcclTransport();
        if (cfg.comm_timeout_s > 0) rt->timeout_s = cfg.comm_timeout_s;
        sc->t = rt;
        *rc = rt->init(cfg.nccl_unique_id, cfg.world, cfg.rank);
        if (*rc) {
            delete sc;
            return nullptr;
        }
    }
    return sc;
}

}  // namespace pgmg

extern "C" {

int pgmg_comm_unique_id(void *out128)
{
    if (!out128) return pgmg::set_err(PGMG_ERR_ARG, "null buffer");
    ncclUniqueId id;
    ncclResult_t r = ncclGetUniqueId(&id);
    if (r != ncclSuccess) return pgmg::set_err(PGMG_ERR_COMM, ncclGetErrorString(r));
    std::memcpy(out128, &id, sizeof(id) < 128 ? sizeof(id) : 128);
    return PGMG_OK;
}

// Self-test of the RCCL transport on one GPU: a world-1 communicator (the only size a
// one-GPU box can form) runs the exact calls of the strip path — a grouped send/recv
// (to itself), allreduce(sum) of doubles and allreduce(min) of u32 — on a stream, and
// checks the results.  0 on success.
int pgmg_rccl_selftest(const void *uid128, int device)
{
    if (!uid128) return pgmg::set_err(PGMG_ERR_ARG, "null unique id");
    if (hipSetDevice(device) != hipSuccess) return pgmg::set_err(PGMG_ERR_HIP, "hipSetDevice");
    pgmg::RcclTransport t;
    int e = t.init(uid128, 1, 0);
    if (e) return e;
    hipStream_t s;
    if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess)
        return pgmg::set_err(PGMG_ERR_HIP, "stream");
    const int n = 1 << 16;
    double *a = nullptr, *b = nullptr;
    unsigned *u = nullptr;
    std::vector<double> h(n), g(n);
    for (int i = 0; i < n; ++i) h[i] = 0.5 * i - 7.0;
    int rc = PGMG_OK;
    if (hipMalloc(&a, n * sizeof(double)) != hipSuccess || hipMalloc(&b, n * sizeof(double)) != hipSuccess ||
        hipMalloc(&u, 4 * sizeof(unsigned)) != hipSuccess)
        rc = pgmg::set_err(PGMG_ERR_NOMEM, "selftest buffers");
    const unsigned hu[4] = {3u, 1u, 4u, 1u};
    unsigned gu[4] = {0, 0, 0, 0};
    if (!rc && (hipMemcpy(a, h.data(), n * sizeof(double), hipMemcpyHostToDevice) != hipSuccess ||
                hipMemset(b, 0, n * sizeof(double)) != hipSuccess ||
                hipMemcpy(u, hu, sizeof(hu), hipMemcpyHostToDevice) != hipSuccess))
        rc = pgmg::set_err(PGMG_ERR_HIP, "selftest upload");
    // the merged pattern of the strips: one group carrying two messages to the same peer
    // (the finest level's held-back halo, then a coarse level's rows), matched in order
    double *c2 = nullptr;
    if (!rc && hipMalloc(&c2, n * sizeof(double)) != hipSuccess)
        rc = pgmg::set_err(PGMG_ERR_HIP, "selftest second buffer");
    if (!rc) rc = t.group_start();
    if (!rc) rc = t.send(a, n * sizeof(double), 0, s);
    if (!rc) rc = t.recv(b, n * sizeof(double), 0, s);
    if (!rc) rc = t.send(a, (n / 2) * sizeof(double), 0, s);
    if (!rc) rc = t.recv(c2, (n / 2) * sizeof(double), 0, s);
    if (!rc) rc = t.group_end(s);
    if (!rc) rc = t.allreduce_sum(a, 3, s);
    if (!rc) rc = t.allreduce_min_u32(u, 4, s);
    if (!rc) rc = t.wait(s);   // polls the stream, the async error state and the progress marks
    if (!rc && hipStreamSynchronize(s) != hipSuccess) rc = pgmg::set_err(PGMG_ERR_HIP, "selftest sync");
    if (!rc && (hipMemcpy(g.data(), c2, (n / 2) * sizeof(double), hipMemcpyDeviceToHost) != hipSuccess ||
                std::memcmp(g.data(), h.data(), (n / 2) * sizeof(double)) != 0))
        rc = pgmg::set_err(PGMG_ERR_COMM, "selftest: the second message of the group differs");
    if (!rc && (hipMemcpy(g.data(), b, n * sizeof(double), hipMemcpyDeviceToHost) != hipSuccess ||
                hipMemcpy(gu, u, sizeof(gu), hipMemcpyDeviceToHost) != hipSuccess))
        rc = pgmg::set_err(PGMG_ERR_HIP, "selftest download");
    if (!rc && std::memcmp(g.data(), h.data(), n * sizeof(double)) != 0)
        rc = pgmg::set_err(PGMG_ERR_COMM, "selftest: received rows differ from the sent rows");
    if (!rc && std::memcmp(gu, hu, sizeof(hu)) != 0)
        rc = pgmg::set_err(PGMG_ERR_COMM, "selftest: allreduce(min) of one rank changed values");
    if (!rc) {
        double a3[3];
        if (hipMemcpy(a3, a, sizeof(a3), hipMemcpyDeviceToHost) != hipSuccess || a3[0] != h[0] ||
            a3[1] != h[1] || a3[2] != h[2])
            rc = pgmg::set_err(PGMG_ERR_COMM, "selftest: allreduce(sum) of one rank changed values");
    }
    (void)hipFree(a);
    (void)hipFree(b);
    (void)hipFree(u);
    if (c2) (void)hipFree(c2);
    (void)hipStreamDestroy(s);
    return rc;
}

// Latency floor of the strips' collectives (world-1 communicator on this device): the three
// kinds of group a V-cycle on row strips enqueues, each timed over `reps` calls with events
int pgmg_rccl_latency(const void *uid128, int device, int reps, double *us3)
{
    if (!uid128 || !us3 || reps < 1) return pgmg::set_err(PGMG_ERR_ARG, "bad argument");
    if (hipSetDevice(device) != hipSuccess) return pgmg::set_err(PGMG_ERR_HIP, "hipSetDevice");
    pgmg::RcclTransport t;
    int rc = t.init(uid128, 1, 0);
    if (rc) return rc;
    hipStream_t s = nullptr;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreate(&e0) != hipSuccess || hipEventCreate(&e1) != hipSuccess)
        return pgmg::set_err(PGMG_ERR_HIP, "latency: stream / events");
    const size_t halo = 2 * 16385 * sizeof(double);
    char *a = nullptr, *b = nullptr;
    if (hipMalloc(&a, halo) != hipSuccess || hipMalloc(&b, halo) != hipSuccess)
        rc = pgmg::set_err(PGMG_ERR_NOMEM, "latency buffers");
    if (!rc && (hipMemset(a, 0, halo) != hipSuccess || hipMemset(b, 0, halo) != hipSuccess))
        rc = pgmg::set_err(PGMG_ERR_HIP, "latency: memset");
    for (int kind = 0; kind < 3 && !rc; ++kind) {
        auto one = [&]() -> int {
            if (kind == 0) {
                int e = t.group_start();
                if (!e) e = t.send(a, halo, 0, s);
                if (!e) e = t.recv(b, halo, 0, s);
                const int e2 = t.group_end(s);
                return e ? e : e2;
            }
            if (kind == 1) return t.allreduce_sum(reinterpret_cast<double *>(a), 3, s);
            return t.allreduce_min_u32(reinterpret_cast<unsigned *>(b), 9, s);
        };
        for (int i = 0; i < 3 && !rc; ++i) rc = one();
        if (!rc) rc = t.wait(s);
        if (!rc && hipEventRecord(e0, s) != hipSuccess) rc = pgmg::set_err(PGMG_ERR_HIP, "event");
        for (int i = 0; i < reps && !rc; ++i) rc = one();
        if (!rc && hipEventRecord(e1, s) != hipSuccess) rc = pgmg::set_err(PGMG_ERR_HIP, "event");
        if (!rc) rc = t.wait(s);
        float ms = 0.f;
        if (!rc && hipEventElapsedTime(&ms, e0, e1) != hipSuccess) rc = pgmg::set_err(PGMG_ERR_HIP, "elapsed");
        if (!rc) us3[kind] = 1e3 * ms / reps;
    }
    if (a) (void)hipFree(a);
    if (b) (void)hipFree(b);
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    (void)hipStreamDestroy(s);
    return rc;
}

int pgmg_loopback_create(int world, void **hub)
{
    if (!hub || world < 1 || world > 64) return pgmg::set_err(PGMG_ERR_ARG, "bad argument");
    auto *h = new pgmg::LoopbackHub();
    h->world = world;
    *hub = h;
    return PGMG_OK;
}

int pgmg_loopback_fail(void *hub, int rank, long long at_group)
{
    auto *h = (pgmg::LoopbackHub *)hub;
    if (!h || rank < 0 || rank >= h->world) return pgmg::set_err(PGMG_ERR_ARG, "bad argument");
    std::lock_guard<std::mutex> g(h->m);
    h->fail_at[rank] = at_group > 0 ? h->groups[rank] + at_group : 0;
    return PGMG_OK;
}

int pgmg_loopback_destroy(void *hub)
{
    delete (pgmg::LoopbackHub *)hub;
    return PGMG_OK;
}

// Host-only: the finest-level row strip [lo, hi) of `rank` and the number of
// strip-distributed levels for an N-point grid over `world` ranks (0 levels: too
// small, every rank runs a replica).  Pure arithmetic, no GPU needed.
int pgmg_plan_strips(int N, int world, int rank, int tail_n, int gather_n, int *lo, int *hi,
                     int *dist_levels)
{
    if (world < 1 || rank < 0 || rank >= world || N < 5)
        return pgmg::set_err(PGMG_ERR_ARG, "bad argument");
    std::vector<int> Ns;
    for (int n = N;; n = (n - 1) / 2 + 1) {
        Ns.push_back(n);
        if (n <= tail_n || n <= 5) break;
    }
    const int nb = (int)Ns.size() - 1;
    const int gn = std::max(gather_n, Ns[nb]);
    int Ld = 0;
    if (world > 1)
        for (int l = 0; l < nb; ++l) {
            if (Ns[l] <= gn || (Ns[l] - 1) / world < pgmg::kMinRows) break;
            Ld = l + 1;
        }
    if (Ld == 0) {
        *lo = 0;
        *hi = N;
        *dist_levels = 0;
        return PGMG_OK;
    }
    const int align = 1 << Ld, G = N - 1;
    auto sp = [&](int r) {
        return r == 0 ? 0 : (r == world ? N : (int)(((long long)r * G / world) / align * align));
    };
    *lo = sp(rank);
    *hi = sp(rank + 1);
    *dist_levels = Ld;
    return PGMG_OK;
}

}  // extern "C"
