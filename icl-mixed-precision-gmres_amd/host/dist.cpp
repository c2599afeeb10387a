// Row-partitioned multi-GPU support (include/mpgmres/dist.h): halo plan,
// RCCL communicator, single-device loopback communicator (P ranks as
// threads, for tests), and the distributed engine entry points.
#include "mpgmres/dist.h"

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <cstdio>
#include <cstring>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "fused_gmres.hpp"
#include "gmres.hpp"
#include "types_hip.hpp"

// Local numbering of one rank's vector (x, w): its own rows at [0, n_local),
// the halo rows owned by LOWER ranks in front of them at [-n_front, 0), the
// rest after them at [n_local, n_ext). A banded matrix's first rows then
// read columns -5..-1 rather than ~n_local, so every slice of the block stays
// within the int16 SELL form and the LDS window.
struct mpg_halo {
    int rank = 0, nranks = 1;
    std::vector<int64_t> row_starts;
    int n_local = 0;
    int n_front = 0;                              // halo rows of lower ranks
    std::vector<int32_t> col_local;
    std::vector<int64_t> halo_global;             // sorted external columns
    std::vector<int32_t> recv_off, recv_cnt;      // per peer, into halo_global
    std::vector<int32_t> recv_pos;                // per peer, local id of its first row
    std::vector<std::vector<int32_t>> send_local; // per peer, local rows to send
    std::vector<bool> send_set;
};

namespace mpg {
namespace {

void nck(ncclResult_t r, const char* what) {
    if (r != ncclSuccess) throw std::runtime_error(std::string("RCCL ") + what + ": " + ncclGetErrorString(r));
}
void hck(hipError_t e, const char* what) {
    if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

// ---------------------------------------------------------------- RCCL
class RcclComm : public Comm {
    std::mutex mu_;  // guards comm_ between the owner's abort and its status queries
    ncclComm_t comm_ = nullptr;
    // a peer rank failed (request_abort, any thread): the owner's bounded wait
    // sees it through async_error() and aborts the communicator on its own
    // thread -- never freed under the owner's enqueues
    std::atomic<bool> abort_req_{false};
    int rank_, size_;
    mpg_ctx_t ctx_;
    std::vector<int32_t> recv_pos_, recv_cnt_;
    std::vector<std::unique_ptr<DevMem>> send_idx_, send_buf_;
    std::vector<int32_t> send_cnt_;
    std::vector<int32_t> send_first_;  // >= 0: the rows sent to q are [first, first + cnt) (sent in place, no pack)

public:
    // one rank per process: the communicator from a broadcast unique id
    RcclComm(mpg_ctx_t ctx, const mpg_halo& h, const char* id, int nranks, int rank)
        : rank_(rank), size_(nranks), ctx_(ctx), recv_pos_(h.recv_pos), recv_cnt_(h.recv_cnt) {
        ncclUniqueId uid;
        std::memcpy(&uid, id, sizeof uid);
        nck(ncclCommInitRank(&comm_, nranks, uid, rank), "ncclCommInitRank");
        plan(h, nranks);
    }
    // one rank per host thread of one process: a communicator of an
    // ncclCommInitAll clique, owned from here on
    RcclComm(mpg_ctx_t ctx, const mpg_halo& h, ncclComm_t comm, int nranks, int rank)
        : comm_(comm), rank_(rank), size_(nranks), ctx_(ctx), recv_pos_(h.recv_pos), recv_cnt_(h.recv_cnt) {
        try {
            plan(h, nranks);
        } catch (...) {
            ncclCommDestroy(comm_);
            throw;
        }
    }

private:
    void plan(const mpg_halo& h, int nranks) {
        send_cnt_.assign(nranks, 0);
        send_first_.assign(nranks, -1);
        send_idx_.resize(nranks);
        send_buf_.resize(nranks);
        for (int q = 0; q < nranks; ++q) {
            const auto& rows = h.send_local[q];
            send_cnt_[q] = (int32_t)rows.size();
            if (rows.empty()) continue;
            bool contiguous = true;  // banded matrices: a run at either end of the block
            for (size_t i = 1; i < rows.size() && contiguous; ++i) contiguous = rows[i] == rows[i - 1] + 1;
            if (contiguous) {
                send_first_[q] = rows[0];
                continue;
            }
            send_idx_[q] = std::make_unique<DevMem>(ctx_, rows.size() * 4);
            check(mpg_memcpy_h2d(ctx_, send_idx_[q]->p, rows.data(), rows.size() * 4), "h2d", ctx_);
            send_buf_[q] = std::make_unique<DevMem>(ctx_, rows.size() * 8);
        }
    }

public:
    ~RcclComm() override {
        if (comm_) ncclCommDestroy(comm_);
    }
    int size() const override { return size_; }
    int rank() const override { return rank_; }
    bool capturable() const override { return true; }
    bool async() const override { return true; }
    std::string async_error() override {
        if (abort_req_.load()) return "another rank failed (abort requested)";
        std::lock_guard<std::mutex> lk(mu_);
        if (!comm_) return "communicator aborted";
        ncclResult_t r = ncclSuccess;
        if (ncclCommGetAsyncError(comm_, &r) != ncclSuccess) return "ncclCommGetAsyncError failed";
        return r == ncclSuccess || r == ncclInProgress ? std::string() : std::string(ncclGetErrorString(r));
    }
    // idempotent; the owning rank's thread only (its wait_event)
    void abort() override {
        std::lock_guard<std::mutex> lk(mu_);
        if (comm_) ncclCommAbort(comm_);
        comm_ = nullptr;
    }
    void request_abort() override { abort_req_.store(true); }
    int transport_ranks() override {
        std::lock_guard<std::mutex> lk(mu_);
        int n = -1;
        if (!comm_ || ncclCommCount(comm_, &n) != ncclSuccess) return -1;
        return n;
    }
    void allreduce_sum(double* dev, int count, hipStream_t s) override {
        nck(ncclAllReduce(dev, dev, (size_t)count, ncclFloat64, ncclSum, comm_, s), "allreduce");
    }
    void allreduce_max(double* dev, int count, hipStream_t s) override {
        nck(ncclAllReduce(dev, dev, (size_t)count, ncclFloat64, ncclMax, comm_, s), "allreduce max");
    }
    void halo(void* vec, int eb, hipStream_t s) override { exchange(nullptr, 0, vec, eb, s); }
    void allreduce_sum_and_halo(double* dev, int count, void* vec, int eb, hipStream_t s) override {
        exchange(dev, count, vec, eb, s);
    }

private:
    // halo send/recv (rows that are not one contiguous run are packed
    // first), with the optional all-reduce in the same RCCL group
    void exchange(double* dev, int count, void* vec, int eb, hipStream_t s) {
        for (int q = 0; q < size_; ++q) {
            if (!send_cnt_[q] || send_first_[q] >= 0) continue;
            const int st = eb == 8 ? mpg_gather_b64(ctx_, send_cnt_[q], send_idx_[q]->as<int32_t>(), vec, send_buf_[q]->p)
                                   : mpg_gather_b32(ctx_, send_cnt_[q], send_idx_[q]->as<int32_t>(), vec, send_buf_[q]->p);
            check(st, "halo pack", ctx_);
        }
        nck(ncclGroupStart(), "group start");
        if (dev) nck(ncclAllReduce(dev, dev, (size_t)count, ncclFloat64, ncclSum, comm_, s), "allreduce");
        for (int q = 0; q < size_; ++q) {
            if (send_cnt_[q]) {
                const void* src = send_first_[q] >= 0 ? static_cast<const char*>(vec) + (size_t)send_first_[q] * eb
                                                      : send_buf_[q]->p;
                nck(ncclSend(src, (size_t)send_cnt_[q] * eb, ncclUint8, q, comm_, s), "send");
            }
            if (recv_cnt_[q]) {
                char* dst = static_cast<char*>(vec) + (ptrdiff_t)recv_pos_[q] * eb;
                nck(ncclRecv(dst, (size_t)recv_cnt_[q] * eb, ncclUint8, q, comm_, s), "recv");
            }
        }
        nck(ncclGroupEnd(), "group end");
    }
};

// ---------------------------------------------------------------- loopback
struct Hub {
    int P;
    std::mutex mu;
    std::condition_variable cv;
    int arrived = 0;
    int64_t generation = 0;
    bool aborted = false;
    std::vector<void*> ptrs;
    std::vector<std::vector<double>> staging;
    explicit Hub(int p) : P(p), ptrs(p), staging(p) {}
    void barrier() {
        std::unique_lock<std::mutex> lk(mu);
        if (aborted) throw std::runtime_error("loopback: another rank failed");
        const int64_t gen = generation;
        if (++arrived == P) {
            arrived = 0;
            ++generation;
            cv.notify_all();
        } else {
            cv.wait(lk, [&] { return generation != gen || aborted; });
            if (aborted) throw std::runtime_error("loopback: another rank failed");
        }
    }
    void abort() {
        std::lock_guard<std::mutex> lk(mu);
        aborted = true;
        cv.notify_all();
    }
};

class LoopbackComm : public Comm {
    Hub& hub_;
    int rank_;
    mpg_ctx_t ctx_;
    std::vector<int32_t> recv_off_, recv_pos_, recv_cnt_;
    std::vector<std::unique_ptr<DevMem>> src_idx_;  // per peer: indices in the peer's numbering

public:
    LoopbackComm(Hub& hub, mpg_ctx_t ctx, const mpg_halo& h)
        : hub_(hub), rank_(h.rank), ctx_(ctx), recv_off_(h.recv_off), recv_pos_(h.recv_pos),
          recv_cnt_(h.recv_cnt) {
        src_idx_.resize(h.nranks);
        for (int q = 0; q < h.nranks; ++q) {
            if (!recv_cnt_[q]) continue;
            std::vector<int32_t> idx(recv_cnt_[q]);
            for (int i = 0; i < recv_cnt_[q]; ++i)
                idx[i] = (int32_t)(h.halo_global[recv_off_[q] + i] - h.row_starts[q]);
            src_idx_[q] = std::make_unique<DevMem>(ctx, idx.size() * 4);
            check(mpg_memcpy_h2d(ctx, src_idx_[q]->p, idx.data(), idx.size() * 4), "h2d", ctx);
        }
    }
    int size() const override { return hub_.P; }
    int rank() const override { return rank_; }
    bool capturable() const override { return false; }
    void allreduce_sum(double* dev, int count, hipStream_t s) override { reduce(dev, count, s, false); }
    void allreduce_max(double* dev, int count, hipStream_t s) override { reduce(dev, count, s, true); }
    void halo(void* vec, int eb, hipStream_t s) override {
        hck(hipStreamSynchronize(s), "sync");
        hub_.ptrs[rank_] = vec;
        hub_.barrier();
        for (int q = 0; q < hub_.P; ++q) {
            if (!recv_cnt_[q]) continue;
            char* dst = static_cast<char*>(vec) + (ptrdiff_t)recv_pos_[q] * eb;
            const int st = eb == 8 ? mpg_gather_b64(ctx_, recv_cnt_[q], src_idx_[q]->as<int32_t>(), hub_.ptrs[q], dst)
                                   : mpg_gather_b32(ctx_, recv_cnt_[q], src_idx_[q]->as<int32_t>(), hub_.ptrs[q], dst);
            check(st, "loopback halo", ctx_);
        }
        hck(hipStreamSynchronize(s), "sync");
        hub_.barrier();
    }

private:
    void reduce(double* dev, int count, hipStream_t s, bool max) {
        auto& mine = hub_.staging[rank_];
        mine.resize((size_t)count);
        hck(hipMemcpyAsync(mine.data(), dev, (size_t)count * 8, hipMemcpyDeviceToHost, s), "d2h");
        hck(hipStreamSynchronize(s), "sync");
        hub_.barrier();
        std::vector<double> out(hub_.staging[0]);
        for (int q = 1; q < hub_.P; ++q)  // rank order: identical on every rank
            for (int c = 0; c < count; ++c)
                out[(size_t)c] = max ? std::max(out[(size_t)c], hub_.staging[q][(size_t)c])
                                     : out[(size_t)c] + hub_.staging[q][(size_t)c];
        hub_.barrier();
        hck(hipMemcpyAsync(dev, out.data(), (size_t)count * 8, hipMemcpyHostToDevice, s), "h2d");
        hck(hipStreamSynchronize(s), "sync");
    }
};

// ---------------------------------------------------------------- host transport
// Collectives through caller-supplied host callbacks (mpg_host_transport,
// dist.h): staging copies through host memory around each call. Lets any
// host transport (e.g. torch.distributed over gloo) drive ranks that share a
// GPU, which RCCL refuses, so the row-partitioned engine runs as separate
// processes on one device. Not capturable (host waits).
class HostComm : public Comm {
    mpg_host_transport t_;
    int rank_, size_;
    mpg_ctx_t ctx_;
    std::vector<int32_t> recv_pos_, recv_cnt_, send_cnt_;
    std::vector<std::unique_ptr<DevMem>> send_idx_, send_dev_;
    std::vector<std::vector<char>> send_host_, recv_host_;
    std::vector<double> red_;

    void call(int st, const char* what) {
        if (st != 0) throw std::runtime_error(std::string("host transport: ") + what + " failed (" + std::to_string(st) + ")");
    }

public:
    HostComm(mpg_ctx_t ctx, const mpg_halo& h, const mpg_host_transport& t, int nranks, int rank)
        : t_(t), rank_(rank), size_(nranks), ctx_(ctx), recv_pos_(h.recv_pos),
          recv_cnt_(h.recv_cnt) {
        send_cnt_.assign(nranks, 0);
        send_idx_.resize(nranks);
        send_dev_.resize(nranks);
        send_host_.resize(nranks);
        recv_host_.resize(nranks);
        for (int q = 0; q < nranks; ++q) {
            const auto& rows = h.send_local[q];
            send_cnt_[q] = (int32_t)rows.size();
            if (rows.empty()) continue;
            send_idx_[q] = std::make_unique<DevMem>(ctx, rows.size() * 4);
            check(mpg_memcpy_h2d(ctx, send_idx_[q]->p, rows.data(), rows.size() * 4), "h2d", ctx);
            send_dev_[q] = std::make_unique<DevMem>(ctx, rows.size() * 8);
        }
    }
    int size() const override { return size_; }
    int rank() const override { return rank_; }
    bool capturable() const override { return false; }
    void allreduce_sum(double* dev, int count, hipStream_t s) override { reduce(dev, count, s, 0); }
    void allreduce_max(double* dev, int count, hipStream_t s) override { reduce(dev, count, s, 1); }
    void halo(void* vec, int eb, hipStream_t s) override {
        std::vector<void*> send(size_, nullptr), recv(size_, nullptr);
        std::vector<int64_t> sb(size_, 0), rb(size_, 0);
        for (int q = 0; q < size_; ++q) {
            if (send_cnt_[q]) {
                const int st = eb == 8 ? mpg_gather_b64(ctx_, send_cnt_[q], send_idx_[q]->as<int32_t>(), vec, send_dev_[q]->p)
                                       : mpg_gather_b32(ctx_, send_cnt_[q], send_idx_[q]->as<int32_t>(), vec, send_dev_[q]->p);
                check(st, "halo pack", ctx_);
                sb[q] = (int64_t)send_cnt_[q] * eb;
                send_host_[q].resize((size_t)sb[q]);
                send[q] = send_host_[q].data();
            }
            if (recv_cnt_[q]) {
                rb[q] = (int64_t)recv_cnt_[q] * eb;
                recv_host_[q].resize((size_t)rb[q]);
                recv[q] = recv_host_[q].data();
            }
        }
        for (int q = 0; q < size_; ++q)
            if (sb[q]) hck(hipMemcpyAsync(send[q], send_dev_[q]->p, (size_t)sb[q], hipMemcpyDeviceToHost, s), "d2h");
        hck(hipStreamSynchronize(s), "sync");
        call(t_.exchange(t_.user, send.data(), sb.data(), recv.data(), rb.data()), "exchange");
        for (int q = 0; q < size_; ++q)
            if (rb[q]) {
                char* dst = static_cast<char*>(vec) + (ptrdiff_t)recv_pos_[q] * eb;
                hck(hipMemcpyAsync(dst, recv[q], (size_t)rb[q], hipMemcpyHostToDevice, s), "h2d");
            }
        hck(hipStreamSynchronize(s), "sync");
    }

private:
    void reduce(double* dev, int count, hipStream_t s, int op) {
        red_.resize((size_t)count);
        hck(hipMemcpyAsync(red_.data(), dev, (size_t)count * 8, hipMemcpyDeviceToHost, s), "d2h");
        hck(hipStreamSynchronize(s), "sync");
        call(t_.allreduce(t_.user, red_.data(), count, op), "allreduce");
        hck(hipMemcpyAsync(dev, red_.data(), (size_t)count * 8, hipMemcpyHostToDevice, s), "h2d");
        hck(hipStreamSynchronize(s), "sync");
    }
};

// rank starts at about equal nnz, rounded down to multiples of `align`
// (the node size, mpg_csr_node_dof)
std::vector<int64_t> nnz_balanced_starts(int n, const int32_t* rowptr, int P, int align = 1) {
    std::vector<int64_t> st((size_t)P + 1, 0);
    const int64_t nnz = rowptr[n];
    int r = 0;
    for (int q = 1; q < P; ++q) {
        const int64_t target = nnz * q / P;
        while (r < n && rowptr[r] < target) ++r;
        st[(size_t)q] = std::max<int64_t>(r / align * align, st[(size_t)q - 1]);
    }
    st[(size_t)P] = n;
    return st;
}

}  // namespace
}  // namespace mpg

using namespace mpg;

extern "C" {

int32_t mpg_csr_node_dof(int32_t n, const int32_t* rowptr, const int32_t* col) {
    if (n <= 0 || n % 3 || !rowptr || !col) return 1;
    for (int32_t r = 0; r < n; r += 3) {
        const int32_t p0 = rowptr[r], p1 = rowptr[r + 1], p2 = rowptr[r + 2], p3 = rowptr[r + 3];
        const int32_t len = p1 - p0;
        if (p2 - p1 != len || p3 - p2 != len || len % 3) return 1;
        for (int32_t t = 0; t < len; t += 3) {
            const int32_t c = col[p0 + t];
            for (int32_t j = 0; j < 3; ++j)
                if (col[p0 + t + j] != c + j || col[p1 + t + j] != c + j || col[p2 + t + j] != c + j) return 1;
        }
    }
    return 3;
}

int mpg_halo_analyze(int32_t rank, int32_t nranks, const int64_t* row_starts, int32_t n_local, const int32_t* rowptr,
                     const int32_t* col_global, mpg_halo_t* out) {
    if (!out || nranks < 1 || rank < 0 || rank >= nranks || !row_starts || !rowptr || n_local < 0) return MPG_ERR_ARG;
    auto* h = new mpg_halo();
    h->rank = rank;
    h->nranks = nranks;
    h->row_starts.assign(row_starts, row_starts + nranks + 1);
    h->n_local = n_local;
    const int64_t r0 = row_starts[rank], r1 = row_starts[rank + 1];
    if (r1 - r0 != n_local) {
        delete h;
        return MPG_ERR_ARG;
    }
    const int64_t nnz = rowptr[n_local];
    for (int64_t k = 0; k < nnz; ++k) {
        const int64_t c = col_global[k];
        if (c < r0 || c >= r1) h->halo_global.push_back(c);
    }
    std::sort(h->halo_global.begin(), h->halo_global.end());
    h->halo_global.erase(std::unique(h->halo_global.begin(), h->halo_global.end()), h->halo_global.end());
    h->n_front = (int)(std::lower_bound(h->halo_global.begin(), h->halo_global.end(), r0) - h->halo_global.begin());
    // local id of the t-th halo row: the lower ones in front of row 0
    auto local_of = [&](int64_t t) {
        return t < h->n_front ? (int32_t)(t - h->n_front) : (int32_t)(n_local + (t - h->n_front));
    };
    h->col_local.resize((size_t)nnz);
    for (int64_t k = 0; k < nnz; ++k) {
        const int64_t c = col_global[k];
        if (c >= r0 && c < r1) {
            h->col_local[(size_t)k] = (int32_t)(c - r0);
        } else {
            const auto it = std::lower_bound(h->halo_global.begin(), h->halo_global.end(), c);
            h->col_local[(size_t)k] = local_of(it - h->halo_global.begin());
        }
    }
    h->recv_off.assign(nranks, 0);
    h->recv_cnt.assign(nranks, 0);
    h->recv_pos.assign(nranks, 0);
    size_t pos = 0;
    for (int q = 0; q < nranks; ++q) {
        h->recv_off[q] = (int32_t)pos;
        while (pos < h->halo_global.size() && h->halo_global[pos] < row_starts[q + 1]) ++pos;
        h->recv_cnt[q] = (int32_t)(pos - h->recv_off[q]);
        h->recv_pos[q] = local_of(h->recv_off[q]);
    }
    h->send_local.assign(nranks, {});
    h->send_set.assign(nranks, false);
    h->send_set[rank] = true;
    *out = h;
    return MPG_OK;
}

int32_t mpg_halo_n_ext(mpg_halo_t h) {
    return h ? h->n_local + (int32_t)h->halo_global.size() - h->n_front : -1;
}
int32_t mpg_halo_n_front(mpg_halo_t h) { return h ? h->n_front : -1; }
int32_t mpg_halo_recv_pos(mpg_halo_t h, int32_t q) {
    return h && q >= 0 && q < h->nranks ? h->recv_pos[q] : INT32_MIN;
}
int32_t mpg_halo_recv_count(mpg_halo_t h, int32_t q) {
    return h && q >= 0 && q < h->nranks ? h->recv_cnt[q] : -1;
}
int mpg_halo_recv_rows(mpg_halo_t h, int32_t q, int64_t* rows) {
    if (!h || q < 0 || q >= h->nranks || (!rows && h->recv_cnt[q])) return MPG_ERR_ARG;
    for (int i = 0; i < h->recv_cnt[q]; ++i) rows[i] = h->halo_global[(size_t)h->recv_off[q] + i];
    return MPG_OK;
}
int mpg_halo_set_send(mpg_halo_t h, int32_t q, int32_t count, const int64_t* rows) {
    if (!h || q < 0 || q >= h->nranks || count < 0 || (count && !rows)) return MPG_ERR_ARG;
    const int64_t r0 = h->row_starts[h->rank], r1 = h->row_starts[h->rank + 1];
    auto& v = h->send_local[q];
    v.resize((size_t)count);
    for (int i = 0; i < count; ++i) {
        if (rows[i] < r0 || rows[i] >= r1) return MPG_ERR_ARG;
        v[(size_t)i] = (int32_t)(rows[i] - r0);
    }
    h->send_set[q] = true;
    return MPG_OK;
}
int mpg_halo_local_cols(mpg_halo_t h, int32_t* out) {
    if (!h || !out) return MPG_ERR_ARG;
    std::copy(h->col_local.begin(), h->col_local.end(), out);
    return MPG_OK;
}
void mpg_halo_free(mpg_halo_t h) { delete h; }

int mpg_rccl_unique_id(char* id_out, int len) {
    if (!id_out || len < (int)sizeof(ncclUniqueId)) return MPG_ERR_ARG;
    ncclUniqueId uid;
    if (ncclGetUniqueId(&uid) != ncclSuccess) return MPG_ERR_RCCL;
    std::memcpy(id_out, &uid, sizeof uid);
    return MPG_OK;
}

int mpg_engine_create_dist(const mpg_solve_args* a, mpg_halo_t plan, const char* id, int32_t nranks, int32_t rank,
                           mpg_engine_t* out, char* err, int errlen) {
    if (!a || !plan || !id || !out || plan->nranks != nranks || plan->rank != rank || plan->n_local != a->n)
        return MPG_ERR_ARG;
    for (int q = 0; q < nranks; ++q)
        if (!plan->send_set[q]) {
            if (err) std::snprintf(err, (size_t)errlen, "halo plan: send list of peer %d not set", q);
            return MPG_ERR_ARG;
        }
    *out = nullptr;
    auto* e = new mpg_engine();
    try {
        set_quiet(!a->verbose || rank != 0);
        check(mpg_ctx_create(a->device, &e->ctx), "mpg_ctx_create");
        ScopedContext scope(e->ctx);
        e->comm = std::make_unique<RcclComm>(e->ctx, *plan, id, nranks, rank);
        mpg_solve_args local = *a;
        local.col = plan->col_local.data();
        e->eng = std::make_unique<FusedEngine>(e->ctx, local, e->comm.get(), mpg_halo_n_ext(plan), plan->n_front);
    } catch (const std::exception& ex) {
        if (err && errlen > 0) std::snprintf(err, (size_t)errlen, "%s", ex.what());
        mpg_engine_destroy(e);
        return MPG_ERR_RCCL;
    }
    *out = e;
    return MPG_OK;
}

int mpg_engine_create_dist_host(const mpg_solve_args* a, mpg_halo_t plan, const mpg_host_transport* t,
                                int32_t nranks, int32_t rank, mpg_engine_t* out, char* err, int errlen) {
    if (!a || !plan || !t || !t->allreduce || !t->exchange || !out || plan->nranks != nranks || plan->rank != rank ||
        plan->n_local != a->n)
        return MPG_ERR_ARG;
    for (int q = 0; q < nranks; ++q)
        if (!plan->send_set[q]) {
            if (err) std::snprintf(err, (size_t)errlen, "halo plan: send list of peer %d not set", q);
            return MPG_ERR_ARG;
        }
    *out = nullptr;
    auto* e = new mpg_engine();
    try {
        set_quiet(!a->verbose || rank != 0);
        check(mpg_ctx_create(a->device, &e->ctx), "mpg_ctx_create");
        ScopedContext scope(e->ctx);
        e->comm = std::make_unique<HostComm>(e->ctx, *plan, *t, nranks, rank);
        mpg_solve_args local = *a;
        local.col = plan->col_local.data();
        e->eng = std::make_unique<FusedEngine>(e->ctx, local, e->comm.get(), mpg_halo_n_ext(plan), plan->n_front);
    } catch (const std::exception& ex) {
        if (err && errlen > 0) std::snprintf(err, (size_t)errlen, "%s", ex.what());
        mpg_engine_destroy(e);
        return MPG_ERR_ARG;
    }
    *out = e;
    return MPG_OK;
}

int mpg_solve_loopback(const mpg_solve_args* a, int32_t P, mpg_solve_result* r) {
    return mpg_solve_loopback_ex(a, P, r, nullptr);
}

}  // extern "C"

namespace mpg {
namespace {

using CommFactory = std::function<std::unique_ptr<Comm>(int q, mpg_ctx_t ctx, const mpg_halo& plan)>;

// calls `done` when it leaves scope (before the communicator it follows is destroyed)
struct OnExit {
    std::function<void()> done;
    ~OnExit() {
        if (done) done();
    }
};

// P ranks as host threads of this process, rank q on devices[q], rows split
// evenly by nnz; `make_comm` gives each rank its communicator (loopback hub
// or an RCCL clique). The result gathers x from every rank and the history
// from rank 0, as mpg_solve reports them.
int solve_rank_threads(const mpg_solve_args* a, int32_t P, mpg_solve_result* r, mpg_rank_layout* layouts,
                       const std::vector<int>& devices, const CommFactory& make_comm,
                       const std::function<void()>& on_error,
                       const std::function<void(int)>& on_comm_gone = nullptr) {
    const int n = a->n;
    const auto starts = nnz_balanced_starts(n, a->rowptr, P, mpg_csr_node_dof(n, a->rowptr, a->col));
    // per-rank row slices and halo plans
    std::vector<std::vector<int32_t>> rp(P), cg(P);
    std::vector<mpg_halo_t> plans(P, nullptr);
    auto free_plans = [&] {
        for (auto p : plans) mpg_halo_free(p);
    };
    for (int q = 0; q < P; ++q) {
        const int64_t r0 = starts[q], r1 = starts[q + 1];
        const int32_t base = a->rowptr[r0];
        rp[q].resize((size_t)(r1 - r0) + 1);
        for (int64_t i = r0; i <= r1; ++i) rp[q][(size_t)(i - r0)] = a->rowptr[i] - base;
        cg[q].assign(a->col + base, a->col + a->rowptr[r1]);
        if (mpg_halo_analyze(q, P, starts.data(), (int32_t)(r1 - r0), rp[q].data(), cg[q].data(), &plans[q])) {
            free_plans();
            return MPG_ERR_ARG;
        }
    }
    for (int q = 0; q < P; ++q)
        for (int p = 0; p < P; ++p) {
            if (p == q) continue;
            const int c = mpg_halo_recv_count(plans[p], q);  // what p needs from q
            std::vector<int64_t> rows((size_t)c);
            mpg_halo_recv_rows(plans[p], q, rows.data());
            mpg_halo_set_send(plans[q], p, c, rows.data());
        }
    std::vector<std::string> errors(P);
    std::vector<double> seconds((size_t)P, 0.0);
    std::vector<std::thread> th;
    for (int q = 0; q < P; ++q) {
        th.emplace_back([&, q] {
            mpg_ctx_t ctx = nullptr;
            try {
                check(mpg_ctx_create(devices[(size_t)q], &ctx), "mpg_ctx_create");
                ScopedContext scope(ctx);
                {
                    std::unique_ptr<Comm> comm = make_comm(q, ctx, *plans[q]);
                    OnExit gone{on_comm_gone ? std::function<void()>([&, q] { on_comm_gone(q); }) : nullptr};
                    const int64_t r0 = starts[q], r1 = starts[q + 1];
                    const int32_t base = a->rowptr[r0];
                    mpg_solve_args la = *a;
                    la.n = (int32_t)(r1 - r0);
                    la.nnz = rp[q].back();
                    la.rowptr = rp[q].data();
                    la.col = plans[q]->col_local.data();
                    la.val = a->val + base;
                    la.b = a->b + r0;
                    la.x_true = a->x_true ? a->x_true + r0 : nullptr;
                    la.device = devices[(size_t)q];
                    if (q != 0) la.verbose = 0;
                    FusedEngine e(ctx, la, comm.get(), mpg_halo_n_ext(plans[q]), plans[q]->n_front);
                    if (layouts) {
                        mpg_rank_layout& L = layouts[q];
                        L = mpg_rank_layout{};
                        int64_t stored = 0;
                        check(mpg_arnoldi_spmv_layout(e.arnoldi(), &L.format, &L.vec_width, nullptr, &stored,
                                                      &L.window), "layout", ctx);
                        check(mpg_arnoldi_sell_columns(e.arnoldi(), &L.col_form, &L.csr_slices, &L.implicit_slices),
                              "columns", ctx);
                        L.n_local = la.n;
                        L.n_front = plans[q]->n_front;
                        L.n_ext = mpg_halo_n_ext(plans[q]);
                        L.row0 = r0;
                        L.half_rows_scaled = e.half_stats()[0];
                        L.givens_folded = e.givens_folded() ? 1 : 0;
                        L.device = devices[(size_t)q];
                        L.transport_ranks = comm->transport_ranks();
                    }
                    const auto t1 = std::chrono::steady_clock::now();
                    bool done = false;
                    while (!done) e.run(1 << 20, done);
                    e.sync();
                    seconds[(size_t)q] = std::chrono::duration<double>(std::chrono::steady_clock::now() - t1).count();
                    mpg_solve_result mine{};
                    mine.x_out = r->x_out ? r->x_out + r0 : nullptr;
                    e.finish_report(&mine);
                    if (q == 0) {
                        fill_history(e, r);
                        r->res_norm = mine.res_norm;
                        r->err_norm = mine.err_norm;
                    }
                }
            } catch (const std::exception& ex) {
                errors[q] = ex.what();
                on_error();
            }
            if (ctx) mpg_ctx_destroy(ctx);
        });
    }
    for (auto& t : th) t.join();
    free_plans();
    r->gmres_seconds = *std::max_element(seconds.begin(), seconds.end());  // the slowest rank's solve
    for (int q = 0; q < P; ++q)
        if (!errors[q].empty()) {
            r->status = MPG_RESULT_ERROR;
            std::snprintf(r->message, sizeof r->message, "rank %d: %s", q, errors[q].c_str());
            return MPG_ERR_ARG;
        }
    return MPG_OK;
}

}  // namespace
}  // namespace mpg

extern "C" {

int mpg_solve_loopback_ex(const mpg_solve_args* a, int32_t P, mpg_solve_result* r, mpg_rank_layout* layouts) {
    if (!a || !r || P < 1 || a->n < P) return MPG_ERR_ARG;
    r->status = MPG_RESULT_ERROR;
    r->message[0] = 0;
    Hub hub(P);
    const std::vector<int> devices((size_t)P, a->device);
    return solve_rank_threads(
        a, P, r, layouts, devices,
        [&](int, mpg_ctx_t ctx, const mpg_halo& h) -> std::unique_ptr<Comm> {
            return std::make_unique<LoopbackComm>(hub, ctx, h);
        },
        [&] { hub.abort(); });
}

int mpg_solve_multi_gpu(const mpg_solve_args* a, int32_t ngpus, const int32_t* devices_in, mpg_solve_result* r,
                        mpg_rank_layout* layouts) {
    if (!a || !r || ngpus < 1 || a->n < ngpus) return MPG_ERR_ARG;
    r->status = MPG_RESULT_ERROR;
    r->message[0] = 0;
    int visible = 0;
    if (hipGetDeviceCount(&visible) != hipSuccess) visible = 0;
    std::vector<int> devices((size_t)ngpus);
    for (int q = 0; q < ngpus; ++q) devices[(size_t)q] = devices_in ? devices_in[q] : q;
    for (int q = 0; q < ngpus; ++q) {
        const int d = devices[(size_t)q];
        if (d < 0 || d >= visible) {
            std::snprintf(r->message, sizeof r->message,
                          "%d GPU(s) requested but %d visible: rank %d would run on device %d", ngpus, visible, q, d);
            return MPG_ERR_ARG;
        }
        for (int p = 0; p < q; ++p)
            if (devices[(size_t)p] == d) {
                std::snprintf(r->message, sizeof r->message,
                              "device %d named twice (ranks %d and %d): RCCL runs one rank per GPU", d, p, q);
                return MPG_ERR_ARG;
            }
    }
    std::vector<ncclComm_t> comms((size_t)ngpus, nullptr);
    const ncclResult_t nr = ncclCommInitAll(comms.data(), ngpus, devices.data());
    if (nr != ncclSuccess) {
        std::snprintf(r->message, sizeof r->message, "ncclCommInitAll over %d GPU(s): %s", ngpus,
                      ncclGetErrorString(nr));
        return MPG_ERR_RCCL;
    }
    std::vector<std::atomic<bool>> taken((size_t)ngpus);
    for (auto& t : taken) t = false;
    std::mutex mu;
    std::vector<RcclComm*> live((size_t)ngpus, nullptr);
    const int st = solve_rank_threads(
        a, ngpus, r, layouts, devices,
        [&](int q, mpg_ctx_t ctx, const mpg_halo& h) -> std::unique_ptr<Comm> {
            taken[(size_t)q] = true;  // the RcclComm owns (or on failure destroyed) comms[q]
            auto c = std::make_unique<RcclComm>(ctx, h, comms[(size_t)q], ngpus, q);
            std::lock_guard<std::mutex> lk(mu);
            live[(size_t)q] = c.get();
            return c;
        },
        [&] {
            // a failed rank: every live peer is asked to abort; its bounded
            // wait (FusedEngine::wait_event) sees the request, aborts its own
            // communicator on its own thread and fails (aborting
            // them from here freed communicators their owners were using)
            std::lock_guard<std::mutex> lk(mu);
            for (auto* c : live)
                if (c) c->request_abort();
        },
        [&](int q) {
            std::lock_guard<std::mutex> lk(mu);
            live[(size_t)q] = nullptr;
        });
    for (int q = 0; q < ngpus; ++q)
        if (!taken[(size_t)q] && comms[(size_t)q]) ncclCommDestroy(comms[(size_t)q]);
    return st == MPG_OK ? MPG_OK : (std::strstr(r->message, "RCCL") ? MPG_ERR_RCCL : st);
}

}  // extern "C"
