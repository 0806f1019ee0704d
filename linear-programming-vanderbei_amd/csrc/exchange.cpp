// exchange.cpp -- RCCL and host-callback implementations of Exchange.
#include "exchange.h"

#include <rccl/rccl.h>

#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "hip_util.h"

namespace ipo {
namespace {

void nccl_check(ncclResult_t r, const char* what) {
    if (r != ncclSuccess) throw std::runtime_error(std::string("rccl ") + what + ": " + ncclGetErrorString(r));
}

class RcclExchange final : public Exchange {
  public:
    RcclExchange(const void* id, int nranks, int rank) : rank_(rank), size_(nranks) {
        ncclUniqueId uid;
        std::memcpy(&uid, id, sizeof(uid));
        nccl_check(ncclCommInitRank(&comm_, nranks, uid, rank), "ncclCommInitRank");
    }
    ~RcclExchange() override {
        if (comm_) (void)ncclCommDestroy(comm_);
    }
    int rank() const override { return rank_; }
    int size() const override { return size_; }
    void allreduce(double* d, size_t n, RedOp op, hipStream_t s) override {
        if (n == 0) return;           // one rank still goes through RCCL (tests of this path)
        const ncclRedOp_t o = op == RedOp::Sum ? ncclSum : op == RedOp::Max ? ncclMax : ncclMin;
        nccl_check(ncclAllReduce(d, d, n, ncclDouble, o, comm_, s), "ncclAllReduce");
    }

  private:
    ncclComm_t comm_ = nullptr;
    int rank_, size_;
};

class HostExchange final : public Exchange {
  public:
    HostExchange(int nranks, int rank, HostAllreduceFn fn, void* user)
        : rank_(rank), size_(nranks), fn_(fn), user_(user) {}
    ~HostExchange() override {
        if (buf_) (void)hipHostFree(buf_);
    }
    int rank() const override { return rank_; }
    int size() const override { return size_; }
    void allreduce(double* d, size_t n, RedOp op, hipStream_t s) override {
        if (n == 0 || size_ == 1) return;
        if (n > cap_) {
            if (buf_) IPO_HIP_CHECK(hipHostFree(buf_));
            IPO_HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&buf_), n * sizeof(double), hipHostMallocDefault));
            cap_ = n;
        }
        IPO_HIP_CHECK(hipMemcpyAsync(buf_, d, n * sizeof(double), hipMemcpyDeviceToHost, s));
        IPO_HIP_CHECK(hipStreamSynchronize(s));
        if (fn_(user_, buf_, static_cast<long>(n), static_cast<int>(op)) != 0)
            throw std::runtime_error("host exchange: allreduce callback failed");
        IPO_HIP_CHECK(hipMemcpyAsync(d, buf_, n * sizeof(double), hipMemcpyHostToDevice, s));
        IPO_HIP_CHECK(hipStreamSynchronize(s));   // buf_ is reused by the next call
    }

  private:
    int rank_, size_;
    HostAllreduceFn fn_;
    void* user_;
    double* buf_ = nullptr;
    size_t cap_ = 0;
};

}  // namespace

Exchange* make_rccl_exchange(const void* unique_id, int nranks, int rank) {
    return new RcclExchange(unique_id, nranks, rank);
}

void rccl_unique_id(void* out128) {
    ncclUniqueId uid;
    nccl_check(ncclGetUniqueId(&uid), "ncclGetUniqueId");
    static_assert(sizeof(uid) == 128, "ncclUniqueId size");
    std::memcpy(out128, &uid, sizeof(uid));
}

Exchange* make_host_exchange(int nranks, int rank, HostAllreduceFn fn, void* user) {
    if (!fn) throw std::invalid_argument("host exchange needs a callback");
    return new HostExchange(nranks, rank, fn, user);
}

}  // namespace ipo
