// exchange.h -- cross-shard reductions of the block-angular sharded solve
// (not in the reference, which is single-process C).
//
// A block-angular LP is split so that shard k owns whole diagonal blocks
// (their rows and columns) and a replica of every linking row.  With the
// linking rows forced into the dense tail of the KKT factor
// (kkt_plan.h, nforced), everything below the tail is shard-local and the
// shards meet only in:
//   * the tail's Schur complement  S = -E_link - sum_k L_k D_k^-1 L_k'
//     (one allreduce of the nt x nt tail block per factorisation);
//   * the tail part of each forward sweep's right-hand side (nt values);
//   * linking-row products A_link x (nt values) for residuals;
//   * the scalars of the iteration: dot products, norms, the ratio test.
// Replicated quantities (linking-row y, w, the tail factor and solution)
// come out bitwise identical on every shard because every shard applies
// the same kernels to the same allreduced inputs.
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>

namespace ipo {

enum class RedOp { Sum = 0, Max = 1, Min = 2 };

class Exchange {
  public:
    virtual ~Exchange() = default;
    virtual int rank() const = 0;
    virtual int size() const = 0;
    // in-place allreduce of n doubles in device memory, ordered on stream s
    virtual void allreduce(double* d, size_t n, RedOp op, hipStream_t s) = 0;
};

// RCCL over xGMI: one process per GPU, communicator from a unique id that
// the caller distributes (rank 0 creates it).
Exchange* make_rccl_exchange(const void* unique_id, int nranks, int rank);
void rccl_unique_id(void* out128);

// Host callback (tests, or hosts that bring their own transport): device
// data is staged through pinned host memory and reduced by fn(user, buf,
// n, op) with op 0 = sum, 1 = max, 2 = min; fn returns 0 on success.
using HostAllreduceFn = int (*)(void* user, double* buf, long n, int op);
Exchange* make_host_exchange(int nranks, int rank, HostAllreduceFn fn, void* user);

}  // namespace ipo
