// kkt_kernels.h -- what the KKT kernel translation units share: the device
// view of the symbolic plan and the launchers of the dense per-panel kernels
// (kkt_dense.hip), which live in their own translation unit because their
// fully unrolled register code dominates compile time.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <vector>

#include "kkt_device.h"
#include "kkt_plan.h"

namespace ipo {

struct PlanView {
    const int* col0;
    const int* rowptr;
    const int* rows;
    const int64_t* off;
    const int* unit_sup;
    const int* unit_tile;
    const int* task_ptr;
    const int* task_pair;
    const int* task_i0;
    const int* task_i1;
    const int* upd_src;
    const int* upd_r0;
    const int* upd_r1;
    const int64_t* relptr;
    const int* rel;
    double* Lx;
    double* dg;
    int* live;
    int* flags;      // [0] dependent pivots, [1] fused panel kernel bail-out, [2] 1 + bailed tail block
    const int* sign; // node class per new index: -1 y-node, +1 x-node
    double* dscale;  // sum of |terms| that formed each pivot (zero-pivot test)
    double tau;      // pivot d is "zero" when |d| <= tau * dscale
    int* incons;     // [r]: right-hand side r met a dropped column with |z| > eps (ldlt.c:462)
    const int* ybase; // per supernode: first ybuf slot of its forward update values
    int xcd;          // k_update launches of at least xcd chunks: consecutive chunks on one XCD (0: never)
};

// Workgroup b of a G-workgroup launch runs on XCD b mod 8 (round-robin
// placement, MI355X_MICROARCH.md).  xcd_chunk(b, G) gives XCD x the
// contiguous chunk range [start_x, start_x + count_x), in dispatch order,
// so neighbouring chunks (the tiles of one target panel, which read the same
// source columns for their B operand) share one L2.  A bijection on [0, G).
static __device__ __forceinline__ int xcd_chunk(int b, int G) {
    const int q = G >> 3, r = G & 7, x = b & 7, i = b >> 3;
    return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + i;
}

// sc1 (agent-scope relaxed atomic) accesses: they bypass the CU's L1, the
// hand-off form of MI355X_MICROARCH.md (stores all sc1, loads all sc1, one
// lane signals after every storing wave's vmcnt(0) and a barrier) for data
// one workgroup passes to another inside a launch
static __device__ __forceinline__ void sc1_store(double* p, double v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
static __device__ __forceinline__ double sc1_load(const double* p) {
    return __hip_atomic_load(const_cast<double*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
static __device__ __forceinline__ int sc1_load_int(const int* p) {
    return __hip_atomic_load(const_cast<int*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// a handed-off value (SC) or a plain one
template <bool SC>
static __device__ __forceinline__ double ld_h(const double* p) {
    if constexpr (SC) return sc1_load(p);
    else return *p;
}
template <bool SC>
static __device__ __forceinline__ void st_h(double* p, double v) {
    if constexpr (SC) sc1_store(p, v);
    else *p = v;
}

// value of v in lane j (j wave-uniform), via two v_readlane_b32
static __device__ __forceinline__ double lane_bcast(double v, int j) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane(static_cast<int>(b), j);
    const int hi = __builtin_amdgcn_readlane(static_cast<int>(b >> 32), j);
    return __longlong_as_double((static_cast<long long>(hi) << 32) | static_cast<unsigned int>(lo));
}

// Diagonal-block LDL' of every supernode of one level (level_sups[q0..q0+count)),
// or, with level_sups == nullptr, of block column kb of the dense tail.
void launch_diag(const PlanView& pv, const int* level_sups, int q0, int count, const TailView& tv, int kb,
                 hipStream_t s);
// L21 = A21 L11^-T D^-1 for factor units [u0, u0+count), or, with
// count < 0, for the rows below block column kb of the dense tail.
void launch_trsm(const PlanView& pv, int u0, int count, const TailView& tv, int kb, hipStream_t s);
// Fused diagonal block + panel rows (the fast path of launch_diag +
// launch_trsm): fused units [f0, f0+count) of a sparse level, or, with
// fu_sup == nullptr, block column kb of the dense tail.  A pivot that fails
// the zero test sets flags[1] and leaves the panel unwritten.
void launch_panel(const PlanView& pv, const int* fu_sup, const int* fu_j, int f0, int count, const TailView& tv,
                  int kb, hipStream_t s);
// Look-ahead dense tail (fused path with k_panel_w): step t = panel of block
// column t (which first applies block t - 1's update to its own rows) beside
// the deferred trailing updates ("visits") scheduled for launch t -- one
// launch per block column.  W = L21 D is formed from L and D where used.
void launch_tail_step(const PlanView& pv, const TailView& tv, int t, hipStream_t s);
// visit tiles of launch t (tail of ntb block columns, chunks of K blocks)
int tail_visit_tiles(int ntb, int t, int K);
// The visits of every look-ahead launch placed so that no launch needs more
// than `cap` workgroups (one round on `cap` CUs): visit_hi's chunks, with
// tiles' first chunks moved into earlier launches where a launch would
// overflow.  Returns the list (TailView::vlist layout) and ptr[0..ntb].
std::vector<unsigned> tail_visit_schedule(int ntb, int nt, int K, int cap, std::vector<int>& ptr);
// Items per launch t (ptr[t] .. ptr[t + 1]): panel workgroups (j, t | chunks
// of column t << 8 | 1 << 31), then visits (bi | c << 8 | b0 << 16 | b1 << 24,
// t | chunk index << 8), column t + 1's first.  Column c's chunks: the latest
// L blocks before c - 1 in launch c - 1, then K at a time in launches c - 2,
// ...; launches over `cap` items move first chunks earlier.
std::vector<uint2> tail_run_schedule(int ntb, int nt, int K, int L, int cap, std::vector<int>& ptr);
void launch_tail_run(const PlanView& pv, const TailView& tv, const TailRun& rc, hipStream_t s);
// The chain launch (k_tail_chain_run, kkt_dense.hip): the chain item, then per
// launch t the tile items (t, R >= t + 2) and the visits of tail_run_schedule
// (ptr as there; the chain item is item 0, before ptr[0]).
std::vector<uint2> tail_chain_schedule(int ntb, int nt, int K, int L, int cap, std::vector<int>& ptr);
void launch_tail_chain(const PlanView& pv, const TailView& tv, const ChainRun& rc, hipStream_t s);
// algorithmic flops / bytes of every visit of one factorisation
void tail_visit_work(int ntb, int nt, int K, double& flops, double& bytes);
// Repair path, block column kb of the dense tail with the dependent-pivot
// rule: one round (k_tail_dep); sti = two copies of {k0, 1 + pending column,
// done, ndep}, both zeroed before round 0; round r reads copy r & 1 and
// writes copy (r + 1) & 1, rounds until the written copy's done flag (one
// round per dependent pivot + 1).  st: tail_dep_state_doubles(ntb) (two copies).
void launch_tail_dep_round(const PlanView& pv, const TailView& tv, int kb, int round, double* st, int* sti,
                           hipStream_t s);
size_t tail_dep_state_doubles(int ntb);
// Block t's update of block column t + 1 alone.
void launch_tail_colupdate(const PlanView& pv, const TailView& tv, int t, hipStream_t s);
// Block column kb as it was before a failed dependent-pivot pass (k_tail_restore).
void launch_tail_restore(const PlanView& pv, const TailView& tv, int kb, hipStream_t s);
// Fused panel of supernodes sups[q0 .. q0+count) that have at most 16
// columns and 64 rows (one wave each, k_panel_s); same bail-out contract.
// a level's fused panel units and small panels in one launch (k_panel_ws)
void launch_panel_ws(const PlanView& pv, const int* fu_sup, const int* fu_j, int f0, int nfu, const TailView& tv,
                     const int* ssups, int s0, int nsm, int dep, hipStream_t s);
// the first n1 of them single-column panels of <= 8 rows, eight to a wave (k_panel_s1)
void launch_panel_small(const PlanView& pv, const int* sups, int q0, int count, int dep, hipStream_t s, int n1 = 0);

}  // namespace ipo
