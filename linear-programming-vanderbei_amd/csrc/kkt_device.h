// kkt_device.h -- device-resident numeric LDL^T of the ipo KKT matrix.
//
// Replaces the numeric half of src/ipo/ldlt.c:
//   factor()   <- inv_num  ldlt.c:164-309 (assembly, lltnum :517-636,
//                 dependent-pivot rule :600-614, eps_diag growth :293-306)
//   solve()    <- solve    ldlt.c:327-425 (iterative refinement) with
//                 rawsolve ldlt.c:433-505 as supernodal level sweeps
// Everything stays in HBM between calls; only a few scalars (refinement
// residual, min |d|, dependent-pivot count) come back to the host.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <memory>
#include <vector>

#include "hip_util.h"
#include "exchange.h"
#include "kkt_plan.h"

namespace ipo {

// Device view of the dense tail (see kkt_plan.h): S = nt x nt column-major.
// Blocks per visit of the look-ahead dense tail (kkt_dense.hip, visit_hi):
// IPO_HIP_VISIT_BLOCKS overrides.
// Measured on dfl001's tail (tools/ubench_tail): per-step launches (round 4)
// 4 -> 2.43 ms, 6 -> 2.26, 8 -> 2.55; the persistent run with the window
// hand-off (round 6, latest chunk L in brackets) 3 -> 1.92 (3), 4 -> 1.79
// (4), 5 -> 1.80 (2-4), 6 -> 1.85 (2), 7 -> 1.96, 8 -> 2.08
constexpr int kTailVisitBlocks = 4;
// the persistent tail's latest chunk per column (tail_run_schedule): it must
// finish within one step (IPO_HIP_VISIT_LATEST overrides); equal to the
// chunk, every tile receives the per-step launches' chunks (bitwise them)
constexpr int kTailVisitLatest = 4;
struct TailView {
    double* S;
    int nt, ntb, tc;
    const int* task_ptr;
    const TailTask* tasks;
    double* W;        // nt x 64 workspace: L21 * D of the current block column
    int vk = kTailVisitBlocks;   // blocks per deferred trailing update (visit) of a tile
    int dep = 1;      // dependent pivots inside the look-ahead panel (kkt_dense.hip panel_w_body; 0: bail to the host)
    // visit schedule (tail_visit_schedule): launch t's visits are vlist[vptr[t] ..
    // vptr[t + 1]), each (bi | c << 8 | b0 << 16 | b1 << 24); vlist on the
    // device, vptr on the host; null: the visit_hi formula alone
    const unsigned* vlist = nullptr;
    const int* vptr = nullptr;
    int sdep = 1;     // dependent pivots inside the sparse fused panels (k_panel_w, k_panel_s; 0: redo the factor)
};

// The look-ahead dense tail as ONE persistent launch (k_tail_run): the
// items of launches [t0, ntb) of tail_run_schedule, drawn by ticket.
// Counters: pdone[t] = panel workgroups of step t done, vseq[bi * ntb + c] =
// visits of tile (bi, c) done -- both zeroed before a factorisation's first
// run and kept for a run resumed after a repair; ticket zeroed before every run.
struct TailRun {
    const uint2* items;   // the run's first item (launch t0's)
    int n;                // items in the run
    int t0;               // its first launch
    int* ticket;
    int* pdone;
    int* vseq;
    // window hand-off (kkt_dense.hip RunPub; null: off): tile window (t, j, w)
    // at pub + (((t & 1) ntb + j) 4 + w) kTailPubWin once wflag[(t ntb + j) 4
    // + w] == epoch (one epoch per launch, never reused: no reset)
    double* pub = nullptr;
    int* wflag = nullptr;
    int* pread = nullptr;     // [ntb] panels of step t done reading step t - 1's windows
    int epoch = 0;
    // developer trace (tools/ubench_tail UB_TRACE): per item {drawn, ready,
    // done} in s_memrealtime ticks (100 MHz) and the workgroup's XCC id; null: off
    unsigned long long* trace = nullptr;
};

// one published tile window: 16 columns of 64 rows of L, then the 16 pivots d
constexpr int kTailPubWin = 16 * 64 + 16;

// The dense tail as one launch around a chain workgroup (k_tail_chain_run):
// the chain item factors every diagonal block and solves tile t + 1 of each
// step, keeping block t's L in LDS for block t + 1's pre-update; tile items
// solve the other tiles against its published windows; visits as in TailRun.
// Every counter and flag is zeroed before each launch (chain_zero_ints).
struct ChainRun {
    const uint2* items;   // tail_chain_schedule
    int n;
    int* ticket;          // [1]
    int* abort;           // [1] a contradicted speculation / a bail: the host redoes the factorisation
    int* pdone;           // [ntb] row tiles of block column t final (the chain 1, the tile items 1 each)
    int* rdone;           // [ntb * ntb] rows of tile R in block column t final (t * ntb + R)
    int* vseq;            // [ntb * ntb] visits of tile (bi, c) done (bi * ntb + c)
    int* dwin;            // [ntb * 4] diagonal window w of block t published (t * 4 + w)
    double* dpub;         // [ntb * 4 * kChainWinPub] the published windows
    double* save;         // [2 * 64 * 64 + 64] the chain's step inputs (a dependent-pivot rerun)
    int latest;           // the visit schedule's latest-chunk blocks (tail_run_schedule's L)
    int novisit = 0;      // developer timing only (tools/ubench_tail UB_NOVISIT): the schedule holds no visits
    unsigned long long* trace = nullptr;   // as TailRun::trace
};
// ints of ChainRun's counters for ntb block columns (ticket, abort, pdone, rdone, vseq, dwin)
inline size_t chain_zero_ints(int ntb) { return 2 + ntb + 2 * static_cast<size_t>(ntb) * ntb + 4 * static_cast<size_t>(ntb); }
constexpr int kChainWinPub = 16 * 64 + 32;   // one window: c = l d of the block rows (16 x 64), d (16), mark (16)

// Device-time phases of the KKT core (timing mode), with the algorithmic
// work of one occurrence (one factorisation / one substitution sweep).
// kPhTail: the look-ahead dense-tail factor (k_tail_pr and its repair launches).
enum KktPhase { kPhGather = 0, kPhDiag, kPhTrsm, kPhSyrk, kPhForward, kPhBackward, kPhTail, kNumPhases };

struct KktTimers {
    double phase_ms[kNumPhases] = {};       // accumulated device time per phase
    long phase_launches[kNumPhases] = {};   // kernel launches per phase
    long phase_count[kNumPhases] = {};      // occurrences (factorisations / sweeps)
    double factor_ms = 0.0;   // accumulated device time of factor()
    double solve_ms = 0.0;    // accumulated device time of solve()
    double sweep_ms = 0.0;    // forward + backward substitution sweeps (timing mode)
    long factors = 0, solves = 0, rawsolves = 0;
    long panel_redos = 0;     // factorisations redone without the fused panel kernels
    long redo_where[4] = {0, 0, 0, 0};   // ... by the kernel that bailed (k_panel, k_panel_w sparse / tail, k_panel_s)
    long tail_repairs = 0;    // dense-tail block columns redone in place (look-ahead resumed after them)
    long tail_dep_rounds = 0; // k_tail_dep launches of those repairs
    long tail_chain_aborts = 0;   // k_tail_chain_run launches aborted (the factorisation redone per step)
};

// The Q block of ldlt.c's K (ldlt.c:253-256, 391-394) on the y-nodes:
// K_yy = -max(E, eps) - qmax Q, Q m x m full symmetric CSC (kkt_plan.h
// QPattern), qmax = the reference's lp->max (-1 max, 1 min).
struct QBlock {
    const int* kQ = nullptr;
    const int* iQ = nullptr;
    const double* Q = nullptr;
    int qmax = 1;
};

class KktDevice {
  public:
    // A is the solver's m x n matrix (CSC).  The plan (ordering, supernodes)
    // is computed here on the host.  kA/iA/A must outlive nothing: copied.
    // nforced > 0: the last nforced rows (linking rows of a block-angular
    // shard) form the dense tail (kkt_plan.h); with an Exchange set, the
    // tail Schur complement, the tail right-hand sides and the refinement
    // residual of those rows are summed over the shards (exchange.h).
    // qb: an optional Q block (not with nforced > 0).
    KktDevice(int m, int n, const int* kA, const int* iA, const double* A, hipStream_t stream, int nforced = 0,
              const QBlock* qb = nullptr);
    ~KktDevice();
    KktDevice(const KktDevice&) = delete;
    KktDevice& operator=(const KktDevice&) = delete;

    const KktPlan& plan() const { return plan_; }
    void set_exchange(Exchange* x) { xch_ = x; }
    int nforced() const { return nforced_; }
    int m() const { return m_; }
    int n() const { return n_; }
    hipStream_t stream() const { return stream_; }

    // Device copies of the constraint matrix in both orientations.
    const int* kA() const { return dkA_.get(); }
    const int* iA() const { return diA_.get(); }
    const double* A() const { return dA_.get(); }
    const int* kAt() const { return dkAt_.get(); }
    const int* iAt() const { return diAt_.get(); }
    const double* At() const { return dAt_.get(); }

    // Numeric factorisation of K(E, D); E (m), D (n) are device vectors.
    void factor(const double* dE, const double* dD);
    // In-place refined solve of  -E dy + A dx = fy,  A' dy + D dx = fx.
    // Returns the rawsolve consistency flag of the last pass (1 = consistent).
    int solve(const double* dE, const double* dD, double* dfy, double* dfx);
    // Two independent refined solves with the same factor (hsd.c:218-224),
    // their substitution sweeps batched; each keeps its own refinement loop.
    int solve2(const double* dE, const double* dD, double* dfy1, double* dfx1, double* dfy2, double* dfx2);
    void solve_multi(int R, const double* dE, const double* dD, double* const* dfy, double* const* dfx, int* ok);

    // One unrefined sweep L D L' z = rhs on R permuted device vectors at dz + r K.
    void rawsolve(double* dz, int R = 1);

    // What a factorisation changes on the host side (eps_diag growth,
    // dependent-pivot count, timers and counters): saved before a
    // speculative factorisation and put back when the caller ends up not
    // using it (the overlapped HSD iteration that finds mu < 1e-12).
    struct HostState {
        double epsdiag;
        int ndep;
        KktTimers tm;
    };
    HostState host_state() const { return {epsdiag_, ndep_, tm_}; }
    void restore_host_state(const HostState& h) { epsdiag_ = h.epsdiag; ndep_ = h.ndep; tm_ = h.tm; }

    double epsdiag() const { return epsdiag_; }
    void set_pivot_tolerance(double t) { pivot_tol_ = t; }
    void set_epsdiag(double e) { epsdiag_ = e; }
    // The refinement's residual takes rows row0..m-1 (trailing long rows, an
    // unsharded solve) from one wave each (launch_link_ax: lanes strided,
    // then a wave sum -- a fixed order, not sparse_dot's) instead of one
    // thread's serial sparse_dot.  For LPs on the segmented-dot policy only
    // (IpmSolver, dev_common.h kOrderedMaxLen).
    void set_long_rows(int row0);
    double pivot_tolerance() const { return pivot_tol_; }
    int ndep() const { return ndep_; }
    int last_passes() const { return last_passes_; }
    const KktTimers& timers() const { return tm_; }
    void enable_timing(bool on) { timing_ = on; }
    void reset_timers() { tm_ = KktTimers(); }

    // Diagnostics: copy numeric factor to host (panels + D), for tests.
    void download_factor(double* lx, double* d, int* live = nullptr) const;
    double* device_lx() const { return dLx_.get(); }
    double* device_diag() const { return dDg_.get(); }

  private:
    void factor_core(const double* dE, const double* dD);
    void dump_factor(const double* dE, const double* dD, double eps_in);
    int dump_count_ = 0;
    TailView tail_view() const;
    template <int R>
    void sweep(double* dz, const double* epsp);
    void sweep_blocked(double* dz, const double* epsp);
    void tail_rhs_begin(double* dz, int R);
    void tail_rhs_end(double* dz, int R);
    size_t ybuf_stride_ = 1, partial_stride_ = 1;
    DevBuf<int> dIncons_;          // per right-hand side: inconsistent-system flag
    int launch_gather(const struct PlanView& pv, const TailView& tv, int tail, int group, hipStream_t s);
    int fwd_launches_ = 0, bwd_launches_ = 0;   // kernel launches per substitution sweep
    void launch_reduce_maxabs2(const double* a, int na, const double* b, int nb, double* dst);

    int m_, n_, T_;
    int nforced_ = 0;
    Exchange* xch_ = nullptr;      // not owned
    DevBuf<double> dLinkAx_;       // [2 * nforced] linking-row products A_link dx per right-hand side
    int long_row0_ = -1;           // set_long_rows: rows >= it by one wave each (-1: none)
    DevBuf<double> dLongAx_;       // [2 * (m - long_row0_)] their products A dx per right-hand side
    bool shard_minor() const { return xch_ && xch_->rank() != 0; }   // holds replicas of the linking rows
    void xsum(double* d, size_t n, RedOp op) { if (xch_) xch_->allreduce(d, n, op, stream_); }
    hipStream_t stream_;
    KktPlan plan_;
    double epsdiag_ = 1.0e-14;     // ldlt.c:31, grows x10 (ldlt.c:301-305)
    int ndep_ = 0;
    // Zero-pivot test |d| <= tol * sum|terms| (the reference tests d == 0,
    // which in its own operation order catches exact cancellations; a
    // different summation order can leave a residue below one ulp of the
    // largest term instead).  1e-17 was chosen by sweeps over the netlib
    // set (a host emulation of the GPU factor in round 1, tools/tau_sweep.py on the GPU):
    // 2^-46 over-flags twin-column pivots the reference keeps, exact zero
    // under-flags; 1e-17 matched the most hsd and intpt iteration counts.
    double pivot_tol_ = 1.0e-17;
    int last_passes_ = 0;
    bool timing_ = false;
    KktTimers tm_;
    hipEvent_t ev0_ = nullptr, ev1_ = nullptr, ev2_ = nullptr, ev3_ = nullptr;
    std::vector<hipEvent_t> kev_;   // event pool (timing mode)
    size_t kev_used_ = 0;
    struct PhaseMark { hipEvent_t b, e; int phase, launches; };
    std::vector<PhaseMark> marks_;
    hipEvent_t mark_b_ = nullptr;
    hipEvent_t next_event();
    void ph_begin(hipStream_t s);
    void ph_end(int phase, int launches, hipStream_t s);
    void ph_collect();               // after a stream sync
  public:
    // algorithmic flops / bytes of one occurrence of each phase
    double work_flops[kNumPhases] = {}, work_bytes[kNumPhases] = {};
  private:

    // matrix
    DevBuf<int> dkA_, diA_, dkAt_, diAt_;
    DevBuf<double> dA_, dAt_;
    // Q block (qnz_ > 0): CSC, its assembly map, its diagonal by y-node (old order)
    int qnz_ = 0, qmax_ = 1;
    DevBuf<int> dkQ_, diQ_;
    DevBuf<double> dQ_, dQdiag_;
    DevBuf<int64_t> dqmap_;
    // plan
    DevBuf<int> dcol0_, drowptr_, drows_, dperm_, diperm_;
    DevBuf<int64_t> doff_, damap_, ddslot_, drelptr_;
    DevBuf<int> dunit_sup_, dunit_tile_, dtask_ptr_, dtask_pair_, dtask_i0_, dtask_i1_;
    DevBuf<int> dupd_src_, dupd_r0_, dupd_r1_, drel_, dlevel_sups_;
    DevBuf<int> dyrow_ptr_, dyrow_idx_;
    // deep trees: the narrow range's update lists without the values from
    // below the range, and those values' lists for the pre-pass (k_fwd_pre)
    int pre_cols_ = 0;
    DevBuf<int> dylate_ptr_, dylate_idx_, dpre_col_, dpre_ptr_, dpre_idx_;
    DevBuf<double> dYbuf_;
    // sync-free top levels of the sweeps (k_fwd_sf / k_bwd_sf)
    void build_sync_free_plan();
    int sf_level_ = 0;                    // first level of the range (nlevels: none)
    int nsf_f_ = 0, nsf_b_ = 0, sf_grid_ = 1;
    int sf_fwd_epoch_ = 0, sf_bwd_epoch_ = 0;
    long long sf_ticket_next_[2] = {0, 0};   // work-item ticket counters (forward, backward): next launch's base
    std::vector<int2> h_sf_items_f_;         // forward sync-free items (host copy, developer stamps)
    int sf_tbase(int d, int nitems);
    size_t zpad_stride_ = 1;
    std::vector<int> h_chunk0_;           // per supernode: first solve chunk (-1: not chunked)
    DevBuf<int2> dsf_items_f_, dsf_items_b_;
    DevBuf<int> dsf_need_, dsf_par_, dsf_zbase_, dsf_zpi_, dsf_fcnt_, dsf_fflag_, dsf_bcnt_, dsf_bflag_, dsf_ticket_;
    DevBuf<int> dybase_;                  // per supernode: first ybuf slot of its update values
    DevBuf<double> dZpad_;                // padded z slices of the range, 2 right-hand sides
    std::vector<int> fu_ptr_;             // per level: fused panel units [fu_ptr_[l], fu_ptr_[l+1])
    DevBuf<int> dfu_sup_, dfu_j_;         // fused panel unit -> supernode, tile pair index
    std::vector<int> small_ptr_;          // per level: small panels [small_ptr_[l], small_ptr_[l+1]) (k_panel_s)
    std::vector<char> split_level_;       // per level: k_diag + k_trsm instead of the fused panels (wide levels)
    std::vector<int> small1_cnt_;         // per level: leading single-column small panels of <= 8 rows (k_panel_s1)
    DevBuf<int> dsmall_sups_;
    bool use_panel_ = true;               // fused diagonal-block + panel kernels (IPO_HIP_PANEL=0: off)
    bool factor_pass(const double* dE, const double* dD, bool fused, bool tail_fused);
    void enqueue_levels(const PlanView& pv, const TailView& tv, bool fused, hipStream_t s);
    bool graph_on_ = false;               // the levels' fused launches replayed as one HIP graph (IPO_HIP_GRAPH=1: on)
    hipGraphExec_t lvl_exec_ = nullptr;   // that graph, captured at the first fused factorisation
    bool finish_pass(bool fused);
    void repair_tail();
    std::vector<int> chunk_ptr_;          // per level: solve chunks [chunk_ptr_[l], chunk_ptr_[l+1])
    std::vector<int> leaf_cnt_;           // per level: leading single-column supernodes of dsweep_sups_
    std::vector<int> leaf8_cnt_;          // per level: the first of them, small leaves (k_fwd_leaf8 / k_bwd_leaf8)
    bool merge_levels_ = true;            // a level's leaves and other supernodes in one sweep launch (IPO_HIP_MERGE_LEVELS)
    bool merge_panels_ = true;            // a level's fused and small panels in one launch (k_panel_ws; the same knob)
    int small_leaves_ = 0;                // levels with at least this many small leaves pack them (IPO_HIP_SMALL_LEAVES; 0: never)
    DevBuf<int> dsweep_sups_;             // level_sups in sweep order (leaves first on unchunked levels)
    DevBuf<int> dchunk_sup_, dchunk_r0_, dsup_chunk0_;
    DevBuf<double> dPartial_;    // backward partial sums, one 64-vector per chunk
    // split-K gather chunks per group (sparse level l, group nlevels = tail)
    bool visits_ = false;
    int gst_group_ = -1, gst_n_ = 0;   // developer gather stamps (IPO_HIP_GATHER_STAMPS)
    DevBuf<long long> dGStamp_;        // deep trees: early gather slots as visits in lower levels' launches
    std::vector<int> ck_kind_;   // per gather group: 0 k_update, 1 k_update_flat, 2 k_update_quad
    std::vector<bool> ck_wide_;   // ck_flat_: k_update_flat (latency-bound launches of deep trees)      // per gather group: k_update<4> (few chunks, units split >= 4 ways)
    std::vector<int> ck_ptr_, sp_ptr_;
    DevBuf<int> dck_u_, dck_b_, dck_e_, dck_part_, dsp_u_, dsp_p0_, dsp_n_;
    DevBuf<int> dck_q_;          // split-unit index of each chunk (-1: unsplit)
    DevBuf<int> dSplitCnt_;      // arrival counters of the split units (fused split-K), zero between launches
    bool eps_cleared_ = false;   // solve_multi's k_perm_in has zeroed the sweep's eps slots
    DevBuf<double> dPartialTile_;
    DevBuf<TaskSrc> dusrc_, dtsrc_;   // per gather task: source panel descriptor
    DevBuf<SlotRec> dslot_rec_, dtail_slot_rec_;   // per gather k-slot record (sparse units, dense tail)
    DevBuf<unsigned long long> dChainGran_;   // dense-tail sweep chains: z of every block as epoch-tagged granules
    int chain_epoch_ = 0;      // the chains' launch epoch (one per launch, never reused)
    int visit_blocks_ = kTailVisitBlocks;   // TailView::vk (IPO_HIP_VISIT_BLOCKS)
    double epsdiag_cap_ = 0.0;     // IPO_HIP_EPSDIAG_MAX (diagnostics; 0: the reference's unbounded growth)
    int tail_spec_ = 1;            // TailView::dep when the host repair backs it (IPO_HIP_TAIL_SPEC: 0 off, 2 tests)
    int sparse_dep_ = 1;           // TailView::sdep (IPO_HIP_SPARSE_DEP)
    bool chain_pairs_ = false; // dense-tail chains with two blocks per workgroup (k_tail_fwd_pair / _bwd_pair)
    bool chain_lead_ = false;  // forward dense-tail sweep by one lead workgroup + helpers (k_tail_fwd_lead)
    DevBuf<int> dtail_task_ptr_, dtail_kslot_, dtail_kslot_ptr_;
    DevBuf<int> dlead_ticket_;         // k_tail_fwd_lead's role tickets (never reset within a run)
    long long lead_ticket_next_ = 0;
    DevBuf<unsigned> dvisit_list_;     // TailView::vlist (tail_visit_schedule; IPO_HIP_VISIT_SCHED=0: none)
    std::vector<int> visit_ptr_;       // TailView::vptr
    // the dense tail as one persistent launch (k_tail_run; IPO_HIP_TAIL_RUN=0: one launch per step)
    bool tail_run_ = false;
    DevBuf<uint2> drun_items_;         // tail_run_schedule
    std::vector<int> run_ptr_;         // first item of each launch
    DevBuf<int> drun_cnt_;             // ticket, pdone[ntb], vseq[ntb * ntb], pread[ntb]
    // the run's window hand-off (TailRun::pub; IPO_HIP_TAIL_WINPUB=0: off)
    bool run_winpub_ = true;
    DevBuf<double> drun_pub_;          // [2 * ntb * 4 * kTailPubWin]
    DevBuf<int> drun_wflag_;           // [ntb * ntb * 4], zeroed once
    int run_epoch_ = 0;
    // the run of launches [t0, ntb) (reset: a factorisation's first run, counters zeroed)
    void launch_tail_from(int t0, bool reset);
    // the dense tail around a chain workgroup (k_tail_chain_run; IPO_HIP_TAIL_CHAIN=0: the run above)
    bool tail_chain_ = false;
    bool chain_off_ = false;           // this factorisation is being redone after an aborted chain launch
    int run_latest_ = kTailVisitLatest;
    DevBuf<uint2> dchain_items_;
    int chain_n_ = 0;
    DevBuf<int> dchain_cnt_;           // chain_zero_ints(ntb) counters
    DevBuf<double> dchain_pub_, dchain_save_;
    void launch_tail_chain_run();
    DevBuf<uint64_t> dtail_tasks_, dutasks_;
    DevBuf<double> dW_;
    DevBuf<double> dDepSt_;        // k_tail_dep's block state and per-tile maxima
    DevBuf<int> dDepI_;            // its round counters
    // numeric
    DevBuf<double> dLx_, dDg_;
    DevBuf<int> dLive_;
    DevBuf<double> dDscale_;
    DevBuf<int> dFlags_;           // [0] ndep, [1] fused bail bits, [2] 1 + bailed tail block, [4..] node sign
    DevBuf<double> dZ_, dDy_, dDx_, dRy_, dRx_;
    DevBuf<double> dPart_, dScal_;
    double* hScal_ = nullptr;      // pinned
    int* hFlags_ = nullptr;        // pinned
};

}  // namespace ipo
