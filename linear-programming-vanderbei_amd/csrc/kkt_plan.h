// kkt_plan.h -- host-side symbolic analysis of the quasi-definite KKT system
//
//        K = [ -E   A ]      E = w/y (m rows, "y-nodes")
//            [  A'  D ]      D = z/x (n cols, "x-nodes")
//
// that ipo factors every interior-point iteration (src/ipo/ldlt.c:164-309,
// called from hsd.c:218 / intpt.c:197).  Symbolic work stays on the host,
// as the reference does it once per process (ldlt.c:211-223):
//
//   * ordering   -- the reference's tiered minimum-degree ordering
//                   (ldlt.c:638-1262), re-implemented here so the GPU
//                   factor has exactly the reference's fill pattern;
//   * supernodes -- consecutive columns with nested structure, split into
//                   panels of at most kPanelCols columns;
//   * schedule   -- supernodal elimination tree levels, per-target update
//                   lists with relative row positions, assembly maps from
//                   A's nonzeros to panel slots.
//
// Node numbering before permutation: y-nodes 0..m-1, x-nodes m..m+n-1.
#pragma once
#include <cstdint>
#include <vector>

namespace ipo {

constexpr int kPanelCols = 64;     // max columns per supernode panel
constexpr int kTileRows = 64;      // rows per factor work unit
constexpr int kSlab = 16;         // k-columns staged per MFMA gather step
constexpr int kTailMin = 128;      // smallest dense tail handled as a dense block
constexpr int kTailMaxWiden = 8192;   // a widened dense tail stays within 8192 columns (512 MB)
constexpr double kTailDensity = 0.7;  // default suffix density of the widened tail (measured)

struct KktOrdering {
    int m = 0, n = 0, T = 0;
    std::vector<int> perm, iperm;  // perm[new] = old
    std::vector<int> Lp, Li;       // strict-lower pattern of L, new indices, sorted
    int pdf = 0;                   // 1 = y-nodes tier 0 ("primal"), 2 = x-nodes tier 0
    int denwin = 0;                // first column of the reference's dense window
    double narth = 0.0;            // reference op count (ldlt.c:1243-1248)
};

// Sparsity of the Q block of ldlt.c's K (ldlt.c:253-256: -max Q added to the
// first node class, here the y-nodes): m x m, full symmetric CSC (both
// triangles and the diagonal, rows sorted in every column, as iolp.c:733-793
// leaves QUADS).  Its off-diagonal entries are edges of the KKT graph
// (ldlt.c:729-745) and make the problem non-separable (ldlt.c:675-682).
struct QPattern {
    const int* kQ = nullptr;
    const int* iQ = nullptr;
    bool separable(int m) const;
};

// ldlt.c:638-858 (inv_sym) + ldlt.c:860-1262 (lltsym), method _MD, dense = 3.
//
// nforced > 0 (not in the reference; block-angular sharding, SURVEY.md
// §8(e)): the last nforced y-nodes (rows m-nforced..m-1, the linking rows)
// are left out of the minimum-degree graph and placed last in natural
// order, and the factor's dense tail is exactly those rows -- the role the
// reference's tier penalty (ldlt.c:994-999) plays for its dense window.
// Every other column's pattern is then independent of the rest of the
// problem, so blocks that share only the linking rows factor apart and meet
// in the tail.  nforced = 0 is the reference ordering, unchanged.
KktOrdering order_tiered_min_degree(int m, int n, const int* kA, const int* iA,
                                    const int* kAt, const int* iAt, int nforced = 0, const QPattern* q = nullptr);

// Nested dissection (kkt_order_nd.cpp; not in the reference): the
// elimination order used instead of the reference's on problems of at least
// kNdMinNodes KKT nodes (every netlib problem is below: ken-11 has 72,086),
// whose minimum-degree trees are thousands of levels deep on banded LPs.
// perm[new] = old; forced rows last in natural order as above.  Pieces of
// at most leaf_rows y-nodes are ordered x-nodes first, then y-nodes.
std::vector<int> nested_dissection_perm(int m, int n, const int* kA, const int* iA, const int* kAt, const int* iAt,
                                        int nforced, int leaf_rows, const QPattern* q = nullptr);
// The symbolic factor (Lp, Li, iperm) of o.perm over the free nodes; forced
// rows get empty columns (add the dense tail after).
void symbolic_from_perm(KktOrdering& o, const int* kA, const int* iA, const int* kAt, const int* iAt, int nforced,
                        const QPattern* q = nullptr);
// Pad chains of columns (parent(j) = j + 1) below column tc into panels of
// at most kPanelCols columns holding at most zfrac explicit zeros (relaxed
// supernodes; the padded entries stay exact zeros in the factor).
void relax_supernodes(KktOrdering& o, int tc, double zfrac);
// nested dissection, Lp/Li, forced tail, relaxed supernodes, narth (of the
// unpadded pattern): the KktOrdering of that order
KktOrdering order_nested_dissection(int m, int n, const int* kA, const int* iA, const int* kAt, const int* iAt,
                                    int nforced, int leaf_rows, double zfrac, const QPattern* q = nullptr);
constexpr int kNdMinNodes = 100000;
constexpr int kNdDense = 64;         // smallest degree of a dense node (also > 10x its class mean)
constexpr int kNdLeafRows = 1024;   // measured on configs[3]: 4.5e10 factor flops, 62 levels (256: 5.5e10, 61)
constexpr double kNdRelax = 0.1;      // explicit-zero fraction of a relaxed panel
// Which order build_kkt_plan uses: IPO_HIP_ORDER = md | nd | auto (default:
// nd from kNdMinNodes KKT nodes up); true = nested dissection
bool use_nested_dissection(int T);
// Host threads of the parallel setup steps (the nested-dissection pieces):
// IPO_HIP_SETUP_THREADS, default min(16, hardware threads)
int setup_threads();

// One gather task into a 64x64 tile of the dense tail: the tail rows of
// source panel `src` whose positions inside the tile's row block (rmask)
// and column block (cmask) are given as bit masks; R_src indices start at
// rbase / cbase and follow the mask bit order.
struct TailTask {
    uint64_t rmask, cmask;
    int src, rbase, cbase, pad;
};

// Where a gather task's source panel lives: Lx + colbase + k * hd is column
// k of its row set R_d; d_k = dg[cd0 + k].
struct TaskSrc {
    int64_t colbase;
    int hd, cd0;
};

// One gather k-slot, resolved on the host (32 B): L(row, k) of the tile's
// r-th marked row is Lx[roff + popcount(rmask below r)], L(col, k) of its
// c-th marked column Lx[roff + cdelta + popcount(cmask below c)], d_k = dg[dk].
// Padding slots: masks 0.
struct SlotRec {
    uint64_t rmask, cmask;
    int64_t roff;
    int cdelta, dk;
};

constexpr int kMaxChunkSlots = 512;   // largest split-K chunk of the gather
constexpr int kVisitLevels = 256;     // trees at least this deep gather early slots as visits (kkt_device.hip)
constexpr int kVisitSlots = 64;       // slots per visit
constexpr int kFlatMaxChunks = 2048;
constexpr int kQuadMaxUnits = 512;    // quadrant gathers for deep-tree launches of at most this many units / visits

struct KktPlan {
    int m = 0, n = 0, T = 0;
    std::vector<int> perm, iperm;

    // supernodal panels: supernode s owns columns [col0[s], col0[s+1]),
    // its below-block rows are rows[rowptr[s] .. rowptr[s+1]) (sorted, new
    // indices).  Panel = h x nc column-major, ld = h = nc + |R_s|; rows of
    // the panel are the nc block rows followed by R_s.
    int nsup = 0;
    std::vector<int> col0;          // [nsup+1]
    std::vector<int> rowptr;        // [nsup+1]
    std::vector<int> rows;          // concatenated R_s
    std::vector<int64_t> off;       // [nsup+1] offset of panel s in Lx
    std::vector<int> parent;        // supernodal etree
    std::vector<int> sup_of;        // [T] column -> supernode
    std::vector<int> level;         // [nsup]
    int nlevels = 0;
    std::vector<int> level_ptr;     // [nlevels+1]
    std::vector<int> level_sups;    // supernodes, grouped by level

    // left-looking update pairs, grouped by target supernode:
    //   for target s, pairs upd_ptr[s]..upd_ptr[s+1]; source d = upd_src[p];
    //   rows R_d[upd_r0[p] .. |R_d|) land in s, the first upd_r1[p]-upd_r0[p]
    //   of them inside s's columns; their panel rows are rel[relptr[p] + i].
    std::vector<int> upd_ptr, upd_src, upd_r0, upd_r1;
    std::vector<int64_t> relptr;
    std::vector<int> rel;

    // assembly: A nonzero k (CSC order) -> slot in Lx; node v (new) -> diagonal slot
    std::vector<int64_t> amap;
    // Q nonzero k (CSC order) -> its slot in Lx where its new row is below its
    // new column, -1 where the symmetric twin carries it, -2 on the diagonal
    std::vector<int64_t> qmap;
    std::vector<int64_t> dslot;     // [T]
    std::vector<int> dsign;         // [T] -1 for y-nodes, +1 for x-nodes (new index)
    int64_t lx_size = 0;

    // dense tail: columns [tail_c0, T) form a full lower triangle (the
    // reference's dense window); stored as an nt x nt column-major block at
    // Lx + off_tail and factored right-looking in 64-column blocks.
    int tail_c0 = 0, nt = 0, ntb = 0;
    int64_t off_tail = 0;
    std::vector<int> tail_r0;          // per sparse panel: first R_s index inside the tail
    std::vector<int> tail_task_ptr;    // per tile (bi*(bi+1)/2 + bj)
    std::vector<TailTask> tail_tasks;
    double flops_tail_update = 0.0, bytes_tail_update = 0.0, flops_tail_factor = 0.0;

    // GPU work decomposition (filled by build_kkt_plan)
    //  factor units: one per (supernode, 64-row tile of its panel), grouped
    //  by level; unit u gathers tasks task_ptr[u]..task_ptr[u+1], each a
    //  slice [task_i0, task_i1) of one update pair's rows.
    std::vector<int> unit_level_ptr;   // [nlevels+1]
    std::vector<int> unit_sup, unit_tile;
    std::vector<int> task_ptr, task_pair, task_i0, task_i1;
    std::vector<TailTask> utasks;      // the same tasks as row/column bit masks
    //  k-slot lists for the MFMA gather: the inner dimension of a unit's
    //  (or tail tile's) update is the concatenation of its tasks' source
    //  columns; slot = (task << 6) | column-in-source, -1 = padding, each
    //  list padded to a multiple of kSlab.
    std::vector<int> kslot, kslot_ptr;            // per factor unit
    std::vector<int> tail_kslot, tail_kslot_ptr;  // per tail tile
    //  forward-solve update lists.  After supernode s is solved, the forward
    //  sweep stores y_s = L21_s z_s in ybuf[rowptr[s] .. rowptr[s+1]) (one
    //  value per row of R_s); row v later subtracts every y entry aimed at
    //  it: ybuf[yrow_idx[yrow_ptr[v] .. yrow_ptr[v+1])], ascending s.
    std::vector<int> yrow_ptr;         // [T+1]
    std::vector<int> yrow_idx;

    // reference statistics
    int64_t lnz = 0;                // nnz strict lower L (reference pattern)
    double narth = 0.0;
    // narth by the phase doing each column's work (build_kkt_plan): the dense
    // tail's columns, the sparse columns' products beyond their supernode
    // (gather) and the rest (panels); they sum to narth
    double narth_tail = 0.0, narth_gather = 0.0, narth_panel = 0.0;
    int64_t lnz_tail = 0;           // entries of L's pattern in the dense tail's columns
    int pdf = 0, denwin = 0;
    int max_h = 0, max_nc = 0;
    double flops_factor = 0.0;      // sum over updates of 2*ra*rc*nc (approx)
    double flops_update = 0.0;      // exact flops of k_update per factorisation (2 per multiply-add, +1 d-scale)
    double bytes_update = 0.0;      // algorithmic bytes of k_update per factorisation
};

// tail_density < 1: the dense tail starts at the longest suffix of columns
// whose lower triangle is at least that full (1: only the full triangle,
// the reference's dense window)
KktPlan build_kkt_plan(int m, int n, const int* kA, const int* iA, const int* kAt, const int* iAt,
                       int nforced = 0, double tail_density = 1.0, const QPattern* q = nullptr);

}  // namespace ipo
