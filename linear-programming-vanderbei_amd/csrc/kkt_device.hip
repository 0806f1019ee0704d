// kkt_device.hip -- supernodal LDL^T of the quasi-definite KKT matrix on
// gfx950 (see kkt_device.h for the reference mapping).
//
// Data layout in HBM
//   Lx    supernode panels, column-major, panel s = h_s x nc_s (ld = h_s):
//         rows 0..nc-1 are the diagonal block (unit lower L11 after the
//         factor, diagonal slots hold K's diagonal on input), rows nc..h-1
//         are the rows R_s of L21.  One contiguous array, 8-B aligned.
//   dg    D of L D L' (new index order), live = the reference's mark[].
//
// Factor = per elimination-tree level three kernels:
//   k_update  one workgroup per (panel, 64-row tile): left-looking gather
//             of every descendant panel's rank-nc_d update into an LDS tile
//             (fixed task order -> bitwise reproducible), then subtract.
//   k_diag    one workgroup per panel: dense LDL' of the diagonal block in
//             LDS with the dependent-pivot rule of ldlt.c:600-614; L11' is
//             stored in the block's unused upper triangle.
//   k_trsm    one workgroup per 64-row tile: L21 = A21 L11^-T D^-1.
// Solve = per level: forward row-gather + in-wave block substitution +
// diagonal scaling (bottom-up), then column-gather + block back substitution
// (top-down).  Refinement loop as ldlt.c:367-416.
#include <hip/hip_runtime.h>

#include <chrono>
#include <algorithm>
#include <climits>
#include <array>
#include <map>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "dev_common.h"
#include "kkt_device.h"
#include "kkt_kernels.h"
#include "lp_io.h"

namespace ipo {

namespace {

constexpr int TR = kTileRows;     // 64
constexpr int PC = kPanelCols;    // 64
constexpr int NT = 256;           // threads per workgroup

// ---------------------------------------------------------------- assembly
__global__ void __launch_bounds__(NT)
k_assemble_A(int nz, const double* __restrict__ A, const int64_t* __restrict__ amap, double* __restrict__ Lx) {
    const int k = blockIdx.x * NT + threadIdx.x;
    if (k < nz) Lx[amap[k]] = A[k];
}

// -max Q below the diagonal (ldlt.c:253-256: the entry whose new row is below
// its new column; its symmetric twin and the diagonal have qmap < 0)
__global__ void __launch_bounds__(NT)
k_assemble_Q(int nq, const double* __restrict__ Q, const int64_t* __restrict__ qmap, double qmax,
             double* __restrict__ Lx) {
    const int k = blockIdx.x * NT + threadIdx.x;
    if (k < nq && qmap[k] >= 0) Lx[qmap[k]] = -qmax * Q[k];
}

// K's diagonal: -max(E, eps) on y-nodes, +max(D, eps) on x-nodes (ldlt.c:235-236),
// then -max Q_jj on the y-nodes of a Q block (ldlt.c:256); |terms| of each
__global__ void __launch_bounds__(NT)
k_assemble_diag(int T, int m, const int* __restrict__ perm, const double* __restrict__ E,
                const double* __restrict__ D, double eps, const int64_t* __restrict__ dslot,
                double* __restrict__ Lx, int* __restrict__ live, double* __restrict__ dscale, int tail_from,
                int* __restrict__ flags, const double* __restrict__ qdiag, double qmax) {
    const int v = blockIdx.x * NT + threadIdx.x;
    if (v < 4) flags[v] = 0;      // the factorisation's flags (no fill launch of their own)
    if (v >= T) return;
    const int old = perm[v];
    // columns >= tail_from: replicated linking rows of a non-leading shard,
    // whose diagonal enters the summed tail once (from shard 0)
    double a = v >= tail_from ? 0.0 : old < m ? -ref_max(E[old], eps) : ref_max(D[old - m], eps);
    double sc = fabs(a);
    if (qdiag && old < m) {
        const double q = qmax * qdiag[old];
        a = a - q;
        sc = sc + fabs(q);
    }
    Lx[dslot[v]] = a;
    dscale[v] = sc;
    live[v] = 1;
}

// The dense tail's lower block triangle zeroed (column c from the first row
// of its diagonal block on): nothing reads the tail above its diagonal
// blocks (gathers, visits and panels write tiles bi >= bj, the sweeps read
// those and the diagonal blocks' upper slots), so the factorisation's clear
// skips that half of the nt x nt block.  One workgroup per column.
__global__ void __launch_bounds__(NT) k_zero_tail_lower(double* __restrict__ S, int nt) {
    const int c = blockIdx.x;
    double* col = S + (size_t)c * nt;
    for (int r = (c / kPanelCols) * kPanelCols + static_cast<int>(threadIdx.x); r < nt; r += NT) col[r] = 0.0;
}

// ------------------------------------------------------- left-looking gather
// out(r, c) -= sum_tasks sum_k L(row, k) * (d_k * L(col, k))     (ldlt.c:572,583)
// for one 64-row x (<= 64)-column output tile.  The inner dimension is the
// concatenation of every task's source columns (the plan's k-slot list);
// kSlab slots at a time are staged in LDS as A(r, k) = L(row(r), k) and
// B(c, k) = d_k L(col(c), k) -- zero where a task's row / column masks
// (TailTask) leave the tile entry untouched -- and multiplied with
// v_mfma_f64_16x16x4_f64, each of the 4 waves owning a 32x32 quarter.
// Slabs are double-buffered: the global loads of slab s+1 are in flight
// while slab s is multiplied.  The fixed slot order makes the sum bitwise
// reproducible.  Entries above the diagonal ((row0 + r) < (col0 + c)) are
// not written; on the diagonal the |terms| are added to dscale.
typedef double double4_t __attribute__((ext_vector_type(4)));
constexpr int KS = kSlab;

// What a k-slot needs (SlotRec, kkt_plan.h: masks, the source column's
// first row-set entry for the tile's rows, the column offset, d_k's index),
// expanded per slot on the host so that one coalesced load per slot stages a
// chunk's records in LDS; the values are then issued without a dependent
// metadata round trip.  ra = L(row, k), rb = d_k * L(col, k) (the reference
// form, ldlt.c:572,583), zero where the task leaves the tile entry untouched.
// The loads are unconditional (an unmarked lane reads the slot's first
// entry) and the mask / d_k product are applied after them (slot_fin): a
// load under a lane branch whose result the branch itself consumes makes
// the compiler wait for it before the branch joins -- one memory round trip
// per slot, measured as ~0.45 us per slot and wave (IPO_HIP_GATHER_STAMPS).
struct SlotLd {
    double a, b, d;
    bool ra, rb;
};
__device__ __forceinline__ SlotLd slot_ld(const SlotRec& m, const double* __restrict__ Lx,
                                          const double* __restrict__ dg, int lane) {
    const uint64_t below = (1ull << lane) - 1ull;
    SlotLd v;
    v.ra = (m.rmask >> lane) & 1ull;
    v.rb = (m.cmask >> lane) & 1ull;
    v.a = Lx[v.ra ? m.roff + __popcll(m.rmask & below) : m.roff];
    v.b = Lx[v.rb ? m.roff + m.cdelta + __popcll(m.cmask & below) : m.roff];
    v.d = dg[m.dk];
    return v;
}
__device__ __forceinline__ void slot_fin(const SlotLd& v, double& ra, double& rb) {
    ra = v.ra ? v.a : 0.0;
    rb = v.rb ? v.d * v.b : 0.0;
}

// Output tile of one gather unit: a 64-row tile of a sparse panel
// (tail < 0) or tile `tail` of the dense tail.
struct GatherTile {
    double* out;
    size_t ld;
    int nrow, ncol, row0, col0;
    double* dscale_col;      // non-null on tiles that hold diagonal entries
};

__device__ __forceinline__ GatherTile unit_tile(const PlanView& p, const TailView& tv, int u, int tail) {
    GatherTile g;
    if (tail < 0) {
        const int s = p.unit_sup[u], t = p.unit_tile[u];
        const int c0 = p.col0[s], nc = p.col0[s + 1] - c0;
        const int h = nc + (p.rowptr[s + 1] - p.rowptr[s]);
        const int rbase = t * TR;
        g.out = p.Lx + p.off[s] + rbase;
        g.ld = h;
        g.nrow = min(TR, h - rbase);
        g.ncol = nc;
        g.row0 = rbase;
        g.col0 = 0;
        g.dscale_col = t == 0 ? p.dscale + c0 : nullptr;
    } else {
        int bi = 0;
        while ((bi + 1) * (bi + 2) / 2 <= u) bi++;
        const int bj = u - bi * (bi + 1) / 2;
        g.out = tv.S + bi * TR + (size_t)(bj * TR) * tv.nt;
        g.ld = tv.nt;
        g.nrow = min(TR, tv.nt - bi * TR);
        g.ncol = min(TR, tv.nt - bj * TR);
        g.row0 = bi * TR;
        g.col0 = bj * TR;
        g.dscale_col = bi == bj ? p.dscale + tv.tc + bj * TR : nullptr;
    }
    return g;
}

// MFMA accumulation of slots [kb, ke) into this thread's 16 tile entries
// (acc[a][b][i] = entry (wr + 16a + (lane>>4) + 4i, wc + 16b + (lane&15)))
// and, for lanes on a diagonal entry, the |terms| of that entry (dabs).
// Pipeline: the slot values of slab sb + 1 are issued while slab sb is
// multiplied, the wave-uniform records of the slab after that one step
// ahead of its values (scalar loads, no LDS), LDS double-buffered.  (Deeper
// register rings, fragment skipping and a 4-waves-per-SIMD build were
// measured slower in round 2 and are gone: DESIGN.md section 6.)
__device__ void gather_acc(const PlanView& p, const SlotRec* __restrict__ recs, int kb, int ke, int dcol,
                           bool has_diag, double4_t (&acc)[2][2], double& dabs) {
    __shared__ double As[2][TR][KS + 1];
    __shared__ double Bs[2][TR][KS + 1];
    const int tid = threadIdx.x;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
    const int wr = (wv & 1) * 32, wc = (wv >> 1) * 32;
    const int li = lane & 15, lk = lane >> 4;
#pragma unroll
    for (int a = 0; a < 2; a++)
#pragma unroll
        for (int b = 0; b < 2; b++) acc[a][b] = (double4_t){0.0, 0.0, 0.0, 0.0};
    dabs = 0.0;
    const int nk = ke - kb, nslab = nk / KS;
    double ra[KS / 4], rb[KS / 4];
    const double* __restrict__ Lx = p.Lx;
    const double* __restrict__ dg = p.dg;
    const SlotRec* __restrict__ wrec = recs + kb + wv * (KS / 4);
    SlotRec mn[KS / 4];
    auto fetch = [&](int slab) {
#pragma unroll
        for (int j = 0; j < KS / 4; j++) mn[j] = wrec[slab * KS + j];
    };
    auto issue = [&]() {
        SlotLd v[KS / 4];
#pragma unroll
        for (int j = 0; j < KS / 4; j++) v[j] = slot_ld(mn[j], Lx, dg, lane);
#pragma unroll
        for (int j = 0; j < KS / 4; j++) slot_fin(v[j], ra[j], rb[j]);
    };
    if (nslab > 0) { fetch(0); issue(); }
    if (1 < nslab) fetch(1);
#pragma unroll
    for (int j = 0; j < KS / 4; j++) { As[0][lane][wv * (KS / 4) + j] = ra[j]; Bs[0][lane][wv * (KS / 4) + j] = rb[j]; }
    __syncthreads();
    for (int sb = 0; sb < nslab; sb++) {
        const int cur = sb & 1;
        if (sb + 1 < nslab) {
            issue();
            if (sb + 2 < nslab) fetch(sb + 2);
        }
#pragma unroll
        for (int kk = 0; kk < KS; kk += 4) {
            double av[2], bv[2];
#pragma unroll
            for (int a = 0; a < 2; a++) av[a] = As[cur][wr + a * 16 + li][kk + lk];
#pragma unroll
            for (int b = 0; b < 2; b++) bv[b] = Bs[cur][wc + b * 16 + li][kk + lk];
#pragma unroll
            for (int a = 0; a < 2; a++)
#pragma unroll
                for (int b = 0; b < 2; b++)
                    acc[a][b] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[a], bv[b], acc[a][b], 0, 0, 0);
        }
        if (has_diag) {
#pragma unroll
            for (int j = 0; j < KS / 4; j++) {
                const int k = wv * (KS / 4) + j;
                dabs += fabs(As[cur][lane][k] * Bs[cur][dcol][k]);
            }
        }
        if (sb + 1 < nslab) {
#pragma unroll
            for (int j = 0; j < KS / 4; j++) {
                As[cur ^ 1][lane][wv * (KS / 4) + j] = ra[j];
                Bs[cur ^ 1][lane][wv * (KS / 4) + j] = rb[j];
            }
        }
        __syncthreads();
    }
}

// The tile's current values (read before the first store: the compiler
// cannot tell that the 16 entries are distinct and would otherwise
// serialise 16 round trips)
__device__ __forceinline__ void gather_old(const GatherTile& g, double (&old)[2][2][4]) {
    const int tid = threadIdx.x, wv = tid >> 6, lane = tid & 63;
    const int wr = (wv & 1) * 32, wc = (wv >> 1) * 32;
#pragma unroll
    for (int a = 0; a < 2; a++)
#pragma unroll
        for (int b = 0; b < 2; b++)
#pragma unroll
            for (int i = 0; i < 4; i++) {
                const int rr = wr + a * 16 + (lane >> 4) + 4 * i;
                const int cc = wc + b * 16 + (lane & 15);
                const bool ok = rr < g.nrow && cc < g.ncol && g.row0 + rr >= g.col0 + cc;
                old[a][b][i] = ok ? g.out[rr + (size_t)cc * g.ld] : 0.0;
            }
}

// out = old - acc on the tile's lower part; dscale += the four waves' dabs in order
__device__ void gather_put(const GatherTile& g, const double (&old)[2][2][4], const double4_t (&acc)[2][2], double dabs,
                           bool has_diag, int dcol) {
    __shared__ double dred[4][TR];
    const int tid = threadIdx.x, wv = tid >> 6, lane = tid & 63;
    const int wr = (wv & 1) * 32, wc = (wv >> 1) * 32;
#pragma unroll
    for (int a = 0; a < 2; a++)
#pragma unroll
        for (int b = 0; b < 2; b++)
#pragma unroll
            for (int i = 0; i < 4; i++) {
                const int rr = wr + a * 16 + (lane >> 4) + 4 * i;
                const int cc = wc + b * 16 + (lane & 15);
                if (rr >= g.nrow || cc >= g.ncol || g.row0 + rr < g.col0 + cc) continue;
                g.out[rr + (size_t)cc * g.ld] = old[a][b][i] - acc[a][b][i];
            }
    if (g.dscale_col) {
        dred[wv][lane] = dabs;
        __syncthreads();
        if (wv == 0 && has_diag) g.dscale_col[dcol] += ((dred[0][lane] + dred[1][lane]) + dred[2][lane]) + dred[3][lane];
    }
}

__device__ __forceinline__ void gather_store(const GatherTile& g, const double4_t (&acc)[2][2], double dabs, bool has_diag,
                                             int dcol) {
    double old[2][2][4];
    gather_old(g, old);
    gather_put(g, old, acc, dabs, has_diag, dcol);
}

// Sum the np partial tiles of a split unit (slots p0.., thread-fragment
// order) in chunk order: acc = ((0 + P_0) + P_1) + ...  The partials were
// handed off inside this launch (sc1 loads, bypassing the CU's L1).
template <int SG>
__device__ __forceinline__ void split_sum(const double* __restrict__ partial, int p0, int np, double4_t (&acc)[2][2],
                                          double& dabs) {
    const int tid = threadIdx.x;
#pragma unroll
    for (int a = 0; a < 2; a++)
#pragma unroll
        for (int b = 0; b < 2; b++) acc[a][b] = (double4_t){0.0, 0.0, 0.0, 0.0};
    dabs = 0.0;
    // SG partials' loads in flight at once (each a dependent round trip
    // otherwise: 12 partials took 12 of them), added in chunk order
    for (int j0 = 0; j0 < np; j0 += SG) {
        double v[SG][17];
#pragma unroll
        for (int g = 0; g < SG; g++) {
            const double* src = partial + (size_t)(p0 + min(j0 + g, np - 1)) * (TR * TR + 4 * TR);
#pragma unroll
            for (int e = 0; e < 16; e++) v[g][e] = sc1_load(src + e * NT + tid);
            v[g][16] = sc1_load(src + TR * TR + tid);
        }
#pragma unroll
        for (int g = 0; g < SG; g++) {
            if (j0 + g >= np) break;
#pragma unroll
            for (int a = 0; a < 2; a++)
#pragma unroll
                for (int b = 0; b < 2; b++)
#pragma unroll
                    for (int i = 0; i < 4; i++) acc[a][b][i] += v[g][(a * 2 + b) * 4 + i];
            dabs += v[g][16];
        }
    }
}

// Gather chunks: chunk c covers slots [ck_b[c], ck_e[c]) of unit ck_u[c].
// ck_part[c] < 0: the unit's only chunk, subtract directly.  Else the chunks
// of split unit q = ck_q[c] store their partial tiles (thread-fragment
// order) and dabs write-through (sc1) at partial slot ck_part[c], drain them,
// and one lane adds to the unit's arrival counter; the chunk whose add comes
// last sums all partials in chunk order (sc1 loads) and stores the tile
// (MI355X_MICROARCH.md hand-off table row 1: last arriver told by its own
// add's return value).  It resets the counter for the next factorisation.
// tail >= 0: units are dense-tail tiles.
// OCC: workgroups per CU the registers are sized for (1: the compiler's
// choice, 160 VGPRs = 3 per CU; 4 (default for SG = 1): 116 VGPRs, no
// spills -- one more workgroup's slab loads in flight per CU: dfl001's
// gather 51.1 -> 47.9 ms per solve, configs[3] / [4] +3 / +7 %;
// IPO_HIP_UPDATE_OCC=1 restores the compiler's choice)
template <int SG, int OCC>
__global__ void __launch_bounds__(NT, OCC)
k_update(PlanView p, TailView tv, int tail, const SlotRec* __restrict__ recs,
         const int* __restrict__ ck_u, const int* __restrict__ ck_b, const int* __restrict__ ck_e,
         const int* __restrict__ ck_part, int c0, double* __restrict__ partial,
         const int* __restrict__ ck_q, const int* __restrict__ sp_p0, const int* __restrict__ sp_n,
         int* __restrict__ split_cnt) {
    const int c = c0 + (p.xcd > 0 && static_cast<int>(gridDim.x) >= p.xcd ? xcd_chunk(blockIdx.x, gridDim.x)
                                                                     : static_cast<int>(blockIdx.x));
    const int u = ck_u[c], kb = ck_b[c], ke = ck_e[c], pi = ck_part[c];
    const GatherTile g = unit_tile(p, tv, u, tail);
    const int lane = threadIdx.x & 63;
    const int dcol = g.row0 + lane - g.col0;
    const bool has_diag = g.dscale_col && dcol >= 0 && dcol < g.ncol && lane < g.nrow;
    double4_t acc[2][2];
    double dabs;
    gather_acc(p, recs, kb, ke, dcol, has_diag, acc, dabs);
    if (pi < 0) {
        gather_store(g, acc, dabs, has_diag, dcol);
        return;
    }
    double* dst = partial + (size_t)pi * (TR * TR + 4 * TR);
    const int tid = threadIdx.x;
#pragma unroll
    for (int a = 0; a < 2; a++)
#pragma unroll
        for (int b = 0; b < 2; b++)
#pragma unroll
            for (int i = 0; i < 4; i++) sc1_store(dst + ((a * 2 + b) * 4 + i) * NT + tid, acc[a][b][i]);
    sc1_store(dst + TR * TR + tid, dabs);
    __shared__ int last;
    const int q = ck_q[c];
    const int np = sp_n[q];
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
        const int prev = __hip_atomic_fetch_add(split_cnt + q, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        last = prev == np - 1;
        if (prev == np - 1) __hip_atomic_store(split_cnt + q, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    if (!last) return;
    split_sum<SG>(partial, sp_p0[q], np, acc, dabs);
    gather_store(g, acc, dabs, has_diag, dcol);
}

// Flat gather for latency-bound launches (the level chain of deep trees,
// where a launch holds one small gather per unit and nothing hides the
// pipelined form's memory round trip per 16-slot slab -- 2.5 us each,
// measured): up to 64 slots per round, their records staged in LDS by one
// coalesced load, then every value of the round issued at once (32 loads
// in flight per lane), one barrier, the MFMA steps.  Slot k of a round is
// staged by the wave gather_acc gives it (k mod 16 in [4 wv, 4 wv + 4)) and
// the MFMA steps and |terms| run in gather_acc's order: bitwise the same.
constexpr int FK = 64;
#define GST(k) do { if (st && threadIdx.x == 0) st[k] = __builtin_amdgcn_s_memrealtime(); } while (0)
__device__ void gather_acc_flat(const PlanView& p, const SlotRec* __restrict__ recs, int kb, int ke, int dcol,
                                bool has_diag, double4_t (&acc)[2][2], double& dabs, long long* st = nullptr) {
    __shared__ double As[TR][FK + 1];
    __shared__ double Bs[TR][FK + 1];
    __shared__ SlotRec rl[FK];
    const int tid = threadIdx.x;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
    const int wr = (wv & 1) * 32, wc = (wv >> 1) * 32;
    const int li = lane & 15, lk = lane >> 4;
#pragma unroll
    for (int a = 0; a < 2; a++)
#pragma unroll
        for (int b = 0; b < 2; b++) acc[a][b] = (double4_t){0.0, 0.0, 0.0, 0.0};
    dabs = 0.0;
    for (int k0 = kb; k0 < ke; k0 += FK) {
        const int nk = min(FK, ke - k0), nsl = nk / KS;
        if (tid < nk * 4)
            reinterpret_cast<uint64_t*>(rl)[tid] = reinterpret_cast<const uint64_t*>(recs + k0)[tid];
        __syncthreads();
        if (k0 == kb) GST(1);
        double ra[FK / 16 * 4], rb[FK / 16 * 4];
        SlotLd v[FK / 16 * 4];
#pragma unroll
        for (int sb = 0; sb < FK / KS; sb++)
#pragma unroll
            for (int j = 0; j < 4; j++)
                if (sb < nsl) v[sb * 4 + j] = slot_ld(rl[sb * KS + wv * 4 + j], p.Lx, p.dg, lane);
#pragma unroll
        for (int sb = 0; sb < FK / KS; sb++)
#pragma unroll
            for (int j = 0; j < 4; j++) {
                ra[sb * 4 + j] = 0.0;
                rb[sb * 4 + j] = 0.0;
                if (sb < nsl) slot_fin(v[sb * 4 + j], ra[sb * 4 + j], rb[sb * 4 + j]);
            }
#pragma unroll
        for (int sb = 0; sb < FK / KS; sb++)
#pragma unroll
            for (int j = 0; j < 4; j++)
                if (sb < nsl) {
                    As[lane][sb * KS + wv * 4 + j] = ra[sb * 4 + j];
                    Bs[lane][sb * KS + wv * 4 + j] = rb[sb * 4 + j];
                }
        __syncthreads();
        if (k0 == kb) GST(2);
        for (int kk = 0; kk < nk; kk += 4) {
            double av[2], bv[2];
#pragma unroll
            for (int a = 0; a < 2; a++) av[a] = As[wr + a * 16 + li][kk + lk];
#pragma unroll
            for (int b = 0; b < 2; b++) bv[b] = Bs[wc + b * 16 + li][kk + lk];
#pragma unroll
            for (int a = 0; a < 2; a++)
#pragma unroll
                for (int b = 0; b < 2; b++)
                    acc[a][b] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[a], bv[b], acc[a][b], 0, 0, 0);
        }
        if (has_diag) {
            for (int sb = 0; sb < nsl; sb++)
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    const int k = sb * KS + wv * 4 + j;
                    dabs += fabs(As[lane][k] * Bs[dcol][k]);
                }
        }
        __syncthreads();
        if (k0 == kb) GST(3);
    }
}

// k_update with the flat gather; an unsplit chunk reads its tile's old
// values before the gather (no workgroup writes a tile its launch reads:
// one chunk per unsplit unit, split units stored by their last chunk only)
template <int SG>
__global__ void __launch_bounds__(NT)
k_update_flat(PlanView p, TailView tv, int tail, const SlotRec* __restrict__ recs,
              const int* __restrict__ ck_u, const int* __restrict__ ck_b, const int* __restrict__ ck_e,
              const int* __restrict__ ck_part, int c0, double* __restrict__ partial,
              const int* __restrict__ ck_q, const int* __restrict__ sp_p0, const int* __restrict__ sp_n,
              int* __restrict__ split_cnt, long long* __restrict__ stamps) {
    long long* st = stamps && blockIdx.x < 1024 ? stamps + blockIdx.x * 8 : nullptr;
    GST(0);
    const int c = c0 + blockIdx.x;
    const int u = ck_u[c], kb = ck_b[c], ke = ck_e[c], pi = ck_part[c];
    const GatherTile g = unit_tile(p, tv, u, tail);
    const int lane = threadIdx.x & 63;
    const int dcol = g.row0 + lane - g.col0;
    const bool has_diag = g.dscale_col && dcol >= 0 && dcol < g.ncol && lane < g.nrow;
    double4_t acc[2][2];
    double dabs;
    if (st && threadIdx.x == 0) st[6] = ke - kb;
    if (pi < 0) {
        double old[2][2][4];
        gather_old(g, old);
        gather_acc_flat(p, recs, kb, ke, dcol, has_diag, acc, dabs, st);
        GST(4);
        gather_put(g, old, acc, dabs, has_diag, dcol);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        GST(5);
        return;
    }
    gather_acc_flat(p, recs, kb, ke, dcol, has_diag, acc, dabs, st);
    double* dst = partial + (size_t)pi * (TR * TR + 4 * TR);
    const int tid = threadIdx.x;
#pragma unroll
    for (int a = 0; a < 2; a++)
#pragma unroll
        for (int b = 0; b < 2; b++)
#pragma unroll
            for (int i = 0; i < 4; i++) sc1_store(dst + ((a * 2 + b) * 4 + i) * NT + tid, acc[a][b][i]);
    sc1_store(dst + TR * TR + tid, dabs);
    __shared__ int last;
    const int q = ck_q[c];
    const int np = sp_n[q];
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
        const int prev = __hip_atomic_fetch_add(split_cnt + q, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        last = prev == np - 1;
        if (prev == np - 1) __hip_atomic_store(split_cnt + q, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    if (!last) return;
    split_sum<SG>(partial, sp_p0[q], np, acc, dabs);
    gather_store(g, acc, dabs, has_diag, dcol);
}

// Quadrant gather for the level chain of deep trees.  Measured there
// (IPO_HIP_GATHER_STAMPS): a 64-slot flat round spends ~7.5 us staging its
// values -- the CU's outstanding misses, ~8 cache lines per slot from as
// many source columns -- not in the MFMA steps.  Here a unit's tile is
// gathered by up to four workgroups, one per 32 x 32 quadrant (the ones
// outside the tile or above the diagonal are not launched), each fetching
// only its 32 rows and 32 columns of every slot (lanes 0-31 the rows, 32-63
// the columns: one load per slot); wave w owns the quadrant's 16 x 16
// fragment (w & 1, w >> 1).  Every tile entry sees gather_acc's MFMA steps
// in its k order, and the diagonal's |terms| are summed in its four wave
// partials, so the factor is bitwise k_update's with one chunk per unit.
// ck_part holds -1 - quadrant (no split K: a quadrant loops over rounds).
__global__ void __launch_bounds__(NT)
k_update_quad(PlanView p, TailView tv, const SlotRec* __restrict__ recs, const int* __restrict__ ck_u,
              const int* __restrict__ ck_b, const int* __restrict__ ck_e, const int* __restrict__ ck_part, int c0,
              long long* __restrict__ stamps) {
    __shared__ double As[32][FK + 1];
    __shared__ double Bs[32][FK + 1];
    __shared__ SlotRec rl[FK];
    long long* st = stamps && blockIdx.x < 1024 ? stamps + blockIdx.x * 8 : nullptr;
    GST(0);
    const int c = c0 + blockIdx.x;
    const int u = ck_u[c], kb = ck_b[c], ke = ck_e[c], q = -1 - ck_part[c];
    const int qr = 32 * (q & 1), qc = 32 * (q >> 1);
    const GatherTile g = unit_tile(p, tv, u, -1);
    const int tid = threadIdx.x;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
    const int fr = 16 * (wv & 1), fc = 16 * (wv >> 1);      // the wave's fragment inside the quadrant
    const int li = lane & 15, lk = lane >> 4;
    // the tile's old values of this lane's 4 fragment entries, before the gather
    double old[4];
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const int rr = qr + fr + lk + 4 * i, cc = qc + fc + li;
        const bool ok = rr < g.nrow && cc < g.ncol && g.row0 + rr >= g.col0 + cc;
        old[i] = ok ? g.out[rr + (size_t)cc * g.ld] : 0.0;
    }
    // diagonal quadrant of a tile with diagonal entries: wave 0's lanes < 32
    // keep the four wave partials of row qr + lane's |terms|
    const bool dq = g.dscale_col && qr == qc;
    const int drow = qr + (lane & 31), dcol = g.row0 + drow - g.col0;
    const bool has_diag = dq && wv == 0 && lane < 32 && dcol >= 0 && dcol < g.ncol && drow < g.nrow;
    double dp[4] = {0.0, 0.0, 0.0, 0.0};
    double4_t acc = (double4_t){0.0, 0.0, 0.0, 0.0};
    const int half = lane >> 5, idx = lane & 31;
    const uint64_t bl = (1ull << ((half ? qc : qr) + idx)) - 1ull;
    const int bit = (half ? qc : qr) + idx;
    for (int k0 = kb; k0 < ke; k0 += FK) {
        const int nk = min(FK, ke - k0);
        if (tid < nk * 4)
            reinterpret_cast<uint64_t*>(rl)[tid] = reinterpret_cast<const uint64_t*>(recs + k0)[tid];
        __syncthreads();
        if (k0 == kb) GST(1);
        // wave w stages slots w, w + 4, ... (16 per 64-slot round, one load each)
        // every load issued before any is used (unconditional, clamped to the
        // slot's first entry; see slot_ld)
        double v[FK / 4], dv[FK / 4];
        bool on[FK / 4];
#pragma unroll
        for (int j = 0; j < FK / 4; j++) {
            const int k = min(wv + 4 * j, nk - 1);
            const SlotRec m = rl[k];
            const uint64_t mk = half ? m.cmask : m.rmask;
            on[j] = wv + 4 * j < nk && ((mk >> bit) & 1ull);
            v[j] = p.Lx[on[j] ? m.roff + (half ? m.cdelta : 0) + __popcll(mk & bl) : m.roff];
            dv[j] = p.dg[m.dk];
        }
#pragma unroll
        for (int j = 0; j < FK / 4; j++) v[j] = on[j] ? (half ? dv[j] * v[j] : v[j]) : 0.0;
#pragma unroll
        for (int j = 0; j < FK / 4; j++) {
            const int k = wv + 4 * j;
            if (k < nk) {
                if (half) Bs[idx][k] = v[j];
                else As[idx][k] = v[j];
            }
        }
        __syncthreads();
        if (k0 == kb) GST(2);
        for (int kk = 0; kk < nk; kk += 4)
            acc = __builtin_amdgcn_mfma_f64_16x16x4f64(As[fr + li][kk + lk], Bs[fc + li][kk + lk], acc, 0, 0, 0);
        if (has_diag) {
            // gather_acc's wave partials: wave w's slots k % 16 in [4w, 4w + 4)
            for (int sb = 0; sb < nk / KS; sb++)
#pragma unroll
                for (int w = 0; w < 4; w++)
#pragma unroll
                    for (int j = 0; j < 4; j++) {
                        const int k = sb * KS + w * 4 + j;
                        dp[w] += fabs(As[idx][k] * Bs[idx][k]);
                    }
        }
        __syncthreads();
        if (k0 == kb) GST(3);
    }
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const int rr = qr + fr + lk + 4 * i, cc = qc + fc + li;
        if (rr < g.nrow && cc < g.ncol && g.row0 + rr >= g.col0 + cc) g.out[rr + (size_t)cc * g.ld] = old[i] - acc[i];
    }
    if (has_diag) g.dscale_col[dcol] += ((dp[0] + dp[1]) + dp[2]) + dp[3];
    if (st) { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); GST(5); }
}

// ------------------------------------------------- diagonal block LDL'
// Dense LDL' of an nc x nc diagonal block (nc <= 64) of a panel with leading
// dimension ld and h rows (rows nc..h-1 lie below the block); c0 is the
// block's first global column.  Reads the block's lower triangle, factors it
// right-looking in LDS with the dependent-pivot rule of ldlt.c:600-614 and
// the reference's update form l_r * (l_c * d), and stores L11' in the
// block's UPPER triangle (the lower one keeps the input), D in dg, mark in
// live.  One 256-thread workgroup.
// ======================================================== dense tail
// S = Lx + off_tail, nt x nt column-major (ld = nt), columns tail_c0.. .
// (TailView is declared in kkt_device.h)



// Trailing update S(bi, bj) -= L(bi, kb) * W(bj, kb)'  for bi >= bj > kb,
// with v_mfma_f64_16x16x4_f64: 4 waves, each a 32x32 quarter (2x2 MFMA tiles).

__global__ void __launch_bounds__(NT)
k_tail_syrk(PlanView p, TailView tv, int kb) {
    __shared__ double As[TR][PC + 1];    // L rows of block bi   [row][k]
    __shared__ double Bs[TR][PC + 1];    // W rows of block bj   [row][k]
    const int nb = tv.ntb - kb - 1;      // trailing blocks
    const int tile = blockIdx.x;
    int ti = 0;
    while ((ti + 1) * (ti + 2) / 2 <= tile) ti++;
    const int tj = tile - ti * (ti + 1) / 2;
    if (ti >= nb) return;
    const int bi = kb + 1 + ti, bj = kb + 1 + tj;
    const int k0 = kb * PC;
    const int nc = min(PC, tv.nt - k0);
    const int nt = tv.nt;
    const int tid = threadIdx.x;
    const double* Lcol = tv.S + (size_t)k0 * nt;      // column k0 of S
    // W rows are stored relative to the block column: W[(row - k0) + k * nt].
    // All 32 loads of a thread are issued before its first LDS store.
    {
        double va[TR * PC / NT], vb[TR * PC / NT];
#pragma unroll
        for (int u = 0; u < TR * PC / NT; u++) {
            const int idx = tid + u * NT, rr = idx % TR, k = idx / TR;
            const int ra = bi * TR + rr, rb = bj * TR + rr;
            const bool oka = k < nc && ra < nt, okb = k < nc && rb < nt;
            const double x = Lcol[oka ? ra + (size_t)k * nt : 0];
            const double y = tv.W[okb ? (rb - k0) + (size_t)k * nt : 0];
            va[u] = oka ? x : 0.0;
            vb[u] = okb ? y : 0.0;
        }
#pragma unroll
        for (int u = 0; u < TR * PC / NT; u++) {
            const int idx = tid + u * NT;
            As[idx % TR][idx / TR] = va[u];
            Bs[idx % TR][idx / TR] = vb[u];
        }
    }
    __syncthreads();
    const int wv = tid >> 6, lane = tid & 63;
    const int wr = (wv & 1) * 32, wc = (wv >> 1) * 32;
    double4_t acc[2][2];
    for (int a = 0; a < 2; a++)
        for (int b = 0; b < 2; b++) acc[a][b] = (double4_t){0.0, 0.0, 0.0, 0.0};
    const int li = lane & 15, lk = lane >> 4;
    for (int kk = 0; kk < PC; kk += 4) {
        double av[2], bv[2];
        for (int a = 0; a < 2; a++) av[a] = As[wr + a * 16 + li][kk + lk];
        for (int b = 0; b < 2; b++) bv[b] = Bs[wc + b * 16 + li][kk + lk];
        for (int a = 0; a < 2; a++)
            for (int b = 0; b < 2; b++) acc[a][b] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[a], bv[b], acc[a][b], 0, 0, 0);
    }
    const bool diag_tile = bi == bj;
    double old[2][2][4];      // all loads before the first store (see gather_store)
#pragma unroll
    for (int a = 0; a < 2; a++)
#pragma unroll
        for (int b = 0; b < 2; b++)
#pragma unroll
            for (int i = 0; i < 4; i++) {
                const int rr = wr + a * 16 + (lane >> 4) + 4 * i;
                const int cc = wc + b * 16 + (lane & 15);
                const int rg = bi * TR + rr, cg = bj * TR + cc;
                const bool ok = rg < nt && cg < nt && !(diag_tile && cc > rr);
                old[a][b][i] = ok ? tv.S[rg + (size_t)cg * nt] : 0.0;
            }
#pragma unroll
    for (int a = 0; a < 2; a++)
#pragma unroll
        for (int b = 0; b < 2; b++)
#pragma unroll
            for (int i = 0; i < 4; i++) {
                const int rr = wr + a * 16 + (lane >> 4) + 4 * i;
                const int cc = wc + b * 16 + (lane & 15);
                const int rg = bi * TR + rr, cg = bj * TR + cc;
                if (rg >= nt || cg >= nt || (diag_tile && cc > rr)) continue;
                tv.S[rg + (size_t)cg * nt] = old[a][b][i] - acc[a][b][i];
            }
    if (diag_tile && tid < TR) {           // |terms| of the diagonal for the zero-pivot test
        const int rg = bi * TR + tid;
        if (rg < nt) {
            double as = 0.0;
            for (int k = 0; k < nc; k++) as += fabs(As[tid][k] * Bs[tid][k]);
            p.dscale[tv.tc + rg] += as;
        }
    }
}

// -------------------------------------------------------------- solves
// Every sweep kernel handles R right-hand sides at once (R = 1 or 2; hsd and
// hsdls solve two systems with the same factor per iteration, hsd.c:218-224):
// vector r of a family lives at base + r * stride.  The dependency chain of a
// sweep is the same for both, so the second vector rides along almost free.
//
// One wave solves a unit-lower nc x nc block in place: lane r holds z_r on
// entry and on exit; Ls[r][j] = L(r, j) (zero for j >= r).  Lane r keeps its
// row of L in registers; z_j is broadcast by v_readlane.  A dropped column j
// (mark false) keeps z_j when |z_j| > eps (and the system is flagged
// inconsistent), else z_j = 0 -- ldlt.c:446-470.
// Fast form when every column of the block is live (the common case):
// NS = 16, 32 or 64 >= nc steps with no per-step branch (a step j >= nc
// subtracts L(r, j) z_j = 0 * 0 and changes nothing), so the chain is one
// basic block the compiler can schedule; the same mul-then-subtract per
// entry as the general form (bitwise the same result).
// The lane index, opaque to the optimiser (OPQ solves): a solve inside a
// loop would otherwise have its 64 per-step lane masks hoisted out of the
// loop (128 scalar registers, spilled: the sync-free sweeps, the lead
// sweep).  Outside loops the hoisted masks are cheaper (OPQ = false).
__device__ __forceinline__ int opaque_lane() {
    int lane = threadIdx.x & 63;
    asm volatile("" : "+v"(lane));
    return lane;
}
template <int R, int NS, bool OPQ>
__device__ __forceinline__ void tri_lower_live(double (&zr)[R], const double (*Ls)[PC + 1]) {
    const int lane = OPQ ? opaque_lane() : (int)(threadIdx.x & 63);
    double lr[NS];
#pragma unroll
    for (int j = 0; j < NS; j++) lr[j] = Ls[lane][j];
#pragma unroll
    for (int j = 0; j < NS; j++) {
#pragma unroll
        for (int r = 0; r < R; r++) {
            const double zj = lane_bcast(zr[r], j);
            const double nz = zr[r] - lr[j] * zj;
            zr[r] = lane > j ? nz : zr[r];
        }
    }
}
template <int R, int NS, bool OPQ>
__device__ __forceinline__ void tri_upper_live(double (&zr)[R], const double (*Ls)[PC + 1]) {
    const int lane = OPQ ? opaque_lane() : (int)(threadIdx.x & 63);
    double lc[NS];
#pragma unroll
    for (int j = 0; j < NS; j++) lc[j] = Ls[j][lane];
#pragma unroll
    for (int j = NS - 1; j >= 0; j--) {
#pragma unroll
        for (int r = 0; r < R; r++) {
            const double zj = lane_bcast(zr[r], j);
            const double nz = zr[r] - lc[j] * zj;
            zr[r] = lane < j ? nz : zr[r];
        }
    }
}

template <int R, bool OPQ = false>
__device__ __forceinline__ void tri_lower(double (&zr)[R], const double (*Ls)[PC + 1], const int* lv, int nc,
                                          const double (&eps)[R], int (&bad)[R]) {
    const int lane = OPQ ? opaque_lane() : (int)(threadIdx.x & 63);
    const uint64_t lm = __ballot(lane < nc && lv[lane]);
    if (lm == (nc >= 64 ? ~0ull : (1ull << nc) - 1ull)) {     // every column live (wave-uniform)
        if (nc <= 16) tri_lower_live<R, 16, OPQ>(zr, Ls);
        else if (nc <= 32) tri_lower_live<R, 32, OPQ>(zr, Ls);
        else tri_lower_live<R, 64, OPQ>(zr, Ls);
        return;
    }
    double lr[PC];
#pragma unroll
    for (int j = 0; j < PC; j++) lr[j] = lane < nc ? Ls[lane][j] : 0.0;
#pragma unroll
    for (int j = 0; j < PC; j++) {
        if (j < nc) {
            const bool alive = (lm >> j) & 1ull;
#pragma unroll
            for (int r = 0; r < R; r++) {
                if (!alive && lane == j) {
                    if (fabs(zr[r]) > eps[r]) bad[r] = 1;
                    else zr[r] = 0.0;
                }
                const double zj = lane_bcast(zr[r], j);
                if (alive && lane > j) zr[r] -= lr[j] * zj;
            }
        }
    }
}

// unit-upper (L11') counterpart; Ls[j][r] = L(j, r) (zero for r >= j)
template <int R, bool OPQ = false>
__device__ __forceinline__ void tri_upper(double (&zr)[R], const double (*Ls)[PC + 1], const int* lv, int nc,
                                          const double (&eps)[R], int (&bad)[R]) {
    const int lane = OPQ ? opaque_lane() : (int)(threadIdx.x & 63);
    const uint64_t lm = __ballot(lane < nc && lv[lane]);
    if (lm == (nc >= 64 ? ~0ull : (1ull << nc) - 1ull)) {     // every column live (wave-uniform)
        if (nc <= 16) tri_upper_live<R, 16, OPQ>(zr, Ls);
        else if (nc <= 32) tri_upper_live<R, 32, OPQ>(zr, Ls);
        else tri_upper_live<R, 64, OPQ>(zr, Ls);
        return;
    }
    double lc[PC];
#pragma unroll
    for (int j = 0; j < PC; j++) lc[j] = j < nc ? Ls[j][lane] : 0.0;
#pragma unroll
    for (int j = PC - 1; j >= 0; j--) {
        if (j < nc) {
            const bool alive = (lm >> j) & 1ull;
#pragma unroll
            for (int r = 0; r < R; r++) {
                if (!alive && lane == j) {
                    if (fabs(zr[r]) > eps[r]) bad[r] = 1;
                    else zr[r] = 0.0;
                }
                const double zj = lane_bcast(zr[r], j);
                if (alive && lane < j) zr[r] -= lc[j] * zj;
            }
        }
    }
}

// Column sums of a wave's 16 (x R) per-lane partials without 16 R serial
// chains of cross-lane permutes: each wave writes its partials to LDS
// scratch (rows padded to PC + 1 doubles: conflict-free column writes and
// row reads), then one thread per (right-hand side, column) redoes
// wave_sum's shfl_down tree (v[l] += v[l + o], o = 32 .. 1, result in lane
// 0) on its row -- the same adds in the same order, so bitwise the same.
// Scratch: R * PC * (PC + 1) doubles; a __syncthreads between the two.
template <int R>
__device__ __forceinline__ void colsum_put(double* red, const double (&v)[R][16], int kq, int nq, int lane) {
#pragma unroll
    for (int r = 0; r < R; r++)
#pragma unroll
        for (int q = 0; q < 16; q++)
            if (q < nq) red[(size_t)(r * PC + kq + q) * (PC + 1) + lane] = v[r][q];
}
__device__ __forceinline__ double colsum_tree(const double* red, int r, int c) {
    const double* __restrict__ x = red + (size_t)(r * PC + c) * (PC + 1);
    double s[32];
#pragma unroll
    for (int l = 0; l < 32; l++) s[l] = x[l] + x[l + 32];
#pragma unroll
    for (int o = 16; o > 0; o >>= 1)
#pragma unroll
        for (int l = 0; l < o; l++) s[l] += s[l + o];
    return s[0];
}

template <int R>
__device__ __forceinline__ void flag_bad(const PlanView& p, const int (&bad)[R]) {
#pragma unroll
    for (int r = 0; r < R; r++)
        if (bad[r]) atomicOr(&p.incons[r], 1);
}

template <int R>
__device__ __forceinline__ void load_eps(const double* epsp, double (&eps)[R]) {
#pragma unroll
    for (int r = 0; r < R; r++) eps[r] = epsp[r];
}

// D^{-1} with the dropped-column rule (ldlt.c:473-480)
__device__ __forceinline__ double dscale_rule(const PlanView& p, int v, double zv, double eps, int& bad) {
    if (p.live[v]) return zv / p.dg[v];
    if (fabs(zv) > eps) bad = 1;
    else zv = 0.0;
    return zv;
}

// Stage L11 of a panel (ld = h) from the upper-triangle slot image:
// Ls[r][j] = L(r, j) for j < r, 0 elsewhere.  Each wave issues all its
// loads before the first LDS store (addresses clamped in bounds).
// Waves wv of nw (default: the whole workgroup) share the loads.
__device__ __forceinline__ void stage_l11(const double* panel, size_t ld, int nc, double (*Ls)[PC + 1], int wv,
                                          int nw) {
    const int lane = threadIdx.x & 63;
    for (int r0 = wv; r0 < PC; r0 += 16 * nw) {
        double t[16];
#pragma unroll
        for (int q = 0; q < 16; q++) {
            const int r = r0 + q * nw;
            const bool ok = r < nc && lane < r;
            t[q] = panel[ok ? lane + (size_t)r * ld : 0];
            t[q] = ok ? t[q] : 0.0;
        }
#pragma unroll
        for (int q = 0; q < 16; q++) {
            const int r = r0 + q * nw;
            if (r < PC) Ls[r][lane] = t[q];
        }
    }
}
__device__ __forceinline__ void stage_l11(const double* panel, size_t ld, int nc, double (*Ls)[PC + 1]) {
    stage_l11(panel, ld, nc, Ls, threadIdx.x >> 6, blockDim.x >> 6);
}

// Vector families of a sweep: z (K entries each) and the forward update
// values ybuf (one per row of every R_s).
struct SweepVecs {
    double* z;
    size_t zs;          // stride between right-hand sides
    double* y;
    size_t ys;
};

// Forward, diagonal part of supernode s: subtract the y values of solved
// descendants from its rows, solve L11.  Leaves z_s in zl[r] and in z.
// 4 threads per row; partial sums combined as (p0 + p1) + (p2 + p3).
// per-item wall-clock stamps of the last forward sync-free sweep (developer
// build with -DIPO_SF_STAMPS; dumped by ~KktDevice)
#ifdef IPO_SF_STAMPS
__device__ long long g_sfst[1 << 15][10];
#define SF_STAMP(it, slot) do { if (threadIdx.x == 0 && (it) >= 0 && (it) < (1 << 15)) g_sfst[it][slot] = __builtin_amdgcn_s_memrealtime(); } while (0)
#define SF_NOTE(it, slot, v) do { if (threadIdx.x == 0 && (it) >= 0 && (it) < (1 << 15)) g_sfst[it][slot] = (v); } while (0)
#else
#define SF_STAMP(it, slot) do {} while (0)
#define SF_NOTE(it, slot, v) do {} while (0)
#endif

// sidx != nullptr: the supernode's update-list indices, yrow_idx[yrow_ptr[c0]
// ..], already staged in LDS by the caller (before its hand-off wait), so
// only the value loads remain on the chain -- sixteen in flight per thread.
template <int R, bool SC = false, bool STAGED = false>
__device__ void fwd_diag(const PlanView& p, int s, const int* __restrict__ yrow_ptr, const int* __restrict__ yrow_idx,
                         const SweepVecs& V, const double (&eps)[R], double (*zl)[PC], double (*Ls)[PC + 1], int* lv,
                         const int* sidx = nullptr, int stamp_it = -1, const int* sptr = nullptr,
                         double* zout = nullptr, size_t zos = 0) {
    const int c0 = p.col0[s], nc = p.col0[s + 1] - c0;
    const int h = nc + (p.rowptr[s + 1] - p.rowptr[s]);
    const int tid = threadIdx.x, wv = tid >> 6, lane = tid & 63;
    if (!STAGED) {              // else the caller staged L11 and the marks already
        stage_l11(p.Lx + p.off[s], h, nc, Ls);
        if (tid < nc) lv[tid] = p.live[c0 + tid];
    }
    // P threads per row (P = 256 / nc rounded down to a power of two, 4..64):
    // part q sums the entries q, q + P, ... of the row's list in list order
    // (sixteen loads in flight), then a fixed xor-butterfly combines the P
    // partial sums -- the same order in every kernel that calls this.
    const int P = nc > 32 ? 4 : nc > 16 ? 8 : nc > 8 ? 16 : nc > 4 ? 32 : 64;
    // sptr: the rows' list bounds yrow_ptr[c0 .. c0 + nc], staged in LDS by the caller
    const int ebase = sidx ? (sptr ? sptr[0] : yrow_ptr[c0]) : 0;
    // list index e: the staged LDS copy or the global list (no pointer
    // arithmetic across address spaces)
    auto lidx = [&](int e) { return sidx ? sidx[e - ebase] : yrow_idx[e]; };
    for (int base = 0; base < nc; base += blockDim.x / P) {
        const int k = base + tid / P, part = tid & (P - 1);
        double acc[R];
#pragma unroll
        for (int r = 0; r < R; r++) acc[r] = 0.0;
        if (k < nc) {
            const int v = c0 + k;
            const int e1 = sptr ? sptr[k + 1] : yrow_ptr[v + 1];
            int e = (sptr ? sptr[k] : yrow_ptr[v]) + part;
#ifdef IPO_SF_STAMPS
            if (tid == 0 && stamp_it >= 0) { g_sfst[stamp_it][9] = e1 + e; SF_STAMP(stamp_it, 7); }
#endif
            for (; e + 31 * P < e1; e += 32 * P) {     // 32 loads in flight per right-hand side
                int ix[32];
#pragma unroll
                for (int u = 0; u < 32; u++) ix[u] = lidx(e + u * P);
                double yv[R][32];
#pragma unroll
                for (int r = 0; r < R; r++)
#pragma unroll
                    for (int u = 0; u < 32; u++) yv[r][u] = ld_h<SC>(V.y + r * V.ys + ix[u]);
#pragma unroll
                for (int r = 0; r < R; r++)
#pragma unroll
                    for (int u = 0; u < 32; u++) acc[r] += yv[r][u];
            }
            for (; e + 15 * P < e1; e += 16 * P) {
                int ix[16];
#pragma unroll
                for (int u = 0; u < 16; u++) ix[u] = lidx(e + u * P);
#pragma unroll
                for (int r = 0; r < R; r++) {
                    const double* yb = V.y + r * V.ys;
                    double yv[16];
#pragma unroll
                    for (int u = 0; u < 16; u++) yv[u] = ld_h<SC>(yb + ix[u]);
#pragma unroll
                    for (int u = 0; u < 16; u++) acc[r] += yv[u];
                }
            }
            for (; e + 3 * P < e1; e += 4 * P) {
                const int i0 = lidx(e), i1 = lidx(e + P), i2 = lidx(e + 2 * P), i3 = lidx(e + 3 * P);
#pragma unroll
                for (int r = 0; r < R; r++) {
                    const double* yb = V.y + r * V.ys;
                    const double y0 = ld_h<SC>(yb + i0), y1 = ld_h<SC>(yb + i1), y2 = ld_h<SC>(yb + i2),
                                 y3 = ld_h<SC>(yb + i3);
                    acc[r] += y0;
                    acc[r] += y1;
                    acc[r] += y2;
                    acc[r] += y3;
                }
            }
            for (; e < e1; e += P) {
                const int i0 = lidx(e);
#pragma unroll
                for (int r = 0; r < R; r++) acc[r] += ld_h<SC>(V.y + r * V.ys + i0);
            }
        }
#ifdef IPO_SF_STAMPS
        if (tid == 0 && stamp_it >= 0) { g_sfst[stamp_it][9] += (long long)acc[0]; SF_STAMP(stamp_it, 8); }
#endif
#pragma unroll
        for (int r = 0; r < R; r++) {
            double pr = acc[r];
            for (int o = 1; o < P; o <<= 1) {
                const double ot = __shfl_xor(pr, o, 64);
                pr = (part & o) ? ot + pr : pr + ot;
            }
            if (part == 0 && k < nc) zl[r][k] = V.z[r * V.zs + c0 + k] - pr;
        }
    }
    __syncthreads();
    SF_STAMP(stamp_it, 5);
    if (wv < R) {                 // wave r solves right-hand side r (independent chains)
        const int r = wv;
        int bad[1] = {};
        double zr[1] = {lane < nc ? zl[r][lane] : 0.0};
        const double e1[1] = {r == 0 ? eps[0] : eps[R - 1]};
        tri_lower<1, true>(zr, Ls, lv, nc, e1, bad);
        if (lane < nc) {
            // zout: z_s goes to a mirror instead (the chunk items of one
            // supernode each solve it and must all read its right-hand side)
            if (zout) sc1_store(zout + r * zos + lane, zr[0]);
            else V.z[r * V.zs + c0 + lane] = zr[0];
            zl[r][lane] = zr[0];
        }
        if (bad[0]) atomicOr(&p.incons[r], 1);
    }
    __syncthreads();
}

// Forward, one level of small supernodes per launch, one workgroup each:
// diagonal part, then y_s = L21 z_s for the ancestors (one row per thread).
// D^{-1} is applied at the start of the backward sweep.
template <int R>
__device__ __forceinline__ void forward_body(const PlanView& p, const int* __restrict__ level_sups, int q0,
                                             const int* __restrict__ yrow_ptr, const int* __restrict__ yrow_idx,
                                             const SweepVecs& V, const double* __restrict__ epsp, int bid) {
    __shared__ double zl[R][PC];
    __shared__ double Ls[PC][PC + 1];
    __shared__ int lv[PC];
    double eps[R];
    load_eps<R>(epsp, eps);
    const int s = level_sups[q0 + bid];
    fwd_diag<R>(p, s, yrow_ptr, yrow_idx, V, eps, zl, Ls, lv);
    const int c0 = p.col0[s], nc = p.col0[s + 1] - c0;
    const int hb = p.rowptr[s + 1] - p.rowptr[s], h = nc + hb;
    const double* panel = p.Lx + p.off[s];
    for (int i = threadIdx.x; i < hb; i += NT) {
        const double* __restrict__ row = panel + nc + i;
        double acc[R];
#pragma unroll
        for (int r = 0; r < R; r++) acc[r] = 0.0;
#pragma unroll 8
        for (int k = 0; k < nc; k++) {
            const double l = row[(size_t)k * h];
#pragma unroll
            for (int r = 0; r < R; r++) acc[r] += l * zl[r][k];
        }
#pragma unroll
        for (int r = 0; r < R; r++) V.y[r * V.ys + p.ybase[s] + i] = acc[r];
    }
}

template <int R>
__global__ void __launch_bounds__(NT)
k_forward(PlanView p, const int* __restrict__ level_sups, int q0, const int* __restrict__ yrow_ptr,
          const int* __restrict__ yrow_idx, SweepVecs V, const double* __restrict__ epsp) {
    forward_body<R>(p, level_sups, q0, yrow_ptr, yrow_idx, V, epsp, blockIdx.x);
}

// Single-column supernodes with at most 64 rows below (the bulk of the
// bottom level: one per x-node of a large LP, 10^6 on configs[3]), one wave
// each, four per workgroup -- k_forward / k_backward spend a 256-thread
// workgroup, an L11 staging and two barriers on each.  The same operations
// in the same order as those kernels' nc = 1 case (the update list summed
// by 64 parts, part q taking entries q, q + 64, ... in list order, the
// parts combined by the xor butterfly; the backward products summed by
// wave_sum), so bitwise the same sweep.
template <int R>
__device__ __forceinline__ void fwd_leaf_body(const PlanView& p, const int* __restrict__ sups, int q0, int cnt,
                                              const int* __restrict__ yrow_ptr, const int* __restrict__ yrow_idx,
                                              const SweepVecs& V, const double* __restrict__ epsp, int bid) {
    const int w = bid * (NT / 64) + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (w >= cnt) return;
    const int s = sups[q0 + w];
    const int c0 = p.col0[s], hb = p.rowptr[s + 1] - p.rowptr[s];
    double pr[R];
#pragma unroll
    for (int r = 0; r < R; r++) pr[r] = 0.0;
    for (int e = yrow_ptr[c0] + lane; e < yrow_ptr[c0 + 1]; e += 64) {
        const int ix = yrow_idx[e];
#pragma unroll
        for (int r = 0; r < R; r++) pr[r] += V.y[r * V.ys + ix];
    }
    double z[R];
#pragma unroll
    for (int r = 0; r < R; r++) {
        for (int o = 1; o < 64; o <<= 1) {
            const double ot = __shfl_xor(pr[r], o, 64);
            pr[r] = (lane & o) ? ot + pr[r] : pr[r] + ot;
        }
        z[r] = __shfl(V.z[r * V.zs + c0] - pr[r], 0, 64);
    }
    if (!p.live[c0]) {          // dropped column (ldlt.c:446-470)
        double eps[R];
        load_eps<R>(epsp, eps);
        int bad[R] = {};
#pragma unroll
        for (int r = 0; r < R; r++) {
            if (fabs(z[r]) > eps[r]) bad[r] = 1;
            else z[r] = 0.0;
        }
        if (lane == 0) flag_bad<R>(p, bad);
    }
    if (lane == 0) {
#pragma unroll
        for (int r = 0; r < R; r++) V.z[r * V.zs + c0] = z[r];
    }
    if (lane < hb) {
        const double l = p.Lx[p.off[s] + 1 + lane];
#pragma unroll
        for (int r = 0; r < R; r++) {
            double acc = 0.0;
            acc += l * z[r];
            V.y[r * V.ys + p.ybase[s] + lane] = acc;
        }
    }
}

template <int R>
__global__ void __launch_bounds__(NT)
k_fwd_leaf(PlanView p, const int* __restrict__ sups, int q0, int cnt, const int* __restrict__ yrow_ptr,
           const int* __restrict__ yrow_idx, SweepVecs V, const double* __restrict__ epsp) {
    fwd_leaf_body<R>(p, sups, q0, cnt, yrow_ptr, yrow_idx, V, epsp, blockIdx.x);
}

// One launch per level for a level's leaves and its other supernodes
// (workgroups [0, nlb): four leaves each, fwd_leaf_body; the rest one
// supernode each, forward_body) -- the two launches' work in one launch: the
// solve phase's launches are host-bound (the device idles 4-13 us between
// them), so every launch saved is time saved.
template <int R>
__global__ void __launch_bounds__(NT)
k_fwd_level(PlanView p, const int* __restrict__ sups, int q0, int nl, int nlb, const int* __restrict__ yrow_ptr,
            const int* __restrict__ yrow_idx, SweepVecs V, const double* __restrict__ epsp) {
    if (static_cast<int>(blockIdx.x) < nlb) fwd_leaf_body<R>(p, sups, q0, nl, yrow_ptr, yrow_idx, V, epsp, blockIdx.x);
    else forward_body<R>(p, sups, q0 + nl, yrow_ptr, yrow_idx, V, epsp, blockIdx.x - nlb);
}

template <int R>
__device__ __forceinline__ void bwd_leaf_body(const PlanView& p, const int* __restrict__ sups, int q0, int cnt,
                                              const SweepVecs& V, const double* __restrict__ epsp, int bid) {
    const int w = bid * (NT / 64) + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (w >= cnt) return;
    const int s = sups[q0 + w];
    const int c0 = p.col0[s], hb = p.rowptr[s + 1] - p.rowptr[s];
    double acc[R];
#pragma unroll
    for (int r = 0; r < R; r++) acc[r] = 0.0;
    if (lane < hb) {
        const int ri = p.rows[p.rowptr[s] + lane];
        const double t = p.Lx[p.off[s] + 1 + lane];
#pragma unroll
        for (int r = 0; r < R; r++) acc[r] += t * V.z[r * V.zs + ri];
    }
    double eps[R];
    load_eps<R>(epsp, eps);
    int bad[R] = {};
#pragma unroll
    for (int r = 0; r < R; r++) {
        const double xs = wave_sum(acc[r]);
        if (lane == 0) {
            double zr = dscale_rule(p, c0, V.z[r * V.zs + c0], eps[r], bad[r]) - xs;
            if (!p.live[c0]) {
                if (fabs(zr) > eps[r]) bad[r] = 1;
                else zr = 0.0;
            }
            V.z[r * V.zs + c0] = zr;
        }
    }
    if (lane == 0) flag_bad<R>(p, bad);
}

template <int R>
__global__ void __launch_bounds__(NT)
k_bwd_leaf(PlanView p, const int* __restrict__ sups, int q0, int cnt, SweepVecs V, const double* __restrict__ epsp) {
    bwd_leaf_body<R>(p, sups, q0, cnt, V, epsp, blockIdx.x);
}

// Small leaves (<= 8 rows below, <= 8 update-list entries: the x-node
// leaves of a large LP) eight to a wave, lanes 8q .. 8q + 7 for leaf q.
// k_fwd_leaf's butterfly over 64 lanes, with entry e in lane e, reduces to
// the three in-group stages followed by adds of +0.0 from the empty lanes
// (one `+ 0.0`: further ones change nothing); k_bwd_leaf's wave_sum reaches
// lane 0 through lanes 0-7 the same way (three adds of +0.0, then the
// row-down steps 4, 2, 1).  Bitwise the one-wave kernels.
constexpr int kSmallLeaf = 8;
constexpr int kSmallLeafMinCount = 32768;     // per level, else one wave per leaf

template <int R>
__global__ void __launch_bounds__(NT)
k_fwd_leaf8(PlanView p, const int* __restrict__ sups, int q0, int cnt, const int* __restrict__ yrow_ptr,
            const int* __restrict__ yrow_idx, SweepVecs V, const double* __restrict__ epsp) {
    const int w = (blockIdx.x * NT + threadIdx.x) / kSmallLeaf, lq = threadIdx.x & (kSmallLeaf - 1);
    if (w >= cnt) return;          // whole groups leave together
    const int s = sups[q0 + w];
    const int c0 = p.col0[s], hb = p.rowptr[s + 1] - p.rowptr[s];
    const int e0 = yrow_ptr[c0], e1 = yrow_ptr[c0 + 1];
    double pr[R];
#pragma unroll
    for (int r = 0; r < R; r++) pr[r] = 0.0;
    if (e0 + lq < e1) {
        const int ix = yrow_idx[e0 + lq];
#pragma unroll
        for (int r = 0; r < R; r++) pr[r] += V.y[r * V.ys + ix];
    }
    double z[R];
#pragma unroll
    for (int r = 0; r < R; r++) {
        for (int o = 1; o < kSmallLeaf; o <<= 1) {
            const double ot = __shfl_xor(pr[r], o, kSmallLeaf);
            pr[r] = (lq & o) ? ot + pr[r] : pr[r] + ot;
        }
        pr[r] = pr[r] + 0.0;
        z[r] = __shfl(V.z[r * V.zs + c0] - pr[r], 0, kSmallLeaf);
    }
    if (!p.live[c0]) {          // dropped column (ldlt.c:446-470)
        double eps[R];
        load_eps<R>(epsp, eps);
        int bad[R] = {};
#pragma unroll
        for (int r = 0; r < R; r++) {
            if (fabs(z[r]) > eps[r]) bad[r] = 1;
            else z[r] = 0.0;
        }
        if (lq == 0) flag_bad<R>(p, bad);
    }
    if (lq == 0) {
#pragma unroll
        for (int r = 0; r < R; r++) V.z[r * V.zs + c0] = z[r];
    }
    if (lq < hb) {
        const double l = p.Lx[p.off[s] + 1 + lq];
#pragma unroll
        for (int r = 0; r < R; r++) {
            double acc = 0.0;
            acc += l * z[r];
            V.y[r * V.ys + p.ybase[s] + lq] = acc;
        }
    }
}

template <int R>
__global__ void __launch_bounds__(NT)
k_bwd_leaf8(PlanView p, const int* __restrict__ sups, int q0, int cnt, SweepVecs V, const double* __restrict__ epsp) {
    const int w = (blockIdx.x * NT + threadIdx.x) / kSmallLeaf, lq = threadIdx.x & (kSmallLeaf - 1);
    if (w >= cnt) return;
    const int s = sups[q0 + w];
    const int c0 = p.col0[s], hb = p.rowptr[s + 1] - p.rowptr[s];
    double acc[R];
#pragma unroll
    for (int r = 0; r < R; r++) acc[r] = 0.0;
    if (lq < hb) {
        const int ri = p.rows[p.rowptr[s] + lq];
        const double t = p.Lx[p.off[s] + 1 + lq];
#pragma unroll
        for (int r = 0; r < R; r++) acc[r] += t * V.z[r * V.zs + ri];
    }
    double eps[R];
    load_eps<R>(epsp, eps);
    int bad[R] = {};
#pragma unroll
    for (int r = 0; r < R; r++) {
        double v = acc[r] + 0.0;                      // wave_sum's steps from lanes 32+, 16+, 8+
        v += __shfl_down(v, 4, kSmallLeaf);
        v += __shfl_down(v, 2, kSmallLeaf);
        v += __shfl_down(v, 1, kSmallLeaf);
        if (lq == 0) {
            double zr = dscale_rule(p, c0, V.z[r * V.zs + c0], eps[r], bad[r]) - v;
            if (!p.live[c0]) {
                if (fabs(zr) > eps[r]) bad[r] = 1;
                else zr = 0.0;
            }
            V.z[r * V.zs + c0] = zr;
        }
    }
    if (lq == 0) flag_bad<R>(p, bad);
}

// Forward for levels with large panels, part 1: diagonal parts only.
template <int R>
__global__ void __launch_bounds__(NT)
k_fwd_diag(PlanView p, const int* __restrict__ level_sups, int q0, const int* __restrict__ yrow_ptr,
           const int* __restrict__ yrow_idx, SweepVecs V, const double* __restrict__ epsp) {
    __shared__ double zl[R][PC];
    __shared__ double Ls[PC][PC + 1];
    __shared__ int lv[PC];
    double eps[R];
    load_eps<R>(epsp, eps);
    fwd_diag<R>(p, level_sups[q0 + blockIdx.x], yrow_ptr, yrow_idx, V, eps, zl, Ls, lv);
}

// part 2: y = L21 z_s over one 64-row chunk of R_s; wave w takes columns
// 16w..16w+15, the four partial sums are added in wave order.
template <int R>
__global__ void __launch_bounds__(NT)
k_fwd_gemv(PlanView p, const int* __restrict__ chunk_sup, const int* __restrict__ chunk_r0, int cb, SweepVecs V) {
    __shared__ double zs[R][PC];
    __shared__ double red[R][4][64];
    const int c = cb + blockIdx.x;
    const int s = chunk_sup[c], r0 = chunk_r0[c];
    const int c0 = p.col0[s], nc = p.col0[s + 1] - c0;
    const int hb = p.rowptr[s + 1] - p.rowptr[s], h = nc + hb;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    if (tid < nc) {
#pragma unroll
        for (int r = 0; r < R; r++) zs[r][tid] = V.z[r * V.zs + c0 + tid];
    }
    __syncthreads();
    const int i = r0 + lane, kq = wv * 16, nq = min(16, nc - kq);
    double acc[R];
#pragma unroll
    for (int r = 0; r < R; r++) acc[r] = 0.0;
    if (i < hb && nq > 0) {
        const double* __restrict__ row = p.Lx + p.off[s] + nc + i + (size_t)kq * h;
        double t[16];
#pragma unroll
        for (int q = 0; q < 16; q++) t[q] = row[(size_t)min(q, nq - 1) * h];
#pragma unroll
        for (int q = 0; q < 16; q++)
            if (q < nq) {
#pragma unroll
                for (int r = 0; r < R; r++) acc[r] += t[q] * zs[r][kq + q];
            }
    }
#pragma unroll
    for (int r = 0; r < R; r++) red[r][wv][lane] = acc[r];
    __syncthreads();
    if (wv == 0 && i < hb) {
#pragma unroll
        for (int r = 0; r < R; r++)
            V.y[r * V.ys + p.ybase[s] + i] = ((red[r][0][lane] + red[r][1][lane]) + red[r][2][lane]) + red[r][3][lane];
    }
}

// Backward, one level of small supernodes per launch, one workgroup each:
// z_s = D^{-1} z_s - L21' z_R, then L11'.  Wave w owns columns 16w..16w+15,
// lanes stride the rows (coalesced column reads).
template <int R>
__device__ __forceinline__ void backward_body(const PlanView& p, const int* __restrict__ level_sups, int q0,
                                              const SweepVecs& V, const double* __restrict__ epsp, int bid) {
    __shared__ double xs[R][PC];
    __shared__ double Ls[PC][PC + 1];     // Ls[j][r] = L(j, r)
    __shared__ int lv[PC];
    const int s = level_sups[q0 + bid];
    const int c0 = p.col0[s], nc = p.col0[s + 1] - c0;
    const int hb = p.rowptr[s + 1] - p.rowptr[s];
    const int h = nc + hb;
    const double* panel = p.Lx + p.off[s];
    const int* __restrict__ rows = p.rows + p.rowptr[s];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    stage_l11(panel, h, nc, Ls);
    if (tid < nc) lv[tid] = p.live[c0 + tid];
    const int kq = wv * 16, nq = min(16, nc - kq);
    if (nq > 0) {
        double acc[R][16];
#pragma unroll
        for (int r = 0; r < R; r++)
#pragma unroll
            for (int q = 0; q < 16; q++) acc[r][q] = 0.0;
        for (int i = lane; i < hb; i += 64) {
            const int ri = rows[i];
            double zi[R];
#pragma unroll
            for (int r = 0; r < R; r++) zi[r] = V.z[r * V.zs + ri];
            const double* __restrict__ col = panel + nc + i + (size_t)kq * h;
            double t[16];
#pragma unroll
            for (int q = 0; q < 16; q++) t[q] = col[(size_t)min(q, nq - 1) * h];
#pragma unroll
            for (int q = 0; q < 16; q++)
                if (q < nq) {
#pragma unroll
                    for (int r = 0; r < R; r++) acc[r][q] += t[q] * zi[r];
                }
        }
#pragma unroll
        for (int r = 0; r < R; r++)
#pragma unroll
            for (int q = 0; q < 16; q++) {
                if (q >= nq) break;           // columns of the wave beyond nc: no reduction
                const double t = wave_sum(acc[r][q]);
                if (lane == 0) xs[r][kq + q] = t;
            }
    }
    __syncthreads();
    if (wv >= R) return;
    // wave r solves right-hand side r (independent chains, one wave each)
    const int r = wv;
    const double e1[1] = {epsp[r]};
    int bad[1] = {};
    double zr[1];
    zr[0] = lane < nc ? dscale_rule(p, c0 + lane, V.z[r * V.zs + c0 + lane], e1[0], bad[0]) - xs[r][lane] : 0.0;
    tri_upper<1>(zr, Ls, lv, nc, e1, bad);
    if (lane < nc) V.z[r * V.zs + c0 + lane] = zr[0];
    if (bad[0]) atomicOr(&p.incons[r], 1);
}

template <int R>
__global__ void __launch_bounds__(NT)
k_backward(PlanView p, const int* __restrict__ level_sups, int q0, SweepVecs V, const double* __restrict__ epsp) {
    backward_body<R>(p, level_sups, q0, V, epsp, blockIdx.x);
}

// k_fwd_level's backward counterpart
template <int R>
__global__ void __launch_bounds__(NT)
k_bwd_level(PlanView p, const int* __restrict__ sups, int q0, int nl, int nlb, SweepVecs V,
            const double* __restrict__ epsp) {
    if (static_cast<int>(blockIdx.x) < nlb) bwd_leaf_body<R>(p, sups, q0, nl, V, epsp, blockIdx.x);
    else backward_body<R>(p, sups, q0 + nl, V, epsp, blockIdx.x - nlb);
}

// Backward for levels with large panels, part 1: per 64-row chunk of R_s,
// part[c][k] = sum over the chunk's rows of L(row, k) z_row.
template <int R>
__global__ void __launch_bounds__(NT)
k_bwd_partial(PlanView p, const int* __restrict__ chunk_sup, const int* __restrict__ chunk_r0, int cb, SweepVecs V,
              double* __restrict__ part, size_t ps) {
    const int c = cb + blockIdx.x;
    const int s = chunk_sup[c], r0 = chunk_r0[c];
    const int c0 = p.col0[s], nc = p.col0[s + 1] - c0;
    const int hb = p.rowptr[s + 1] - p.rowptr[s], h = nc + hb;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int kq = wv * 16, nq = min(16, nc - kq);
    if (nq <= 0) return;
    const int i = r0 + lane;
    const bool okr = i < hb;
    const int ic = okr ? i : 0;
    const int ri = p.rows[p.rowptr[s] + ic];
    double zi[R];
#pragma unroll
    for (int r = 0; r < R; r++) zi[r] = V.z[r * V.zs + ri];
    const double* __restrict__ col = p.Lx + p.off[s] + nc + ic + (size_t)kq * h;
    double t[16];
#pragma unroll
    for (int q = 0; q < 16; q++) t[q] = col[(size_t)min(q, nq - 1) * h];
#pragma unroll
    for (int r = 0; r < R; r++)
#pragma unroll
        for (int q = 0; q < 16; q++) {
            if (q >= nq) break;
            const double v = wave_sum(okr ? t[q] * zi[r] : 0.0);
            if (lane == 0) part[r * ps + (size_t)c * PC + kq + q] = v;
        }
}

// part 2: sum the chunks of each supernode (wave w: chunks w, w+4, ...; the
// four partials added in wave order), then D^{-1} and L11'.
template <int R>
__global__ void __launch_bounds__(NT)
k_bwd_finish(PlanView p, const int* __restrict__ level_sups, int q0, const int* __restrict__ sup_chunk0,
             const double* __restrict__ part, size_t ps, SweepVecs V, const double* __restrict__ epsp) {
    __shared__ double Ls[PC][PC + 1];
    __shared__ int lv[PC];
    __shared__ double xs[R][4][PC];
    const int s = level_sups[q0 + blockIdx.x];
    const int c0 = p.col0[s], nc = p.col0[s + 1] - c0;
    const int hb = p.rowptr[s + 1] - p.rowptr[s], h = nc + hb;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    stage_l11(p.Lx + p.off[s], h, nc, Ls);
    if (tid < nc) lv[tid] = p.live[c0 + tid];
    {
        const int cf = sup_chunk0[s], nch = (hb + 63) / 64;
        double x[R];
#pragma unroll
        for (int r = 0; r < R; r++) x[r] = 0.0;
        if (lane < nc)
            for (int c = wv; c < nch; c += 4) {
#pragma unroll
                for (int r = 0; r < R; r++) x[r] += part[r * ps + (size_t)(cf + c) * PC + lane];
            }
#pragma unroll
        for (int r = 0; r < R; r++) xs[r][wv][lane] = x[r];
    }
    __syncthreads();
    if (wv >= R) return;
    // wave r solves right-hand side r (independent chains, one wave each)
    const int r = wv;
    const double e1[1] = {epsp[r]};
    int bad[1] = {};
    double zr[1];
    zr[0] = lane < nc ? dscale_rule(p, c0 + lane, V.z[r * V.zs + c0 + lane], e1[0], bad[0]) -
                            (((xs[r][0][lane] + xs[r][1][lane]) + xs[r][2][lane]) + xs[r][3][lane])
                      : 0.0;
    tri_upper<1>(zr, Ls, lv, nc, e1, bad);
    if (lane < nc) V.z[r * V.zs + c0 + lane] = zr[0];
    if (bad[0]) atomicOr(&p.incons[r], 1);
}

// ---------------------------------------------------- dense-tail solves
// forward, part 1: tail rows subtract the y values the sparse panels left
template <int R>
__global__ void __launch_bounds__(NT)
k_tail_gather(TailView tv, const int* __restrict__ yrow_ptr, const int* __restrict__ yrow_idx, SweepVecs V) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int i = blockIdx.x * 4 + wv;
    if (i >= tv.nt) return;
    const int v = tv.tc + i;
    double acc[R];
#pragma unroll
    for (int r = 0; r < R; r++) acc[r] = 0.0;
    for (int e = yrow_ptr[v] + lane; e < yrow_ptr[v + 1]; e += 64) {
        const int i0 = yrow_idx[e];
#pragma unroll
        for (int r = 0; r < R; r++) acc[r] += V.y[r * V.ys + i0];
    }
#pragma unroll
    for (int r = 0; r < R; r++) {
        const double a = wave_sum(acc[r]);
        if (lane == 0) V.z[r * V.zs + v] = V.z[r * V.zs + v] - a;
    }
}

// Per-block fallbacks for very large dense tails (ntb > kChainMaxBlocks),
// one right-hand side.  forward, part 2, block kb: every workgroup solves
// the block's L11 in wave 0 (identical arithmetic, identical results;
// workgroup 0 stores it), then updates 64 rows below it.
__global__ void __launch_bounds__(NT)
k_tail_fwd(PlanView p, TailView tv, int kb, double* __restrict__ z, const double* __restrict__ epsp) {
    __shared__ double Ls[PC][PC + 1];
    __shared__ double zb[PC];
    __shared__ int lv[PC];
    __shared__ double red[4][64];
    const int nt = tv.nt, tc = tv.tc, k0 = kb * PC, nc = min(PC, nt - k0);
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    stage_l11(tv.S + k0 + (size_t)k0 * nt, nt, nc, Ls);
    if (tid < nc) lv[tid] = p.live[tc + k0 + tid];
    __syncthreads();
    if (wv == 0) {
        int bad[1] = {0};
        double eps[1] = {*epsp};
        double zr[1] = {lane < nc ? z[tc + k0 + lane] : 0.0};
        tri_lower<1>(zr, Ls, lv, nc, eps, bad);
        if (lane < nc) zb[lane] = zr[0];
        if (blockIdx.x == 0) {
            if (lane < nc) z[tc + k0 + lane] = zr[0];
            flag_bad<1>(p, bad);
        }
    }
    __syncthreads();
    const int r = k0 + nc + blockIdx.x * 64 + lane;
    const int kq = wv * 16, nq = min(16, nc - kq);
    double acc = 0.0;
    if (r < nt && nq > 0) {
        const double* __restrict__ row = tv.S + r + (size_t)(k0 + kq) * nt;
        double t[16];
#pragma unroll
        for (int q = 0; q < 16; q++) t[q] = row[(size_t)min(q, nq - 1) * nt];
#pragma unroll
        for (int q = 0; q < 16; q++)
            if (q < nq) acc += t[q] * zb[kq + q];
    }
    red[wv][lane] = acc;
    __syncthreads();
    if (wv == 0 && r < nt) z[tc + r] = z[tc + r] - (((red[0][lane] + red[1][lane]) + red[2][lane]) + red[3][lane]);
}

// backward, part 1: D^{-1} on the tail with the dropped-column rule
__global__ void __launch_bounds__(NT)
k_tail_dscale(PlanView p, TailView tv, double* __restrict__ z, const double* __restrict__ epsp) {
    const int i = blockIdx.x * NT + threadIdx.x;
    if (i >= tv.nt) return;
    const int v = tv.tc + i;
    int bad[1] = {0};
    z[v] = dscale_rule(p, v, z[v], *epsp, bad[0]);
    flag_bad<1>(p, bad);
}

// backward, part 2, block kb: L11' solve (every workgroup, workgroup 0
// stores), then 64 columns j < k0 left of it.
__global__ void __launch_bounds__(NT)
k_tail_bwd(PlanView p, TailView tv, int kb, double* __restrict__ z, const double* __restrict__ epsp) {
    __shared__ double Ls[PC][PC + 1];     // Ls[j][r] = L(j, r)
    __shared__ double zb[PC];
    __shared__ int lv[PC];
    __shared__ double red[4][64];
    const int nt = tv.nt, tc = tv.tc, k0 = kb * PC, nc = min(PC, nt - k0);
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    stage_l11(tv.S + k0 + (size_t)k0 * nt, nt, nc, Ls);
    if (tid < nc) lv[tid] = p.live[tc + k0 + tid];
    __syncthreads();
    if (wv == 0) {
        int bad[1] = {0};
        double eps[1] = {*epsp};
        double zr[1] = {lane < nc ? z[tc + k0 + lane] : 0.0};
        tri_upper<1>(zr, Ls, lv, nc, eps, bad);
        if (lane < nc) zb[lane] = zr[0];
        if (blockIdx.x == 0) {
            if (lane < nc) z[tc + k0 + lane] = zr[0];
            flag_bad<1>(p, bad);
        }
    }
    __syncthreads();
    const int j = blockIdx.x * 64 + lane;
    const int kq = wv * 16, nq = min(16, nc - kq);
    double acc = 0.0;
    if (j < k0 && nq > 0) {
        const double* __restrict__ col = tv.S + (k0 + kq) + (size_t)j * nt;
        double t[16];
#pragma unroll
        for (int q = 0; q < 16; q++) t[q] = col[min(q, nq - 1)];
#pragma unroll
        for (int q = 0; q < 16; q++)
            if (q < nq) acc += t[q] * zb[kq + q];
    }
    red[wv][lane] = acc;
    __syncthreads();
    if (wv == 0 && j < k0) z[tc + j] = z[tc + j] - (((red[0][lane] + red[1][lane]) + red[2][lane]) + red[3][lane]);
}

// ------------------------------------------- dense-tail sweeps, one launch
// Sync-free block-row chains: workgroup i owns 64-row block i of the tail
// and waits, block by block, for the blocks it depends on.  Each block's z
// is handed on as epoch-tagged granules (gran_put / gran_wait above,
// MI355X_MICROARCH.md hand-off table row R2: the data is the flag -- one
// store round trip on the producer, one load round trip on the consumer;
// round 2's sc1 payload + drained flag took two of each).  One workgroup
// per CU is enforced with dynamic LDS.  Every workgroup only waits on blocks
// of lower rank in its own launch order, so the grid drains as long as it
// is resident (ntb <= kChainMaxBlocks).
constexpr int kChainMaxBlocks = 200;
constexpr size_t kChainLds = 96 * 1024;
static_assert(2 * PC * (PC + 1) * sizeof(double) <= kChainLds, "k_tail_bwd_chain scratch");

#ifndef IPO_POLL_SLEEP
#define IPO_POLL_SLEEP 1
#endif
__device__ __forceinline__ void chain_wait(const int* flags, int j, int epoch) {
    if (threadIdx.x == 0)
        while (__hip_atomic_load(const_cast<int*>(flags + j), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < epoch)
            __builtin_amdgcn_s_sleep(IPO_POLL_SLEEP);
    __syncthreads();
}
__device__ __forceinline__ void chain_publish(int* flags, int i, int epoch) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_store(flags + i, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Data-tagged hand-off of a block's z (MI355X_MICROARCH.md hand-off table,
// row R2): every double travels as two naturally aligned 8-byte granules
// {tag = epoch, 32-bit half}, each written by ONE relaxed agent-scope
// (sc1) store -- no flag, no drain, no barrier on the producer; the consumer
// re-reads its granules until every tag is the launch's epoch and has the
// data with the match.  Epochs grow by one per launch and are never reused
// (the buffer starts zeroed, the first epoch is 1), so no reset per launch.
// Block j, right-hand side r, row q: granules ((j R + r) 64 + q) 2 + {0, 1}.
typedef unsigned long long gran_t;
__device__ __forceinline__ void gran_put(gran_t* g, unsigned epoch, double v) {
    const unsigned long long b = static_cast<unsigned long long>(__double_as_longlong(v));
    const unsigned long long e = static_cast<unsigned long long>(epoch) << 32;
    __hip_atomic_store(g, e | (b & 0xffffffffull), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(g + 1, e | (b >> 32), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// one wave: lane q < nr waits for row q of block j's R values
template <int R>
__device__ __forceinline__ void gran_wait(const gran_t* g, unsigned epoch, int lane, int nr, double (&v)[R]) {
    for (;;) {
        bool ok = true;
#pragma unroll
        for (int r = 0; r < R; r++) {
            if (lane < nr) {
                const gran_t* q = g + ((size_t)r * 64 + lane) * 2;
                const unsigned long long lo = __hip_atomic_load(const_cast<gran_t*>(q), __ATOMIC_RELAXED,
                                                                __HIP_MEMORY_SCOPE_AGENT);
                const unsigned long long hi = __hip_atomic_load(const_cast<gran_t*>(q + 1), __ATOMIC_RELAXED,
                                                                __HIP_MEMORY_SCOPE_AGENT);
                ok &= (lo >> 32) == epoch && (hi >> 32) == epoch;
                v[r] = __longlong_as_double(static_cast<long long>(((hi & 0xffffffffull) << 32) | (lo & 0xffffffffull)));
            } else {
                v[r] = 0.0;
            }
        }
        if (__all(ok)) return;
        __builtin_amdgcn_s_sleep(IPO_POLL_SLEEP);
    }
}

// forward: z_i -= sum_{j<i} L(i, j) z_j, then the unit-lower L11 solve of block i
template <int R>
__global__ void __launch_bounds__(NT)
k_tail_fwd_chain(PlanView p, TailView tv, SweepVecs V, const double* __restrict__ epsp, gran_t* __restrict__ gran,
                 unsigned epoch) {
    extern __shared__ double lds_pad[];
    __shared__ double Ls[PC][PC + 1];
    __shared__ int lv[PC];
    __shared__ double zb[R][PC];
    __shared__ double red[R][4][64];
    const int nt = tv.nt, tc = tv.tc, i = blockIdx.x, k0 = i * PC, nc = min(PC, nt - k0);
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    // the own block's right-hand side and eps do not depend on the chain
    double eps[R], zown[R];
    load_eps<R>(epsp, eps);
#pragma unroll
    for (int r = 0; r < R; r++) zown[r] = (wv == 0 && lane < nc) ? V.z[r * V.zs + tc + k0 + lane] : 0.0;
    if (tid == 0) lds_pad[0] = 0.0;
    stage_l11(tv.S + k0 + (size_t)k0 * nt, nt, nc, Ls);
    if (tid < nc) lv[tid] = p.live[tc + k0 + tid];
    const int row = k0 + (lane < nc ? lane : 0);
    double acc[R];
#pragma unroll
    for (int r = 0; r < R; r++) acc[r] = 0.0;
    for (int j = 0; j < i; j++) {
        // the L(i, j) tile does not depend on z: load it before waiting
        const double* __restrict__ col = tv.S + row + (size_t)(j * PC + wv * 16) * nt;
        double t[16];
#pragma unroll
        for (int q = 0; q < 16; q++) t[q] = col[(size_t)q * nt];
        if (wv == 0) {
            double zj[R];
            gran_wait<R>(gran + (size_t)j * R * 128, epoch, lane, PC, zj);
#pragma unroll
            for (int r = 0; r < R; r++) zb[r][lane] = zj[r];
        }
        __syncthreads();
#pragma unroll
        for (int q = 0; q < 16; q++) {
#pragma unroll
            for (int r = 0; r < R; r++) acc[r] += t[q] * zb[r][wv * 16 + q];
        }
        __syncthreads();
    }
#pragma unroll
    for (int r = 0; r < R; r++) red[r][wv][lane] = acc[r];
    __syncthreads();
    if (wv == 0) {
        int bad[R] = {};
        double zr[R];
#pragma unroll
        for (int r = 0; r < R; r++)
            zr[r] = lane < nc ? zown[r] - (((red[r][0][lane] + red[r][1][lane]) + red[r][2][lane]) + red[r][3][lane])
                              : 0.0;
        tri_lower<R>(zr, Ls, lv, nc, eps, bad);
        if (lane < nc) {
#pragma unroll
            for (int r = 0; r < R; r++) {
                gran_put(gran + (((size_t)i * R + r) * 64 + lane) * 2, epoch, zr[r]);
                V.z[r * V.zs + tc + k0 + lane] = zr[r];
            }
        }
        flag_bad<R>(p, bad);
    }
}

// backward (launch order = blocks from the last): z_i = D^{-1} z_i
// - sum_{j>i} L(j, i)' z_j, then the L11' solve.  Wave w owns 16 columns of
// block i, lanes stride the rows of block j (coalesced column reads).
template <int R>
__global__ void __launch_bounds__(NT)
k_tail_bwd_chain(PlanView p, TailView tv, SweepVecs V, const double* __restrict__ epsp, gran_t* __restrict__ gran,
                 unsigned epoch) {
    extern __shared__ double lds_pad[];
    __shared__ double Ls[PC][PC + 1];     // Ls[j][r] = L(j, r)
    __shared__ int lv[PC];
    __shared__ double zb[R][PC];
    __shared__ double xs[R][PC];
    const int nt = tv.nt, tc = tv.tc, ntb = tv.ntb;
    const int i = ntb - 1 - blockIdx.x, k0 = i * PC, nc = min(PC, nt - k0);
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    if (tid == 0) lds_pad[0] = 0.0;
    stage_l11(tv.S + k0 + (size_t)k0 * nt, nt, nc, Ls);
    if (tid < nc) lv[tid] = p.live[tc + k0 + tid];
    const int kq = wv * 16, nq = min(16, nc - kq);
    // D^{-1} z of the own block does not depend on the chain: formed first,
    // by the wave that solves its right-hand side (wave r solves r: the two
    // triangular solves of R = 2 are independent chains, one wave each runs
    // them at about twice the pace of one wave interleaving both)
    double eps[R], zd[R];
    int bad[R] = {};
    load_eps<R>(epsp, eps);
#pragma unroll
    for (int r = 0; r < R; r++)
        zd[r] = (wv == r && lane < nc) ? dscale_rule(p, tc + k0 + lane, V.z[r * V.zs + tc + k0 + lane], eps[r], bad[r])
                                       : 0.0;
    double acc[R][16];
#pragma unroll
    for (int r = 0; r < R; r++)
#pragma unroll
        for (int q = 0; q < 16; q++) acc[r][q] = 0.0;
    for (int j = ntb - 1; j > i; j--) {
        const int r0 = j * PC, nr = min(PC, nt - r0);
        const int rr = r0 + (lane < nr ? lane : 0);
        const double* __restrict__ col = tv.S + rr + (size_t)(k0 + (nq > 0 ? kq : 0)) * nt;
        double t[16];
#pragma unroll
        for (int q = 0; q < 16; q++) t[q] = col[(size_t)min(q, max(nq, 1) - 1) * nt];
        if (wv == 0) {
            double zj[R];
            gran_wait<R>(gran + (size_t)j * R * 128, epoch, lane, nr, zj);
#pragma unroll
            for (int r = 0; r < R; r++) zb[r][lane] = zj[r];
        }
        __syncthreads();
#pragma unroll
        for (int r = 0; r < R; r++) {
            const double zr = lane < nr ? zb[r][lane] : 0.0;
#pragma unroll
            for (int q = 0; q < 16; q++) acc[r][q] += t[q] * zr;
        }
        __syncthreads();
    }
    double* red = lds_pad;   // colsum scratch
    if (nq > 0) colsum_put<R>(red, acc, kq, nq, lane);
    __syncthreads();
    if (tid < R * PC && tid % PC < nc) xs[tid / PC][tid % PC] = colsum_tree(red, tid / PC, tid % PC);
    __syncthreads();
    if (wv < R) {
        const int r = wv;
        double zr[1] = {lane < nc ? zd[r] - (i < ntb - 1 ? xs[r][lane] : 0.0) : 0.0};
        const double e1[1] = {eps[r]};
        int b1[1] = {bad[r]};
        tri_upper<1>(zr, Ls, lv, nc, e1, b1);
        if (lane < nc) {
            gran_put(gran + (((size_t)i * R + r) * 64 + lane) * 2, epoch, zr[0]);
            V.z[r * V.zs + tc + k0 + lane] = zr[0];
        }
        if (b1[0]) atomicOr(&p.incons[r], 1);
    }
}

// The same chains with two 64-row blocks per workgroup ("pairs"): the
// first block's z is handed to the second inside the workgroup (through LDS
// after a barrier) instead of through memory, one hand-off per pair instead
// of per block, while the first block's z is published at once for the
// workgroups further down the chain.  Every entry sees the arithmetic of
// k_tail_fwd_chain / k_tail_bwd_chain in the same order (the per-wave
// partial sums over the earlier blocks, the internal block as their last
// term, the same wave / column reductions and triangular solves): bitwise
// the same sweep.  Forward: workgroup g owns blocks a = 2g, b = 2g + 1.
constexpr size_t kPairFwdLds = 64 * 1024;                                   // dynamic pad: one per CU
constexpr size_t kPairBwdLds = 2 * PC * (PC + 1) * sizeof(double);           // colsum scratch (R <= 2)

template <int R>
__global__ void __launch_bounds__(NT)
k_tail_fwd_pair(PlanView p, TailView tv, SweepVecs V, const double* __restrict__ epsp, gran_t* __restrict__ gran,
                unsigned epoch) {
    extern __shared__ double lds_pad[];
    __shared__ double Ls[2][PC][PC + 1];
    __shared__ int lv[2][PC];
    __shared__ double zb[R][PC];
    __shared__ double red[R][4][64];
    const int nt = tv.nt, tc = tv.tc, ntb = tv.ntb;
    const int a = 2 * blockIdx.x, b = a + 1;
    const bool hasb = b < ntb;
    const int ka = a * PC, nca = min(PC, nt - ka), kb = b * PC, ncb = hasb ? min(PC, nt - kb) : 0;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    double eps[R], zown_a[R], zown_b[R];
    load_eps<R>(epsp, eps);
#pragma unroll
    for (int r = 0; r < R; r++) {
        zown_a[r] = (wv == 0 && lane < nca) ? V.z[r * V.zs + tc + ka + lane] : 0.0;
        zown_b[r] = (wv == 0 && lane < ncb) ? V.z[r * V.zs + tc + kb + lane] : 0.0;
    }
    if (tid == 0) lds_pad[0] = 0.0;
    stage_l11(tv.S + ka + (size_t)ka * nt, nt, nca, Ls[0]);
    if (hasb) stage_l11(tv.S + kb + (size_t)kb * nt, nt, ncb, Ls[1]);
    if (tid < nca) lv[0][tid] = p.live[tc + ka + tid];
    if (tid < ncb) lv[1][tid] = p.live[tc + kb + tid];
    const int rowa = ka + (lane < nca ? lane : 0), rowb = kb + (lane < ncb ? lane : ka - kb);
    double acca[R], accb[R];
#pragma unroll
    for (int r = 0; r < R; r++) { acca[r] = 0.0; accb[r] = 0.0; }
    for (int j = 0; j < a; j++) {
        const size_t c0 = (size_t)(j * PC + wv * 16) * nt;
        double ta[16], tb[16];
#pragma unroll
        for (int q = 0; q < 16; q++) { ta[q] = tv.S[rowa + c0 + (size_t)q * nt]; tb[q] = tv.S[rowb + c0 + (size_t)q * nt]; }
        if (wv == 0) {
            double zj[R];
            gran_wait<R>(gran + (size_t)j * R * 128, epoch, lane, PC, zj);
#pragma unroll
            for (int r = 0; r < R; r++) zb[r][lane] = zj[r];
        }
        __syncthreads();
#pragma unroll
        for (int q = 0; q < 16; q++) {
#pragma unroll
            for (int r = 0; r < R; r++) {
                acca[r] += ta[q] * zb[r][wv * 16 + q];
                accb[r] += tb[q] * zb[r][wv * 16 + q];
            }
        }
        __syncthreads();
    }
    // block b's term of block a (rows of b, columns of a): loaded before a's solve
    double tba[16];
    {
        const size_t c0 = (size_t)(ka + wv * 16) * nt;
#pragma unroll
        for (int q = 0; q < 16; q++) tba[q] = tv.S[rowb + c0 + (size_t)q * nt];
    }
#pragma unroll
    for (int r = 0; r < R; r++) red[r][wv][lane] = acca[r];
    __syncthreads();
    if (wv == 0) {
        int bad[R] = {};
        double zr[R];
#pragma unroll
        for (int r = 0; r < R; r++)
            zr[r] = lane < nca ? zown_a[r] - (((red[r][0][lane] + red[r][1][lane]) + red[r][2][lane]) + red[r][3][lane])
                               : 0.0;
        tri_lower<R>(zr, Ls[0], lv[0], nca, eps, bad);
        if (lane < nca) {
#pragma unroll
            for (int r = 0; r < R; r++) {
                gran_put(gran + (((size_t)a * R + r) * 64 + lane) * 2, epoch, zr[r]);
                V.z[r * V.zs + tc + ka + lane] = zr[r];
            }
        }
#pragma unroll
        for (int r = 0; r < R; r++) zb[r][lane] = lane < nca ? zr[r] : 0.0;
        flag_bad<R>(p, bad);
    }
    if (!hasb) return;
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 16; q++) {
#pragma unroll
        for (int r = 0; r < R; r++) accb[r] += tba[q] * zb[r][wv * 16 + q];
    }
#pragma unroll
    for (int r = 0; r < R; r++) red[r][wv][lane] = accb[r];
    __syncthreads();
    if (wv == 0) {
        int bad[R] = {};
        double zr[R];
#pragma unroll
        for (int r = 0; r < R; r++)
            zr[r] = lane < ncb ? zown_b[r] - (((red[r][0][lane] + red[r][1][lane]) + red[r][2][lane]) + red[r][3][lane])
                               : 0.0;
        tri_lower<R>(zr, Ls[1], lv[1], ncb, eps, bad);
        if (lane < ncb) {
#pragma unroll
            for (int r = 0; r < R; r++) {
                gran_put(gran + (((size_t)b * R + r) * 64 + lane) * 2, epoch, zr[r]);
                V.z[r * V.zs + tc + kb + lane] = zr[r];
            }
        }
        flag_bad<R>(p, bad);
    }
}

// Backward pairs, from the last block: workgroup g owns blocks hi = ntb - 1
// - 2g and lo = hi - 1 (none for an odd count's first workgroup).
template <int R>
__global__ void __launch_bounds__(NT)
k_tail_bwd_pair(PlanView p, TailView tv, SweepVecs V, const double* __restrict__ epsp, gran_t* __restrict__ gran,
                unsigned epoch) {
    extern __shared__ double lds_pad[];
    __shared__ double Ls[2][PC][PC + 1];     // [0] block hi, [1] block lo; Ls[j][r] = L(j, r)
    __shared__ int lv[2][PC];
    __shared__ double zb[R][PC];
    __shared__ double xs[R][PC];
    const int nt = tv.nt, tc = tv.tc, ntb = tv.ntb;
    const int hi = ntb - 1 - 2 * blockIdx.x, lo = hi - 1;
    const bool haslo = lo >= 0;
    const int kh = hi * PC, nch = min(PC, nt - kh), kl = haslo ? lo * PC : kh, ncl = haslo ? PC : 0;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    stage_l11(tv.S + kh + (size_t)kh * nt, nt, nch, Ls[0]);
    if (haslo) stage_l11(tv.S + kl + (size_t)kl * nt, nt, ncl, Ls[1]);
    if (tid < nch) lv[0][tid] = p.live[tc + kh + tid];
    if (tid < ncl) lv[1][tid] = p.live[tc + kl + tid];
    const int kq = wv * 16, nqh = min(16, nch - kq), nql = min(16, ncl - kq);
    double eps[R], zdh[R], zdl[R];
    int badh[R] = {}, badl[R] = {};
    load_eps<R>(epsp, eps);
#pragma unroll
    for (int r = 0; r < R; r++) {
        zdh[r] = (wv == 0 && lane < nch) ? dscale_rule(p, tc + kh + lane, V.z[r * V.zs + tc + kh + lane], eps[r], badh[r])
                                         : 0.0;
        zdl[r] = (wv == 0 && lane < ncl) ? dscale_rule(p, tc + kl + lane, V.z[r * V.zs + tc + kl + lane], eps[r], badl[r])
                                         : 0.0;
    }
    double acch[R][16], accl[R][16];
#pragma unroll
    for (int r = 0; r < R; r++)
#pragma unroll
        for (int q = 0; q < 16; q++) { acch[r][q] = 0.0; accl[r][q] = 0.0; }
    for (int j = ntb - 1; j > hi; j--) {
        const int r0 = j * PC, nr = min(PC, nt - r0);
        const int rr = r0 + (lane < nr ? lane : 0);
        const double* __restrict__ colh = tv.S + rr + (size_t)(kh + (nqh > 0 ? kq : 0)) * nt;
        const double* __restrict__ coll = tv.S + rr + (size_t)(kl + (nql > 0 ? kq : 0)) * nt;
        double th[16], tl[16];
#pragma unroll
        for (int q = 0; q < 16; q++) {
            th[q] = colh[(size_t)min(q, max(nqh, 1) - 1) * nt];
            tl[q] = coll[(size_t)min(q, max(nql, 1) - 1) * nt];
        }
        if (wv == 0) {
            double zj[R];
            gran_wait<R>(gran + (size_t)j * R * 128, epoch, lane, nr, zj);
#pragma unroll
            for (int r = 0; r < R; r++) zb[r][lane] = zj[r];
        }
        __syncthreads();
#pragma unroll
        for (int r = 0; r < R; r++) {
            const double zr = lane < nr ? zb[r][lane] : 0.0;
#pragma unroll
            for (int q = 0; q < 16; q++) {
                acch[r][q] += th[q] * zr;
                accl[r][q] += tl[q] * zr;
            }
        }
        __syncthreads();
    }
    // block lo's term of block hi (rows of hi, columns of lo): loaded before hi's solve
    double tlh[16];
    {
        const int rr = kh + (lane < nch ? lane : 0);
        const double* __restrict__ col = tv.S + rr + (size_t)(kl + (nql > 0 ? kq : 0)) * nt;
#pragma unroll
        for (int q = 0; q < 16; q++) tlh[q] = col[(size_t)min(q, max(nql, 1) - 1) * nt];
    }
    double* red = lds_pad;   // colsum scratch
    if (hi < ntb - 1) {
        if (nqh > 0) colsum_put<R>(red, acch, kq, nqh, lane);
        __syncthreads();
        if (tid < R * PC && tid % PC < nch) xs[tid / PC][tid % PC] = colsum_tree(red, tid / PC, tid % PC);
        __syncthreads();
    }
    if (wv == 0) {
        double zr[R];
#pragma unroll
        for (int r = 0; r < R; r++) zr[r] = lane < nch ? zdh[r] - (hi < ntb - 1 ? xs[r][lane] : 0.0) : 0.0;
        tri_upper<R>(zr, Ls[0], lv[0], nch, eps, badh);
        if (lane < nch) {
#pragma unroll
            for (int r = 0; r < R; r++) {
                gran_put(gran + (((size_t)hi * R + r) * 64 + lane) * 2, epoch, zr[r]);
                V.z[r * V.zs + tc + kh + lane] = zr[r];
            }
        }
#pragma unroll
        for (int r = 0; r < R; r++) zb[r][lane] = zr[r];
        flag_bad<R>(p, badh);
    }
    if (!haslo) return;
    __syncthreads();
#pragma unroll
    for (int r = 0; r < R; r++) {
        const double zr = lane < nch ? zb[r][lane] : 0.0;
#pragma unroll
        for (int q = 0; q < 16; q++) accl[r][q] += tlh[q] * zr;
    }
    if (nql > 0) colsum_put<R>(red, accl, kq, nql, lane);
    __syncthreads();
    if (tid < R * PC && tid % PC < ncl) xs[tid / PC][tid % PC] = colsum_tree(red, tid / PC, tid % PC);
    __syncthreads();
    if (wv == 0) {
        double zr[R];
#pragma unroll
        for (int r = 0; r < R; r++) zr[r] = lane < ncl ? zdl[r] - xs[r][lane] : 0.0;
        tri_upper<R>(zr, Ls[1], lv[1], ncl, eps, badl);
        if (lane < ncl) {
#pragma unroll
            for (int r = 0; r < R; r++) {
                gran_put(gran + (((size_t)lo * R + r) * 64 + lane) * 2, epoch, zr[r]);
                V.z[r * V.zs + tc + kl + lane] = zr[r];
            }
        }
        flag_bad<R>(p, badl);
    }
}

// ------------------------------------ forward tail sweep: a lead workgroup
// The chain above hands every block's z across CUs (a granule round trip per
// block on the critical path).  Here ONE lead workgroup solves all blocks in
// order, z_{i-1} reaching block i through LDS.  Of block i's products
// L(i, j) z_j the lead forms only the last K = kLeadBlocks (j = i-K .. i-1);
// helper workgroup i - K (one per block i > K) sums j = 0 .. i-K-1 from the
// granules of z the lead publishes and hands its per-lane partials to the
// lead as granules.  Each lane's sum is k_tail_fwd_chain's wave partial --
// the same terms in the same order, continued by the lead -- and the column
// reduction and L11 solve are the same: bitwise the same sweep.
// Lead: wave 0 solves; four "product waves" (column group g owns columns
// 16g .. 16g+15 of every block; waves 1, 2, 3, 5 -- wave 4, which would share
// the solver's SIMD, leaves at once) form the partials and, while wave 0
// solves block i, already sum block i+1's partial up to j = i-1, store the
// L11 of block i+1 (loaded a step earlier) and issue the loads of step i+2
// (tiles, L11, the helper partial).  Measured on dfl001 (70 blocks, R = 2,
// IPO_LEAD_STAMPS): 2.8 us per step -- solve 2.0, waits 0.8 -- against
// ~3.5 us per block of the per-block chain, whose cross-CU hand-off this
// removes.  Step i, barriers A_i and B_i:
//   products: acc = pre_i + L(i, i-1) z_{i-1} -> red  |A_i|  pre_{i+1} =
//             helper partial + L(i+1, j) z_j for j = i+1-K .. i-1; loads
//             for step i+2; L11(i+1) staged  |B_i|
//   solver:   |A_i|  z_i = L11 \ (z_i - sum of red), published  |B_i|
// Residency: a helper waits only on z the lead publishes, the lead only on
// helpers' partials over earlier z -- acyclic while the grid (<= ntb
// workgroups, one per CU by the dynamic LDS) is resident.
constexpr int kLeadBlocks = 2;     // K = 1 measured: forward sweep 380 -> 387 us (helpers' partials late)
// developer stamps (-DIPO_LEAD_STAMPS; compiled out otherwise): one launch's
// per-step split printed from the device
#ifdef IPO_LEAD_STAMPS
__device__ double g_lead_stats[8][4];
#define LEAD_T(v) const long long v = wall_clock64()
#else
#define LEAD_T(v) do {} while (0)
#endif
// raw buffer over the tail S (nt <= kChainMaxBlocks * PC: byte offsets fit an int)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t tail_rsrc(const double* S) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<double*>(S), 0, 0x7fffffff, 0x00020000);
}
__device__ __forceinline__ double buf_ld(__amdgpu_buffer_rsrc_t rs, int voff, int soff) {
    typedef int i32x2 __attribute__((ext_vector_type(2)));
    const i32x2 v = __builtin_amdgcn_raw_buffer_load_b64(rs, voff, soff, 0);
    return __builtin_bit_cast(double, v);
}
constexpr int kLeadNT = 448;
constexpr int kHelpBatch = 4;
// helper partials: block i, right-hand side r, column group g, lane l ->
// granules ((((i R + r) 4 + g) 64 + l) 2 + {0, 1}
__device__ __forceinline__ gran_t* part_slot(gran_t* pg, int i, int R, int r, int g, int lane) {
    return pg + (((((size_t)i * R + r) * 4 + g) * 64) + lane) * 2;
}
__device__ __forceinline__ void lds_sync() {     // LDS-only barrier: global stores need not drain
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

template <int R>
__global__ void __launch_bounds__(kLeadNT)
k_tail_fwd_lead(PlanView p, TailView tv, SweepVecs V, const double* __restrict__ epsp, gran_t* __restrict__ gran,
                gran_t* __restrict__ pgran, unsigned epoch, int* __restrict__ ticket, int tbase) {
    extern __shared__ double lds[];
    constexpr int K = kLeadBlocks;
    const int nt = tv.nt, tc = tv.tc, ntb = tv.ntb;
    // waves: 0 solves (right-hand side 0; 6, on SIMD 2, solves 1 when R = 2:
    // two independent chains at one wave each); 1, 2, 3 and 5 are column
    // groups 0-3; 4 (which would share wave 0's SIMD) leaves at once
    const int tid = threadIdx.x, lane = tid & 63, wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int g = wv <= 3 ? wv - 1 : wv - 2;     // wave-uniform (scalar buffer offsets)
    const int pl = g * 64 + lane;
    // roles by ticket, not by blockIdx: the workgroup that draws ticket 0 is
    // the lead, ticket t > 0 the helper of block t + K.  A helper waits only
    // on z the lead publishes and the lead only on partials of helpers with
    // lower tickets, each drawn by a workgroup that is running or done, so
    // the grid drains on any share of the CUs (co-tenant kernels, shards on
    // one device) without relying on dispatch order (ADVICE/VERDICT r04)
    __shared__ int role_sh;
    if (tid == 0) role_sh = __hip_atomic_fetch_add(ticket, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - tbase;
    __syncthreads();
    const int role = role_sh;
    if (wv == 4 || (wv == 6 && (R == 1 || role > 0))) return;
    if (role > 0) {              // helper of block i
        const int i = role + K, k0 = i * PC, nc = min(PC, nt - k0), jend = i - K;
        double* zb = lds;        // zb[(b R + r) PC + c]
        const __amdgpu_buffer_rsrc_t rs = tail_rsrc(tv.S);
        const int nt8 = nt * 8, g16 = __builtin_amdgcn_readfirstlane(g * 16);
        const int voff = (k0 + (lane < nc ? lane : 0)) * 8;
        double acc[R];
#pragma unroll
        for (int r = 0; r < R; r++) acc[r] = 0.0;
        for (int j0 = 0; j0 < jend; j0 += kHelpBatch) {
            double t[kHelpBatch][16];
            if (wv > 0) {
#pragma unroll
                for (int b = 0; b < kHelpBatch; b++) {
                    const int s0 = (min(j0 + b, jend - 1) * PC + g16) * nt8;
#pragma unroll
                    for (int q = 0; q < 16; q++) t[b][q] = buf_ld(rs, voff, s0 + q * nt8);
                }
            } else {
#pragma unroll
                for (int b = 0; b < kHelpBatch; b++) {
                    if (j0 + b < jend) {
                        double zj[R];
                        gran_wait<R>(gran + (size_t)(j0 + b) * R * 128, epoch, lane, PC, zj);
#pragma unroll
                        for (int r = 0; r < R; r++) zb[(b * R + r) * PC + lane] = zj[r];
                    }
                }
            }
            lds_sync();
            if (wv > 0) {
#pragma unroll
                for (int b = 0; b < kHelpBatch; b++) {
                    if (j0 + b < jend) {
#pragma unroll
                        for (int q = 0; q < 16; q++) {
#pragma unroll
                            for (int r = 0; r < R; r++) acc[r] += t[b][q] * zb[(b * R + r) * PC + g * 16 + q];
                        }
                    }
                }
            }
            lds_sync();
        }
        if (wv > 0) {
#pragma unroll
            for (int r = 0; r < R; r++) gran_put(part_slot(pgran, i, R, r, g, lane), epoch, acc[r]);
        }
        return;
    }
    double(*Ls)[PC][PC + 1] = reinterpret_cast<double(*)[PC][PC + 1]>(lds);     // two buffers
    double* zh = lds + 2 * PC * (PC + 1);     // z of the last K blocks: zh[((j % K) R + r) PC + c]
    double* red = zh + K * R * PC;            // red[(r 4 + g) 64 + lane]
    int* lv = reinterpret_cast<int*>(red + R * 4 * 64);    // lv[buf PC + c]
    if (wv == 0 || wv == 6) {
        // ---- solver wave(s): right-hand side rs
        const int rs = wv == 0 ? 0 : 1;
        double eps[1] = {epsp[rs]}, zown[1];
        int bad[1] = {};
        zown[0] = lane < min(PC, nt) ? V.z[rs * V.zs + tc + lane] : 0.0;
#ifdef IPO_LEAD_STAMPS
        long long sa = 0, st = 0, sb = 0;
#endif
        lds_sync();                                                      // B_{-1}
        for (int i = 0; i < ntb; i++) {
            LEAD_T(t0);
            const int k0 = i * PC, nc = min(PC, nt - k0);
            double znext;
            const int k1 = k0 + PC, nc1 = i + 1 < ntb ? min(PC, nt - k1) : 0;
            znext = lane < nc1 ? V.z[rs * V.zs + tc + k1 + lane] : 0.0;
            lds_sync();                                                  // A_i
            LEAD_T(t1);
            double zr[1];
            {
                const double* rd = red + rs * 4 * 64 + lane;
                zr[0] = lane < nc ? zown[0] - (((rd[0] + rd[64]) + rd[128]) + rd[192]) : 0.0;
            }
            tri_lower<1, true>(zr, Ls[i & 1], lv + (i & 1) * PC, nc, eps, bad);
            LEAD_T(t2);
            if (lane < nc) {
                gran_put(gran + (((size_t)i * R + rs) * 64 + lane) * 2, epoch, zr[0]);
                V.z[rs * V.zs + tc + k0 + lane] = zr[0];
            }
            zh[((i % K) * R + rs) * PC + lane] = lane < nc ? zr[0] : 0.0;
            zown[0] = znext;
            lds_sync();                                                  // B_i
#ifdef IPO_LEAD_STAMPS
            LEAD_T(t3);
            sa += t1 - t0; st += t2 - t1; sb += t3 - t2;
#endif
        }
#ifdef IPO_LEAD_STAMPS
        if (lane == 0 && wv == 0) {
            g_lead_stats[0][0] = sa * 0.01 / ntb; g_lead_stats[0][1] = st * 0.01 / ntb;
            g_lead_stats[0][2] = sb * 0.01 / ntb;
        }
#endif
        if (bad[0]) atomicOr(&p.incons[rs], 1);
        return;
    }
    // ---- product waves
    // buffer loads: the per-column offsets are scalars, only the row offset
    // is a per-lane register (64 global loads would each hold a 64-bit address)
    const __amdgpu_buffer_rsrc_t rs = tail_rsrc(tv.S);
    const int nt8 = nt * 8, g16 = __builtin_amdgcn_readfirstlane(g * 16);
    auto load_tiles = [&](int i, double(&t)[K][16]) {     // L(i, j), j = i-K .. i-1 (j >= 0)
        const int k0 = i * PC, nc = min(PC, nt - k0);
        const int voff = (k0 + (lane < nc ? lane : 0)) * 8;
#pragma unroll
        for (int b = 0; b < K; b++) {
            const int s0 = (max(i - K + b, 0) * PC + g16) * nt8;
#pragma unroll
            for (int q = 0; q < 16; q++) t[b][q] = buf_ld(rs, voff, s0 + q * nt8);
        }
    };
    // L11 of block i (stage_l11's rows r = g + 4q of Ls[r][c] = L(r, c), c < r)
    // and its live marks, loaded into registers a step before they are stored
    auto l11_load = [&](int i, double(&t)[16], int& lvv) {
        const int k0 = i * PC, nc = min(PC, nt - k0);
        const int voff = (k0 + lane) * 8;
#pragma unroll
        for (int q = 0; q < 16; q++) {
            const int r = g + 4 * q;
            const bool ok = r < nc && lane < r;
            t[q] = buf_ld(rs, ok ? voff : 0, min(k0 + r, nt - 1) * nt8);   // masked when stored
        }
        lvv = p.live[tc + k0 + min(pl, nc - 1)];
    };
    auto l11_store = [&](int i, const double(&t)[16], int lvv) {
        const int nc = min(PC, nt - i * PC);
#pragma unroll
        for (int q = 0; q < 16; q++) {
            const int r = g + 4 * q;
            Ls[i & 1][r][lane] = r < nc && lane < r ? t[q] : 0.0;
        }
        if (pl < nc) lv[(i & 1) * PC + pl] = lvv;
    };
    unsigned long long praw[R][2];
    auto part_load = [&](int i) {
#pragma unroll
        for (int r = 0; r < R; r++) {
            const gran_t* q = part_slot(pgran, i, R, r, g, lane);
            praw[r][0] = __hip_atomic_load(const_cast<gran_t*>(q), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            praw[r][1] = __hip_atomic_load(const_cast<gran_t*>(q + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    };
    double pre[R];
#pragma unroll
    for (int r = 0; r < R; r++) pre[r] = 0.0;
    double tA[K][16], tB[K][16], lA[16], lB[16];
    int vA, vB;
#ifdef IPO_LEAD_STAMPS
    long long pw = 0, p3 = 0, p4 = 0;
    int polls = 0;
#endif
    l11_load(0, lA, vA);
    l11_store(0, lA, vA);
    load_tiles(min(1, ntb - 1), tB);
    l11_load(min(1, ntb - 1), lB, vB);
    part_load(min(1, ntb - 1));
    lds_sync();                                                          // B_{-1}
    // cur / lcur: step i's tiles (and the L11 slot to refill), nxt / lnxt: step i+1's
    auto step = [&](int i, double(&cur)[K][16], double(&nxt)[K][16], double(&lcur)[16], int& vcur,
                    double(&lnxt)[16], int& vnxt) {
        double acc[R];
#pragma unroll
        for (int r = 0; r < R; r++) acc[r] = pre[r];
        if (i >= 1) {                                  // the last term: z_{i-1}
            const double* z = zh + ((i - 1) % K) * R * PC + g * 16;
#pragma unroll
            for (int q = 0; q < 16; q++) {
#pragma unroll
                for (int r = 0; r < R; r++) acc[r] += cur[K - 1][q] * z[r * PC + q];
            }
        }
#pragma unroll
        for (int r = 0; r < R; r++) red[(r * 4 + g) * 64 + lane] = acc[r];
        lds_sync();                                                      // A_i
        LEAD_T(u0);
        if (i + 1 < ntb) {
            l11_store(i + 1, lnxt, vnxt);
            if (i + 1 > K) {                           // helper i+1-K's partial (j <= i-K)
                for (;;) {
                    bool ok = true;
#pragma unroll
                    for (int r = 0; r < R; r++) ok &= (praw[r][0] >> 32) == epoch && (praw[r][1] >> 32) == epoch;
                    if (__all(ok)) break;
#ifdef IPO_LEAD_STAMPS
                    polls++;
#endif
                    __builtin_amdgcn_s_sleep(IPO_POLL_SLEEP);
                    part_load(i + 1);
                }
                LEAD_T(u1);
#ifdef IPO_LEAD_STAMPS
                pw += u1 - u0;
#endif
#pragma unroll
                for (int r = 0; r < R; r++)
                    pre[r] = __longlong_as_double(static_cast<long long>(((praw[r][1] & 0xffffffffull) << 32) |
                                                                         (praw[r][0] & 0xffffffffull)));
            } else {
#pragma unroll
                for (int r = 0; r < R; r++) pre[r] = 0.0;
            }
#pragma unroll
            for (int b = 0; b < K - 1; b++) {          // j = i+1-K .. i-1, in order
                const int j = i + 1 - K + b;
                if (j >= 0) {
                    const double* z = zh + (j % K) * R * PC + g * 16;
#pragma unroll
                    for (int q = 0; q < 16; q++) {
#pragma unroll
                        for (int r = 0; r < R; r++) pre[r] += nxt[b][q] * z[r * PC + q];
                    }
                }
                __builtin_amdgcn_sched_barrier(0);     // z reads one tile at a time (registers)
            }
        }
        LEAD_T(u2);
        // step i+2's loads, unconditional (clamped in range: a conditional
        // load would keep the old registers live across the branch)
        const int i2 = min(i + 2, ntb - 1);
        load_tiles(i2, cur);
        l11_load(i2, lcur, vcur);
        part_load(i2);
        LEAD_T(u3);
#ifdef IPO_LEAD_STAMPS
        p3 += u2 - u0; p4 += u3 - u2;
#endif
        lds_sync();                                                      // B_i
    };
    int i = 0;
    for (; i + 1 < ntb; i += 2) {      // two steps per trip, unconditionally (no register merges)
        step(i, tA, tB, lA, vA, lB, vB);
        step(i + 1, tB, tA, lB, vB, lA, vA);
    }
    if (i < ntb) step(i, tA, tB, lA, vA, lB, vB);
#ifdef IPO_LEAD_STAMPS
    if (lane == 0) {
        g_lead_stats[wv][0] = pw * 0.01 / ntb; g_lead_stats[wv][1] = polls;
        g_lead_stats[wv][2] = p3 * 0.01 / ntb; g_lead_stats[wv][3] = p4 * 0.01 / ntb;
    }
#endif
}

// ------------------------------------------- sync-free sweeps, top levels
// The narrow top of the elimination tree (levels >= sf_level_, a few
// supernodes each) in one persistent launch per direction instead of one or
// two launches per level.  One workgroup per CU (dynamic LDS).  Workgroups
// draw the work items in list order from a global ticket counter (one
// agent-scope atomic per item, drawn one item ahead), and an item only waits
// on items earlier in the list (descendants forward, ancestors backward).
// An item is therefore only ever held by a running workgroup, and every item
// it waits on was drawn earlier by a running workgroup: the grid drains
// whatever share of the CUs the launch gets (co-tenant kernels, several
// shards on one device).  The counter is never reset within a run: each
// launch draws exactly nitems + gridDim.x tickets (every workgroup stops at
// its first ticket past the list), so the host passes the launch's base.  Items: (s, -1) a whole supernode, (s, -2) the
// diagonal part (forward) / the finish (backward) of a chunked supernode,
// (s, c >= 0) its 64-row chunk c.  Hand-offs follow MI355X_MICROARCH.md
// (inter-workgroup visibility, table row 1): the producer writes the values
// with sc1 stores, waits vmcnt(0), joins a barrier, and one lane adds to
// the consumer's counter or stores a flag (agent scope); the consumer polls
// from one lane, joins a barrier and reads the values with sc1 loads.  Each
// handed-off value sits in 128-B lines of its own producer (padded ybuf
// slices, the zpad mirror, per-chunk partials), written once per sweep, so
// no consumer can have cached a line before its producer wrote it.  The
// arithmetic per supernode is that of the per-level kernels (bitwise).
constexpr int kSfIdx = static_cast<int>(kChainLds / sizeof(int));   // update-list indices staged per item

struct SfView {
    const int2* items;
    int nitems;
    int* cnt;           // per supernode: arrivals (forward: child y producers; backward: chunks)
    int* flag;          // per supernode: epoch of its completed diagonal part (fwd) / finish (bwd)
    const int* need;    // per supernode: forward arrivals per sweep
    const int* parent;  // per supernode: parent inside the range, else -1
    const int* zbase;   // per supernode: its padded z slice
    const int* zpi;     // per column: padded z position, -1 outside the range
    double* zpad;       // padded z slices of R right-hand sides
    size_t zps;
    int epoch;
    int* ticket;        // work-item counter (see above)
    int tbase;          // its value when this launch starts
};

// next work item of this workgroup: thread 0's ticket, through LDS
__device__ __forceinline__ int sf_draw(const SfView& sf) {
    return __hip_atomic_fetch_add(sf.ticket, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - sf.tbase;
}
// End of an item: the next ticket goes to LDS before the item's last
// barrier (no extra barrier), then the hand-off of MI355X_MICROARCH.md.
__device__ __forceinline__ void sf_next(int* tk, int nxt) {
    if (threadIdx.x == 0) *tk = nxt;
    __syncthreads();
}

__device__ __forceinline__ void sf_arrive_next(int* c, int* tk, int nxt) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (threadIdx.x == 0) *tk = nxt;
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_fetch_add(c, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void sf_publish_next(int* flags, int i, int epoch, int* tk, int nxt) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (threadIdx.x == 0) *tk = nxt;
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_store(flags + i, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}


// Forward pre-pass of deep trees (build_sync_free_plan): z_c -= the sum of
// the update values column c of the narrow range receives from below the
// range, in list order, one thread per column (eight loads in flight).
template <int R>
__global__ void __launch_bounds__(NT)
k_fwd_pre(int ncols, const int* __restrict__ col, const int* __restrict__ eptr, const int* __restrict__ eidx,
          SweepVecs V) {
    const int j = blockIdx.x * NT + threadIdx.x;
    if (j >= ncols) return;
    const int c = col[j];
    double acc[R];
#pragma unroll
    for (int r = 0; r < R; r++) acc[r] = 0.0;
    int e = eptr[j];
    const int e1 = eptr[j + 1];
    for (; e + 7 < e1; e += 8) {
        int ix[8];
#pragma unroll
        for (int u = 0; u < 8; u++) ix[u] = eidx[e + u];
#pragma unroll
        for (int r = 0; r < R; r++) {
            double yv[8];
#pragma unroll
            for (int u = 0; u < 8; u++) yv[u] = V.y[r * V.ys + ix[u]];
#pragma unroll
            for (int u = 0; u < 8; u++) acc[r] += yv[u];
        }
    }
    for (; e < e1; e++) {
        const int i0 = eidx[e];
#pragma unroll
        for (int r = 0; r < R; r++) acc[r] += V.y[r * V.ys + i0];
    }
#pragma unroll
    for (int r = 0; r < R; r++) V.z[r * V.zs + c] -= acc[r];
}

template <int R>
__global__ void __launch_bounds__(NT)
k_fwd_sf(PlanView p, SfView sf, const int* __restrict__ yrow_ptr, const int* __restrict__ yrow_idx,
         const int* __restrict__ chunk_r0, SweepVecs V, const double* __restrict__ epsp) {
    extern __shared__ double lds_pad[];
    __shared__ double zl[R][PC];
    __shared__ double Ls[PC][PC + 1];
    __shared__ int lv[PC];
    __shared__ double red[R][4][64];
    __shared__ int sptr[PC + 1];
    double eps[R];
    load_eps<R>(epsp, eps);
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    __shared__ int tk[2];
    if (tid == 0) { lds_pad[0] = 0.0; tk[0] = sf_draw(sf); }
    __syncthreads();
    for (int par_ = 0;; par_ ^= 1) {
        const int it = tk[par_];
        if (it >= sf.nitems) break;
        // the next item's ticket is drawn once this item's wait is over (its
        // atomic then overlaps the item's work, not the wait) and stored at
        // the item's last barrier
        int nxt = 0;
        int* const slot = &tk[par_ ^ 1];
        SF_STAMP(it, 0);
        const int2 w = sf.items[it];
        const int s = w.x, code = w.y;
        const int c0 = p.col0[s], nc = p.col0[s + 1] - c0;
        const int hb = p.rowptr[s + 1] - p.rowptr[s], h = nc + hb;
        const int par = sf.parent[s];
        const double* panel = p.Lx + p.off[s];
        if (code == -1) {
            // the factor does not depend on the hand-off: L11, the marks and
            // (whole supernodes, hb <= 128 rows: one per thread) this
            // thread's row of L21 are loaded before the wait
            double lr[PC];
            const bool pre = code == -1 && hb <= NT && tid < hb;
            if (code == -1 && hb > 0) {
                const double* __restrict__ row = panel + nc + min(tid, hb - 1);
#pragma unroll
                for (int k = 0; k < PC; k++) lr[k] = row[(size_t)min(k, nc - 1) * h];
            }
            stage_l11(panel, h, nc, Ls);
            if (tid < nc) lv[tid] = p.live[c0 + tid];
            // the update-list indices do not depend on the hand-off either
            const int eb = yrow_ptr[c0], ne = yrow_ptr[c0 + nc] - eb;
            int* sidx = reinterpret_cast<int*>(lds_pad);
            const bool stg = ne <= kSfIdx;
            if (stg)
                for (int e = tid; e < ne; e += NT) sidx[e] = yrow_idx[eb + e];
            if (tid <= nc) sptr[tid] = yrow_ptr[c0 + tid];
            chain_wait(sf.cnt, s, sf.epoch * sf.need[s]);
            SF_STAMP(it, 1);
            if (tid == 0) nxt = sf_draw(sf);
            SF_NOTE(it, 6, ne);
            fwd_diag<R, true, true>(p, s, yrow_ptr, yrow_idx, V, eps, zl, Ls, lv, stg ? sidx : nullptr, it,
                                    stg ? sptr : nullptr);
            SF_STAMP(it, 2);
            if (code == -1) {       // y_s = L21 z_s, one row per thread (k_forward)
                if (pre) {
                    double acc[R];
#pragma unroll
                    for (int r = 0; r < R; r++) acc[r] = 0.0;
#pragma unroll
                    for (int k = 0; k < PC; k++)
                        if (k < nc) {
#pragma unroll
                            for (int r = 0; r < R; r++) acc[r] += lr[k] * zl[r][k];
                        }
#pragma unroll
                    for (int r = 0; r < R; r++) sc1_store(V.y + r * V.ys + p.ybase[s] + tid, acc[r]);
                }
                for (int i = hb <= NT ? hb : tid; i < hb; i += NT) {
                    const double* __restrict__ row = panel + nc + i;
                    double acc[R];
#pragma unroll
                    for (int r = 0; r < R; r++) acc[r] = 0.0;
#pragma unroll 8
                    for (int k = 0; k < nc; k++) {
                        const double l = row[(size_t)k * h];
#pragma unroll
                        for (int r = 0; r < R; r++) acc[r] += l * zl[r][k];
                    }
#pragma unroll
                    for (int r = 0; r < R; r++) sc1_store(V.y + r * V.ys + p.ybase[s] + i, acc[r]);
                }
                if (par >= 0) { SF_STAMP(it, 3); sf_arrive_next(sf.cnt + par, slot, nxt); SF_STAMP(it, 4); }
                else { SF_STAMP(it, 3); sf_next(slot, nxt); SF_STAMP(it, 4); }
            }
        } else {
            // one 64-row chunk of a chunked supernode: the diagonal part
            // (every chunk item of the supernode solves it, so the chain
            // has one hand-off per level, not two; z_s to the zpad mirror,
            // whence the backward sweep takes it), then y over the chunk's
            // rows (k_fwd_gemv)
            const int i = chunk_r0[code] + lane, kq = wv * 16, nq = min(16, nc - kq);
            double t[16];             // the factor tile, L11, the marks and the list indices before the wait
            {
                const double* __restrict__ row = panel + nc + min(i, hb - 1) + (size_t)(nq > 0 ? kq : 0) * h;
#pragma unroll
                for (int q = 0; q < 16; q++) t[q] = row[(size_t)min(q, max(nq, 1) - 1) * h];
            }
            stage_l11(panel, h, nc, Ls);
            if (tid < nc) lv[tid] = p.live[c0 + tid];
            const int eb = yrow_ptr[c0], ne = yrow_ptr[c0 + nc] - eb;
            int* sidx = reinterpret_cast<int*>(lds_pad);
            const bool stg = ne <= kSfIdx;
            if (stg)
                for (int e = tid; e < ne; e += NT) sidx[e] = yrow_idx[eb + e];
            if (tid <= nc) sptr[tid] = yrow_ptr[c0 + tid];
            chain_wait(sf.cnt, s, sf.epoch * sf.need[s]);
            SF_STAMP(it, 1);
            if (tid == 0) nxt = sf_draw(sf);
            fwd_diag<R, true, true>(p, s, yrow_ptr, yrow_idx, V, eps, zl, Ls, lv, stg ? sidx : nullptr, it,
                                    stg ? sptr : nullptr, sf.zpad + sf.zbase[s], sf.zps);
            SF_STAMP(it, 2);
            double acc[R];
#pragma unroll
            for (int r = 0; r < R; r++) acc[r] = 0.0;
            if (i < hb && nq > 0) {
#pragma unroll
                for (int q = 0; q < 16; q++)
                    if (q < nq) {
#pragma unroll
                        for (int r = 0; r < R; r++) acc[r] += t[q] * zl[r][kq + q];
                    }
            }
#pragma unroll
            for (int r = 0; r < R; r++) red[r][wv][lane] = acc[r];
            __syncthreads();
            if (wv == 0 && i < hb) {
#pragma unroll
                for (int r = 0; r < R; r++)
                    sc1_store(V.y + r * V.ys + p.ybase[s] + i,
                              ((red[r][0][lane] + red[r][1][lane]) + red[r][2][lane]) + red[r][3][lane]);
            }
            if (par >= 0) { SF_STAMP(it, 3); sf_arrive_next(sf.cnt + par, slot, nxt); SF_STAMP(it, 4); }
            else { SF_STAMP(it, 3); sf_next(slot, nxt); SF_STAMP(it, 4); }
        }
    }
}

// z of row ri for the backward sweep: the padded mirror inside the range
// (pi = sf.zpi[ri], looked up before the hand-off wait)
template <int R>
__device__ __forceinline__ void sf_zrow(const SfView& sf, const SweepVecs& V, int ri, int pi, double (&zi)[R]) {
#pragma unroll
    for (int r = 0; r < R; r++) zi[r] = pi >= 0 ? sc1_load(sf.zpad + r * sf.zps + pi) : V.z[r * V.zs + ri];
}

// Wave r of a backward item solves right-hand side r (the R chains are
// independent; one wave each): z_s = D^-1 z_s - sub (dscale_rule on the
// prefetched own z, d, mark; ldlt.c:473-480), then L11', z_s to z and to the
// zpad mirror.  sub = the four wave partials of xs summed in k_bwd_finish's
// order (chunked supernodes) or xs[r][0] (whole ones).
template <int R>
__device__ __forceinline__ void bwd_sf_solve(const PlanView& p, const SfView& sf, const SweepVecs& V, int s, int c0,
                                             int nc, bool chunked, double zo, int lvo, double dgo,
                                             const double (&eps)[R], const double (*Ls)[PC + 1], const int* lv,
                                             const double (*xs)[4][PC], int r) {
    const int lane = threadIdx.x & 63;
    const double e1[1] = {r == 0 ? eps[0] : eps[R - 1]};
    int bad[1] = {};
    double zr[1];
    {
        const double sub = chunked ? ((xs[r][0][lane] + xs[r][1][lane]) + xs[r][2][lane]) + xs[r][3][lane]
                                   : xs[r][0][lane];
        double zd = 0.0;
        if (lane < nc) {
            zd = zo;
            if (lvo) zd = zd / dgo;
            else if (fabs(zd) > e1[0]) bad[0] = 1;
            else zd = 0.0;
        }
        zr[0] = lane < nc ? zd - sub : 0.0;
    }
    tri_upper<1, true>(zr, Ls, lv, nc, e1, bad);
    if (lane < nc) {
        V.z[r * V.zs + c0 + lane] = zr[0];
        sc1_store(sf.zpad + r * sf.zps + sf.zbase[s] + lane, zr[0]);
    }
    if (bad[0]) atomicOr(&p.incons[r], 1);
}

template <int R>
__global__ void __launch_bounds__(NT)
k_bwd_sf(PlanView p, SfView sf, const int* __restrict__ chunk_r0, const int* __restrict__ sup_chunk0,
         double* __restrict__ part, size_t ps, SweepVecs V, const double* __restrict__ epsp) {
    extern __shared__ double lds_pad[];
    __shared__ double Ls[PC][PC + 1];     // Ls[j][r] = L(j, r)
    __shared__ int lv[PC];
    __shared__ double xs[R][4][PC];
    double eps[R];
    load_eps<R>(epsp, eps);
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    double* red = lds_pad;   // colsum scratch
    __shared__ int tk[2];
    __shared__ int lastc;
    if (tid == 0) { lds_pad[0] = 0.0; tk[0] = sf_draw(sf); }
    __syncthreads();
    for (int par_ = 0;; par_ ^= 1) {
        const int it = tk[par_];
        if (it >= sf.nitems) break;
        int nxt = 0;                // next ticket: drawn after this item's wait, stored at its last barrier
        int* const slot = &tk[par_ ^ 1];
        const int2 w = sf.items[it];
        const int s = w.x, code = w.y;
        const int c0 = p.col0[s], nc = p.col0[s + 1] - c0;
        const int hb = p.rowptr[s + 1] - p.rowptr[s], h = nc + hb;
        const int par = sf.parent[s];
        const double* panel = p.Lx + p.off[s];
        const int* __restrict__ rows = p.rows + p.rowptr[s];
        const int kq = wv * 16, nq = min(16, nc - kq);
        if (code >= 0) {
            // partial sums of one 64-row chunk (k_bwd_partial); the chunk
            // whose arrival comes last finishes the supernode (k_bwd_finish:
            // the partials in its order, D^-1, L11') -- one hand-off per
            // level instead of a finish item waiting on the chunks
            const int i = chunk_r0[code] + lane;
            const bool okr = i < hb;
            const int ic = okr ? i : 0;
            const int ri = rows[ic];
            const int pi = sf.zpi[ri];
            double t[16];             // the factor tile, L11, the own z / d / mark before the wait
            const double* __restrict__ col = panel + nc + ic + (size_t)(nq > 0 ? kq : 0) * h;
#pragma unroll
            for (int q = 0; q < 16; q++) t[q] = col[(size_t)min(q, max(nq, 1) - 1) * h];
            stage_l11(panel, h, nc, Ls);
            if (tid < nc) lv[tid] = p.live[c0 + tid];
            double zown = 0.0, dgo = 1.0;     // of the right-hand side wave wv < R solves
            int lvo = 1;
            if (wv < R && lane < nc) {
                zown = sc1_load(sf.zpad + wv * sf.zps + sf.zbase[s] + lane);
                lvo = p.live[c0 + lane];
                dgo = p.dg[c0 + lane];
            }
            if (par >= 0) chain_wait(sf.flag, par, sf.epoch);
            if (tid == 0) nxt = sf_draw(sf);
            if (nq > 0) {
                double zi[R], v[R][16];
                sf_zrow<R>(sf, V, ri, pi, zi);
#pragma unroll
                for (int r = 0; r < R; r++)
#pragma unroll
                    for (int q = 0; q < 16; q++) v[r][q] = okr ? t[q] * zi[r] : 0.0;
                colsum_put<R>(red, v, kq, nq, lane);
            }
            __syncthreads();
            if (tid < R * PC && tid % PC < nc)
                sc1_store(part + (tid / PC) * ps + (size_t)code * PC + tid % PC, colsum_tree(red, tid / PC, tid % PC));
            const int nch = (hb + 63) / 64;
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            if (tid == 0) {
                const int prev = __hip_atomic_fetch_add(sf.cnt + s, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                lastc = prev + 1 == sf.epoch * nch;
                *slot = nxt;
            }
            __syncthreads();
            if (!lastc) continue;
            const int cf = sup_chunk0[s];
            double x[R];
#pragma unroll
            for (int r = 0; r < R; r++) x[r] = 0.0;
            if (lane < nc)
                for (int c = wv; c < nch; c += 4) {
#pragma unroll
                    for (int r = 0; r < R; r++) x[r] += sc1_load(part + r * ps + (size_t)(cf + c) * PC + lane);
                }
#pragma unroll
            for (int r = 0; r < R; r++) xs[r][wv][lane] = x[r];
            __syncthreads();
            if (wv < R) bwd_sf_solve<R>(p, sf, V, s, c0, nc, true, zown, lvo, dgo, eps, Ls, lv, xs, wv);
            sf_publish_next(sf.flag, s, sf.epoch, slot, nxt);
            continue;
        }
        // nothing below depends on the hand-off but the z values of the
        // ancestors' rows and the chunk partials: L11, the marks, this
        // block's own z / d / mark (D^-1 z) and, for a whole supernode
        // (hb <= 128: two rows per lane at most), its L21 tiles and row
        // lookups are loaded before the wait
        stage_l11(panel, h, nc, Ls);
        if (tid < nc) lv[tid] = p.live[c0 + tid];
        double zown = 0.0, dgo = 1.0;     // of the right-hand side wave wv < R solves
        int lvo = 1;
        if (wv < R && lane < nc) {
            // a chunked supernode's forward z_s is in the zpad mirror (k_fwd_sf)
            zown = code == -2 ? sc1_load(sf.zpad + wv * sf.zps + sf.zbase[s] + lane) : V.z[wv * V.zs + c0 + lane];
            lvo = p.live[c0 + lane];
            dgo = p.dg[c0 + lane];
        }
        constexpr int kPre = 2;       // rows per lane prefetched (hb <= 128)
        double tp[kPre][16];
        int rip[kPre], pip[kPre];
        const bool pre = code == -1 && hb <= 64 * kPre && nq > 0;
        if (pre) {
#pragma unroll
            for (int u = 0; u < kPre; u++) {
                const int i = min(lane + 64 * u, max(hb - 1, 0));
                rip[u] = hb > 0 ? rows[i] : 0;
                const double* __restrict__ col = panel + nc + i + (size_t)kq * h;
#pragma unroll
                for (int q = 0; q < 16; q++) tp[u][q] = col[(size_t)min(q, nq - 1) * h];
            }
#pragma unroll
            for (int u = 0; u < kPre; u++) pip[u] = hb > 0 ? sf.zpi[rip[u]] : -1;
        }
        if (code == -2) chain_wait(sf.cnt, s, sf.epoch * ((hb + 63) / 64));
        else if (par >= 0) chain_wait(sf.flag, par, sf.epoch);
        if (tid == 0) nxt = sf_draw(sf);
        if (code == -2) {           // chunk partials in the order of k_bwd_finish
            const int cf = sup_chunk0[s], nch = (hb + 63) / 64;
            double x[R];
#pragma unroll
            for (int r = 0; r < R; r++) x[r] = 0.0;
            if (lane < nc)
                for (int c = wv; c < nch; c += 4) {
#pragma unroll
                    for (int r = 0; r < R; r++) x[r] += sc1_load(part + r * ps + (size_t)(cf + c) * PC + lane);
                }
#pragma unroll
            for (int r = 0; r < R; r++) xs[r][wv][lane] = x[r];
        } else if (pre) {           // L21' z_R from the prefetched tiles (same sums as below)
            double acc[R][16];
#pragma unroll
            for (int r = 0; r < R; r++)
#pragma unroll
                for (int q = 0; q < 16; q++) acc[r][q] = 0.0;
            double zi[kPre][R];
#pragma unroll
            for (int u = 0; u < kPre; u++)
                if (lane + 64 * u < hb) sf_zrow<R>(sf, V, rip[u], pip[u], zi[u]);
#pragma unroll
            for (int u = 0; u < kPre; u++)
                if (lane + 64 * u < hb) {
#pragma unroll
                    for (int q = 0; q < 16; q++)
                        if (q < nq) {
#pragma unroll
                            for (int r = 0; r < R; r++) acc[r][q] += tp[u][q] * zi[u][r];
                        }
                }
            colsum_put<R>(red, acc, kq, nq, lane);
        } else if (nq > 0) {        // L21' z_R over all rows (k_backward)
            double acc[R][16];
#pragma unroll
            for (int r = 0; r < R; r++)
#pragma unroll
                for (int q = 0; q < 16; q++) acc[r][q] = 0.0;
            for (int i = lane; i < hb; i += 64) {
                double zi[R];
                sf_zrow<R>(sf, V, rows[i], sf.zpi[rows[i]], zi);
                const double* __restrict__ col = panel + nc + i + (size_t)kq * h;
                double t[16];
#pragma unroll
                for (int q = 0; q < 16; q++) t[q] = col[(size_t)min(q, nq - 1) * h];
#pragma unroll
                for (int q = 0; q < 16; q++)
                    if (q < nq) {
#pragma unroll
                        for (int r = 0; r < R; r++) acc[r][q] += t[q] * zi[r];
                    }
            }
            colsum_put<R>(red, acc, kq, nq, lane);
        }
        __syncthreads();
        if (code != -2) {
            if (tid < R * PC && tid % PC < nc) xs[tid / PC][0][tid % PC] = colsum_tree(red, tid / PC, tid % PC);
            __syncthreads();
        }
        if (wv < R) bwd_sf_solve<R>(p, sf, V, s, c0, nc, code == -2, zown, lvo, dgo, eps, Ls, lv, xs, wv);
        sf_publish_next(sf.flag, s, sf.epoch, slot, nxt);
    }
}

// -------------------------------------------------------- refinement glue
// The refinement pass's per-system launches, both active systems in one
// launch (blockIdx.y = the system's slot q; the refinement phase is
// host-bound, so a launch saved is time saved)
struct PermJobs {
    const double* fy[2];
    const double* fx[2];
    double* z[2];
    double* dy[2];
    double* dx[2];
    int mode[2];
};
// z[v] = rhs(perm[v]) with rhs = (fy | fx); the pass's first permutation also
// clears the consistency flags and the dropped-column eps of its sweep
// (zi[0..1], zd[0..1]; no fill launches)
__global__ void __launch_bounds__(NT)
k_perm_in2(int T, int m, const int* __restrict__ perm, PermJobs J, int* __restrict__ zi, double* __restrict__ zd) {
    const int v = blockIdx.x * NT + threadIdx.x, q = blockIdx.y;
    if (q == 0 && v < 2 && zi) { zi[v] = 0; zd[v] = 0.0; }
    if (v >= T) return;
    const int o = perm[v];
    J.z[q][v] = o < m ? J.fy[q][o] : J.fx[q][o - m];
}
// dy/dx (=|+=|-=) z[iperm[.]]
__global__ void __launch_bounds__(NT)
k_perm_out2(int T, int m, const int* __restrict__ iperm, PermJobs J) {
    const int o = blockIdx.x * NT + threadIdx.x, q = blockIdx.y;
    if (o >= T) return;
    const double v = J.z[q][iperm[o]];
    double* dst = o < m ? J.dy[q] + o : J.dx[q] + (o - m);
    const int mode = J.mode[q];
    if (mode == 0) *dst = v;
    else if (mode == 1) *dst = *dst + v;
    else *dst = *dst - v;
}

// dy/dx (=|+=|-=) z[iperm[.]]
__global__ void __launch_bounds__(NT)
k_perm_out(int T, int m, const int* __restrict__ iperm, const double* __restrict__ z, double* __restrict__ dy,
           double* __restrict__ dx, int mode) {
    const int o = blockIdx.x * NT + threadIdx.x;
    if (o >= T) return;
    const double v = z[iperm[o]];
    double* dst = o < m ? dy + o : dx + (o - m);
    if (mode == 0) *dst = v;
    else if (mode == 1) *dst = *dst + v;
    else *dst = *dst - v;
}

// KKT residual (ldlt.c:389-398):
//   ry_j = fy_j - ((A dx)_j - E_j dy_j)        row gather over CSR
//   rx_i = fx_i - ((A' dy)_i + D_i dx_i)       column gather over CSC
// plus max-abs partials of both (ldlt.c:401).
__device__ __forceinline__ void kkt_residual_body(
    int m, int n, const int* __restrict__ kAt, const int* __restrict__ iAt, const double* __restrict__ At,
    const int* __restrict__ kA, const int* __restrict__ iA, const double* __restrict__ A, const double* __restrict__ E,
    const double* __restrict__ D, const double* __restrict__ fy, const double* __restrict__ fx,
    const double* __restrict__ dy, const double* __restrict__ dx, double* __restrict__ ry, double* __restrict__ rx,
    double* __restrict__ part, int mrow, const double* __restrict__ axl, const int* __restrict__ kQ,
    const int* __restrict__ iQ, const double* __restrict__ Q, double qmax) {
    __shared__ double sh[kResThreads / 64];
    double mx = 0.0;
    for (int i = blockIdx.x * kResThreads + threadIdx.x; i < m + n; i += kRedBlocks * kResThreads) {
        if (i < m) {
            double s = 0.0;
            if (i >= mrow) s = axl[i - mrow];      // linking row: product summed over the shards
            else
                s = sparse_dot(kAt[i], kAt[i + 1], At, iAt, dx);
            // a Q block: fy - ((A dx - E dy) - max Q dy), ldlt.c:391-394
            // (Q symmetric: row i of Q dy summed over its column i in order)
            const double r = kQ ? fy[i] - ((s - E[i] * dy[i]) - qmax * sparse_dot(kQ[i], kQ[i + 1], Q, iQ, dy))
                                : fy[i] - (s - E[i] * dy[i]);
            ry[i] = r;
            mx = fmax(mx, ref_abs(r));
        } else {
            const int j = i - m;
            double s = 0.0;
            s = sparse_dot(kA[j], kA[j + 1], A, iA, dy);
            const double r = fx[j] - (s + D[j] * dx[j]);
            rx[j] = r;
            mx = fmax(mx, ref_abs(r));
        }
    }
    mx = block_max_w<kResThreads / 64>(mx, sh);
    if (threadIdx.x == 0) part[blockIdx.x] = mx;
}


struct ResJobs {
    const double* fy[2];
    const double* fx[2];
    const double* dy[2];
    const double* dx[2];
    double* ry[2];
    double* rx[2];
    const double* axl[2];
};
// the active systems' residuals, one launch: system q = blockIdx.y writes
// the partials of slot q (part + q kRedBlocks)
__global__ void __launch_bounds__(kResThreads)
k_kkt_residual2(int m, int n, const int* __restrict__ kAt, const int* __restrict__ iAt, const double* __restrict__ At,
                const int* __restrict__ kA, const int* __restrict__ iA, const double* __restrict__ A,
                const double* __restrict__ E, const double* __restrict__ D, ResJobs J, double* __restrict__ part,
                int mrow, const int* __restrict__ kQ, const int* __restrict__ iQ, const double* __restrict__ Q,
                double qmax) {
    const int q = blockIdx.y;
    kkt_residual_body(m, n, kAt, iAt, At, kA, iA, A, E, D, J.fy[q], J.fx[q], J.dy[q], J.dx[q], J.ry[q], J.rx[q],
                      part + (size_t)q * kRedBlocks, mrow, J.axl[q], kQ, iQ, Q, qmax);
}

// -min|d| partials, so that the max-finisher yields -min|d| (negated on host)
__global__ void __launch_bounds__(NT)
k_min_abs_partial(const double* __restrict__ d, int T, double* __restrict__ part) {
    __shared__ double sh[4];
    double mn = HUGE_VAL;
    for (int i = blockIdx.x * NT + threadIdx.x; i < T; i += kRedBlocks * NT) mn = fmin(mn, ref_abs(d[i]));
    const double r = block_max(-mn, sh);
    if (threadIdx.x == 0) part[blockIdx.x] = r;
}

__global__ void k_scale_scalar(double* e, int n, double f) { if (static_cast<int>(threadIdx.x) < n) e[threadIdx.x] *= f; }
// dst[2r] <- src[2r] (m values), dst[2r+1] <- src[2r+1] (n values), r < R
struct CopyOut {
    const double* src[4];
    double* dst[4];
    int m, n, R;
};
__global__ void __launch_bounds__(NT) k_copy_out(CopyOut c) {
    const int i = blockIdx.x * NT + threadIdx.x, per = c.m + c.n;
    if (i >= c.R * per) return;
    const int r = i / per, k = i - r * per;
    if (k < c.m) c.dst[2 * r][k] = c.src[2 * r][k];
    else c.dst[2 * r + 1][k - c.m] = c.src[2 * r + 1][k - c.m];
}
// n ints copied bit for bit into the doubles at out (one host read-back with them)
__global__ void k_pack_ints(const int* f, int n, double* out) {
    if (static_cast<int>(threadIdx.x) < n) reinterpret_cast<int*>(out)[threadIdx.x] = f[threadIdx.x];
}
__global__ void k_flag_to_scalar(const int* f, double* d) { d[0] = static_cast<double>(f[0]); }

}  // namespace

// ======================================================================
KktDevice::KktDevice(int m, int n, const int* kA, const int* iA, const double* A, hipStream_t stream, int nforced,
                     const QBlock* qb)
    : m_(m), n_(n), T_(m + n), nforced_(nforced), stream_(stream) {
    if (qb && !qb->kQ) qb = nullptr;
    if (qb && nforced > 0) throw std::invalid_argument("kkt: a Q block with forced rows is not supported");
    QPattern qpat;
    if (qb) { qpat.kQ = qb->kQ; qpat.iQ = qb->iQ; }
    // IPO_HIP_SETUP_TIMES: where the host setup goes, to stderr
    const bool st_on = std::getenv("IPO_HIP_SETUP_TIMES") != nullptr;
    const auto st0 = std::chrono::steady_clock::now();
    auto mark = [&](const char* what) {
        if (st_on)
            std::fprintf(stderr, "setup %-28s %9.1f ms\n", what,
                         std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - st0).count());
    };
    std::vector<int> kat, iat;
    std::vector<double> at;
    csc_transpose(m, n, kA, iA, A, kat, iat, at);
    // the dense tail reaches down to the longest suffix at least 70 % full
    // (IPO_HIP_TAIL_DENSITY=1: only the reference's full dense window)
    double tail_density = kTailDensity;
    if (const char* e = std::getenv("IPO_HIP_TAIL_DENSITY")) tail_density = std::atof(e);
    mark("transpose");
    plan_ = build_kkt_plan(m, n, kA, iA, kat.data(), iat.data(), nforced, tail_density, qb ? &qpat : nullptr);
    mark("ordering + symbolic plan");
    if (nforced > 0) dLinkAx_.alloc(2 * static_cast<size_t>(nforced));
    const int nz = kA[n];
    hipStream_t s = stream_;
    dkA_.upload(kA, n + 1, s);
    diA_.upload(iA, nz, s);
    dA_.upload(A, nz, s);
    dkAt_.upload(kat, s);
    diAt_.upload(iat, s);
    dAt_.upload(at, s);

    dcol0_.upload(plan_.col0, s);
    drowptr_.upload(plan_.rowptr, s);
    drows_.upload(plan_.rows, s);
    dperm_.upload(plan_.perm, s);
    diperm_.upload(plan_.iperm, s);
    doff_.upload(plan_.off, s);
    damap_.upload(plan_.amap, s);
    if (qb) {
        qnz_ = qb->kQ[m];
        qmax_ = qb->qmax;
        dkQ_.upload(qb->kQ, m + 1, s);
        diQ_.upload(qb->iQ, qnz_ > 0 ? qnz_ : 1, s);
        dQ_.upload(qb->Q, qnz_ > 0 ? qnz_ : 1, s);
        dqmap_.upload(plan_.qmap, s);
        std::vector<double> qd(m > 0 ? m : 1, 0.0);
        for (int j = 0; j < m; j++)
            for (int k = qb->kQ[j]; k < qb->kQ[j + 1]; k++)
                if (qb->iQ[k] == j) qd[j] = qb->Q[k];
        dQdiag_.upload(qd, s);
        IPO_HIP_CHECK(hipStreamSynchronize(s));
    }
    ddslot_.upload(plan_.dslot, s);
    drelptr_.upload(plan_.relptr, s);
    dunit_sup_.upload(plan_.unit_sup, s);
    dunit_tile_.upload(plan_.unit_tile, s);
    dtask_ptr_.upload(plan_.task_ptr, s);
    dtask_pair_.upload(plan_.task_pair, s);
    dtask_i0_.upload(plan_.task_i0, s);
    dtask_i1_.upload(plan_.task_i1, s);
    dupd_src_.upload(plan_.upd_src, s);
    dupd_r0_.upload(plan_.upd_r0, s);
    dupd_r1_.upload(plan_.upd_r1, s);
    drel_.upload(plan_.rel, s);
    dlevel_sups_.upload(plan_.level_sups, s);
    mark("fused panel units (k_panel_w");
    {   // fused panel units (k_panel_w): per supernode max(1, tiles - 1) workgroups,
        // workgroup j holding the diagonal block and 64-row tile j + 1
        // (supernodes of at most 16 columns and 64 rows go to the one-wave
        // small-panel kernel instead: list small_sups_, per level small_ptr_)
        std::vector<int> fs, fj, ss;
        fu_ptr_.assign(plan_.nlevels + 1, 0);
        small_ptr_.assign(plan_.nlevels + 1, 0);
        for (int l = 0; l < plan_.nlevels; l++) {
            for (int q = plan_.level_ptr[l]; q < plan_.level_ptr[l + 1]; q++) {
                const int sp = plan_.level_sups[q];
                const int nc = plan_.col0[sp + 1] - plan_.col0[sp];
                const int h = nc + plan_.rowptr[sp + 1] - plan_.rowptr[sp];
                if (nc <= 16 && h <= kTileRows) { ss.push_back(sp); continue; }
                const int nw = std::max(1, ceil_div(h, kTileRows) - 1);
                for (int j = 0; j < nw; j++) { fs.push_back(sp); fj.push_back(j); }
            }
            fu_ptr_[l + 1] = static_cast<int>(fs.size());
            small_ptr_[l + 1] = static_cast<int>(ss.size());
        }
        // Levels whose fused units outnumber their supernodes many times
        // over and fill the device several times (the separator levels of
        // nested dissection: 1,000-3,500 units, 7-14 per supernode) run the
        // per-phase kernels instead: the fused units each refactor their
        // supernode's diagonal block, k_diag factors it once and k_trsm's
        // tiles only read it.  The same operations on every entry in the
        // same order (the IPO_HIP_PANEL=0 path), so bitwise the fused one.
        // IPO_HIP_PANEL_SPLIT: the unit count from which a level splits (0: never)
        int split_min = 768;
        if (const char* e = std::getenv("IPO_HIP_PANEL_SPLIT")) split_min = std::max(0, std::atoi(e));
        split_level_.assign(plan_.nlevels, 0);
        for (int l = 0; l < plan_.nlevels && split_min > 0; l++) {
            const int nfu = fu_ptr_[l + 1] - fu_ptr_[l];
            int nsup = 0;
            for (int q = fu_ptr_[l]; q < fu_ptr_[l + 1]; q++) nsup += fj[q] == 0;
            split_level_[l] = nfu >= split_min && nfu >= 4 * nsup;
        }
        // single-column small panels of <= 8 rows first in each level's list,
        // eight to a wave (k_panel_s1) on levels of many of them (the leaf
        // sweeps' threshold, IPO_HIP_SMALL_LEAVES)
        small1_cnt_.assign(plan_.nlevels, 0);
        {
            int thr = kSmallLeafMinCount;
            if (const char* e = std::getenv("IPO_HIP_SMALL_LEAVES")) thr = std::max(0, std::atoi(e));
            for (int l = 0; l < plan_.nlevels && thr > 0; l++) {
                const auto b = ss.begin() + small_ptr_[l], e = ss.begin() + small_ptr_[l + 1];
                const auto mid = std::stable_partition(b, e, [&](int sp) {
                    return plan_.col0[sp + 1] - plan_.col0[sp] == 1 && 1 + plan_.rowptr[sp + 1] - plan_.rowptr[sp] <= 8;
                });
                if (mid - b >= thr) small1_cnt_[l] = static_cast<int>(mid - b);
            }
        }
        dfu_sup_.upload(fs, s);
        dfu_j_.upload(fj, s);
        dsmall_sups_.upload(ss, s);
        IPO_HIP_CHECK(hipStreamSynchronize(s));
        // IPO_HIP_PANEL=0: per-phase kernels only (k_diag + k_trsm + k_tail_syrk,
        // the dependent-pivot path), the bitwise reference of the fused ones
        if (const char* e = std::getenv("IPO_HIP_PANEL")) use_panel_ = std::atoi(e) != 0;
    }
    mark("solve chunks: levels holding");
    {   // solve chunks: levels holding a panel with more than kChunkRows rows below
        // its diagonal block are solved in 64-row chunks (two launches each way)
        constexpr int kChunkRows = 128;
        std::vector<int> csup, cr0, chunk0(plan_.nsup, -1);
        chunk_ptr_.assign(plan_.nlevels + 1, 0);
        for (int l = 0; l < plan_.nlevels; l++) {
            bool big = false;
            for (int q = plan_.level_ptr[l]; q < plan_.level_ptr[l + 1]; q++) {
                const int sp = plan_.level_sups[q];
                big |= plan_.rowptr[sp + 1] - plan_.rowptr[sp] > kChunkRows;
            }
            if (big)
                for (int q = plan_.level_ptr[l]; q < plan_.level_ptr[l + 1]; q++) {
                    const int sp = plan_.level_sups[q], hb = plan_.rowptr[sp + 1] - plan_.rowptr[sp];
                    chunk0[sp] = static_cast<int>(csup.size());
                    for (int r0 = 0; r0 < hb; r0 += 64) { csup.push_back(sp); cr0.push_back(r0); }
                }
            chunk_ptr_[l + 1] = static_cast<int>(csup.size());
        }
        dchunk_sup_.upload(csup, s);
        dchunk_r0_.upload(cr0, s);
        dsup_chunk0_.upload(chunk0, s);
        partial_stride_ = csup.empty() ? 1 : csup.size() * kPanelCols;
        dPartial_.alloc(2 * partial_stride_);
        IPO_HIP_CHECK(hipStreamSynchronize(s));   // csup / cr0 / chunk0 are stack vectors
        h_chunk0_ = chunk0;
    }
    mark("sweep order of each level");
    {   // sweep order of each level: on levels without solve chunks the
        // single-column supernodes with <= 64 rows below come first (one wave
        // each, k_fwd_leaf / k_bwd_leaf), the rest after them
        std::vector<int> ss(plan_.level_sups);
        leaf_cnt_.assign(plan_.nlevels, 0);
        leaf8_cnt_.assign(plan_.nlevels, 0);
        small_leaves_ = kSmallLeafMinCount;
        if (const char* e = std::getenv("IPO_HIP_MERGE_LEVELS")) merge_levels_ = merge_panels_ = std::atoi(e) != 0;
        if (const char* e = std::getenv("IPO_HIP_SMALL_LEAVES")) small_leaves_ = std::max(0, std::atoi(e));
        for (int l = 0; l < plan_.nlevels; l++) {
            if (chunk_ptr_[l + 1] > chunk_ptr_[l]) continue;
            const auto b = ss.begin() + plan_.level_ptr[l], e = ss.begin() + plan_.level_ptr[l + 1];
            const auto mid = std::stable_partition(b, e, [&](int sp) {
                return plan_.col0[sp + 1] - plan_.col0[sp] == 1 && plan_.rowptr[sp + 1] - plan_.rowptr[sp] <= 64;
            });
            leaf_cnt_[l] = static_cast<int>(mid - b);
            if (small_leaves_ > 0) {   // the small ones first (k_fwd_leaf8 / k_bwd_leaf8)
                const auto mid8 = std::stable_partition(b, mid, [&](int sp) {
                    const int c = plan_.col0[sp];
                    return plan_.rowptr[sp + 1] - plan_.rowptr[sp] <= kSmallLeaf &&
                           plan_.yrow_ptr[c + 1] - plan_.yrow_ptr[c] <= kSmallLeaf;
                });
                leaf8_cnt_[l] = static_cast<int>(mid8 - b);
                // a wave of eight leaves touches eight times the cache lines
                // per load: slower on latency-bound levels (dfl001's sweeps
                // 4 ms slower per solve), faster from tens of thousands of
                // leaves on (configs[3]: 10^6)
                if (leaf8_cnt_[l] < small_leaves_) leaf8_cnt_[l] = 0;
            }
        }
        dsweep_sups_.upload(ss, s);
        IPO_HIP_CHECK(hipStreamSynchronize(s));
    }
    dyrow_ptr_.upload(plan_.yrow_ptr, s);
    build_sync_free_plan();
    // Deep elimination trees (at least kVisitLevels levels, e.g. the banded
    // BASELINE configs[3]: 2,785 levels, most of them one or two 64-column
    // supernodes): a level's gather would wait on every descendant's update,
    // although 93 % of its k-slots come from supernodes finished several
    // levels earlier.  There each unit's slots are ordered by the level of
    // their source (stable), and only the slabs that hold a source of the
    // level just below ("late") stay in the unit's own level's gather; the
    // earlier slabs become visits of at most kVisitSlots slots, scheduled as
    // late as their sources allow into the gather launches of the levels
    // below (one visit per unit per launch, each a read-modify-write of the
    // unit's tile in slot order).  The level chain then waits per level on
    // one small gather and the panel, the visits ride in the same launches
    // beside them.  IPO_HIP_VISITS=1/0 forces the schedule on / off.
    std::vector<int> kslot_v;
    mark("gather chunks (split K)");
    {   // gather chunks (split K): groups = sparse levels, then the dense tail
        const int nu = static_cast<int>(plan_.unit_sup.size());
        const char* ve = std::getenv("IPO_HIP_VISITS");
        visits_ = ve ? std::atoi(ve) != 0 : plan_.nlevels >= kVisitLevels;
        // flat gathers (k_update_flat) for the latency-bound launches of
        // deep trees: IPO_HIP_GATHER_FLAT=0 never, 1 (default) deep trees,
        // 2 every launch of at most kFlatMaxChunks chunks
        int flat_mode = 1;
        if (const char* e = std::getenv("IPO_HIP_GATHER_STAMPS")) gst_group_ = std::atoi(e);
        if (const char* e = std::getenv("IPO_HIP_GRAPH")) graph_on_ = std::atoi(e) != 0;
        // quadrant gathers (k_update_quad) on the narrow levels of deep trees
        // (IPO_HIP_GATHER_QUAD=0: off)
        bool quad_mode = true;
        if (const char* e = std::getenv("IPO_HIP_GATHER_QUAD")) quad_mode = std::atoi(e) != 0;
        if (const char* e = std::getenv("IPO_HIP_GATHER_FLAT")) flat_mode = std::atoi(e);
        int visit_slabs = kVisitSlots / kSlab;
        if (const char* e = std::getenv("IPO_HIP_VISIT_SLOTS")) visit_slabs = std::max(1, std::atoi(e) / kSlab);
        std::vector<int> kptr_v, late_b;
        std::vector<std::vector<int3>> vis(plan_.nlevels + 1);   // per group: (unit, slot begin, slot end)
        if (visits_) {
            kptr_v.assign(nu + 1, 0);
            late_b.assign(nu, 0);
            std::vector<std::pair<int, int>> sl;   // (source level, slot)
            std::vector<int> rl;
            for (int l = 1; l < plan_.nlevels; l++)
                for (int u = plan_.unit_level_ptr[l]; u < plan_.unit_level_ptr[l + 1]; u++) {
                    sl.clear();
                    for (int i = plan_.kslot_ptr[u]; i < plan_.kslot_ptr[u + 1]; i++) {
                        const int k = plan_.kslot[i];
                        if (k >= 0) sl.push_back({plan_.level[plan_.utasks[k >> 6].src], k});
                    }
                    std::stable_sort(sl.begin(), sl.end(),
                                     [](const std::pair<int, int>& a, const std::pair<int, int>& b) { return a.first < b.first; });
                    const int kb = static_cast<int>(kslot_v.size());
                    rl.clear();
                    for (size_t i = 0; i < sl.size(); i++) {
                        kslot_v.push_back(sl[i].second);
                        if (i % kSlab == 0) rl.push_back(sl[i].first);
                        else rl.back() = std::max(rl.back(), sl[i].first);
                    }
                    while (kslot_v.size() % kSlab) kslot_v.push_back(-1);
                    kptr_v[u + 1] = static_cast<int>(kslot_v.size());
                    const int nsl = static_cast<int>(rl.size());
                    int j = nsl;
                    while (j > 0 && rl[j - 1] >= l - 1) j--;
                    late_b[u] = kb + kSlab * j;
                    // early slabs [0, j), backwards, as late as their sources allow
                    int t = l - 1, end = j, cur = j;
                    while (cur > 0) {
                        if (end - cur >= visit_slabs && rl[cur - 1] <= t - 2) {
                            vis[t].push_back(make_int3(u, kb + kSlab * cur, kb + kSlab * end));
                            t--;
                            end = cur;
                        }
                        cur--;
                    }
                    if (end > 0) vis[t].push_back(make_int3(u, kb, kb + kSlab * end));
                }
            // groups visit their units in unit order
            for (auto& g : vis)
                std::sort(g.begin(), g.end(), [](const int3& a, const int3& b) { return a.x < b.x; });
        }
        std::vector<int> cu, cb, ce, cp, cq, su, sp0, sn;
        ck_ptr_.assign(plan_.nlevels + 2, 0);
        sp_ptr_.assign(plan_.nlevels + 2, 0);
        size_t max_part = 0;
        const int wg_target = 512;
        int min_chunk = 64;     // 64: measured best of 16-256 on configs[3] and dfl001 (IPO_HIP_MIN_CHUNK)
        if (const char* e = std::getenv("IPO_HIP_MIN_CHUNK")) min_chunk = std::max(kSlab, std::atoi(e) / kSlab * kSlab);
        // units [u0, u1), slots [kbeg(u), kend(u)) each, then the group's visits
        // a sparse unit's 32 x 32 quadrants that hold lower-triangle entries (k_update_quad)
        auto quadrants = [&](int u, int kb, int ke) {
            const int sp = plan_.unit_sup[u], t = plan_.unit_tile[u];
            const int nc = plan_.col0[sp + 1] - plan_.col0[sp], h = nc + plan_.rowptr[sp + 1] - plan_.rowptr[sp];
            const int nrow = std::min(kTileRows, h - t * kTileRows);
            for (int q = 0; q < 4; q++) {
                const int qr = q & 1, qc = q >> 1;
                if (32 * qr >= nrow || 32 * qc >= nc || (t == 0 && qc > qr)) continue;
                cu.push_back(u); cb.push_back(kb); ce.push_back(ke); cp.push_back(-1 - q); cq.push_back(-1);
            }
        };
        auto group = [&](int u0, int u1, auto kbeg, auto kend, const std::vector<int3>* visits) {
            const long nck0 = static_cast<long>(cu.size());
            long sumk = 0, nun = 0;
            for (int u = u0; u < u1; u++) { sumk += kend(u) - kbeg(u); nun += kend(u) > kbeg(u); }
            // deep trees' narrow levels: quadrant gathers, one chunk per unit
            const bool quad = quad_mode && visits && nun + static_cast<long>(visits->size()) <= kQuadMaxUnits;
            if (quad) {
                for (int u = u0; u < u1; u++)
                    if (kend(u) > kbeg(u)) quadrants(u, kbeg(u), kend(u));
                for (const int3& v : *visits) quadrants(v.x, v.y, v.z);
                ck_wide_.push_back(false);
                ck_kind_.push_back(2);
                return;
            }
            // aim at >= wg_target workgroups per launch, chunks of min_chunk..512 slots
            long kmax = (sumk / wg_target + kSlab - 1) / kSlab * kSlab;
            kmax = std::max<long>(min_chunk, std::min<long>(kMaxChunkSlots, kmax));
            int np = 0, mx = 0;
            for (int u = u0; u < u1; u++) {
                const int kb = kbeg(u), ke = kend(u);
                if (ke == kb) continue;
                const int nch = static_cast<int>((ke - kb + kmax - 1) / kmax);
                mx = std::max(mx, nch);
                if (nch > 1) { su.push_back(u); sp0.push_back(np); sn.push_back(nch); }
                for (int j = 0; j < nch; j++) {
                    cu.push_back(u);
                    cb.push_back(kb + static_cast<int>(j * kmax));
                    ce.push_back(std::min<int>(ke, kb + static_cast<int>((j + 1) * kmax)));
                    cp.push_back(nch > 1 ? np++ : -1);
                    cq.push_back(nch > 1 ? static_cast<int>(su.size()) - 1 : -1);
                }
            }
            if (visits)
                for (const int3& v : *visits) {
                    cu.push_back(v.x); cb.push_back(v.y); ce.push_back(v.z); cp.push_back(-1); cq.push_back(-1);
                }
            max_part = std::max<size_t>(max_part, np);
            // a group of few chunks (about one per CU: occupancy does not
            // matter) whose units are split many ways waits on its partial
            // sums: sum them several at a time
            ck_wide_.push_back(mx >= 4 && static_cast<long>(cu.size()) - nck0 <= 512);
            ck_kind_.push_back(quad ? 2 : (flat_mode == 2 || (flat_mode == 1 && visits_)) &&
                                               static_cast<long>(cu.size()) - nck0 <= kFlatMaxChunks ? 1 : 0);
        };
        const std::vector<int>& kp = plan_.kslot_ptr;
        ck_wide_.clear();
        ck_kind_.clear();
        for (int l = 0; l < plan_.nlevels; l++) {
            if (l == 0) { ck_wide_.push_back(false); ck_kind_.push_back(0); }
            else if (visits_)
                group(plan_.unit_level_ptr[l], plan_.unit_level_ptr[l + 1], [&](int u) { return late_b[u]; },
                      [&](int u) { return kptr_v[u + 1]; }, &vis[l]);
            else
                group(plan_.unit_level_ptr[l], plan_.unit_level_ptr[l + 1], [&](int u) { return kp[u]; },
                      [&](int u) { return kp[u + 1]; }, nullptr);
            ck_ptr_[l + 1] = static_cast<int>(cu.size());
            sp_ptr_[l + 1] = static_cast<int>(su.size());
        }
        const std::vector<int>& tp = plan_.tail_kslot_ptr;
        if (plan_.nt > 0)
            group(0, plan_.ntb * (plan_.ntb + 1) / 2, [&](int u) { return tp[u]; }, [&](int u) { return tp[u + 1]; },
                  nullptr);
        else { ck_wide_.push_back(false); ck_kind_.push_back(0); }
        ck_ptr_[plan_.nlevels + 1] = static_cast<int>(cu.size());
        sp_ptr_[plan_.nlevels + 1] = static_cast<int>(su.size());
        dck_u_.upload(cu, s);
        dck_b_.upload(cb, s);
        dck_e_.upload(ce, s);
        dck_part_.upload(cp, s);
        dsp_u_.upload(su, s);
        dsp_p0_.upload(sp0, s);
        dsp_n_.upload(sn, s);
        dck_q_.upload(cq, s);
        dSplitCnt_.alloc(std::max<size_t>(1, su.size()));
        IPO_HIP_CHECK(hipMemsetAsync(dSplitCnt_.get(), 0, std::max<size_t>(1, su.size()) * sizeof(int), s));
        dPartialTile_.alloc(std::max<size_t>(1, max_part) * (kTileRows * kTileRows + 4 * kTileRows));
        IPO_HIP_CHECK(hipStreamSynchronize(s));
    }
    mark("launches per sweep and algor");
    {   // launches per sweep and algorithmic work per phase occurrence
        fwd_launches_ = bwd_launches_ = sf_level_ < plan_.nlevels ? 1 : 0;
        for (int l = 0; l < sf_level_; l++) {
            const int nsl = plan_.level_ptr[l + 1] - plan_.level_ptr[l];
            const int nl = leaf_cnt_[l], n8 = leaf8_cnt_[l];
            const int k = chunk_ptr_[l + 1] > chunk_ptr_[l] ? 2
                        : (n8 > 0) + (nl > n8 && nsl > nl && merge_levels_ ? 1 : (nl > n8) + (nsl > nl));
            fwd_launches_ += k;
            bwd_launches_ += k;
        }
        if (plan_.nt > 0) {
            const int chain = plan_.ntb <= kChainMaxBlocks;
            fwd_launches_ += 1 + (chain ? 1 : plan_.ntb);
            bwd_launches_ += chain ? 1 : 1 + plan_.ntb;
        }
        const auto& P = plan_;
        double gf = 0, gb = 0;
        auto tasks_work = [&](const std::vector<TailTask>& ts) {
            for (const TailTask& t : ts) {
                const double ncd = P.col0[t.src + 1] - P.col0[t.src];
                const double nr = __builtin_popcountll(t.rmask), ncl = __builtin_popcountll(t.cmask);
                gf += 2.0 * ncd * nr * ncl;
                gb += 8.0 * ncd * (nr + ncl);
            }
        };
        tasks_work(P.utasks);
        tasks_work(P.tail_tasks);
        double df = 0, db = 0, tf = 0, tb = 0, sf = 0, sb = 0, lxs = 0;
        for (int sp = 0; sp < P.nsup; sp++) {
            const double nc = P.col0[sp + 1] - P.col0[sp], hb = P.rowptr[sp + 1] - P.rowptr[sp];
            df += 2.0 * nc * nc * nc / 3.0;
            db += 8.0 * 1.5 * nc * nc;
            tf += hb * nc * nc;
            tb += 16.0 * hb * nc;
            lxs += (nc + hb) * nc;
            gb += 16.0 * (nc + hb) * nc;      // read-modify-write of every target panel
        }
        const double sdf = df, sdb = db, stf = tf, stb = tb;     // sparse panels alone
        for (int kb = 0; kb < P.ntb; kb++) {
            const double nc = std::min(kPanelCols, P.nt - kb * kPanelCols), below = P.nt - kb * kPanelCols - nc;
            df += 2.0 * nc * nc * nc / 3.0;
            db += 8.0 * 1.5 * nc * nc;
            tf += below * nc * nc;
            tb += 16.0 * below * nc;                                // L21 read + write
            const double nb = P.ntb - kb - 1;
            sf += 2.0 * nc * (nb * (nb + 1) / 2) * kTileRows * kTileRows;
            sb += (nb * (nb + 1) / 2) * (16.0 * kTileRows * kTileRows + 16.0 * kTileRows * nc);
        }
        gb += 16.0 * 0.5 * P.nt * P.nt;                                 // tail block read-modify-write
        work_flops[kPhGather] = gf; work_bytes[kPhGather] = gb;
        work_flops[kPhDiag] = df; work_bytes[kPhDiag] = db;
        work_flops[kPhTrsm] = tf; work_bytes[kPhTrsm] = tb;
        work_flops[kPhSyrk] = sf; work_bytes[kPhSyrk] = sb;
        // Algorithmic flops per factorisation in SURVEY.md 8(d)'s unit: the
        // reference's narth (ldlt.c:1243-1248), split by the phase doing each
        // column's work (kkt_plan.h: narth_tail / narth_gather / narth_panel,
        // which sum to narth).  What the kernels execute (plan flops above,
        // the dense tail's explicit zeros) is not the work.  Bytes: each
        // phase's entries of L read and written once (+ the gather's source
        // reads from the plan).
        (void)sdf; (void)stf; (void)df; (void)tf; (void)sf; (void)lxs;
        work_flops[kPhGather] = P.narth_gather;
        if (use_panel_) {   // k_panel_w does both: the diag phase carries the sparse trsm work;
            // the dense tail is its own phase (k_tail_pr: panels + deferred
            // trailing updates; its repair launches)
            work_flops[kPhDiag] = P.narth_panel; work_bytes[kPhDiag] = sdb + stb;
            work_flops[kPhTrsm] = work_bytes[kPhTrsm] = 0;
            work_flops[kPhSyrk] = work_bytes[kPhSyrk] = 0;
            work_flops[kPhTail] = P.narth_tail;
            work_bytes[kPhTail] = 16.0 * (static_cast<double>(P.lnz_tail) + P.nt);
        } else {            // per-phase path: the tail's work goes with its trailing updates
            work_flops[kPhDiag] = P.narth_panel;
            work_flops[kPhTrsm] = 0;
            work_flops[kPhSyrk] = P.narth_tail;
        }
        // a sweep (s (4 nnz(L) + N) per iteration, a solve
        // being one forward and one backward sweep): 2 nnz(L) + N / 2 flops,
        // every entry of L read once (12 B with its index) and the vector
        // values in and out
        for (int ph : {kPhForward, kPhBackward}) {
            work_flops[ph] = 2.0 * static_cast<double>(P.lnz) + 0.5 * T_;
            work_bytes[ph] = 12.0 * static_cast<double>(P.lnz) + 16.0 * T_;
        }
    }
    mark("per-task source descriptors ");
    {   // per-task source descriptors for the gather
        auto build = [&](const std::vector<TailTask>& ts, DevBuf<TaskSrc>& dst) {
            std::vector<TaskSrc> v(ts.size());
            for (size_t t = 0; t < ts.size(); t++) {
                const int d = ts[t].src, ncd = plan_.col0[d + 1] - plan_.col0[d];
                v[t].colbase = plan_.off[d] + ncd;
                v[t].hd = ncd + (plan_.rowptr[d + 1] - plan_.rowptr[d]);
                v[t].cd0 = plan_.col0[d];
            }
            dst.upload(v, s);
            IPO_HIP_CHECK(hipStreamSynchronize(s));
        };
        build(plan_.utasks, dusrc_);
        if (plan_.nt > 0) build(plan_.tail_tasks, dtsrc_);
        // per k-slot records of the gather (SlotRec), expanded from the
        // slot -> task -> source panel indirection
        auto expand = [&](const std::vector<int>& kslot, const std::vector<TailTask>& ts, DevBuf<SlotRec>& dst) {
            std::vector<SlotRec> v(kslot.size());
            for (size_t i = 0; i < kslot.size(); i++) {
                const int sl = kslot[i];
                SlotRec& r = v[i];
                if (sl < 0) { r.rmask = r.cmask = 0; r.roff = 0; r.cdelta = 0; r.dk = 0; continue; }
                const TailTask& t = ts[sl >> 6];
                const int kl = sl & 63, d = t.src, ncd = plan_.col0[d + 1] - plan_.col0[d];
                const int64_t hd = ncd + (plan_.rowptr[d + 1] - plan_.rowptr[d]);
                r.rmask = t.rmask;
                r.cmask = t.cmask;
                r.roff = plan_.off[d] + ncd + kl * hd + t.rbase;
                r.cdelta = t.cbase - t.rbase;
                r.dk = plan_.col0[d] + kl;
            }
            dst.upload(v, s);
            IPO_HIP_CHECK(hipStreamSynchronize(s));
        };
        expand(visits_ ? kslot_v : plan_.kslot, plan_.utasks, dslot_rec_);
        if (plan_.nt > 0) expand(plan_.tail_kslot, plan_.tail_tasks, dtail_slot_rec_);
    }
    mark("dutasks_.upload(reinterpret_");
    dutasks_.upload(reinterpret_cast<const uint64_t*>(plan_.utasks.data()), plan_.utasks.size() * 4, s);
    if (plan_.nt > 0) {
        dtail_task_ptr_.upload(plan_.tail_task_ptr, s);
        dtail_kslot_.upload(plan_.tail_kslot, s);
        dtail_kslot_ptr_.upload(plan_.tail_kslot_ptr, s);
        static_assert(sizeof(TailTask) == 32, "TailTask layout");
        dtail_tasks_.upload(reinterpret_cast<const uint64_t*>(plan_.tail_tasks.data()), plan_.tail_tasks.size() * 4, s);
        dW_.alloc(static_cast<size_t>(plan_.nt) * kPanelCols);   // W = L21 D of one block column (per-phase path)
        dDepSt_.alloc(tail_dep_state_doubles(plan_.ntb));
        dDepI_.alloc(8);
        // R <= 2 right-hand sides: z of every block, then k_tail_fwd_lead's helper partials
        dChainGran_.alloc(static_cast<size_t>(plan_.ntb) * (2 * 128 + 2 * 4 * 64 * 2));
        dlead_ticket_.alloc(1);
        IPO_HIP_CHECK(hipMemsetAsync(dlead_ticket_.get(), 0, sizeof(int), s));
        lead_ticket_next_ = 0;
        IPO_HIP_CHECK(hipMemsetAsync(dChainGran_.get(), 0, dChainGran_.bytes(), s));
        if (plan_.ntb <= kChainMaxBlocks) {
            for (const void* f : {reinterpret_cast<const void*>(&k_tail_fwd_chain<1>),
                                  reinterpret_cast<const void*>(&k_tail_fwd_chain<2>),
                                  reinterpret_cast<const void*>(&k_tail_bwd_chain<1>),
                                  reinterpret_cast<const void*>(&k_tail_bwd_chain<2>)})
                IPO_HIP_CHECK(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, kChainLds));
            for (const void* f : {reinterpret_cast<const void*>(&k_tail_fwd_pair<1>),
                                  reinterpret_cast<const void*>(&k_tail_fwd_pair<2>)})
                IPO_HIP_CHECK(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, kPairFwdLds));
            for (const void* f : {reinterpret_cast<const void*>(&k_tail_bwd_pair<1>),
                                  reinterpret_cast<const void*>(&k_tail_bwd_pair<2>)})
                IPO_HIP_CHECK(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, kPairBwdLds));
            // two 64-row blocks per chain workgroup (IPO_HIP_CHAIN_PAIRS=1; default: one)
            const char* cp = std::getenv("IPO_HIP_CHAIN_PAIRS");
            chain_pairs_ = cp && std::atoi(cp) != 0;
            for (const void* f : {reinterpret_cast<const void*>(&k_tail_fwd_lead<1>),
                                  reinterpret_cast<const void*>(&k_tail_fwd_lead<2>)})
                IPO_HIP_CHECK(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, kChainLds));
            // the forward sweep by a lead workgroup (default; IPO_HIP_CHAIN_LEAD=0: the per-block chain)
            const char* cl = std::getenv("IPO_HIP_CHAIN_LEAD");
            chain_lead_ = !(cl && std::atoi(cl) == 0);
        }
    }
    if (const char* vb = std::getenv("IPO_HIP_VISIT_BLOCKS")) visit_blocks_ = std::max(1, std::atoi(vb));
    if (plan_.nt > 0 && plan_.ntb <= 255) {
        // look-ahead launches of at most one workgroup per CU (tail_visit_schedule)
        const char* vs = std::getenv("IPO_HIP_VISIT_SCHED");
        if (!vs || std::atoi(vs) != 0) {
            int dev = 0, cus = 0;
            IPO_HIP_CHECK(hipGetDevice(&dev));
            IPO_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
            const std::vector<unsigned> vl = tail_visit_schedule(plan_.ntb, plan_.nt, visit_blocks_, cus, visit_ptr_);
            dvisit_list_.upload(vl, s);
            IPO_HIP_CHECK(hipStreamSynchronize(s));   // vl is a local
        }
        // the persistent run (k_tail_run, default; its bails end in the same
        // state as the per-step launches', so the repair and the sharded
        // solve's per-phase redo are unchanged); the latest chunk of each
        // column IPO_HIP_VISIT_LATEST blocks
        const char* tr = std::getenv("IPO_HIP_TAIL_RUN");
        tail_run_ = !(tr && std::atoi(tr) == 0);
        if (tail_run_) {
            int dev = 0, cus = 0;
            IPO_HIP_CHECK(hipGetDevice(&dev));
            IPO_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
            const char* vl = std::getenv("IPO_HIP_VISIT_LATEST");
            const int latest = vl ? std::max(1, std::atoi(vl)) : kTailVisitLatest;
            run_latest_ = latest;
            const std::vector<uint2> items =
                tail_run_schedule(plan_.ntb, plan_.nt, visit_blocks_, latest, cus, run_ptr_);
            drun_items_.upload(items, s);
            drun_cnt_.alloc(1 + plan_.ntb + static_cast<size_t>(plan_.ntb) * plan_.ntb + plan_.ntb);
            // each step's tile windows handed to the next step's pre-update as
            // they complete (kkt_dense.hip RunPub; IPO_HIP_TAIL_WINPUB=0: the
            // pre-update waits for the whole previous step and reads S)
            const char* wp = std::getenv("IPO_HIP_TAIL_WINPUB");
            run_winpub_ = !(wp && std::atoi(wp) == 0);
            if (run_winpub_) {
                drun_pub_.alloc(2 * static_cast<size_t>(plan_.ntb) * 4 * kTailPubWin);
                drun_wflag_.alloc(static_cast<size_t>(plan_.ntb) * plan_.ntb * 4);
                IPO_HIP_CHECK(hipMemsetAsync(drun_wflag_.get(), 0, drun_wflag_.bytes(), s));
                run_epoch_ = 0;
            }
            IPO_HIP_CHECK(hipStreamSynchronize(s));   // items is a local
            // the chain launch (IPO_HIP_TAIL_CHAIN=1, where the tail has tiles
            // below its blocks; used when TailView::dep == 1, else the run above)
            const char* tc = std::getenv("IPO_HIP_TAIL_CHAIN");
            tail_chain_ = plan_.ntb >= 3 && tc && std::atoi(tc) != 0;
            if (tail_chain_) {
                std::vector<int> cptr;
                const std::vector<uint2> citems =
                    tail_chain_schedule(plan_.ntb, plan_.nt, visit_blocks_, latest, cus, cptr);
                chain_n_ = static_cast<int>(citems.size());
                dchain_items_.upload(citems, s);
                dchain_cnt_.alloc(chain_zero_ints(plan_.ntb));
                dchain_pub_.alloc(static_cast<size_t>(plan_.ntb) * 4 * kChainWinPub);
                dchain_save_.alloc(2 * kPanelCols * kPanelCols + kPanelCols);
                IPO_HIP_CHECK(hipStreamSynchronize(s));
            }
        }
    }
    if (const char* ts = std::getenv("IPO_HIP_TAIL_SPEC")) tail_spec_ = std::atoi(ts);
    if (const char* sd = std::getenv("IPO_HIP_SPARSE_DEP")) sparse_dep_ = std::atoi(sd);
    if (const char* em = std::getenv("IPO_HIP_EPSDIAG_MAX")) epsdiag_cap_ = std::atof(em);

    mark("dLx_.alloc(plan_.lx_size > 0");
    dLx_.alloc(plan_.lx_size > 0 ? plan_.lx_size : 1);
    dDg_.alloc(T_ > 0 ? T_ : 1);
    dLive_.alloc(T_ > 0 ? T_ : 1);
    dDscale_.alloc(T_ > 0 ? T_ : 1);
    if (const char* e = std::getenv("IPO_HIP_PIVTOL")) pivot_tol_ = std::atof(e);
    // flags: [0] ndep, [1] fused panel bail-out bits, [2] 1 + the dense-tail
    // block column whose look-ahead panel bailed, [4..4+T) node class sign
    dFlags_.alloc(4 + T_);
    {
        std::vector<int> fl(4 + T_, 0);
        for (int v = 0; v < T_; v++) fl[4 + v] = plan_.dsign[v];
        dFlags_.upload(fl, s);
    }
    dZ_.alloc(2 * (T_ > 0 ? T_ : 1));
    dDy_.alloc(2 * (m > 0 ? m : 1));
    dRy_.alloc(2 * (m > 0 ? m : 1));
    dDx_.alloc(2 * (n > 0 ? n : 1));
    dRx_.alloc(2 * (n > 0 ? n : 1));
    dIncons_.alloc(2);
    dPart_.alloc(8 * kRedBlocks);
    dScal_.alloc(16);
    IPO_HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&hScal_), 16 * sizeof(double), hipHostMallocDefault));
    IPO_HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&hFlags_), 8 * sizeof(int), hipHostMallocDefault));
    IPO_HIP_CHECK(hipEventCreate(&ev0_));
    IPO_HIP_CHECK(hipEventCreate(&ev1_));
    IPO_HIP_CHECK(hipEventCreate(&ev2_));
    IPO_HIP_CHECK(hipEventCreate(&ev3_));
    IPO_HIP_CHECK(hipStreamSynchronize(s));
    mark("done");
}

// Sync-free top levels (k_fwd_sf / k_bwd_sf): from sf_level_ up every level
// is at most kSfWidth supernodes wide (IPO_HIP_SF_WIDTH): 300 for factors
// of fewer than 2^25 entries, 64 above.  Measured on one box: dfl001 64 /
// 150 / 300 / 450 / 600 / all -> 290.9 / 292.5 / 292.7 / 292.7 / 292.1 /
// 224.4 it/s (every level in the launch starves the wide bottom ones),
// 25fv47 by intpt 932 -> 963 at 300; but banded configs[3] 76.9 -> 68.5 and
// block-angular configs[4] 47.6 -> 39.3 at 300 (their upper levels hold
// large chunked supernodes, which the per-level launches spread wider).  Their forward update values get
// ybuf slices, and their z values zpad slices, of their own 128-B lines;
// work items, per-supernode arrival counts and parents.  Called from the
// constructor after the solve chunks are built.
void KktDevice::build_sync_free_plan() {
    int kSfWidth = plan_.lx_size < (int64_t(1) << 25) ? 300 : 64;
    if (const char* e = std::getenv("IPO_HIP_SF_WIDTH")) kSfWidth = std::max(1, std::atoi(e));
    hipStream_t s = stream_;
    const KktPlan& P = plan_;
    const int ns = P.nsup;
    sf_level_ = P.nlevels;
    while (sf_level_ > 0 && P.level_ptr[sf_level_] - P.level_ptr[sf_level_ - 1] <= kSfWidth) sf_level_--;
    if (P.nlevels - sf_level_ < 2) sf_level_ = P.nlevels;
    if (const char* e = std::getenv("IPO_HIP_SF"))
        if (std::atoi(e) == 0) sf_level_ = P.nlevels;
    auto chunked = [&](int sp) { const int l = P.level[sp]; return chunk_ptr_[l + 1] > chunk_ptr_[l]; };
    auto nchunks = [&](int sp) { return (P.rowptr[sp + 1] - P.rowptr[sp] + 63) / 64; };
    std::vector<int> ybase(ns + 1), zbase(ns, -1), zpi(T_ > 0 ? T_ : 1, -1), need(ns, 0), par(ns, -1);
    size_t yend = P.rowptr.empty() ? 0 : P.rowptr.back(), zend = 0;
    for (int sp = 0; sp < ns; sp++) {
        if (P.level[sp] < sf_level_) { ybase[sp] = P.rowptr[sp]; continue; }
        yend = (yend + 15) & ~size_t(15);
        ybase[sp] = static_cast<int>(yend);
        yend += P.rowptr[sp + 1] - P.rowptr[sp];
        zend = (zend + 15) & ~size_t(15);
        zbase[sp] = static_cast<int>(zend);
        for (int c = P.col0[sp]; c < P.col0[sp + 1]; c++) zpi[c] = static_cast<int>(zend + c - P.col0[sp]);
        zend += P.col0[sp + 1] - P.col0[sp];
        const int pa = P.parent[sp];
        if (pa >= 0) { par[sp] = pa; need[pa] += chunked(sp) ? nchunks(sp) : 1; }
    }
    ybase[ns] = static_cast<int>(yend);
    std::vector<int> yidx(P.yrow_idx);
    if (sf_level_ < P.nlevels) {       // update-value positions of the moved slices
        std::vector<int> pos(yidx.empty() ? 1 : P.rowptr.back());
        for (int sp = 0; sp < ns; sp++)
            for (int i = P.rowptr[sp]; i < P.rowptr[sp + 1]; i++) pos[i] = ybase[sp] + (i - P.rowptr[sp]);
        for (int& e : yidx) e = pos[e];
    }
    dyrow_idx_.upload(yidx, s);
    dybase_.upload(ybase, s);
    // Deep trees: the update values a narrow-range column receives from
    // supernodes below the range (on configs[3] the 10^6 leaves and the wide
    // levels: ~30 scattered values per row, ~5 us of the chain item's loads)
    // are all known once the bottom levels are swept.  They are subtracted
    // from the right-hand side by one pre-pass launch (k_fwd_pre: per column,
    // in list order), and the sync-free items sum only the values of
    // supernodes inside the range (their own lists, ylate_*).
    pre_cols_ = 0;
    {
        const char* ve = std::getenv("IPO_HIP_VISITS");
        const bool deep = ve ? std::atoi(ve) != 0 : P.nlevels >= kVisitLevels;
        if (deep && sf_level_ < P.nlevels) {
            auto src_of = [&](int i) {        // the supernode whose row set holds R entry i
                return static_cast<int>(std::upper_bound(P.rowptr.begin(), P.rowptr.end(), i) - P.rowptr.begin()) - 1;
            };
            std::vector<int> lptr(T_ + 1, 0), lidx, ecol, eptr{0}, eidx;
            for (int v = 0; v < T_; v++) {
                const int sv = v < P.tail_c0 ? P.sup_of[v] : -1;
                const bool in_range = sv >= 0 && P.level[sv] >= sf_level_;
                bool any_early = false;
                // (columns outside the range keep empty late lists: only k_fwd_sf reads these)
                for (int e = in_range ? P.yrow_ptr[v] : 0; e < (in_range ? P.yrow_ptr[v + 1] : 0); e++) {
                    const bool early = P.level[src_of(P.yrow_idx[e])] < sf_level_;
                    if (early) {
                        if (!any_early) { ecol.push_back(v); any_early = true; }
                        eidx.push_back(yidx[e]);
                    } else {
                        lidx.push_back(yidx[e]);
                    }
                }
                if (any_early) eptr.push_back(static_cast<int>(eidx.size()));
                lptr[v + 1] = static_cast<int>(lidx.size());
            }
            pre_cols_ = static_cast<int>(ecol.size());
            dylate_ptr_.upload(lptr, s);
            dylate_idx_.upload(lidx.empty() ? std::vector<int>{0} : lidx, s);
            dpre_col_.upload(ecol.empty() ? std::vector<int>{0} : ecol, s);
            dpre_ptr_.upload(eptr, s);
            dpre_idx_.upload(eidx.empty() ? std::vector<int>{0} : eidx, s);
            IPO_HIP_CHECK(hipStreamSynchronize(s));
        }
    }
    ybuf_stride_ = std::max<size_t>(yend, 1);
    dYbuf_.alloc(2 * ybuf_stride_);
    std::vector<int2> fi, bi;
    for (int l = sf_level_; l < P.nlevels; l++)
        for (int q = P.level_ptr[l]; q < P.level_ptr[l + 1]; q++) {
            const int sp = P.level_sups[q];
            if (!chunked(sp)) { fi.push_back(make_int2(sp, -1)); continue; }
            for (int c = 0; c < nchunks(sp); c++) fi.push_back(make_int2(sp, h_chunk0_[sp] + c));
        }
    for (int l = P.nlevels - 1; l >= sf_level_; l--)
        for (int q = P.level_ptr[l]; q < P.level_ptr[l + 1]; q++) {
            const int sp = P.level_sups[q];
            if (!chunked(sp)) { bi.push_back(make_int2(sp, -1)); continue; }
            for (int c = 0; c < nchunks(sp); c++) bi.push_back(make_int2(sp, h_chunk0_[sp] + c));
        }
    nsf_f_ = static_cast<int>(fi.size());
    nsf_b_ = static_cast<int>(bi.size());
    if (sf_level_ < P.nlevels) {
        dsf_items_f_.upload(fi, s);
        h_sf_items_f_ = fi;
        dsf_items_b_.upload(bi, s);
        dsf_need_.upload(need, s);
        dsf_par_.upload(par, s);
        dsf_zbase_.upload(zbase, s);
        dsf_zpi_.upload(zpi, s);
        zpad_stride_ = std::max<size_t>(zend, 1);
        dZpad_.alloc(2 * zpad_stride_);
        for (DevBuf<int>* b : {&dsf_fcnt_, &dsf_fflag_, &dsf_bcnt_, &dsf_bflag_}) {
            b->alloc(ns);
            IPO_HIP_CHECK(hipMemsetAsync(b->get(), 0, ns * sizeof(int), s));
        }
        dsf_ticket_.alloc(2);
        IPO_HIP_CHECK(hipMemsetAsync(dsf_ticket_.get(), 0, 2 * sizeof(int), s));
        sf_ticket_next_[0] = sf_ticket_next_[1] = 0;
        int dev = 0;
        IPO_HIP_CHECK(hipGetDevice(&dev));
        IPO_HIP_CHECK(hipDeviceGetAttribute(&sf_grid_, hipDeviceAttributeMultiprocessorCount, dev));
        for (const void* f : {reinterpret_cast<const void*>(&k_fwd_sf<1>), reinterpret_cast<const void*>(&k_fwd_sf<2>),
                              reinterpret_cast<const void*>(&k_bwd_sf<1>), reinterpret_cast<const void*>(&k_bwd_sf<2>)})
            IPO_HIP_CHECK(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, kChainLds));
    }
    IPO_HIP_CHECK(hipStreamSynchronize(s));   // the host vectors above are locals
}

#ifdef IPO_SF_STAMPS
// Per-level summary of the last forward sync-free sweep's stamps (10 ns
// ticks): items, mean wait / diag (gather + L11 solve) / rest / hand-off,
// and when the level's last item finished.
static void dump_sf_stamps(const std::vector<int2>& items, const KktPlan& P) {
    std::vector<long long> st((size_t)(1 << 15) * 10);
    if (hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(g_sfst), st.size() * sizeof(long long)) != hipSuccess) return;
    const int n = std::min<int>(items.size(), 1 << 15);
    long long t0 = LLONG_MAX;
    for (int i = 0; i < n; i++) t0 = std::min(t0, st[i * 10]);
    std::map<int, std::array<double, 7>> lv;   // level -> items, wait, diag, rest, end, handoff, ...
    for (int i = 0; i < n; i++) {
        const long long* x = &st[i * 10];
        auto& a = lv[P.level[items[i].x]];
        a[0] += 1; a[1] += x[1] - x[0]; a[2] += x[2] - x[1]; a[3] += x[3] - x[2]; a[4] = std::max<double>(a[4], x[4] - t0);
        a[5] += x[4] - x[3];
    }
    if (const char* f = std::getenv("IPO_SF_STAMPS_FILE")) {
        if (FILE* fo = std::fopen(f, "w")) {
            for (int i = 0; i < n; i++) {
                const long long* x = &st[i * 10];
                std::fprintf(fo, "%d %d %d %d %lld %lld %lld %lld %lld %lld %lld %lld %lld\n", items[i].x, items[i].y,
                             P.level[items[i].x], P.parent[items[i].x], x[0] - t0, x[1] - t0, x[2] - t0, x[3] - t0,
                             x[4] - t0, x[5] - t0, x[6], x[7] - t0, x[8] - t0);
            }
            std::fclose(fo);
        }
    }
    std::fprintf(stderr, "sf forward: level items wait diag rest handoff end(us)\n");
    for (auto& [l, a] : lv)
        std::fprintf(stderr, "  %3d %4.0f %7.2f %7.2f %7.2f %6.2f %8.1f\n", l, a[0], a[1] / a[0] / 100, a[2] / a[0] / 100,
                     a[3] / a[0] / 100, a[5] / a[0] / 100, a[4] / 100);
}
#endif

KktDevice::~KktDevice() {
#ifdef IPO_SF_STAMPS
    if (!h_sf_items_f_.empty()) dump_sf_stamps(h_sf_items_f_, plan_);
#endif
    if (std::getenv("IPO_HIP_DEBUG_REDO"))
        std::fprintf(stderr, "kkt: %ld factorisations, %ld redone; bails (unused) %ld, k_panel_w sparse %ld, tail %ld, "
                             "k_panel_s %ld; tail block columns repaired %ld in %ld rounds\n", tm_.factors,
                     tm_.panel_redos, tm_.redo_where[0], tm_.redo_where[1], tm_.redo_where[2], tm_.redo_where[3],
                     tm_.tail_repairs, tm_.tail_dep_rounds);
    if (hScal_) (void)hipHostFree(hScal_);
    if (hFlags_) (void)hipHostFree(hFlags_);
    if (ev0_) (void)hipEventDestroy(ev0_);
    if (ev1_) (void)hipEventDestroy(ev1_);
    if (ev2_) (void)hipEventDestroy(ev2_);
    if (ev3_) (void)hipEventDestroy(ev3_);
    for (hipEvent_t e : kev_) (void)hipEventDestroy(e);
    if (lvl_exec_) (void)hipGraphExecDestroy(lvl_exec_);
}

static PlanView make_view(const KktPlan&, const DevBuf<int>& col0, const DevBuf<int>& rowptr, const DevBuf<int>& rows,
                          const DevBuf<int64_t>& off, const DevBuf<int>& us, const DevBuf<int>& ut,
                          const DevBuf<int>& tp, const DevBuf<int>& tq, const DevBuf<int>& t0, const DevBuf<int>& t1,
                          const DevBuf<int>& src, const DevBuf<int>& r0, const DevBuf<int>& r1,
                          const DevBuf<int64_t>& relptr, const DevBuf<int>& rel, const DevBuf<double>& lx,
                          const DevBuf<double>& dg, const DevBuf<int>& live, const DevBuf<int>& flags) {
    PlanView v;
    v.col0 = col0.get(); v.rowptr = rowptr.get(); v.rows = rows.get(); v.off = off.get();
    v.unit_sup = us.get(); v.unit_tile = ut.get(); v.task_ptr = tp.get(); v.task_pair = tq.get();
    v.task_i0 = t0.get(); v.task_i1 = t1.get(); v.upd_src = src.get(); v.upd_r0 = r0.get(); v.upd_r1 = r1.get();
    v.relptr = relptr.get(); v.rel = rel.get(); v.Lx = lx.get(); v.dg = dg.get(); v.live = live.get();
    v.flags = flags.get();
    v.sign = flags.get() + 4;
    return v;
}

#define IPO_VIEW() with_scale(make_view(plan_, dcol0_, drowptr_, drows_, doff_, dunit_sup_, dunit_tile_, dtask_ptr_, \
                             dtask_pair_, dtask_i0_, dtask_i1_, dupd_src_, dupd_r0_, dupd_r1_, drelptr_, drel_, \
                             dLx_, dDg_, dLive_, dFlags_), dDscale_.get(), pivot_tol_, dIncons_.get(), \
                             dybase_.get())

static PlanView with_scale(PlanView v, double* dscale, double tau, int* incons, const int* ybase) {
    static const int xcd = [] {
        const char* e = std::getenv("IPO_HIP_UPDATE_XCD");     // launches of at least this many chunks (0: off)
        return e ? std::max(0, std::atoi(e)) : 1024;
    }();
    v.xcd = xcd;
    v.dscale = dscale;
    v.tau = tau;
    v.incons = incons;
    v.ybase = ybase;
    return v;
}

TailView KktDevice::tail_view() const {
    TailView t;
    t.S = dLx_.get() + plan_.off_tail;
    t.nt = plan_.nt;
    t.ntb = plan_.ntb;
    t.tc = plan_.tail_c0;
    t.task_ptr = dtail_task_ptr_.get();
    t.tasks = reinterpret_cast<const TailTask*>(dtail_tasks_.get());
    t.W = dW_.get();
    t.vk = visit_blocks_;
    if (!visit_ptr_.empty()) {
        t.vlist = dvisit_list_.get();
        t.vptr = visit_ptr_.data();
    }
    // dependent pivots in the look-ahead panel: its failed checks fall back on
    // the host repair, which the sharded solve does not use
    const char* rp = std::getenv("IPO_HIP_TAIL_REPAIR");
    t.dep = use_panel_ && !xch_ && (!rp || std::atoi(rp) != 0) ? tail_spec_ : 0;
    // in the sparse panels a failed check falls back on redoing the factor
    // from the assembly, on every shard alike (the bail flags are reduced)
    t.sdep = sparse_dep_;
    return t;
}

// Developer diagnostics (IPO_HIP_DUMP_DIR=dir): every factorisation's input
// (E, D, eps_diag) and outcome (live marks, D, |terms| sums, ndep) to
// dir/fNNNN.bin, for tools/dep_compare.py, which refactors the same input
// with the oracle and compares the dependent-pivot classification.
// Layout: int32 m, n, T, ndep; f64 eps_in, eps_out; f64 E[m], D[n];
// int32 perm[T]; int32 live[T]; f64 dg[T]; f64 dscale[T] (new order).
void KktDevice::dump_factor(const double* dE, const double* dD, double eps_in) {
    const char* dir = std::getenv("IPO_HIP_DUMP_DIR");
    if (!dir) return;
    std::vector<double> E(m_), D(n_), dg(T_), dsc(T_);
    std::vector<int> live(T_);
    IPO_HIP_CHECK(hipStreamSynchronize(stream_));
    if (m_) IPO_HIP_CHECK(hipMemcpy(E.data(), dE, m_ * sizeof(double), hipMemcpyDeviceToHost));
    if (n_) IPO_HIP_CHECK(hipMemcpy(D.data(), dD, n_ * sizeof(double), hipMemcpyDeviceToHost));
    dLive_.download(live.data(), T_, stream_);
    dDg_.download(dg.data(), T_, stream_);
    dDscale_.download(dsc.data(), T_, stream_);
    IPO_HIP_CHECK(hipStreamSynchronize(stream_));
    char path[4096];
    std::snprintf(path, sizeof path, "%s/f%04d.bin", dir, dump_count_++);
    FILE* f = std::fopen(path, "wb");
    if (!f) return;
    const int hdr[4] = {m_, n_, T_, ndep_};
    const double eps[2] = {eps_in, epsdiag_};
    std::fwrite(hdr, sizeof(int), 4, f);
    std::fwrite(eps, sizeof(double), 2, f);
    std::fwrite(E.data(), sizeof(double), m_, f);
    std::fwrite(D.data(), sizeof(double), n_, f);
    std::fwrite(plan_.perm.data(), sizeof(int), T_, f);
    std::fwrite(live.data(), sizeof(int), T_, f);
    std::fwrite(dg.data(), sizeof(double), T_, f);
    std::fwrite(dsc.data(), sizeof(double), T_, f);
    std::fclose(f);
}

void KktDevice::factor(const double* dE, const double* dD) {
    const double eps_in = epsdiag_;
    factor_core(dE, dD);
    dump_factor(dE, dD, eps_in);
}

void KktDevice::factor_core(const double* dE, const double* dD) {
    // fast path: fused diagonal-block + panel kernels; a pivot that fails
    // the zero test makes them stop unwritten.  A bail in the dense tail
    // only: the look-ahead resumes from the bailed block column (repair);
    // in the sparse levels: the factorisation is redone with the per-phase
    // kernels there, which own the dependent-pivot rule, and the tail again
    // by the look-ahead (its own bails repaired the same way) -- a per-phase
    // tail costs a single-workgroup partial substitution per block column
    const char* rp = std::getenv("IPO_HIP_TAIL_REPAIR");
    const bool repair = use_panel_ && !xch_ && (!rp || std::atoi(rp) != 0);
    bool ok = factor_pass(dE, dD, use_panel_, use_panel_);
    if (!ok && (hFlags_[1] & 64)) {
        // the chain launch aborted (a tile contradicted a dropped column): the
        // factorisation again with the per-step look-ahead and its repairs
        tm_.tail_chain_aborts++;
        chain_off_ = true;
        ok = factor_pass(dE, dD, use_panel_, use_panel_);
        chain_off_ = false;
    }
    if (!ok) {
        tm_.panel_redos++;
        for (int b = 0; b < 4; b++) tm_.redo_where[b] += (hFlags_[1] >> b) & 1;
        // bit 16: a dependent-pivot pass of the tail failed its check (restore first)
        const bool tail_only = (hFlags_[1] & ~16) == 4 && hFlags_[4] > 0;
        if (repair && tail_only) repair_tail();
        else if (!factor_pass(dE, dD, false, repair) && repair && (hFlags_[1] & ~16) == 4 && hFlags_[4] > 0)
            repair_tail();
    }
    tm_.factors++;
    // one occurrence per factorisation, whatever redos and repairs it took
    // (their launches and time stay in the phases: the work is priced once)
    if (timing_)
        for (int ph : {kPhGather, kPhDiag, kPhTrsm, kPhSyrk, kPhTail}) tm_.phase_count[ph]++;
    ndep_ = xch_ ? static_cast<int>(hScal_[1]) : hFlags_[0];
    if (-hScal_[0] < 1.0e-14) epsdiag_ *= 10;
    // developer diagnostics (IPO_HIP_EPSDIAG_MAX, tools/status_loss_probe.py):
    // a cap on the growth above, to measure what a stalled solve owes to it
    if (epsdiag_cap_ > 0.0 && epsdiag_ > epsdiag_cap_) epsdiag_ = epsdiag_cap_;
}

// One numeric factorisation, the sparse levels by the fused kernels (fused)
// or the per-phase ones, the dense tail by the look-ahead (tail_fused) or
// the per-phase kernels; returns false when fused kernels bailed out
// (flags[1] says where; nothing of a bailed part may then be used).
bool KktDevice::factor_pass(const double* dE, const double* dD, bool fused, bool tail_fused) {
    hipStream_t s = stream_;
    if (timing_) IPO_HIP_CHECK(hipEventRecord(ev0_, s));
    const PlanView pv = IPO_VIEW();
    const int nz = static_cast<int>(plan_.amap.size());
    if (plan_.nt > 0 && !xch_) {
        // the sparse panels, then the tail's lower block triangle only (the
        // sharded solve sums the whole tail across shards: cleared whole)
        if (plan_.off_tail > 0) IPO_HIP_CHECK(hipMemsetAsync(dLx_.get(), 0, plan_.off_tail * sizeof(double), s));
        hipLaunchKernelGGL(k_zero_tail_lower, dim3(plan_.nt), dim3(NT), 0, s, dLx_.get() + plan_.off_tail, plan_.nt);
    } else {
        IPO_HIP_CHECK(hipMemsetAsync(dLx_.get(), 0, dLx_.bytes(), s));
    }
    if (nz > 0) hipLaunchKernelGGL(k_assemble_A, dim3(ceil_div(nz, NT)), dim3(NT), 0, s, nz, dA_.get(), damap_.get(), dLx_.get());
    if (qnz_ > 0)
        hipLaunchKernelGGL(k_assemble_Q, dim3(ceil_div(qnz_, NT)), dim3(NT), 0, s, qnz_, dQ_.get(), dqmap_.get(),
                           static_cast<double>(qmax_), dLx_.get());
    hipLaunchKernelGGL(k_assemble_diag, dim3(ceil_div(T_, NT)), dim3(NT), 0, s, T_, m_, dperm_.get(), dE, dD, epsdiag_,
                       ddslot_.get(), dLx_.get(), dLive_.get(), dDscale_.get(), shard_minor() ? plan_.tail_c0 : T_,
                       dFlags_.get(), dkQ_.get() ? dQdiag_.get() : static_cast<const double*>(nullptr),
                       static_cast<double>(qmax_));
    const TailView tv = tail_view();
    // the sparse levels and the dense tail's gather: the same launches every
    // factorisation of a plan (fixed arguments), so the fused form can be
    // captured once as a HIP graph and replayed (IPO_HIP_GRAPH=1, opt-in;
    // per-phase timing and the gather stamps launch them one by one).
    // Measured: dfl001 unchanged (292.9 / 292.8 against 293.7 / 291.5 it/s),
    // 25fv47 by intpt +1-3 %; the launches' cost is on the device (~4.5 us
    // per dispatch), not the host's enqueue, and rocprofv3 --kernel-trace
    // --stats crashed in the runtime on the replayed graph, so off
    if (graph_on_ && fused && !timing_ && gst_group_ < 0 && !xch_) {
        if (!lvl_exec_) {
            hipGraph_t g = nullptr;
            IPO_HIP_CHECK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
            enqueue_levels(pv, tv, fused, s);
            IPO_HIP_CHECK(hipStreamEndCapture(s, &g));
            const hipError_t e = hipGraphInstantiate(&lvl_exec_, g, nullptr, nullptr, 0);
            (void)hipGraphDestroy(g);
            IPO_HIP_CHECK(e);
        }
        IPO_HIP_CHECK(hipGraphLaunch(lvl_exec_, s));
    } else {
        enqueue_levels(pv, tv, fused, s);
    }
    if (plan_.nt > 0) {
        // shards: S = sum of every shard's assembled + gathered tail (exchange.h)
        xsum(tv.S, static_cast<size_t>(plan_.nt) * plan_.nt, RedOp::Sum);
        xsum(dDscale_.get() + plan_.tail_c0, plan_.nt, RedOp::Sum);
        if (tail_fused && tail_chain_ && !chain_off_ && tv.dep == 1) {   // kkt_dense.hip, k_tail_chain_run
            launch_tail_chain_run();
        } else if (tail_fused && tail_run_) {     // one persistent launch (kkt_dense.hip, k_tail_run)
            launch_tail_from(0, true);
        } else if (tail_fused) {     // look-ahead steps (kkt_dense.hip, k_tail_pr)
            // one event pair around the steps (a pair per launch added its
            // own ~2.5 us to every launch's time: the phase's average launch
            // would not be the kernel's)
            ph_begin(s);
            for (int t = 0; t < plan_.ntb; t++) launch_tail_step(pv, tv, t, s);
            ph_end(kPhTail, plan_.ntb, s);
        } else
        for (int kb = 0; kb < plan_.ntb; kb++) {
            const int k0 = kb * kPanelCols, nc = std::min(kPanelCols, plan_.nt - k0);
            const int below = plan_.nt - k0 - nc;
            ph_begin(s);
            {
                launch_diag(pv, nullptr, 0, 1, tv, kb, s);
                ph_end(kPhDiag, 1, s);
                if (below > 0) {
                    ph_begin(s);
                    launch_trsm(pv, 0, -1, tv, kb, s);
                    ph_end(kPhTrsm, 1, s);
                }
            }
            if (below > 0) {
                const int nb = plan_.ntb - kb - 1;
                ph_begin(s);
                hipLaunchKernelGGL(k_tail_syrk, dim3(nb * (nb + 1) / 2), dim3(NT), 0, s, pv, tv, kb);
                ph_end(kPhSyrk, 1, s);
            }
        }
    }
    return finish_pass(fused || tail_fused);
}

// The sparse levels (gather, then panels, level by level) and the dense
// tail's gather of one factorisation, enqueued on s.
void KktDevice::enqueue_levels(const PlanView& pv, const TailView& tv, bool fused, hipStream_t s) {
    for (int l = 0; l < plan_.nlevels; l++) {
        const int u0 = plan_.unit_level_ptr[l], u1 = plan_.unit_level_ptr[l + 1];
        if (u1 <= u0) continue;
        if (l > 0) {
            ph_begin(s);
            const int nl = launch_gather(pv, tv, -1, l, s);
            ph_end(kPhGather, nl, s);
        }
        const int q0 = plan_.level_ptr[l], q1 = plan_.level_ptr[l + 1];
        ph_begin(s);
        if (fused && split_level_[l]) {
            launch_diag(pv, dlevel_sups_.get(), q0, q1 - q0, tv, 0, s);
            launch_trsm(pv, u0, u1 - u0, tv, 0, s);
            ph_end(kPhDiag, 2, s);
        } else if (fused) {
            const int nsm = small_ptr_[l + 1] - small_ptr_[l], nfu = fu_ptr_[l + 1] - fu_ptr_[l];
            const int n1 = small1_cnt_[l];
            if (merge_panels_ && nfu > 0 && nsm > n1) {
                launch_panel_small(pv, dsmall_sups_.get(), small_ptr_[l], n1, tv.sdep, s, n1);
                launch_panel_ws(pv, dfu_sup_.get(), dfu_j_.get(), fu_ptr_[l], nfu, tv, dsmall_sups_.get(),
                                small_ptr_[l] + n1, nsm - n1, tv.sdep, s);
                ph_end(kPhDiag, 1 + (n1 > 0), s);
            } else {
                launch_panel_small(pv, dsmall_sups_.get(), small_ptr_[l], nsm, tv.sdep, s, n1);
                launch_panel(pv, dfu_sup_.get(), dfu_j_.get(), fu_ptr_[l], nfu, tv, -1, s);
                ph_end(kPhDiag, (nsm > 0) + (nfu > 0), s);
            }
        } else {
            launch_diag(pv, dlevel_sups_.get(), q0, q1 - q0, tv, 0, s);
            ph_end(kPhDiag, 1, s);
            ph_begin(s);
            launch_trsm(pv, u0, u1 - u0, tv, 0, s);
            ph_end(kPhTrsm, 1, s);
        }
    }
    if (plan_.nt > 0) {
        ph_begin(s);
        const int nl = launch_gather(pv, tv, 0, plan_.nlevels, s);
        ph_end(kPhGather, nl, s);
    }
}

// min |d| over the factor (ldlt.c:293-306), the dependent-pivot count and
// the fused kernels' bail-out flags, to the host
bool KktDevice::finish_pass(bool fused) {
    hipStream_t s = stream_;
    IPO_HIP_CHECK(hipGetLastError());
    hipLaunchKernelGGL(k_min_abs_partial, dim3(kRedBlocks), dim3(NT), 0, s, dDg_.get(), T_, dPart_.get());
    if (xch_) {   // every shard must take the same eps_diag / dependent-pivot / redo decisions
        hipLaunchKernelGGL(k_finish_reduce, dim3(1), dim3(kRedThreads), 0, s, dPart_.get(), 1, 1u, dScal_.get());
        hipLaunchKernelGGL(k_flag_to_scalar, dim3(1), dim3(1), 0, s, dFlags_.get(), dScal_.get() + 1);
        hipLaunchKernelGGL(k_flag_to_scalar, dim3(1), dim3(1), 0, s, dFlags_.get() + 1, dScal_.get() + 2);
        xsum(dScal_.get(), 3, RedOp::Max);
        hipLaunchKernelGGL(k_pack_ints, dim3(1), dim3(3), 0, s, dFlags_.get(), 3, dScal_.get() + 3);
    } else {
        // min|d| and the three flags in one read-back, one launch
        hipLaunchKernelGGL(k_finish_reduce_pack, dim3(1), dim3(kRedThreads), 0, s, dPart_.get(), 1, 1u, dScal_.get(),
                           static_cast<const int*>(dFlags_.get()), 3, dScal_.get() + 3);
    }
    IPO_HIP_CHECK(hipMemcpyAsync(hScal_, dScal_.get(), 5 * sizeof(double), hipMemcpyDeviceToHost, s));
    if (timing_) IPO_HIP_CHECK(hipEventRecord(ev1_, s));
    IPO_HIP_CHECK(hipStreamSynchronize(s));
    if (gst_n_ > 0) {      // developer stamps of one gather launch (IPO_HIP_GATHER_STAMPS)
        std::vector<long long> st(1024 * 8);
        IPO_HIP_CHECK(hipMemcpy(st.data(), dGStamp_.get(), st.size() * sizeof(long long), hipMemcpyDeviceToHost));
        long long t0 = st[0];
        for (int b = 0; b < std::min(gst_n_, 1024); b++) t0 = std::min(t0, st[b * 8]);
        std::fprintf(stderr, "gather stamps group %d, %d workgroups (us from first start: start rec val mfma acc put slots)\n",
                     gst_group_, gst_n_);
        for (int b = 0; b < std::min(gst_n_, 1024); b++) {
            const long long* q = st.data() + b * 8;
            std::fprintf(stderr, "  wg %4d: %6.2f %6.2f %6.2f %6.2f %6.2f %6.2f  %lld\n", b, (q[0] - t0) / 100.0,
                         (q[1] - t0) / 100.0, (q[2] - t0) / 100.0, (q[3] - t0) / 100.0, (q[4] - t0) / 100.0,
                         (q[5] - t0) / 100.0, q[6]);
        }
        gst_n_ = 0;
        gst_group_ = -1;
    }
    {
        int f[3];
        std::memcpy(f, hScal_ + 3, sizeof(f));
        hFlags_[0] = f[0];
        hFlags_[1] = f[1];
        hFlags_[4] = f[2];
    }
    if (timing_) {
        float ms = 0;
        IPO_HIP_CHECK(hipEventElapsedTime(&ms, ev0_, ev1_));
        tm_.factor_ms += ms;
        ph_collect();
    }
    const bool bail = xch_ ? hScal_[2] > 0 : hFlags_[1] != 0;
    return !(fused && bail);
}

// The dense tail's look-ahead steps [t0, ntb) as one persistent launch
// (k_tail_run).  reset: the factorisation's first run (every counter
// zeroed); a run resumed by repair_tail keeps pdone / vseq, which hold
// exactly the items of launches <= tb (later items were skipped uncounted).
void KktDevice::launch_tail_from(int t0, bool reset) {
    hipStream_t s = stream_;
    const PlanView pv = IPO_VIEW();
    const size_t ncnt = reset ? drun_cnt_.size() : 1;
    IPO_HIP_CHECK(hipMemsetAsync(drun_cnt_.get(), 0, ncnt * sizeof(int), s));
    TailRun rc;
    rc.items = drun_items_.get() + run_ptr_[t0];
    rc.n = run_ptr_[plan_.ntb] - run_ptr_[t0];
    rc.t0 = t0;
    rc.ticket = drun_cnt_.get();
    rc.pdone = drun_cnt_.get() + 1;
    rc.vseq = drun_cnt_.get() + 1 + plan_.ntb;
    if (run_winpub_) {
        if (run_epoch_ == INT_MAX) {      // (never within a process's life: one epoch per factorisation)
            IPO_HIP_CHECK(hipMemsetAsync(drun_wflag_.get(), 0, drun_wflag_.bytes(), s));
            run_epoch_ = 0;
        }
        rc.pub = drun_pub_.get();
        rc.wflag = drun_wflag_.get();
        rc.pread = rc.vseq + static_cast<size_t>(plan_.ntb) * plan_.ntb;
        // a resumed run: steps >= t0 count their readers afresh
        if (!reset) IPO_HIP_CHECK(hipMemsetAsync(rc.pread + t0, 0, (plan_.ntb - t0) * sizeof(int), s));
        rc.epoch = ++run_epoch_;
    }
    ph_begin(s);
    launch_tail_run(pv, tail_view(), rc, s);
    ph_end(kPhTail, rc.n > 0, s);
}

// The dense tail around a chain workgroup (kkt_dense.hip, k_tail_chain_run):
// every counter zeroed, one launch of the whole schedule.
void KktDevice::launch_tail_chain_run() {
    hipStream_t s = stream_;
    const PlanView pv = IPO_VIEW();
    IPO_HIP_CHECK(hipMemsetAsync(dchain_cnt_.get(), 0, dchain_cnt_.bytes(), s));
    const int ntb = plan_.ntb;
    ChainRun rc;
    rc.items = dchain_items_.get();
    rc.n = chain_n_;
    rc.ticket = dchain_cnt_.get();
    rc.abort = rc.ticket + 1;
    rc.pdone = rc.ticket + 2;
    rc.rdone = rc.pdone + ntb;
    rc.vseq = rc.rdone + static_cast<size_t>(ntb) * ntb;
    rc.dwin = rc.vseq + static_cast<size_t>(ntb) * ntb;
    rc.dpub = dchain_pub_.get();
    rc.save = dchain_save_.get();
    rc.latest = run_latest_;
    ph_begin(s);
    launch_tail_chain(pv, tail_view(), rc, s);
    ph_end(kPhTail, 1, s);
}

// The look-ahead dense tail bailed at block column tb (a pivot failed the
// zero test; launches after it did nothing): the sparse factor and block
// columns < tb stand, column tb holds the updates of blocks <= tb - 2 (its
// panel stores S only once it holds) and every column right of it what its
// visits up to launch tb gave it.  Apply block tb - 1 to column tb, factor
// column tb with the dependent-pivot rounds (k_tail_dep), and resume
// the look-ahead at tb + 1 with the same visit schedule: the fast path's
// operations with block column tb's panel replaced by k_diag + k_trsm.
// Repeats while a later column bails.
void KktDevice::repair_tail() {
    hipStream_t s = stream_;
    const PlanView pv = IPO_VIEW();
    for (;;) {
        const int tb = hFlags_[4] - 1;
        tm_.tail_repairs++;
        if (timing_) IPO_HIP_CHECK(hipEventRecord(ev0_, s));
        IPO_HIP_CHECK(hipMemsetAsync(dFlags_.get() + 1, 0, 2 * sizeof(int), s));
        TailView tv = tail_view();
        if (hFlags_[1] & 16) launch_tail_restore(pv, tv, tb, s);   // other workgroups of the DEP pass wrote
        ph_begin(s);
        if (tb > 0) launch_tail_colupdate(pv, tv, tb - 1, s);
        ph_end(kPhTail, tb > 0, s);
        // block column tb with the dependent-pivot rule, one round per dependent pivot
        IPO_HIP_CHECK(hipMemsetAsync(dDepI_.get(), 0, 8 * sizeof(int), s));
        // rounds enqueued kDepBatch at a time (a round after the last is a
        // no-op), one host read-back per batch instead of per round; round r
        // writes state copy (r + 1) & 1, so the batch's last round wrote
        // copy (r + kDepBatch) & 1
        constexpr int kDepBatch = 4;
        for (int r = 0;; r += kDepBatch) {
            if (r > kPanelCols + 1) throw std::runtime_error("kkt: dense-tail dependent-pivot rounds did not finish");
            ph_begin(s);
            for (int b = 0; b < kDepBatch; b++)
                launch_tail_dep_round(pv, tv, tb, r + b, dDepSt_.get(), dDepI_.get(), s);
            ph_end(kPhTail, kDepBatch, s);
            IPO_HIP_CHECK(hipMemcpyAsync(hFlags_ + 6, dDepI_.get() + 4 * ((r + kDepBatch) & 1) + 2, sizeof(int),
                                         hipMemcpyDeviceToHost, s));
            IPO_HIP_CHECK(hipStreamSynchronize(s));
            tm_.tail_dep_rounds += kDepBatch;
            if (hFlags_[6]) break;
        }
        if (tail_run_) {
            launch_tail_from(tb + 1, false);
        } else {
            ph_begin(s);
            for (int t = tb + 1; t < plan_.ntb; t++) launch_tail_step(pv, tail_view(), t, s);
            ph_end(kPhTail, plan_.ntb - tb - 1, s);
        }
        if (finish_pass(true)) break;
        if ((hFlags_[1] & ~16) != 4 || hFlags_[4] - 1 <= tb)   // cannot happen: a later tail column or nothing
            throw std::runtime_error("kkt: dense-tail repair did not advance");
    }
}

// Gather launch of one level (tail < 0) or of the dense tail (group =
// nlevels): every chunk; split units combined by their last-arriving chunk.
int KktDevice::launch_gather(const PlanView& pv, const TailView& tv, int tail, int group, hipStream_t s) {
    const int c0 = ck_ptr_[group], c1 = ck_ptr_[group + 1];
    if (c1 <= c0) return 0;
    const SlotRec* recs = tail < 0 ? dslot_rec_.get() : dtail_slot_rec_.get();
    // groups whose split units have many chunks sum their partials four
    // at a time (more registers: three waves per SIMD drop to two, which
    // the gathers of the other groups would pay for)
    // developer stamps (IPO_HIP_GATHER_STAMPS=<group>): per workgroup
    // s_memrealtime at start / records / values / MFMA / put / stores
    long long* stq = nullptr;
    if (gst_group_ == group && tail < 0 && ck_kind_[group] > 0) {
        if (!dGStamp_.get()) dGStamp_.alloc(1024 * 8);
        stq = dGStamp_.get();
        gst_n_ = c1 - c0;
    }
    if (ck_kind_[group] == 2) {
        hipLaunchKernelGGL(k_update_quad, dim3(c1 - c0), dim3(NT), 0, s, pv, tv, recs, dck_u_.get(), dck_b_.get(),
                           dck_e_.get(), dck_part_.get(), c0, stq);
        return 1;
    }
    if (ck_kind_[group] == 1) {
        if (ck_wide_[group])
        hipLaunchKernelGGL(k_update_flat<4>, dim3(c1 - c0), dim3(NT), 0, s, pv, tv, tail, recs, dck_u_.get(),
                           dck_b_.get(), dck_e_.get(), dck_part_.get(), c0, dPartialTile_.get(), dck_q_.get(),
                           dsp_p0_.get(), dsp_n_.get(), dSplitCnt_.get(), stq);
        else
        hipLaunchKernelGGL(k_update_flat<1>, dim3(c1 - c0), dim3(NT), 0, s, pv, tv, tail, recs, dck_u_.get(),
                           dck_b_.get(), dck_e_.get(), dck_part_.get(), c0, dPartialTile_.get(), dck_q_.get(),
                           dsp_p0_.get(), dsp_n_.get(), dSplitCnt_.get(), stq);
        return 1;
    }
    static const int occ = [] {
        const char* e = std::getenv("IPO_HIP_UPDATE_OCC");
        return e ? std::atoi(e) : 4;
    }();
    auto go = [&](auto kern) {
        hipLaunchKernelGGL(kern, dim3(c1 - c0), dim3(NT), 0, s, pv, tv, tail, recs, dck_u_.get(), dck_b_.get(),
                           dck_e_.get(), dck_part_.get(), c0, dPartialTile_.get(), dck_q_.get(), dsp_p0_.get(),
                           dsp_n_.get(), dSplitCnt_.get());
    };
    if (ck_wide_[group]) {
        // (four partials in flight spill at 128 and at 168 VGPRs; 3 per CU
        // with 16 spilled measured no faster than 2 per CU)
        go(k_update<4, 1>);
    } else {
        if (occ == 4) go(k_update<1, 4>);
        else go(k_update<1, 1>);
    }
    return 1;
}

hipEvent_t KktDevice::next_event() {
    if (kev_used_ == kev_.size()) {
        hipEvent_t e;
        IPO_HIP_CHECK(hipEventCreate(&e));
        kev_.push_back(e);
    }
    return kev_[kev_used_++];
}

void KktDevice::ph_begin(hipStream_t s) {
    if (!timing_) return;
    mark_b_ = next_event();
    IPO_HIP_CHECK(hipEventRecord(mark_b_, s));
}

void KktDevice::ph_end(int phase, int launches, hipStream_t s) {
    if (!timing_) return;
    hipEvent_t e = next_event();
    IPO_HIP_CHECK(hipEventRecord(e, s));
    marks_.push_back({mark_b_, e, phase, launches});
}

void KktDevice::ph_collect() {
    for (const PhaseMark& mk : marks_) {
        float ms = 0;
        IPO_HIP_CHECK(hipEventElapsedTime(&ms, mk.b, mk.e));
        tm_.phase_ms[mk.phase] += ms;
        tm_.phase_launches[mk.phase] += mk.launches;
    }
    marks_.clear();
    kev_used_ = 0;
}

// Substitution sweeps for R right-hand sides stored at dz + r * K.
template <int R>
void KktDevice::sweep(double* dz, const double* epsp) {
    hipStream_t s = stream_;
    const PlanView pv = IPO_VIEW();
    const SweepVecs V{dz, static_cast<size_t>(T_), dYbuf_.get(), ybuf_stride_};
    const size_t ps = partial_stride_;
    if (timing_) IPO_HIP_CHECK(hipEventRecord(ev2_, s));
    ph_begin(s);
    for (int l = 0; l < sf_level_; l++) {
        const int q0 = plan_.level_ptr[l], q1 = plan_.level_ptr[l + 1];
        const int cb = chunk_ptr_[l], ce = chunk_ptr_[l + 1];
        if (ce > cb) {
            hipLaunchKernelGGL(k_fwd_diag<R>, dim3(q1 - q0), dim3(NT), 0, s, pv, dlevel_sups_.get(), q0,
                               dyrow_ptr_.get(), dyrow_idx_.get(), V, epsp);
            hipLaunchKernelGGL(k_fwd_gemv<R>, dim3(ce - cb), dim3(NT), 0, s, pv, dchunk_sup_.get(), dchunk_r0_.get(), cb,
                               V);
        } else {
            const int nl = leaf_cnt_[l], n8 = leaf8_cnt_[l];
            if (n8 > 0)
                hipLaunchKernelGGL(k_fwd_leaf8<R>, dim3(ceil_div(n8, NT / kSmallLeaf)), dim3(NT), 0, s, pv,
                                   dsweep_sups_.get(), q0, n8, dyrow_ptr_.get(), dyrow_idx_.get(), V, epsp);
            if (nl > n8 && q1 - q0 > nl && merge_levels_) {
                const int nlb = ceil_div(nl - n8, NT / 64);
                hipLaunchKernelGGL(k_fwd_level<R>, dim3(nlb + q1 - q0 - nl), dim3(NT), 0, s, pv, dsweep_sups_.get(),
                                   q0 + n8, nl - n8, nlb, dyrow_ptr_.get(), dyrow_idx_.get(), V, epsp);
            } else {
                if (nl > n8)
                    hipLaunchKernelGGL(k_fwd_leaf<R>, dim3(ceil_div(nl - n8, NT / 64)), dim3(NT), 0, s, pv,
                                       dsweep_sups_.get(), q0 + n8, nl - n8, dyrow_ptr_.get(), dyrow_idx_.get(), V,
                                       epsp);
                if (q1 - q0 > nl)
                    hipLaunchKernelGGL(k_forward<R>, dim3(q1 - q0 - nl), dim3(NT), 0, s, pv, dsweep_sups_.get(),
                                       q0 + nl, dyrow_ptr_.get(), dyrow_idx_.get(), V, epsp);
            }
        }
    }
    if (sf_level_ < plan_.nlevels) {      // the narrow top levels in one launch
        const SfView sf{dsf_items_f_.get(), nsf_f_, dsf_fcnt_.get(), dsf_fflag_.get(), dsf_need_.get(), dsf_par_.get(),
                        dsf_zbase_.get(), dsf_zpi_.get(), dZpad_.get(), zpad_stride_, ++sf_fwd_epoch_,
                        dsf_ticket_.get(), sf_tbase(0, nsf_f_)};
        const bool pre = pre_cols_ > 0 || dylate_ptr_.get();
        if (pre_cols_ > 0)
            hipLaunchKernelGGL(k_fwd_pre<R>, dim3(ceil_div(pre_cols_, NT)), dim3(NT), 0, s, pre_cols_, dpre_col_.get(),
                               dpre_ptr_.get(), dpre_idx_.get(), V);
        hipLaunchKernelGGL(k_fwd_sf<R>, dim3(std::min(sf_grid_, nsf_f_)), dim3(NT), kChainLds, s, pv, sf,
                           pre ? dylate_ptr_.get() : dyrow_ptr_.get(), pre ? dylate_idx_.get() : dyrow_idx_.get(),
                           dchunk_r0_.get(), V, epsp);
    }
    if (plan_.nt > 0) {
        const TailView tv = tail_view();
        tail_rhs_begin(dz, R);
        hipLaunchKernelGGL(k_tail_gather<R>, dim3(ceil_div(plan_.nt, 4)), dim3(NT), 0, s, tv, dyrow_ptr_.get(),
                           dyrow_idx_.get(), V);
        tail_rhs_end(dz, R);
        if (chain_lead_) {
            const int grid = 1 + std::max(0, plan_.ntb - 1 - kLeadBlocks);
            if (lead_ticket_next_ + grid > (1LL << 30)) {
                IPO_HIP_CHECK(hipMemsetAsync(dlead_ticket_.get(), 0, sizeof(int), s));
                lead_ticket_next_ = 0;
            }
            const int tb = static_cast<int>(lead_ticket_next_);
            lead_ticket_next_ += grid;
            hipLaunchKernelGGL(k_tail_fwd_lead<R>, dim3(grid), dim3(kLeadNT), kChainLds, s, pv, tv, V, epsp,
                               dChainGran_.get(), dChainGran_.get() + static_cast<size_t>(plan_.ntb) * 2 * 128,
                               ++chain_epoch_, dlead_ticket_.get(), tb);
        } else if (chain_pairs_)
            hipLaunchKernelGGL(k_tail_fwd_pair<R>, dim3((plan_.ntb + 1) / 2), dim3(NT), kPairFwdLds, s, pv, tv, V, epsp,
                               dChainGran_.get(), ++chain_epoch_);
        else
            hipLaunchKernelGGL(k_tail_fwd_chain<R>, dim3(plan_.ntb), dim3(NT), kChainLds, s, pv, tv, V, epsp,
                               dChainGran_.get(), ++chain_epoch_);
#ifdef IPO_LEAD_STAMPS
        if (chain_lead_ && chain_epoch_ % 64 == 41) {
            double st[8][4];
            IPO_HIP_CHECK(hipStreamSynchronize(s));
            IPO_HIP_CHECK(hipMemcpyFromSymbol(st, HIP_SYMBOL(g_lead_stats), sizeof(st)));
            std::fprintf(stderr, "lead R %d ntb %d per step us: solver wait-A %.3f tri %.3f wait-B %.3f\n", R, plan_.ntb,
                         st[0][0], st[0][1], st[0][2]);
            for (int w = 1; w <= 4; w++)
                std::fprintf(stderr, "  wave %d: partial wait %.3f (%g polls) phase3 %.3f loads %.3f\n", w, st[w][0],
                             st[w][1], st[w][2], st[w][3]);
        }
#endif
    }
    ph_end(kPhForward, fwd_launches_, s);
    ph_begin(s);
    if (plan_.nt > 0) {
        const TailView tv = tail_view();
        if (chain_pairs_)
            hipLaunchKernelGGL(k_tail_bwd_pair<R>, dim3((plan_.ntb + 1) / 2), dim3(NT), kPairBwdLds, s, pv, tv, V, epsp,
                               dChainGran_.get(), ++chain_epoch_);
        else
            hipLaunchKernelGGL(k_tail_bwd_chain<R>, dim3(plan_.ntb), dim3(NT), kChainLds, s, pv, tv, V, epsp,
                               dChainGran_.get(), ++chain_epoch_);
    }
    if (sf_level_ < plan_.nlevels) {
        const SfView sf{dsf_items_b_.get(), nsf_b_, dsf_bcnt_.get(), dsf_bflag_.get(), dsf_need_.get(), dsf_par_.get(),
                        dsf_zbase_.get(), dsf_zpi_.get(), dZpad_.get(), zpad_stride_, ++sf_bwd_epoch_,
                        dsf_ticket_.get() + 1, sf_tbase(1, nsf_b_)};
        hipLaunchKernelGGL(k_bwd_sf<R>, dim3(std::min(sf_grid_, nsf_b_)), dim3(NT), kChainLds, s, pv, sf,
                           dchunk_r0_.get(), dsup_chunk0_.get(), dPartial_.get(), ps, V, epsp);
    }
    for (int l = sf_level_ - 1; l >= 0; l--) {
        const int q0 = plan_.level_ptr[l], q1 = plan_.level_ptr[l + 1];
        const int cb = chunk_ptr_[l], ce = chunk_ptr_[l + 1];
        if (ce > cb) {
            hipLaunchKernelGGL(k_bwd_partial<R>, dim3(ce - cb), dim3(NT), 0, s, pv, dchunk_sup_.get(), dchunk_r0_.get(),
                               cb, V, dPartial_.get(), ps);
            hipLaunchKernelGGL(k_bwd_finish<R>, dim3(q1 - q0), dim3(NT), 0, s, pv, dlevel_sups_.get(), q0,
                               dsup_chunk0_.get(), dPartial_.get(), ps, V, epsp);
        } else {
            const int nl = leaf_cnt_[l], n8 = leaf8_cnt_[l];
            if (n8 > 0)
                hipLaunchKernelGGL(k_bwd_leaf8<R>, dim3(ceil_div(n8, NT / kSmallLeaf)), dim3(NT), 0, s, pv,
                                   dsweep_sups_.get(), q0, n8, V, epsp);
            if (nl > n8 && q1 - q0 > nl && merge_levels_) {
                const int nlb = ceil_div(nl - n8, NT / 64);
                hipLaunchKernelGGL(k_bwd_level<R>, dim3(nlb + q1 - q0 - nl), dim3(NT), 0, s, pv, dsweep_sups_.get(),
                                   q0 + n8, nl - n8, nlb, V, epsp);
            } else {
                if (nl > n8)
                    hipLaunchKernelGGL(k_bwd_leaf<R>, dim3(ceil_div(nl - n8, NT / 64)), dim3(NT), 0, s, pv,
                                       dsweep_sups_.get(), q0 + n8, nl - n8, V, epsp);
                if (q1 - q0 > nl)
                    hipLaunchKernelGGL(k_backward<R>, dim3(q1 - q0 - nl), dim3(NT), 0, s, pv, dsweep_sups_.get(),
                                       q0 + nl, V, epsp);
            }
        }
    }
    ph_end(kPhBackward, bwd_launches_, s);
    IPO_HIP_CHECK(hipGetLastError());
    if (timing_) {
        IPO_HIP_CHECK(hipEventRecord(ev3_, s));
        IPO_HIP_CHECK(hipEventSynchronize(ev3_));
        float ms = 0;
        IPO_HIP_CHECK(hipEventElapsedTime(&ms, ev2_, ev3_));
        tm_.sweep_ms += ms;
        ph_collect();
        tm_.phase_count[kPhForward]++;
        tm_.phase_count[kPhBackward]++;
    }
}

// Ticket base of the next sync-free launch of direction d over nitems items:
// each launch draws nitems + grid tickets; the counter is cleared (in stream
// order) before it could overflow.
int KktDevice::sf_tbase(int d, int nitems) {
    const long long draw = static_cast<long long>(nitems) + std::min(sf_grid_, nitems);
    if (sf_ticket_next_[d] + draw > (1LL << 30)) {
        IPO_HIP_CHECK(hipMemsetAsync(dsf_ticket_.get() + d, 0, sizeof(int), stream_));
        sf_ticket_next_[d] = 0;
    }
    const int base = static_cast<int>(sf_ticket_next_[d]);
    sf_ticket_next_[d] += draw;
    return base;
}

// Very large dense tails (more blocks than the chain kernels keep resident):
// one right-hand side, per-block launches.
void KktDevice::sweep_blocked(double* dz, const double* epsp) {
    hipStream_t s = stream_;
    const PlanView pv = IPO_VIEW();
    const SweepVecs V{dz, static_cast<size_t>(T_), dYbuf_.get(), ybuf_stride_};
    const size_t ps = partial_stride_;
    for (int l = 0; l < plan_.nlevels; l++) {
        const int q0 = plan_.level_ptr[l], q1 = plan_.level_ptr[l + 1];
        const int cb = chunk_ptr_[l], ce = chunk_ptr_[l + 1];
        if (ce > cb) {
            hipLaunchKernelGGL(k_fwd_diag<1>, dim3(q1 - q0), dim3(NT), 0, s, pv, dlevel_sups_.get(), q0,
                               dyrow_ptr_.get(), dyrow_idx_.get(), V, epsp);
            hipLaunchKernelGGL(k_fwd_gemv<1>, dim3(ce - cb), dim3(NT), 0, s, pv, dchunk_sup_.get(), dchunk_r0_.get(), cb,
                               V);
        } else {
            hipLaunchKernelGGL(k_forward<1>, dim3(q1 - q0), dim3(NT), 0, s, pv, dlevel_sups_.get(), q0,
                               dyrow_ptr_.get(), dyrow_idx_.get(), V, epsp);
        }
    }
    const TailView tv = tail_view();
    const int nt = plan_.nt;
    tail_rhs_begin(dz, 1);
    hipLaunchKernelGGL(k_tail_gather<1>, dim3(ceil_div(nt, 4)), dim3(NT), 0, s, tv, dyrow_ptr_.get(), dyrow_idx_.get(),
                       V);
    tail_rhs_end(dz, 1);
    for (int kb = 0; kb < plan_.ntb; kb++) {
        const int below = nt - std::min(nt, (kb + 1) * kPanelCols);
        hipLaunchKernelGGL(k_tail_fwd, dim3(std::max(1, ceil_div(below, 64))), dim3(NT), 0, s, pv, tv, kb, dz, epsp);
    }
    hipLaunchKernelGGL(k_tail_dscale, dim3(ceil_div(nt, NT)), dim3(NT), 0, s, pv, tv, dz, epsp);
    for (int kb = plan_.ntb - 1; kb >= 0; kb--) {
        const int left = kb * kPanelCols;
        hipLaunchKernelGGL(k_tail_bwd, dim3(std::max(1, ceil_div(left, 64))), dim3(NT), 0, s, pv, tv, kb, dz, epsp);
    }
    for (int l = plan_.nlevels - 1; l >= 0; l--) {
        const int q0 = plan_.level_ptr[l], q1 = plan_.level_ptr[l + 1];
        const int cb = chunk_ptr_[l], ce = chunk_ptr_[l + 1];
        if (ce > cb) {
            hipLaunchKernelGGL(k_bwd_partial<1>, dim3(ce - cb), dim3(NT), 0, s, pv, dchunk_sup_.get(), dchunk_r0_.get(),
                               cb, V, dPartial_.get(), ps);
            hipLaunchKernelGGL(k_bwd_finish<1>, dim3(q1 - q0), dim3(NT), 0, s, pv, dlevel_sups_.get(), q0,
                               dsup_chunk0_.get(), dPartial_.get(), ps, V, epsp);
        } else {
            hipLaunchKernelGGL(k_backward<1>, dim3(q1 - q0), dim3(NT), 0, s, pv, dlevel_sups_.get(), q0, V, epsp);
        }
    }
    IPO_HIP_CHECK(hipGetLastError());
}

// Sharded sweeps: the tail rows' right-hand side enters once (shard 0), and
// after the gather each shard holds its own blocks' contributions: sum them.
void KktDevice::tail_rhs_begin(double* dz, int R) {
    if (!shard_minor()) return;
    for (int r = 0; r < R; r++)
        IPO_HIP_CHECK(hipMemsetAsync(dz + (size_t)r * T_ + plan_.tail_c0, 0, sizeof(double) * plan_.nt, stream_));
}
void KktDevice::tail_rhs_end(double* dz, int R) {
    for (int r = 0; r < R; r++) xsum(dz + (size_t)r * T_ + plan_.tail_c0, plan_.nt, RedOp::Sum);
}

void KktDevice::set_long_rows(int row0) {
    if (xch_ || row0 < 0 || row0 >= m_) return;
    long_row0_ = row0;
    dLongAx_.alloc(2 * static_cast<size_t>(m_ - row0));
}

// rawsolve (ldlt.c:433-505) of R right-hand sides at dz + r * K, in place.
void KktDevice::rawsolve(double* dz, int R) {
    hipStream_t s = stream_;
    double* epsp = dScal_.get() + 4;        // eps of right-hand side r at epsp[r]
    if (ndep_ > 0) {
        // eps = epssol * max|z[0..n)| (ldlt.c:446: first n entries of the permuted vector)
        RedJobs j{};
        j.nj = R;
        for (int r = 0; r < R; r++) { j.a[r] = dz + (size_t)r * T_; j.b[r] = nullptr; j.len[r] = n_; j.op[r] = 1; }
        launch_reduce(j, dPart_.get(), epsp, s);
        hipLaunchKernelGGL(k_scale_scalar, dim3(1), dim3(64), 0, s, epsp, R, 1.0e-6);
        xsum(epsp, R, RedOp::Max);
    } else if (!eps_cleared_) {
        IPO_HIP_CHECK(hipMemsetAsync(epsp, 0, R * sizeof(double), s));
    }
    if (plan_.nt > 0 && plan_.ntb > kChainMaxBlocks) {
        for (int r = 0; r < R; r++) sweep_blocked(dz + (size_t)r * T_, epsp + r);
    } else if (R == 2) {
        sweep<2>(dz, epsp);
    } else {
        sweep<1>(dz, epsp);
    }
    tm_.rawsolves += R;
}

// Refined solves of R systems K [dy; dx] = [fy_r; fx_r] with the current
// factor, in place (ldlt.c:327-425).  Each right-hand side runs the
// reference's own refinement loop (first pass from the right-hand side,
// further passes on the KKT residual while it exceeds 1e-10 (max|b| + 1)
// and halves, the last correction undone if the residual grew); passes of
// both systems share one sweep.  Returns the reference's consistency flag
// of each system in ok[r].
void KktDevice::solve_multi(int R, const double* dE, const double* dD, double* const* dfy, double* const* dfx,
                            int* ok) {
    hipStream_t s = stream_;
    if (timing_) IPO_HIP_CHECK(hipEventRecord(ev0_, s));
    const int m = m_, n = n_, T = T_;
    {   // maxbc_r = MAX(maxv(fx_r), maxv(fy_r)) + 1   (ldlt.c:367)
        RedJobs j{};
        j.nj = 2 * R;
        for (int r = 0; r < R; r++) {
            j.a[2 * r] = dfx[r]; j.b[2 * r] = nullptr; j.len[2 * r] = n; j.op[2 * r] = 1;
            j.a[2 * r + 1] = dfy[r]; j.b[2 * r + 1] = nullptr; j.len[2 * r + 1] = m; j.op[2 * r + 1] = 1;
        }
        // read back with the first pass's residuals (no copy or wait of its own)
        launch_reduce(j, dPart_.get(), dScal_.get() + 8, s);
        xsum(dScal_.get() + 8, 2 * R, RedOp::Max);
    }
    double maxbc[2] = {0.0, 0.0}, rs[2] = {HUGE_VAL, HUGE_VAL}, rs_old[2] = {HUGE_VAL, HUGE_VAL};
    int pass[2] = {0, 0};
    bool active[2] = {R > 0, R > 1};
    auto zv = [&](int r) { return dZ_.get() + (size_t)r * T; };
    auto dyv = [&](int r) { return dDy_.get() + (size_t)r * m; };
    auto dxv = [&](int r) { return dDx_.get() + (size_t)r * n; };
    auto ryv = [&](int r) { return dRy_.get() + (size_t)r * m; };
    auto rxv = [&](int r) { return dRx_.get() + (size_t)r * n; };
    // the reference's consistency flag is that of each system's last rawsolve
    // (ldlt.c:379, 424): flags are cleared before every sweep, and the sweep's
    // right-hand-side slot q of an active system is read back after it
    int incons[2] = {0, 0};
    while (active[0] || active[1]) {
        {
            PermJobs J{};
            int na = 0;
            for (int r = 0; r < R; r++)
                if (active[r]) {
                    J.fy[na] = pass[r] == 0 ? dfy[r] : ryv(r);
                    J.fx[na] = pass[r] == 0 ? dfx[r] : rxv(r);
                    J.z[na] = zv(r);
                    na++;
                }
            hipLaunchKernelGGL(k_perm_in2, dim3(ceil_div(T, NT), na), dim3(NT), 0, s, T, m, dperm_.get(), J,
                               dIncons_.get(), dScal_.get() + 4);
        }
        eps_cleared_ = true;
        if (active[0] && active[1]) rawsolve(zv(0), 2);
        else rawsolve(zv(active[0] ? 0 : 1), 1);
        eps_cleared_ = false;
        int nq = 0;
        {
            PermJobs P{};
            ResJobs J{};
            const int mrow = xch_ ? m - nforced_ : long_row0_ >= 0 ? long_row0_ : m;
            for (int r = 0; r < R; r++) {
                if (!active[r]) continue;
                P.z[nq] = zv(r); P.dy[nq] = dyv(r); P.dx[nq] = dxv(r); P.mode[nq] = pass[r] == 0 ? 0 : 1;
                J.fy[nq] = dfy[r]; J.fx[nq] = dfx[r]; J.dy[nq] = dyv(r); J.dx[nq] = dxv(r);
                J.ry[nq] = ryv(r); J.rx[nq] = rxv(r);
                J.axl[nq] = xch_ ? dLinkAx_.get() + (size_t)r * nforced_
                                 : long_row0_ >= 0 ? dLongAx_.get() + (size_t)r * (m - long_row0_) : nullptr;
                nq++;
            }
            hipLaunchKernelGGL(k_perm_out2, dim3(ceil_div(T, NT), nq), dim3(NT), 0, s, T, m, diperm_.get(), P);
            for (int q = 0; q < nq; q++) {
                double* axl = const_cast<double*>(J.axl[q]);
                if (xch_) {
                    launch_link_ax(mrow, m, dkAt_.get(), diAt_.get(), dAt_.get(), J.dx[q], axl, s);
                    xsum(axl, nforced_, RedOp::Sum);
                } else if (long_row0_ >= 0) {
                    launch_link_ax(mrow, m, dkAt_.get(), diAt_.get(), dAt_.get(), J.dx[q], axl, s);
                }
            }
            hipLaunchKernelGGL(k_kkt_residual2, dim3(kRedBlocks, nq), dim3(kResThreads), 0, s, m, n, dkAt_.get(),
                               diAt_.get(), dAt_.get(), dkA_.get(), diA_.get(), dA_.get(), dE, dD, J, dPart_.get(), mrow,
                               dkQ_.get() ? dkQ_.get() : static_cast<const int*>(nullptr), diQ_.get(), dQ_.get(),
                               static_cast<double>(qmax_));
        }
        // residuals and the consistency flags in one read-back
        if (xch_) {
            hipLaunchKernelGGL(k_finish_reduce, dim3(1), dim3(kRedThreads), 0, s, dPart_.get(), nq, (1u << nq) - 1u,
                               dScal_.get());
            xsum(dScal_.get(), nq, RedOp::Max);
            hipLaunchKernelGGL(k_pack_ints, dim3(1), dim3(2), 0, s, dIncons_.get(), 2, dScal_.get() + 6);
        } else {
            hipLaunchKernelGGL(k_finish_reduce_pack, dim3(1), dim3(kRedThreads), 0, s, dPart_.get(), nq,
                               (1u << nq) - 1u, dScal_.get(), static_cast<const int*>(dIncons_.get()), 2,
                               dScal_.get() + 6);
        }
        IPO_HIP_CHECK(hipMemcpyAsync(hScal_, dScal_.get(), (pass[0] + pass[1] == 0 ? 8 + 2 * R : 7) * sizeof(double),
                                     hipMemcpyDeviceToHost, s));
        IPO_HIP_CHECK(hipStreamSynchronize(s));
        if (pass[0] + pass[1] == 0)
            for (int r = 0; r < R; r++)
                maxbc[r] = (hScal_[8 + 2 * r] > hScal_[8 + 2 * r + 1] ? hScal_[8 + 2 * r] : hScal_[8 + 2 * r + 1]) + 1;
        std::memcpy(hFlags_ + 2, hScal_ + 6, 2 * sizeof(int));
        int q = 0;
        for (int r = 0; r < R; r++) {
            if (!active[r]) continue;
            incons[r] = hFlags_[2 + q];
            rs_old[r] = rs[r];
            rs[r] = hScal_[q++];
            pass[r]++;
            active[r] = rs[r] > 1.0e-10 * maxbc[r] && rs[r] < rs_old[r] / 2;
        }
    }
    CopyOut co{};
    for (int r = 0; r < R; r++) {
        if (rs[r] > rs_old[r] && pass[r] > 1)
            hipLaunchKernelGGL(k_perm_out, dim3(ceil_div(T, NT)), dim3(NT), 0, s, T, m, diperm_.get(), zv(r), dyv(r),
                               dxv(r), 2);
        co.src[2 * r] = dyv(r); co.dst[2 * r] = dfy[r];
        co.src[2 * r + 1] = dxv(r); co.dst[2 * r + 1] = dfx[r];
    }
    // the solutions back into the callers' vectors: one launch for all
    // 2R copies (four copy-engine calls cost four host round trips)
    co.m = m;
    co.n = n;
    co.R = R;
    if (R > 0 && m + n > 0) hipLaunchKernelGGL(k_copy_out, dim3(ceil_div(R * (m + n), NT)), dim3(NT), 0, s, co);
    if (timing_) {   // otherwise the caller's next read-back orders the copies
        IPO_HIP_CHECK(hipEventRecord(ev1_, s));
        IPO_HIP_CHECK(hipStreamSynchronize(s));
        float ms = 0;
        IPO_HIP_CHECK(hipEventElapsedTime(&ms, ev0_, ev1_));
        tm_.solve_ms += ms;
    }
    tm_.solves += R;
    last_passes_ = pass[0] + pass[1];
    for (int r = 0; r < R; r++) ok[r] = incons[r] ? 0 : 1;
}

int KktDevice::solve(const double* dE, const double* dD, double* dfy, double* dfx) {
    int ok[1];
    solve_multi(1, dE, dD, &dfy, &dfx, ok);
    return ok[0];
}

int KktDevice::solve2(const double* dE, const double* dD, double* dfy1, double* dfx1, double* dfy2, double* dfx2) {
    double* fy[2] = {dfy1, dfy2};
    double* fx[2] = {dfx1, dfx2};
    int ok[2];
    solve_multi(2, dE, dD, fy, fx, ok);
    return ok[0] && ok[1];
}

void KktDevice::download_factor(double* lx, double* d, int* live) const {
    if (lx) dLx_.download(lx, plan_.lx_size, stream_);
    if (d) dDg_.download(d, T_, stream_);
    if (live) dLive_.download(live, T_, stream_);
    IPO_HIP_CHECK(hipStreamSynchronize(stream_));
}

}  // namespace ipo
