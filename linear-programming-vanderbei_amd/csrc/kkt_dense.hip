// kkt_dense.hip -- dense per-panel kernels of the supernodal LDL':
// diagonal-block factorisation (register fast path + the dependent-pivot
// path of ldlt.c:600-614) and the panel triangular solve L21 = A21 L11^-T D^-1.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <stdexcept>

#include "dev_common.h"
#include "hip_util.h"
#include "kkt_kernels.h"

namespace ipo {

namespace {

constexpr int TR = kTileRows;     // 64
constexpr int PC = kPanelCols;    // 64
constexpr int NT = 256;

// What the diagonal-block routines need from the plan, passed by value: a
// reference to the kernel's PlanView argument would force a copy of it into
// scratch memory (and a scratch load per use) once a non-inlined callee
// takes its address.
struct DiagCtx {
    double* dscale;
    double* dg;
    int* live;
    int* flags;
    const int* sign;
    double tau;
};

// Thread (row r = lane, part q0 = wave) of a 256-thread workgroup keeps
// the entries (r, 4q + q0), q = 0..15, of a 64-column row in registers.
// Column k = 4 qk + pk is visited with qk unrolled (a static register
// index) and pk a runtime loop, which keeps the code small: the dependency
// chain, not the flops, bounds these kernels, and a fully unrolled 64 x 64
// body does not fit the instruction cache.
// Fast path of the diagonal-block LDL' (256 threads, layout above).  Same
// operations in the same order as factor_diag_block below (bitwise
// identical results); returns false -- having written nothing -- as soon as
// a pivot fails the zero test, and the caller reruns the block with
// factor_diag_block, which owns the dependent-pivot rule (ldlt.c:600-614).
// On success stores L11' in the block's upper triangle, D in dg, mark = 1.
__device__ __forceinline__ bool factor_diag_fast(const DiagCtx p, double* panel, int ld, int nc, int c0,
                                                 double (*B)[PC + 1]) {
    __shared__ double colk[2][PC];        // double-buffered: one barrier per column
    __shared__ double dks[2];
    __shared__ int tinys[2];
    __shared__ double dv[PC];
    const int tid = threadIdx.x, r = tid & 63, q0 = tid >> 6;
    double a[16];
#pragma unroll
    for (int q = 0; q < 16; q++) {
        const int c = 4 * q + q0;
        const bool ok = r < nc && c <= r;
        const double t = panel[ok ? r + (size_t)c * ld : 0];
        a[q] = ok ? t : 0.0;
    }
    double dsc = (r < nc && (r & 3) == q0) ? p.dscale[c0 + r] : 0.0;   // kept by the diagonal's owner
    // k = 4 qk + pk: qk unrolled (static register index), pk a runtime loop.
    // Column k (pivot included) lives entirely in wave pk: that wave reads
    // the pivot by v_readlane, scales the column and publishes it; one
    // barrier later every wave applies the rank-1 update to its columns.
    bool tiny = false;
#pragma unroll
    for (int qk = 0; qk < 16; qk++) {
        for (int pk = 0; pk < 4; pk++) {
            const int k = 4 * qk + pk;
            if (k >= nc || tiny) break;
            const int buf = k & 1;
            if (q0 == pk) {
                const double dk = lane_bcast(a[qk], k);
                const double dsk = lane_bcast(dsc, k);
                const bool tz = fabs(dk) <= p.tau * dsk;      // uniform in the wave
                const bool below = !tz && r > k && r < nc;
                const double l = below ? a[qk] / dk : 0.0;
                if (below) a[qk] = l;
                colk[buf][r] = l;
                if (r == 0) { dks[buf] = dk; tinys[buf] = tz; dv[k] = dk; }
            }
            __syncthreads();
            if (tinys[buf]) { tiny = true; break; }
            const double dk = dks[buf];
            if (r > k && r < nc) {
                // all LDS reads first, then branch-free selects
                const double lr = colk[buf][r];
                double ck[16];
#pragma unroll
                for (int q = qk; q < 16; q++) ck[q] = colk[buf][4 * q + q0];
#pragma unroll
                for (int q = qk; q < 16; q++) {
                    const int c = 4 * q + q0;
                    const double tk = lr * (ck[q] * dk);
                    const bool u = c > k && c <= r;
                    a[q] = u ? a[q] - tk : a[q];
                    dsc = (u && c == r) ? dsc + fabs(tk) : dsc;
                }
            }
        }
    }
    if (tiny) return false;
    __syncthreads();
    // L11(r, c) -> upper slot (c, r) through an LDS transpose
#pragma unroll
    for (int q = 0; q < 16; q++) B[r][4 * q + q0] = a[q];
    __syncthreads();
    for (int rr = q0; rr < nc; rr += 4)
        if (r < rr) panel[r + (size_t)rr * ld] = B[rr][r];
    if (tid < nc) { p.dg[c0 + tid] = dv[tid]; p.live[c0 + tid] = 1; }
    return true;
}

__device__ __attribute__((noinline)) void factor_diag_block(double* dscale, double* dgp, int* livep, int* flags,
                                                          const int* sign, double tau, double* panel, int ld, int nc, int h,
                                                          int c0) {
    const DiagCtx p{dscale, dgp, livep, flags, sign, tau};
    __shared__ double B[PC][PC + 1];
    __shared__ double dv[PC];
    __shared__ int lv[PC];
    __shared__ double dsc[PC];
    __shared__ double red[4];
    __shared__ int ndep_sh;
    const int tid = threadIdx.x, nthr = blockDim.x, np = nthr >> 6;
    const int tr = tid & 63, tp = tid >> 6;     // row, part (np parts stride the columns)
    for (int c = tp; c < nc; c += np) B[tr][c] = (tr < nc && tr >= c) ? panel[tr + (size_t)c * ld] : 0.0;
    for (int k = tid; k < nc; k += nthr) dsc[k] = p.dscale[c0 + k];
    if (tid == 0) ndep_sh = 0;
    __syncthreads();
    for (int k = 0; k < nc; k++) {
        double dk = B[k][k];
        int alive = 1;
        if (fabs(dk) <= p.tau * dsc[k]) {         // ldlt.c:600 with a rounding-aware zero test
            // largest off-diagonal magnitude of column k after every update
            // from columns < k; rows below the block are rebuilt from the
            // (not yet solved) panel by a partial forward substitution
            // Only "mx < 1e-2" matters: the block's own rows are reduced
            // first, and when they already reach the threshold the costly
            // rows below (a partial substitution each) cannot change the
            // decision and are skipped.
            double mx = 0.0;
            for (int r = k + 1 + tid; r < nc; r += nthr) mx = ref_max(mx, ref_abs(B[r][k]));
            mx = wave_max(mx);
            if (tr == 0) red[tp] = mx;
            __syncthreads();
            if (tid == 0) {
                double m2 = red[0];
                for (int q = 1; q < np; q++) m2 = ref_max(m2, red[q]);
                red[0] = m2;
            }
            __syncthreads();
            const double mblk = red[0];
            __syncthreads();
            mx = 0.0;
            if (!(mblk >= 1.0e+6 * 1.0e-8)) {
                for (int rr = nc + tid; rr < h; rr += nthr) {
                    double w[PC];
                    for (int c = 0; c <= k; c++) w[c] = panel[rr + (size_t)c * ld];
                    for (int j = 0; j < k; j++) {
                        const double lj = lv[j] ? w[j] / dv[j] : 0.0;
                        for (int c = j + 1; c <= k; c++) w[c] -= lj * (B[c][j] * dv[j]);
                    }
                    mx = ref_max(mx, ref_abs(w[k]));
                }
            }
            mx = wave_max(mx);
            if (tr == 0) red[tp] = mx;
            __syncthreads();
            if (tid == 0) {
                double m2 = mblk;
                for (int q = 0; q < np; q++) m2 = ref_max(m2, red[q]);
                red[0] = m2;
            }
            __syncthreads();
            mx = red[0];
            if (mx < 1.0e+6 * 1.0e-8) alive = 0;                    // column dropped, d keeps its value
            else dk = (p.sign[c0 + k] < 0 ? -1.0 : 1.0) * 1.0e-8;   // y-nodes -, x-nodes +
            if (tid == 0) ndep_sh++;
            __syncthreads();
        }
        if (tid == 0) { dv[k] = dk; lv[k] = alive; }
        // scale column k first (lij = a / d), then update with lij * (ljk * d)
        for (int r = k + 1 + tid; r < nc; r += nthr) B[r][k] = alive ? B[r][k] / dk : 0.0;
        __syncthreads();
        if (alive && tr > k && tr < nc) {
            const double lr = B[tr][k];
            for (int c = k + 1 + tp; c <= tr; c += np) {
                const double tk = lr * (B[c][k] * dk);
                B[tr][c] -= tk;
                if (tr == c) dsc[c] += fabs(tk);
            }
        }
        __syncthreads();
    }
    // L11(r, c) -> upper slot (c, r): thread tr writes row c = tr of the slot image
    for (int r = tp; r < nc; r += np)
        if (tr < r) panel[tr + (size_t)r * ld] = B[r][tr];
    for (int k = tid; k < nc; k += nthr) { p.dg[c0 + k] = dv[k]; p.live[c0 + k] = lv[k]; }
    if (tid == 0 && ndep_sh) atomicAdd(&p.flags[0], ndep_sh);
}


// ------------------------------------------------------- L21 = A21 L11^-T D^-1
// Rows [rlo, rhi) (at most 64) of a panel (ld, nc columns starting at global
// column c0), against the factored diagonal block (L11' in its upper
// triangle); 256 threads, row r = lane, columns 4q + wave in registers.
// Bl(c, k) = L11(c, k) d_k in LDS.  With wbuf != nullptr also writes
// W = L21 D (ldw, rows relative to wrow0) for the dense tail's trailing
// update.  Reference form: l = w / d, w -= l * (l11 * d).
__device__ void solve_rows(const DiagCtx p, double* panel, int ld, int nc, int c0, int rlo, int rhi,
                           double* wbuf, int ldw, int wrow0) {
    __shared__ double Bl[PC][PC + 1];     // Bl[c][k] = L11(c, k) * d_k
    __shared__ double dv[PC];
    __shared__ int lv[PC];
    __shared__ double lk[2][64];          // double-buffered: one barrier per column
    const int tid = threadIdx.x, r = tid & 63, q0 = tid >> 6;
    for (int k = tid; k < nc; k += NT) { dv[k] = p.dg[c0 + k]; lv[k] = p.live[c0 + k]; }
    __syncthreads();
    for (int idx = tid; idx < PC * PC; idx += NT) {
        const int k = idx & 63, c = idx >> 6;        // slot (k, c) holds L11(c, k)
        Bl[c][k] = (k < c && c < nc) ? panel[k + (size_t)c * ld] * dv[k] : 0.0;
    }
    const int row = rlo + r;
    const bool okr = row < rhi;
    double a[16];
#pragma unroll
    for (int q = 0; q < 16; q++) {
        const int c = 4 * q + q0;
        const bool ok = okr && c < nc;
        const double t = panel[ok ? row + (size_t)c * ld : 0];
        a[q] = ok ? t : 0.0;
    }
    __syncthreads();
#pragma unroll
    for (int qk = 0; qk < 16; qk++) {
        for (int pk = 0; pk < 4; pk++) {
            const int k = 4 * qk + pk;
            if (k >= nc) break;
            const int buf = k & 1;
            if (q0 == pk) {
                const double l = lv[k] ? a[qk] / dv[k] : 0.0;
                a[qk] = l;
                lk[buf][r] = l;
            }
            __syncthreads();
            const double l = lk[buf][r];
            double bk[16];
#pragma unroll
            for (int q = qk; q < 16; q++) bk[q] = Bl[4 * q + q0][k];
#pragma unroll
            for (int q = qk; q < 16; q++) {
                const int c = 4 * q + q0;
                a[q] = c > k ? a[q] - l * bk[q] : a[q];   // Bl = 0 beyond nc
            }
        }
    }
    if (okr) {
#pragma unroll
        for (int q = 0; q < 16; q++) {
            const int c = 4 * q + q0;
            if (c < nc) {
                panel[row + (size_t)c * ld] = a[q];
                if (wbuf) wbuf[(wrow0 + r) + (size_t)c * ldw] = a[q] * dv[c];
            }
        }
    }
}


// one kernel for both the sparse panels (level_sups != nullptr) and the
// dense tail, so the unrolled fast path is compiled once
__global__ void __launch_bounds__(NT)
k_diag(PlanView p, const int* __restrict__ level_sups, int q0, TailView tv, int kb) {
    __shared__ double Bt[PC][PC + 1];
    __shared__ int ok;
    double* panel;
    int ld, nc, h, c0;
    if (level_sups) {
        const int s = level_sups[q0 + blockIdx.x];
        c0 = p.col0[s];
        nc = p.col0[s + 1] - c0;
        h = nc + (p.rowptr[s + 1] - p.rowptr[s]);
        ld = h;
        panel = p.Lx + p.off[s];
    } else {
        const int k0 = kb * PC;
        nc = min(PC, tv.nt - k0);
        ld = tv.nt;
        h = tv.nt - k0;
        c0 = tv.tc + k0;
        panel = tv.S + k0 + (size_t)k0 * tv.nt;
    }
    const DiagCtx dc{p.dscale, p.dg, p.live, p.flags, p.sign, p.tau};
    const bool f = factor_diag_fast(dc, panel, ld, nc, c0, Bt);
    if (threadIdx.x == 0) ok = f;
    __syncthreads();
    if (!ok) factor_diag_block(p.dscale, p.dg, p.live, p.flags, p.sign, p.tau, panel, ld, nc, h, c0);
}

__global__ void __launch_bounds__(NT)
k_trsm(PlanView p, int u0, TailView tv, int kb) {
    double* panel;
    double* wbuf = nullptr;
    int ld, nc, c0, rlo, rhi, ldw = 0, wrow0 = 0;
    if (kb < 0) {
        const int u = u0 + blockIdx.x;
        const int s = p.unit_sup[u], t = p.unit_tile[u];
        c0 = p.col0[s];
        nc = p.col0[s + 1] - c0;
        ld = nc + (p.rowptr[s + 1] - p.rowptr[s]);
        rlo = max(t * TR, nc);
        rhi = min(t * TR + TR, ld);
        panel = p.Lx + p.off[s];
    } else {
        const int k0 = kb * PC;
        nc = min(PC, tv.nt - k0);
        rlo = nc + blockIdx.x * TR;            // rows relative to the block column
        rhi = min(rlo + TR, tv.nt - k0);
        ld = tv.nt;
        c0 = tv.tc + k0;
        panel = tv.S + k0 + (size_t)k0 * tv.nt;
        wbuf = tv.W;
        ldw = tv.nt;
        wrow0 = rlo;
    }
    if (rhi <= rlo) return;
    solve_rows(DiagCtx{p.dscale, p.dg, p.live, p.flags, p.sign, p.tau}, panel, ld, nc, c0, rlo, rhi, wbuf, ldw, wrow0);
}

// ----------------------------------------- dense tail, dependent pivots
// Block column kb of the dense tail when the look-ahead panel bailed on a
// pivot that fails the zero test (the repair path): diagonal block + every
// row below with the reference's rule (ldlt.c:600-614), in rounds of one
// launch each.  Workgroup g factors the diagonal block redundantly in LDS
// (factor_diag_block's operations) and keeps its own 64-row tile of the rows
// below solved column by column (solve_rows': l = a / d_k on live columns,
// a -= l (L11 d)), so at a failing pivot k every tile holds column k after
// the updates of columns < k -- the values the rule's largest off-diagonal
// magnitude is taken over.  A round runs until such a column whose decision
// is not known yet: each workgroup publishes its tile's largest magnitude
// (the diagonal block's rows included) and its rows' state in place,
// workgroup 0 the block's state, and the round ends; the next round (the
// kernel boundary orders everything) reloads the state, reduces the
// published maxima in workgroup order -- every workgroup the same values,
// the same decision: drop, or +-1e-8 by node class -- and goes on.  No grid
// barrier, no co-residency assumption: one launch per dependent pivot.
// State: st = B (PC x PC) | dv | lv | dsc | gmax[G]; sti = k0, 1 + pending
// column (0: none), done, ndep.  Two copies of each, selected by the round's
// parity: round r reads copy r & 1 and writes copy (r + 1) & 1, so nothing a
// launch reads is written in that launch (workgroups of one grid are not
// ordered: a workgroup starting after workgroup 0 ended must still see the
// round's input state, and the maxima of the pending column must not be
// overwritten by those of the next failing column while a slower workgroup
// still reduces them).
constexpr int kDepState = PC * PC + 3 * PC;

__global__ void __launch_bounds__(NT)
k_tail_dep(PlanView p, TailView tv, int kb, const double* __restrict__ st_in, double* __restrict__ st_out,
           const int* __restrict__ sti_in, int* __restrict__ sti_out) {
    __shared__ double B[PC][PC + 1];
    __shared__ double dv[PC];
    __shared__ int lv[PC];
    __shared__ double dsc[PC];
    __shared__ double red[4];
    __shared__ double lk[PC];
    __shared__ int ndep_sh;
    const int k0b = kb * PC, nt = tv.nt, ld = nt;
    const int nc = min(PC, nt - k0b), h = nt - k0b, c0 = tv.tc + k0b;
    double* panel = tv.S + k0b + (size_t)k0b * nt;
    const int G = gridDim.x, g = blockIdx.x;
    const int tid = threadIdx.x, tr = tid & 63, tp = tid >> 6, np = NT >> 6;
    const int row = nc + g * TR + tr;
    const bool rok = row < h;
    if (sti_in[2]) {              // the block column is done: a round enqueued past the end is a no-op
        if (g == 0 && tid == 0) sti_out[2] = 1;
        return;
    }
    const int kstart = sti_in[0], pending = sti_in[1] - 1;
    const double* gmax_in = st_in + kDepState;
    double* gmax_out = st_out + kDepState;
    const double* st = st_in;
    if (kstart == 0) {
        for (int c = tp; c < nc; c += np) B[tr][c] = (tr < nc && tr >= c) ? panel[tr + (size_t)c * ld] : 0.0;
        for (int k = tid; k < nc; k += NT) { dsc[k] = p.dscale[c0 + k]; dv[k] = 0.0; lv[k] = 1; }
    } else {
        for (int c = tp; c < nc; c += np) B[tr][c] = st[tr * PC + c];
        for (int k = tid; k < nc; k += NT) {
            dv[k] = st[PC * PC + k];
            lv[k] = static_cast<int>(st[PC * PC + PC + k]);
            dsc[k] = st[PC * PC + 2 * PC + k];
        }
    }
    double a[16];
#pragma unroll
    for (int q = 0; q < 16; q++) {
        const int c = 4 * q + tp;
        const bool ok = rok && c < nc;
        const double t = panel[ok ? row + (size_t)c * ld : 0];
        a[q] = ok ? t : 0.0;
    }
    if (tid == 0) ndep_sh = kstart == 0 ? 0 : sti_in[3];
    __syncthreads();
#pragma unroll
    for (int qk = 0; qk < 16; qk++) {
        for (int pk = 0; pk < 4; pk++) {
            const int k = 4 * qk + pk;
            if (k >= nc) break;
            if (k < kstart) continue;
            double dk = B[k][k];
            int alive = 1;
            if (fabs(dk) <= p.tau * dsc[k]) {           // wave-uniform (LDS values)
                if (pending != k) {
                    // publish this tile's largest magnitude of column k and the
                    // state, end the round
                    double mx = 0.0;
                    for (int r = k + 1 + tid; r < nc; r += NT) mx = ref_max(mx, ref_abs(B[r][k]));
                    if (tp == pk && rok) mx = ref_max(mx, ref_abs(a[qk]));
                    mx = wave_max(mx);
                    if (tr == 0) red[tp] = mx;
                    __syncthreads();
                    if (tid == 0) {
                        double m2 = red[0];
                        for (int q = 1; q < np; q++) m2 = ref_max(m2, red[q]);
                        gmax_out[g] = m2;
                    }
                    if (rok) {
#pragma unroll
                        for (int q = 0; q < 16; q++) {
                            const int c = 4 * q + tp;
                            if (c < nc) panel[row + (size_t)c * ld] = a[q];
                        }
                    }
                    if (g == 0) {
                        for (int c = tp; c < nc; c += np) st_out[tr * PC + c] = B[tr][c];
                        for (int kk = tid; kk < nc; kk += NT) {
                            st_out[PC * PC + kk] = dv[kk];
                            st_out[PC * PC + PC + kk] = lv[kk];
                            st_out[PC * PC + 2 * PC + kk] = dsc[kk];
                        }
                        if (tid == 0) { sti_out[0] = k; sti_out[1] = k + 1; sti_out[2] = 0; sti_out[3] = ndep_sh; }
                    }
                    return;
                }
                double mx = gmax_in[0];
                for (int q = 1; q < G; q++) mx = ref_max(mx, gmax_in[q]);
                if (mx < 1.0e+6 * 1.0e-8) alive = 0;
                else dk = (p.sign[c0 + k] < 0 ? -1.0 : 1.0) * 1.0e-8;
                if (tid == 0) ndep_sh++;
            }
            if (tid == 0) { dv[k] = dk; lv[k] = alive; }
            for (int r = k + 1 + tid; r < nc; r += NT) B[r][k] = alive ? B[r][k] / dk : 0.0;
            if (tp == pk) {
                const double l = alive ? a[qk] / dk : 0.0;
                a[qk] = l;
                lk[tr] = l;
            }
            __syncthreads();
            if (alive && tr > k && tr < nc) {
                const double lr = B[tr][k];
                for (int c = k + 1 + tp; c <= tr; c += np) {
                    const double tk = lr * (B[c][k] * dk);
                    B[tr][c] -= tk;
                    if (tr == c) dsc[c] += fabs(tk);
                }
            }
            {
                const double l = lk[tr];
#pragma unroll
                for (int q = 0; q < 16; q++) {
                    const int c = 4 * q + tp;
                    const double bk = (k < c && c < nc) ? B[c][k] * dk : 0.0;
                    a[q] = c > k ? a[q] - l * bk : a[q];
                }
            }
            __syncthreads();
        }
    }
    if (rok) {
#pragma unroll
        for (int q = 0; q < 16; q++) {
            const int c = 4 * q + tp;
            if (c < nc) panel[row + (size_t)c * ld] = a[q];
        }
    }
    if (g != 0) return;
    for (int r = tp; r < nc; r += np)
        if (tr < r) panel[tr + (size_t)r * ld] = B[r][tr];
    for (int k = tid; k < nc; k += NT) { p.dg[c0 + k] = dv[k]; p.live[c0 + k] = lv[k]; }
    if (tid == 0) {
        if (ndep_sh) atomicAdd(&p.flags[0], ndep_sh);
        sti_out[2] = 1;
    }
}

// ------------------------------------------------------------ fused panel
// Diagonal block and the rows below it in one launch: the fast path of
// k_diag + k_trsm (k_panel_w below).  A pivot that fails the zero test stops
// every workgroup of the panel before it writes anything and raises
// flags[1]: the host then redoes the factorisation with k_diag / k_trsm,
// which own the dependent-pivot rule (ldlt.c:600-614).  (Round 1's 8-wave
// one-barrier-per-column k_panel, bitwise the same, measured slower and is
// gone.)
constexpr int PNT = 512;

// ------------------------------------------------------- windowed panel
// Fused diagonal block + panel rows, the column chain cut into four
// 16-column windows (one workgroup barrier per window).  Wave
// w of half 0 (waves 0-3) keeps window w (columns 16w..16w+15) of the
// block's 64 rows, wave w of half 1 (waves 4-7) window w of tile j + 1.
// Phase t (one workgroup barrier each):
//   half 0: every wave w >= t applies the 16 rank-1 updates of window t-1
//           to its columns (in k order), then wave t factors window t
//           right-looking on its own, every cross-lane value (pivot, its
//           |terms|, the window's c_j) by v_readlane -- no LDS round trip
//           and no workgroup barrier inside a window;
//   half 1: one phase behind: waves w >= t-1 apply the updates of tile
//           window t-2, then wave t-1 solves window t-1 of the tile rows
//           (l = b(k) / d_k, b(j) -= l Ct[k][j]).
// What crosses waves lives in LDS: Ct[k][r] = l(r, k) d_k (a row of
// L11 D: the update operand of both halves), Lr[k][r] / Lb[k][r] = l(r, k)
// of the block rows / tile rows.  Every entry sees the updates k = 0, 1,
// ... in order with the operations of factor_diag_fast / solve_rows (l =
// a / d, a -= l (l_j d_k), |terms| of each pivot in dscale order), so the
// factor is bitwise that of k_panel and of k_diag + k_trsm.  A pivot that
// fails the zero test raises a flag the whole workgroup reads after the
// phase's barrier; the panel then stops unwritten (flags[1]), as k_panel.
constexpr int WIN = 16;
constexpr int CTS = PC + 2;           // Ct row stride: 16-B aligned rows for ds_read_b128

// in-kernel clock stamps for tools/ubench_panel.hip (compiled out otherwise)
#ifdef IPO_PANEL_STAMPS
__device__ long long g_stamps[8][16];
#define PANEL_STAMP(slot)                                                                         \
    do {                                                                                          \
        if (blockIdx.x == 0 && (threadIdx.x & 63) == 0) g_stamps[threadIdx.x >> 6][slot] = clock64(); \
    } while (0)
#else
#define PANEL_STAMP(slot) do {} while (0)
#endif

__device__ __forceinline__ void win_row(const double* __restrict__ row, double (&c)[WIN]) {
#pragma unroll
    for (int q = 0; q < WIN; q += 2) {
        const double2 v = *reinterpret_cast<const double2*>(row + q);
        c[q] = v.x;
        c[q + 1] = v.y;
    }
}

// The window routines come in a FULL form (all 16 columns inside the
// block: no per-column guard, so a window is one basic block the compiler
// can schedule across -- the next step's pivot chain in the shadow of the
// previous step's updates) and a guarded form for the last, partial window.
// Progress counters of the windows (LDS): a wave publishes how many columns
// of its window it has written (Ct / Lr / Lb / dv), the waves that apply or
// solve against that window wait for the column they need -- a dataflow
// between the waves instead of one workgroup barrier per window.  One wave's
// LDS operations execute in issue order, so data stored before a count is
// visible to a wave that has read the count; the wavefront fences only keep
// the compiler from moving LDS accesses across the count.
__device__ __forceinline__ void df_publish(int* prog, int v) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __hip_atomic_store(prog, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

__device__ __forceinline__ void df_wait(const int* prog, int v, int& seen) {
    if (seen < v) {
        int x;
        while ((x = __builtin_amdgcn_readfirstlane(__hip_atomic_load(prog, __ATOMIC_RELAXED,
                                                                     __HIP_MEMORY_SCOPE_WORKGROUP))) < v)
            __builtin_amdgcn_s_sleep(1);
        seen = x;
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Window factorisation (half 0, wave w): every cross-lane value by
// v_readlane; column i of the window is published after its pivot step.
// Software-pipelined: step i forms pivot i + 1 (its column updated first,
// by v_readlane) before the rest of its updates, so the division of the next
// pivot issues interleaved with them instead of after them.
// DEP (the dense tail's second pass after a pivot failed the zero test, see
// panel_w_body): such a pivot takes the dependent-pivot rule of ldlt.c:600-614
// in the chain -- +-1e-8 by node class when some entry of the column below it
// reaches 1e-2, else the column is dropped (l = 0, d kept, live 0).  The
// block's own rows decide "keep" for certain; "drop" also needs the rows
// below the block, which other workgroups hold: each workgroup checks its
// tile against the decision (win_solve) and the panel bails if one fails.
struct DepState {
    const int* sign;       // node class of the block's columns (c0-relative)
    int* lv;               // LDS: per column 1 live, 0 dropped, 2 kept with +-1e-8 (dependent), published with dv
    int* spec;             // LDS: the speculation failed (or met a NaN)
    int ndep;              // dependent pivots of this wave's window
    int specv = 1;         // what a failure stores in *spec (k_tail_chain_run: its pass, so no reset is needed)
};

__device__ __forceinline__ void dep_pivot(double col, int k, int lane, int h0, double& dk, int& alive, DepState& ds) {
    const bool in = lane > k && lane < h0;
    const bool big = __ballot(in && !(fabs(col) < 1.0e+6 * 1.0e-8)) != 0;   // includes NaN
    const bool nan = __ballot(in && col != col) != 0;
    if (nan && lane == 0) *ds.spec = ds.specv;   // the host repair decides it (the reference's NaN-order max)
    if (big) dk = (ds.sign[k] < 0 ? -1.0 : 1.0) * 1.0e-8;   // y-nodes -, x-nodes +
    else alive = 0;                                        // dropped, d keeps its value
    ds.ndep++;
}

// pb (all window routines): the progress counters' base -- a window's
// column i is published as pb + i + 1, so a workgroup that runs several
// passes (k_tail_chain_run) needs no reset barrier between them.
template <bool FULL, bool DEP>
__device__ __forceinline__ void win_factor(double (&a)[WIN], double& dsc, bool& tz_any, int cw0, int nc, int lane,
                                           int h0, double tau, double (*Ct)[CTS], double (*Lr)[PC], double* dv,
                                           int* prog, DepState& ds, int pb = 0) {
    double dk = lane_bcast(a[0], cw0);
    int alive = 1, mark = 1;
    if (DEP) {
        if (fabs(dk) <= tau * lane_bcast(dsc, cw0)) {
            dep_pivot(a[0], cw0, lane, h0, dk, alive, ds);
            mark = alive ? 2 : 0;
        }
    } else {
        tz_any |= fabs(dk) <= tau * lane_bcast(dsc, cw0);   // no short-circuit: no branch
    }
    double l = alive && lane > cw0 && lane < h0 ? a[0] / dk : 0.0;
#pragma unroll
    for (int i = 0; i < WIN; i++) {
        const int k = cw0 + i;
        if (FULL || k < nc) {
            const bool below = lane > k && lane < h0;
            a[i] = below ? l : a[i];
            const double c = l * dk;
            Ct[k][lane] = c;
            Lr[k][lane] = l;
            dv[k] = dk;                   // every lane stores the same value: no EXEC branch
            if (DEP) ds.lv[k] = mark;
            // the wavefront fence orders the reads of the row just written
            // (and the published count) after the writes for the compiler;
            // the LDS runs one wave's operations in issue order
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
            __hip_atomic_store(prog, pb + i + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            if (i == WIN - 1) PANEL_STAMP(5);
            dsc = dsc + fabs(l * c);
            double cc[WIN];
            if (i + 2 < WIN) win_row(&Ct[k][cw0], cc);
            const double lk = l;
            if (i + 1 < WIN && (FULL || k + 1 < nc)) {
                // pivot k + 1: its column by v_readlane, then l of the next step
                a[i + 1] = a[i + 1] - lk * lane_bcast(c, k + 1);
                dk = lane_bcast(a[i + 1], k + 1);
                if (DEP) {
                    alive = 1;
                    mark = 1;
                    if (fabs(dk) <= tau * lane_bcast(dsc, k + 1)) {
                        dep_pivot(a[i + 1], k + 1, lane, h0, dk, alive, ds);
                        mark = alive ? 2 : 0;
                    }
                } else {
                    tz_any |= fabs(dk) <= tau * lane_bcast(dsc, k + 1);
                }
                l = alive && lane > k + 1 && lane < h0 ? a[i + 1] / dk : 0.0;
            }
#pragma unroll
            for (int q = i + 2; q < WIN; q++) a[q] = a[q] - lk * cc[q];
        }
    }
}

// Rank-1 updates k = kw .. kw + 15 of an earlier (always full) window, in k
// order, on this wave's 16 columns (L = Lr for block rows, Lb for tile rows;
// DSC: also the |terms| of the diagonal entries this wave owns), each as soon
// as the window's owner has published column k.  (The 16 column multipliers
// come as one broadcast LDS row: by v_readlane from the lanes holding them
// the updates ran at half the speed.)
template <bool DSC>
__device__ __forceinline__ void win_apply(double (&a)[WIN], double& dsc, int kw, int lane, int cw0,
                                          double (*Ct)[CTS], double (*L)[PC], const int* prog, int pb = 0) {
    // software-pipelined: step i + 1's LDS operands are read before step i's
    // arithmetic, so the read latency hides under the updates
    int seen = 0;
    double l, ck = 0.0, cc[WIN];
    df_wait(prog, pb + 1, seen);
    l = L[kw][lane];
    if (DSC) ck = Ct[kw][lane];
    win_row(&Ct[kw][cw0], cc);
#pragma unroll 2
    for (int i = 0; i < WIN; i++) {
        const int k = kw + i;
        double ln = 0.0, ckn = 0.0, cn[WIN];
        if (i + 1 < WIN) {
            df_wait(prog, pb + i + 2, seen);
            if (i + 2 == WIN) PANEL_STAMP(6);
            ln = L[k + 1][lane];
            if (DSC) ckn = Ct[k + 1][lane];
            win_row(&Ct[k + 1][cw0], cn);
        }
#pragma unroll
        for (int q = 0; q < WIN; q++) a[q] = a[q] - l * cc[q];
        if (DSC) dsc = dsc + fabs(l * ck);
        l = ln;
        ck = ckn;
#pragma unroll
        for (int q = 0; q < WIN; q++) cc[q] = cn[q];
    }
    PANEL_STAMP(7);
}

// Window solve of the tile rows (half 1, wave w): solve_rows' form, step i
// once half 0 has published pivot i of the window (wprog); publishes Lb.
// DEP: a dropped column (lv 0) gives l = 0, and this tile's entries of it
// must stay below 1e-2 (the speculation of dep_pivot), else the panel bails;
// below a dependent pivot kept from the block's rows (lv 2) a NaN in the tile
// bails too (the reference's max fold over the whole column is order-
// dependent with a NaN in it: the host repair decides it).
template <bool FULL, bool DEP>
__device__ __forceinline__ void win_solve(double (&a)[WIN], int cw0, int nc, bool rok, int lane, double (*Ct)[CTS],
                                          double (*Lb)[PC], const double* dv, const int* wprog, int* prog,
                                          DepState& ds, int pb = 0) {
    int seen = 0;
#pragma unroll
    for (int i = 0; i < WIN; i++) {
        const int k = cw0 + i;
        if (FULL || k < nc) {
            df_wait(wprog, pb + i + 1, seen);
            double l;
            if (DEP && !ds.lv[k]) {
                if (__ballot(rok && !(fabs(a[i]) < 1.0e+6 * 1.0e-8)) != 0 && lane == 0) *ds.spec = ds.specv;
                l = 0.0;
            } else {
                if (DEP && ds.lv[k] == 2 && __ballot(rok && a[i] != a[i]) != 0 && lane == 0) *ds.spec = ds.specv;
                l = rok ? a[i] / dv[k] : 0.0;
            }
            a[i] = l;
            Lb[k][lane] = l;
            df_publish(prog, pb + i + 1);
            double cc[WIN];
            win_row(&Ct[k][cw0], cc);
#pragma unroll
            for (int q = i + 1; q < WIN; q++) a[q] = a[q] - l * cc[q];
        }
    }
}

typedef double double4_t __attribute__((ext_vector_type(4)));

// Dense-tail panels of the look-ahead factorisation first apply block
// column t - 1's update to their own rows (the diagonal block and tile j +
// 1), the way k_tail_syrk would: operands staged here, products (old - acc
// is formed by the panel on its loaded values) left in Ad / Aj as [row][col].
// Row stride 66: the MFMA operand reads (16 rows x 4 k per wave) hit at
// most two lanes per bank, a 16-lane column of one k none.
constexpr int PRS = PC + 2;
struct PreLds {
    double Ad[TR][PRS];
    double Aj[TR][PRS];
    double Bs[TR][PRS];
};

// LDS image of the windowed panel (one raw buffer, so a kernel can share it
// with the trailing-update tiles below)
struct PanelLds {
    double Ct[PC][CTS];
    double Lr[PC][PC];
    double Lb[PC][PC];
    double dv[PC];
    int lv[PC];                           // DEP pass: live mark per column
    int prog[8];                          // published columns: windows of half 0, then of half 1
    int tiny;
    int spec;                             // DEP pass: a tile (or a NaN) contradicts a dropped column
    int ndep;                             // DEP pass: dependent pivots of the block
    int wverd[4];                         // half 0's window w factored: 1 every pivot passed the zero test, 2 not
};

// Workgroup `bid` of a windowed panel: fused unit f0 + bid of a sparse level
// (fu_sup != nullptr) or block column kb of the dense tail, whose W = L21 D
// goes to wtail.
// Dependent pivots in the dense tail (dep != 0, k_tail_pr): the first pass
// (DEP false) ends unwritten as soon as the diagonal block has a pivot that
// fails the zero test -- every workgroup of the panel sees it, the block is
// factored identically in each -- and returns true; the caller reruns the
// panel with DEP true, which applies ldlt.c:600-614 in the chain (dep_pivot):
// a column "kept" with +-1e-8 is certain from the block's rows alone; a
// dropped one is checked by every workgroup on its own tile (win_solve).  A
// workgroup whose tile contradicts a drop (or meets a NaN) bails as the first
// pass would have (flags[1] bit 4 | 16, flags[2]), and the host resumes the
// look-ahead from this block column (KktDevice::repair_tail) after putting
// back what the other workgroups wrote: the DEP pass saves its tile rows and
// workgroup 0 the block's |terms| into tv.W (unused by the look-ahead) before
// anything is written, and workgroup 0 leaves the dependent pivots it added
// to flags[0] in flags[3] (k_tail_restore).  Where the speculation holds (122
// of the 124 dependent pivots of the oracle's dfl001_100/110/114 factors that
// fall in the GPU's dense tail), the block costs one more panel pass instead
// of the host round trips and relaunches of a repair; the factor is bitwise
// the repair path's (tests/test_gpu_panel.py).  dep == 2 (IPO_HIP_TAIL_SPEC=2,
// tests only) treats every drop as contradicted, which exercises the restore.
// SC (k_tail_run, the persistent dense tail): every access to what other
// workgroups of the launch write or read (S, dg, dscale, the DEP saves) is
// an sc1 access (kkt_kernels.h), and pre_wait() -- called once this
// workgroup's own entries are loading, before block t - 1's operands are --
// waits for the panels of step t - 1 (false: skip the item, the tail bailed).
struct NoWait {
    __device__ bool operator()() const { return true; }
};
// post(bailed): called by every thread once the handed-off results are
// stored (the tile rows and, workgroup 0, D) -- k_tail_run signals step t
// there, before workgroup 0's L11' / mark / |terms| stores, which only later
// launches read -- or with true when the panel bails
struct NoPost {
    __device__ void operator()(bool) const {}
};
// A panel workgroup that bails adds 1 + kRunBail to pdone[t]: a waiter on
// the panels of step t learns both in one load.
constexpr int kRunBail = 1 << 16;

// one lane polls until pdone counter c0 (null: none) reaches v0 and vseq
// counter c1 (null: none) reaches v1; the workgroup joins a barrier and gets
// false for "skip the item": step t - 1 bailed (c0's bail bit), or, while a
// counter is short, a panel of a launch before t has bailed (flags[2]: then
// the counter may never complete)
__device__ __forceinline__ bool run_wait(const int* c0, int v0, const int* c1, int v1, const int* bailp, int t,
                                         int* sh) {
    if (threadIdx.x == 0) {
        int ok = 1;
        for (;;) {
            const int x0 = c0 ? sc1_load_int(c0) : v0;
            const int x1 = c1 ? sc1_load_int(c1) : v1;
            if ((x0 & (kRunBail - 1)) >= v0 && x1 >= v1) {
                ok = x0 < kRunBail;
                break;
            }
            const int b = sc1_load_int(bailp);
            if (b && b - 1 < t) {
                ok = 0;
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
        *sh = ok;
    }
    __syncthreads();
    return *sh != 0;
}

// Window hand-off of the persistent tail (k_tail_run; pub null: off).  A
// tile window of step t is final once it is solved and the diagonal windows
// up to it passed the zero test (a first pass that meets a dependent pivot
// in window v reruns with DEP, which computes windows before v again with the
// same operations): half 1's wave publishes it at once -- its 64 rows of L
// and the window's 16 pivots, sc1 stores, vmcnt(0), then the flag
// (t, j, w) = epoch -- and the panels of step t + 1 form their pre-update
// window by window from those of tiles 0 (their diagonal rows) and j + 1
// (their tile rows): the MFMA k-steps in the same order, so the same
// products, bitwise the pre-update that reads S once step t is done.  They
// wait for the whole step t (pdone: every panel done, none bailed) only after
// their own window chains, before their first global write.  The first step
// of a run (t0: after a repair, S holds step t0 - 1) reads S.
__device__ __forceinline__ void run_signal(int* cnt, int v = 1) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_fetch_add(cnt, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// The buffer of step t's windows (t & 1) takes step t + 2's next: a panel
// of step t counts itself in pread[t] once it has read step t - 1's
// windows, and step t + 1's half-1 waves wait for that count before they
// publish into it (a DEP pass reads S, not the buffer).
// Such a panel also waits for the visits of its own tiles (vd, vt: vseq
// counters, q chunks each) only after that pre-update's products, right
// before it loads its own entries: the visits of its column end late in the
// previous step and gate nothing else.
struct RunPub {
    double* pub = nullptr;     // TailRun::pub
    const int* wflag = nullptr;
    int* wflag_w = nullptr;
    int* pread = nullptr;      // TailRun::pread
    int t0 = 0;
    int epoch = 0;
    const int* vd = nullptr;   // the vseq counters of the panel's diagonal tile and tile (null: none)
    const int* vt = nullptr;
    int q = 0;
    int* sh = nullptr;         // run_wait's LDS word
};

template <bool DEP = false, bool SC = false, class PreWait = NoWait, class Post = NoPost>
__device__ __forceinline__ bool panel_w_body(const PlanView& p, const int* __restrict__ fu_sup,
                                             const int* __restrict__ fu_j, int f0, const TailView& tv, int kb, int bid,
                                             PanelLds& S, double* wtail, bool pre = false,
                                             const int* bailp = nullptr, int bt = 0, int dep = 0,
                                             PreWait pre_wait = PreWait{}, Post post = Post{},
                                             RunPub rp = RunPub{}) {
    // a bail flag of an earlier step (dense tail, see k_tail_pr): read first,
    // tested once this workgroup's operand loads are in flight
    const int bailed = bailp ? *bailp : 0;
    double (*Ct)[CTS] = S.Ct;
    double (*Lr)[PC] = S.Lr;
    double (*Lb)[PC] = S.Lb;
    double* dv = S.dv;
    int& tiny_sh = S.tiny;
    double* panel;
    double* wbuf = nullptr;
    int ld, nc, h, c0, j;
    if (fu_sup) {
        const int s = fu_sup[f0 + bid];
        j = fu_j[f0 + bid];
        c0 = p.col0[s];
        nc = p.col0[s + 1] - c0;
        h = nc + (p.rowptr[s + 1] - p.rowptr[s]);
        ld = h;
        panel = p.Lx + p.off[s];
    } else {
        const int k0 = kb * PC;
        j = bid;
        nc = min(PC, tv.nt - k0);
        h = tv.nt - k0;
        ld = tv.nt;
        c0 = tv.tc + k0;
        panel = tv.S + k0 + (size_t)k0 * tv.nt;
        wbuf = wtail;
    }
    const int tid = threadIdx.x, lane = tid & 63, wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    PANEL_STAMP(15);
    const bool h1 = wv >= 4;
    // half 1 takes the windows in the order 2 3 0 1, so the waves sharing a
    // SIMD (wv, wv + 4) never both own the last window's long chain
    const int w = h1 ? (wv + 2) & 3 : wv, cw0 = WIN * w;
    const int h0 = min(PC, h);
    const int row = h1 ? TR * (j + 1) + lane : lane;
    const bool rok = h1 ? row < h : row < h0;
    const bool tile = TR * (j + 1) < h;             // workgroup has tile rows
    const int nwin = (nc + WIN - 1) / WIN;
    double a[WIN];
    // |terms| of the pivots of this wave's window (half 0; lane r <-> (r, r))
    double dsc = 0.0;
    auto load_own = [&]() {
#pragma unroll
        for (int q = 0; q < WIN; q++) {
            const int c = cw0 + q;
            const bool ok = rok && c < nc && (h1 || c <= row);
            const double t = ld_h<SC>(panel + (ok ? row + (size_t)c * ld : 0));
            a[q] = ok ? t : 0.0;
        }
        dsc = (!h1 && lane < nc && (lane >> 4) == w) ? ld_h<SC>(p.dscale + c0 + lane) : 0.0;
    };
    auto dep_save = [&]() {
        if (DEP && !fu_sup) {
            // what this pass may overwrite, saved for k_tail_restore: the tile
            // rows (rows >= 64 of the block column, as in S) and workgroup 0's
            // |terms| of the block's pivots (rows 0..nc-1 of W's column 0)
            if (h1 && rok && tile) {
#pragma unroll
                for (int q = 0; q < WIN; q++) {
                    const int c = cw0 + q;
                    if (c < nc) st_h<SC>(tv.W + row + (size_t)c * tv.nt, a[q]);
                }
            }
            if (j == 0 && !h1 && lane < nc && (lane >> 4) == w) st_h<SC>(tv.W + lane, dsc);
        }
    };
    // the pre-update from the previous step's published windows (RunPub):
    // the own entries are loaded after its products
    // (not in a DEP pass: step kb - 1 is complete by then and S holds it --
    // the same values; its buffer may already take step kb + 1's windows)
    const bool winpub = !DEP && SC && rp.pub && pre && kb - 1 >= rp.t0;
    if (!winpub) load_own();
    double dsc_pre = 0.0;                  // pivot |terms| after the pre-update (stored once the panel holds)
    if (!pre && bailed && bailed - 1 < bt) return false;
    if (!winpub) dep_save();
    if (pre) {
        if (!winpub && !pre_wait()) return false;     // workgroup-uniform
        // dense tail, block column kb > 0: block kb - 1's update of this
        // workgroup's rows, k_tail_syrk's MFMA fragments and order; the
        // entries get old - acc and the pivots' |terms| old + sum_k |l w|,
        // the operations of k_tail_syrk's tile, without a launch of its own
        PreLds& P = *reinterpret_cast<PreLds*>(&S);
        const int nt = tv.nt, kp = (kb - 1) * PC;
        const double* Lcol = tv.S + (size_t)kp * nt;
        constexpr int NU = TR * PC / PNT;
        // |terms| of the pivots (half 0, the wave's 16 diagonal rows), k in
        // order, interleaved with the MFMA steps that read the same k
        const bool holder = !h1 && lane < nc && (lane >> 4) == w;
        double asum = 0.0;
        const int wr = (w & 1) * 32, wc = (w >> 1) * 32, li = lane & 15, lk = lane >> 4;
        double (*Am)[PRS] = h1 ? P.Aj : P.Ad;
        double4_t acc[2][2];
#pragma unroll
        for (int x = 0; x < 2; x++)
#pragma unroll
            for (int y = 0; y < 2; y++) acc[x][y] = (double4_t){0.0, 0.0, 0.0, 0.0};
        auto mfma_k = [&](int kk) {
            double av[2], bv[2];
#pragma unroll
            for (int x = 0; x < 2; x++) av[x] = Am[wr + x * 16 + li][kk + lk];
#pragma unroll
            for (int y = 0; y < 2; y++) bv[y] = P.Bs[wc + y * 16 + li][kk + lk];
#pragma unroll
            for (int x = 0; x < 2; x++)
#pragma unroll
                for (int y = 0; y < 2; y++)
                    acc[x][y] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[x], bv[y], acc[x][y], 0, 0, 0);
            if (holder) {
#pragma unroll
                for (int u = 0; u < 4; u++) asum += fabs(P.Ad[lane][kk + u] * P.Bs[lane][kk + u]);
            }
        };
        if (winpub) {
            // window by window as step kb - 1 publishes them: its tile 0 holds
            // this panel's diagonal rows (and the pivots), tile j + 1 its tile rows
            __shared__ int pub_ok;
            const int tp = kb - 1, ntb = tv.ntb;
            const bool hasj = (kb + j + 1) * TR < nt;
            const double* p0 = rp.pub + (size_t)(tp & 1) * ntb * 4 * kTailPubWin;
            const double* pj = p0 + (size_t)(j + 1) * 4 * kTailPubWin;
            const int* f0 = rp.wflag + (size_t)tp * ntb * 4;
            const int* fj = f0 + (j + 1) * 4;
            const int rr = tid % TR, rd = kb * TR + rr, rj = (kb + j + 1) * TR + rr;
            const bool okd = rd < nt, okj = rj < nt;
            for (int v = 0; v < 4; v++) {
                if (tid == 0) {
                    int ok = 1;
                    for (;;) {
                        if (sc1_load_int(f0 + v) == rp.epoch && (!hasj || sc1_load_int(fj + v) == rp.epoch)) break;
                        const int b = sc1_load_int(p.flags + 2);
                        if (b && b - 1 < bt) {     // an earlier step bailed: its windows may never come
                            ok = 0;
                            break;
                        }
                        __builtin_amdgcn_s_sleep(1);
                    }
                    pub_ok = ok;
                }
                __syncthreads();
                if (!pub_ok) return false;
                const double* q0 = p0 + v * kTailPubWin;
                const double* qj = pj + v * kTailPubWin;
                constexpr int NW = TR * WIN / PNT;
                double vd[NW], vj[NW], vw[NW];
#pragma unroll
                for (int u = 0; u < NW; u++) {
                    const int kl = (tid + u * PNT) / TR;
                    const double x = sc1_load(q0 + (okd ? kl * TR + rr : 0));
                    const double y = sc1_load(qj + (okj ? kl * TR + rr : 0));
                    const double dk = sc1_load(q0 + WIN * TR + kl);
                    vd[u] = okd ? x : 0.0;
                    vj[u] = okj ? y : 0.0;
                    vw[u] = okd ? x * dk : 0.0;
                }
#pragma unroll
                for (int u = 0; u < NW; u++) {
                    const int k = WIN * v + (tid + u * PNT) / TR;
                    P.Ad[rr][k] = vd[u];
                    P.Aj[rr][k] = vj[u];
                    P.Bs[rr][k] = vw[u];
                }
                __syncthreads();
#pragma unroll
                for (int kk = WIN * v; kk < WIN * (v + 1); kk += 4) mfma_k(kk);
            }
            run_signal(rp.pread + kb);     // step kb - 1's windows read (their loads complete)
            PANEL_STAMP(3);
            // the visits of this panel's tiles, then its own entries (and a
            // DEP pass's saves of them)
            if (!run_wait(rp.vd, rp.q, rp.vt, rp.q, p.flags + 2, bt, rp.sh)) return false;
            load_own();
            dep_save();
        } else {
            // all 3 NU loads in flight, then into LDS
            double vd[NU], vj[NU], vw[NU];
            const int rr = tid % TR, rd = kb * TR + rr, rj = (kb + j + 1) * TR + rr;
            const bool okd = rd < nt, okj = rj < nt;
#pragma unroll
            for (int u = 0; u < NU; u++) {
                const int k = (tid + u * PNT) / TR;
                const double x = ld_h<SC>(Lcol + (okd ? rd + (size_t)k * nt : 0));
                const double y = ld_h<SC>(Lcol + (okj ? rj + (size_t)k * nt : 0));
                // W = L21 D of block t - 1 formed here, the product its panel
                // would have stored (l * d, the same operands: bitwise)
                const double dk = ld_h<SC>(p.dg + tv.tc + kp + k);
                vd[u] = okd ? x : 0.0;
                vj[u] = okj ? y : 0.0;
                vw[u] = okd ? x * dk : 0.0;
            }
            if (bailed && bailed - 1 < bt) return false;     // workgroup-uniform
#pragma unroll
            for (int u = 0; u < NU; u++) {
                const int k = (tid + u * PNT) / TR;
                P.Ad[rr][k] = vd[u];
                P.Aj[rr][k] = vj[u];
                P.Bs[rr][k] = vw[u];
            }
            __syncthreads();
            PANEL_STAMP(3);
#pragma unroll
            for (int kk = 0; kk < PC; kk += 4) mfma_k(kk);
        }
        PANEL_STAMP(4);
        __syncthreads();                   // every operand read: Ad / Aj take the products, [col][row]
#pragma unroll
        for (int x = 0; x < 2; x++)
#pragma unroll
            for (int y = 0; y < 2; y++)
#pragma unroll
                for (int i = 0; i < 4; i++)
                    Am[wc + y * 16 + (lane & 15)][wr + x * 16 + (lane >> 4) + 4 * i] = acc[x][y][i];
        __syncthreads();
#pragma unroll
        for (int q = 0; q < WIN; q++) {
            const int c = cw0 + q;
            if (rok && c < nc && (h1 || c <= row)) a[q] = a[q] - Am[c][lane];
        }
        dsc = dsc + asum;
        dsc_pre = dsc;
        __syncthreads();                   // the panel's LDS image overwrites P from here
        PANEL_STAMP(14);
    }
    if (tid < 8) S.prog[tid] = 0;
    if (tid < 4) S.wverd[tid] = 0;
    if (tid == 0) { tiny_sh = 0; S.spec = dep == 2 ? -1 : 0; S.ndep = 0; }
    __syncthreads();
    DepState ds{p.sign + c0, S.lv, &S.spec, 0};
    PANEL_STAMP(0);
    // half 0, wave w: updates of windows 0 .. w - 1, then factor window w;
    // half 1, wave w: the same updates on the tile rows, then solve window w.
    // Issue priority: the window chains (factor, solve) and the updates that
    // gate them over the rest.
    if (w < nwin && (!h1 || tile)) {
        int* const prog = S.prog + (h1 ? 4 : 0);
        double unused = 0.0;
        for (int t = 0; t < w; t++) {
            // the updates of window w - 1 gate this wave's own chain
            if (t + 1 < w) {
                if (h1) __builtin_amdgcn_s_setprio(0);
                else __builtin_amdgcn_s_setprio(1);
            } else {
                if (h1) __builtin_amdgcn_s_setprio(2);
                else __builtin_amdgcn_s_setprio(3);
            }
            if (!h1) win_apply<true>(a, dsc, WIN * t, lane, cw0, Ct, Lr, prog + t);
            else win_apply<false>(a, unused, WIN * t, lane, cw0, Ct, Lb, prog + t);
        }
        PANEL_STAMP(1);
        if (!h1) {
            bool tz_any = false;
            __builtin_amdgcn_s_setprio(3);
            if (cw0 + WIN <= nc) win_factor<true, DEP>(a, dsc, tz_any, cw0, nc, lane, h0, p.tau, Ct, Lr, dv, prog + w, ds);
            else win_factor<false, DEP>(a, dsc, tz_any, cw0, nc, lane, h0, p.tau, Ct, Lr, dv, prog + w, ds);
            if (tz_any && lane == 0) tiny_sh = 1;
            if (DEP && ds.ndep && lane == 0) atomicAdd(&S.ndep, ds.ndep);
            if (lane == 0) __hip_atomic_store(S.wverd + w, tz_any ? 2 : 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        } else {
            __builtin_amdgcn_s_setprio(3);
            if (cw0 + WIN <= nc) win_solve<true, DEP>(a, cw0, nc, rok, lane, Ct, Lb, dv, S.prog + w, prog + w, ds);
            else win_solve<false, DEP>(a, cw0, nc, rok, lane, Ct, Lb, dv, S.prog + w, prog + w, ds);
            if (SC && rp.pub && kb + 1 < tv.ntb) {
                // hand the window to step kb + 1 (RunPub) once the diagonal
                // windows up to it passed the zero test (a DEP pass: at once;
                // its checks decide at the step's end, which the consumers await)
                bool ok = true;
                if (!DEP) {
                    for (int v = 0; v <= w; v++) {
                        int x;
                        while ((x = __hip_atomic_load(S.wverd + v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) == 0)
                            __builtin_amdgcn_s_sleep(1);
                        ok = ok && x == 1;
                    }
                }
                // the buffer's previous windows (step kb - 2's) read by every
                // panel of step kb - 1 that took them (kb - 1 > t0)
                if (ok && kb - 1 > rp.t0) {
                    const int need = max(1, (tv.nt - (kb - 1) * PC + TR - 1) / TR - 1);   // tail_gp(nt, kb - 1)
                    int got = 0;
                    if (lane == 0) {
                        for (;;) {
                            got = sc1_load_int(rp.pread + kb - 1);
                            if (got >= need) break;
                            const int b = sc1_load_int(p.flags + 2);
                            if (b && b - 1 < kb) break;        // the launch is being abandoned
                            __builtin_amdgcn_s_sleep(1);
                        }
                    }
                    ok = __builtin_amdgcn_readfirstlane(got) >= need;
                }
                if (ok) {
                    double* pb = rp.pub + (((size_t)(kb & 1) * tv.ntb + j) * 4 + w) * kTailPubWin;
                    if (rok) {
#pragma unroll
                        for (int q = 0; q < WIN; q++)
                            if (cw0 + q < nc) sc1_store(pb + q * TR + lane, a[q]);
                    }
                    if (lane < WIN) sc1_store(pb + WIN * TR + lane, dv[cw0 + lane]);
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    if (lane == 0)
                        __hip_atomic_store(rp.wflag_w + ((size_t)kb * tv.ntb + j) * 4 + w, rp.epoch, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
                }
            }
        }
        __builtin_amdgcn_s_setprio(0);
        PANEL_STAMP(2);
        // this wave's rows out as soon as its window is done: half 1 its
        // rows of L21 (and W = L21 D on the dense tail), half 0 of workgroup
        // 0 the rows of R_s inside the first 64 rows.  A sparse panel that
        // bails is redone from the assembly on, so what it wrote is moot; a
        // dense-tail panel that bails is resumed from its block column
        // (KktDevice::repair_tail), so its rows of S wait for the check
        // below (W is rewritten by the repair).
        if (wbuf && (h1 ? rok : (j == 0 && lane >= nc && lane < h0))) {
            double dw[WIN];
            win_row(&dv[cw0], dw);        // one LDS round trip, not one per column
#pragma unroll
            for (int q = 0; q < WIN; q++) {
                const int c = cw0 + q;
                if (c < nc) wbuf[row + (size_t)c * ld] = a[q] * dw[q];
            }
        }
    }
    // LDS-only barrier: the global stores above need not drain first
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
    // a pre-update from published windows: the whole of step kb - 1 done and
    // none of it bailed, before anything of this panel is written (a DEP
    // pass's saves included)
    if (winpub && !pre_wait()) return false;
    PANEL_STAMP(12);
    if (!DEP && tiny_sh && dep) return true;      // every workgroup of the panel: rerun with DEP
    // DEP: spec < 0 (dep == 2) with a dropped column in the block counts as contradicted
    const bool fail = DEP ? (S.spec > 0 || (S.spec < 0 && S.ndep > 0 && [&] {
                                 for (int k = 0; k < nc; k++)
                                     if (!S.lv[k]) return true;
                                 return false;
                             }()))
                          : tiny_sh != 0;
    if (fail) {
        if (tid == 0) {
            atomicOr(&p.flags[1], fu_sup ? 2 : DEP ? 4 | 16 : 4);   // bit: where it bailed (16: restore first)
            if (!fu_sup) atomicMax(&p.flags[2], kb + 1);   // the dense-tail block column
            if (DEP && !fu_sup && j == 0)                  // workgroup 0 added no dependent pivots
                __hip_atomic_store(p.flags + 3, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        post(true);
        return false;
    }
    // the rows of L21 (half 1) and of R_s inside the first 64 rows (half 0 of
    // workgroup 0), once the panel holds: a first pass that meets a dependent
    // pivot ends unwritten, so its DEP pass starts from the same input
    if (w < nwin && (h1 ? rok && tile : (j == 0 && lane >= nc && lane < h0))) {
#pragma unroll
        for (int q = 0; q < WIN; q++) {
            const int c = cw0 + q;
            if (c < nc) st_h<SC>(panel + row + (size_t)c * ld, a[q]);
        }
    }
    if (j == 0 && tid < nc) { st_h<SC>(p.dg + c0 + tid, dv[tid]); p.live[c0 + tid] = DEP ? S.lv[tid] != 0 : 1; }
    post(false);
    if (!fu_sup && pre && j == 0 && !h1 && lane < nc && (lane >> 4) == w) st_h<SC>(p.dscale + c0 + lane, dsc_pre);
    if (j != 0) return false;
    // workgroup 0: L11' into the upper slot through an LDS transpose (Ct is
    // free again)
    if (!h1) {
#pragma unroll
        for (int q = 0; q < WIN; q++) Ct[lane][cw0 + q] = a[q];
    }
    __syncthreads();
    for (int rr = 1 + wv; rr < nc; rr += PNT / 64)
        if (lane < rr) st_h<SC>(panel + lane + (size_t)rr * ld, Ct[rr][lane]);
    if (DEP && tid == 0) {
        if (S.ndep) atomicAdd(&p.flags[0], S.ndep);
        if (!fu_sup)                                // taken back by k_tail_restore if a later check fails
            __hip_atomic_store(p.flags + 3, S.ndep, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    PANEL_STAMP(13);
    return false;
}

__global__ void __launch_bounds__(PNT)
k_panel_w(PlanView p, const int* __restrict__ fu_sup, const int* __restrict__ fu_j, int f0, TailView tv, int kb) {
    __shared__ __attribute__((aligned(16))) char lds[sizeof(PanelLds)];
    PanelLds& S = *reinterpret_cast<PanelLds*>(lds);
    // sparse panels: a dependent pivot is resolved by a second, DEP pass
    // (panel_w_body); a failed check there bails to the redo from the assembly
    const int dep = fu_sup ? (tv.sdep ? 1 : 0) : 0;
    if (panel_w_body<false>(p, fu_sup, fu_j, f0, tv, kb, blockIdx.x, S, tv.W, false, nullptr, 0, dep)) {
        __syncthreads();
        panel_w_body<true>(p, fu_sup, fu_j, f0, tv, kb, blockIdx.x, S, tv.W, false, nullptr, 0, dep);
    }
}

// ------------------------------------------- dense tail: look-ahead steps
// Trailing update of the dense tail, one 64 x 64 tile (bi, bj) by 512
// threads: S(bi, bj) -= L(bi, kb) W(bj, kb)' with v_mfma_f64_16x16x4_f64,
// every 16 x 16 fragment accumulated over k = 0..63 in the order of
// k_tail_syrk (bitwise the same update); wave w owns rows 32 (w & 1) ..
// + 31, columns 16 (w >> 1) .. + 15.  On a diagonal tile the |terms| go to
// dscale as k_tail_syrk adds them.

// k-major, row stride SKS = 80 doubles: a wave's MFMA operand read (16
// consecutive rows x 4 k) puts the four k at bank offsets 0, 32, 0, 32 --
// two lanes per bank, the minimum for 64 eight-byte reads -- and a store of
// one k's 64 rows is conflict-free.  ([row][k] with stride 65 had up to four
// lanes on a bank on the operand reads.)
constexpr int SKS = PC + 16;
struct SyrkLds {
    double As[PC][SKS];
    double Bs[PC][SKS];
};

// |terms| of a diagonal tile's pivots over one block: as += |L(r, k) W(r, k)|
// for k = 0 .. nc - 1 in order (lane r = row r).  Sixteen products are read
// and formed ahead of their adds, so the LDS latency is paid once per
// sixteen terms instead of once per term (a rolled loop made the diagonal
// tile the slowest workgroup of every step: ~2.7 us per block).
template <int S>
__device__ __forceinline__ double diag_terms(const double (*As)[S], const double (*Bs)[S], int r, int nc, double as) {
    int k = 0;
    for (; k + 16 <= nc; k += 16) {
        double pr[16];
#pragma unroll
        for (int u = 0; u < 16; u++) pr[u] = fabs(As[k + u][r] * Bs[k + u][r]);
#pragma unroll
        for (int u = 0; u < 16; u++) as += pr[u];
    }
    for (; k < nc; k++) as += fabs(As[k][r] * Bs[k][r]);
    return as;
}
__device__ __forceinline__ double diag_terms(const SyrkLds& L, int r, int nc, double as) {
    return diag_terms<SKS>(L.As, L.Bs, r, nc, as);
}

// A wave's 32 x 16 block of a 64 x 64 product over one 64-column block
// from the k-major LDS tiles: rows wr .. wr + 31 of As, columns wc .. wc + 15
// of Bs, sixteen MFMA k-steps in order (acc[0] rows wr.., acc[1] rows
// wr + 16..).
__device__ __forceinline__ void mfma_32x16(const SyrkLds& L, int wr, int wc, int li, int lk, double4_t (&acc)[2]) {
#pragma unroll
    for (int kk = 0; kk < PC; kk += 4) {
        double av[2];
#pragma unroll
        for (int a = 0; a < 2; a++) av[a] = L.As[kk + lk][wr + a * 16 + li];
        const double bv = L.Bs[kk + lk][wc + li];
#pragma unroll
        for (int a = 0; a < 2; a++) acc[a] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[a], bv, acc[a], 0, 0, 0);
    }
}

// developer clock stamps of the visits (tools/ubench_visit.hip built with
// -DIPO_VISIT_STAMPS; compiled out otherwise): workgroup 0, per block
#ifdef IPO_VISIT_STAMPS
__device__ long long g_vstamps[8][16][6];
#define VISIT_STAMP(blk, slot)                                                                          \
    do {                                                                                                \
        if (blockIdx.x == 0 && (threadIdx.x & 63) == 0 && (blk) < 16)                                   \
            g_vstamps[threadIdx.x >> 6][(blk)][(slot)] = clock64();                                     \
    } while (0)
#else
#define VISIT_STAMP(blk, slot) do {} while (0)
#endif

__device__ __forceinline__ void syrk_tile512(const PlanView& p, const TailView& tv, int kb, int bi, int bj,
                                             SyrkLds& L) {
    const int nt = tv.nt, k0 = kb * PC, nc = min(PC, nt - k0), tid = threadIdx.x;
    const double* Lcol = tv.S + (size_t)k0 * nt;
    {
        double va[TR * PC / PNT], vb[TR * PC / PNT];
#pragma unroll
        for (int u = 0; u < TR * PC / PNT; u++) {
            const int idx = tid + u * PNT, rr = idx % TR, k = idx / TR;
            const int ra = bi * TR + rr, rb = bj * TR + rr;
            const bool oka = k < nc && ra < nt, okb = k < nc && rb < nt;
            const double x = Lcol[oka ? ra + (size_t)k * nt : 0];
            const double y = Lcol[okb ? rb + (size_t)k * nt : 0];    // W = L21 D formed here (bitwise its store)
            const double d = p.dg[tv.tc + k0 + (k < nc ? k : 0)];
            va[u] = oka ? x : 0.0;
            vb[u] = okb ? y * d : 0.0;
        }
#pragma unroll
        for (int u = 0; u < TR * PC / PNT; u++) {
            const int idx = tid + u * PNT;
            L.As[idx / TR][idx % TR] = va[u];
            L.Bs[idx / TR][idx % TR] = vb[u];
        }
    }
    __syncthreads();
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
    const int wr = (wv & 1) * 32, wc = (wv >> 1) * 16;
    double4_t acc[2];
#pragma unroll
    for (int a = 0; a < 2; a++) acc[a] = (double4_t){0.0, 0.0, 0.0, 0.0};
    const int li = lane & 15, lk = lane >> 4;
    mfma_32x16(L, wr, wc, li, lk, acc);
    const bool diag_tile = bi == bj;
    double old[2][4];
#pragma unroll
    for (int a = 0; a < 2; a++)
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const int rr = wr + a * 16 + (lane >> 4) + 4 * i, cc = wc + (lane & 15);
            const int rg = bi * TR + rr, cg = bj * TR + cc;
            const bool ok = rg < nt && cg < nt && !(diag_tile && cc > rr);
            old[a][i] = ok ? tv.S[rg + (size_t)cg * nt] : 0.0;
        }
#pragma unroll
    for (int a = 0; a < 2; a++)
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const int rr = wr + a * 16 + (lane >> 4) + 4 * i, cc = wc + (lane & 15);
            const int rg = bi * TR + rr, cg = bj * TR + cc;
            if (rg < nt && cg < nt && !(diag_tile && cc > rr)) tv.S[rg + (size_t)cg * nt] = old[a][i] - acc[a][i];
        }
    if (diag_tile && tid < TR) {
        const int rg = bi * TR + tid;
        if (rg < nt) {
            p.dscale[tv.tc + rg] += diag_terms(L, tid, nc, 0.0);
        }
    }
}


// Deferred trailing update of the dense tail ("visit"): tile (bi, bj) of S
// receives the updates of blocks b0 .. b1 - 1 (at most TailView::vk) in one
// pass, S(bi, bj) -= sum_b L(bi, b) W(bj, b)', W = L D formed on the load
// (no W array: bitwise the product the panel would store), the products summed
// in the MFMA accumulators (k ascending inside a block, blocks ascending),
// one read-modify-write of the tile for all of them.  Block b + 1's operands
// are loaded into registers while block b's are multiplied from LDS (two
// blocks in flight measured no faster: tools/ubench_tail, round 4).  On a
// diagonal tile the |terms| of every block go to dscale (one add).
// SC: the persistent tail's hand-off form (sc1 loads and stores, panel_w_body).
template <bool SC = false>
__device__ __forceinline__ void visit_tile512(const PlanView& p, const TailView& tv, int bi, int bj, int b0, int b1,
                                              SyrkLds& L, const int* bailp = nullptr, int bt = 0) {
    // a bail flag of an earlier step (see k_tail_pr), read in the shadow of
    // the first operand loads
    const int bailed = bailp ? *bailp : 0;
    const int nt = tv.nt, tid = threadIdx.x;
    constexpr int NU = TR * PC / PNT;
    // raw operand loads of a block: L rows of tile bi (x) and of tile bj
    // (y), and D (d); nothing is computed from them until the block is
    // staged into LDS -- arithmetic on a load right after it is issued
    // makes the wave wait for it there, before the previous block's MFMA
    // steps, and the load latency is then paid once per block
    double rx[NU], ry[NU], rd[NU];
    // element offsets of this thread's operands inside a block column,
    // the same for every block (rows clamped into the tail): a block's loads
    // are a uniform base plus these, no per-block address arithmetic (the
    // 64-bit address of every load took ~2,000 cycles per block to issue)
    int offa[NU], offb[NU];
#pragma unroll
    for (int u = 0; u < NU; u++) {
        const int idx = tid + u * PNT, rr = idx % TR, k = idx / TR;
        offa[u] = min(bi * TR + rr, nt - 1) + k * nt;
        offb[u] = min(bj * TR + rr, nt - 1) + k * nt;
    }
    auto load = [&](int b, double (&xx)[NU], double (&yy)[NU], double (&dd)[NU]) {
        const int k0 = b * PC;
        const double* __restrict__ Lcol = tv.S + (size_t)k0 * nt;
        const double* __restrict__ dgb = p.dg + tv.tc + k0;
        if (k0 + PC <= nt) {
#pragma unroll
            for (int u = 0; u < NU; u++) {
                xx[u] = ld_h<SC>(Lcol + offa[u]);
                yy[u] = ld_h<SC>(Lcol + offb[u]);
                dd[u] = ld_h<SC>(dgb + (tid + u * PNT) / TR);
            }
        } else {                       // the last, partial block column: columns clamped too
            const int kmax = nt - 1 - k0;
#pragma unroll
            for (int u = 0; u < NU; u++) {
                const int idx = tid + u * PNT, k = idx / TR, kc = min(k, kmax);
                xx[u] = ld_h<SC>(Lcol + offa[u] - (k - kc) * nt);
                yy[u] = ld_h<SC>(Lcol + offb[u] - (k - kc) * nt);
                dd[u] = ld_h<SC>(dgb + kc);
            }
        }
    };
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
    const int wr = (wv & 1) * 32, wc = (wv >> 1) * 16;
    const int li = lane & 15, lk = lane >> 4;
    const bool diag_tile = bi == bj;
    double4_t acc[2];
#pragma unroll
    for (int a = 0; a < 2; a++) acc[a] = (double4_t){0.0, 0.0, 0.0, 0.0};
    double as = 0.0;
    load(b0, rx, ry, rd);
    // the tile's own entries (no other workgroup of the launch touches
    // them), read now so their latency hides under the products; column-
    // coalesced (wave wv holds columns wv, wv + 8, ..., lane = row: one
    // 512-byte column segment per load), the products come to this layout
    // through LDS at the end
    double old[8];
    const int rgl = bi * TR + lane;
#pragma unroll
    for (int u = 0; u < 8; u++) {
        const int cc = wv + 8 * u, cg = bj * TR + cc;
        const bool ok = rgl < nt && cg < nt && !(diag_tile && cc > lane);
        old[u] = ld_h<SC>(tv.S + (ok ? rgl + (size_t)cg * nt : 0));
    }
    if (bailed && bailed - 1 < bt) return;
    // block b: operands from registers into LDS, block b + 1's loads into
    // the freed registers, then block b's MFMA steps
    auto step = [&](int b, double (&xx)[NU], double (&yy)[NU], double (&dd)[NU]) {
        VISIT_STAMP(b - b0, 0);
        const int nc = min(PC, nt - b * PC);
#pragma unroll
        for (int u = 0; u < NU; u++) {
            const int idx = tid + u * PNT, rr = idx % TR, k = idx / TR;
            const bool oka = k < nc && bi * TR + rr < nt, okb = k < nc && bj * TR + rr < nt;
            L.As[k][rr] = oka ? xx[u] : 0.0;
            L.Bs[k][rr] = okb ? yy[u] * dd[u] : 0.0;    // W = L21 D of block b, formed as its panel forms it (bitwise)
        }
        VISIT_STAMP(b - b0, 1);
        __syncthreads();
        VISIT_STAMP(b - b0, 2);
        if (b + 1 < b1) load(b + 1, xx, yy, dd);
        VISIT_STAMP(b - b0, 3);
        mfma_32x16(L, wr, wc, li, lk, acc);
        VISIT_STAMP(b - b0, 4);
        if (diag_tile && tid < TR) as = diag_terms(L, tid, min(PC, nt - b * PC), as);
        __syncthreads();
        VISIT_STAMP(b - b0, 5);
    };
    for (int b = b0; b < b1; b++) step(b, rx, ry, rd);
    // the products to [column][row] in LDS (free after the last step's barrier)
#pragma unroll
    for (int a = 0; a < 2; a++)
#pragma unroll
        for (int i = 0; i < 4; i++) L.As[wc + (lane & 15)][wr + a * 16 + (lane >> 4) + 4 * i] = acc[a][i];
    __syncthreads();
#pragma unroll
    for (int u = 0; u < 8; u++) {
        const int cc = wv + 8 * u, cg = bj * TR + cc;
        if (rgl < nt && cg < nt && !(diag_tile && cc > lane)) st_h<SC>(tv.S + rgl + (size_t)cg * nt, old[u] - L.As[cc][lane]);
    }
    if (diag_tile && tid < TR && bi * TR + tid < nt) {
        double* dp = p.dscale + tv.tc + bi * TR + tid;
        st_h<SC>(dp, ld_h<SC>(dp) + as);
    }
}

constexpr size_t kTailStepLds0 = sizeof(PanelLds) > sizeof(SyrkLds) ? sizeof(PanelLds) : sizeof(SyrkLds);
constexpr size_t kTailStepLds = kTailStepLds0 > sizeof(PreLds) ? kTailStepLds0 : sizeof(PreLds);

// Visits of launch t (tail_visit_cols): block column c receives the updates
// of blocks 0 .. c - 2 in chunks of K = TailView::vk, the latest chunk in launch
// c - 1, the one before in launch c - 2, ...: launch c - 1 - k applies blocks
// [c - 1 - 4 (k + 1), c - 1 - 4 k) (clipped at 0) -- every block available
// (b < t) and every column done before its panel, block c - 1 being the
// panel's own pre-update.  Each entry still receives blocks 0, 1, ... in
// order; the work is spread over the launches (late-as-possible, so the
// early steps, once 3x the panel's time under the right-looking update, are
// panel-bound) and a tile is read and written once per chunk, not per block.
__host__ __device__ __forceinline__ int visit_hi(int t, int c, int K) { return c - 1 - K * (c - 1 - t); }

// Step t of the look-ahead dense-tail factorisation, one launch:
//   workgroups [0, gp):  panel of block column t (k_panel_w's body);
//   the rest:            the visits of launch t, one tile each, columns
//                        t + 1, t + 2, ... (visit_hi above).
// Block column t holds every update from blocks <= t - 2 (earlier visits);
// the panel workgroups apply block t - 1's to their own rows first
// (panel_w_body's pre-update, k_tail_syrk's fragments and order).
__global__ void __launch_bounds__(PNT)
k_tail_pr(PlanView p, TailView tv, int t, int gp, int vbase) {
    __shared__ __attribute__((aligned(16))) char lds[kTailStepLds];
    // a panel of an earlier step bailed (flags[2] = 1 + its block column;
    // not this launch's own, whose visits must complete): the host
    // resumes the look-ahead from there
    if ((int)blockIdx.x < gp) {
        PanelLds& S = *reinterpret_cast<PanelLds*>(lds);
        if (panel_w_body<false>(p, nullptr, nullptr, 0, tv, t, blockIdx.x, S, nullptr, t > 0, p.flags + 2, t, tv.dep)) {
            __syncthreads();           // every wave has read the first pass's verdict
            panel_w_body<true>(p, nullptr, nullptr, 0, tv, t, blockIdx.x, S, nullptr, t > 0, p.flags + 2, t, tv.dep);
        }
        return;
    }
    if (tv.vlist) {
        const unsigned v = tv.vlist[vbase + blockIdx.x - gp];
        visit_tile512(p, tv, v & 255, (v >> 8) & 255, (v >> 16) & 255, v >> 24, *reinterpret_cast<SyrkLds*>(lds),
                      p.flags + 2, t);
        return;
    }
    int tile = blockIdx.x - gp, c = t + 1;
    while (tile >= tv.ntb - c) { tile -= tv.ntb - c; c++; }
    const int b1 = visit_hi(t, c, tv.vk);
    visit_tile512(p, tv, c + tile, c, max(0, b1 - tv.vk), b1, *reinterpret_cast<SyrkLds*>(lds), p.flags + 2, t);
}

// ----------------------------------------- dense tail: one persistent launch
// The look-ahead steps t0 .. ntb - 1 as work items of ONE launch
// (tail_run_schedule): each workgroup draws one item from a ticket counter
// when it starts (schedule order) and runs it to completion --
//   panel (t, j): workgroup j of k_tail_pr's panel of step t (pre-update of
//                 block t - 1 on its rows, then the windowed panel);
//   visit:        one deferred trailing update of launch t (visit_tile512).
// An item waits only on items with smaller tickets: every item of launch t
// on the panels of step t - 1 (what the launch boundary gave k_tail_pr), a
// panel on the visits of its two tiles (per-tile sequence counters vseq), a
// visit on the chunks of its tile before it.  So no launch gap separates the
// steps, a panel starts as soon as its own inputs are final, its entries
// load before it waits for step t - 1, and the grid drains on any share of
// the CUs (a ticket is only drawn by a running workgroup).  Hand-offs: the
// data sc1 both ways, every storing wave's vmcnt(0) and a barrier before one
// lane's agent-scope add (MI355X_MICROARCH.md's first row).  A panel that
// bails (flags[2]) still counts itself, so its step's visits complete as in
// k_tail_pr; every item of a later launch reads the flag after its wait and
// is skipped without counting, and the host repair resumes the run from
// step tb + 1 with the counters as they are.
__host__ __device__ __forceinline__ int tail_gp(int nt, int t) { return max(1, (nt - t * PC + TR - 1) / TR - 1); }
// visits (chunks) of block column c in the persistent schedules (run_chunks)
__host__ __device__ __forceinline__ int run_chunk_count(int c, int K, int L) {
    return c <= 1 ? 0 : 1 + (max(0, c - 1 - L) + K - 1) / K;
}


__global__ void __launch_bounds__(PNT)
k_tail_run(PlanView p, TailView tv, TailRun rc) {
    __shared__ __attribute__((aligned(16))) char lds[kTailStepLds];
    // the two waits of a panel item report through different words: no
    // barrier separates a slow wave's read of the first from the second's write
    __shared__ int sh_item, sh_ok, sh_ok2;
    const int ntb = tv.ntb;
    const int* bailp = p.flags + 2;
    // one item per workgroup, drawn when the workgroup starts (a loop over
    // items in a persistent grid kept more registers live: 256 VGPRs and
    // spills against k_tail_pr's 218; the dispatcher starts a workgroup as
    // soon as a CU frees, so the items still flow in ticket order)
    if (threadIdx.x == 0) sh_item = __hip_atomic_fetch_add(rc.ticket, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    const int it = sh_item;
    if (it >= rc.n) return;
    const uint2 rec = rc.items[it];
    const int t = rec.y & 0xff, q = (rec.y >> 8) & 0xff;
    unsigned long long* tr = rc.trace ? rc.trace + 4 * (size_t)it : nullptr;
    if (tr && threadIdx.x == 0) {
        tr[0] = __builtin_amdgcn_s_memrealtime();
        tr[3] = __builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (3 << 11));   // HW_REG_XCC_ID bits 0..3
    }
    if (rec.y >> 31) {
        // panel (t, j): column t's visits done for the diagonal tile and tile t + j + 1
        const int j = rec.x;
        const int* vd = q ? rc.vseq + t * ntb + t : nullptr;
        const int* vt = q && t + j + 1 < ntb ? rc.vseq + (t + j + 1) * ntb + t : nullptr;
        // (with the window hand-off the panel waits for them itself, after
        // its pre-update's products: RunPub)
        const bool winpub = rc.pub && t > 0 && t - 1 >= rc.t0;
        if (!winpub && !run_wait(vd, q, vt, q, bailp, t, &sh_ok)) return;
        // (the first step of a run resumed after a repair waits for nothing
        // before it: the repair's launches came first)
        auto pw = [&]() {
            const bool go = t == rc.t0 || run_wait(rc.pdone + t - 1, tail_gp(tv.nt, t - 1), nullptr, 0, bailp, t, &sh_ok2);
            if (tr && threadIdx.x == 0) tr[1] = __builtin_amdgcn_s_memrealtime();
            return go;
        };
        auto post = [&](bool bailed) { run_signal(rc.pdone + t, bailed ? 1 + kRunBail : 1); };
        if (tr && threadIdx.x == 0 && t == 0) tr[1] = __builtin_amdgcn_s_memrealtime();
        PanelLds& S = *reinterpret_cast<PanelLds*>(lds);
        const RunPub rp{rc.pub, rc.wflag, rc.wflag, rc.pread, rc.t0, rc.epoch, vd, vt, q, &sh_ok};
        if (panel_w_body<false, true>(p, nullptr, nullptr, 0, tv, t, j, S, nullptr, t > 0, nullptr, t, tv.dep, pw,
                                      post, rp)) {
            __syncthreads();           // every wave has read the first pass's verdict
            panel_w_body<true, true>(p, nullptr, nullptr, 0, tv, t, j, S, nullptr, t > 0, nullptr, t, tv.dep, NoWait{},
                                     post, rp);
        }
    } else {
        // visit: chunk q of tile (bi, c), once the panels of step t - 1 are done
        const int bi = rec.x & 255, c = (rec.x >> 8) & 255, b0 = (rec.x >> 16) & 255, b1 = rec.x >> 24;
        int* vs = rc.vseq + bi * ntb + c;
        if (!run_wait(t > rc.t0 ? rc.pdone + t - 1 : nullptr, t > rc.t0 ? tail_gp(tv.nt, t - 1) : 0, q ? vs : nullptr,
                      q, bailp, t, &sh_ok))
            return;
        if (tr && threadIdx.x == 0) tr[1] = __builtin_amdgcn_s_memrealtime();
        visit_tile512<true>(p, tv, bi, c, b0, b1, *reinterpret_cast<SyrkLds*>(lds));
        run_signal(vs);
    }
    if (tr && threadIdx.x == 0) tr[2] = __builtin_amdgcn_s_memrealtime();
}

// ------------------------------- dense tail: one launch around a chain workgroup
// k_tail_chain_run (opt-in, IPO_HIP_TAIL_CHAIN=1; slower than k_tail_run, DESIGN.md
// section 6.3): the steps of the
// look-ahead factorisation as ticketed items of one launch, like k_tail_run,
// but the critical path -- diagonal block t, the tile t + 1 below it, block t
// + 1's pre-update by block t -- stays inside ONE long-lived workgroup (the
// chain item, ticket 0, one pass over every block column):
//   waves 0-3 (half 0) factor diagonal block t by windows (win_factor), and
//     publish each window, once it and every window before it passed the
//     zero test, to global memory (c = l d of the block rows, d, marks:
//     dpub, flag dwin) for the tile items;
//   waves 4-7 (half 1) solve tile t + 1 against the block's windows through
//     LDS (win_solve), as k_panel_w's workgroup 0 does;
//   block t + 1's pre-update by block t, L(t+1, t) W(t+1, t)' with W = L D
//     (the products k_tail_pr's next launch would reload and form), is
//     accumulated in the MFMA registers of half 0 as half 1 completes each
//     window of tile t + 1 -- the operands never leave LDS -- and the |terms|
//     of block t + 1's pivots beside it, k in order;
//   tile t + 2's pre-update by block t, L(t+2, t) W(t+1, t)', is formed by
//     half 1 once the tile item (t, t + 2) has stored its rows, while half 0
//     already factors block t + 1.
// Every entry receives the same products in the same order as in k_tail_pr
// (the same MFMA fragments, k ascending, then old - acc; the same window
// operations), so the factor is bitwise that of k_tail_run with the same
// visit chunks.  Tile items (t, R), R >= t + 2: the tile's pre-update (as
// k_tail_pr's panel workgroups), then tile R solved window by window against
// the chain's published windows.  Visits: as in k_tail_run.  A dependent
// pivot in block t: the chain reruns the block with the rule of ldlt.c:600-614
// from its saved inputs (what it published before the failing window is
// unchanged); a tile that contradicts a dropped column, a NaN in the rule, or
// a zero pivot without the in-panel rule (TailView::dep == 0) aborts the
// launch (flags[1] bit 64) and the host redoes the factorisation with the
// per-step look-ahead and its repairs.  Waits poll the abort flag, so the
// grid always drains.
struct ChainLds {
    PanelLds P;               // Ct, Lr, Lb, dv, lv, prog[8], tiny, spec, ndep
    double T[PC][CTS];        // half 1: L(t + 2, t) as [k][row], then the product as [col][row]
    double dvp[PC];           // D of block t (half 1's product runs while block t + 1 overwrites dv)
    int hs[2];                // half-0 / half-1 meeting counters (monotonic)
    int winok[4];             // diagonal window verdicts of the current pass: pass << 2 | 1 clean, | 2 zero pivot
    int arrive;               // half-1 waves whose step results have drained (monotonic)
    int sh[2];                // workgroup wait verdicts
};
constexpr size_t kChainItemLds = sizeof(ChainLds) > kTailStepLds ? sizeof(ChainLds) : kTailStepLds;

__host__ __device__ __forceinline__ int chain_target(int ntb, int t) { return 1 + max(0, ntb - t - 2); }

__device__ __forceinline__ void chain_abort(const PlanView& p, int* abortp) {
    atomicOr(&p.flags[1], 64);
    __hip_atomic_store(abortp, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// the four waves of one half meet (the other half runs on): each wave bumps
// an LDS counter once per meeting; gen counts this wave's meetings
__device__ __forceinline__ void half_sync(int* cnt, int& gen) {
    gen += 4;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    if ((threadIdx.x & 63) == 0) __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    while (__builtin_amdgcn_readfirstlane(__hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) < gen)
        __builtin_amdgcn_s_sleep(1);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// one wave waits until *c >= v (lane 0 polls); false: the launch aborted
__device__ __forceinline__ bool wave_poll(const int* c, int v, const int* abortp) {
    int ok = 1;
    if ((threadIdx.x & 63) == 0) {
        while (sc1_load_int(c) < v) {
            if (sc1_load_int(abortp)) {
                ok = 0;
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
    }
    return __builtin_amdgcn_readfirstlane(ok) != 0;
}

// the workgroup waits until *c0 >= v0 and *c1 >= v1 (null: none); false: abort
__device__ __forceinline__ bool chain_wg_wait(const int* c0, int v0, const int* c1, int v1, const int* abortp, int* sh) {
    if (threadIdx.x == 0) {
        int ok = 1;
        for (;;) {
            if ((!c0 || sc1_load_int(c0) >= v0) && (!c1 || sc1_load_int(c1) >= v1)) break;
            if (sc1_load_int(abortp)) {
                ok = 0;
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
        *sh = ok;
    }
    __syncthreads();
    return *sh != 0;
}

// lower 16 x 16 fragments (fx >= fy) of block t + 1's pre-update, three per
// half-0 wave for waves 0-1, two for 2-3
__device__ constexpr int kPdFx[12] = {0, 1, 2, 3, 1, 2, 3, 2, 3, 3, -1, -1};
__device__ constexpr int kPdFy[12] = {0, 0, 0, 0, 1, 1, 1, 2, 2, 3, -1, -1};

// block column k1's diagonal block after its visits: this wave's window of
// columns (lower triangle), and the |terms| of the pivots it holds
__device__ __forceinline__ void chain_load_diag(const TailView& tv, const PlanView& p, int k1, int nc1, int h01, int cw0,
                                                int lane, int w, double (&sd)[WIN], double& dscl) {
    const int nt = tv.nt;
    const bool rk = lane < h01;
#pragma unroll
    for (int q = 0; q < WIN; q++) {
        const int c = cw0 + q;
        const bool ok = rk && c < nc1 && c <= lane;
        const double x = sc1_load(tv.S + (ok ? k1 + lane + (size_t)(k1 + c) * nt : 0));
        sd[q] = ok ? x : 0.0;
    }
    dscl = (lane < nc1 && (lane >> 4) == w) ? sc1_load(p.dscale + tv.tc + k1 + lane) : 0.0;
}

// developer trace of the chain (ChainRun::trace): per step and wave four
// stamps after the items' records: e 0 own window begins, 1 it ends, 2 the
// pass's work done, 3 after the pass's barriers
#define CHAIN_STAMP(t, e)                                                                              \
    do {                                                                                               \
        if (rc.trace && (threadIdx.x & 63) == 0)                                                       \
            rc.trace[4 * ((size_t)rc.n + tv.ntb) + (size_t)(t) * 32 + (threadIdx.x >> 6) * 4 + (e)] =   \
                __builtin_amdgcn_s_memrealtime();                                                      \
    } while (0)

// The chain item is two loops over the block columns, one per half of the
// workgroup (waves 0-3 and 4-7), meeting at the same workgroup barriers (two
// per pass) and through LDS counters: each half keeps only its own state
// live (written as one interleaved loop the two halves' registers added up
// and spilled).
// Half 0: block t's windows, their publication, block t + 1's pre-update.
__device__ __forceinline__ void chain_half0(const PlanView& p, const TailView& tv, const ChainRun& rc,
                                                      ChainLds& C) {
    PanelLds& S = C.P;
    const int nt = tv.nt, ntb = tv.ntb, tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6), cw0 = WIN * w;
    const int li = lane & 15, lk = lane >> 4;
    int passes = 0, g0 = 0;
    double a[WIN], dsc;
    {
        // step 0: S(0, 0)'s lower triangle and the |terms| of its pivots
        const int nc = min(PC, nt);
#pragma unroll
        for (int q = 0; q < WIN; q++) {
            const int c = cw0 + q;
            const bool ok = lane < nc && c < nc && c <= lane;
            const double x = sc1_load(tv.S + (ok ? lane + (size_t)c * nt : 0));
            a[q] = ok ? x : 0.0;
        }
        dsc = (lane < nc && (lane >> 4) == w) ? sc1_load(p.dscale + tv.tc + lane) : 0.0;
    }
    for (int t = 0; t < ntb; t++) {
        const int k0 = t * PC, nc = min(PC, nt - k0), h = nt - k0, h0 = min(PC, h), c0 = tv.tc + k0;
        double* panel = tv.S + k0 + (size_t)k0 * nt;
        const bool next = t + 1 < ntb;
        const int nwin = (nc + WIN - 1) / WIN;
        const bool holder = lane < nc && (lane >> 4) == w;
        unsigned long long* tr = rc.trace ? rc.trace + 4 * (size_t)(rc.n + t) : nullptr;
        if (tr && tid == 0) tr[0] = __builtin_amdgcn_s_memrealtime();
        // the step's inputs, for a dependent-pivot rerun (each wave reloads its own)
#pragma unroll
        for (int q = 0; q < WIN; q++) sc1_store(rc.save + (cw0 + q) * PC + lane, a[q]);
        if (holder) sc1_store(rc.save + 2 * PC * PC + lane, dsc);
        const double dsc_in = dsc;         // |terms| before the block's own steps: dscale(t)
        double4_t pacc[3];
        double asum = 0.0, sd[WIN], dscl = 0.0;
        bool have_sd = false, dep_pass = false;
        for (;;) {
            passes++;
            const int pb = WIN * passes;
            if (tid == 0) S.ndep = 0;
#pragma unroll
            for (int f = 0; f < 3; f++) pacc[f] = (double4_t){0.0, 0.0, 0.0, 0.0};
            asum = 0.0;
            if (w < nwin) {
                DepState ds{p.sign + c0, S.lv, &S.spec, 0, passes};
                int* const prog = S.prog;
                for (int t2 = 0; t2 < w; t2++) {
                    if (t2 + 1 < w) __builtin_amdgcn_s_setprio(1);
                    else __builtin_amdgcn_s_setprio(3);
                    win_apply<true>(a, dsc, WIN * t2, lane, cw0, S.Ct, S.Lr, prog + t2, pb);
                }
                __builtin_amdgcn_s_setprio(3);
                CHAIN_STAMP(t, 0);
                bool tz = false;
                const bool full = cw0 + WIN <= nc;
                if (dep_pass) {
                    if (full) win_factor<true, true>(a, dsc, tz, cw0, nc, lane, h0, p.tau, S.Ct, S.Lr, S.dv, prog + w, ds, pb);
                    else win_factor<false, true>(a, dsc, tz, cw0, nc, lane, h0, p.tau, S.Ct, S.Lr, S.dv, prog + w, ds, pb);
                    if (ds.ndep && lane == 0) atomicAdd(&S.ndep, ds.ndep);
                } else {
                    if (full) win_factor<true, false>(a, dsc, tz, cw0, nc, lane, h0, p.tau, S.Ct, S.Lr, S.dv, prog + w, ds, pb);
                    else win_factor<false, false>(a, dsc, tz, cw0, nc, lane, h0, p.tau, S.Ct, S.Lr, S.dv, prog + w, ds, pb);
                }
                __builtin_amdgcn_s_setprio(0);
                CHAIN_STAMP(t, 1);
                if (tz && lane == 0) S.tiny = passes;
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
                if (lane == 0)
                    __hip_atomic_store(&C.winok[w], passes << 2 | (tz ? 2 : 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                // publish the window when it and every window before it passed the
                // zero test (the dependent-pivot pass: all of them)
                bool clean = !tz || dep_pass;
                for (int v = 0; v < w; v++) {
                    int x;
                    while (((x = __builtin_amdgcn_readfirstlane(__hip_atomic_load(&C.winok[v], __ATOMIC_RELAXED,
                                                                                   __HIP_MEMORY_SCOPE_WORKGROUP))) >> 2) != passes)
                        __builtin_amdgcn_s_sleep(1);
                    clean = clean && (dep_pass || (x & 3) == 1);
                }
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
                if (clean && t + 2 < ntb) {
                    double* dst = rc.dpub + ((size_t)t * 4 + w) * kChainWinPub;
#pragma unroll
                    for (int kk = 0; kk < WIN; kk++) sc1_store(dst + kk * PC + lane, S.Ct[cw0 + kk][lane]);
                    if (lane < WIN) {
                        sc1_store(dst + WIN * PC + lane, S.dv[cw0 + lane]);
                        sc1_store(dst + WIN * PC + WIN + lane, dep_pass ? static_cast<double>(S.lv[cw0 + lane]) : 1.0);
                    }
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    if (lane == 0) __hip_atomic_store(rc.dwin + t * 4 + w, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
                // block t + 1's pre-update by block t, as half 1 completes each
                // window of tile t + 1: the fragments k ascending, the |terms| of
                // block t + 1's pivots (lane r = its row r) beside them
                if (next) {
                    const int k1 = k0 + PC, nc1 = min(PC, nt - k1);
                    for (int v = 0; v < 4; v++) {
                        if (v == 3 && !have_sd) {
                            // block t + 1 after its visits, ahead of the step's end (after
                            // an abort the wait falls through: the chain runs on with
                            // garbage to its end, every wave in step, and the host
                            // discards the launch)
                            wave_poll(rc.vseq + (t + 1) * ntb + t + 1, (rc.novisit ? 0 : run_chunk_count(t + 1, tv.vk, rc.latest)), rc.abort);
                            chain_load_diag(tv, p, k1, nc1, min(PC, nt - k1), cw0, lane, w, sd, dscl);
                            have_sd = true;
                        }
                        int seen = 0;
                        df_wait(S.prog + 4 + v, pb + WIN, seen);
#pragma unroll
                        for (int f = 0; f < 3; f++) {
                            const int fi = w + 4 * f, fx = kPdFx[fi], fy = kPdFy[fi];
                            if (fx < 0) continue;
#pragma unroll
                            for (int s4 = 0; s4 < 4; s4++) {
                                const int kk = WIN * v + 4 * s4 + lk;
                                const double av = S.Lb[kk][fx * 16 + li];
                                const double bv = S.Lb[kk][fy * 16 + li] * S.dv[kk];
                                pacc[f] = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, pacc[f], 0, 0, 0);
                            }
                        }
                        if (lane < nc1 && (lane >> 4) == w) {
#pragma unroll
                            for (int u = 0; u < WIN; u++) {
                                const double x = S.Lb[WIN * v + u][lane];
                                asum += fabs(x * (x * S.dv[WIN * v + u]));
                            }
                        }
                    }
                }
            }
            CHAIN_STAMP(t, 2);
            __syncthreads();
            const bool tiny = S.tiny == passes;
            const bool spec = S.spec == passes;
            __syncthreads();           // read by every wave before any can overwrite them
            CHAIN_STAMP(t, 3);
            if (!dep_pass && tiny && tv.dep) {
                // rerun the block with the dependent-pivot rule from the saved inputs
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
                for (int q = 0; q < WIN; q++) a[q] = sc1_load(rc.save + (cw0 + q) * PC + lane);
                dsc = holder ? sc1_load(rc.save + 2 * PC * PC + lane) : 0.0;
                dep_pass = true;
                continue;
            }
            if (spec || (!dep_pass && tiny)) {
                if (tid == 0) chain_abort(p, rc.abort);
                return;
            }
            break;
        }
        if (tr && tid == 0) tr[1] = __builtin_amdgcn_s_memrealtime();
        // L11' into the block's upper slot (Lr[c][r] = l(r, c)), the rows of the
        // block below nc (the last, partial block), marks, |terms|
        for (int rr = 1 + w; rr < nc; rr += 4)
            if (lane < rr) sc1_store(panel + lane + (size_t)rr * nt, S.Lr[lane][rr]);
        if (lane >= nc && lane < h0) {
#pragma unroll
            for (int q = 0; q < WIN; q++)
                if (cw0 + q < nc) sc1_store(panel + lane + (size_t)(cw0 + q) * nt, S.Lr[cw0 + q][lane]);
        }
        if (tid < nc) p.live[c0 + tid] = dep_pass ? S.lv[tid] != 0 : 1;
        if (holder && t > 0) sc1_store(p.dscale + c0 + lane, dsc_in);
        if (dep_pass && tid == 0 && S.ndep) atomicAdd(&p.flags[0], S.ndep);
        if (tr && tid == 0) tr[2] = __builtin_amdgcn_s_memrealtime();
        if (!next) break;
        // block t + 1: its entries after the visits minus block t's product
        const int k1 = k0 + PC, nc1 = min(PC, nt - k1), h01 = min(PC, nt - k1);
        if (!have_sd) {
            wave_poll(rc.vseq + (t + 1) * ntb + t + 1, (rc.novisit ? 0 : run_chunk_count(t + 1, tv.vk, rc.latest)), rc.abort);
            chain_load_diag(tv, p, k1, nc1, h01, cw0, lane, w, sd, dscl);
        }
        // the fragments to LDS as [col][row] (Ct is free: every window of block t is done)
#pragma unroll
        for (int f = 0; f < 3; f++) {
            const int fi = w + 4 * f, fx = kPdFx[fi], fy = kPdFy[fi];
            if (fx < 0) continue;
#pragma unroll
            for (int i = 0; i < 4; i++) S.Ct[fy * 16 + li][fx * 16 + lk + 4 * i] = pacc[f][i];
        }
        half_sync(&C.hs[0], g0);
        const bool rk = lane < h01;
#pragma unroll
        for (int q = 0; q < WIN; q++) {
            const int c = cw0 + q;
            a[q] = (rk && c < nc1 && c <= lane) ? sd[q] - S.Ct[c][lane] : 0.0;
        }
        dsc = (lane < nc1 && (lane >> 4) == w) ? dscl + asum : 0.0;
        // (each wave reads only its own columns of the product, which it alone
        // overwrites next, with block t + 1's window: no second meeting)
    }
}

// Half 1: tile t + 1 against block t's windows; its rows, D and the step's
// signal; tile t + 2's pre-update by block t for the next step.
__device__ __forceinline__ void chain_half1(const PlanView& p, const TailView& tv, const ChainRun& rc,
                                                      ChainLds& C) {
    PanelLds& S = C.P;
    const int nt = tv.nt, ntb = tv.ntb, tid = threadIdx.x, lane = tid & 63;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6), w = (wv + 2) & 3, cw0 = WIN * w;
    const int li = lane & 15, lk = lane >> 4;
    int passes = 0, g1 = 0;
    double a[WIN];
    {
        // step 0: tile 1's entries (the rows 64 .. 127 of block column 0)
        const int nc = min(PC, nt), row = TR + lane;
#pragma unroll
        for (int q = 0; q < WIN; q++) {
            const int c = cw0 + q;
            const bool ok = row < nt && c < nc;
            const double x = sc1_load(tv.S + (ok ? row + (size_t)c * nt : 0));
            a[q] = ok ? x : 0.0;
        }
    }
    for (int t = 0; t < ntb; t++) {
        const int k0 = t * PC, nc = min(PC, nt - k0), h = nt - k0, c0 = tv.tc + k0;
        double* panel = tv.S + k0 + (size_t)k0 * nt;
        const int row = TR + lane;
        const bool rok = row < h;
        const bool tile = TR < h;
        const int nwin = (nc + WIN - 1) / WIN;
#pragma unroll
        for (int q = 0; q < WIN; q++) sc1_store(rc.save + PC * PC + (cw0 + q) * PC + lane, a[q]);
        bool dep_pass = false;
        for (;;) {
            passes++;
            const int pb = WIN * passes;
            if (w < nwin && tile) {
                DepState ds{p.sign + c0, S.lv, &S.spec, 0, passes};
                int* const prog = S.prog + 4;
                double unused = 0.0;
                for (int t2 = 0; t2 < w; t2++) {
                    if (t2 + 1 < w) __builtin_amdgcn_s_setprio(0);
                    else __builtin_amdgcn_s_setprio(2);
                    win_apply<false>(a, unused, WIN * t2, lane, cw0, S.Ct, S.Lb, prog + t2, pb);
                }
                __builtin_amdgcn_s_setprio(3);
                CHAIN_STAMP(t, 0);
                const bool full = cw0 + WIN <= nc;
                if (dep_pass) {
                    if (full) win_solve<true, true>(a, cw0, nc, rok, lane, S.Ct, S.Lb, S.dv, S.prog + w, prog + w, ds, pb);
                    else win_solve<false, true>(a, cw0, nc, rok, lane, S.Ct, S.Lb, S.dv, S.prog + w, prog + w, ds, pb);
                } else {
                    if (full) win_solve<true, false>(a, cw0, nc, rok, lane, S.Ct, S.Lb, S.dv, S.prog + w, prog + w, ds, pb);
                    else win_solve<false, false>(a, cw0, nc, rok, lane, S.Ct, S.Lb, S.dv, S.prog + w, prog + w, ds, pb);
                }
                __builtin_amdgcn_s_setprio(0);
                CHAIN_STAMP(t, 1);
            }
            CHAIN_STAMP(t, 2);
            __syncthreads();
            const bool tiny = S.tiny == passes;
            const bool spec = S.spec == passes;
            __syncthreads();
            CHAIN_STAMP(t, 3);
            if (!dep_pass && tiny && tv.dep) {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
                for (int q = 0; q < WIN; q++) a[q] = sc1_load(rc.save + PC * PC + (cw0 + q) * PC + lane);
                dep_pass = true;
                continue;
            }
            if (spec || (!dep_pass && tiny)) return;
            break;
        }
        // tile t + 1's rows of L, D of block t; the last half-1 wave whose
        // stores drained signals the step (pdone, and tile t + 1's rows)
        if (w < nwin && tile && rok) {
#pragma unroll
            for (int q = 0; q < WIN; q++) {
                const int c = cw0 + q;
                if (c < nc) sc1_store(panel + row + (size_t)c * nt, a[q]);
            }
        }
        if (wv == 4 && lane < nc) sc1_store(p.dg + c0 + lane, S.dv[lane]);
        if (wv == 5) C.dvp[lane] = S.dv[lane];
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        int last = 0;
        if (lane == 0) last = __hip_atomic_fetch_add(&C.arrive, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) == 4 * t + 3;
        if (__builtin_amdgcn_readfirstlane(last) && lane == 0) {
            if (tile) __hip_atomic_store(rc.rdone + t * ntb + t + 1, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_fetch_add(rc.pdone + t, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (t + 2 >= ntb) continue;
        // tile t + 2 after the visits minus block t's product L(t+2, t) W(t+1, t)':
        // its rows of block column t from the tile item (t, t + 2)
        const int k1 = k0 + PC, nc1 = min(PC, nt - k1);
        wave_poll(rc.rdone + t * ntb + t + 2, 1, rc.abort);
        const int r2 = (t + 2) * TR + lane;
        const bool ok2 = r2 < nt;
#pragma unroll
        for (int q = 0; q < WIN; q++) {
            const double x = sc1_load(tv.S + (ok2 ? r2 + (size_t)(k0 + cw0 + q) * nt : 0));
            C.T[cw0 + q][lane] = ok2 ? x : 0.0;
        }
        wave_poll(rc.vseq + (t + 2) * ntb + t + 1, (rc.novisit ? 0 : run_chunk_count(t + 1, tv.vk, rc.latest)), rc.abort);
        double st[WIN];
#pragma unroll
        for (int q = 0; q < WIN; q++) {
            const int c = cw0 + q;
            const bool ok = ok2 && c < nc1;
            const double x = sc1_load(tv.S + (ok ? r2 + (size_t)(k1 + c) * nt : 0));
            st[q] = ok ? x : 0.0;
        }
        half_sync(&C.hs[1], g1);       // T holds L(t + 2, t); dvp holds D of block t
        double4_t acc[4];
#pragma unroll
        for (int y = 0; y < 4; y++) acc[y] = (double4_t){0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int kk = 0; kk < PC; kk += 4) {
            const double av = C.T[kk + lk][w * 16 + li];
#pragma unroll
            for (int y = 0; y < 4; y++) {
                const double bv = S.Lb[kk + lk][y * 16 + li] * C.dvp[kk + lk];
                acc[y] = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc[y], 0, 0, 0);
            }
        }
        half_sync(&C.hs[1], g1);       // every operand read
#pragma unroll
        for (int y = 0; y < 4; y++)
#pragma unroll
            for (int i = 0; i < 4; i++) C.T[y * 16 + li][w * 16 + lk + 4 * i] = acc[y][i];
        half_sync(&C.hs[1], g1);
#pragma unroll
        for (int q = 0; q < WIN; q++) {
            const int c = cw0 + q;
            a[q] = (ok2 && c < nc1) ? st[q] - C.T[c][lane] : 0.0;
        }
    }
}

// the chain item (see above)
__device__ void chain_body(const PlanView& p, const TailView& tv, const ChainRun& rc, ChainLds& C) {
    const int tid = threadIdx.x;
    if (tid < 8) C.P.prog[tid] = 0;
    if (tid < 4) C.winok[tid] = 0;
    if (tid == 0) {
        C.P.tiny = 0;
        C.P.spec = 0;
        C.P.ndep = 0;
        C.hs[0] = C.hs[1] = 0;
        C.arrive = 0;
    }
    __syncthreads();
    if (__builtin_amdgcn_readfirstlane(tid >> 6) >= 4) chain_half1(p, tv, rc, C);
    else chain_half0(p, tv, rc, C);
}

// tile item (t, R), R >= t + 2: tile R's rows of block column t.  Waves 4-7
// solve it (k_panel_w's half 1) against the chain's published windows of
// block t, which waves 0-3 load into LDS as the chain publishes them; first
// block t - 1's update of the tile (k_tail_pr's pre-update, tile half: the
// same fragments, k ascending, old - acc).
__device__ __attribute__((noinline)) void chain_tile_body(const PlanView& p, const TailView& tv, const ChainRun& rc, int t, int R, char* lds,
                                int* sh) {
    PanelLds& S = *reinterpret_cast<PanelLds*>(lds);
    const int nt = tv.nt, ntb = tv.ntb, tid = threadIdx.x, lane = tid & 63;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const bool solver = wv >= 4;
    const int w = solver ? (wv + 2) & 3 : wv, cw0 = WIN * w;
    const int k0 = t * PC, c0 = tv.tc + k0;       // block t is full: a tile lies below it
    const int row = R * TR + lane;
    const bool rok = row < nt;
    const int li = lane & 15, lk = lane >> 4;
    // the visits of this tile are done: its entries
    if (!chain_wg_wait(rc.vseq + R * ntb + t, (rc.novisit ? 0 : run_chunk_count(t, tv.vk, rc.latest)), nullptr, 0, rc.abort, sh)) return;
    double a[WIN];
#pragma unroll
    for (int q = 0; q < WIN; q++) {
        const double x = sc1_load(tv.S + (solver && rok ? row + (size_t)(k0 + cw0 + q) * nt : 0));
        a[q] = solver && rok ? x : 0.0;
    }
    if (t > 0) {
        // block t - 1's update: the tile's rows of block column t - 1 (tile item
        // (t - 1, R)) and block t's (the chain), W = L D formed on the load
        if (!chain_wg_wait(rc.rdone + (t - 1) * ntb + R, 1, rc.rdone + (t - 1) * ntb + t, 1, rc.abort, sh + 1)) return;
        PreLds& P = *reinterpret_cast<PreLds*>(lds);
        const int kp = k0 - PC;
        const double* Lcol = tv.S + (size_t)kp * nt;
        constexpr int NU = TR * PC / PNT;
        double vj[NU], vw[NU];
        const int rr = tid % TR, rd = k0 + rr, rj = R * TR + rr;
        const bool okj = rj < nt;
#pragma unroll
        for (int u = 0; u < NU; u++) {
            const int k = (tid + u * PNT) / TR;
            const double x = sc1_load(Lcol + rd + (size_t)k * nt);
            const double y = sc1_load(Lcol + (okj ? rj + (size_t)k * nt : 0));
            const double dk = sc1_load(p.dg + tv.tc + kp + k);
            vj[u] = okj ? y : 0.0;
            vw[u] = x * dk;
        }
#pragma unroll
        for (int u = 0; u < NU; u++) {
            const int k = (tid + u * PNT) / TR;
            P.Aj[rr][k] = vj[u];
            P.Bs[rr][k] = vw[u];
        }
        __syncthreads();
        // 16 fragments over 8 waves: rows fx of the tile, columns fy, fy + 1 of W
        const int fx = wv & 3, fy0 = 2 * (wv >> 2);
        double4_t acc[2];
        acc[0] = acc[1] = (double4_t){0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int kk = 0; kk < PC; kk += 4) {
            const double av = P.Aj[fx * 16 + li][kk + lk];
#pragma unroll
            for (int y = 0; y < 2; y++)
                acc[y] = __builtin_amdgcn_mfma_f64_16x16x4f64(av, P.Bs[(fy0 + y) * 16 + li][kk + lk], acc[y], 0, 0, 0);
        }
        __syncthreads();
#pragma unroll
        for (int y = 0; y < 2; y++)
#pragma unroll
            for (int i = 0; i < 4; i++) P.Ad[(fy0 + y) * 16 + li][fx * 16 + lk + 4 * i] = acc[y][i];
        __syncthreads();
        if (solver && rok) {
#pragma unroll
            for (int q = 0; q < WIN; q++) a[q] = a[q] - P.Ad[cw0 + q][lane];
        }
        __syncthreads();           // the panel's LDS image overwrites P from here
    }
    if (tid < 8) S.prog[tid] = 0;
    if (tid == 0) S.spec = 0;
    if (tid == 8) S.tiny = 0;      // here: the launch aborted while this item waited for a window
    __syncthreads();
    DepState ds{p.sign + c0, S.lv, &S.spec, 0};
    if (!solver) {
        // window w of block t, as the chain publishes it (after an abort: the
        // window is marked and the solve runs on, so that every wave ends)
        const bool ok = wave_poll(rc.dwin + t * 4 + w, 1, rc.abort);
        const double* src = rc.dpub + ((size_t)t * 4 + w) * kChainWinPub;
        double v[WIN];
#pragma unroll
        for (int kk = 0; kk < WIN; kk++) v[kk] = ok ? sc1_load(src + kk * PC + lane) : 0.0;
        double dd = 1.0, mk = 1.0;
        if (ok && lane < WIN) {
            dd = sc1_load(src + WIN * PC + lane);
            mk = sc1_load(src + WIN * PC + WIN + lane);
        }
#pragma unroll
        for (int kk = 0; kk < WIN; kk++) S.Ct[cw0 + kk][lane] = v[kk];
        if (lane < WIN) {
            S.dv[cw0 + lane] = dd;
            S.lv[cw0 + lane] = static_cast<int>(mk);
        }
        if (!ok && lane == 0) S.tiny = 1;
        df_publish(S.prog + w, WIN);
    } else {
        double unused = 0.0;
        for (int t2 = 0; t2 < w; t2++) win_apply<false>(a, unused, WIN * t2, lane, cw0, S.Ct, S.Lb, S.prog + 4 + t2);
        win_solve<true, true>(a, cw0, PC, rok, lane, S.Ct, S.Lb, S.dv, S.prog + w, S.prog + 4 + w, ds);
    }
    __syncthreads();
    if (S.tiny) return;                 // the launch aborted: nothing of it is used
    if (S.spec) {                        // a tile entry contradicts a dropped column
        if (tid == 0) chain_abort(p, rc.abort);
        return;
    }
    if (solver && rok) {
#pragma unroll
        for (int q = 0; q < WIN; q++) sc1_store(tv.S + row + (size_t)(k0 + cw0 + q) * nt, a[q]);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
        __hip_atomic_store(rc.rdone + t * ntb + R, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_fetch_add(rc.pdone + t, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

__global__ void __launch_bounds__(PNT)
k_tail_chain_run(PlanView p, TailView tv, ChainRun rc) {
    __shared__ __attribute__((aligned(16))) char lds[kChainItemLds];
    __shared__ int sh_item, sh_ok[2];
    const int ntb = tv.ntb;
    if (threadIdx.x == 0) sh_item = __hip_atomic_fetch_add(rc.ticket, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    const int it = sh_item;
    if (it >= rc.n) return;
    const uint2 rec = rc.items[it];
    const int t = rec.y & 0xff, q = (rec.y >> 8) & 0xff;
    unsigned long long* tr = rc.trace ? rc.trace + 4 * (size_t)it : nullptr;
    if (tr && threadIdx.x == 0) {
        tr[0] = __builtin_amdgcn_s_memrealtime();
        tr[3] = __builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (3 << 11));
    }
    if (rec.y & (1u << 30)) {
        chain_body(p, tv, rc, *reinterpret_cast<ChainLds*>(lds));
    } else if (rec.y >> 31) {
        if (tr && threadIdx.x == 0) tr[1] = __builtin_amdgcn_s_memrealtime();
        chain_tile_body(p, tv, rc, t, static_cast<int>(rec.x), lds, sh_ok);
    } else {
        const int bi = rec.x & 255, c = (rec.x >> 8) & 255, b0 = (rec.x >> 16) & 255, b1 = rec.x >> 24;
        int* vs = rc.vseq + bi * ntb + c;
        if (!chain_wg_wait(t > 0 ? rc.pdone + t - 1 : nullptr, t > 0 ? chain_target(ntb, t - 1) : 0, q ? vs : nullptr,
                           q, rc.abort, sh_ok))
            return;
        if (tr && threadIdx.x == 0) tr[1] = __builtin_amdgcn_s_memrealtime();
        visit_tile512<true>(p, tv, bi, c, b0, b1, *reinterpret_cast<SyrkLds*>(lds));
        run_signal(vs);
    }
    if (tr && threadIdx.x == 0) tr[2] = __builtin_amdgcn_s_memrealtime();
}

// A DEP pass of block column kb failed its check in some workgroup (flags[1]
// bit 16) after others had written: put back the tile rows and the block's
// |terms| it saved in tv.W and the dependent pivots workgroup 0 added, so the
// host repair starts from the column as the look-ahead left it.
__global__ void __launch_bounds__(256)
k_tail_restore(PlanView p, TailView tv, int kb) {
    const int nt = tv.nt, k0 = kb * PC, nc = min(PC, nt - k0), h = nt - k0, c = blockIdx.y;
    double* panel = tv.S + k0 + (size_t)k0 * nt;
    for (int row = nc + blockIdx.x * 256 + threadIdx.x; row < h; row += gridDim.x * 256)
        panel[row + (size_t)c * nt] = tv.W[row + (size_t)c * nt];
    if (blockIdx.x == 0 && c == 0) {
        if ((int)threadIdx.x < nc) p.dscale[tv.tc + k0 + threadIdx.x] = tv.W[threadIdx.x];
        if (threadIdx.x == 0) {
            p.flags[0] -= p.flags[3];
            p.flags[3] = 0;
        }
    }
}

// Block t's update of block column t + 1 only (tiles (bi, t + 1), bi > t):
// what the look-ahead panel of step t + 1 applies to its own rows, for the
// repair path that resumes the look-ahead after a dependent pivot.
__global__ void __launch_bounds__(PNT)
k_tail_col(PlanView p, TailView tv, int t) {
    __shared__ __attribute__((aligned(16))) char lds[sizeof(SyrkLds)];
    syrk_tile512(p, tv, t, t + 1 + blockIdx.x, t + 1, *reinterpret_cast<SyrkLds*>(lds));
}

// ------------------------------------------------------- small panels
// Supernodes with at most 16 columns and 64 rows (the bulk of the bottom
// levels): one wave each, four per workgroup, no barrier and no LDS.  Lane
// r keeps row r, columns 0..15 in registers; column step k: pivot and its
// |terms| by v_readlane, l = a / d_k below the diagonal, c_r = l d_k, and
// a_r(q) -= l c_q with c_q by v_readlane -- the operations and order of
// factor_diag_fast per entry (bitwise the same factor).  A pivot that fails
// the zero test stops the wave before it writes anything and raises
// flags[1], as the other fused kernels.
constexpr int SNC = 16;

__device__ __forceinline__ void panel_s_body(const PlanView& p, const int* __restrict__ sups, int q0, int q, int dep) {
    const int lane = threadIdx.x & 63;
    const int s = sups[q0 + q];
    const int c0 = p.col0[s], nc = p.col0[s + 1] - c0;
    const int h = nc + (p.rowptr[s + 1] - p.rowptr[s]), ld = h;
    double* panel = p.Lx + p.off[s];
    const bool rok = lane < h;
    double a[SNC];
#pragma unroll
    for (int c = 0; c < SNC; c++) {
        const bool ok = rok && c < nc && c <= lane;
        const double t = panel[ok ? lane + (size_t)c * ld : 0];
        a[c] = ok ? t : 0.0;
    }
    double dsc = lane < nc ? p.dscale[c0 + lane] : 0.0;
    double mydv = 0.0;
    int mylive = 1, ndep = 0;
#pragma unroll
    for (int k = 0; k < SNC; k++) {
        if (k < nc) {
            double dk = lane_bcast(a[k], k);
            const double dsk = lane_bcast(dsc, k);
            int alive = 1;
            if (fabs(dk) <= p.tau * dsk) {          // wave-uniform
                // ldlt.c:600-614: every row of the column is in this wave
                // (the supernode's rows and R_s), so the largest entry below
                // the pivot decides here: +-1e-8 by node class if it reaches
                // 1e-2, else the column is dropped; a NaN (whose place in the
                // reference's max fold matters) goes to the redo
                const bool in = lane > k && rok;
                const bool nan = __ballot(in && a[k] != a[k]) != 0;
                if (!dep || nan) {
                    if (lane == 0) atomicOr(&p.flags[1], 8);
                    return;
                }
                if (__ballot(in && !(fabs(a[k]) < 1.0e+6 * 1.0e-8)) != 0) dk = (p.sign[c0 + k] < 0 ? -1.0 : 1.0) * 1.0e-8;
                else alive = 0;
                ndep++;
            }
            mylive = lane == k ? alive : mylive;
            const bool below = lane > k && rok;
            const double l = alive && below ? a[k] / dk : 0.0;     // a dropped column's L is 0
            a[k] = below ? l : a[k];
            mydv = lane == k ? dk : mydv;
            const double c = l * dk;
            dsc = dsc + fabs(l * c);
#pragma unroll
            for (int qq = k + 1; qq < SNC; qq++)
                if (qq < nc) a[qq] = a[qq] - l * lane_bcast(c, qq);
        }
    }
    // rows of R_s: L21; rows of the block: L11' into the upper slot
    if (rok) {
#pragma unroll
        for (int c = 0; c < SNC; c++) {
            if (c < nc && lane >= nc) panel[lane + (size_t)c * ld] = a[c];
            else if (c < lane && lane < nc) panel[c + (size_t)lane * ld] = a[c];
        }
    }
    if (lane < nc) { p.dg[c0 + lane] = mydv; p.live[c0 + lane] = mylive; }
    if (ndep && lane == 0) atomicAdd(&p.flags[0], ndep);
}

__global__ void __launch_bounds__(256)
k_panel_s(PlanView p, const int* __restrict__ sups, int q0, int count, int dep) {
    const int q = blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (q >= count) return;
    panel_s_body(p, sups, q0, q, dep);
}

// A sparse level's fused panel units (workgroups [0, nfu): k_panel_w's
// work) and its small panels (the rest: eight per workgroup, one a wave,
// k_panel_s's work) in one launch: the level chain of a problem like
// dfl001 is a sequence of small latency-bound launches, and the two
// kernels of a level are independent.  The same bodies, so bitwise.
__global__ void __launch_bounds__(PNT)
k_panel_ws(PlanView p, const int* __restrict__ fu_sup, const int* __restrict__ fu_j, int f0, int nfu, TailView tv,
           const int* __restrict__ ssups, int s0, int nsm, int dep) {
    __shared__ __attribute__((aligned(16))) char lds[sizeof(PanelLds)];
    if (static_cast<int>(blockIdx.x) >= nfu) {
        const int q = (blockIdx.x - nfu) * (PNT / 64) + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
        if (q < nsm) panel_s_body(p, ssups, s0, q, dep);
        return;
    }
    PanelLds& S = *reinterpret_cast<PanelLds*>(lds);
    const int sdep = tv.sdep ? 1 : 0;
    if (panel_w_body<false>(p, fu_sup, fu_j, f0, tv, -1, blockIdx.x, S, tv.W, false, nullptr, 0, sdep)) {
        __syncthreads();
        panel_w_body<true>(p, fu_sup, fu_j, f0, tv, -1, blockIdx.x, S, tv.W, false, nullptr, 0, sdep);
    }
}

// Single-column small panels with at most 8 rows (the x-node leaves of a
// large LP, 10^6 on configs[3]) eight to a wave, lanes 8q .. 8q + 7 for
// panel q: k_panel_s's nc = 1 step lane for lane (the pivot and its |terms|
// from the group's lane 0, the zero test, the dependent-pivot rule over the
// group's rows, l = a / d below it), so bitwise the same factor.  A group
// that bails stores nothing, as k_panel_s's wave.
constexpr int kPanel1Rows = 8;

__global__ void __launch_bounds__(256)
k_panel_s1(PlanView p, const int* __restrict__ sups, int q0, int count, int dep) {
    const int lane = threadIdx.x & 63, lq = lane & (kPanel1Rows - 1), gb = lane & ~(kPanel1Rows - 1);
    const int q = (blockIdx.x * 256 + threadIdx.x) / kPanel1Rows;
    if (q >= count) return;           // whole groups leave together
    const int s = sups[q0 + q];
    const int c0 = p.col0[s];
    const int h = 1 + (p.rowptr[s + 1] - p.rowptr[s]);
    double* panel = p.Lx + p.off[s];
    const bool rok = lq < h;
    const double a = rok ? panel[lq] : 0.0;
    const double dsc = lq == 0 ? p.dscale[c0] : 0.0;
    double dk = __shfl(a, 0, kPanel1Rows);
    const double dsk = __shfl(dsc, 0, kPanel1Rows);
    int alive = 1, ndep = 0;
    const unsigned long long gmask = 0xffull << gb;
    if (fabs(dk) <= p.tau * dsk) {                 // group-uniform
        const bool in = lq > 0 && rok;
        const bool nan = (__ballot(in && a != a) & gmask) != 0;
        if (!dep || nan) {
            if (lq == 0) atomicOr(&p.flags[1], 8);
            return;
        }
        if ((__ballot(in && !(fabs(a) < 1.0e+6 * 1.0e-8)) & gmask) != 0) dk = (p.sign[c0] < 0 ? -1.0 : 1.0) * 1.0e-8;
        else alive = 0;
        ndep++;
    }
    const bool below = lq > 0 && rok;
    const double l = alive && below ? a / dk : 0.0;     // a dropped column's L is 0
    if (below) panel[lq] = l;
    if (lq == 0) {
        p.dg[c0] = dk;
        p.live[c0] = alive;
        if (ndep) atomicAdd(&p.flags[0], ndep);
    }
}

}  // namespace

int tail_visit_tiles(int ntb, int t, int K) {
    int n = 0;
    for (int c = t + 1; c < ntb && visit_hi(t, c, K) > 0; c++) n += ntb - c;
    return t > 0 ? n : 0;
}

// Launch t runs panel t on gp(t) workgroups beside its visits; with one
// workgroup per CU (the kernel's LDS) a launch of more than `cap` workgroups
// takes two rounds of visits: on dfl001 launches 21-37 under visit_hi's
// chunks (up to 286 workgroups, 37-47 us against ~30).  Those launches carry
// the first chunks of later columns' tiles (blocks 0 .. b1 - 1 with b1 <= 6),
// which are ready from launch b1 on: moved, latest-first, into the latest
// earlier launch with room.  Every tile keeps its chunks and their order (its
// first chunk only comes earlier), so the factor is bitwise the same.
std::vector<unsigned> tail_visit_schedule(int ntb, int nt, int K, int cap, std::vector<int>& ptr) {
    struct V { int bi, c, b0, b1; };
    std::vector<std::vector<V>> L(ntb);
    std::vector<int> tot(ntb, 0);
    for (int t = 0; t < ntb; t++) {
        const int h = nt - t * PC;
        tot[t] = std::max(1, (h + TR - 1) / TR - 1);          // launch_tail_step's panel workgroups
        if (t == 0) continue;
        for (int c = t + 1; c < ntb && visit_hi(t, c, K) > 0; c++) {
            const int b1 = visit_hi(t, c, K), b0 = std::max(0, b1 - K);
            for (int bi = c; bi < ntb; bi++) L[t].push_back({bi, c, b0, b1});
        }
        tot[t] += static_cast<int>(L[t].size());
    }
    for (int t = ntb - 1; t > 1; t--) {
        while (tot[t] > cap) {
            // a first chunk of this launch, the one ready earliest (then the
            // farthest column: its tiles have the longest wait before their
            // panel anyway)
            int best = -1;
            for (int q = 0; q < static_cast<int>(L[t].size()); q++) {
                const V& v = L[t][q];
                if (v.b0 != 0) continue;
                if (best < 0 || v.b1 < L[t][best].b1 || (v.b1 == L[t][best].b1 && v.c > L[t][best].c)) best = q;
            }
            if (best < 0) break;
            int dst = -1;
            for (int u = t - 1; u >= std::max(1, L[t][best].b1); u--)
                if (tot[u] < cap) { dst = u; break; }
            if (dst < 0) break;
            L[dst].push_back(L[t][best]);
            tot[dst]++;
            L[t].erase(L[t].begin() + best);
            tot[t]--;
        }
    }
    // XCD grouping (speed only, never correctness): workgroups b and b + 8
    // share an XCD and its L2 (MI355X_MICROARCH.md, round-robin placement),
    // and every visit of column c reads the same blocks L(c, b0 .. b1 - 1)
    // (the B operand, W = L D): the visits of column c go to workgroup ids of
    // one residue mod 8 where possible, so those blocks come from one L2
    std::vector<unsigned> out;
    ptr.assign(ntb + 1, 0);
    const bool xcd = !std::getenv("IPO_HIP_VISIT_XCD") || std::atoi(std::getenv("IPO_HIP_VISIT_XCD")) != 0;
    for (int t = 0; t < ntb; t++) {
        ptr[t] = static_cast<int>(out.size());
        std::vector<V> order;
        if (xcd && !L[t].empty()) {
            const int gp = tot[t] - static_cast<int>(L[t].size());
            std::vector<std::vector<V>> q(8);
            for (const V& v : L[t]) q[v.c % 8].push_back(v);
            std::vector<size_t> head(8, 0);
            for (size_t e = 0; e < L[t].size(); e++) {
                int x = (gp + static_cast<int>(e)) % 8;
                if (head[x] == q[x].size()) {           // this residue's columns are used up: the fullest other
                    size_t best = 0;
                    for (int y = 0; y < 8; y++)
                        if (q[y].size() - head[y] > best) { best = q[y].size() - head[y]; x = y; }
                }
                order.push_back(q[x][head[x]++]);
            }
        } else {
            order = L[t];
        }
        for (const V& v : order)
            out.push_back(static_cast<unsigned>(v.bi) | static_cast<unsigned>(v.c) << 8 |
                          static_cast<unsigned>(v.b0) << 16 | static_cast<unsigned>(v.b1) << 24);
    }
    ptr[ntb] = static_cast<int>(out.size());
    return out;
}

// Chunks of column c of the persistent tail, latest first: blocks [0, c - 1)
// (block c - 1 is its panel's pre-update), the latest L blocks one chunk (a
// visit that must finish within one step: it needs block c - 2, final at the
// end of step c - 2, before panel c), then K at a time downwards.
static std::vector<std::pair<int, int>> run_chunks(int c, int K, int L) {
    std::vector<std::pair<int, int>> v;
    int b1 = c - 1;
    for (int k = 0; b1 > 0; k++) {
        const int b0 = std::max(0, b1 - (k == 0 ? L : K));
        v.push_back({b0, b1});
        b1 = b0;
    }
    return v;
}

std::vector<uint2> tail_run_schedule(int ntb, int nt, int K, int L, int cap, std::vector<int>& ptr) {
    struct V { int bi, c, b0, b1, q; };
    std::vector<std::vector<V>> Ls(ntb);
    std::vector<int> tot(ntb, 0), nch(ntb, 0);
    for (int c = 0; c < ntb; c++) {
        const std::vector<std::pair<int, int>> ch = run_chunks(c, K, L);
        nch[c] = static_cast<int>(ch.size());
        // the k-th chunk from the top in launch c - 1 - k (its blocks < b1 <= c - 1 - k)
        for (int k = 0; k < nch[c]; k++)
            for (int bi = c; bi < ntb; bi++) Ls[c - 1 - k].push_back({bi, c, ch[k].first, ch[k].second, nch[c] - 1 - k});
    }
    for (int t = 0; t < ntb; t++) tot[t] = tail_gp(nt, t) + static_cast<int>(Ls[t].size());
    // launches over `cap` items: first chunks (q = 0) into the latest earlier
    // launch with room where they are ready (launch >= b1), as tail_visit_schedule
    for (int t = ntb - 1; t > 1; t--) {
        while (tot[t] > cap) {
            int best = -1;
            for (int i = 0; i < static_cast<int>(Ls[t].size()); i++) {
                const V& v = Ls[t][i];
                if (v.q != 0) continue;
                if (best < 0 || v.b1 < Ls[t][best].b1 || (v.b1 == Ls[t][best].b1 && v.c > Ls[t][best].c)) best = i;
            }
            if (best < 0) break;
            int dst = -1;
            for (int u = t - 1; u >= std::max(1, Ls[t][best].b1); u--)
                if (tot[u] < cap) { dst = u; break; }
            if (dst < 0) break;
            Ls[dst].push_back(Ls[t][best]);
            tot[dst]++;
            Ls[t].erase(Ls[t].begin() + best);
            tot[t]--;
        }
    }
    std::vector<uint2> out;
    ptr.assign(ntb + 1, 0);
    for (int t = 0; t < ntb; t++) {
        ptr[t] = static_cast<int>(out.size());
        for (int j = 0; j < tail_gp(nt, t); j++)
            out.push_back(make_uint2(static_cast<unsigned>(j), static_cast<unsigned>(t) |
                                                                  static_cast<unsigned>(nch[t]) << 8 | 1u << 31));
        // column t + 1's visits first (its panel waits for them), then by column
        std::vector<V>& vv = Ls[t];
        std::stable_sort(vv.begin(), vv.end(), [t](const V& a, const V& b) {
            const bool ua = a.c == t + 1, ub = b.c == t + 1;
            if (ua != ub) return ua;
            return a.c != b.c ? a.c < b.c : a.bi < b.bi;
        });
        for (const V& v : vv)
            out.push_back(make_uint2(static_cast<unsigned>(v.bi) | static_cast<unsigned>(v.c) << 8 |
                                         static_cast<unsigned>(v.b0) << 16 | static_cast<unsigned>(v.b1) << 24,
                                     static_cast<unsigned>(t) | static_cast<unsigned>(v.q) << 8));
    }
    ptr[ntb] = static_cast<int>(out.size());
    return out;
}

// Items of k_tail_chain_run: the chain item first, then per launch t the
// tile items (t, R), R = t + 2 .. ntb - 1 (R = t + 2 first: the chain waits
// for it), then launch t's visits as tail_run_schedule places them, with
// room for the chain's CU.
std::vector<uint2> tail_chain_schedule(int ntb, int nt, int K, int L, int cap, std::vector<int>& ptr) {
    std::vector<int> rptr;
    const std::vector<uint2> run = tail_run_schedule(ntb, nt, K, L, cap - 1, rptr);
    std::vector<uint2> out;
    out.push_back(make_uint2(0u, 1u << 30));
    ptr.assign(ntb + 1, 0);
    for (int t = 0; t < ntb; t++) {
        ptr[t] = static_cast<int>(out.size());
        for (int R = t + 2; R < ntb; R++) out.push_back(make_uint2(static_cast<unsigned>(R), static_cast<unsigned>(t) | 1u << 31));
        for (int i = rptr[t]; i < rptr[t + 1]; i++)
            if (!(run[i].y >> 31)) out.push_back(run[i]);          // the visits (panels are the chain's now)
    }
    ptr[ntb] = static_cast<int>(out.size());
    return out;
}

void launch_tail_chain(const PlanView& pv, const TailView& tv, const ChainRun& rc, hipStream_t s) {
    if (rc.n > 0) hipLaunchKernelGGL(k_tail_chain_run, dim3(rc.n), dim3(PNT), 0, s, pv, tv, rc);
}

void launch_tail_run(const PlanView& pv, const TailView& tv, const TailRun& rc, hipStream_t s) {
    if (rc.n > 0) hipLaunchKernelGGL(k_tail_run, dim3(rc.n), dim3(PNT), 0, s, pv, tv, rc);
}

void tail_visit_work(int ntb, int nt, int K, double& flops, double& bytes) {
    flops = bytes = 0.0;
    for (int t = 1; t < ntb; t++)
        for (int c = t + 1; c < ntb && visit_hi(t, c, K) > 0; c++) {
            const int b1 = visit_hi(t, c, K), b0 = std::max(0, b1 - K);
            for (int bi = c; bi < ntb; bi++) {
                const double rows = std::min(TR, nt - bi * TR), cols = std::min(TR, nt - c * TR);
                for (int b = b0; b < b1; b++) {
                    const double k = std::min(PC, nt - b * PC);
                    flops += 2.0 * rows * cols * k;
                    bytes += 8.0 * k * (rows + cols);          // L rows of bi and of c (W = L D formed on load)
                }
                bytes += 16.0 * rows * cols;                   // one read-modify-write of the tile
            }
        }
}

void launch_tail_step(const PlanView& pv, const TailView& tv, int t, hipStream_t s) {
    const int h = tv.nt - t * PC;
    const int gp = std::max(1, (h + TR - 1) / TR - 1);
    const int nr = tv.vlist ? tv.vptr[t + 1] - tv.vptr[t] : tail_visit_tiles(tv.ntb, t, tv.vk);
    hipLaunchKernelGGL(k_tail_pr, dim3(gp + nr), dim3(PNT), 0, s, pv, tv, t, gp, tv.vlist ? tv.vptr[t] : 0);
}

void launch_tail_restore(const PlanView& pv, const TailView& tv, int kb, hipStream_t s) {
    const int nc = std::min(PC, tv.nt - kb * PC), rows = tv.nt - kb * PC - nc;
    hipLaunchKernelGGL(k_tail_restore, dim3(std::max(1, std::min(64, (rows + 255) / 256)), nc), dim3(256), 0, s, pv, tv,
                       kb);
}

void launch_tail_colupdate(const PlanView& pv, const TailView& tv, int t, hipStream_t s) {
    if (tv.ntb - t - 1 > 0) hipLaunchKernelGGL(k_tail_col, dim3(tv.ntb - t - 1), dim3(PNT), 0, s, pv, tv, t);
}

int tail_dep_tiles(const TailView& tv, int kb) {
    const int below = tv.nt - kb * PC - std::min(PC, tv.nt - kb * PC);
    return std::max(1, (below + TR - 1) / TR);
}

size_t tail_dep_state_doubles(int ntb) { return 2 * (kDepState + static_cast<size_t>(std::max(1, ntb))); }

void launch_tail_dep_round(const PlanView& pv, const TailView& tv, int kb, int round, double* st, int* sti,
                           hipStream_t s) {
    const size_t half = tail_dep_state_doubles(tv.ntb) / 2;
    const int in = round & 1, out = in ^ 1;
    hipLaunchKernelGGL(k_tail_dep, dim3(tail_dep_tiles(tv, kb)), dim3(NT), 0, s, pv, tv, kb, st + in * half,
                       st + out * half, sti + 4 * in, sti + 4 * out);
}

void launch_panel_small(const PlanView& pv, const int* sups, int q0, int count, int dep, hipStream_t s, int n1) {
    if (n1 > 0)
        hipLaunchKernelGGL(k_panel_s1, dim3((n1 + 256 / kPanel1Rows - 1) / (256 / kPanel1Rows)), dim3(256), 0, s, pv,
                           sups, q0, n1, dep);
    if (count > n1)
        hipLaunchKernelGGL(k_panel_s, dim3((count - n1 + 3) / 4), dim3(256), 0, s, pv, sups, q0 + n1, count - n1, dep);
}

void launch_panel_ws(const PlanView& pv, const int* fu_sup, const int* fu_j, int f0, int nfu, const TailView& tv,
                     const int* ssups, int s0, int nsm, int dep, hipStream_t s) {
    hipLaunchKernelGGL(k_panel_ws, dim3(nfu + (nsm + PNT / 64 - 1) / (PNT / 64)), dim3(PNT), 0, s, pv, fu_sup, fu_j, f0,
                       nfu, tv, ssups, s0, nsm, dep);
}

void launch_panel(const PlanView& pv, const int* fu_sup, const int* fu_j, int f0, int count, const TailView& tv,
                  int kb, hipStream_t s) {
    // kb < 0: fused units of a sparse level (whose list pointer is null when
    // the problem has none, so the pointer cannot tell the modes apart)
    if (kb < 0) {
        if (count <= 0) return;
        if (!fu_sup || !fu_j) throw std::runtime_error("launch_panel: sparse units without a unit list");
        hipLaunchKernelGGL(k_panel_w, dim3(count), dim3(PNT), 0, s, pv, fu_sup, fu_j, f0, tv, -1);
    } else {
        const int h = tv.nt - kb * PC;
        const int g = std::max(1, (h + TR - 1) / TR - 1);
        hipLaunchKernelGGL(k_panel_w, dim3(g), dim3(PNT), 0, s, pv, nullptr, nullptr, 0, tv, kb);
    }
}

void launch_diag(const PlanView& pv, const int* level_sups, int q0, int count, const TailView& tv, int kb,
                 hipStream_t s) {
    hipLaunchKernelGGL(k_diag, dim3(level_sups ? count : 1), dim3(NT), 0, s, pv, level_sups, q0, tv, kb);
}

void launch_trsm(const PlanView& pv, int u0, int count, const TailView& tv, int kb, hipStream_t s) {
    if (count >= 0) {
        hipLaunchKernelGGL(k_trsm, dim3(count), dim3(NT), 0, s, pv, u0, tv, -1);
    } else {
        const int below = tv.nt - kb * PC - min(PC, tv.nt - kb * PC);
        if (below > 0) hipLaunchKernelGGL(k_trsm, dim3((below + TR - 1) / TR), dim3(NT), 0, s, pv, 0, tv, kb);
    }
}

}  // namespace ipo
