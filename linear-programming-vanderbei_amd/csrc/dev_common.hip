// dev_common.hip -- deterministic multi-job reductions (see dev_common.h).
#include "dev_common.h"

#include <algorithm>
#include <cstdlib>
#include <stdexcept>
#include <vector>
#include "hip_util.h"

namespace ipo {

__global__ void __launch_bounds__(kRedThreads)
k_reduce_jobs(RedJobs jobs, double* __restrict__ part) {
    __shared__ double sh[4];
    for (int j = 0; j < jobs.nj; j++) {
        const double* a = jobs.a[j];
        const double* b = jobs.b[j];
        const int len = jobs.len[j];
        const int op = jobs.op[j];
        double acc = op == 0 ? 0.0 : (op == 2 ? 0.0 : 0.0);
        for (int i = blockIdx.x * kRedThreads + threadIdx.x; i < len; i += kRedBlocks * kRedThreads) {
            if (op == 0) acc += a[i] * b[i];
            else if (op == 1) acc = fmax(acc, ref_abs(a[i]));
            else acc = fmax(acc, -a[i] / b[i]);      // NaN ratios are ignored like hsd.c:249-258
        }
        const double r = op == 0 ? block_sum(acc, sh) : block_max(acc, sh);
        if (threadIdx.x == 0) part[j * kRedBlocks + blockIdx.x] = r;
    }
}

__global__ void __launch_bounds__(kRedThreads)
k_finish_reduce(const double* __restrict__ part, int nq, unsigned maxmask, double* __restrict__ out) {
    __shared__ double sh[4];
    for (int q = 0; q < nq; q++) {
        const bool mx = (maxmask >> q) & 1u;
        double v = part[q * kRedBlocks + threadIdx.x];   // kRedBlocks == kRedThreads
        const double r = mx ? block_max(v, sh) : block_sum(v, sh);
        if (threadIdx.x == 0) out[q] = r;
    }
}

// k_finish_reduce, then the nf ints at f copied into the doubles at outi
// (one launch for a read-back's scalars and flags)
__global__ void __launch_bounds__(kRedThreads)
k_finish_reduce_pack(const double* __restrict__ part, int nq, unsigned maxmask, double* __restrict__ out,
                     const int* __restrict__ f, int nf, double* __restrict__ outi) {
    __shared__ double sh[4];
    for (int q = 0; q < nq; q++) {
        const bool mx = (maxmask >> q) & 1u;
        double v = part[q * kRedBlocks + threadIdx.x];
        const double r = mx ? block_max(v, sh) : block_sum(v, sh);
        if (threadIdx.x == 0) out[q] = r;
    }
    if (static_cast<int>(threadIdx.x) < nf) reinterpret_cast<int*>(outi)[threadIdx.x] = f[threadIdx.x];
}

// dotprod() of linalg.c:17-25 in its own order: one running sum, i = 0..n-1.
// One 256-thread block per job: one wave forms a chunk's products (eight
// loads in flight per lane) and compacts them into LDS while one lane adds
// the previous chunk's in index order, its LDS reads one 16-value batch
// ahead of the adds, so that only the dependent adds remain on the chain.
// Max-type jobs are order-free.
constexpr int kOrdThreads = 256;

__global__ void __launch_bounds__(kOrdThreads)
k_reduce_ordered(RedJobs jobs, double* __restrict__ out) {
    const int j = blockIdx.x;
    const double* a = jobs.a[j];
    const double* b = jobs.b[j];
    const int len = jobs.len[j];
    const int op = jobs.op[j];
    const int tid = threadIdx.x;
    if (job_segmented(jobs, j)) return;     // k_dot_segments / k_dot_finish (launch_reduce)
    if (op != 0) {
        // maxima are order-free: eight loads in flight per thread
        __shared__ double sh[4];
        double acc = 0.0;
        for (int i0 = 0; i0 < len; i0 += 8 * kOrdThreads) {
            double va[8], vb[8];
#pragma unroll
            for (int u = 0; u < 8; u++) {
                const int i = i0 + u * kOrdThreads + tid;
                va[u] = i < len ? a[i] : 0.0;
                vb[u] = op == 2 && i < len ? b[i] : 1.0;
            }
#pragma unroll
            for (int u = 0; u < 8; u++) {
                if (i0 + u * kOrdThreads + tid >= len) continue;
                if (op == 1) acc = fmax(acc, ref_abs(va[u]));
                else acc = fmax(acc, -va[u] / vb[u]);
            }
        }
        acc = block_max(acc, sh);
        if (tid == 0) out[j] = acc;
        return;
    }
    // Zero products leave the running sum unchanged: it starts at +0, and a
    // sum of round-to-nearest adds is never -0 unless it adds -0 to -0, so
    // s + (+-0) == s at every step.  Wave 1 forms each chunk's products and
    // compacts the non-zero ones in index order (a ballot per 64 products,
    // no block barrier) into one of two LDS buffers, while lane 0 of wave 0
    // adds the previous chunk's: the same sum, bit for bit (NaN products
    // are not zero and stay), over half the chain on dfl001's b'y and c'x
    // (27 / 51 % of b / c non-zero), the forming of chunk k + 1 under the
    // adds of chunk k.  Hand-offs through LDS words (ready: chunk k + 1
    // written, freed: chunk k added), release / acquire at workgroup scope.
    constexpr int CH = 4096;
    __shared__ __attribute__((aligned(16))) double comp[2][CH + 16];   // + one batch of read-ahead
    __shared__ int nzc[2], ready[2], freed[2];
    if (tid < 2) {
        ready[tid] = 0;
        freed[tid] = 0;
    }
    __syncthreads();
    const int nch = (len + CH - 1) / CH, lane = tid & 63, wv = tid >> 6;
    if (wv == 1) {
        for (int k = 0; k < nch; k++) {
            const int buf = k & 1;
            if (k >= 2)
                while (__hip_atomic_load(&freed[buf], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < k - 1)
                    __builtin_amdgcn_s_sleep(1);
            const int base = k * CH, cnt = min(CH, len - base);
            int off = 0;
            for (int i0 = 0; i0 < cnt; i0 += 8 * 64) {
                double pa[8], pb[8];
#pragma unroll
                for (int u = 0; u < 8; u++) {
                    const int i = i0 + u * 64 + lane;
                    pa[u] = i < cnt ? a[base + i] : 0.0;
                    pb[u] = i < cnt ? b[base + i] : 0.0;
                }
#pragma unroll
                for (int u = 0; u < 8; u++) {
                    const double v = pa[u] * pb[u];
                    const bool nzf = i0 + u * 64 + lane < cnt && v != 0.0;
                    const unsigned long long m = __ballot(nzf);
                    if (nzf) comp[buf][off + __popcll(m & ((1ull << lane) - 1ull))] = v;
                    off += __popcll(m);
                }
            }
            if (lane == 0) {
                nzc[buf] = off;
                __hip_atomic_store(&ready[buf], k + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
        }
        return;
    }
    if (tid != 0) return;
    double s = 0.0e0;
    for (int k = 0; k < nch; k++) {
        const int buf = k & 1;
        while (__hip_atomic_load(&ready[buf], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < k + 1)
            __builtin_amdgcn_s_sleep(1);
        const int nz = nzc[buf];
        const double2* pp = reinterpret_cast<const double2*>(comp[buf]);
        double2 cur[8];
#pragma unroll
        for (int u = 0; u < 8; u++) cur[u] = pp[u];
        int i = 0;
        for (; i + 16 <= nz; i += 16) {
            double2 nxt[8];
#pragma unroll
            for (int u = 0; u < 8; u++) nxt[u] = pp[(i + 16) / 2 + u];
#pragma unroll
            for (int u = 0; u < 8; u++) { s += cur[u].x; s += cur[u].y; }
#pragma unroll
            for (int u = 0; u < 8; u++) cur[u] = nxt[u];
        }
        for (; i < nz; i++) s += comp[buf][i];
        __hip_atomic_store(&freed[buf], k + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    out[j] = s;
}

// Test entry (ipo_hip_dot_ordered): the ordered dot of two host vectors
// through launch_reduce, on the default stream.
double dot_ordered_host(const double* a, const double* b, int n) {
    DevBuf<double> da(std::max(1, n)), db(std::max(1, n)), dout(8), dpart(8 * kRedBlocks);
    IPO_HIP_CHECK(hipMemcpy(da.get(), a, n * sizeof(double), hipMemcpyHostToDevice));
    IPO_HIP_CHECK(hipMemcpy(db.get(), b, n * sizeof(double), hipMemcpyHostToDevice));
    RedJobs j{};
    j.nj = 1;
    j.a[0] = da.get(); j.b[0] = db.get(); j.len[0] = n; j.op[0] = 0;
    launch_reduce(j, dpart.get(), dout.get(), nullptr);
    double r = 0.0;
    IPO_HIP_CHECK(hipMemcpy(&r, dout.get(), sizeof(double), hipMemcpyDeviceToHost));
    return r;
}

// Segmented jobs (job_segmented): dots of at least kOrderedMaxLen entries
// (or the job set's segmin -- synthetic LPs of 10^6 columns; no netlib
// problem comes near) and long maxima.  One sequential chain of len adds
// took 4.3 ms at 10^6, one 256-thread block 1.1 ms, and the serial chain of
// a 2 x 10^5 dot ~1 ms.  Fixed segmented order instead: the vector in
// kRedBlocks contiguous segments, segment g reduced by block g (thread t
// takes its entries i = t, t + 256, ... in index order, the 256 partials
// added in thread order), the segment results added in segment order by
// k_dot_finish -- deterministic, not the reference's rounding (maxima are
// order-free, so theirs is exact).
__global__ void __launch_bounds__(kOrdThreads)
k_dot_segments(RedJobs jobs, double* __restrict__ part) {
    const int j = blockIdx.y, g = blockIdx.x, tid = threadIdx.x;
    const int len = jobs.len[j], op = jobs.op[j];
    if (!job_segmented(jobs, j)) return;
    const long seg = (static_cast<long>(len) + kRedBlocks - 1) / kRedBlocks;
    const long b = seg * g, e = min(static_cast<long>(len), b + seg);
    const double* a = jobs.a[j];
    const double* bb = jobs.b[j];
    __shared__ double sh[kOrdThreads];
    double acc = 0.0;
    for (long i0 = b; i0 < e; i0 += 8 * kOrdThreads) {
        double pa[8], pb[8];
#pragma unroll
        for (int u = 0; u < 8; u++) {
            const long i = i0 + u * kOrdThreads + tid;
            pa[u] = i < e ? a[i] : 0.0;
            pb[u] = i < e && op != 1 ? bb[i] : 1.0;
        }
#pragma unroll
        for (int u = 0; u < 8; u++) {
            if (i0 + u * kOrdThreads + tid >= e) continue;
            if (op == 0) acc += pa[u] * pb[u];
            else if (op == 1) acc = fmax(acc, ref_abs(pa[u]));
            else acc = fmax(acc, -pa[u] / pb[u]);      // NaN ratios are ignored like hsd.c:249-258
        }
    }
    sh[tid] = acc;
    __syncthreads();
    if (tid == 0) {
        double s = 0.0;
        for (int t = 0; t < kOrdThreads; t++) s = op == 0 ? s + sh[t] : fmax(s, sh[t]);
        part[j * kRedBlocks + g] = s;
    }
}

__global__ void __launch_bounds__(64)
k_dot_finish(RedJobs jobs, const double* __restrict__ part, double* __restrict__ out) {
    const int j = threadIdx.x;
    if (j >= jobs.nj || !job_segmented(jobs, j)) return;
    const bool mx = jobs.op[j] != 0;
    double s = 0.0;
    for (int g = 0; g < kRedBlocks; g++) s = mx ? fmax(s, part[j * kRedBlocks + g]) : s + part[j * kRedBlocks + g];
    out[j] = s;
}

__global__ void __launch_bounds__(256)
k_link_ax(int mrow, int m, const int* __restrict__ kAt, const int* __restrict__ iAt, const double* __restrict__ At,
          const double* __restrict__ x, double* __restrict__ out) {
    const int i = mrow + blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (i >= m) return;
    double s = 0.0;
    for (int k = kAt[i] + lane; k < kAt[i + 1]; k += 64) s += At[k] * x[iAt[k]];
    s = wave_sum(s);
    if (lane == 0) out[i - mrow] = s;
}

void launch_link_ax(int mrow, int m, const int* kAt, const int* iAt, const double* At, const double* x, double* out,
                    hipStream_t st) {
    if (m <= mrow) return;
    hipLaunchKernelGGL(k_link_ax, dim3((m - mrow + 3) / 4), dim3(256), 0, st, mrow, m, kAt, iAt, At, x, out);
    IPO_HIP_CHECK(hipGetLastError());
}

// Column-sliced row products (A x, row i summed over its columns in
// ascending order like sparse_dot): pass p adds the entries of the columns
// of slice p to the carried sum, so each pass gathers from one slice of x
// that stays in the L2 of every XCD instead of a random line of all of x per
// entry; the per-row sequence of additions is sparse_dot's, so the result is
// bitwise the same.  A slice's entries are stored by jagged diagonals (rows
// of the slice by entry count, longest first; diagonal k = the k-th entry of
// every row that has one, in that row order): thread r takes the r-th row of
// the order and its k-th entry at dptr[k] + r, so the 64 lanes of a wave
// read consecutive addresses (one row per lane on CSR would read 64 lines
// per load) and run for about the same number of entries.
__global__ void __launch_bounds__(256)
k_rows_ax_jds(int rows, const int* __restrict__ perm, const int* __restrict__ dptr, const int* __restrict__ dlen,
              int nd, const int* __restrict__ cols, const double* __restrict__ vals, const double* __restrict__ x,
              int first, double* __restrict__ ax) {
    const int r = blockIdx.x * 256 + threadIdx.x;
    if (r >= rows) return;
    const int i = perm[r];
    double s = first ? 0.0 : ax[i];
    // eight diagonals at a time, their loads in flight together (the row's
    // entries still added in order); a row has entry k iff r < dlen[k], and
    // dlen does not increase with k
    for (int k = 0; k < nd; k += 8) {
        if (r >= dlen[k]) break;
        int c[8];
        double a[8], b[8];
        bool ok[8];
#pragma unroll
        for (int u = 0; u < 8; u++) {
            ok[u] = k + u < nd && r < dlen[k + u];
            if (ok[u]) {
                const int q = dptr[k + u] + r;
                c[u] = cols[q];
                a[u] = vals[q];
            }
        }
#pragma unroll
        for (int u = 0; u < 8; u++)
            if (ok[u]) b[u] = x[c[u]];
#pragma unroll
        for (int u = 0; u < 8; u++)
            if (ok[u]) s += a[u] * b[u];
    }
    ax[i] = s;
}

// Measured on BASELINE configs[3]'s uniform LP (x 8 MB): one pass 72.6 us
// per residual launch, 2 / 3 / 4 / 8 column slices 77.5 / 79.1 / 85 / 123 us
// (the jagged-diagonal entry loads made the slices' locality worth less than
// their extra passes), so large problems take one pass by default.
int rows_ax_blocks(int n) {
    if (const char* e = std::getenv("IPO_HIP_AX_BLOCKS")) return std::max(1, std::atoi(e));
    (void)n;
    return 1;
}

bool rows_ax_sliced(int n) {
    if (const char* e = std::getenv("IPO_HIP_AX_JDS")) return std::atoi(e) != 0;
    return rows_ax_blocks(n) > 1 || static_cast<long>(n) * static_cast<long>(sizeof(double)) > kAxSliceBytes;
}

void RowAxPlan::build(int m, int n, const int* kA, const int* iA, const double* A, int npass, hipStream_t st) {
    m_ = m;
    np_ = std::max(1, npass);
    const int per = (n + np_ - 1) / np_;
    auto slice = [&](int j) { return per > 0 ? std::min(np_ - 1, j / per) : 0; };
    // entries per (pass, row), the rows of each pass by count (descending,
    // row order among equal counts), the diagonals
    std::vector<int> cnt(static_cast<size_t>(np_) * m, 0);
    for (int j = 0; j < n; j++)
        for (int k = kA[j]; k < kA[j + 1]; k++) cnt[static_cast<size_t>(slice(j)) * m + iA[k]]++;
    std::vector<int> perm(static_cast<size_t>(np_) * m), rank(static_cast<size_t>(np_) * m), dptr, dlen;
    rows_.assign(np_, 0);
    nd_.assign(np_, 0);
    dbase_.assign(np_ + 1, 0);
    long nz = 0;
    for (int p = 0; p < np_; p++) {
        const int* c = cnt.data() + static_cast<size_t>(p) * m;
        int mx = 0;
        for (int i = 0; i < m; i++) mx = std::max(mx, c[i]);
        std::vector<int> bucket(mx + 2, 0);          // rows with count >= v start at bucket[mx - v]
        for (int i = 0; i < m; i++) bucket[mx - c[i] + 1]++;
        for (int v = 0; v <= mx; v++) bucket[v + 1] += bucket[v];
        int* pp = perm.data() + static_cast<size_t>(p) * m;
        int* rk = rank.data() + static_cast<size_t>(p) * m;
        for (int i = 0; i < m; i++) { const int r = bucket[mx - c[i]]++; pp[r] = i; rk[i] = r; }
        // pass 0 writes every row (a row with no entry in it gets 0); later
        // passes only the rows that have entries in their slice
        int active = 0;
        while (active < m && c[pp[active]] > 0) active++;
        rows_[p] = p == 0 ? m : active;
        nd_[p] = mx;
        for (int k = 0, len = active; k < mx; k++) {
            while (len > 0 && c[pp[len - 1]] <= k) len--;
            dptr.push_back(static_cast<int>(nz));
            dlen.push_back(len);
            nz += len;
        }
        dbase_[p + 1] = static_cast<int>(dptr.size());
    }
    if (nz > static_cast<long>(INT32_MAX)) throw std::length_error("row products: more than 2^31 entries");
    std::vector<int> cols(nz), fill(static_cast<size_t>(np_) * m, 0);
    std::vector<double> vals(nz);
    for (int j = 0; j < n; j++) {
        const int p = slice(j);
        for (int k = kA[j]; k < kA[j + 1]; k++) {
            const size_t pi = static_cast<size_t>(p) * m + iA[k];
            const int q = dptr[dbase_[p] + fill[pi]++] + rank[pi];
            cols[q] = j;
            vals[q] = A[k];
        }
    }
    perm_.upload(perm, st);
    dptr_.upload(dptr, st);
    dlen_.upload(dlen, st);
    cols_.upload(cols, st);
    vals_.upload(vals, st);
    IPO_HIP_CHECK(hipStreamSynchronize(st));     // the host vectors go out of scope
}

void RowAxPlan::launch(const double* x, double* ax, hipStream_t st) const {
    for (int p = 0; p < np_; p++) {
        if (rows_[p] <= 0) continue;
        hipLaunchKernelGGL(k_rows_ax_jds, dim3((rows_[p] + 255) / 256), dim3(256), 0, st, rows_[p],
                           perm_.get() + static_cast<size_t>(p) * m_, dptr_.get() + dbase_[p], dlen_.get() + dbase_[p],
                           nd_[p], cols_.get(), vals_.get(), x, p == 0 ? 1 : 0, ax);
    }
    IPO_HIP_CHECK(hipGetLastError());
}

bool g_ordered_reductions = true;

void launch_reduce(const RedJobs& jobs, double* part, double* out, hipStream_t st) {
    if (g_ordered_reductions) {
        hipLaunchKernelGGL(k_reduce_ordered, dim3(jobs.nj), dim3(kOrdThreads), 0, st, jobs, out);
        bool longdot = false;
        for (int j = 0; j < jobs.nj; j++) longdot |= job_segmented(jobs, j);
        if (longdot) {     // part holds kRedBlocks partials per job (the callers' buffers: 8 jobs)
            hipLaunchKernelGGL(k_dot_segments, dim3(kRedBlocks, jobs.nj), dim3(kOrdThreads), 0, st, jobs, part);
            hipLaunchKernelGGL(k_dot_finish, dim3(1), dim3(64), 0, st, jobs, part, out);
        }
        IPO_HIP_CHECK(hipGetLastError());
        return;
    }
    unsigned mask = 0;
    for (int j = 0; j < jobs.nj; j++) if (jobs.op[j] != 0) mask |= 1u << j;
    hipLaunchKernelGGL(k_reduce_jobs, dim3(kRedBlocks), dim3(kRedThreads), 0, st, jobs, part);
    hipLaunchKernelGGL(k_finish_reduce, dim3(1), dim3(kRedThreads), 0, st, part, jobs.nj, mask, out);
    IPO_HIP_CHECK(hipGetLastError());
}

}  // namespace ipo
