// kkt_order_nd.cpp -- nested-dissection ordering of the KKT graph and the
// symbolic factor of an arbitrary elimination order (not in the reference).
//
// The reference orders K by tiered minimum degree (ldlt.c:638-1262), and so
// does this library for every problem of the size the reference was built
// for (order_tiered_min_degree, identical permutation, kkt_symbolic.cpp).
// On large banded LPs (BASELINE configs[3], the blocks of configs[4]) that
// order eliminates the band's interior one column after another: a chain of
// ~130 k columns, 2,785 supernodal levels on configs[3], every level a few
// dependent kernel launches.  K is quasi-definite, so it factors stably
// under any symmetric permutation (the reason ldlt.c can order it freely);
// nested dissection cuts the band into pieces whose subtrees factor side by
// side and meet at separators, giving an elimination tree of a few dozen
// levels.
//
// Separators come from BFS level structures (George's automatic nested
// dissection): from a pseudo-peripheral node of the piece, the levels of
// the breadth-first search are vertex separators.  K's graph is bipartite
// (y-nodes meet only x-nodes), so the levels alternate node class and the
// separator is taken among the y-levels (rows: ~band width of them on a
// banded LP) near the median.  Pieces of at most `leaf_rows` y-nodes are
// leaves: their x-nodes first (independent single-column supernodes), then
// their y-nodes in natural order (one dense band segment, nested columns).
#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <cstdlib>
#include <exception>
#include <mutex>
#include <stdexcept>
#include <thread>
#include <vector>

#include "kkt_plan.h"

namespace ipo {

namespace {

struct Job {
    int lo;                 // first new index of this piece
    std::vector<int> nodes;
};

}  // namespace

std::vector<int> nested_dissection_perm(int m, int n, const int* kA, const int* iA, const int* kAt, const int* iAt,
                                        int nforced, int leaf_rows, const QPattern* q) {
    const int T = m + n, mf = m - nforced, Tfree = T - nforced;
    const bool hasq = q && q->kQ;
    if (hasq && nforced > 0) throw std::invalid_argument("kkt: a Q block with forced rows is not supported");
    // free graph in CSR (forced rows left out, as in order_tiered_min_degree);
    // a Q block adds y-y edges, and the graph is then no longer bipartite
    std::vector<int> xadj(T + 1, 0), adj;
    adj.reserve(2 * static_cast<size_t>(kA[n]) + (hasq ? q->kQ[m] : 0));
    for (int r = 0; r < m; r++) {
        if (r < mf) {
            for (int k = kAt[r]; k < kAt[r + 1]; k++) adj.push_back(m + iAt[k]);
            if (hasq)
                for (int k = q->kQ[r]; k < q->kQ[r + 1]; k++)
                    if (q->iQ[k] != r) adj.push_back(q->iQ[k]);
        }
        xadj[r + 1] = static_cast<int>(adj.size());
    }
    for (int c = 0; c < n; c++) {
        for (int k = kA[c]; k < kA[c + 1]; k++)
            if (iA[k] < mf) adj.push_back(iA[k]);
        xadj[m + c + 1] = static_cast<int>(adj.size());
    }
    std::vector<int> perm(T, -1);
    for (int k = 0; k < nforced; k++) perm[Tfree + k] = mf + k;
    // dense nodes (rows or columns of more than ten times their class's mean
    // degree, and more than kNdDense: the linking rows of a block-angular LP
    // passed whole) would put every piece within two BFS levels of each
    // other; they leave the graph and go last, in natural order, before the
    // forced rows (their columns then form the dense tail)
    std::vector<int> dense;
    {
        double sy = 0, sx = 0;
        for (int r = 0; r < mf; r++) sy += xadj[r + 1] - xadj[r];
        for (int c = m; c < T; c++) sx += xadj[c + 1] - xadj[c];
        const double ty = std::max<double>(kNdDense, 10.0 * sy / std::max(1, mf));
        const double tx = std::max<double>(kNdDense, 10.0 * sx / std::max(1, n));
        for (int v = 0; v < T; v++) {
            if (v >= mf && v < m) continue;
            if (xadj[v + 1] - xadj[v] > (v < m ? ty : tx)) dense.push_back(v);
        }
        if (!dense.empty()) {
            std::vector<char> isd(T, 0);
            for (int v : dense) isd[v] = 1;
            std::vector<int> x2(T + 1, 0), a2;
            a2.reserve(adj.size());
            for (int v = 0; v < T; v++) {
                if (!isd[v])
                    for (int k = xadj[v]; k < xadj[v + 1]; k++)
                        if (!isd[adj[k]]) a2.push_back(adj[k]);
                x2[v + 1] = static_cast<int>(a2.size());
            }
            xadj.swap(x2);
            adj.swap(a2);
            std::copy(dense.begin(), dense.end(), perm.begin() + (Tfree - static_cast<int>(dense.size())));
        }
    }

    // The pieces are independent: a pool of threads takes them from a shared
    // list (large pieces) or a private stack (small ones).  Each piece's
    // outcome depends only on its own node list and first index, so the
    // permutation does not depend on the schedule.  Every thread marks the
    // nodes of its piece in arrays of its own (stamps are unique per piece):
    // shared mark arrays would have the threads' writes to neighbouring
    // nodes of different pieces contend for the same cache lines.
    std::atomic<int> stamp{0};
    std::vector<Job> shared;
    std::mutex mu;
    std::condition_variable cv;
    int busy = 0;
    {
        Job root;
        root.lo = 0;
        root.nodes.reserve(Tfree);
        std::vector<char> isd(T, 0);
        for (int v : dense) isd[v] = 1;
        for (int v = 0; v < T; v++)
            if ((v < mf || v >= m) && !isd[v]) root.nodes.push_back(v);
        shared.push_back(std::move(root));
    }
    constexpr size_t kSharedMin = 16384;      // pieces at least this large go to the shared list

    // a worker that throws (bad_alloc on its per-thread arrays, ...) stores
    // the first exception and stops the pool; it is rethrown after the join,
    // so the C API's try / catch sees it instead of std::terminate
    std::exception_ptr failure;
    std::atomic<bool> failed{false};
    auto work = [&]() {
        std::vector<int> inset(T, -1), dist(T, -1), order;
        auto inset_of = [&](int w) { return inset[w]; };
        auto set_inset = [&](int w, int st) { inset[w] = st; };
        std::vector<Job> local;
        // BFS inside the set stamped `st`; fills dist (relative), returns the number of levels
        auto bfs = [&](int src, int st, std::vector<int>& ord) -> int {
            ord.clear();
            ord.push_back(src);
            dist[src] = 0;
            int nl = 1;
            for (size_t h = 0; h < ord.size(); h++) {
                const int v = ord[h], dv = dist[v];
                for (int k = xadj[v]; k < xadj[v + 1]; k++) {
                    const int w = adj[k];
                    if (inset_of(w) == st && dist[w] < 0) {
                        dist[w] = dv + 1;
                        nl = std::max(nl, dv + 2);
                        ord.push_back(w);
                    }
                }
            }
            return nl;
        };
        auto leaf = [&](Job& J) {
            std::vector<int>& v = J.nodes;
            // x-nodes first, then y-nodes, each in natural order
            const auto mid = std::partition(v.begin(), v.end(), [&](int a) { return a >= m; });
            std::sort(v.begin(), mid);
            std::sort(mid, v.end());
            std::copy(v.begin(), v.end(), perm.begin() + J.lo);
        };
        auto emit = [&](Job&& c) {
            if (c.nodes.size() >= kSharedMin) {
                std::lock_guard<std::mutex> g(mu);
                shared.push_back(std::move(c));
                cv.notify_one();
            } else {
                local.push_back(std::move(c));
            }
        };
        // one piece: a leaf, its connected components, or two halves and a separator
        auto split = [&](Job J) {
            const int size = static_cast<int>(J.nodes.size());
            if (size == 0) return;
            int ny = 0;
            for (int v : J.nodes) ny += v < m;
            if (ny <= leaf_rows) { leaf(J); return; }
            const int st = ++stamp;
            for (int v : J.nodes) { set_inset(v, st); dist[v] = -1; }
            // connected components: each its own piece (independent subtrees)
            int nl = bfs(J.nodes[0], st, order);
            if (static_cast<int>(order.size()) < size) {
                std::vector<Job> comps;
                int lo = J.lo;
                auto take = [&]() {
                    Job c;
                    c.lo = lo;
                    c.nodes = order;
                    for (int w : order) set_inset(w, -2);
                    lo += static_cast<int>(order.size());
                    comps.push_back(std::move(c));
                };
                take();
                for (int v : J.nodes)
                    if (inset[v] == st) { bfs(v, st, order); take(); }
                for (int v : J.nodes) { set_inset(v, -1); dist[v] = -1; }
                for (auto& c : comps) emit(std::move(c));
                return;
            }
            // pseudo-peripheral root: restart from a minimum-degree node of the
            // last level while the eccentricity grows
            int root = J.nodes[0];
            for (int it = 0; it < 4; it++) {
                int best = -1, bdeg = 0;
                for (size_t q = order.size(); q-- > 0;) {
                    const int v = order[q];
                    if (dist[v] != nl - 1) break;
                    const int d = xadj[v + 1] - xadj[v];
                    if (best < 0 || d < bdeg) { best = v; bdeg = d; }
                }
                for (int v : order) dist[v] = -1;
                const int nl2 = bfs(best, st, order);
                if (nl2 > nl) { root = best; nl = nl2; continue; }
                if (nl2 == nl) { root = best; break; }
                for (int v : order) dist[v] = -1;     // shorter: back to the previous root
                nl = bfs(root, st, order);
                break;
            }
            // level sizes; y-levels are those of the root's class parity
            std::vector<int> cnt(nl, 0);
            for (int v : order) cnt[dist[v]]++;
            const int ypar = root < m ? 0 : 1;
            std::vector<long> before(nl + 1, 0);
            for (int l = 0; l < nl; l++) before[l + 1] = before[l] + cnt[l];
            int sep = -1;
            {
                long bestc = -1;
                for (int l = 1; l + 1 < nl; l++) {
                    if (!hasq && (l & 1) != ypar) continue;
                    const long b = before[l], a = size - before[l + 1];
                    const long rest = b + a;
                    if (10 * std::min(a, b) < 3 * rest) continue;        // both sides >= 30 %
                    if (bestc < 0 || cnt[l] < bestc) { bestc = cnt[l]; sep = l; }
                }
                if (sep < 0) {        // no balanced y-level: the one nearest the median
                    long bd = -1;
                    for (int l = 1; l + 1 < nl; l++) {
                        if (!hasq && (l & 1) != ypar) continue;
                        const long d = std::labs(before[l] - (size - before[l + 1]));
                        if (bd < 0 || d < bd) { bd = d; sep = l; }
                    }
                }
            }
            if (sep < 0) {            // no interior y-level
                for (int v : J.nodes) { set_inset(v, -1); dist[v] = -1; }
                leaf(J);
                return;
            }
            Job P1, P2;
            std::vector<int> S;
            // one allocation each (big vectors grown by doubling come and go
            // through mmap / munmap, and every munmap stalls all threads)
            P1.nodes.reserve(before[sep + 1]);
            P2.nodes.reserve(size - before[sep + 1]);
            for (int v : order) {
                const int d = dist[v];
                if (d < sep) P1.nodes.push_back(v);
                else if (d > sep) P2.nodes.push_back(v);
                else {
                    // a separator node with no neighbour beyond the separator
                    // belongs to the near side
                    bool far = false;
                    for (int k = xadj[v]; k < xadj[v + 1]; k++) {
                        const int w = adj[k];
                        if (inset_of(w) == st && dist[w] == sep + 1) { far = true; break; }
                    }
                    if (far) S.push_back(v);
                    else P1.nodes.push_back(v);
                }
            }
            for (int v : J.nodes) { set_inset(v, -1); dist[v] = -1; }
            std::sort(S.begin(), S.end());
            P1.lo = J.lo;
            P2.lo = J.lo + static_cast<int>(P1.nodes.size());
            std::copy(S.begin(), S.end(), perm.begin() + P2.lo + static_cast<int>(P2.nodes.size()));
            emit(std::move(P2));
            emit(std::move(P1));
        };
        for (;;) {
            Job J;
            {
                std::unique_lock<std::mutex> g(mu);
                cv.wait(g, [&] { return failed || !shared.empty() || busy == 0; });
                if (failed || shared.empty()) return;  // nothing queued and nobody working: done
                J = std::move(shared.back());
                shared.pop_back();
                busy++;
            }
            split(std::move(J));
            while (!local.empty() && !failed) {
                Job c = std::move(local.back());
                local.pop_back();
                split(std::move(c));
            }
            {
                std::lock_guard<std::mutex> g(mu);
                busy--;
                if (busy == 0 && shared.empty()) cv.notify_all();
            }
        }
    };
    auto worker = [&]() {
        try {
            work();
        } catch (...) {
            std::lock_guard<std::mutex> g(mu);
            if (!failed) failure = std::current_exception();
            failed = true;
            cv.notify_all();
        }
    };
    const int nth = setup_threads();
    std::vector<std::thread> pool;
    for (int i = 1; i < nth; i++) pool.emplace_back(worker);
    worker();
    for (auto& th : pool) th.join();
    if (failure) std::rethrow_exception(failure);
    for (int v = 0; v < T; v++)
        if (perm[v] < 0) throw std::logic_error("nested dissection: incomplete permutation");
    return perm;
}

// Strict-lower pattern of L for the elimination order perm over the free
// nodes [0, Tfree) (forced rows excluded): column j holds K's entries below
// j and every child's pattern below j (the row-merge rule over the
// elimination tree, parent = first row).
void symbolic_from_perm(KktOrdering& o, const int* kA, const int* iA, const int* kAt, const int* iAt, int nforced,
                        const QPattern* q) {
    const int m = o.m, T = o.T, Tfree = T - nforced, mf = m - nforced;
    o.iperm.assign(T, -1);
    for (int j = 0; j < T; j++) o.iperm[o.perm[j]] = j;
    const std::vector<int>& iperm = o.iperm;
    std::vector<int> Lp(T + 1, 0), Li;
    Li.reserve(static_cast<size_t>(kA[o.n]) * 4);
    std::vector<int> mark(Tfree, -1), head(Tfree, -1), next(Tfree, -1), rest;
    for (int j = 0; j < Tfree; j++) {
        const size_t start = Li.size();
        mark[j] = j;
        const int v = o.perm[j];
        // the longest child's pattern below j is already sorted: it is merged
        // with the sorted rest (K's entries, the other children) instead of
        // sorting the whole column
        int big = -1;
        for (int c = head[j]; c >= 0; c = next[c])
            if (big < 0 || Lp[c + 1] - Lp[c] > Lp[big + 1] - Lp[big]) big = c;
        if (big >= 0)
            for (int k = Lp[big] + 1; k < Lp[big + 1]; k++) mark[Li[k]] = j;   // Li[Lp[big]] == j
        rest.clear();
        auto add = [&](int i) {
            if (i > j && i < Tfree && mark[i] != j) { mark[i] = j; rest.push_back(i); }
        };
        if (v < m) {
            for (int k = kAt[v]; k < kAt[v + 1]; k++) add(iperm[m + iAt[k]]);
            if (q && q->kQ)
                for (int k = q->kQ[v]; k < q->kQ[v + 1]; k++) add(iperm[q->iQ[k]]);
        } else {
            for (int k = kA[v - m]; k < kA[v - m + 1]; k++)
                if (iA[k] < mf) add(iperm[iA[k]]);
        }
        for (int c = head[j]; c >= 0; c = next[c])
            if (c != big)
                for (int k = Lp[c]; k < Lp[c + 1]; k++) add(Li[k]);
        std::sort(rest.begin(), rest.end());
        const size_t nb = big >= 0 ? static_cast<size_t>(Lp[big + 1] - Lp[big] - 1) : 0;
        if (start + nb + rest.size() > static_cast<size_t>(INT32_MAX))
            throw std::length_error("symbolic: more than 2^31 nonzeros in L");
        Li.resize(start + nb + rest.size());
        const int* bp = Li.data() + (big >= 0 ? Lp[big] + 1 : 0);
        std::merge(bp, bp + nb, rest.begin(), rest.end(), Li.begin() + start);
        Lp[j + 1] = static_cast<int>(Li.size());
        if (Li.size() > start) {
            const int p = Li[start];
            next[j] = head[p];
            head[p] = j;
        }
    }
    for (int j = Tfree; j < T; j++) Lp[j + 1] = Lp[Tfree];
    o.Lp.swap(Lp);
    o.Li.swap(Li);
}

// Relaxed supernodes: columns j, j + 1 with parent(j) = j + 1 share a panel
// when the panel padded to the nested pattern (every column k of a panel
// [c, e] gets rows {k+1..e} U struct(e)) holds at most `zfrac` explicit zeros
// and kPanelCols columns.  The padded entries are zero in exact arithmetic
// and stay exact zeros in the factor (every term that forms them is a
// product with a structural zero), and struct(k) \ {k + 1} is contained in
// struct(k + 1) along the chain, so no other column's pattern changes.
void relax_supernodes(KktOrdering& o, int tc, double zfrac) {
    if (zfrac <= 0.0) return;
    const int T = o.T;
    std::vector<int> cnt(T);
    for (int j = 0; j < T; j++) cnt[j] = o.Lp[j + 1] - o.Lp[j];
    std::vector<int> pstart;          // panel starts, [c, next start)
    pstart.push_back(0);
    for (int j = 0; j + 1 < tc; j++) {
        const int c = pstart.back();
        const int width = j + 1 - c;
        bool join = false;
        if (cnt[j] > 0 && o.Li[o.Lp[j]] == j + 1 && width < kPanelCols) {
            double e2 = 0.0, nz2 = 0.0;
            for (int k = c; k <= j + 1; k++) { e2 += (j + 1 - k) + cnt[j + 1]; nz2 += cnt[k]; }
            join = e2 - nz2 <= zfrac * e2;
        }
        if (!join) pstart.push_back(j + 1);
    }
    pstart.push_back(tc);
    bool padded = false;
    for (size_t q = 0; q + 1 < pstart.size(); q++) {
        const int c = pstart[q], e = pstart[q + 1] - 1;
        for (int k = c; k < e; k++)
            if (cnt[k] != (e - k) + cnt[e]) { padded = true; break; }
        if (padded) break;
    }
    if (!padded) return;
    std::vector<int> Lp(T + 1, 0), Li;
    size_t tot = 0;
    for (size_t q = 0; q + 1 < pstart.size(); q++) {
        const int c = pstart[q], e = pstart[q + 1] - 1;
        for (int k = c; k <= e; k++) tot += (e - k) + cnt[e];
    }
    for (int j = tc; j < T; j++) tot += cnt[j];
    Li.reserve(tot);
    for (size_t q = 0; q + 1 < pstart.size(); q++) {
        const int c = pstart[q], e = pstart[q + 1] - 1;
        for (int k = c; k <= e; k++) {
            for (int r = k + 1; r <= e; r++) Li.push_back(r);
            Li.insert(Li.end(), o.Li.begin() + o.Lp[e], o.Li.begin() + o.Lp[e + 1]);
            Lp[k + 1] = static_cast<int>(Li.size());
        }
    }
    for (int j = tc; j < T; j++) {
        Li.insert(Li.end(), o.Li.begin() + o.Lp[j], o.Li.begin() + o.Lp[j + 1]);
        Lp[j + 1] = static_cast<int>(Li.size());
    }
    o.Lp.swap(Lp);
    o.Li.swap(Li);
}

}  // namespace ipo
