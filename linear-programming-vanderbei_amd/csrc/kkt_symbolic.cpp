// kkt_symbolic.cpp -- host symbolic phase for the GPU KKT factorisation.
// See kkt_plan.h.  Reference behaviour restated (not translated):
//   ordering   src/ipo/ldlt.c:638-858 (inv_sym), :860-1262 (lltsym)
//   heap       src/ipo/ldlt.c:1305-1349
#include "kkt_plan.h"

#include <algorithm>
#include <atomic>
#include <functional>
#include <iterator>
#include <memory>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <mutex>
#include <stdexcept>
#include <thread>

namespace ipo {

namespace {

// Min-heap of node ids keyed by an external key array, 1-based positions.
// The sift rules (strict comparisons, right child preferred only when
// strictly smaller) decide ties and therefore the ordering; they follow
// ldlt.c:1305-1349.
struct KeyHeap {
    std::vector<int> slot;   // slot[pos] = node, pos in 1..count
    std::vector<int> at;     // at[node]  = pos
    int count = 0;
    const std::vector<int>* key = nullptr;

    void exchange(int a, int b) {
        std::swap(slot[a], slot[b]);
        std::swap(at[slot[a]], at[slot[b]]);
    }
    void sink(int pos) {
        const auto& k = *key;
        for (int ch = 2 * pos; ch <= count; ch = 2 * pos) {
            if (ch < count && k[slot[ch + 1]] < k[slot[ch]]) ch++;
            if (!(k[slot[pos]] > k[slot[ch]])) return;
            exchange(pos, ch);
            pos = ch;
        }
    }
    void swim(int pos) {
        const auto& k = *key;
        for (int par = pos / 2; par > 0; par = pos / 2) {
            if (!(k[slot[par]] > k[slot[pos]])) return;
            exchange(pos, par);
            pos = par;
        }
    }
};

// Threads for the bit-matrix clique steps of the minimum-degree ordering:
// run(fn) calls fn(tid) on every thread (tid 0 = the caller) and returns
// when all have; between steps the workers spin briefly, then yield.
class StepPool {
  public:
    explicit StepPool(int nth) {
        for (int i = 1; i < nth; i++) th_.emplace_back([this, i] { loop(i); });
    }
    ~StepPool() {
        stop_.store(true, std::memory_order_relaxed);
        gen_.fetch_add(1, std::memory_order_release);
        for (auto& t : th_) t.join();
    }
    // An exception thrown by fn on any thread (bad_alloc in a clique step)
    // is kept, the step still completes on every thread, and the first one
    // is rethrown here after the join, so it reaches the C API's catch.
    template <class F>
    void run(F&& f) {
        fn_ = std::ref(f);
        err_ = nullptr;
        done_.store(0, std::memory_order_relaxed);
        gen_.fetch_add(1, std::memory_order_release);
        try {
            f(0);
        } catch (...) {
            keep(std::current_exception());
        }
        while (done_.load(std::memory_order_acquire) != static_cast<int>(th_.size())) relax();
        if (err_) std::rethrow_exception(err_);
    }

  private:
    static void relax() { __builtin_ia32_pause(); }
    void loop(int tid) {
        unsigned seen = 0;
        for (;;) {
            unsigned g;
            for (int spins = 0; (g = gen_.load(std::memory_order_acquire)) == seen; spins++) {
                if (spins < 4096) relax();
                else std::this_thread::yield();
            }
            seen = g;
            if (stop_.load(std::memory_order_relaxed)) return;
            try {
                fn_(tid);
            } catch (...) {
                keep(std::current_exception());
            }
            done_.fetch_add(1, std::memory_order_release);
        }
    }
    void keep(std::exception_ptr e) {
        std::lock_guard<std::mutex> g(err_mu_);
        if (!err_) err_ = e;
    }
    std::vector<std::thread> th_;
    std::function<void(int)> fn_;
    std::mutex err_mu_;
    std::exception_ptr err_;
    std::atomic<unsigned> gen_{0};
    std::atomic<int> done_{0};
    std::atomic<bool> stop_{false};
};
constexpr size_t kPoolMinGroup = 256;   // smaller groups stay on the caller
constexpr size_t kPoolChunk = 8;        // members per claim

// Forced tail (kkt_plan.h): the free columns [0, Tfree) are ordered and
// their free-row pattern is known; the forced rows (y-nodes mf..m-1) go
// last in natural order.  No path between two free nodes runs through a
// forced node (those come later), so the free pattern is unchanged and the
// forced part of column s is  F(s) = adjF(s) U (F(c) of every etree child c),
// the standard row-merge rule restricted to the forced rows.
void add_forced_tail(KktOrdering& o, int m, const int* kA, const int* iA, int nforced) {
    const int T = o.T, Tfree = T - nforced, mf = m - nforced;
    for (int k = 0; k < nforced; k++) {
        o.perm[Tfree + k] = mf + k;
        o.iperm[mf + k] = Tfree + k;
    }
    std::vector<std::vector<int>> F(Tfree);
    for (int s = 0; s < Tfree; s++) {
        const int v = o.perm[s];
        std::vector<int>& f = F[s];
        if (v >= m) {                                   // x-node: its forced rows
            std::vector<int> a;
            for (int k = kA[v - m]; k < kA[v - m + 1]; k++)
                if (iA[k] >= mf) a.push_back(Tfree + iA[k] - mf);
            std::sort(a.begin(), a.end());
            std::vector<int> u;
            std::set_union(f.begin(), f.end(), a.begin(), a.end(), std::back_inserter(u));
            f.swap(u);
        }
        // parent: first free row below, else the first forced row
        int par = -1;
        if (o.Lp[s + 1] > o.Lp[s]) par = o.Li[o.Lp[s]];
        if (par >= 0 && par < Tfree) {
            std::vector<int>& g = F[par];
            std::vector<int> u;
            std::set_union(g.begin(), g.end(), f.begin(), f.end(), std::back_inserter(u));
            g.swap(u);
        }
    }
    std::vector<int> Lp(T + 1, 0), Li;
    size_t tot = static_cast<size_t>(o.Lp[Tfree]);
    for (int s = 0; s < Tfree; s++) tot += F[s].size();
    tot += static_cast<size_t>(nforced) * (nforced - 1) / 2;
    Li.reserve(tot);
    for (int s = 0; s < Tfree; s++) {
        Li.insert(Li.end(), o.Li.begin() + o.Lp[s], o.Li.begin() + o.Lp[s + 1]);
        Li.insert(Li.end(), F[s].begin(), F[s].end());
        std::vector<int>().swap(F[s]);
        Lp[s + 1] = static_cast<int>(Li.size());
    }
    for (int k = 0; k < nforced; k++) {                 // dense lower triangle
        for (int r = Tfree + k + 1; r < T; r++) Li.push_back(r);
        Lp[Tfree + k + 1] = static_cast<int>(Li.size());
    }
    o.Lp.swap(Lp);
    o.Li.swap(Li);
    o.denwin = Tfree;
}

}  // namespace

bool QPattern::separable(int m) const {
    if (!kQ) return true;
    for (int j = 0; j < m; j++)
        for (int k = kQ[j]; k < kQ[j + 1]; k++)
            if (iQ[k] != j) return false;
    return true;
}

KktOrdering order_nested_dissection(int m, int n, const int* kA, const int* iA, const int* kAt, const int* iAt,
                                    int nforced, int leaf_rows, double zfrac, const QPattern* q) {
    KktOrdering o;
    o.m = m; o.n = n; o.T = m + n;
    o.perm = nested_dissection_perm(m, n, kA, iA, kAt, iAt, nforced, leaf_rows, q);
    symbolic_from_perm(o, kA, iA, kAt, iAt, nforced, q);
    const int T = o.T;
    if (nforced > 0) {
        add_forced_tail(o, m, kA, iA, nforced);
    } else {
        int tc = T;
        while (tc > 0 && o.Lp[tc] - o.Lp[tc - 1] == T - tc) tc--;
        o.denwin = tc;
    }
    double na = 0.0;
    for (int v = 0; v < T; v++) { double c = o.Lp[v + 1] - o.Lp[v]; na += c * c; }
    o.narth = na + 3.0 * o.Lp[T] + T;
    relax_supernodes(o, nforced > 0 ? T - nforced : o.denwin, zfrac);
    return o;
}

bool use_nested_dissection(int T) {
    const char* e = std::getenv("IPO_HIP_ORDER");
    if (e && !std::strcmp(e, "md")) return false;
    if (e && !std::strcmp(e, "nd")) return true;
    return T >= kNdMinNodes;
}

int setup_threads() {
    if (const char* e = std::getenv("IPO_HIP_SETUP_THREADS")) return std::max(1, std::atoi(e));
    const int hw = static_cast<int>(std::thread::hardware_concurrency());
    return std::max(1, std::min(16, hw));
}

KktOrdering order_tiered_min_degree(int m, int n, const int* kA, const int* iA,
                                    const int* kAt, const int* iAt, int nforced, const QPattern* q) {
    const bool hasq = q && q->kQ;
    if (hasq && nforced > 0) throw std::invalid_argument("kkt: a Q block with forced rows is not supported");
    KktOrdering o;
    o.m = m; o.n = n; o.T = m + n;
    const int T = o.T;

    // which node class goes first: compare the reference's fill estimates
    // for eliminating y-nodes first ("primal") vs x-nodes first ("dual")
    double keep = 1.0;
    for (int r = 0; r < m; r++) {
        double dens = static_cast<double>(kAt[r + 1] - kAt[r]) / (n + 1);
        keep = keep * (1.0 - dens * dens);
    }
    const double fill_y_first = 0.5 * n * n * (1.0 - keep);
    keep = 1.0;
    for (int c = 0; c < n; c++) {
        double dens = static_cast<double>(kA[c + 1] - kA[c]) / (m + 1);
        keep = keep * (1.0 - dens * dens);
    }
    const double fill_x_first = 0.5 * m * m * (1.0 - keep);
    // the primal priority needs a separable problem (ldlt.c:675-682, 710)
    o.pdf = (3 * fill_y_first <= fill_x_first && (!hasq || q->separable(m))) ? 1 : 2;

    // adjacency of K, y-node r lists its x-nodes (column order), x-node c its rows
    // forced rows (y-nodes mf..m-1, see kkt_plan.h) stay out of the graph
    const int mf = m - nforced;
    std::vector<std::vector<int>> nb(T);
    std::vector<int> tier(T);
    for (int r = 0; r < mf; r++) {
        nb[r].reserve(kAt[r + 1] - kAt[r] + (hasq ? q->kQ[r + 1] - q->kQ[r] : 0));
        for (int k = kAt[r]; k < kAt[r + 1]; k++) nb[r].push_back(m + iAt[k]);
        if (hasq)            // then the Q neighbours (ldlt.c:737-742)
            for (int k = q->kQ[r]; k < q->kQ[r + 1]; k++)
                if (q->iQ[k] != r) nb[r].push_back(q->iQ[k]);
        tier[r] = o.pdf == 1 ? 0 : 1;
    }
    for (int r = mf; r < m; r++) tier[r] = 0;
    for (int c = 0; c < n; c++) {
        nb[m + c].reserve(kA[c + 1] - kA[c]);
        for (int k = kA[c]; k < kA[c + 1]; k++)
            if (iA[k] < mf) nb[m + c].push_back(iA[k]);
        tier[m + c] = o.pdf == 1 ? 1 : 0;
    }
    // the reference's dense-column threshold always evaluates to 3 for ipo
    // (no free variables, no finite ranges: ldlt.c:814-846)
    const int dense_deg = 3;
    const int penalty = T;

    // deg[v]: live neighbours of v.  Eliminated nodes are not erased from
    // the survivors' lists as they leave (an O(degree) find + shift per
    // survivor and pivot); they stay as dead entries, skipped where a list
    // is read, and a list is compacted (order kept) once it is mostly dead.
    // Every decision reads the same live neighbours in the same order as the
    // eager form, so the ordering is unchanged.
    std::vector<int> deg(T), ndead(T, 0);
    std::vector<char> dead(T, 0);
    for (int v = 0; v < T; v++) deg[v] = static_cast<int>(nb[v].size());
    auto compact = [&](int w) {
        auto& lst = nb[w];
        lst.erase(std::remove_if(lst.begin(), lst.end(), [&](int q) { return dead[q] != 0; }), lst.end());
        ndead[w] = 0;
    };

    std::vector<int> key(T);
    for (int v = 0; v < T; v++) {
        int d = deg[v];
        if (d > dense_deg && tier[v] == 0) tier[v] = 1;
        key[v] = d + tier[v] * penalty;
    }
    for (int r = mf; r < m; r++) key[r] = 4 * penalty;    // never chosen before the free nodes
    KeyHeap hp;
    hp.key = &key;
    hp.slot.assign(T + 1, 0);
    hp.at.assign(T, 0);
    hp.count = T;
    for (int v = T - 1; v >= 0; v--) { hp.at[v] = v + 1; hp.slot[v + 1] = v; hp.sink(v + 1); }

    std::vector<int>& perm = o.perm;
    std::vector<int>& iperm = o.iperm;
    perm.assign(T, -1);
    iperm.assign(T, -1);
    std::vector<int> seen(T, 0), group;
    group.reserve(T);
    o.Lp.assign(T + 1, 0);
    std::vector<int> lrows;          // original ids until the final relabel
    lrows.reserve(static_cast<size_t>(kA[n]) * 2);

    int stamp = 0, step = 0, denwin = T;
    const int Tfree = T - nforced;
    constexpr int kBitsNodes = 8192;
    int bw = 0;                                  // words per bit-matrix row (0: lists only)
    std::vector<uint64_t> bits;
    std::vector<int> cidx(T, -1), cnode, gpos;  // bit-matrix column of a node and back
    std::vector<uint64_t> gmask, alive;
    std::vector<std::vector<uint64_t>> pmask(1);  // per pool thread
    std::unique_ptr<StepPool> pool;
    while (step < Tfree) {
        const int piv = hp.slot[1];
        const int dg = deg[piv];
        if (dg >= T - 1 - step) denwin = step;
        perm[step] = piv;
        iperm[piv] = step;
        if (ndead[piv]) compact(piv);

        // neighbours are tagged with the current step; twins (same degree,
        // same tier, neighbourhood inside piv's closed neighbourhood) are
        // eliminated together with piv
        int next = step + 1;
        group.clear();
        for (int w : nb[piv]) iperm[w] = step;
        // (on the bit matrix: w's live row inside piv's row plus piv)
        const uint64_t* prow = bw > 0 ? bits.data() + static_cast<size_t>(cidx[piv]) * bw : nullptr;
        for (int w : nb[piv]) {
            bool twin = false;
            if (deg[w] == dg && tier[w] == tier[piv]) {
                twin = true;
                if (bw > 0) {
                    const uint64_t* row = bits.data() + static_cast<size_t>(cidx[w]) * bw;
                    const int cp = cidx[piv];
                    for (int k = 0; k < bw && twin; k++) {
                        uint64_t x = row[k] & alive[k] & ~prow[k];
                        if (k == (cp >> 6)) x &= ~(1ull << (cp & 63));
                        twin = x == 0;
                    }
                } else {
                    for (int q : nb[w])
                        if (!dead[q] && iperm[q] < step) { twin = false; break; }
                }
            }
            if (twin) { perm[next] = w; iperm[w] = next; next++; }
            else group.push_back(w);
        }

        // L's column s: its live neighbours after it (their order is free:
        // the relabel sorts every column)
        int width = dg;
        for (int s = step; s < next; s++) {
            const int v = perm[s];
            o.Lp[s + 1] = o.Lp[s] + width;
            auto take = [&](int w) {
                const int r = iperm[w];
                if (r > s || (r == step && w != piv)) lrows.push_back(w);
            };
            if (bw > 0) {
                const uint64_t* row = bits.data() + static_cast<size_t>(cidx[v]) * bw;
                for (int k = 0; k < bw; k++)
                    for (uint64_t x = row[k] & alive[k]; x; x &= x - 1) take(cnode[(k << 6) + __builtin_ctzll(x)]);
            } else {
                for (int w : nb[v])
                    if (!dead[w]) take(w);
            }
            width--;
        }

        // piv and its twins leave the survivors' lists (as dead entries)
        const int nel = next - step;
        for (int s = step; s < next; s++) {
            const int v = perm[s];
            dead[v] = 1;
            if (bw > 0) alive[cidx[v] >> 6] &= ~(1ull << (cidx[v] & 63));
        }
        for (int w : group) { deg[w] -= nel; ndead[w] += nel; }
        for (int s = step; s < next; s++) {      // leave the heap
            const int v = perm[s];
            const int pos = hp.at[v];
            const int old_key = key[hp.slot[pos]];
            hp.slot[pos] = hp.slot[hp.count];
            hp.at[hp.slot[pos]] = pos;
            hp.count--;
            if (old_key < key[hp.slot[pos]]) hp.sink(pos);
            else hp.swim(pos);
        }
        // clique on the survivors: w gains, in group order, every member of
        // the group it is not adjacent to yet (the pairwise loop below appends
        // exactly that sequence to every list).  Nothing to add once the
        // survivors form a complete graph (the reference's dense window:
        // every survivor a neighbour of piv and of each other)
        const int nsurv = Tfree - next;
        bool complete = static_cast<int>(group.size()) == nsurv;
        for (size_t a = 0; complete && a < group.size(); a++) complete = deg[group[a]] == nsurv - 1;
        if (complete) {
        } else if (bw > 0) {
            // The pairwise loop below adds a missing pair (a, b), a before b
            // in group order, at a's turn to both lists; whether it is
            // missing depends only on the adjacency at the step's start.  So
            // every member w gains exactly the members it was not adjacent
            // to, in group order (those before it from their turns, those
            // after it from its own).  Word-parallel here: the missing
            // members of w are gmask & ~row(w) over the group's words; each
            // list grows by its own appends only (no scattered pushes), and
            // the rows take the whole clique afterwards.
            int wlo = bw, whi = -1;
            for (size_t a = 0; a < group.size(); a++) {
                const int c = cidx[group[a]];
                gpos[c] = static_cast<int>(a);
                gmask[c >> 6] |= 1ull << (c & 63);
                wlo = std::min(wlo, c >> 6);
                whi = std::max(whi, c >> 6);
            }
            // A member reads and writes only its own row, list and degree,
            // so large groups are split over the step pool's threads (the
            // result is the serial loop's, bit for bit).
            const size_t pw = (group.size() + 63) / 64;
            auto member = [&](size_t a, uint64_t* pm) {
                const int w = group[a], cw = cidx[w];
                uint64_t* row = bits.data() + static_cast<size_t>(cw) * bw;
                // missing members into a bit set over group positions,
                // read back in position order (no sort)
                int nmiss = 0;
                for (int k = wlo; k <= whi; k++) {
                    uint64_t x = gmask[k] & ~row[k];
                    if (k == (cw >> 6)) x &= ~(1ull << (cw & 63));
                    while (x) {
                        const int b = gpos[(k << 6) + __builtin_ctzll(x)];
                        pm[b >> 6] |= 1ull << (b & 63);
                        nmiss++;
                        x &= x - 1;
                    }
                    row[k] |= gmask[k];                 // the row takes the whole clique
                }
                row[cw >> 6] &= ~(1ull << (cw & 63));
                if (nmiss == 0) return;
                auto& lst = nb[w];
                for (size_t k = 0; k < pw; k++) {
                    uint64_t x = pm[k];
                    if (!x) continue;
                    pm[k] = 0;
                    const int* gk = group.data() + (k << 6);
                    while (x) {
                        lst.push_back(gk[__builtin_ctzll(x)]);
                        x &= x - 1;
                    }
                }
                deg[w] += nmiss;
            };
            if (pool && group.size() >= kPoolMinGroup) {
                std::atomic<size_t> next_a{0};
                pool->run([&](int tid) {
                    auto& pm = pmask[tid];
                    if (pm.size() < pw) pm.resize(pw, 0ull);
                    for (size_t a0; (a0 = next_a.fetch_add(kPoolChunk, std::memory_order_relaxed)) < group.size();)
                        for (size_t a = a0; a < std::min(group.size(), a0 + kPoolChunk); a++) member(a, pm.data());
                });
            } else {
                auto& pm = pmask[0];
                if (pm.size() < pw) pm.resize(pw, 0ull);
                for (size_t a = 0; a < group.size(); a++) member(a, pm.data());
            }
            for (int k = wlo; k <= whi; k++) gmask[k] = 0;
        } else {
            for (size_t a = 0; a < group.size(); a++) {
                const int w = group[a];
                if (ndead[w] > deg[w]) compact(w);
                ++stamp;
                for (int q : nb[w]) seen[q] = stamp;
                for (size_t b = a + 1; b < group.size(); b++) {
                    const int w2 = group[b];
                    if (seen[w2] != stamp) { nb[w].push_back(w2); nb[w2].push_back(w); deg[w]++; deg[w2]++; }
                }
            }
        }
        for (int w : group) {
            key[w] = deg[w] + (tier[w] != 0 ? tier[w] * penalty : 0);
            hp.swim(hp.at[w]);
            hp.sink(hp.at[w]);
        }
        for (int s = step; s < next; s++) { std::vector<int>().swap(nb[perm[s]]); }
        step = next;
        // once few nodes remain (the graph turns dense towards the reference's
        // dense window), adjacency tests go to a bit matrix over the
        // survivors: the clique step then costs |group|^2 bit tests instead of
        // a scan of every survivor's list
        if (bw == 0 && Tfree - step <= kBitsNodes && Tfree - step > 0) {
            const int R = Tfree - step;
            bw = (R + 63) / 64;
            bits.assign(static_cast<size_t>(R) * bw, 0ull);
            const int nth = setup_threads();
            if (nth > 1) {
                pool = std::make_unique<StepPool>(nth);
                pmask.resize(nth);
            }
            gmask.assign(bw, 0ull);
            gpos.assign(R, -1);
            cnode.assign(R, -1);
            alive.assign(bw, 0ull);
            int c = 0;
            for (int k = 1; k <= hp.count; k++) {
                const int v = hp.slot[k];
                if (v >= mf && v < m) continue;          // forced rows: outside the graph
                cnode[c] = v;
                alive[c >> 6] |= 1ull << (c & 63);
                cidx[v] = c++;
            }
            for (int k = 1; k <= hp.count; k++) {
                const int v = hp.slot[k];
                if (cidx[v] < 0) continue;
                uint64_t* row = bits.data() + static_cast<size_t>(cidx[v]) * bw;
                for (int q : nb[v])
                    if (!dead[q] && cidx[q] >= 0) row[cidx[q] >> 6] |= 1ull << (cidx[q] & 63);
            }
        }
    }
    o.denwin = denwin;
    // relabel and sort every column: with the step pool, every column sorted
    // on its own, columns split over the threads; else bucket the entries by
    // row (columns ascending inside a row) and deal the rows out in order
    const size_t nz = lrows.size();
    o.Li.resize(nz);
    if (pool) {
        std::atomic<int> next_s{0};
        pool->run([&](int) {
            constexpr int kCols = 64;
            for (int s0; (s0 = next_s.fetch_add(kCols, std::memory_order_relaxed)) < Tfree;)
                for (int s = s0; s < std::min(Tfree, s0 + kCols); s++) {
                    int* li = o.Li.data() + o.Lp[s];
                    const int len = o.Lp[s + 1] - o.Lp[s];
                    for (int k = 0; k < len; k++) li[k] = iperm[lrows[o.Lp[s] + k]];
                    std::sort(li, li + len);
                }
        });
    } else {
        std::vector<int> rptr(T + 1, 0), rcol(nz);
        for (size_t k = 0; k < nz; k++) rptr[iperm[lrows[k]] + 1]++;
        for (int v = 0; v < T; v++) rptr[v + 1] += rptr[v];
        std::vector<int> fill(rptr.begin(), rptr.end() - 1);
        for (int s = 0; s < Tfree; s++)
            for (int k = o.Lp[s]; k < o.Lp[s + 1]; k++) rcol[fill[iperm[lrows[k]]]++] = s;
        std::copy(o.Lp.begin(), o.Lp.end() - 1, fill.begin());
        for (int r = 0; r < T; r++)
            for (int k = rptr[r]; k < rptr[r + 1]; k++) o.Li[fill[rcol[k]]++] = r;
    }
    std::vector<int>().swap(lrows);
    if (nforced > 0) add_forced_tail(o, m, kA, iA, nforced);
    double na = 0.0;
    for (int v = 0; v < T; v++) { double c = o.Lp[v + 1] - o.Lp[v]; na += c * c; }
    o.narth = na + 3.0 * o.Lp[T] + T;
    return o;
}

KktPlan build_kkt_plan(int m, int n, const int* kA, const int* iA, const int* kAt, const int* iAt, int nforced,
                       double tail_density, const QPattern* q) {
    int leaf = kNdLeafRows;
    if (const char* e = std::getenv("IPO_HIP_ND_LEAF")) leaf = std::max(1, std::atoi(e));
    double relax = kNdRelax;
    if (const char* e = std::getenv("IPO_HIP_ND_RELAX")) relax = std::atof(e);
    KktOrdering o = use_nested_dissection(m + n)
                        ? order_nested_dissection(m, n, kA, iA, kAt, iAt, nforced, leaf, relax, q)
                        : order_tiered_min_degree(m, n, kA, iA, kAt, iAt, nforced, q);
    KktPlan P;
    P.m = m; P.n = n; P.T = o.T;
    const int T = o.T;
    P.perm = o.perm; P.iperm = o.iperm;
    P.lnz = o.Lp[T];
    P.narth = o.narth;
    P.pdf = o.pdf;
    P.denwin = o.denwin;

    std::vector<int> cnt(T);
    for (int j = 0; j < T; j++) cnt[j] = o.Lp[j + 1] - o.Lp[j];

    // ---- dense tail: the maximal suffix of columns whose L column is full
    //      (the reference's dense window, ldlt.c:1027 / :587-590)
    int tc = T;
    if (nforced > 0) {
        tc = T - nforced;               // the tail is exactly the forced rows
    } else {
        while (tc > 0 && cnt[tc - 1] == T - tc) tc--;
        // optionally widen the dense tail to the longest suffix whose lower
        // triangle is still at least `rho` full (structural zeros stay exact
        // zeros in the dense factor): the narrow, tall supernodes just below
        // the reference's dense window then become 64-column MFMA blocks
        // instead of one elimination level each
        if (tail_density < 1.0 && tc < T) {
            double nnz = 0.5 * double(T - tc) * double(T - tc - 1);
            int best = tc;
            for (int j = tc - 1; j >= 0 && T - j <= kTailMaxWiden; j--) {
                nnz += cnt[j];
                const double nt = T - j;
                if (nnz >= tail_density * 0.5 * nt * (nt - 1)) best = j;
                else if (nnz < 0.5 * tail_density * 0.5 * nt * (nt - 1)) break;
            }
            tc = best;
        }
        if (T - tc < kTailMin) tc = T;
    }
    P.tail_c0 = tc;
    P.nt = T - tc;
    P.ntb = (P.nt + kTileRows - 1) / kTileRows;

    // ---- sparse supernodes on [0, tc): column j+1 joins j's panel when
    //      struct(L_j+1) = struct(L_j) \ {j+1}; panels hold <= kPanelCols columns
    P.col0.clear();
    if (tc > 0) {
        P.col0.push_back(0);
        for (int j = 0; j + 1 < tc; j++) {
            const int width = j + 1 - P.col0.back();
            const bool nested = cnt[j] > 0 && o.Li[o.Lp[j]] == j + 1 && cnt[j + 1] == cnt[j] - 1;
            if (!nested || width >= kPanelCols) P.col0.push_back(j + 1);
        }
        P.col0.push_back(tc);
    } else {
        P.col0.push_back(0);
    }
    P.nsup = static_cast<int>(P.col0.size()) - 1;
    const int ns = P.nsup;
    P.sup_of.assign(T, -1);
    for (int s = 0; s < ns; s++)
        for (int j = P.col0[s]; j < P.col0[s + 1]; j++) P.sup_of[j] = s;

    P.rowptr.assign(ns + 1, 0);
    for (int s = 0; s < ns; s++) P.rowptr[s + 1] = P.rowptr[s] + cnt[P.col0[s + 1] - 1];
    P.rows.resize(P.rowptr[ns]);
    P.off.assign(ns + 1, 0);
    for (int s = 0; s < ns; s++) {
        const int last = P.col0[s + 1] - 1;
        std::copy(o.Li.begin() + o.Lp[last], o.Li.begin() + o.Lp[last + 1], P.rows.begin() + P.rowptr[s]);
        const int nc = P.col0[s + 1] - P.col0[s];
        const int h = nc + cnt[last];
        P.off[s + 1] = P.off[s] + static_cast<int64_t>(h) * nc;
        P.max_h = std::max(P.max_h, h);
        P.max_nc = std::max(P.max_nc, nc);
    }
    P.off_tail = P.off[ns];
    P.lx_size = P.off_tail + static_cast<int64_t>(P.nt) * P.nt;

    auto panel_h = [&](int s) { return P.col0[s + 1] - P.col0[s] + (P.rowptr[s + 1] - P.rowptr[s]); };

    // ---- narth (ldlt.c:1243-1248: sum_j c_j^2 + 3 nnz(L) + N) split by the
    //      phase whose kernels do each column's work (SURVEY.md 8(d)'s unit
    //      per phase): a tail column's c_j^2 + 3 c_j + 1 is the dense tail's;
    //      a sparse column's outer product over the rows beyond its supernode,
    //      min(c_j, |R_s|)^2, the gather's; the rest (the products inside the
    //      panel, the scaling, the pivot) the panels'.  The three sum to narth.
    {
        double tail = 0.0, gath = 0.0;
        for (int j = tc; j < T; j++) {
            const double c = cnt[j];
            tail += c * c + 3.0 * c + 1.0;
            P.lnz_tail += cnt[j];
        }
        for (int j = 0; j < tc; j++) {
            const int s = P.sup_of[j];
            const double r = std::min(cnt[j], P.rowptr[s + 1] - P.rowptr[s]);
            gath += r * r;
        }
        P.narth_tail = std::min(tail, P.narth);
        P.narth_gather = std::min(gath, P.narth - P.narth_tail);
        P.narth_panel = P.narth - P.narth_tail - P.narth_gather;
    }

    // ---- sparse supernodal tree + levels (children have smaller indices)
    P.parent.assign(ns, -1);
    P.level.assign(ns, 0);
    for (int s = 0; s < ns; s++) {
        if (P.rowptr[s + 1] > P.rowptr[s]) {
            const int r = P.rows[P.rowptr[s]];
            P.parent[s] = r < tc ? P.sup_of[r] : -1;
        }
    }
    for (int s = 0; s < ns; s++)
        if (P.parent[s] >= 0) P.level[P.parent[s]] = std::max(P.level[P.parent[s]], P.level[s] + 1);
    P.nlevels = 0;
    for (int s = 0; s < ns; s++) P.nlevels = std::max(P.nlevels, P.level[s] + 1);
    P.level_ptr.assign(P.nlevels + 1, 0);
    for (int s = 0; s < ns; s++) P.level_ptr[P.level[s] + 1]++;
    for (int l = 0; l < P.nlevels; l++) P.level_ptr[l + 1] += P.level_ptr[l];
    P.level_sups.resize(ns);
    {
        std::vector<int> fill(P.level_ptr.begin(), P.level_ptr.end() - 1);
        for (int s = 0; s < ns; s++) P.level_sups[fill[P.level[s]]++] = s;
    }

    // ---- sparse update pairs (targets below the tail)
    struct Pair { int tgt, src, r0, r1; };
    std::vector<Pair> pairs;
    P.tail_r0.assign(ns, 0);
    for (int d = 0; d < ns; d++) {
        const int b = P.rowptr[d], e = P.rowptr[d + 1];
        int i = b;
        while (i < e && P.rows[i] < tc) {
            const int t = P.sup_of[P.rows[i]];
            int j = i;
            while (j < e && P.rows[j] < tc && P.sup_of[P.rows[j]] == t) j++;
            pairs.push_back({t, d, i - b, j - b});
            i = j;
        }
        P.tail_r0[d] = i - b;       // R_d[tail_r0 ..] are tail rows
    }
    // grouped by target, sources in ascending order inside a group (a
    // stable counting sort of the source-ordered list)
    P.upd_ptr.assign(ns + 1, 0);
    for (const Pair& q : pairs) P.upd_ptr[q.tgt + 1]++;
    for (int s = 0; s < ns; s++) P.upd_ptr[s + 1] += P.upd_ptr[s];
    {
        std::vector<Pair> sorted(pairs.size());
        std::vector<int> fill(P.upd_ptr.begin(), P.upd_ptr.end() - 1);
        for (const Pair& q : pairs) sorted[fill[q.tgt]++] = q;
        pairs.swap(sorted);
    }
    const size_t np = pairs.size();
    P.upd_src.resize(np); P.upd_r0.resize(np); P.upd_r1.resize(np); P.relptr.assign(np + 1, 0);
    for (size_t q = 0; q < np; q++) {
        const Pair& pr = pairs[q];
        const int hd = P.rowptr[pr.src + 1] - P.rowptr[pr.src];
        P.upd_src[q] = pr.src; P.upd_r0[q] = pr.r0; P.upd_r1[q] = pr.r1;
        P.relptr[q + 1] = P.relptr[q] + (hd - pr.r0);
    }
    P.rel.resize(P.relptr[np]);
    for (size_t q = 0; q < np; q++) {
        const Pair& pr = pairs[q];
        const int* rd = P.rows.data() + P.rowptr[pr.src];
        const int hd = P.rowptr[pr.src + 1] - P.rowptr[pr.src];
        int64_t o2 = P.relptr[q];
        const int c0 = P.col0[pr.tgt], c1 = P.col0[pr.tgt + 1];
        const int* rt = P.rows.data() + P.rowptr[pr.tgt];
        const int ht = P.rowptr[pr.tgt + 1] - P.rowptr[pr.tgt];
        int it = 0;
        for (int i = pr.r0; i < hd; i++) {
            const int row = rd[i];
            if (row < c1) { P.rel[o2++] = row - c0; continue; }
            while (it < ht && rt[it] < row) it++;
            if (it == ht || rt[it] != row) throw std::logic_error("kkt plan: structure not nested");
            P.rel[o2++] = (c1 - c0) + it;
        }
    }

    // ---- sparse GPU work units: (supernode, row tile), level by level
    {
        std::vector<int> unit_first(ns + 1, 0);
        P.unit_level_ptr.assign(P.nlevels + 1, 0);
        for (int l = 0; l < P.nlevels; l++) {
            for (int q = P.level_ptr[l]; q < P.level_ptr[l + 1]; q++) {
                const int s = P.level_sups[q];
                const int nt = (panel_h(s) + kTileRows - 1) / kTileRows;
                unit_first[s] = static_cast<int>(P.unit_sup.size());
                for (int t = 0; t < nt; t++) { P.unit_sup.push_back(s); P.unit_tile.push_back(t); }
            }
            P.unit_level_ptr[l + 1] = static_cast<int>(P.unit_sup.size());
        }
        const int nu = static_cast<int>(P.unit_sup.size());
        std::vector<std::vector<int>> tk(nu);
        for (int s = 0; s < ns; s++) {
            for (int q = P.upd_ptr[s]; q < P.upd_ptr[s + 1]; q++) {
                const int len = static_cast<int>(P.relptr[q + 1] - P.relptr[q]);
                const int* rl = P.rel.data() + P.relptr[q];
                int i = 0;
                while (i < len) {
                    const int t = rl[i] / kTileRows;
                    int j = i;
                    while (j < len && rl[j] / kTileRows == t) j++;
                    auto& v = tk[unit_first[s] + t];
                    v.push_back(q); v.push_back(i); v.push_back(j);
                    i = j;
                }
            }
        }
        P.task_ptr.assign(nu + 1, 0);
        for (int u = 0; u < nu; u++) P.task_ptr[u + 1] = P.task_ptr[u] + static_cast<int>(tk[u].size() / 3);
        P.task_pair.resize(P.task_ptr[nu]); P.task_i0.resize(P.task_ptr[nu]); P.task_i1.resize(P.task_ptr[nu]);
        P.utasks.resize(P.task_ptr[nu]);
        for (int u = 0; u < nu; u++) {
            const int s = P.unit_sup[u];
            const int nc = P.col0[s + 1] - P.col0[s];
            for (size_t e = 0; e < tk[u].size() / 3; e++) {
                const int q = tk[u][3 * e], i0 = tk[u][3 * e + 1], i1 = tk[u][3 * e + 2];
                P.task_pair[P.task_ptr[u] + e] = q;
                P.task_i0[P.task_ptr[u] + e] = i0;
                P.task_i1[P.task_ptr[u] + e] = i1;
                const int* rl = P.rel.data() + P.relptr[q];
                {
                    TailTask tt{};
                    tt.src = P.upd_src[q];
                    tt.rbase = P.upd_r0[q] + i0;
                    tt.cbase = P.upd_r0[q];
                    const int rb = P.unit_tile[u] * kTileRows;
                    for (int i = i0; i < i1; i++) tt.rmask |= 1ull << (rl[i] - rb);
                    for (int jj = 0; jj < P.upd_r1[q] - P.upd_r0[q]; jj++) tt.cmask |= 1ull << rl[jj];
                    P.utasks[P.task_ptr[u] + e] = tt;
                }
                const double ncd = P.col0[P.upd_src[q] + 1] - P.col0[P.upd_src[q]];
                const int ncols = P.upd_r1[q] - P.upd_r0[q];
                long prs = 0;
                for (int jj = 0; jj < ncols; jj++) {
                    const int* lo = std::lower_bound(rl + i0, rl + i1, rl[jj]);
                    prs += (rl + i1) - lo;
                }
                P.flops_update += 3.0 * ncd * prs;
                P.bytes_update += 8.0 * ncd * ((i1 - i0) + ncols);
            }
            if (!tk[u].empty()) {
                const int rows = std::min(kTileRows, panel_h(s) - P.unit_tile[u] * kTileRows);
                P.bytes_update += 16.0 * rows * nc;
            }
        }
    }

    // ---- dense-tail gather tasks: every sparse supernode with tail rows
    //      touches the 64x64 tiles (bi >= bj) its tail rows span
    if (P.nt > 0) {
        const int nb = P.ntb;
        const int ntiles = nb * (nb + 1) / 2;
        std::vector<std::vector<TailTask>> tt(ntiles);
        for (int d = 0; d < ns; d++) {
            const int b = P.rowptr[d], e = P.rowptr[d + 1];
            const int q0 = b + P.tail_r0[d];
            if (q0 >= e) continue;
            // segments of tail rows per 64-row block
            std::vector<int> sb, ss, se;
            std::vector<uint64_t> sm;
            int i = q0;
            while (i < e) {
                const int blk = (P.rows[i] - tc) / kTileRows;
                int j = i;
                uint64_t mask = 0;
                while (j < e && (P.rows[j] - tc) / kTileRows == blk) { mask |= 1ull << ((P.rows[j] - tc) % kTileRows); j++; }
                sb.push_back(blk); ss.push_back(i - b); se.push_back(j - b); sm.push_back(mask);
                i = j;
            }
            const double ncd = P.col0[d + 1] - P.col0[d];
            for (size_t x = 0; x < sb.size(); x++)
                for (size_t y = 0; y <= x; y++) {
                    TailTask t{};
                    t.src = d;
                    t.rbase = ss[x]; t.cbase = ss[y];
                    t.rmask = sm[x]; t.cmask = sm[y];
                    tt[sb[x] * (sb[x] + 1) / 2 + sb[y]].push_back(t);
                    const double ra = se[x] - ss[x], rc = se[y] - ss[y];
                    P.flops_tail_update += 3.0 * ncd * ra * rc;
                    P.bytes_tail_update += 8.0 * ncd * (ra + rc);
                }
        }
        P.tail_task_ptr.assign(ntiles + 1, 0);
        for (int t = 0; t < ntiles; t++) P.tail_task_ptr[t + 1] = P.tail_task_ptr[t] + static_cast<int>(tt[t].size());
        P.tail_tasks.reserve(P.tail_task_ptr[ntiles]);
        for (int t = 0; t < ntiles; t++) P.tail_tasks.insert(P.tail_tasks.end(), tt[t].begin(), tt[t].end());
        const double N = P.nt;
        P.flops_tail_factor = N * N * N / 3.0 * 2.0;
    }

    // ---- k-slot lists (inner dimension of the MFMA gather)
    {
        auto build = [&](const std::vector<int>& tptr, const std::vector<TailTask>& tasks, std::vector<int>& ks,
                         std::vector<int>& kp) {
            const int nu = static_cast<int>(tptr.size()) - 1;
            if (static_cast<int64_t>(tasks.size()) >= (int64_t(1) << 25))
                throw std::length_error("kkt plan: too many gather tasks for 25-bit slot ids");
            kp.assign(nu + 1, 0);
            ks.clear();
            for (int u = 0; u < nu; u++) {
                for (int t = tptr[u]; t < tptr[u + 1]; t++) {
                    const int d = tasks[t].src, ncd = P.col0[d + 1] - P.col0[d];
                    for (int k = 0; k < ncd; k++) ks.push_back((t << 6) | k);
                }
                while (ks.size() % kSlab) ks.push_back(-1);
                kp[u + 1] = static_cast<int>(ks.size());
            }
        };
        build(P.task_ptr, P.utasks, P.kslot, P.kslot_ptr);
        if (P.nt > 0) build(P.tail_task_ptr, P.tail_tasks, P.tail_kslot, P.tail_kslot_ptr);
    }

    // ---- forward-solve update lists (rows of every sparse panel, by row)
    {
        P.yrow_ptr.assign(T + 1, 0);
        for (int i = 0; i < P.rowptr[ns]; i++) P.yrow_ptr[P.rows[i] + 1]++;
        for (int v = 0; v < T; v++) P.yrow_ptr[v + 1] += P.yrow_ptr[v];
        P.yrow_idx.resize(P.yrow_ptr[T]);
        std::vector<int> fill(P.yrow_ptr.begin(), P.yrow_ptr.end() - 1);
        for (int i = 0; i < P.rowptr[ns]; i++) P.yrow_idx[fill[P.rows[i]]++] = i;
    }

    for (int s = 0; s < ns; s++) {
        const double nc = P.col0[s + 1] - P.col0[s], h = panel_h(s);
        P.flops_factor += nc * nc * nc / 3.0 + (h - nc) * nc * nc;
    }
    P.flops_factor += P.flops_update * 2.0 / 3.0 + P.flops_tail_update * 2.0 / 3.0 + P.flops_tail_factor;

    // ---- assembly maps
    auto slot_of = [&](int row, int col) -> int64_t {   // row >= col, new indices
        if (col >= tc) return P.off_tail + static_cast<int64_t>(col - tc) * P.nt + (row - tc);
        const int s = P.sup_of[col];
        const int c0 = P.col0[s], c1 = P.col0[s + 1];
        const int h = panel_h(s);
        int pos;
        if (row < c1) pos = row - c0;
        else {
            auto bgn = P.rows.begin() + P.rowptr[s], end = P.rows.begin() + P.rowptr[s + 1];
            auto it = std::lower_bound(bgn, end, row);
            if (it == end || *it != row) throw std::logic_error("kkt plan: A entry outside the pattern");
            pos = (c1 - c0) + static_cast<int>(it - bgn);
        }
        return P.off[s] + static_cast<int64_t>(col - c0) * h + pos;
    };
    P.dslot.resize(T);
    P.dsign.resize(T);
    for (int v = 0; v < T; v++) {
        P.dslot[v] = slot_of(v, v);
        P.dsign[v] = P.perm[v] < m ? -1 : 1;
    }
    P.amap.resize(kA[n]);
    for (int c = 0; c < n; c++)
        for (int k = kA[c]; k < kA[c + 1]; k++) {
            const int a = P.iperm[iA[k]], b = P.iperm[m + c];
            P.amap[k] = slot_of(std::max(a, b), std::min(a, b));
        }
    if (q && q->kQ) {       // ldlt.c:253-256: row > col stored, row == col on the diagonal
        P.qmap.resize(q->kQ[m]);
        for (int j = 0; j < m; j++)
            for (int k = q->kQ[j]; k < q->kQ[j + 1]; k++) {
                const int row = P.iperm[q->iQ[k]], col = P.iperm[j];
                P.qmap[k] = row > col ? slot_of(row, col) : row == col ? -2 : -1;
            }
    }
    return P;
}

}  // namespace ipo
