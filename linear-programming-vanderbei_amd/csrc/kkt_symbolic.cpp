// kkt_symbolic.cpp -- host symbolic phase for the GPU KKT factorisation.
// See kkt_plan.h.  Reference behaviour restated (not translated):
//   ordering   src/ipo/ldlt.c:638-858 (inv_sym), :860-1262 (lltsym)
//   heap       src/ipo/ldlt.c:1305-1349
#include "kkt_plan.h"

#include <algorithm>
#include <cmath>
#include <stdexcept>

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

}  // namespace

KktOrdering order_tiered_min_degree(int m, int n, const int* kA, const int* iA,
                                    const int* kAt, const int* iAt) {
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
    o.pdf = (3 * fill_y_first <= fill_x_first) ? 1 : 2;

    // adjacency of K, y-node r lists its x-nodes (column order), x-node c its rows
    std::vector<std::vector<int>> nb(T);
    std::vector<int> tier(T);
    for (int r = 0; r < m; r++) {
        nb[r].reserve(kAt[r + 1] - kAt[r]);
        for (int k = kAt[r]; k < kAt[r + 1]; k++) nb[r].push_back(m + iAt[k]);
        tier[r] = o.pdf == 1 ? 0 : 1;
    }
    for (int c = 0; c < n; c++) {
        nb[m + c].reserve(kA[c + 1] - kA[c]);
        for (int k = kA[c]; k < kA[c + 1]; k++) nb[m + c].push_back(iA[k]);
        tier[m + c] = o.pdf == 1 ? 1 : 0;
    }
    // the reference's dense-column threshold always evaluates to 3 for ipo
    // (no free variables, no finite ranges: ldlt.c:814-846)
    const int dense_deg = 3;
    const int penalty = T;

    std::vector<int> key(T);
    for (int v = 0; v < T; v++) {
        int d = static_cast<int>(nb[v].size());
        if (d > dense_deg && tier[v] == 0) tier[v] = 1;
        key[v] = d + tier[v] * penalty;
    }
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
    while (step < T) {
        const int piv = hp.slot[1];
        const int dg = static_cast<int>(nb[piv].size());
        if (dg >= T - 1 - step) denwin = step;
        perm[step] = piv;
        iperm[piv] = step;

        // neighbours are tagged with the current step; twins (same degree,
        // same tier, neighbourhood inside piv's closed neighbourhood) are
        // eliminated together with piv
        int next = step + 1;
        group.clear();
        for (int w : nb[piv]) iperm[w] = step;
        for (int w : nb[piv]) {
            bool twin = false;
            if (static_cast<int>(nb[w].size()) == dg && tier[w] == tier[piv]) {
                twin = true;
                for (int q : nb[w]) if (iperm[q] < step) { twin = false; break; }
            }
            if (twin) { perm[next] = w; iperm[w] = next; next++; }
            else group.push_back(w);
        }

        int width = dg;
        for (int s = step; s < next; s++) {
            const int v = perm[s];
            o.Lp[s + 1] = o.Lp[s] + width;
            for (int w : nb[v]) {
                int r = iperm[w];
                if (r > s || (r == step && w != piv)) lrows.push_back(w);
            }
            width--;
        }

        for (int w : group) {                    // drop piv from the survivors
            auto& lst = nb[w];
            lst.erase(std::find(lst.begin(), lst.end(), piv));
        }
        if (next > step + 1) {                   // ... and the twins
            for (int w : group) {
                auto& lst = nb[w];
                lst.erase(std::remove_if(lst.begin(), lst.end(),
                                         [&](int q) { return iperm[q] > step; }),
                          lst.end());
            }
        }
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
        for (size_t a = 0; a < group.size(); a++) {   // clique on the survivors
            const int w = group[a];
            ++stamp;
            for (int q : nb[w]) seen[q] = stamp;
            for (size_t b = a + 1; b < group.size(); b++) {
                const int w2 = group[b];
                if (seen[w2] != stamp) { nb[w].push_back(w2); nb[w2].push_back(w); }
            }
        }
        for (int w : group) {
            key[w] = static_cast<int>(nb[w].size()) + (tier[w] != 0 ? tier[w] * penalty : 0);
            hp.swim(hp.at[w]);
            hp.sink(hp.at[w]);
        }
        for (int s = step; s < next; s++) { std::vector<int>().swap(nb[perm[s]]); }
        step = next;
    }
    o.denwin = denwin;
    o.Li.resize(lrows.size());
    for (size_t k = 0; k < lrows.size(); k++) o.Li[k] = iperm[lrows[k]];
    for (int v = 0; v < T; v++) std::sort(o.Li.begin() + o.Lp[v], o.Li.begin() + o.Lp[v + 1]);
    double na = 0.0;
    for (int v = 0; v < T; v++) { double c = o.Lp[v + 1] - o.Lp[v]; na += c * c; }
    o.narth = na + 3.0 * o.Lp[T] + T;
    return o;
}

KktPlan build_kkt_plan(int m, int n, const int* kA, const int* iA, const int* kAt, const int* iAt) {
    KktOrdering o = order_tiered_min_degree(m, n, kA, iA, kAt, iAt);
    KktPlan P;
    P.m = m; P.n = n; P.T = o.T;
    const int T = o.T;
    P.perm = o.perm; P.iperm = o.iperm;
    P.lnz = o.Lp[T];
    P.narth = o.narth;
    P.pdf = o.pdf;
    P.denwin = o.denwin;

    // ---- supernodes: column j+1 joins j's panel when struct(L_j+1) = struct(L_j) \ {j+1}
    std::vector<int> cnt(T);
    for (int j = 0; j < T; j++) cnt[j] = o.Lp[j + 1] - o.Lp[j];
    P.col0.clear();
    P.col0.push_back(0);
    for (int j = 0; j + 1 < T; j++) {
        const int width = j + 1 - P.col0.back();
        const bool nested = cnt[j] > 0 && o.Li[o.Lp[j]] == j + 1 && cnt[j + 1] == cnt[j] - 1;
        if (!nested || width >= kPanelCols) P.col0.push_back(j + 1);
    }
    P.col0.push_back(T);
    P.nsup = static_cast<int>(P.col0.size()) - 1;
    const int ns = P.nsup;

    P.sup_of.assign(T, 0);
    for (int s = 0; s < ns; s++)
        for (int j = P.col0[s]; j < P.col0[s + 1]; j++) P.sup_of[j] = s;

    // below-block rows of each panel = rows of its last column
    P.rowptr.assign(ns + 1, 0);
    for (int s = 0; s < ns; s++) {
        const int last = P.col0[s + 1] - 1;
        P.rowptr[s + 1] = P.rowptr[s] + cnt[last];
    }
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
    P.lx_size = P.off[ns];

    // ---- supernodal tree + levels (children have smaller indices)
    P.parent.assign(ns, -1);
    P.level.assign(ns, 0);
    for (int s = 0; s < ns; s++) {
        if (P.rowptr[s + 1] > P.rowptr[s]) P.parent[s] = P.sup_of[P.rows[P.rowptr[s]]];
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

    // position of a global row inside panel s
    auto panel_pos = [&](int s, int row) -> int {
        const int c0 = P.col0[s], c1 = P.col0[s + 1];
        if (row < c1) return row - c0;
        auto b = P.rows.begin() + P.rowptr[s], e = P.rows.begin() + P.rowptr[s + 1];
        auto it = std::lower_bound(b, e, row);
        if (it == e || *it != row) throw std::logic_error("kkt plan: row not in target panel");
        return (c1 - c0) + static_cast<int>(it - b);
    };

    // ---- update pairs: source d touches every supernode owning one of its rows
    struct Pair { int tgt, src, r0, r1; };
    std::vector<Pair> pairs;
    for (int d = 0; d < ns; d++) {
        const int b = P.rowptr[d], e = P.rowptr[d + 1];
        int i = b;
        while (i < e) {
            const int t = P.sup_of[P.rows[i]];
            int j = i;
            while (j < e && P.sup_of[P.rows[j]] == t) j++;
            pairs.push_back({t, d, i - b, j - b});
            i = j;
        }
    }
    std::stable_sort(pairs.begin(), pairs.end(), [](const Pair& a, const Pair& b) { return a.tgt < b.tgt; });
    P.upd_ptr.assign(ns + 1, 0);
    for (const Pair& p : pairs) P.upd_ptr[p.tgt + 1]++;
    for (int s = 0; s < ns; s++) P.upd_ptr[s + 1] += P.upd_ptr[s];
    const size_t np = pairs.size();
    P.upd_src.resize(np); P.upd_r0.resize(np); P.upd_r1.resize(np); P.relptr.assign(np + 1, 0);
    for (size_t q = 0; q < np; q++) {
        const Pair& p = pairs[q];
        const int hd = P.rowptr[p.src + 1] - P.rowptr[p.src];
        P.upd_src[q] = p.src; P.upd_r0[q] = p.r0; P.upd_r1[q] = p.r1;
        P.relptr[q + 1] = P.relptr[q] + (hd - p.r0);
        const double ra = hd - p.r0, rc = p.r1 - p.r0, nc = P.col0[p.src + 1] - P.col0[p.src];
        P.flops_factor += 2.0 * nc * rc * (ra - 0.5 * rc);
    }
    P.rel.resize(P.relptr[np]);
    for (size_t q = 0; q < np; q++) {
        const Pair& p = pairs[q];
        const int* rd = P.rows.data() + P.rowptr[p.src];
        const int hd = P.rowptr[p.src + 1] - P.rowptr[p.src];
        int64_t o2 = P.relptr[q];
        // rows are sorted in both lists: merge instead of searching
        const int c0 = P.col0[p.tgt], c1 = P.col0[p.tgt + 1];
        const int* rt = P.rows.data() + P.rowptr[p.tgt];
        const int ht = P.rowptr[p.tgt + 1] - P.rowptr[p.tgt];
        int it = 0;
        for (int i = p.r0; i < hd; i++) {
            const int row = rd[i];
            if (row < c1) { P.rel[o2++] = row - c0; continue; }
            while (it < ht && rt[it] < row) it++;
            if (it == ht || rt[it] != row) throw std::logic_error("kkt plan: structure not nested");
            P.rel[o2++] = (c1 - c0) + it;
        }
    }
    for (int s = 0; s < ns; s++) {      // dense factor + trsm of each panel
        const double nc = P.col0[s + 1] - P.col0[s], h = nc + (P.rowptr[s + 1] - P.rowptr[s]);
        P.flops_factor += nc * nc * nc / 3.0 + (h - nc) * nc * nc;
    }

    // ---- GPU work units: (supernode, row tile), level by level
    {
        std::vector<int> unit_first(ns + 1, 0);      // first unit of supernode s
        P.unit_level_ptr.assign(P.nlevels + 1, 0);
        for (int l = 0; l < P.nlevels; l++) {
            for (int q = P.level_ptr[l]; q < P.level_ptr[l + 1]; q++) {
                const int s = P.level_sups[q];
                const int h = P.col0[s + 1] - P.col0[s] + (P.rowptr[s + 1] - P.rowptr[s]);
                const int nt = (h + kTileRows - 1) / kTileRows;
                unit_first[s] = static_cast<int>(P.unit_sup.size());
                for (int t = 0; t < nt; t++) { P.unit_sup.push_back(s); P.unit_tile.push_back(t); }
            }
            P.unit_level_ptr[l + 1] = static_cast<int>(P.unit_sup.size());
        }
        const int nu = static_cast<int>(P.unit_sup.size());
        std::vector<std::vector<int>> tk(nu);          // flattened (pair, i0, i1)
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
        // exact work of the gather kernel: every (i, j) pair with panel row >= panel col
        for (int u = 0; u < nu; u++) {
            const int s = P.unit_sup[u];
            for (size_t e = 0; e < tk[u].size() / 3; e++) {
                const int q = tk[u][3 * e], i0 = tk[u][3 * e + 1], i1 = tk[u][3 * e + 2];
                const int* rl = P.rel.data() + P.relptr[q];
                const int d = P.upd_src[q];
                const double ncd = P.col0[d + 1] - P.col0[d];
                const int ncols = P.upd_r1[q] - P.upd_r0[q];
                long pairs = 0;
                for (int jj = 0; jj < ncols; jj++) {
                    // rows i in [i0, i1) with rl[i] >= rl[jj]; rl ascending
                    const int* lo = std::lower_bound(rl + i0, rl + i1, rl[jj]);
                    pairs += (rl + i1) - lo;
                }
                P.flops_update += pairs * ncd * 3.0;
                P.bytes_update += 8.0 * ncd * ((i1 - i0) + ncols);   // L_d rows read once per task
                (void)s;
            }
        }
        for (int u = 0; u < nu; u++) {   // panel tile read-modify-write
            const int s = P.unit_sup[u];
            if (P.task_ptr.empty() && tk[u].empty()) continue;
            if (tk[u].empty()) continue;
            const int nc = P.col0[s + 1] - P.col0[s];
            const int h = nc + (P.rowptr[s + 1] - P.rowptr[s]);
            const int rows = std::min(kTileRows, h - P.unit_tile[u] * kTileRows);
            P.bytes_update += 16.0 * rows * nc;
        }
        P.task_ptr.assign(nu + 1, 0);
        for (int u = 0; u < nu; u++) P.task_ptr[u + 1] = P.task_ptr[u] + static_cast<int>(tk[u].size() / 3);
        P.task_pair.resize(P.task_ptr[nu]); P.task_i0.resize(P.task_ptr[nu]); P.task_i1.resize(P.task_ptr[nu]);
        for (int u = 0; u < nu; u++) {
            for (size_t e = 0; e < tk[u].size() / 3; e++) {
                P.task_pair[P.task_ptr[u] + e] = tk[u][3 * e];
                P.task_i0[P.task_ptr[u] + e] = tk[u][3 * e + 1];
                P.task_i1[P.task_ptr[u] + e] = tk[u][3 * e + 2];
            }
        }
    }
    // ---- forward-solve row lists (entries outside the row's own panel)
    {
        P.frow_ptr.assign(T + 1, 0);
        for (int d = 0; d < ns; d++) {
            const int nc = P.col0[d + 1] - P.col0[d];
            for (int i = P.rowptr[d]; i < P.rowptr[d + 1]; i++) P.frow_ptr[P.rows[i] + 1] += nc;
        }
        for (int v = 0; v < T; v++) P.frow_ptr[v + 1] += P.frow_ptr[v];
        P.frow_col.resize(P.frow_ptr[T]);
        P.frow_pos.resize(P.frow_ptr[T]);
        std::vector<int> fill(P.frow_ptr.begin(), P.frow_ptr.end() - 1);
        for (int d = 0; d < ns; d++) {
            const int nc = P.col0[d + 1] - P.col0[d];
            const int hb = P.rowptr[d + 1] - P.rowptr[d];
            const int h = nc + hb;
            for (int k = 0; k < nc; k++)
                for (int i = 0; i < hb; i++) {
                    const int row = P.rows[P.rowptr[d] + i];
                    const int e = fill[row]++;
                    P.frow_col[e] = P.col0[d] + k;
                    P.frow_pos[e] = P.off[d] + static_cast<int64_t>(k) * h + nc + i;
                }
        }
    }

    // ---- assembly maps
    P.dslot.resize(T);
    P.dsign.resize(T);
    for (int v = 0; v < T; v++) {
        const int s = P.sup_of[v];
        const int h = P.col0[s + 1] - P.col0[s] + (P.rowptr[s + 1] - P.rowptr[s]);
        const int lc = v - P.col0[s];
        P.dslot[v] = P.off[s] + static_cast<int64_t>(lc) * h + lc;
        P.dsign[v] = P.perm[v] < m ? -1 : 1;
    }
    P.amap.resize(kA[n]);
    for (int c = 0; c < n; c++) {
        for (int k = kA[c]; k < kA[c + 1]; k++) {
            const int a = P.iperm[iA[k]], b = P.iperm[m + c];
            const int col = std::min(a, b), row = std::max(a, b);
            const int s = P.sup_of[col];
            const int h = P.col0[s + 1] - P.col0[s] + (P.rowptr[s + 1] - P.rowptr[s]);
            P.amap[k] = P.off[s] + static_cast<int64_t>(col - P.col0[s]) * h + panel_pos(s, row);
        }
    }
    return P;
}

}  // namespace ipo
