// synth.cpp -- synthetic LP generators (see synth.h).
#include "synth.h"

#include <algorithm>
#include <stdexcept>
#include <string>

namespace ipo {
namespace {

inline uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

// Independent stream per (seed, stream id, index).
struct Rng {
    uint64_t s;
    Rng(uint64_t seed, uint64_t stream, uint64_t idx)
        : s(splitmix64(splitmix64(seed ^ (stream * 0xD1B54A32D192ED03ull)) + idx)) {}
    uint64_t next() { s = splitmix64(s); return s; }
    double unif() { return static_cast<double>(next() >> 11) * 0x1.0p-53; }
    uint64_t below(uint64_t k) { return next() % k; }   // k << 2^64: bias negligible
};

enum Stream : uint64_t { kRows = 1, kVals = 2, kX = 3, kW = 4, kY = 5, kZ = 6, kLinkCols = 7, kLinkVals = 8 };

// value U[-1,1] with |v| >= 0.1
inline double draw_value(Rng& r) {
    const double mag = 0.1 + 0.9 * r.unif();
    return (r.next() & 1) ? -mag : mag;
}

// per_col distinct sorted rows of a column from [lo, lo + width)
void draw_rows(Rng& r, int lo, int width, int per_col, int* out) {
    int k = 0;
    while (k < per_col) {
        const int v = lo + static_cast<int>(r.below(static_cast<uint64_t>(width)));
        bool dup = false;
        for (int q = 0; q < k; q++) dup |= (out[q] == v);
        if (!dup) out[k++] = v;
    }
    std::sort(out, out + per_col);
}

void window(int64_t center, int band, int m, int* lo, int* width) {
    if (band <= 0 || band >= m) { *lo = 0; *width = m; return; }
    int64_t l = center - band / 2;
    if (l < 0) l = 0;
    if (l + band > m) l = m - band;
    *lo = static_cast<int>(l);
    *width = band;
}

void check(bool ok, const char* what) {
    if (!ok) throw std::invalid_argument(std::string("synth: ") + what);
}

void interior_point(SynthLP& o, uint64_t seed) {
    o.xs.resize(o.n); o.zs.resize(o.n); o.ws.resize(o.m); o.ys.resize(o.m);
    for (int j = 0; j < o.n; j++) {
        Rng rx(seed, kX, j), rz(seed, kZ, j);
        o.xs[j] = 0.5 + rx.unif();
        o.zs[j] = 0.5 + rz.unif();
    }
    for (int i = 0; i < o.m; i++) {
        Rng rw(seed, kW, i), ry(seed, kY, i);
        o.ws[i] = 0.5 + rw.unif();
        o.ys[i] = 0.5 + ry.unif();
    }
    // b = A x* + w*,  c = A' y* - z*  (column order, fixed)
    o.b.assign(o.m, 0.0);
    o.c.assign(o.n, 0.0);
    for (int j = 0; j < o.n; j++) {
        double cj = 0.0;
        for (int k = o.kA[j]; k < o.kA[j + 1]; k++) {
            o.b[o.iA[k]] += o.A[k] * o.xs[j];
            cj += o.A[k] * o.ys[o.iA[k]];
        }
        o.c[j] = cj - o.zs[j];
    }
    for (int i = 0; i < o.m; i++) o.b[i] += o.ws[i];
}

}  // namespace

void synth_random(int m, int n, int per_col, int band, uint64_t seed, SynthLP& o) {
    check(m > 0 && n > 0 && per_col > 0, "sizes must be positive");
    const int wmin = (band <= 0 || band >= m) ? m : band;
    check(per_col <= wmin, "per_col exceeds the row window");
    check(static_cast<int64_t>(n) * per_col < (int64_t(1) << 31), "nnz exceeds int32");
    o = SynthLP();
    o.m = m; o.n = n;
    o.kA.resize(n + 1);
    o.iA.resize(static_cast<size_t>(n) * per_col);
    o.A.resize(o.iA.size());
    for (int j = 0; j < n; j++) {
        o.kA[j] = j * per_col;
        int lo, width;
        window(static_cast<int64_t>(j) * m / n, band, m, &lo, &width);
        Rng rr(seed, kRows, j), rv(seed, kVals, j);
        draw_rows(rr, lo, width, per_col, &o.iA[o.kA[j]]);
        for (int q = 0; q < per_col; q++) o.A[o.kA[j] + q] = draw_value(rv);
    }
    o.kA[n] = n * per_col;
    interior_point(o, seed);
}

void synth_block_angular(int nblocks, int mb, int nb, int per_col, int band, int nlink, int link_nz,
                         uint64_t seed, SynthLP& o) {
    check(nblocks > 0 && mb > 0 && nb > 0 && per_col > 0 && nlink >= 0 && link_nz >= 0, "bad sizes");
    const int64_t m64 = static_cast<int64_t>(nblocks) * mb + nlink;
    const int64_t n64 = static_cast<int64_t>(nblocks) * nb;
    check(m64 < (int64_t(1) << 31) && n64 < (int64_t(1) << 31), "dimensions exceed int32");
    check(link_nz <= n64, "link_nz exceeds the column count");
    const int wmin = (band <= 0 || band >= mb) ? mb : band;
    check(per_col <= wmin, "per_col exceeds the row window");
    const int64_t nz64 = n64 * per_col + static_cast<int64_t>(nlink) * link_nz;
    check(nz64 < (int64_t(1) << 31), "nnz exceeds int32");
    o = SynthLP();
    o.m = static_cast<int>(m64);
    o.n = static_cast<int>(n64);
    const int n = o.n;

    // linking rows: link_nz distinct uniform columns each
    std::vector<int> lcnt(n + 1, 0);
    std::vector<int> lcol(static_cast<size_t>(nlink) * link_nz);
    std::vector<double> lval(lcol.size());
    {
        std::vector<int> tmp;
        for (int t = 0; t < nlink; t++) {
            Rng rc(seed, kLinkCols, t), rv(seed, kLinkVals, t);
            tmp.clear();
            // rejection against a sorted set: link_nz << n in the configs
            while (static_cast<int>(tmp.size()) < link_nz) {
                const int v = static_cast<int>(rc.below(static_cast<uint64_t>(n)));
                auto it = std::lower_bound(tmp.begin(), tmp.end(), v);
                if (it == tmp.end() || *it != v) tmp.insert(it, v);
            }
            for (int q = 0; q < link_nz; q++) {
                lcol[static_cast<size_t>(t) * link_nz + q] = tmp[q];
                lval[static_cast<size_t>(t) * link_nz + q] = draw_value(rv);
                lcnt[tmp[q] + 1]++;
            }
        }
        for (int j = 0; j < n; j++) lcnt[j + 1] += lcnt[j];
    }
    // CSC: block entries (rows of the column's block), then linking rows
    // (all larger than any block row) in ascending t
    std::vector<int> lrow(lcol.size());
    std::vector<double> lv2(lcol.size());
    {
        std::vector<int> fill(lcnt.begin(), lcnt.end() - 1);
        for (int t = 0; t < nlink; t++)
            for (int q = 0; q < link_nz; q++) {
                const size_t e = static_cast<size_t>(t) * link_nz + q;
                const int p = fill[lcol[e]]++;
                lrow[p] = nblocks * mb + t;
                lv2[p] = lval[e];
            }
    }
    o.kA.resize(n + 1);
    o.iA.resize(static_cast<size_t>(nz64));
    o.A.resize(static_cast<size_t>(nz64));
    int pos = 0;
    for (int j = 0; j < n; j++) {
        o.kA[j] = pos;
        const int blk = j / nb, jl = j % nb;
        int lo, width;
        window(static_cast<int64_t>(jl) * mb / nb, band, mb, &lo, &width);
        Rng rr(seed, kRows, j), rv(seed, kVals, j);
        draw_rows(rr, lo, width, per_col, &o.iA[pos]);
        for (int q = 0; q < per_col; q++) {
            o.iA[pos + q] += blk * mb;
            o.A[pos + q] = draw_value(rv);
        }
        pos += per_col;
        for (int p = lcnt[j]; p < lcnt[j + 1]; p++) {
            o.iA[pos] = lrow[p];
            o.A[pos] = lv2[p];
            pos++;
        }
    }
    o.kA[n] = pos;
    interior_point(o, seed);
}

}  // namespace ipo
