// synth.h -- synthetic LPs of BASELINE.json configs[3] and configs[4]
// (SURVEY.md §8(d) "Configs as inputs", items 4 and 5).
//
// Both are handed to solver() directly in its own form
//      max c'x  s.t.  Ax <= b, x >= 0         (src/common/solve.c:225-235)
// and are feasible and bounded by construction: with x*, w*, y*, z* drawn
// from U[0.5, 1.5],  b = A x* + w*  and  c = A' y* - z*,  so x* is primal
// feasible and y* dual feasible (A'y* - c = z* > 0).
//
// Random:        m rows, n columns, exactly `per_col` distinct rows per
//                column, values U[-1,1] with |v| >= 0.1.  band = 0: rows
//                uniform over [0, m); band > 0: rows from a window of width
//                `band` centred on floor(j m / n) (clipped to [0, m)), which
//                keeps the fill of an exact factorisation bounded.
// Block-angular: `nblocks` diagonal blocks of mb x nb (banded random as
//                above, block-local), followed by `nlink` linking rows with
//                `link_nz` nonzeros each, spread uniformly over all columns.
//                Rows: block k owns [k mb, (k+1) mb), linking rows last.
//                Columns: block k owns [k nb, (k+1) nb).
//
// Every random draw is a pure function of (seed, stream, index) via
// splitmix64, so each column and each linking row can be generated
// independently (and in parallel) with the same result.
#pragma once
#include <cstdint>
#include <vector>

namespace ipo {

struct SynthLP {
    int m = 0, n = 0;
    std::vector<int> kA, iA;          // CSC, rows ascending in each column
    std::vector<double> A, b, c;
    std::vector<double> xs, ws, ys, zs;   // the interior point the data was built from
};

void synth_random(int m, int n, int per_col, int band, uint64_t seed, SynthLP& out);
void synth_block_angular(int nblocks, int mb, int nb, int per_col, int band, int nlink, int link_nz,
                         uint64_t seed, SynthLP& out);

}  // namespace ipo
