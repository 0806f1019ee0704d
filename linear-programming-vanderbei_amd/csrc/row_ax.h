// row_ax.h -- A x by rows in column slices of x (host interface; the kernel
// is k_rows_ax_jds in dev_common.hip).
#pragma once
#include <hip/hip_runtime.h>

#include <vector>

#include "hip_util.h"

namespace ipo {

// A x by rows through jagged diagonals (bitwise sparse_dot's sums, see
// k_rows_ax_jds) when x exceeds kAxSliceBytes: rows_ax_blocks(n) = the
// column slices, one pass each (default 1; IPO_HIP_AX_BLOCKS overrides).  RowAxPlan holds A's
// entries by slice in jagged-diagonal order (built once, on the host, from
// the CSC of A); launch() writes ax[m], one kernel per pass.
constexpr long kAxSliceBytes = 2l << 20;
int rows_ax_blocks(int n);
// whether A x goes through a RowAxPlan: more than one slice, or
// IPO_HIP_AX_JDS=1 (jagged diagonals over a single slice)
bool rows_ax_sliced(int n);
class RowAxPlan {
  public:
    void build(int m, int n, const int* kA, const int* iA, const double* A, int npass, hipStream_t st);
    void launch(const double* x, double* ax, hipStream_t st) const;
    int passes() const { return np_; }

  private:
    int m_ = 0, np_ = 0;
    std::vector<int> rows_, nd_, dbase_;        // per pass: rows launched, diagonals, offset into dptr / dlen
    DevBuf<int> perm_, dptr_, dlen_, cols_;
    DevBuf<double> vals_;
};

}  // namespace ipo
