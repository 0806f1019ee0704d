// lp_io.h -- native front end of ipo-hip: MPS reader and the solvelp()
// normalisation that turns an MPS problem into the form solver() takes.
//
// Behaviour follows the reference front end so the same .mps file reaches
// solver() with the same rows, signs and order:
//   read_mps     src/common/iolp.c:145-838   (fixed columns, L rows negated,
//                                             objective = first N row)
//   to_solver_form src/common/solve.c:28-205 (lower-bound shift, rows
//                                             negated, ranged/E rows split,
//                                             upper bounds appended, CSC
//                                             rebuilt with sorted rows)
#pragma once
#include <cstdio>
#include <string>
#include <vector>

namespace ipo {

struct MpsProblem {
    std::string name;
    int m = 0, n = 0;
    std::vector<int> kA, iA;        // CSC, n+1 / nz
    std::vector<double> A, b, c, r, l, u;
    double f = 0.0;
    int sense = 1;                  // 1 = MIN, -1 = MAX
    std::vector<std::string> warnings;
};

// Returns 0 on success or the reference's error number (2, 11, 26, 35).
int read_mps(const char* path, MpsProblem& out, std::string* err);

struct SolverForm {
    int m = 0, n = 0, nz = 0;       // dimensions seen by solver()
    int m0 = 0, n0 = 0, nz0 = 0;    // before the transform
    std::vector<int> kA, iA;        // CSC, row indices ascending
    std::vector<double> A, b, c;
    double f = 0.0;
    int sense = 1;
    std::vector<double> lshift;     // to undo the lower-bound shift
};

// Returns 0, or 3 ("dual unbounded") when a variable has no lower bound.
int to_solver_form(const MpsProblem& p, SolverForm& s);

// CSC transpose with the reference's stable order (linalg.c:75-103).
void csc_transpose(int m, int n, const int* ka, const int* ia, const double* a,
                   std::vector<int>& kat, std::vector<int>& iat, std::vector<double>& at);

}  // namespace ipo
