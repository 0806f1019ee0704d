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
    double inftol = 1.0e-5;         // INFTOL header keyword (iolp.c:98, :297)
    std::vector<std::string> rowlab, collab;   // field text, trailing blanks kept (iolp.c:387, :422)
    std::vector<std::string> warnings;
    // QUADS (iolp.c:583-645, symmetrised as iolp.c:733-793): n x n, both
    // triangles and the nonzero diagonal, rows sorted in each column; empty
    // kQ when the file has no QUADS section.  solvelp() does not pass Q to
    // solver() (solve.c:24-26 has no Q); the LU plug-in takes it
    // (ipo_hip_ldlt_set_q, ldlt.c:253-256).
    std::vector<int> kQ, iQ;
    std::vector<double> Q;
};

// Returns 0 on success or the reference's error number (2, 11, 26, 35, 36).
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

// Free-variable extension (not in the reference, which aborts with status
// 3, solve.c:79-87): an equivalent problem whose
// every column has a finite lower bound.
//   l = -inf, u = +inf : x = x+ - x-   column j keeps (a_j, c_j), l = 0; a
//                        column (-a_j, -c_j), l = 0, is appended (appended
//                        columns in order of j, after the original n);
//   l = -inf, u finite : x = u - x'    column j becomes (-a_j, -c_j), l = 0,
//                        u = inf; b -= a_j u, f += c_j u.
// colmap[j'] = +(j+1) / -(j+1): x_j' enters x_j with that sign; shift[j] =
// the u of a reflected column.  The same transform as the oracle's
// orc_split_free (test infrastructure), so the two can be compared.
struct FreeMap {
    int n = 0, nfree = 0;
    std::vector<int> colmap;        // [n'] signed 1-based original column
    std::vector<double> shift;      // [n]
    // x (n original columns) from the split problem's x' (n' columns, after
    // the solver's lower-bound shift is undone)
    void recover(const double* xs, double* x) const;
};
int split_free_columns(const MpsProblem& in, MpsProblem& out, FreeMap& map);

// What writesol (iolp.c:976-1045) prints after solvelp has undone its
// transform (solve.c:237-255): per original column x + l and z, per
// original row the dual (negated for MIN) and the quantities writesol
// reads from the LP as solvelp left it -- b (shifted by A l and negated,
// solve.c:105-109, :145), u (shifted by l, :103-104) and the row activity
// of the transformed, negated rows (rowact = -A x).  z is the solver's z:
// the reference frees it in hsd.c:290-291 and writesol then reads freed
// memory; here it is the value solver() returned.
struct SolutionOut {
    std::vector<double> x, z, y, rowact, b, u;
};
SolutionOut untransform(const MpsProblem& p, const SolverForm& s, const double* x, const double* y, const double* z);
// A free-variable split problem's solution mapped back onto the original
// columns (x_j = recovered, z_j = the dual slack of its first image).
void merge_split(const MpsProblem& orig, const FreeMap& fm, SolutionOut& so);
// writesol (iolp.c:976-1045): the COLUMNS / ROWS report to `path`.
int write_sol(const char* path, const MpsProblem& p, const SolutionOut& so, std::string* err);

// CSC transpose with the reference's stable order (linalg.c:75-103).
void csc_transpose(int m, int n, const int* ka, const int* ia, const double* a,
                   std::vector<int>& kat, std::vector<int>& iat, std::vector<double>& at);

}  // namespace ipo
