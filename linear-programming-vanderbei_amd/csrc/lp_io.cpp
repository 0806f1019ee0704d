// lp_io.cpp -- MPS reader + solver-form transform (see lp_io.h).
#include "lp_io.h"

#include <cmath>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <unordered_map>
#include <utility>

namespace ipo {

namespace {

enum class Section { Header, Name, Rows, Columns, Rhs, Ranges, Bounds, Quads, End, Unknown };

Section section_from(const char* head3) {
    if (!std::strcmp(head3, "RHS")) return Section::Rhs;
    if (!std::strcmp(head3, "RAN")) return Section::Ranges;
    if (!std::strcmp(head3, "BOU")) return Section::Bounds;
    if (!std::strcmp(head3, "QUA")) return Section::Quads;
    if (!std::strcmp(head3, "END")) return Section::End;
    return Section::Unknown;
}

// A fixed-format MPS card.  The reference reads with fgets into a 240-byte
// buffer, blanks from the last character read up to column 78 and, outside
// the header, terminates the fields at columns 3, 12, 22, 36, 47, 61 and 79
// (iolp.c:252-261).  Field widths (and trailing blanks inside a label) are
// therefore part of the label identity.
struct Card {
    char buf[240];
    int len = 0;
    const char* kind() const { return buf + 1; }
    const char* name0() const { return buf + 4; }
    const char* name1() const { return buf + 14; }
    const char* num1() const { return buf + 24; }
    const char* name2() const { return buf + 39; }
    const char* num2() const { return buf + 49; }
    void cut_fields() {
        for (int p : {3, 12, 22, 36, 47, 61, 79}) buf[p] = '\0';
    }
};

bool has_substr(const char* s, const char* t) { return *t && std::strstr(s, t) != nullptr; }

}  // namespace

int read_mps(const char* path, MpsProblem& P, std::string* err) {
    P = MpsProblem();
    FILE* fp = std::fopen(path, "r");
    if (!fp) { if (err) *err = std::string("cannot open file ") + path; return 2; }

    std::unordered_map<std::string, int> row_id, col_id;
    std::vector<int> row_kind;          // 0 = E/G, 1 = L (negated), 2 = N (dropped)
    std::vector<std::string> col_name;
    std::string obj_row, rhs_set, rng_set, bnd_set;
    bool quads = false;                       // QUADS section seen
    int q_prev = -1;                          // last QUADS column (iolp.c's j_previous)
    std::vector<int> q_colptr, q_row;         // strictly lower entries by column
    std::vector<double> q_val;
    std::unordered_map<int, double> q_diag;
    char word0[256] = "", word1[256] = "";
    Card cd;
    cd.buf[79] = '\0';
    Section sec = Section::Header;
    int rc = 0;

    auto unknown_section = [&](const char* head) {
        if (err) *err = std::string("unrecognized section label: ") + head;
        rc = 26;
    };

    while (std::fgets(cd.buf, sizeof(cd.buf), fp)) {
        if (cd.buf[0] == '*') continue;
        cd.len = static_cast<int>(std::strlen(cd.buf));
        for (int j = cd.len - 1; j < 79; j++) cd.buf[j] = ' ';
        if (sec != Section::Header) cd.cut_fields();

        switch (sec) {
        case Section::Header:
            std::sscanf(cd.buf, "%255s%255s", word0, word1);   // words persist like iolp.c:265
            if (!std::strncmp(word0, "NAME", 4)) { P.name = word1; sec = Section::Name; }
            else if (!std::strcmp(word0, "MAX")) P.sense = -1;
            else if (!std::strcmp(word0, "MIN")) P.sense = 1;
            else if (!std::strcmp(word0, "OBJ")) obj_row = word1;
            else if (!std::strcmp(word0, "RHS")) rhs_set = word1;
            else if (!std::strcmp(word0, "RANGES")) rng_set = word1;
            else if (!std::strcmp(word0, "BOUNDS")) bnd_set = word1;
            else if (!std::strcmp(word0, "INFTOL")) P.inftol = std::atof(word1);
            break;
        case Section::Name:
            if (!std::strcmp(cd.buf, "ROW")) sec = Section::Rows;
            else P.warnings.push_back(std::string("expected ROWS after NAME instead of ") + cd.buf);
            break;
        case Section::Rows: {
            if (cd.buf[0] != ' ') {
                if (!std::strcmp(cd.buf, "COL")) { sec = Section::Columns; P.b.assign(row_kind.size(), 0.0); }
                else P.warnings.push_back(std::string("expected L, E, G, N, or COLUMNS instead of ") + cd.kind());
                break;
            }
            const char t = cd.kind()[0] == ' ' ? cd.kind()[1] : cd.kind()[0];
            const std::string lab = cd.name0();
            int kind = 0;
            double rng = HUGE_VAL;
            if (t == 'L') kind = 1;
            else if (t == 'E') rng = 0.0;
            else if (t == 'N') {
                if (obj_row.empty()) obj_row = lab;
                if (has_substr(lab.c_str(), obj_row.c_str())) obj_row = lab;
                kind = 2;
            }
            row_id[lab] = static_cast<int>(row_kind.size());
            row_kind.push_back(kind);
            P.rowlab.push_back(lab);
            P.r.push_back(rng);
            break;
        }
        case Section::Columns: {
            if (cd.buf[0] != ' ') {
                P.c.assign(col_name.size(), 0.0);
                P.l.assign(col_name.size(), 0.0);
                sec = section_from(cd.buf);
                if (sec == Section::Unknown) { unknown_section(cd.buf); goto finish; }
                break;
            }
            const std::string lab = cd.name0();
            auto it = col_id.find(lab);
            if (it != col_id.end()) {
                if (col_name.back() != lab) { if (err) *err = "column " + lab + " out of order in COLUMNS section"; rc = 35; goto finish; }
            } else if (std::strcmp(cd.name1(), "'MARKER'") != 0) {
                col_id[lab] = static_cast<int>(col_name.size());
                col_name.push_back(lab);
                P.kA.push_back(static_cast<int>(P.iA.size()));
                P.u.push_back(HUGE_VAL);
            }
            for (int fld = 0; fld < 2; fld++) {
                if (cd.len < (fld ? 50 : 25)) continue;
                const double v = std::atof(fld ? cd.num2() : cd.num1());
                if (v == 0.0) continue;
                auto rt = row_id.find(fld ? cd.name2() : cd.name1());
                if (rt == row_id.end()) { P.warnings.push_back(std::string("row label missing: ") + (fld ? cd.name2() : cd.name1())); continue; }
                P.iA.push_back(rt->second);
                P.A.push_back(v);
            }
            break;
        }
        case Section::Rhs:
        case Section::Ranges: {
            if (cd.buf[0] != ' ') {
                sec = section_from(cd.buf);
                if (sec == Section::Unknown) { unknown_section(cd.buf); goto finish; }
                break;
            }
            std::string& set = sec == Section::Rhs ? rhs_set : rng_set;
            std::vector<double>& dst = sec == Section::Rhs ? P.b : P.r;
            if (set.empty()) set = cd.name0();
            if (!has_substr(cd.name0(), set.c_str())) break;
            // second name/value pair first (iolp.c:481-500)
            if (cd.len >= 50) {
                const double v = std::atof(cd.num2());
                if (v != 0.0) {
                    auto rt = row_id.find(cd.name2());
                    if (rt != row_id.end()) dst[rt->second] = v;
                    else P.warnings.push_back(std::string("row label missing: ") + cd.name2());
                }
            }
            {
                const double v = std::atof(cd.num1());
                if (v != 0.0) {
                    auto rt = row_id.find(cd.name1());
                    if (rt != row_id.end()) dst[rt->second] = v;
                    else P.warnings.push_back(std::string("row label missing: ") + cd.name1());
                }
            }
            break;
        }
        case Section::Bounds: {
            if (cd.buf[0] != ' ') {
                sec = section_from(cd.buf);
                if (sec == Section::Unknown) { unknown_section(cd.buf); goto finish; }
                break;
            }
            if (bnd_set.empty()) bnd_set = cd.name0();
            if (!has_substr(cd.name0(), bnd_set.c_str())) break;
            const double v = std::atof(cd.num1());
            auto ct = col_id.find(cd.name1());
            if (ct == col_id.end()) { P.warnings.push_back(std::string("bound on unknown column ") + cd.name1()); break; }
            const int j = ct->second;
            const std::string k = cd.kind();
            if (k == "LO") P.l[j] = v;
            else if (k == "UP") P.u[j] = v;
            else if (k == "FX") { P.l[j] = v; P.u[j] = v; }
            else if (k == "FR") { P.l[j] = -HUGE_VAL; P.u[j] = HUGE_VAL; }
            else if (k == "PL") P.u[j] = HUGE_VAL;
            else if (k == "MI") { P.u[j] = P.l[j]; P.l[j] = -HUGE_VAL; }
            else if (k == "BV") { P.l[j] = 0.0; P.u[j] = 1.0; }
            else if (k == "LI") P.l[j] = v;
            else if (k == "UI") P.u[j] = v;
            else if (k == "SC") { P.l[j] = 0.0; P.u[j] = v; }
            else P.warnings.push_back("unrecognized bound type " + k);
            break;
        }
        case Section::Quads: {   // iolp.c:583-645: the lower triangle of Q by columns
            if (cd.buf[0] != ' ') {
                sec = section_from(cd.buf);
                if (sec == Section::Unknown) { unknown_section(cd.buf); goto finish; }
                break;
            }
            quads = true;
            auto ct = col_id.find(cd.name0());
            if (ct == col_id.end()) { P.warnings.push_back(std::string("column label missing: ") + cd.name0()); break; }
            const int j = ct->second;
            if (j > q_prev) {
                q_colptr.resize(j + 1, static_cast<int>(q_row.size()));
                q_prev = j;
            } else if (j < q_prev) {
                if (err) *err = "QUADS columns out of order";
                rc = 36;
                goto finish;
            }
            for (int fld = 0; fld < 2; fld++) {
                if (cd.len < (fld ? 50 : 25)) continue;
                const double v = std::atof(fld ? cd.num2() : cd.num1());
                if (v == 0.0) continue;
                auto rt = col_id.find(fld ? cd.name2() : cd.name1());
                if (rt == col_id.end()) { P.warnings.push_back(std::string("column label missing: ") + (fld ? cd.name2() : cd.name1())); continue; }
                const int i = rt->second;
                if (i > j) { q_row.push_back(i); q_val.push_back(v); }
                else if (i == j) q_diag[j] = v;
                else P.warnings.push_back("QUADS entry above the diagonal ignored");
            }
            break;
        }
        default:
            break;
        }
    }
    if (P.name.empty()) { if (err) *err = "NAME not found"; rc = 11; goto finish; }
    if (quads) {   // symmetrise (iolp.c:733-793): both triangles + the nonzero diagonal, rows sorted
        const int n = static_cast<int>(col_name.size());
        q_colptr.resize(n + 1, static_cast<int>(q_row.size()));
        std::vector<std::vector<std::pair<int, double>>> col(n);
        for (int j = 0; j < n; j++) {
            for (int k = q_colptr[j]; k < q_colptr[j + 1]; k++) col[j].push_back({q_row[k], q_val[k]});
            auto d = q_diag.find(j);
            if (d != q_diag.end() && d->second != 0.0) col[j].push_back({j, d->second});
            for (int k = q_colptr[j]; k < q_colptr[j + 1]; k++) col[q_row[k]].push_back({j, q_val[k]});
        }
        P.kQ.assign(1, 0);
        for (int j = 0; j < n; j++) {
            std::stable_sort(col[j].begin(), col[j].end(),
                             [](const std::pair<int, double>& a, const std::pair<int, double>& b) { return a.first < b.first; });
            for (const auto& e : col[j]) { P.iQ.push_back(e.first); P.Q.push_back(e.second); }
            P.kQ.push_back(static_cast<int>(P.iQ.size()));
        }
    }
    if (sec != Section::End) P.warnings.push_back("ENDATA not found");
    {
        const int n = static_cast<int>(col_name.size());
        const int mrows = static_cast<int>(row_kind.size());
        if (P.c.size() != static_cast<size_t>(n)) { P.c.assign(n, 0.0); P.l.assign(n, 0.0); }
        if (P.b.size() != static_cast<size_t>(mrows)) P.b.assign(mrows, 0.0);
        P.kA.push_back(static_cast<int>(P.iA.size()));

        // objective row -> c, N rows dropped, L rows negated, rows renumbered
        auto ot = row_id.find(obj_row);
        const int ic = ot == row_id.end() ? -1 : ot->second;
        if (ic == -1 || row_kind[ic] != 2) P.warnings.push_back("objective function " + obj_row + " not found");
        int keep = 0;
        for (int j = 0; j < n; j++) {
            const int k0 = P.kA[j], k1 = P.kA[j + 1];
            P.kA[j] = keep;
            for (int k = k0; k < k1; k++) {
                const int i = P.iA[k];
                if (i == ic) { P.c[j] = P.A[k]; continue; }
                if (row_kind[i] == 2) continue;
                P.A[keep] = row_kind[i] == 1 ? -P.A[k] : P.A[k];
                P.iA[keep] = i;
                keep++;
            }
        }
        P.kA[n] = keep;
        P.A.resize(keep);
        P.iA.resize(keep);
        std::vector<int> renum(mrows, -1);
        int mm = 0;
        for (int i = 0; i < mrows; i++) {
            if (i == ic || row_kind[i] == 2) continue;
            renum[i] = mm;
            P.b[mm] = row_kind[i] == 1 ? -P.b[i] : P.b[i];
            P.r[mm] = P.r[i];
            P.rowlab[mm] = P.rowlab[i];
            mm++;
        }
        for (int& i : P.iA) i = renum[i];
        P.b.resize(mm);
        P.r.resize(mm);
        P.rowlab.resize(mm);
        P.collab = col_name;
        P.m = mm;
        P.n = n;
    }
finish:
    std::fclose(fp);
    return rc;
}

int split_free_columns(const MpsProblem& P, MpsProblem& Q, FreeMap& map) {
    const int n = P.n, m = P.m;
    Q = P;
    map = FreeMap();
    map.n = n;
    map.shift.assign(n, 0.0);
    std::vector<int> split;
    for (int j = 0; j < n; j++)
        if (P.l[j] == -HUGE_VAL) {
            map.nfree++;
            if (P.u[j] == HUGE_VAL) split.push_back(j);
        }
    const int n2 = n + static_cast<int>(split.size());
    Q.n = n2;
    Q.kA.assign(1, 0);
    Q.iA.clear();
    Q.A.clear();
    Q.c.assign(n2, 0.0);
    Q.l.assign(n2, 0.0);
    Q.u.assign(n2, HUGE_VAL);
    map.colmap.assign(n2, 0);
    for (int j = 0; j < n; j++) {
        const bool refl = P.l[j] == -HUGE_VAL && P.u[j] < HUGE_VAL;
        const double sg = refl ? -1.0 : 1.0;
        for (int k = P.kA[j]; k < P.kA[j + 1]; k++) {
            Q.iA.push_back(P.iA[k]);
            Q.A.push_back(sg * P.A[k]);
            if (refl) Q.b[P.iA[k]] -= P.A[k] * P.u[j];
        }
        Q.kA.push_back(static_cast<int>(Q.iA.size()));
        Q.c[j] = sg * P.c[j];
        map.colmap[j] = refl ? -(j + 1) : (j + 1);
        if (refl) {
            Q.f += P.c[j] * P.u[j];
            map.shift[j] = P.u[j];
        } else {
            Q.l[j] = P.l[j] == -HUGE_VAL ? 0.0 : P.l[j];
            Q.u[j] = P.u[j];
        }
    }
    int jn = n;
    for (int j : split) {
        for (int k = P.kA[j]; k < P.kA[j + 1]; k++) { Q.iA.push_back(P.iA[k]); Q.A.push_back(-P.A[k]); }
        Q.kA.push_back(static_cast<int>(Q.iA.size()));
        Q.c[jn] = -P.c[j];
        map.colmap[jn] = -(j + 1);
        jn++;
    }
    (void)m;
    return map.nfree;
}

void FreeMap::recover(const double* xs, double* x) const {
    for (int j = 0; j < n; j++) x[j] = shift[j];
    for (size_t q = 0; q < colmap.size(); q++) {
        const int c = colmap[q];
        if (c > 0) x[c - 1] += xs[q];
        else x[-c - 1] -= xs[q];
    }
}

SolutionOut untransform(const MpsProblem& p, const SolverForm& s, const double* x, const double* y, const double* z) {
    const int m = p.m, n = p.n;
    SolutionOut o;
    o.x.resize(n);
    o.z.resize(n);
    o.y.resize(m);
    o.u = p.u;
    o.b.resize(m);
    for (int j = 0; j < n; j++) {
        o.x[j] = x[j] + p.l[j];                         // solve.c:241
        o.z[j] = z[j];
        if (o.u[j] != HUGE_VAL) o.u[j] -= p.l[j];       // solve.c:103-104, in place in the reference's LP
    }
    // b - A l, negated (solve.c:105-109, :145); the y of the first m rows,
    // negated for MIN (solve.c:247-250)
    std::vector<double> al(m, 0.0);
    for (int j = 0; j < n; j++)
        for (int k = p.kA[j]; k < p.kA[j + 1]; k++) al[p.iA[k]] += p.A[k] * p.l[j];
    for (int i = 0; i < m; i++) {
        o.b[i] = -(p.b[i] - al[i]);
        o.y[i] = s.sense == 1 ? -y[i] : y[i];
    }
    // rowact of writesol (iolp.c:1003-1007): the rebuilt A, whose first m rows
    // are the negated originals (solve.c:142-146), times the shifted-back x
    o.rowact.assign(m, 0.0);
    for (int j = 0; j < n; j++)
        for (int k = p.kA[j]; k < p.kA[j + 1]; k++) o.rowact[p.iA[k]] += o.x[j] * -p.A[k];
    return o;
}

void merge_split(const MpsProblem& orig, const FreeMap& fm, SolutionOut& so) {
    const int n = orig.n;
    std::vector<double> x(n), z(n, 0.0);
    fm.recover(so.x.data(), x.data());
    for (int j = 0; j < n; j++) z[j] = fm.colmap[j] < 0 ? -so.z[j] : so.z[j];
    // rows: the same rows, activity of the original columns
    std::vector<double> ract(orig.m, 0.0);
    for (int j = 0; j < n; j++)
        for (int k = orig.kA[j]; k < orig.kA[j + 1]; k++) ract[orig.iA[k]] += x[j] * -orig.A[k];
    std::vector<double> u(orig.u);
    for (int j = 0; j < n; j++)
        if (u[j] != HUGE_VAL && orig.l[j] != -HUGE_VAL) u[j] -= orig.l[j];
    std::vector<double> al(orig.m, 0.0), b(orig.m);
    for (int j = 0; j < n; j++)
        if (orig.l[j] != -HUGE_VAL)
            for (int k = orig.kA[j]; k < orig.kA[j + 1]; k++) al[orig.iA[k]] += orig.A[k] * orig.l[j];
    for (int i = 0; i < orig.m; i++) b[i] = -(orig.b[i] - al[i]);
    so.x.swap(x);
    so.z.swap(z);
    so.rowact.swap(ract);
    so.u.swap(u);
    so.b.swap(b);
}

int write_sol(const char* path, const MpsProblem& p, const SolutionOut& so, std::string* err) {
    FILE* fp = std::fopen(path, "w");
    if (!fp) { if (err) *err = std::string("cannot open file ") + path; return 2; }
    const double eps = p.inftol * 1.2;
    const std::vector<double>& l = p.l;
    std::fprintf(fp, "COLUMNS SECTION\n");
    std::fprintf(fp, "   index       label  primal_val reduced_cst");
    std::fprintf(fp, "    lower_bd    upper_bd   OB_flag\n");
    for (int j = 0; j < p.n; j++) {
        const char* lab = p.collab[j].c_str();
        const double x = so.x[j], z = so.z[j], u = so.u[j];
        if (l[j] > -HUGE_VAL && u < HUGE_VAL) std::fprintf(fp, "%8d  %10s %11.4e %11.4e %11.4e %11.4e", j, lab, x, z, l[j], u);
        else if (l[j] > -HUGE_VAL) std::fprintf(fp, "%8d  %10s %11.4e %11.4e %11.4e    Infinity", j, lab, x, z, l[j]);
        else if (u < HUGE_VAL) std::fprintf(fp, "%8d  %10s %11.4e %11.4e   -Infinity %11.4e", j, lab, x, z, u);
        else std::fprintf(fp, "%8d  %10s %11.4e %11.4e   -Infinity    Infinity", j, lab, x, z);
        if (x < l[j] - eps || x > u + eps) std::fprintf(fp, "      OB\n");
        else std::fprintf(fp, "\n");
    }
    std::fprintf(fp, "ROWS SECTION\n");
    std::fprintf(fp, "   index       label    dual_val  row_actvty");
    std::fprintf(fp, " rght_hnd_sd       range   OB_flag\n");
    for (int i = 0; i < p.m; i++) {
        const char* lab = p.rowlab[i].c_str();
        const double r = p.r[i], b = so.b[i], ra = so.rowact[i];
        if (r < HUGE_VAL) std::fprintf(fp, "%8d  %10s %11.4e %11.4e %11.4e %11.4e", i, lab, so.y[i], ra, b, r);
        else std::fprintf(fp, "%8d  %10s %11.4e %11.4e %11.4e    Infinity", i, lab, so.y[i], ra, b);
        if (ra < b - eps || ra > b + r + eps) std::fprintf(fp, "     OB\n");
        else std::fprintf(fp, "\n");
    }
    std::fprintf(fp, "ENDOUT\n");
    std::fclose(fp);
    return 0;
}

void csc_transpose(int m, int n, const int* ka, const int* ia, const double* a,
                   std::vector<int>& kat, std::vector<int>& iat, std::vector<double>& at) {
    const int nz = ka[n];
    kat.assign(m + 1, 0);
    iat.resize(nz);
    at.resize(nz);
    for (int k = 0; k < nz; k++) kat[ia[k] + 1]++;
    for (int i = 0; i < m; i++) kat[i + 1] += kat[i];
    std::vector<int> fill(kat.begin(), kat.end() - 1);
    for (int j = 0; j < n; j++)
        for (int k = ka[j]; k < ka[j + 1]; k++) {
            const int d = fill[ia[k]]++;
            iat[d] = j;
            at[d] = a[k];
        }
}

int to_solver_form(const MpsProblem& p, SolverForm& s) {
    s = SolverForm();
    const int m = p.m, n = p.n;
    s.m0 = m; s.n0 = n; s.nz0 = p.kA.empty() ? 0 : p.kA[n];
    s.sense = p.sense;
    s.m = m; s.n = n;
    for (int j = 0; j < n; j++)
        if (p.l[j] == -HUGE_VAL) return 3;

    // shift x <- x - l (solve.c:103-110)
    std::vector<double> u(p.u), b(p.b);
    for (int j = 0; j < n; j++) if (u[j] != HUGE_VAL) u[j] -= p.l[j];
    {
        std::vector<double> al(m, 0.0);
        for (int j = 0; j < n; j++)
            for (int k = p.kA[j]; k < p.kA[j + 1]; k++) al[p.iA[k]] += p.A[k] * p.l[j];
        for (int i = 0; i < m; i++) b[i] -= al[i];
    }
    double f = p.f;
    {
        double dot = 0.0;
        for (int j = 0; j < n; j++) dot += p.c[j] * p.l[j];
        f += dot;
    }

    // rows: all original rows negated, then +copies of ranged rows, then bounds
    std::vector<int> rp, ci;
    std::vector<double> rv;
    csc_transpose(m, n, p.kA.data(), p.iA.data(), p.A.data(), rp, ci, rv);
    std::vector<int> rp2(rp);
    std::vector<int> extra_ci;
    std::vector<double> extra_rv, extra_b;
    std::vector<int> extra_len;
    for (int i = 0; i < m; i++) {
        const bool ranged = p.r[i] < HUGE_VAL;
        if (ranged) {
            for (int k = rp[i]; k < rp[i + 1]; k++) { extra_ci.push_back(ci[k]); extra_rv.push_back(rv[k]); }
            extra_len.push_back(rp[i + 1] - rp[i]);
            extra_b.push_back(b[i] + p.r[i]);
        }
        for (int k = rp[i]; k < rp[i + 1]; k++) rv[k] *= -1;
        b[i] *= -1;
    }
    for (int j = 0; j < n; j++) {
        if (u[j] < HUGE_VAL) {
            extra_ci.push_back(j); extra_rv.push_back(1.0);
            extra_len.push_back(1);
            extra_b.push_back(u[j]);
        }
    }
    const int mtot = m + static_cast<int>(extra_len.size());
    rp.resize(mtot + 1);
    for (size_t e = 0; e < extra_len.size(); e++) rp[m + e + 1] = rp[m + e] + extra_len[e];
    ci.insert(ci.end(), extra_ci.begin(), extra_ci.end());
    rv.insert(rv.end(), extra_rv.begin(), extra_rv.end());
    b.insert(b.end(), extra_b.begin(), extra_b.end());

    // back to CSC (row indices ascend because rows are visited in order)
    csc_transpose(n, mtot, rp.data(), ci.data(), rv.data(), s.kA, s.iA, s.A);
    s.m = mtot;
    s.n = n;
    s.nz = rp[mtot];
    s.b = std::move(b);
    s.c = p.c;
    s.f = f;
    if (p.sense == 1) {
        for (double& v : s.c) v *= -1;
        s.f *= -1;
    }
    s.lshift = p.l;
    return 0;
}

}  // namespace ipo
