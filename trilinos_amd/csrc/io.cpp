// Matrix ingestion: MatrixMarket coordinate files and Harwell-Boeing
// RUA/RSA files, read on the host into the rows of one rank's uniform row range, then
// handed to crs_create (column map, import plan, device CSR).
//
//   MatrixMarket   Tpetra::MatrixMarket::Reader<CrsMatrix>::readSparseFile
//                  (tpetra/core/inout/MatrixMarket_Tpetra.hpp): "coordinate" real / integer /
//                  pattern, general / symmetric / skew-symmetric; 1-based indices; symmetric
//                  storage is expanded to both triangles (SymmetrizingAdder, skew: -v);
//                  duplicate entries are summed in file order.
//   Harwell-Boeing Trilinos_Util_read_hb (triutils/src/Trilinos_Util_read_hb.cpp) as used by
//                  Belos::Util::createEpetraProblem (belos/epetra/src/BelosEpetraUtils.cpp:
//                  81-160): CSC in Fortran fixed-width fields, converted to MSR, so every row
//                  gets an explicit diagonal entry (0.0 when the file has none), inserted with
//                  InsertGlobalValues; symmetric (RSA) storage expanded to both triangles.
//
// Every rank parses the whole file and keeps its rows (no broadcast: files are read where
// they lie).  Row entries are handed over in file order; crs_create orders each row by local
// column id exactly as Epetra's FillComplete (SortEntries) does.
#include <algorithm>
#include <cctype>
#include <charconv>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include "../../include/migmres.h"
#include "internal.h"
#include "plan.h"
#include "runtime.h"

using namespace migmres;

namespace {

std::string slurp(const char *path) {
  std::ifstream f(path, std::ios::binary);
  if (!f) throw Error(MIGMRES_EINVAL, std::string("cannot open matrix file: ") + path);
  std::ostringstream ss;
  ss << f.rdbuf();
  return ss.str();
}

// Lines of a text buffer as [begin, end) offsets (no terminators).
std::vector<std::pair<size_t, size_t>> split_lines(const std::string &s) {
  std::vector<std::pair<size_t, size_t>> out;
  size_t b = 0;
  while (b < s.size()) {
    size_t e = s.find('\n', b);
    if (e == std::string::npos) e = s.size();
    size_t ee = e;
    if (ee > b && s[ee - 1] == '\r') --ee;
    out.emplace_back(b, ee);
    b = e + 1;
  }
  return out;
}

double parse_double(const char *b, const char *e) {
  // Fortran exponents may be written with D (or be missing the letter: 1.0-3); both occur
  // in Harwell-Boeing files.
  char buf[64];
  size_t n = 0;
  bool digit_seen = false;
  for (const char *p = b; p < e && n < sizeof(buf) - 2; ++p) {
    char c = *p;
    if (c == ' ' || c == '\t') continue;
    if (c == 'D' || c == 'd') c = 'E';
    if ((c == '+' || c == '-') && digit_seen && n > 0 && buf[n - 1] != 'E' && buf[n - 1] != 'e') buf[n++] = 'E';
    if (std::isdigit((unsigned char)c)) digit_seen = true;
    buf[n++] = c;
  }
  buf[n] = 0;
  if (n == 0) throw Error(MIGMRES_EINVAL, "matrix file: empty numeric field");
  double v = 0.0;
  auto r = std::from_chars(buf, buf + n, v);
  if (r.ec != std::errc() || r.ptr != buf + n) throw Error(MIGMRES_EINVAL, std::string("matrix file: bad number '") + buf + "'");
  return v;
}

long long parse_ll(const char *b, const char *e) {
  while (b < e && (*b == ' ' || *b == '\t')) ++b;
  while (e > b && (e[-1] == ' ' || e[-1] == '\t')) --e;
  long long v = 0;
  auto r = std::from_chars(b, e, v);
  if (r.ec != std::errc() || r.ptr != e) throw Error(MIGMRES_EINVAL, "matrix file: bad integer field");
  return v;
}

// Local rows of [first, first + n_local), entries (global column, value) in insertion order;
// duplicates within a row are summed in that order (first occurrence keeps its position).
struct RowSet {
  long long first = 0;
  int n_local = 0;
  std::vector<std::vector<std::pair<long long, double>>> rows;
  void init(long long f, int n) {
    first = f;
    n_local = n;
    rows.assign(n, {});
  }
  void add(long long r, long long c, double v) {
    if (r < first || r >= first + n_local) return;
    rows[r - first].emplace_back(c, v);
  }
  void merge_duplicates() {
    for (auto &row : rows) {
      if (row.size() < 2) continue;
      std::vector<std::pair<long long, double>> out;
      out.reserve(row.size());
      std::vector<std::pair<long long, size_t>> seen;  // (column, index in out), sorted
      for (auto &e : row) {
        auto it = std::lower_bound(seen.begin(), seen.end(), std::make_pair(e.first, (size_t)0));
        if (it != seen.end() && it->first == e.first) {
          out[it->second].second += e.second;
        } else {
          seen.insert(it, {e.first, out.size()});
          out.push_back(e);
        }
      }
      row.swap(out);
    }
  }
  long long nnz() const {
    long long n = 0;
    for (auto &r : rows) n += (long long)r.size();
    return n;
  }
  void flatten(long long *rowptr, long long *gcols, double *vals) const {
    long long q = 0;
    if (rowptr) rowptr[0] = 0;
    for (int i = 0; i < n_local; ++i) {
      for (auto &e : rows[i]) {
        if (gcols) gcols[q] = e.first;
        if (vals) vals[q] = e.second;
        ++q;
      }
      if (rowptr) rowptr[i + 1] = q;
    }
  }
};

struct FileInfo {
  bool mm = false;
  long long nrows = 0, ncols = 0, nnz_file = 0;
  int symmetric = 0;  // 0 general, 1 symmetric, 2 skew-symmetric
};

// ---------------------------------------------------------------- MatrixMarket
struct MmHeader {
  bool pattern = false;
  int sym = 0;
  size_t data_line = 0;
  long long m = 0, n = 0, nnz = 0;
};

MmHeader mm_header(const std::string &s, const std::vector<std::pair<size_t, size_t>> &lines) {
  MmHeader h;
  if (lines.empty()) throw Error(MIGMRES_EINVAL, "MatrixMarket: empty file");
  std::string banner = s.substr(lines[0].first, lines[0].second - lines[0].first);
  std::string low = banner;
  for (auto &c : low) c = (char)std::tolower((unsigned char)c);
  std::istringstream bs(low);
  std::string tag, object, fmt, field, symm;
  bs >> tag >> object >> fmt >> field >> symm;
  if (tag != "%%matrixmarket" || object != "matrix") throw Error(MIGMRES_EINVAL, "MatrixMarket: bad banner");
  if (fmt != "coordinate") throw Error(MIGMRES_EINVAL, "MatrixMarket: only coordinate (sparse) files are read");
  if (field == "complex") throw Error(MIGMRES_EINVAL, "MatrixMarket: complex matrices are not supported");
  if (field != "real" && field != "integer" && field != "pattern" && field != "double")
    throw Error(MIGMRES_EINVAL, "MatrixMarket: unknown field " + field);
  h.pattern = field == "pattern";
  if (symm == "general") h.sym = 0;
  else if (symm == "symmetric") h.sym = 1;
  else if (symm == "skew-symmetric") h.sym = 2;
  else throw Error(MIGMRES_EINVAL, "MatrixMarket: unsupported symmetry " + symm);
  size_t i = 1;
  for (; i < lines.size(); ++i) {
    const char *b = s.data() + lines[i].first, *e = s.data() + lines[i].second;
    while (b < e && std::isspace((unsigned char)*b)) ++b;
    if (b == e || *b == '%') continue;
    std::istringstream ls(std::string(b, e));
    if (!(ls >> h.m >> h.n >> h.nnz)) throw Error(MIGMRES_EINVAL, "MatrixMarket: bad size line");
    break;
  }
  h.data_line = i + 1;
  return h;
}

void mm_read(const std::string &s, RowSet *rs, FileInfo &info) {
  const auto lines = split_lines(s);
  const MmHeader h = mm_header(s, lines);
  info.mm = true;
  info.nrows = h.m;
  info.ncols = h.n;
  info.nnz_file = h.nnz;
  info.symmetric = h.sym;
  if (!rs) return;
  long long count = 0;
  for (size_t li = h.data_line; li < lines.size() && count < h.nnz; ++li) {
    const char *p = s.data() + lines[li].first, *e = s.data() + lines[li].second;
    while (p < e && std::isspace((unsigned char)*p)) ++p;
    if (p == e || *p == '%') continue;
    const char *f[3][2];
    int nf = 0;
    while (p < e && nf < 3) {
      const char *b = p;
      while (p < e && !std::isspace((unsigned char)*p)) ++p;
      f[nf][0] = b;
      f[nf][1] = p;
      ++nf;
      while (p < e && std::isspace((unsigned char)*p)) ++p;
    }
    if (nf < (h.pattern ? 2 : 3)) throw Error(MIGMRES_EINVAL, "MatrixMarket: short entry line");
    const long long i = parse_ll(f[0][0], f[0][1]) - 1, j = parse_ll(f[1][0], f[1][1]) - 1;
    const double v = h.pattern ? 1.0 : parse_double(f[2][0], f[2][1]);
    if (i < 0 || i >= h.m || j < 0 || j >= h.n) throw Error(MIGMRES_EINVAL, "MatrixMarket: index out of range");
    rs->add(i, j, v);
    if (h.sym && i != j) rs->add(j, i, h.sym == 2 ? -v : v);
    ++count;
  }
  if (count != h.nnz) throw Error(MIGMRES_EINVAL, "MatrixMarket: fewer entries than the size line declares");
}

// ---------------------------------------------------------------- Harwell-Boeing
// Fortran edit descriptor of a field list: "(16I5)", "(1P5E16.8)", "(4D20.12)", "(10F8.2)"
struct FFmt {
  int per_line = 1, width = 0;
};

FFmt ffmt(std::string f) {
  std::string u;
  for (char c : f)
    if (!std::isspace((unsigned char)c)) u += (char)std::toupper((unsigned char)c);
  size_t p = u.find('(');
  if (p == std::string::npos) throw Error(MIGMRES_EINVAL, "Harwell-Boeing: bad format " + f);
  u = u.substr(p + 1);
  // drop a scale factor "nP" (and an optional comma after it)
  size_t pp = u.find('P');
  if (pp != std::string::npos && pp < u.size() && pp > 0 && std::isdigit((unsigned char)u[pp - 1])) {
    size_t s0 = pp;
    while (s0 > 0 && std::isdigit((unsigned char)u[s0 - 1])) --s0;
    u = u.substr(0, s0) + u.substr(pp + 1);
    if (!u.empty() && u[0] == ',') u = u.substr(1);
  }
  FFmt r;
  size_t i = 0;
  while (i < u.size() && std::isdigit((unsigned char)u[i])) ++i;
  r.per_line = i ? std::stoi(u.substr(0, i)) : 1;
  if (i >= u.size() || !std::strchr("IEDFG", u[i])) throw Error(MIGMRES_EINVAL, "Harwell-Boeing: bad format " + f);
  ++i;
  size_t j = i;
  while (j < u.size() && std::isdigit((unsigned char)u[j])) ++j;
  r.width = std::stoi(u.substr(i, j - i));
  return r;
}

template <class T, class P>
void hb_fields(const std::string &s, const std::vector<std::pair<size_t, size_t>> &lines, size_t l0, long long nlines,
               const FFmt &fm, long long count, std::vector<T> &out, P parse) {
  out.clear();
  out.reserve(count);
  for (long long li = 0; li < nlines && (long long)out.size() < count; ++li) {
    if (l0 + li >= lines.size()) break;
    const char *b = s.data() + lines[l0 + li].first, *e = s.data() + lines[l0 + li].second;
    for (int k = 0; k < fm.per_line && (long long)out.size() < count; ++k) {
      const char *fb = b + (size_t)k * fm.width;
      if (fb >= e) break;
      const char *fe = std::min(fb + fm.width, e);
      bool blank = true;
      for (const char *q = fb; q < fe; ++q) blank = blank && std::isspace((unsigned char)*q);
      if (blank) break;
      out.push_back(parse(fb, fe));
    }
  }
  if ((long long)out.size() != count) throw Error(MIGMRES_EINVAL, "Harwell-Boeing: short data section");
}

void hb_read(const std::string &s, RowSet *rs, FileInfo &info) {
  const auto lines = split_lines(s);
  if (lines.size() < 4) throw Error(MIGMRES_EINVAL, "Harwell-Boeing: short header");
  auto fld = [&](size_t li, size_t a, size_t w) {
    const size_t b = lines[li].first + a, e = lines[li].second;
    if (b >= e) return std::string();
    return s.substr(b, std::min(w, e - b));
  };
  auto num = [&](size_t li, size_t a, size_t w) {
    std::string t = fld(li, a, w);
    t.erase(std::remove_if(t.begin(), t.end(), [](char c) { return std::isspace((unsigned char)c); }), t.end());
    return t.empty() ? 0LL : std::stoll(t);
  };
  const long long ptrcrd = num(1, 14, 14), indcrd = num(1, 28, 14), valcrd = num(1, 42, 14), rhscrd = num(1, 56, 14);
  std::string type = fld(2, 0, 3);
  for (auto &c : type) c = (char)std::toupper((unsigned char)c);
  const long long nrow = num(2, 14, 14), ncol = num(2, 28, 14), nnz = num(2, 42, 14);
  if (type.size() < 3 || type[0] != 'R') throw Error(MIGMRES_EINVAL, "Harwell-Boeing: only real matrices");
  if (type[2] != 'A') throw Error(MIGMRES_EINVAL, "Harwell-Boeing: only assembled matrices");
  if (nrow != ncol) throw Error(MIGMRES_EINVAL, "Harwell-Boeing: matrix must be square");
  const bool sym = type[1] == 'S';
  info.mm = false;
  info.nrows = nrow;
  info.ncols = ncol;
  info.nnz_file = nnz;
  info.symmetric = sym ? 1 : 0;
  if (!rs) return;
  const FFmt fp = ffmt(fld(3, 0, 16)), fi = ffmt(fld(3, 16, 16)), fv = ffmt(fld(3, 32, 20));
  const size_t l0 = 4 + (rhscrd > 0 ? 1 : 0);
  std::vector<long long> colptr, rowind;
  std::vector<double> vals;
  hb_fields(s, lines, l0, ptrcrd, fp, ncol + 1, colptr, parse_ll);
  hb_fields(s, lines, l0 + ptrcrd, indcrd, fi, nnz, rowind, parse_ll);
  if (valcrd <= 0) throw Error(MIGMRES_EINVAL, "Harwell-Boeing: pattern-only files are not supported");
  hb_fields(s, lines, l0 + ptrcrd + indcrd, valcrd, fv, nnz, vals, parse_double);
  // MSR conversion (Trilinos_Util_csrmsr): the diagonal of every row is explicit; the
  // reference inserts each row's off-diagonal entries, then the diagonal
  // (BelosEpetraUtils.cpp:121-131).  Insertion order does not reach the stored rows
  // (FillComplete sorts them), so rows are built as off-diagonals in CSC scan order + the
  // diagonal last.
  std::vector<double> diag(rs->n_local, 0.0);
  for (long long j = 0; j < ncol; ++j) {
    for (long long q = colptr[j] - 1; q < colptr[j + 1] - 1; ++q) {
      const long long r = rowind[q] - 1;
      const double v = vals[q];
      if (r < 0 || r >= nrow) throw Error(MIGMRES_EINVAL, "Harwell-Boeing: row index out of range");
      if (r == j) {
        if (r >= rs->first && r < rs->first + rs->n_local) diag[r - rs->first] += v;
        continue;
      }
      rs->add(r, j, v);
      if (sym) rs->add(j, r, v);
    }
  }
  for (int i = 0; i < rs->n_local; ++i) rs->rows[i].emplace_back(rs->first + i, diag[i]);
}

FileInfo read_file(const char *path, RowSet *rs, int nranks, int rank) {
  MIG_CHECK(path, "matrix file: null path");
  const std::string s = slurp(path);
  FileInfo info;
  const bool mm = s.compare(0, 14, "%%MatrixMarket") == 0;
  // header pass: sizes for the row map
  if (mm)
    mm_read(s, nullptr, info);
  else
    hb_read(s, nullptr, info);
  if (info.nrows != info.ncols) throw Error(MIGMRES_EINVAL, "matrix file: the operator must be square");
  if (rs) {
    if (rs->n_local < 0) {  // uniform map of this rank
      long long first = 0;
      int n_local = 0;
      uniform_map(info.nrows, nranks, rank, &first, &n_local);
      rs->init(first, n_local);
    }
    if (mm)
      mm_read(s, rs, info);
    else
      hb_read(s, rs, info);
    rs->merge_duplicates();
  }
  return info;
}

}  // namespace

extern "C" int migmres_matrix_file_info(const char *path, long long *n_global, long long *nnz_file, int *symmetric) {
  return guard([&] {
    const FileInfo fi = read_file(path, nullptr, 1, 0);
    if (n_global) *n_global = fi.nrows;
    if (nnz_file) *nnz_file = fi.nnz_file;
    if (symmetric) *symmetric = fi.symmetric;
  });
}

extern "C" int migmres_matrix_file_rows(const char *path, long long first, int n_local, long long *rowptr_out,
                                        long long *gcols_out, double *vals_out, long long *nnz_out) {
  return guard([&] {
    MIG_CHECK(nnz_out && n_local >= 0 && first >= 0, "matrix_file_rows: bad arguments");
    RowSet rs;
    rs.init(first, n_local);
    read_file(path, &rs, 1, 0);
    *nnz_out = rs.nnz();
    if (rowptr_out || gcols_out || vals_out) rs.flatten(rowptr_out, gcols_out, vals_out);
  });
}

extern "C" int migmres_crs_read_file(migmres_ctx *ctx, const char *path, migmres_crs **out) {
  return guard([&] {
    MIG_CHECK(ctx && out, "crs_read_file: null argument");
    RowSet rs;
    rs.n_local = -1;
    const FileInfo fi = read_file(path, &rs, ctx->nranks, ctx->rank);
    std::vector<long long> rp(rs.n_local + 1), gc(rs.nnz());
    std::vector<double> v(gc.size());
    rs.flatten(rp.data(), gc.data(), v.data());
    *out = crs_create(ctx, fi.nrows, rs.first, rs.n_local, rp.data(), gc.data(), v.data());
  });
}
