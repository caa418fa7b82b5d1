// Host-side index maps: uniform row map, Epetra column map, import plan, local CRS and the
// Galeri stencil generators.  Pure C++ (no GPU calls) so the plans are testable on a CPU.
#include "plan.h"

#include <algorithm>
#include <climits>
#include <cstring>
#include <numeric>
#include <unordered_map>
#include <unordered_set>

namespace migmres {

// Epetra_BlockMap::ConstructAutoUniform (epetra/src/Epetra_BlockMap.cpp:60-107).
void uniform_map(long long n_global, int nranks, int rank, long long *first, int *n_local) {
  const long long base = n_global / nranks;
  const long long rem = n_global % nranks;
  long long start = (long long)rank * (base + 1);
  long long n = base;
  if (rank < rem)
    n += 1;
  else
    start -= rank - rem;
  *first = start;
  *n_local = (int)n;
}

int owner_of(long long gid, long long n_global, int nranks) {
  const long long base = n_global / nranks;
  const long long rem = n_global % nranks;
  const long long cut = rem * (base + 1);
  if (gid < cut) return (int)(gid / (base + 1));
  return (int)(rem + (gid - cut) / (base > 0 ? base : 1));
}

// Epetra_Util::Sort, ascending, int keys (epetra/src/Epetra_Util.cpp:113-156): the
// gap-halving shell sort.  Not stable; companions move with their keys.
void epetra_shell_sort(std::vector<int> &keys, std::vector<long long> *c1, std::vector<int> *c2) {
  const int n = (int)keys.size();
  int m = n / 2;
  while (m > 0) {
    const int max = n - m;
    for (int j = 0; j < max; ++j) {
      for (int k = j; k >= 0; k -= m) {
        if (keys[k + m] >= keys[k]) break;
        std::swap(keys[k + m], keys[k]);
        if (c1) std::swap((*c1)[k + m], (*c1)[k]);
        if (c2) std::swap((*c2)[k + m], (*c2)[k]);
      }
    }
    m = m / 2;
  }
}

// Epetra_CrsGraph::MakeColMap_int (epetra/src/Epetra_CrsGraph.cpp:1348-1524), default
// SortGhostsAssociatedWithEachProcessor_ = false.
std::vector<long long> make_colmap(long long n_global, int nranks, long long first, int n_local,
                                   const long long *rowptr, const long long *gcols) {
  std::vector<char> present((size_t)n_local, 0);
  long long n_present = 0;
  std::vector<long long> remote;
  std::unordered_set<long long> seen;
  const long long nnz = rowptr[n_local];
  for (long long e = 0; e < nnz; ++e) {
    const long long g = gcols[e];
    if (g >= first && g < first + n_local) {
      char &p = present[(size_t)(g - first)];
      if (!p) {
        p = 1;
        ++n_present;
      }
    } else if (seen.insert(g).second) {
      remote.push_back(g);
    }
  }
  if (nranks == 1) {
    if (!remote.empty()) throw Error(MIGMRES_EINVAL, "column ids outside the domain map on one rank");
    if (n_present == n_local) {
      std::vector<long long> cm((size_t)n_local);
      std::iota(cm.begin(), cm.end(), first);
      return cm;
    }
  }
  std::vector<int> pids(remote.size());
  for (size_t i = 0; i < remote.size(); ++i) pids[i] = owner_of(remote[i], n_global, nranks);
  epetra_shell_sort(pids, &remote, nullptr);
  std::vector<long long> cm;
  cm.reserve((size_t)n_present + remote.size());
  for (int i = 0; i < n_local; ++i)
    if (present[(size_t)i] || n_present == n_local) cm.push_back(first + i);
  cm.insert(cm.end(), remote.begin(), remote.end());
  return cm;
}

// Remote part of Epetra_Import::Construct (epetra/src/Epetra_Import.cpp:292-440).
RemotePlan make_remotes(long long n_global, int nranks, long long first, int n_local,
                        const long long *colmap, int n_cols) {
  RemotePlan p;
  const int mn = std::min(n_local, n_cols);
  int same = 0;
  while (same < mn && colmap[same] == first + same) ++same;
  p.num_same = same;
  for (int i = same; i < n_cols; ++i) {
    const long long g = colmap[i];
    if (g >= first && g < first + n_local) {
      p.permute_to.push_back(i);
      p.permute_from.push_back((int)(g - first));
    } else {
      p.remote_lids.push_back(i);
      p.remote_gids.push_back(g);
      p.remote_pids.push_back(owner_of(g, n_global, nranks));
    }
  }
  epetra_shell_sort(p.remote_pids, &p.remote_gids, &p.remote_lids);
  return p;
}

// MakeIndicesLocal + SortEntries (epetra/src/Epetra_CrsMatrix.cpp:1147-1199): local ids via
// the column map, each row's entries ordered by ascending local id.
void local_crs(int n_local, const long long *rowptr, const long long *gcols, const double *vals,
               const long long *colmap, int n_cols, long long first, int *lcols_out,
               double *vals_out) {
  // Owned GIDs map by offset when the column map starts with the whole domain.
  int same = 0;
  while (same < std::min(n_local, n_cols) && colmap[same] == first + same) ++same;
  std::unordered_map<long long, int> lut;
  for (int i = same; i < n_cols; ++i) lut.emplace(colmap[i], i);
  std::vector<std::pair<int, double>> row;
  for (int r = 0; r < n_local; ++r) {
    const long long b = rowptr[r], e = rowptr[r + 1];
    row.clear();
    for (long long q = b; q < e; ++q) {
      const long long g = gcols[q];
      int lid;
      if (g >= first && g < first + same)
        lid = (int)(g - first);
      else {
        auto it = lut.find(g);
        if (it == lut.end()) throw Error(MIGMRES_EINVAL, "column id missing from column map");
        lid = it->second;
      }
      row.emplace_back(lid, vals[q]);
    }
    std::sort(row.begin(), row.end(),
              [](const std::pair<int, double> &a, const std::pair<int, double> &b) { return a.first < b.first; });
    for (size_t i = 0; i < row.size(); ++i) {
      lcols_out[b + (long long)i] = row[i].first;
      vals_out[b + (long long)i] = row[i].second;
    }
  }
}

// Galeri Cross2D / Cross3D rows in InsertGlobalValues order
// (galeri/src-epetra/CrsMatrices/Galeri_Cross2D.h, Galeri_Cross3D.h:78-128;
// neighbours: galeri/src-epetra/Galeri_Utils.cpp:331-398); "Brick3D" is the 27-point
// Xpetra Brick3D (galeri/src-xpetra/Galeri_XpetraMatrixTypes.hpp:533-630) with a = 26,
// b..g = -1 and Dirichlet truncation on every face (boundary rows keep 26).
//
// "FlanProxy" (not a Galeri matrix): a stand-in of BASELINE config 4's SuiteSparse
// Flan_1565 (3-D hexahedral FE model of a flange, 3 dofs per node, ~73 nnz per row), which is
// not in this image.  Nodes on an nx x ny x nz grid, 3 dofs each; node v couples to every
// in-range node of its 3x3x3 neighbourhood except a deterministic 1/13 of the edges
// (symmetric: decided on the unordered pair), giving ~73 nnz per row at 81 x 81 x 80 nodes
// (1,574,640 rows).  The node numbering is scrambled along each grid line
// (ix -> (32 ix + 7) mod nx, nx coprime to 32) so a row's columns are irregular, as in an
// unstructured mesh.  Off-diagonal values -(h+1)/997 with h a hash of (row, column); the
// diagonal is 1 + the sum of the row's off-diagonal magnitudes (diagonally dominant).
static inline unsigned long long mix64(unsigned long long x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdULL;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ULL;
  x ^= x >> 33;
  return x;
}

static void flan_proxy_rows(int nx, int ny, int nz, long long first, int n_local, std::vector<long long> &rowptr,
                            std::vector<long long> &gcols, std::vector<double> &vals) {
  MIG_CHECK(nx % 2 == 1 && nx > 1 && ny > 0 && nz > 0, "FlanProxy: nx must be odd (coprime to 32)");
  int ainv = 1;  // 32^-1 mod nx
  while ((32LL * ainv) % nx != 1) ++ainv;
  auto perm = [&](long long ix) { return (32 * ix + 7) % nx; };
  auto unperm = [&](long long px) { return ((px - 7) % nx + nx) % nx * ainv % nx; };
  const long long nxy = (long long)nx * ny;
  rowptr.assign((size_t)n_local + 1, 0);
  gcols.clear();
  vals.clear();
  gcols.reserve((size_t)n_local * 78);
  vals.reserve((size_t)n_local * 78);
  for (int r = 0; r < n_local; ++r) {
    const long long g = first + r;
    const long long pv = g / 3;
    const long long iz = pv / nxy, iy = (pv % nxy) / nx, ix = unperm(pv % nx);
    const long long v = ix + nx * (iy + ny * iz);
    const size_t row0 = gcols.size();
    size_t diag_at = 0;
    double off = 0.0;
    for (int dz = -1; dz <= 1; ++dz)
      for (int dy = -1; dy <= 1; ++dy)
        for (int dx = -1; dx <= 1; ++dx) {
          const long long jx = ix + dx, jy = iy + dy, jz = iz + dz;
          if (jx < 0 || jx >= nx || jy < 0 || jy >= ny || jz < 0 || jz >= nz) continue;
          const long long u = jx + nx * (jy + ny * jz);
          if (u != v && mix64((unsigned long long)std::min(u, v) * 0x9e3779b97f4a7c15ULL +
                              (unsigned long long)std::max(u, v)) % 13 == 0)
            continue;
          const long long pu = perm(jx) + nx * (jy + ny * jz);
          for (int e = 0; e < 3; ++e) {
            const long long c = 3 * pu + e;
            if (c == g) {
              diag_at = gcols.size();
              gcols.push_back(c);
              vals.push_back(0.0);
              continue;
            }
            const double h = (double)(mix64((unsigned long long)g * 0x100000001b3ULL ^ (unsigned long long)c) % 997);
            const double a = -(h + 1.0) / 997.0;
            gcols.push_back(c);
            vals.push_back(a);
            off += -a;
          }
        }
    (void)row0;
    vals[diag_at] = 1.0 + off;
    rowptr[(size_t)r + 1] = (long long)gcols.size();
  }
}

void galeri_rows(const std::string &kind, int nx, int ny, int nz, long long first, int n_local,
                 std::vector<long long> &rowptr, std::vector<long long> &gcols,
                 std::vector<double> &vals) {
  if (kind == "FlanProxy") {
    flan_proxy_rows(nx, ny, nz, first, n_local, rowptr, gcols, vals);
    return;
  }
  if (kind == "Brick3D") {
    const long long nxy = (long long)nx * ny;
    rowptr.assign((size_t)n_local + 1, 0);
    gcols.clear();
    vals.clear();
    gcols.reserve((size_t)n_local * 27);
    vals.reserve((size_t)n_local * 27);
    for (int r = 0; r < n_local; ++r) {
      const long long g = first + r;
      const long long iz = g / nxy, iy = (g % nxy) / nx, ix = g % nx;
      for (int dz = -1; dz <= 1; ++dz)
        for (int dy = -1; dy <= 1; ++dy)
          for (int dx = -1; dx <= 1; ++dx) {
            if (ix + dx < 0 || ix + dx >= nx || iy + dy < 0 || iy + dy >= ny || iz + dz < 0 || iz + dz >= nz)
              continue;
            gcols.push_back(g + dx + dy * (long long)nx + dz * nxy);
            vals.push_back(dx == 0 && dy == 0 && dz == 0 ? 26.0 : -1.0);
          }
      rowptr[(size_t)r + 1] = (long long)gcols.size();
    }
    return;
  }
  const bool three = kind == "Laplace3D";
  if (!three && kind != "Laplace2D") throw Error(MIGMRES_EINVAL, "unknown Galeri matrix " + kind);
  const long long nxy = (long long)nx * ny;
  const int w = three ? 7 : 5;
  rowptr.assign((size_t)n_local + 1, 0);
  gcols.clear();
  vals.clear();
  gcols.reserve((size_t)n_local * w);
  vals.reserve((size_t)n_local * w);
  const double diag = three ? 6.0 : 4.0;
  for (int r = 0; r < n_local; ++r) {
    const long long g = first + r;
    const long long ixy = three ? g % nxy : g;
    const long long iz = three ? g / nxy : 0;
    const long long ix = ixy % nx, iy = ixy / nx;
    const long long zoff = iz * nxy;
    if (ix != 0) { gcols.push_back(ixy - 1 + zoff); vals.push_back(-1.0); }
    if (ix != nx - 1) { gcols.push_back(ixy + 1 + zoff); vals.push_back(-1.0); }
    if (iy != 0) { gcols.push_back(ixy - nx + zoff); vals.push_back(-1.0); }
    if (iy != ny - 1) { gcols.push_back(ixy + nx + zoff); vals.push_back(-1.0); }
    if (three) {
      if (iz != 0) { gcols.push_back(g - nxy); vals.push_back(-1.0); }
      if (iz != nz - 1) { gcols.push_back(g + nxy); vals.push_back(-1.0); }
    }
    gcols.push_back(g);
    vals.push_back(diag);
    rowptr[(size_t)r + 1] = (long long)gcols.size();
  }
}

bool make_pair_plan(int n_local, const long long *rowptr, const int *xcols, PairPlan &out) {
  const int P = (n_local + 1) / 2;
  out.ptr.assign((size_t)P + 1, 0);
  out.key.clear();
  out.meta.clear();
  out.key.reserve((size_t)(rowptr[n_local] / 2 + 8));
  out.meta.reserve((size_t)(rowptr[n_local] / 2 + 8));
  auto key_of = [&](int c) { return c < n_local ? (c >> 1) : -(1 + ((c - n_local) >> 1)); };
  auto half_of = [&](int c) { return c < n_local ? (c & 1) : ((c - n_local) & 1); };
  // ascending X-space order maps to: owned keys ascending, then ghost keys descending in value
  auto rank_of = [&](int c) { return c < n_local ? (long long)(c >> 1) : (1LL << 40) + ((c - n_local) >> 1); };
  for (int p = 0; p < P; ++p) {
    const int rows[2] = {2 * p, 2 * p + 1};
    long long b[2], e[2];
    for (int h = 0; h < 2; ++h) {
      if (rows[h] < n_local) {
        b[h] = rowptr[rows[h]];
        e[h] = rowptr[rows[h] + 1];
      } else {
        b[h] = e[h] = 0;
      }
      if (e[h] - b[h] > kPairMaxRow) return false;
    }
    long long i0 = b[0], i1 = b[1];
    int nk = 0;
    while (i0 < e[0] || i1 < e[1]) {
      const long long r0 = i0 < e[0] ? rank_of(xcols[i0]) : (1LL << 62);
      const long long r1 = i1 < e[1] ? rank_of(xcols[i1]) : (1LL << 62);
      const long long r = r0 < r1 ? r0 : r1;
      const int key = key_of(r == r0 ? xcols[i0] : xcols[i1]);
      unsigned short m = 0xFFFF;
      long long *it[2] = {&i0, &i1};
      for (int h = 0; h < 2; ++h) {
        // at most two entries of a row share a key (low half first in ascending order)
        while (*it[h] < e[h] && rank_of(xcols[*it[h]]) == r) {
          const int hf = half_of(xcols[*it[h]]);
          const int shift = 4 * (2 * h + hf);
          if (((m >> shift) & 0xF) != 0xF) return false;  // repeated column
          m = (unsigned short)((m & ~(0xF << shift)) | ((int)(*it[h] - b[h]) << shift));
          ++*it[h];
        }
      }
      out.key.push_back(key);
      out.meta.push_back(m);
      if (++nk > kPairMaxKeys) return false;
    }
    if (nk > out.max_keys) out.max_keys = nk;
    out.ptr[(size_t)p + 1] = (int)out.key.size();
  }
  // padding so the kernel's clamped reads of kPairMaxKeys slots stay in bounds
  for (int i = 0; i < kPairMaxKeys; ++i) {
    out.key.push_back(0);
    out.meta.push_back(0xFFFF);
  }
  return true;
}

void make_pair_sell(int n_local, const long long *rowptr, const double *lvals, const PairPlan &plan, PairSell &out) {
  const int P = (n_local + 1) / 2;
  const int nchunks = (P + 63) / 64;
  int rmax = 1;
  for (int r = 0; r < n_local; ++r) rmax = std::max(rmax, (int)(rowptr[r + 1] - rowptr[r]));
  const int maxk = std::max(plan.max_keys, 1);
  out.rmax = rmax;
  out.maxk = maxk;
  out.v.assign((size_t)nchunks * 2 * rmax * 64, 0.0);
  out.k.assign((size_t)nchunks * maxk * 64, 0);
  out.m.assign((size_t)nchunks * maxk * 64, 0xFFFF);
  for (int p = 0; p < P; ++p) {
    const int chunk = p / 64, lane = p % 64;
    for (int h = 0; h < 2; ++h) {
      const int r = 2 * p + h;
      if (r >= n_local) continue;
      for (long long e = rowptr[r]; e < rowptr[r + 1]; ++e)
        out.v[(((size_t)chunk * 2 + h) * rmax + (size_t)(e - rowptr[r])) * 64 + lane] = lvals[e];
    }
    const int u0 = plan.ptr[(size_t)p], nu = plan.ptr[(size_t)p + 1] - u0;
    for (int u = 0; u < maxk; ++u) {
      const size_t at = ((size_t)chunk * maxk + u) * 64 + lane;
      if (u < nu) {
        out.k[at] = plan.key[(size_t)(u0 + u)];
        out.m[at] = plan.meta[(size_t)(u0 + u)];
      } else {
        out.k[at] = nu > 0 ? plan.key[(size_t)(u0 + nu - 1)] : p;  // a valid address, map empty
      }
    }
  }
}

bool make_pair_templates(int n_local, const long long *rowptr, const int *xcols, const double *lvals,
                         PairTemplates &out) {
  const int P = (n_local + 1) / 2;
  out = PairTemplates();
  out.npairs = P;
  out.id.assign((size_t)P, kTplNone);
  std::unordered_map<unsigned long long, int> val_index;  // value bit pattern -> dictionary slot
  // a pair's shape: key count, then per key (offset, packed slots); templates are found by
  // comparing against the previous pair's shape first (runs of interior pairs) and then by
  // a hash of the shape
  std::vector<long long> shape, prev;
  int prev_id = -1;
  std::unordered_map<std::string, int> tpl_index;
  std::vector<std::vector<long long>> shapes;
  auto value_slot = [&](double v, int *slot) {
    unsigned long long bits;
    std::memcpy(&bits, &v, sizeof(bits));
    if (out.vals.size() <= 8) {  // stencils: a handful of values, a linear scan beats hashing
      for (size_t i = 0; i < out.vals.size(); ++i)
        if (std::memcmp(&out.vals[i], &bits, sizeof(bits)) == 0) {
          *slot = (int)i;
          return true;
        }
    }
    auto it = val_index.find(bits);
    if (it != val_index.end()) {
      *slot = it->second;
      return true;
    }
    if (out.vals.size() >= 255) return false;
    *slot = (int)out.vals.size();
    val_index.emplace(bits, *slot);
    out.vals.push_back(v);
    return true;
  };
  for (int p = 0; p < P; ++p) {
    long long b[2], e[2];
    bool ghost = false;
    for (int h = 0; h < 2; ++h) {
      const int r = 2 * p + h;
      b[h] = r < n_local ? rowptr[r] : 0;
      e[h] = r < n_local ? rowptr[r + 1] : 0;
      if (e[h] - b[h] > kTplMaxRow) return false;
      for (long long i = b[h]; i < e[h]; ++i) {
        if (xcols[i] >= n_local) ghost = true;
        if (i > b[h] && xcols[i] <= xcols[i - 1]) return false;  // stored order must ascend
      }
    }
    if (ghost) continue;
    // merge the two rows' keys in ascending order (both rows ascend, so key order is each
    // row's stored order, low half before high half)
    shape.clear();
    shape.push_back(0);
    long long i0 = b[0], i1 = b[1];
    int nk = 0;
    while (i0 < e[0] || i1 < e[1]) {
      const int k0 = i0 < e[0] ? (xcols[i0] >> 1) : INT32_MAX;
      const int k1 = i1 < e[1] ? (xcols[i1] >> 1) : INT32_MAX;
      const int key = k0 < k1 ? k0 : k1;
      unsigned slots = 0xFFFFFFFFu;
      long long *it[2] = {&i0, &i1};
      for (int h = 0; h < 2; ++h)
        while (*it[h] < e[h] && (xcols[*it[h]] >> 1) == key) {
          const int sh = 8 * (2 * h + (xcols[*it[h]] & 1));
          int vs;
          if (!value_slot(lvals[*it[h]], &vs)) return false;
          slots = (slots & ~(0xFFu << sh)) | ((unsigned)vs << sh);
          ++*it[h];
        }
      shape.push_back(key - p);
      shape.push_back((long long)slots);
      if (++nk > kTplMaxKeys) return false;
    }
    shape[0] = nk;
    int t;
    if (prev_id >= 0 && shape == prev) {
      t = prev_id;
    } else {
      std::string s((const char *)shape.data(), sizeof(long long) * shape.size());
      auto it = tpl_index.find(s);
      if (it != tpl_index.end()) {
        t = it->second;
      } else {
        if ((int)shapes.size() >= kTplMaxTemplates) return false;
        t = (int)shapes.size();
        tpl_index.emplace(std::move(s), t);
        shapes.push_back(shape);
      }
      prev = shape;
      prev_id = t;
    }
    out.id[(size_t)p] = (unsigned char)t;
    ++out.n_templated;
    out.maxk = std::max(out.maxk, nk);
  }
  if (out.n_templated == 0) return false;
  out.ntpl = (int)shapes.size();
  out.maxk = std::max(out.maxk, 1);
  out.rec.assign((size_t)out.ntpl * out.maxk * 2, 0);
  for (int t = 0; t < out.ntpl; ++t) {
    const auto &sh = shapes[(size_t)t];
    for (int u = 0; u < out.maxk; ++u) {
      int *r = &out.rec[((size_t)t * out.maxk + u) * 2];
      if (u < sh[0]) {
        r[0] = (int)sh[(size_t)(1 + 2 * u)];
        r[1] = (int)(unsigned)sh[(size_t)(2 + 2 * u)];
      } else {
        r[0] = 0;  // padding key: reads the pair itself, adds nothing
        r[1] = (int)0xFFFFFFFFu;
      }
    }
  }
  return true;
}

void make_sell64(int n_local, const long long *rowptr, const int *lcols, const double *lvals, Sell64 &out) {
  const int nchunks = (n_local + 63) / 64;
  out.off.assign((size_t)nchunks + 1, 0);
  out.len.assign((size_t)n_local, 0);
  for (int c = 0; c < nchunks; ++c) {
    int w = 0;
    for (int r = 64 * c; r < std::min(n_local, 64 * c + 64); ++r) {
      out.len[(size_t)r] = (int)(rowptr[r + 1] - rowptr[r]);
      w = std::max(w, out.len[(size_t)r]);
    }
    out.off[(size_t)c + 1] = out.off[(size_t)c] + (long long)w * 64;
  }
  out.cols.assign((size_t)out.off[(size_t)nchunks], 0);
  out.vals.assign((size_t)out.off[(size_t)nchunks], 0.0);
  for (int c = 0; c < nchunks; ++c) {
    const int w = (int)((out.off[(size_t)c + 1] - out.off[(size_t)c]) / 64);
    for (int lane = 0; lane < 64; ++lane) {
      const int r = 64 * c + lane;
      for (int s = 0; s < w; ++s) {
        const size_t at = (size_t)out.off[(size_t)c] + (size_t)s * 64 + lane;
        if (r < n_local && s < out.len[(size_t)r]) {
          out.cols[at] = lcols[rowptr[r] + s];
          out.vals[at] = lvals[rowptr[r] + s];
        } else {
          out.cols[at] = r < n_local ? r : 0;
        }
      }
    }
  }
}

bool make_bsr3(int n_local, const long long *rowptr, const int *lcols, const double *lvals, Bsr3 &out) {
  out = Bsr3();
  const int nbr = n_local / 3;
  out.nbr = nbr;
  out.len.assign((size_t)nbr, 0);
  long long qual_rows = 0;
  for (int b = 0; b < nbr; ++b) {
    const int r0 = 3 * b;
    const long long n0 = rowptr[r0 + 1] - rowptr[r0];
    bool ok = n0 > 0 && n0 % 3 == 0 && rowptr[r0 + 2] - rowptr[r0 + 1] == n0 && rowptr[r0 + 3] - rowptr[r0 + 2] == n0;
    for (long long e = 0; ok && e < n0; ++e) {
      const int c = lcols[rowptr[r0] + e];
      ok = c < n_local && c == lcols[rowptr[r0 + 1] + e] && c == lcols[rowptr[r0 + 2] + e] &&
           (e % 3 != 0 || (c % 3 == 0 && c + 2 < n_local)) && (e % 3 == 0 || c == lcols[rowptr[r0] + e - 1] + 1);
    }
    if (ok) {
      out.len[(size_t)b] = (int)(n0 / 3);
      qual_rows += 3;
    } else {
      for (int r = r0; r < r0 + 3; ++r) out.rest.push_back(r);
    }
  }
  for (int r = 3 * nbr; r < n_local; ++r) out.rest.push_back(r);
  if (qual_rows == 0 || qual_rows * 8 < 7LL * n_local) return false;
  const int nchunks = (nbr + 63) / 64;
  out.off.assign((size_t)nchunks + 1, 0);
  for (int c = 0; c < nchunks; ++c) {
    int w = 0;
    for (int b = 64 * c; b < std::min(nbr, 64 * c + 64); ++b) w = std::max(w, out.len[(size_t)b]);
    out.off[(size_t)c + 1] = out.off[(size_t)c] + (long long)w * 64;
  }
  out.bcol.assign((size_t)out.off[(size_t)nchunks], 0);
  out.vals.assign((size_t)out.off[(size_t)nchunks] * 9, 0.0);
  for (int b = 0; b < nbr; ++b) {
    const int c = b >> 6, lane = b & 63;
    for (int s = 0; s < out.len[(size_t)b]; ++s) {
      const long long slot = out.off[(size_t)c] + 64LL * s;
      out.bcol[(size_t)(slot + lane)] = lcols[rowptr[3 * b] + 3 * s];
      for (int r = 0; r < 3; ++r)
        for (int e = 0; e < 3; ++e)
          out.vals[bsr3_val_index(slot, 3 * r + e, lane)] = lvals[rowptr[3 * b + r] + 3 * s + e];
    }
  }
  return true;
}

bool make_stencil_groups(const PairTemplates &pt, StencilGroups &out) {
  out = StencilGroups();
  std::vector<int> offs;
  for (int t = 0; t < pt.ntpl; ++t)
    for (int u = 0; u < pt.maxk; ++u)
      if ((unsigned)pt.rec[2 * ((size_t)t * pt.maxk + u) + 1] != 0xFFFFFFFFu)
        offs.push_back(pt.rec[2 * ((size_t)t * pt.maxk + u)]);
  std::sort(offs.begin(), offs.end());
  offs.erase(std::unique(offs.begin(), offs.end()), offs.end());
  // groups from the smallest unclaimed offset o: (o, o + 1, o + 2) around centre o + 1 when
  // o + 1 is a key, else o alone as a centre (a y- or z-neighbour of a 7-point stencil)
  for (size_t i = 0; i < offs.size();) {
    const bool run = i + 1 < offs.size() && offs[i + 1] == offs[i] + 1;
    const int c = run ? offs[i] + 1 : offs[i];
    if (!out.center.empty() && c - out.center.back() < 3) return false;
    out.center.push_back(c);
    while (i < offs.size() && offs[i] <= c + 1) ++i;
  }
  out.G = (int)out.center.size();
  if (out.G < 1 || out.G > 9) return false;
  for (size_t g = 1; g < out.center.size(); ++g)
    if (out.center[g] - out.center[g - 1] < 3) return false;
  out.slots.assign((size_t)pt.ntpl * out.G, ~0ULL);
  for (int t = 0; t < pt.ntpl; ++t)
    for (int u = 0; u < pt.maxk; ++u) {
      const int off = pt.rec[2 * ((size_t)t * pt.maxk + u)];
      const unsigned sl = (unsigned)pt.rec[2 * ((size_t)t * pt.maxk + u) + 1];
      if (sl == 0xFFFFFFFFu) continue;  // padding record
      int g = 0;
      while (g < out.G && !(off >= out.center[g] - 1 && off <= out.center[g] + 1)) ++g;
      if (g == out.G) return false;
      const int d = off - out.center[g];
      const unsigned r0lo = sl & 0xFF, r0hi = (sl >> 8) & 0xFF, r1lo = (sl >> 16) & 0xFF, r1hi = sl >> 24;
      unsigned long long &w = out.slots[(size_t)t * out.G + g];
      auto put = [&](int byte, unsigned v) { w = (w & ~(0xFFULL << (8 * byte))) | ((unsigned long long)v << (8 * byte)); };
      if (d == -1) {
        if (r0lo != kTplUnused || r1lo != kTplUnused || r1hi != kTplUnused) return false;
        put(0, r0hi);
      } else if (d == 0) {
        put(1, r0lo);
        put(2, r0hi);
        put(3, r1lo);
        put(4, r1hi);
      } else {
        if (r0lo != kTplUnused || r0hi != kTplUnused || r1hi != kTplUnused) return false;
        put(5, r1lo);
      }
    }
  return true;
}

bool make_march_geometry(const StencilGroups &sg, int ntpl, int npairs, MarchGeometry &out) {
  out = MarchGeometry();
  const int G = sg.G;
  if (G < 1 || npairs <= 0) return false;
  std::vector<int> pos;
  for (int c : sg.center)
    if (c > 0) pos.push_back(c);
  std::sort(pos.begin(), pos.end());
  if (pos.empty()) return false;
  const int nxp = pos[0];
  std::vector<long long> cand;
  for (int c : pos)
    if (c > nxp) {
      cand.push_back(c);
      cand.push_back((long long)c + nxp);
    }
  for (long long P : cand) {
    if (P % nxp != 0 || P / nxp < 2 || P > (1LL << 30)) continue;
    std::vector<int> ga(G), gb(G);
    bool all = true, deep = false;
    for (int g = 0; g < G && all; ++g) {
      bool found = false;
      for (int a : {0, -1, 1})
        for (int b : {0, -1, 1})
          if (!found && (long long)a * P + (long long)b * nxp == sg.center[(size_t)g]) {
            ga[(size_t)g] = a;
            gb[(size_t)g] = b;
            found = true;
          }
      all = found;
      deep = deep || (found && ga[(size_t)g] != 0);
    }
    if (!all || !deep) continue;
    out.nxp = nxp;
    out.plane = (int)P;
    out.nyl = (int)(P / nxp);
    out.nz = (int)((npairs + P - 1) / P);
    out.ga = ga;
    out.gb = gb;
    out.tb.assign((size_t)4 * ntpl, 0);
    for (int t = 0; t < ntpl; ++t) {
      int *b = &out.tb[(size_t)4 * t];
      bool any = false;
      for (int g = 0; g < G; ++g) {
        const unsigned long long w = sg.slots[(size_t)t * G + g];
        bool used = false;
        for (int byte = 0; byte < 6; ++byte) used = used || ((w >> (8 * byte)) & 0xFF) != kTplUnused;
        if (!used) continue;
        if ((w & 0xFF) != kTplUnused) b[0] = 1;
        if (((w >> 40) & 0xFF) != kTplUnused) b[1] = 1;
        b[2] = any ? std::min(b[2], gb[(size_t)g]) : gb[(size_t)g];
        b[3] = any ? std::max(b[3], gb[(size_t)g]) : gb[(size_t)g];
        any = true;
      }
    }
    return true;
  }
  return false;
}

}  // namespace migmres
