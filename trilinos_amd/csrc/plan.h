// Host-side index maps and import plans (bit-exact restatement of Epetra's rules).
#pragma once

#include <string>
#include <vector>

#include "internal.h"

namespace migmres {

void uniform_map(long long n_global, int nranks, int rank, long long *first, int *n_local);
int owner_of(long long gid, long long n_global, int nranks);
void epetra_shell_sort(std::vector<int> &keys, std::vector<long long> *c1, std::vector<int> *c2);

std::vector<long long> make_colmap(long long n_global, int nranks, long long first, int n_local,
                                   const long long *rowptr, const long long *gcols);

struct RemotePlan {
  int num_same = 0;
  std::vector<int> permute_to, permute_from;
  std::vector<int> remote_lids, remote_pids;
  std::vector<long long> remote_gids;
};

RemotePlan make_remotes(long long n_global, int nranks, long long first, int n_local,
                        const long long *colmap, int n_cols);

void local_crs(int n_local, const long long *rowptr, const long long *gcols, const double *vals,
               const long long *colmap, int n_cols, long long first, int *lcols_out,
               double *vals_out);

// Row-pair gather plan for k_spmm_pair (kernels.hip).  Rows (2p, 2p+1) share 16-byte
// loads of aligned X pairs: for every row pair the sorted distinct pair keys of both rows'
// X-space columns (owned column c -> c >> 1; ghost column n_local + g -> -(1 + (g >> 1))),
// and per key a 16-bit map of which entry of each row reads its low / high half
// (nibbles: row 0 low, row 0 high, row 1 low, row 1 high; 15 = none).  Each row's entries
// stay in stored (ascending X-space) order, so the kernel's sums are the reference's.
// Returns false (no plan) if a row has more than kPairMaxRow entries, a pair needs more
// than kPairMaxKeys keys, or a row repeats a column.
constexpr int kPairMaxRow = 8, kPairMaxKeys = 12;
struct PairPlan {
  std::vector<int> ptr, key;
  std::vector<unsigned short> meta;
  int max_keys = 0;  // largest key count of any pair (the kernel is instantiated for <= 8 and <= 12)
};
bool make_pair_plan(int n_local, const long long *rowptr, const int *xcols, PairPlan &out);

// The pair plan in the layout k_spmm_pair reads ("SELL-64": per wave of 64 row pairs, slot s
// of all 64 pairs is contiguous), so that every lane's coefficient / key loads coalesce:
//   v[((chunk * 2 + h) * rmax + j) * 64 + lane]  entry j of row 2p + h (0 past the row's end)
//   k[(chunk * maxk + u) * 64 + lane], m[...]    key u and its half map (unused: last key, 0xFFFF)
// with p = 64 chunk + lane, rmax = longest row, maxk = plan.max_keys.
struct PairSell {
  std::vector<double> v;
  std::vector<int> k;
  std::vector<unsigned short> m;
  int rmax = 0, maxk = 0;
};
void make_pair_sell(int n_local, const long long *rowptr, const double *lvals, const PairPlan &plan, PairSell &out);

// SELL-64 copy of a local CSR for the general SpMM kernel (k_spmm_sell): rows in chunks of
// 64; chunk c holds its entries slot-major, entry s of row 64c + lane at
// off[c] + s * 64 + lane for s < width[c] (the chunk's longest row); padding slots hold
// column = the row itself and value 0 and are never summed (len[r] bounds the sum).
struct Sell64 {
  std::vector<long long> off;  // nchunks + 1
  std::vector<int> len;        // n_local
  std::vector<int> cols;
  std::vector<double> vals;
};
void make_sell64(int n_local, const long long *rowptr, const int *lcols, const double *lvals, Sell64 &out);

// 3 x 3 block form of a CRS whose rows come in triples with one column set made of whole
// aligned column triples (3 unknowns per mesh node, as in SuiteSparse Flan_1565), DETECTED
// from the local CRS -- nothing is assumed: block row b = rows 3b .. 3b + 2 qualifies when the
// three rows have identical sorted column lists consisting of complete triples 3j, 3j + 1,
// 3j + 2 of owned columns.  Qualifying block rows are stored SELL-64 by block: slot s of the
// 64 block rows of a chunk at off[chunk] + 64 s + lane holds the block's first column 3j in
// bcol and its 9 values (row-major, value 3 r + e at bsr3_val_index(off[chunk] + 64 s, 3 r + e,
// lane)) in vals; len[b] = the block row's blocks (0 for a block row that does not qualify).
// rest lists the rows of non-qualifying block rows (and a last partial triple) for the
// row kernel.  Returns false when fewer than 7/8 of the rows qualify (format not used).
struct Bsr3 {
  int nbr = 0;
  std::vector<long long> off;  // nchunks + 1, in block slots
  std::vector<int> len;        // nbr
  std::vector<int> bcol;
  std::vector<double> vals;
  std::vector<int> rest;
};
bool make_bsr3(int n_local, const long long *rowptr, const int *lcols, const double *lvals, Bsr3 &out);
// Where value e (= 3 r + c, row r and column c of the block) of the block at slot base S
// (= off[chunk] + 64 s) for lane `lane` is stored: the first eight values of the 64 lanes as
// four pair-interleaved strips (value 2 m and 2 m + 1 of a lane adjacent: one 16-byte load
// each), the ninth as a plain strip -- 5 loads per block instead of 9.
__host__ __device__ inline size_t bsr3_val_index(long long S, int e, int lane) {
  return (size_t)(9 * S + (e < 8 ? 128 * (e >> 1) + 2 * lane + (e & 1) : 512 + lane));
}

// Row-pair templates for k_spmm_tpl (kernels.hip): a compressed form of the pair plan for
// matrices whose row pairs repeat a small number of shapes (stencils: the interior pairs of
// a 7- or 27-point operator are all alike, boundary pairs add a few dozen variants).  A
// pair's template is its keys relative to the pair index (owned columns only), and per key
// which entry of which row reads the low / high half, with the coefficient stored as an
// index into a value dictionary.  Per pair the matrix then costs ONE byte (its template id)
// instead of 12 bytes per entry; the sums still run in stored order with the same products,
// so the result is bit-identical to k_spmm / k_spmm_pair.
//   id[p]                   template of pair p (kTplNone: the pair reads a ghost column and
//                           is left to the fallback kernel)
//   rec[(t * maxk + u)]     key u of template t: .x = key offset (X rows 2 (p + off), +1),
//                           .y = four value-dictionary slots (bytes: row 0 low, row 0 high,
//                           row 1 low, row 1 high; kTplUnused = no entry); templates with
//                           fewer keys are padded with (0, all unused)
//   vals[i]                 the value dictionary (distinct coefficients, bit patterns)
// Returns false (format not used) when a row has more than kTplMaxRow entries, a pair more
// than kTplMaxKeys keys, there are more than kTplMaxTemplates templates or more than 255
// distinct values, a row repeats a column, or no pair is templated.
constexpr int kTplMaxRow = 32, kTplMaxKeys = 32, kTplMaxTemplates = 128;
constexpr unsigned char kTplNone = 0xFF, kTplUnused = 0xFF;
struct PairTemplates {
  int ntpl = 0, maxk = 0, npairs = 0, n_templated = 0;
  std::vector<unsigned char> id;
  std::vector<int> rec;  // 2 ints per key: offset, packed slots
  std::vector<double> vals;
};
bool make_pair_templates(int n_local, const long long *rowptr, const int *xcols, const double *lvals,
                         PairTemplates &out);

// Lane-shared form of the templates for k_spmm_tpl3 (kernels.hip): every key offset of every
// template lies in one of G groups of three consecutive pair offsets (c_g - 1, c_g, c_g + 1)
// -- the x-neighbours along one (dy, dz) line of a 3-D stencil on an even-nx grid -- and each
// row reads only the halves a 3-point line stencil reads: row 0 (even x) the high half of
// c_g - 1 and both halves of c_g; row 1 both halves of c_g and the low half of c_g + 1.  A
// lane then loads only the centre pair of each group and takes the neighbours' halves from the
// adjacent lanes.  slots[(t * G + g)] packs the group's six value-dictionary slots (bytes 0-5:
// row 0 from c-1 high, c low, c high; row 1 from c low, c high, c+1 low; kTplUnused = none).
// Groups must be at least 3 apart so each row's sums keep their stored (ascending) order.
// Returns false when the templates do not have this shape.
struct StencilGroups {
  int G = 0;
  std::vector<int> center;
  std::vector<unsigned long long> slots;
};
bool make_stencil_groups(const PairTemplates &pt, StencilGroups &out);

// Geometry of the stencil groups for the 2.5-D march (k_spmm_march, kernels.hip): pair
// offsets nxp (one grid line) and plane = nxp * nyl (one grid plane) such that every group
// centre is ga * plane + gb * nxp with ga, gb in {-1, 0, 1} and some ga != 0 (a 3-D stencil);
// nz = planes covering npairs.  nxp is the smallest positive centre, plane the first
// candidate (a positive centre, or one plus nxp) that decomposes every centre.  tb holds per
// template {uses a left-neighbour half, uses a right-neighbour half, lowest gb, highest gb}
// of its used groups, for the device check that no templated pair's keys leave its line or
// plane under this geometry (march_check).  Returns false when no such geometry exists.
struct MarchGeometry {
  int nxp = 0, nyl = 0, plane = 0, nz = 0;
  std::vector<int> ga, gb, tb;
};
bool make_march_geometry(const StencilGroups &sg, int ntpl, int npairs, MarchGeometry &out);

void galeri_rows(const std::string &kind, int nx, int ny, int nz, long long first, int n_local,
                 std::vector<long long> &rowptr, std::vector<long long> &gcols,
                 std::vector<double> &vals);

}  // namespace migmres
