// SpMM format plans built on the device from the finished local CSR (d_rowptr int32,
// X-space column ids, values): the same arrays plan.cpp's host builders produce
// (make_pair_plan + make_pair_sell, make_sell64, make_bsr3, make_pair_templates) and the
// runtime's rest / interior / boundary lists, so a device FillComplete never brings the CSR
// back to the host.  Every builder reports "not applicable" exactly where the host one
// returns false; tests compare both through migmres_crs_format_digest.
#pragma once

#include <vector>

#include "internal.h"

namespace migmres {

// MIGMRES_HOST_FORMATS=1: plan.cpp's host builders instead (the local CSR is brought to the
// host); read at every CRS construction.
bool host_formats();

struct DevCsr {
  int n_local = 0;
  long long nnz = 0;
  const int *rowptr = nullptr, *cols = nullptr;
  const double *vals = nullptr;
};

// make_pair_plan + make_pair_sell; the device arrays are allocated here (hipMalloc)
struct DevPairSell {
  double *v = nullptr;
  int *k = nullptr;
  unsigned short *m = nullptr;
  int rmax = 0, maxk = 0;
};
bool dev_pair_sell(hipStream_t s, const DevCsr &A, DevPairSell &out);

struct DevSell64 {
  long long *off = nullptr;
  int *len = nullptr, *cols = nullptr;
  double *vals = nullptr;
};
void dev_sell64(hipStream_t s, const DevCsr &A, DevSell64 &out);

struct DevBsr3 {
  int nbr = 0, n_rest = 0;
  long long *off = nullptr;
  int *len = nullptr, *bcol = nullptr, *rest = nullptr;
  double *vals = nullptr;
  long long nslots = 0;     // off[nchunks]
  double rest_bytes = 0.0;  // sum over the rest rows of 12 * length + 4
};
bool dev_bsr3(hipStream_t s, const DevCsr &A, DevBsr3 &out);

// make_pair_templates: id on the device, the (small) template records and value dictionary on
// the host for the runtime (make_stencil_groups reads them)
struct DevTemplates {
  unsigned char *id = nullptr;
  int ntpl = 0, maxk = 0, npairs = 0;
  long long n_templated = 0;
  std::vector<int> rec;
  std::vector<double> vals;
};
// 1: built; 0: not applicable (the host builder also declines); -1: two pair shapes share a
// hash (nothing allocated): build this plan with make_pair_templates on the host instead.
int dev_templates(hipStream_t s, const DevCsr &A, DevTemplates &out);

// Pairs (by_pairs) or rows whose template id is kTplNone, ascending, into a new device array;
// *rest_bytes = sum of 12 * length + 4 over their rows.
int dev_template_rest(hipStream_t s, const DevCsr &A, const unsigned char *id, int npairs, bool by_pairs,
                      int **out, double *rest_bytes);

// Units (row pairs or rows) that read a ghost column (boundary) and those that do not
// (interior), ascending, into new device arrays.
void dev_halo_units(hipStream_t s, const DevCsr &A, bool by_pairs, int **interior, int *n_interior, int **boundary,
                    int *n_boundary);

// The local transpose for Y = A^T X (Epetra_CrsMatrix::Multiply(TransA = true) -> GeneralMTM,
// epetra/src/Epetra_CrsMatrix.cpp:3587-3650): row c (an X-space column of A: owned row c, or
// ghost slot c - n_local) lists A's entries (r, v) of column c in ascending r -- the order in
// which GeneralMTM's scatter loop (y = 0; for i: for j: y[col_j] += v_j * x_i) adds them, so a
// row-kernel SpMM over it reproduces the loop bit for bit.  Arrays allocated here.
struct DevTrans {
  int *rowptr = nullptr, *cols = nullptr;
  double *vals = nullptr;
};
void dev_transpose(hipStream_t s, const DevCsr &A, int n_out, DevTrans &out);

}  // namespace migmres
