// FillComplete on the device: Epetra's column map, local indices and sorted rows, built from a
// CSR (global column ids, insertion order) that already lives in HBM.
//
//   Epetra_CrsGraph::MakeColMap_int      epetra/src/Epetra_CrsGraph.cpp:1348-1524
//   Epetra_CrsMatrix::MakeIndicesLocal +
//   SortEntries                          epetra/src/Epetra_CrsMatrix.cpp:1147-1199
//   Epetra_Import::Construct (remotes)   epetra/src/Epetra_Import.cpp:292-440
//
// What runs where.  Every O(nnz) step is a kernel: classifying entries (owned / remote),
// marking the owned columns that occur, collecting the distinct remote ids in order of first
// appearance (a stable radix sort by id of the (id, entry) pairs, the run heads, then a sort
// of the heads by entry), turning global ids into X-space ids (owned: local row; remote:
// ghost slot, by binary search in the id-sorted remote list) and sorting every row by local
// id.  The one step Epetra defines sequentially -- Epetra_Util::Sort's gap-halving shell
// sort of the distinct remote ids by owner PID (unstable: ties keep the order the shell sort
// leaves them in) -- runs on the host over the n_remote distinct ids (the halo surface, not
// the matrix), exactly as plan.cpp restates it.  The result is identical to crs_create's host
// path (tests/test_gpu_fillcomplete.py): same column map, import plan and local CSR.
#include <hipcub/hipcub.hpp>

#include "formats.h"

#include "plan.h"
#include "runtime.h"

namespace migmres {

namespace {

__global__ void k_fc_rowptr32(const long long *__restrict__ rp, int *__restrict__ rp32, int n1) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < n1) rp32[i] = (int)rp[i];
}

// owned entry: xcol = local row, mark the row's column as present; remote entry: xcol = -1 and
// (id, entry) appended to the remote list (order fixed afterwards by the sorts)
__global__ void k_fc_classify(long long nnz, const long long *__restrict__ gcols, long long first, int n_local,
                              int *__restrict__ xcol, unsigned char *__restrict__ present, long long *rem_g, int *rem_e,
                              int *counter) {
  const long long e = (long long)blockIdx.x * 256 + threadIdx.x;
  if (e >= nnz) return;
  const long long g = gcols[e];
  if (g >= first && g < first + n_local) {
    xcol[e] = (int)(g - first);
    present[g - first] = 1;
  } else {
    xcol[e] = -1;
    const int i = atomicAdd(counter, 1);
    rem_g[i] = g;
    rem_e[i] = (int)e;
  }
}

__global__ void k_fc_heads(const long long *__restrict__ g, int n, unsigned char *__restrict__ head) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < n) head[i] = (i == 0 || g[i] != g[i - 1]) ? 1 : 0;
}

// number of marked owned columns (one atomic per wave)
__global__ void k_fc_count(const unsigned char *__restrict__ present, int n, int *__restrict__ out) {
  int c = 0;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) c += present[i];
  for (int off = 32; off > 0; off >>= 1) c += __shfl_down(c, off, 64);
  if ((threadIdx.x & 63) == 0 && c) atomicAdd(out, c);
}

__global__ void k_fc_iota(int *__restrict__ v, int n) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < n) v[i] = i;
}

// remote entries: ghost slot by binary search of the id in the id-sorted remote list
__global__ void k_fc_remote_xcol(long long nnz, const long long *__restrict__ gcols, int *__restrict__ xcol,
                                 const long long *__restrict__ sg, const int *__restrict__ sslot, int n_remote,
                                 int n_local, int *bad) {
  const long long e = (long long)blockIdx.x * 256 + threadIdx.x;
  if (e >= nnz || xcol[e] >= 0) return;
  const long long g = gcols[e];
  int lo = 0, hi = n_remote - 1;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (sg[mid] < g)
      lo = mid + 1;
    else
      hi = mid;
  }
  if (n_remote > 0 && sg[lo] == g)
    xcol[e] = n_local + sslot[lo];
  else
    atomicAdd(bad, 1);
}

// SortEntries: each row by ascending local id (= ascending X-space id), values with their
// columns; insertion sort, one thread per row (rows are short; a repeated column keeps its
// input order -- matrices are merged on input, io.cpp)
__global__ void k_fc_sort_rows(int n_local, const long long *__restrict__ rp, int *__restrict__ xcol,
                               double *__restrict__ vals) {
  const int r = blockIdx.x * 256 + threadIdx.x;
  if (r >= n_local) return;
  const long long b = rp[r], e = rp[r + 1];
  for (long long i = b + 1; i < e; ++i) {
    const int c = xcol[i];
    const double v = vals[i];
    long long j = i - 1;
    while (j >= b && xcol[j] > c) {
      xcol[j + 1] = xcol[j];
      vals[j + 1] = vals[j];
      --j;
    }
    xcol[j + 1] = c;
    vals[j + 1] = v;
  }
}

inline int nblk(long long n) { return (int)((n + 255) / 256); }

struct DevBuf {
  void *p = nullptr;
  explicit DevBuf(size_t bytes) { MIG_HIP(hipMalloc(&p, bytes > 0 ? bytes : 8)); }
  ~DevBuf() {
    if (p) (void)hipFree(p);
  }
  template <class T>
  T *as() const {
    return static_cast<T *>(p);
  }
  DevBuf(const DevBuf &) = delete;
  DevBuf &operator=(const DevBuf &) = delete;
};

template <class K, class V>
void sort_pairs(hipStream_t s, const K *kin, K *kout, const V *vin, V *vout, int n) {
  if (n <= 0) return;
  size_t tb = 0;
  MIG_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, kin, kout, vin, vout, n, 0, (int)(8 * sizeof(K)), s));
  DevBuf tmp(tb);
  MIG_HIP(hipcub::DeviceRadixSort::SortPairs(tmp.p, tb, kin, kout, vin, vout, n, 0, (int)(8 * sizeof(K)), s));
  MIG_HIP(hipStreamSynchronize(s));
}

template <class T>
int select_flagged(hipStream_t s, const T *in, const unsigned char *flags, T *out, int n) {
  DevBuf cnt(sizeof(int));
  size_t tb = 0;
  MIG_HIP(hipcub::DeviceSelect::Flagged(nullptr, tb, in, flags, out, cnt.as<int>(), n, s));
  DevBuf tmp(tb);
  MIG_HIP(hipcub::DeviceSelect::Flagged(tmp.p, tb, in, flags, out, cnt.as<int>(), n, s));
  int h = 0;
  MIG_HIP(hipMemcpyAsync(&h, cnt.p, sizeof(int), hipMemcpyDeviceToHost, s));
  MIG_HIP(hipStreamSynchronize(s));
  return h;
}

}  // namespace

void fill_complete_device(migmres_crs *A, const long long *d_rowptr, const long long *d_gcols, const double *d_vals_in,
                          std::vector<long long> &rowptr, std::vector<int> &lcols, std::vector<double> &lvals) {
  migmres_ctx *ctx = A->ctx;
  hipStream_t s = ctx->stream;
  const int n_local = A->n_local;
  const long long first = A->first, n_global = A->n_global;
  rowptr.resize((size_t)n_local + 1);
  MIG_HIP(hipMemcpyAsync(rowptr.data(), d_rowptr, sizeof(long long) * (n_local + 1), hipMemcpyDeviceToHost, s));
  MIG_HIP(hipStreamSynchronize(s));
  const long long nnz = rowptr[(size_t)n_local];
  MIG_CHECK(rowptr[0] == 0 && nnz >= 0, "device CRS: rowptr must start at 0");
  MIG_CHECK(nnz < (1LL << 31), "local nnz must fit int32 row offsets");
  A->nnz = nnz;

  // the operator's arrays: int32 row offsets, X-space columns, values padded by 8 zeros
  MIG_HIP(hipMalloc(&A->d_rowptr, sizeof(int) * (n_local + 1)));
  MIG_HIP(hipMalloc(&A->d_cols, sizeof(int) * (nnz > 0 ? nnz : 1)));
  MIG_HIP(hipMalloc(&A->d_vals, sizeof(double) * (nnz + 8)));
  MIG_HIP(hipMemsetAsync(A->d_vals, 0, sizeof(double) * (nnz + 8), s));
  if (nnz) MIG_HIP(hipMemcpyAsync(A->d_vals, d_vals_in, sizeof(double) * nnz, hipMemcpyDeviceToDevice, s));
  k_fc_rowptr32<<<nblk(n_local + 1), 256, 0, s>>>(d_rowptr, A->d_rowptr, n_local + 1);

  setup_mark("fc: rowptr + alloc");
  // 1. classify entries, mark present owned columns, collect remote (id, entry) pairs
  DevBuf present((size_t)n_local), counter(sizeof(int)), bad(sizeof(int));
  DevBuf rem_g(sizeof(long long) * (size_t)nnz), rem_e(sizeof(int) * (size_t)nnz);
  MIG_HIP(hipMemsetAsync(present.p, 0, (size_t)n_local, s));
  MIG_HIP(hipMemsetAsync(counter.p, 0, sizeof(int), s));
  MIG_HIP(hipMemsetAsync(bad.p, 0, sizeof(int), s));
  if (nnz)
    k_fc_classify<<<nblk(nnz), 256, 0, s>>>(nnz, d_gcols, first, n_local, A->d_cols, present.as<unsigned char>(),
                                             rem_g.as<long long>(), rem_e.as<int>(), counter.as<int>());
  int n_rem_entries = 0;
  MIG_HIP(hipMemcpyAsync(&n_rem_entries, counter.p, sizeof(int), hipMemcpyDeviceToHost, s));
  MIG_HIP(hipStreamSynchronize(s));
  MIG_CHECK(!(ctx->nranks == 1 && n_rem_entries > 0), "column ids outside the domain map on one rank");

  // 2. distinct remote ids in order of first appearance: restore entry order (sort by entry),
  //    stable sort by id (each id's run then starts at its first entry), run heads, sort the
  //    heads by entry
  std::vector<long long> remote;  // first-appearance order
  if (n_rem_entries > 0) {
    const int m = n_rem_entries;
    DevBuf e1(sizeof(int) * m), g1(sizeof(long long) * m), g2(sizeof(long long) * m), e2(sizeof(int) * m);
    sort_pairs(s, rem_e.as<int>(), e1.as<int>(), rem_g.as<long long>(), g1.as<long long>(), m);
    sort_pairs(s, g1.as<long long>(), g2.as<long long>(), e1.as<int>(), e2.as<int>(), m);
    DevBuf head((size_t)m), ug(sizeof(long long) * m), ue(sizeof(int) * m);
    k_fc_heads<<<nblk(m), 256, 0, s>>>(g2.as<long long>(), m, head.as<unsigned char>());
    const int nr = select_flagged(s, g2.as<long long>(), head.as<unsigned char>(), ug.as<long long>(), m);
    select_flagged(s, e2.as<int>(), head.as<unsigned char>(), ue.as<int>(), m);
    DevBuf fe(sizeof(int) * nr), fg(sizeof(long long) * nr);
    sort_pairs(s, ue.as<int>(), fe.as<int>(), ug.as<long long>(), fg.as<long long>(), nr);
    remote.resize((size_t)nr);
    MIG_HIP(hipMemcpyAsync(remote.data(), fg.p, sizeof(long long) * nr, hipMemcpyDeviceToHost, s));
    MIG_HIP(hipStreamSynchronize(s));
  }

  setup_mark("fc: classify + remotes");
  // 3. MakeColMap's remote order (Epetra_Util::Sort by owner PID, host: n_remote ids) and the
  //    column map: the owned columns that occur (all of them when every one occurs), then
  //    the remotes
  std::vector<int> pids(remote.size());
  for (size_t i = 0; i < remote.size(); ++i) pids[i] = owner_of(remote[i], n_global, ctx->nranks);
  epetra_shell_sort(pids, &remote, nullptr);
  long long n_present = 0;
  std::vector<unsigned char> pres;
  {
    // count on the host only when some owned column is missing (rare: download the marks)
    int all = 0;
    DevBuf flag(sizeof(int));
    MIG_HIP(hipMemsetAsync(flag.p, 0, sizeof(int), s));
    if (n_local > 0)
      k_fc_count<<<std::min(nblk(n_local), 4096), 256, 0, s>>>(present.as<unsigned char>(), n_local, flag.as<int>());
    MIG_HIP(hipMemcpyAsync(&all, flag.p, sizeof(int), hipMemcpyDeviceToHost, s));
    MIG_HIP(hipStreamSynchronize(s));
    n_present = all;
    if (n_present < n_local) {
      pres.resize((size_t)n_local);
      MIG_HIP(hipMemcpy(pres.data(), present.p, (size_t)n_local, hipMemcpyDeviceToHost));
    }
  }
  A->colmap.clear();
  A->colmap.reserve((size_t)(n_present == n_local ? n_local : n_present) + remote.size());
  for (int i = 0; i < n_local; ++i)
    if (n_present == n_local || pres[(size_t)i]) A->colmap.push_back(first + i);
  A->colmap.insert(A->colmap.end(), remote.begin(), remote.end());
  A->n_cols = (int)A->colmap.size();
  A->plan = make_remotes(n_global, ctx->nranks, first, n_local, A->colmap.data(), A->n_cols);
  const int n_remote = (int)A->plan.remote_gids.size();
  MIG_CHECK(n_remote == (int)remote.size(), "device FillComplete: remote lists disagree");

  setup_mark("fc: colmap + import");
  // 4. remote X-space ids (ghost slot = import order), 5. SortEntries
  if (n_remote > 0) {
    DevBuf rg(sizeof(long long) * n_remote), slot(sizeof(int) * n_remote), sg(sizeof(long long) * n_remote),
        sslot(sizeof(int) * n_remote);
    MIG_HIP(hipMemcpyAsync(rg.p, A->plan.remote_gids.data(), sizeof(long long) * n_remote, hipMemcpyHostToDevice, s));
    k_fc_iota<<<nblk(n_remote), 256, 0, s>>>(slot.as<int>(), n_remote);
    sort_pairs(s, rg.as<long long>(), sg.as<long long>(), slot.as<int>(), sslot.as<int>(), n_remote);
    k_fc_remote_xcol<<<nblk(nnz), 256, 0, s>>>(nnz, d_gcols, A->d_cols, sg.as<long long>(), sslot.as<int>(), n_remote,
                                               n_local, bad.as<int>());
    int nbad = 0;
    MIG_HIP(hipMemcpyAsync(&nbad, bad.p, sizeof(int), hipMemcpyDeviceToHost, s));
    MIG_HIP(hipStreamSynchronize(s));
    MIG_CHECK(nbad == 0, "device FillComplete: remote column missing from the column map");
  }
  if (n_local > 0) k_fc_sort_rows<<<nblk(n_local), 256, 0, s>>>(n_local, d_rowptr, A->d_cols, A->d_vals);
  MIG_HIP(hipGetLastError());

  // the SpMM format plans (pair / template / SELL-64 / 3x3 blocks: this library's, not
  // Epetra's) are built on the device from the finished local CSR (formats.hip); only
  // MIGMRES_HOST_FORMATS=1 brings it to the host for plan.cpp's builders
  if (!host_formats()) return;
  lcols.resize((size_t)nnz);
  lvals.resize((size_t)nnz);
  if (nnz) {
    MIG_HIP(hipMemcpyAsync(lcols.data(), A->d_cols, sizeof(int) * nnz, hipMemcpyDeviceToHost, s));
    MIG_HIP(hipMemcpyAsync(lvals.data(), A->d_vals, sizeof(double) * nnz, hipMemcpyDeviceToHost, s));
  }
  MIG_HIP(hipStreamSynchronize(s));
}

}  // namespace migmres
