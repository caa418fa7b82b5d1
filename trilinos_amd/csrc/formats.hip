// SpMM format plans on the device (see formats.h).  Each kernel restates one host builder of
// plan.cpp over a thread per row pair / row / block row; the orders the host builders fix by
// their sequential scans (value dictionary slots and template ids in order of first
// appearance, rest lists ascending) come from stable radix sorts and ordered stream
// compaction, so the arrays are identical, not merely equivalent.
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "formats.h"
#include "plan.h"

namespace migmres {
namespace {

inline int nblk(long long n) { return (int)((n + 255) / 256); }

struct Buf {
  void *p = nullptr;
  explicit Buf(size_t bytes) { MIG_HIP(hipMalloc(&p, bytes > 0 ? bytes : 8)); }
  ~Buf() {
    if (p) hipFree(p);
  }
  template <class T>
  T *as() const {
    return (T *)p;
  }
  Buf(const Buf &) = delete;
  Buf &operator=(const Buf &) = delete;
};

template <class T>
T dev_max(hipStream_t s, const T *in, int n, T init) {
  if (n <= 0) return init;
  Buf out(sizeof(T));
  size_t tb = 0;
  MIG_HIP(hipcub::DeviceReduce::Reduce(nullptr, tb, in, out.as<T>(), n, hipcub::Max(), init, s));
  Buf tmp(tb);
  MIG_HIP(hipcub::DeviceReduce::Reduce(tmp.p, tb, in, out.as<T>(), n, hipcub::Max(), init, s));
  T h;
  MIG_HIP(hipMemcpyAsync(&h, out.p, sizeof(T), hipMemcpyDeviceToHost, s));
  MIG_HIP(hipStreamSynchronize(s));
  return h;
}

template <class T>
T dev_min(hipStream_t s, const T *in, int n, T init) {
  if (n <= 0) return init;
  Buf out(sizeof(T));
  size_t tb = 0;
  MIG_HIP(hipcub::DeviceReduce::Reduce(nullptr, tb, in, out.as<T>(), n, hipcub::Min(), init, s));
  Buf tmp(tb);
  MIG_HIP(hipcub::DeviceReduce::Reduce(tmp.p, tb, in, out.as<T>(), n, hipcub::Min(), init, s));
  T h;
  MIG_HIP(hipMemcpyAsync(&h, out.p, sizeof(T), hipMemcpyDeviceToHost, s));
  MIG_HIP(hipStreamSynchronize(s));
  return h;
}

template <class T>
T dev_sum(hipStream_t s, const T *in, int n) {
  if (n <= 0) return T(0);
  Buf out(sizeof(T));
  size_t tb = 0;
  MIG_HIP(hipcub::DeviceReduce::Sum(nullptr, tb, in, out.as<T>(), n, s));
  Buf tmp(tb);
  MIG_HIP(hipcub::DeviceReduce::Sum(tmp.p, tb, in, out.as<T>(), n, s));
  T h;
  MIG_HIP(hipMemcpyAsync(&h, out.p, sizeof(T), hipMemcpyDeviceToHost, s));
  MIG_HIP(hipStreamSynchronize(s));
  return h;
}

// out[0] = 0, out[i + 1] = in[0] + ... + in[i]
void dev_offsets(hipStream_t s, const long long *in, long long *out, int n) {
  MIG_HIP(hipMemsetAsync(out, 0, sizeof(long long), s));
  if (n <= 0) return;
  size_t tb = 0;
  MIG_HIP(hipcub::DeviceScan::InclusiveSum(nullptr, tb, in, out + 1, n, s));
  Buf tmp(tb);
  MIG_HIP(hipcub::DeviceScan::InclusiveSum(tmp.p, tb, in, out + 1, n, s));
}

// the ids i < n with flag[i] != 0, ascending
int dev_select_ids(hipStream_t s, const unsigned char *flags, int n, int *out) {
  if (n <= 0) return 0;
  Buf cnt(sizeof(int));
  hipcub::CountingInputIterator<int> ids(0);
  size_t tb = 0;
  MIG_HIP(hipcub::DeviceSelect::Flagged(nullptr, tb, ids, flags, out, cnt.as<int>(), n, s));
  Buf tmp(tb);
  MIG_HIP(hipcub::DeviceSelect::Flagged(tmp.p, tb, ids, flags, out, cnt.as<int>(), n, s));
  int h = 0;
  MIG_HIP(hipMemcpyAsync(&h, cnt.p, sizeof(int), hipMemcpyDeviceToHost, s));
  MIG_HIP(hipStreamSynchronize(s));
  return h;
}

template <class T>
int dev_select(hipStream_t s, const T *in, const unsigned char *flags, int n, T *out) {
  if (n <= 0) return 0;
  Buf cnt(sizeof(int));
  size_t tb = 0;
  MIG_HIP(hipcub::DeviceSelect::Flagged(nullptr, tb, in, flags, out, cnt.as<int>(), n, s));
  Buf tmp(tb);
  MIG_HIP(hipcub::DeviceSelect::Flagged(tmp.p, tb, in, flags, out, cnt.as<int>(), n, s));
  int h = 0;
  MIG_HIP(hipMemcpyAsync(&h, cnt.p, sizeof(int), hipMemcpyDeviceToHost, s));
  MIG_HIP(hipStreamSynchronize(s));
  return h;
}

// stable LSD radix sort (equal keys keep their input order)
template <class K, class V>
void dev_sort_pairs(hipStream_t s, const K *kin, K *kout, const V *vin, V *vout, int n) {
  if (n <= 0) return;
  size_t tb = 0;
  MIG_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, kin, kout, vin, vout, n, 0, (int)(8 * sizeof(K)), s));
  Buf tmp(tb);
  MIG_HIP(hipcub::DeviceRadixSort::SortPairs(tmp.p, tb, kin, kout, vin, vout, n, 0, (int)(8 * sizeof(K)), s));
}

__device__ __forceinline__ int row_len(const int *rowptr, int r, int n) { return r < n ? rowptr[r + 1] - rowptr[r] : 0; }

// ------------------------------------------------------------------ pair plan (make_pair_plan)
__device__ __forceinline__ long long pp_rank(int c, int n) {
  return c < n ? (long long)(c >> 1) : (1LL << 40) + ((c - n) >> 1);
}
__device__ __forceinline__ int pp_key(int c, int n) { return c < n ? (c >> 1) : -(1 + ((c - n) >> 1)); }
__device__ __forceinline__ int pp_half(int c, int n) { return c < n ? (c & 1) : ((c - n) & 1); }

// The merge of make_pair_plan for pair p: emit(u, key, meta) per key; the key count, or -1
// where the host builder returns false.
template <class F>
__device__ int pp_walk(const int *rowptr, const int *cols, int n, int p, F emit) {
  int b[2], e[2];
  for (int h = 0; h < 2; ++h) {
    const int r = 2 * p + h;
    b[h] = r < n ? rowptr[r] : 0;
    e[h] = r < n ? rowptr[r + 1] : 0;
    if (e[h] - b[h] > kPairMaxRow) return -1;
  }
  int i[2] = {b[0], b[1]};
  int nk = 0;
  while (i[0] < e[0] || i[1] < e[1]) {
    const long long r0 = i[0] < e[0] ? pp_rank(cols[i[0]], n) : (1LL << 62);
    const long long r1 = i[1] < e[1] ? pp_rank(cols[i[1]], n) : (1LL << 62);
    const long long rr = r0 < r1 ? r0 : r1;
    const int key = pp_key(rr == r0 ? cols[i[0]] : cols[i[1]], n);
    unsigned m = 0xFFFF;
    for (int h = 0; h < 2; ++h)
      while (i[h] < e[h] && pp_rank(cols[i[h]], n) == rr) {
        const int sh = 4 * (2 * h + pp_half(cols[i[h]], n));
        if (((m >> sh) & 0xF) != 0xF) return -1;  // repeated column
        m = (m & ~(0xFu << sh)) | ((unsigned)(i[h] - b[h]) << sh);
        ++i[h];
      }
    emit(nk, key, (unsigned short)m);
    if (++nk > kPairMaxKeys) return -1;
  }
  return nk;
}

__global__ void k_pp_count(const int *rowptr, const int *cols, int n, int P, int *nk, int *rlen) {
  const int p = blockIdx.x * 256 + threadIdx.x;
  if (p >= P) return;
  nk[p] = pp_walk(rowptr, cols, n, p, [](int, int, unsigned short) {});
  rlen[p] = max(row_len(rowptr, 2 * p, n), row_len(rowptr, 2 * p + 1, n));
}

__global__ void k_pp_fill(const int *rowptr, const int *cols, const double *vals, int n, int P, int rmax, int maxk,
                          double *v, int *kk, unsigned short *mm) {
  const int p = blockIdx.x * 256 + threadIdx.x;
  if (p >= P) return;
  const int chunk = p >> 6, lane = p & 63;
  for (int h = 0; h < 2; ++h) {
    const int r = 2 * p + h;
    if (r >= n) continue;
    for (int e = rowptr[r]; e < rowptr[r + 1]; ++e)
      v[(((size_t)chunk * 2 + h) * rmax + (size_t)(e - rowptr[r])) * 64 + lane] = vals[e];
  }
  int last = p;
  const int nu = pp_walk(rowptr, cols, n, p, [&](int u, int key, unsigned short m) {
    const size_t at = ((size_t)chunk * maxk + u) * 64 + lane;
    kk[at] = key;
    mm[at] = m;
    last = key;
  });
  for (int u = nu > 0 ? nu : 0; u < maxk; ++u) {
    const size_t at = ((size_t)chunk * maxk + u) * 64 + lane;
    kk[at] = last;  // a valid address (the pair's last key, or the pair itself), map empty
    mm[at] = 0xFFFF;
  }
}

// ------------------------------------------------------------------ SELL-64 (make_sell64)
__global__ void k_chunk_width(const int *rowptr, int n, int nunits, int unit_rows, long long *w64) {
  // chunk c of 64 units (rows, or block rows of unit_rows rows whose length is len[])
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= (nunits + 63) / 64) return;
  int w = 0;
  for (int u = 64 * c; u < min(nunits, 64 * c + 64); ++u) w = max(w, row_len(rowptr, u * unit_rows, n));
  w64[c] = (long long)w * 64;
}

__global__ void k_sell_fill(const int *rowptr, const int *cols, const double *vals, int n, const long long *off,
                            int *len, int *scol, double *sval) {
  const int r = blockIdx.x * 256 + threadIdx.x;
  const int nchunks = (n + 63) / 64;
  if (r >= nchunks * 64) return;
  const int c = r >> 6, lane = r & 63;
  const int w = (int)((off[c + 1] - off[c]) / 64);
  const int l = row_len(rowptr, r, n);
  if (r < n) len[r] = l;
  for (int s = 0; s < w; ++s) {
    const size_t at = (size_t)off[c] + (size_t)s * 64 + lane;
    if (r < n && s < l) {
      scol[at] = cols[rowptr[r] + s];
      sval[at] = vals[rowptr[r] + s];
    } else {
      scol[at] = r < n ? r : 0;
      sval[at] = 0.0;
    }
  }
}

// ------------------------------------------------------------------ 3 x 3 blocks (make_bsr3)
__global__ void k_b3_qualify(const int *rowptr, const int *cols, int n, int nbr, int *len, unsigned char *rest_flag,
                             double *rest_bytes) {
  const int r = blockIdx.x * 256 + threadIdx.x;
  if (r >= n) return;
  const int b = r / 3;
  bool ok = false;
  if (b < nbr) {
    const int r0 = 3 * b;
    const int n0 = rowptr[r0 + 1] - rowptr[r0];
    ok = n0 > 0 && n0 % 3 == 0 && rowptr[r0 + 2] - rowptr[r0 + 1] == n0 && rowptr[r0 + 3] - rowptr[r0 + 2] == n0;
    for (int e = 0; ok && e < n0; ++e) {
      const int c = cols[rowptr[r0] + e];
      ok = c < n && c == cols[rowptr[r0 + 1] + e] && c == cols[rowptr[r0 + 2] + e] &&
           (e % 3 != 0 || (c % 3 == 0 && c + 2 < n)) && (e % 3 == 0 || c == cols[rowptr[r0] + e - 1] + 1);
    }
    if (r == r0) len[b] = ok ? n0 / 3 : 0;
  }
  rest_flag[r] = ok ? 0 : 1;
  rest_bytes[r] = ok ? 0.0 : 12.0 * (double)row_len(rowptr, r, n) + 4.0;
}

__global__ void k_b3_width(const int *len, int nbr, long long *w64) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= (nbr + 63) / 64) return;
  int w = 0;
  for (int b = 64 * c; b < min(nbr, 64 * c + 64); ++b) w = max(w, len[b]);
  w64[c] = (long long)w * 64;
}

__global__ void k_b3_fill(const int *rowptr, const int *cols, const double *vals, int nbr, const long long *off,
                          const int *len, int *bcol, double *bval) {
  const int b = blockIdx.x * 256 + threadIdx.x;
  if (b >= nbr) return;
  const int c = b >> 6, lane = b & 63;
  for (int s = 0; s < len[b]; ++s) {
    const long long slot = off[c] + 64LL * s;
    bcol[slot + lane] = cols[rowptr[3 * b] + 3 * s];
    for (int r = 0; r < 3; ++r)
      for (int e = 0; e < 3; ++e) bval[bsr3_val_index(slot, 3 * r + e, lane)] = vals[rowptr[3 * b + r] + 3 * s + e];
  }
}

// ------------------------------------------------------------------ templates (make_pair_templates)
// per pair: 1 = a row has more than kTplMaxRow entries or does not ascend (the host builder
// fails on any pair); ghost = reads a ghost column (left to the fallback kernel); cnt =
// entries of a templated pair
__global__ void k_tpl_check(const int *rowptr, const int *cols, int n, int P, unsigned char *bad,
                            unsigned char *ghost, long long *cnt) {
  const int p = blockIdx.x * 256 + threadIdx.x;
  if (p >= P) return;
  bool fail = false, gh = false;
  int total = 0;
  for (int h = 0; h < 2; ++h) {
    const int r = 2 * p + h;
    if (r >= n) continue;
    const int b = rowptr[r], e = rowptr[r + 1];
    if (e - b > kTplMaxRow) fail = true;
    for (int i = b; i < e; ++i) {
      if (cols[i] >= n) gh = true;
      if (i > b && cols[i] <= cols[i - 1]) fail = true;
    }
    total += e - b;
  }
  bad[p] = fail ? 1 : 0;
  ghost[p] = gh ? 1 : 0;
  cnt[p] = gh ? 0 : total;
}

// The merge of make_pair_templates for a non-ghost pair: visit(key, slot_byte_shift, entry)
// per entry in the host's order (keys ascending; within a key row 0's entries, then row 1's);
// key_done(key) after each key.
template <class V, class K>
__device__ void tpl_walk(const int *rowptr, const int *cols, int n, int p, V visit, K key_done) {
  int b[2], e[2];
  for (int h = 0; h < 2; ++h) {
    const int r = 2 * p + h;
    b[h] = r < n ? rowptr[r] : 0;
    e[h] = r < n ? rowptr[r + 1] : 0;
  }
  int i[2] = {b[0], b[1]};
  while (i[0] < e[0] || i[1] < e[1]) {
    const int k0 = i[0] < e[0] ? (cols[i[0]] >> 1) : INT_MAX;
    const int k1 = i[1] < e[1] ? (cols[i[1]] >> 1) : INT_MAX;
    const int key = k0 < k1 ? k0 : k1;
    for (int h = 0; h < 2; ++h)
      while (i[h] < e[h] && (cols[i[h]] >> 1) == key) {
        visit(key, 8 * (2 * h + (cols[i[h]] & 1)), i[h]);
        ++i[h];
      }
    key_done(key);
  }
}

__global__ void k_tpl_value_stream(const int *rowptr, const int *cols, const double *vals, int n, int P,
                                   const unsigned char *ghost, const long long *eoff, unsigned long long *bits,
                                   long long *visit_id) {
  const int p = blockIdx.x * 256 + threadIdx.x;
  if (p >= P || ghost[p]) return;
  long long at = eoff[p];
  tpl_walk(
      rowptr, cols, n, p,
      [&](int, int, int e) {
        unsigned long long b;
        memcpy(&b, &vals[e], sizeof(b));
        bits[at] = b;
        visit_id[at] = at;
        ++at;
      },
      [](int) {});
}

__global__ void k_run_heads_u64(const unsigned long long *sorted, long long m, unsigned char *head) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= m) return;
  head[i] = (i == 0 || sorted[i] != sorted[i - 1]) ? 1 : 0;
}

__device__ __forceinline__ int lookup_u64(const unsigned long long *keys, const int *slot, int nk,
                                          unsigned long long x) {
  int lo = 0, hi = nk - 1;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (keys[mid] < x)
      lo = mid + 1;
    else
      hi = mid;
  }
  return (nk > 0 && keys[lo] == x) ? slot[lo] : -1;
}

__device__ __forceinline__ unsigned long long mix64d(unsigned long long x) {
  x ^= x >> 33;
  x *= 0xFF51AFD7ED558CCDULL;
  x ^= x >> 33;
  x *= 0xC4CEB9FE1A85EC53ULL;
  x ^= x >> 33;
  return x;
}

// The shape of pair p: emit(u, offset, slots) per key; the key count (kTplMaxKeys + 1 when
// over the limit: the host builder fails).
template <class F>
__device__ int tpl_shape(const int *rowptr, const int *cols, const double *vals, int n, int p,
                         const unsigned long long *vkeys, const int *vslot, int nv, F emit) {
  unsigned slots = 0xFFFFFFFFu;
  int nk = 0;
  tpl_walk(
      rowptr, cols, n, p,
      [&](int, int sh, int e) {
        unsigned long long b;
        memcpy(&b, &vals[e], sizeof(b));
        const int vs = lookup_u64(vkeys, vslot, nv, b);
        slots = (slots & ~(0xFFu << sh)) | ((unsigned)vs << sh);
      },
      [&](int key) {
        if (nk < kTplMaxKeys) emit(nk, key - p, slots);
        ++nk;
        slots = 0xFFFFFFFFu;
      });
  return nk;
}

__global__ void k_tpl_hash(const int *rowptr, const int *cols, const double *vals, int n, int P,
                           const unsigned char *ghost, const unsigned long long *vkeys, const int *vslot, int nv,
                           unsigned long long hmask, unsigned long long *hash, int *nk_out, int *pid) {
  const int p = blockIdx.x * 256 + threadIdx.x;
  if (p >= P) return;
  pid[p] = p;
  if (ghost[p]) {
    hash[p] = ~0ULL;  // sorts last; not a template
    nk_out[p] = 0;
    return;
  }
  unsigned long long h = 0x9E3779B97F4A7C15ULL;
  const int nk = tpl_shape(rowptr, cols, vals, n, p, vkeys, vslot, nv, [&](int, int off, unsigned sl) {
    h = mix64d(h ^ (unsigned long long)(unsigned)off) + 0x632BE59BD9B4E019ULL;
    h = mix64d(h ^ (unsigned long long)sl);
  });
  h = mix64d(h ^ (unsigned long long)nk) & hmask;  // hmask: all ones (a test may truncate it)
  hash[p] = h == ~0ULL ? ~0ULL - 1 : h;
  nk_out[p] = nk;
}

// template id of each pair (kTplNone for ghost pairs) and a check that the pair's shape equals
// its template's representative pair's (a hash collision makes the build fall back)
__global__ void k_tpl_assign(const int *rowptr, const int *cols, const double *vals, int n, int P,
                             const unsigned char *ghost, const unsigned long long *vkeys, const int *vslot, int nv,
                             const unsigned long long *hash, const unsigned long long *tkeys, const int *tslot,
                             const int *trep, int ntpl, unsigned char *id, unsigned char *mismatch) {
  const int p = blockIdx.x * 256 + threadIdx.x;
  if (p >= P) return;
  mismatch[p] = 0;
  if (ghost[p]) {
    id[p] = kTplNone;
    return;
  }
  const int t = lookup_u64(tkeys, tslot, ntpl, hash[p]);
  if (t < 0) {
    mismatch[p] = 1;
    id[p] = kTplNone;
    return;
  }
  id[p] = (unsigned char)t;
  const int q = trep[t];
  if (q == p) return;
  int a_off[kTplMaxKeys];
  unsigned a_sl[kTplMaxKeys];
  const int na = tpl_shape(rowptr, cols, vals, n, p, vkeys, vslot, nv, [&](int u, int off, unsigned sl) {
    a_off[u] = off;
    a_sl[u] = sl;
  });
  bool same = true;
  const int nb = tpl_shape(rowptr, cols, vals, n, q, vkeys, vslot, nv, [&](int u, int off, unsigned sl) {
    if (u >= na || a_off[u] != off || a_sl[u] != sl) same = false;
  });
  if (!same || na != nb) mismatch[p] = 1;
}

__global__ void k_tpl_rec(const int *rowptr, const int *cols, const double *vals, int n, const int *trep, int ntpl,
                          int maxk, const unsigned long long *vkeys, const int *vslot, int nv, int *rec) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  if (t >= ntpl) return;
  const int nk = tpl_shape(rowptr, cols, vals, n, trep[t], vkeys, vslot, nv, [&](int u, int off, unsigned sl) {
    if (u < maxk) {
      rec[2 * ((size_t)t * maxk + u)] = off;
      rec[2 * ((size_t)t * maxk + u) + 1] = (int)sl;
    }
  });
  for (int u = nk; u < maxk; ++u) {  // padding key: reads the pair itself, adds nothing
    rec[2 * ((size_t)t * maxk + u)] = 0;
    rec[2 * ((size_t)t * maxk + u) + 1] = (int)0xFFFFFFFFu;
  }
}

__global__ void k_tpl_rest_flags(const int *rowptr, int n, const unsigned char *id, int P, bool by_pairs,
                                 unsigned char *flag, double *bytes) {
  const int u = blockIdx.x * 256 + threadIdx.x;
  if (by_pairs) {
    if (u >= P) return;
    const bool none = id[u] == kTplNone;
    flag[u] = none ? 1 : 0;
    double b = 0.0;
    if (none)
      for (int r = 2 * u; r < min(n, 2 * u + 2); ++r) b += 12.0 * (double)row_len(rowptr, r, n) + 4.0;
    bytes[u] = b;
  } else {
    if (u >= n) return;
    const bool none = id[u >> 1] == kTplNone;
    flag[u] = none ? 1 : 0;
    bytes[u] = none ? 12.0 * (double)row_len(rowptr, u, n) + 4.0 : 0.0;
  }
}

__global__ void k_unit_ghost(const int *rowptr, const int *cols, int n, int nunits, int unit, unsigned char *bnd,
                             unsigned char *inr) {
  const int u = blockIdx.x * 256 + threadIdx.x;
  if (u >= nunits) return;
  bool g = false;
  for (int r = u * unit; r < min(n, (u + 1) * unit) && !g; ++r)
    for (int e = rowptr[r]; e < rowptr[r + 1]; ++e)
      if (cols[e] >= n) {
        g = true;
        break;
      }
  bnd[u] = g ? 1 : 0;
  inr[u] = g ? 0 : 1;
}

// ------------------------------------------------------------------ transpose (GeneralMTM order)
__global__ void k_tr_rowid(const int *rowptr, int n, int *rowid, int *eid) {
  const int r = blockIdx.x * 256 + threadIdx.x;
  if (r >= n) return;
  for (int e = rowptr[r]; e < rowptr[r + 1]; ++e) {
    rowid[e] = r;
    eid[e] = e;
  }
}
__global__ void k_tr_count(const int *cols, long long nnz, unsigned long long *cnt) {
  const long long e = (long long)blockIdx.x * 256 + threadIdx.x;
  if (e < nnz) atomicAdd(&cnt[cols[e]], 1ULL);  // integer counts: order-independent
}
__global__ void k_tr_fill(const int *sorted_e, const int *rowid, const double *vals, long long nnz, int *tcols,
                          double *tvals) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= nnz) return;
  const int e = sorted_e[i];
  tcols[i] = rowid[e];
  tvals[i] = vals[e];
}
__global__ void k_tr_rowptr32(const long long *off, int n1, int *rp) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < n1) rp[i] = (int)off[i];
}

}  // namespace

void setup_mark(const char *what) {
  static const bool on = [] {
    const char *e = std::getenv("MIGMRES_SETUP_TRACE");
    return e && e[0] == '1';
  }();
  if (!on) return;
  static auto t0 = std::chrono::steady_clock::now();
  static auto last = t0;
  const auto now = std::chrono::steady_clock::now();
  std::fprintf(stderr, "[setup] %-28s +%8.1f ms (%8.1f ms)\n", what,
               std::chrono::duration<double, std::milli>(now - last).count(),
               std::chrono::duration<double, std::milli>(now - t0).count());
  last = now;
}

bool host_formats() {
  const char *e = std::getenv("MIGMRES_HOST_FORMATS");
  return e && e[0] == '1';
}

bool dev_pair_sell(hipStream_t s, const DevCsr &A, DevPairSell &out) {
  const int n = A.n_local, P = (n + 1) / 2;
  if (P <= 0) return false;
  Buf nk(sizeof(int) * P), rlen(sizeof(int) * P);
  setup_mark("formats: pair plan");
  k_pp_count<<<nblk(P), 256, 0, s>>>(A.rowptr, A.cols, n, P, nk.as<int>(), rlen.as<int>());
  MIG_HIP(hipGetLastError());
  if (dev_min<int>(s, nk.as<int>(), P, 0) < 0) return false;  // a pair the plan cannot take
  out.maxk = std::max(dev_max<int>(s, nk.as<int>(), P, 0), 1);
  out.rmax = std::max(dev_max<int>(s, rlen.as<int>(), P, 0), 1);
  const int nchunks = (P + 63) / 64;
  const size_t nv = (size_t)nchunks * 2 * out.rmax * 64, nkk = (size_t)nchunks * out.maxk * 64;
  MIG_HIP(hipMalloc(&out.v, sizeof(double) * nv));
  MIG_HIP(hipMalloc(&out.k, sizeof(int) * nkk));
  MIG_HIP(hipMalloc(&out.m, sizeof(unsigned short) * nkk));
  MIG_HIP(hipMemsetAsync(out.v, 0, sizeof(double) * nv, s));
  MIG_HIP(hipMemsetAsync(out.k, 0, sizeof(int) * nkk, s));
  MIG_HIP(hipMemsetAsync(out.m, 0xFF, sizeof(unsigned short) * nkk, s));
  k_pp_fill<<<nblk(P), 256, 0, s>>>(A.rowptr, A.cols, A.vals, n, P, out.rmax, out.maxk, out.v, out.k, out.m);
  MIG_HIP(hipGetLastError());
  return true;
}

void dev_sell64(hipStream_t s, const DevCsr &A, DevSell64 &out) {
  const int n = A.n_local, nchunks = (n + 63) / 64;
  Buf w(sizeof(long long) * (nchunks > 0 ? nchunks : 1));
  MIG_HIP(hipMalloc(&out.off, sizeof(long long) * (nchunks + 1)));
  MIG_HIP(hipMalloc(&out.len, sizeof(int) * (n > 0 ? n : 1)));
  if (nchunks > 0) k_chunk_width<<<nblk(nchunks), 256, 0, s>>>(A.rowptr, n, n, 1, w.as<long long>());
  dev_offsets(s, w.as<long long>(), out.off, nchunks);
  long long total = 0;
  MIG_HIP(hipMemcpyAsync(&total, out.off + nchunks, sizeof(long long), hipMemcpyDeviceToHost, s));
  MIG_HIP(hipStreamSynchronize(s));
  MIG_HIP(hipMalloc(&out.cols, sizeof(int) * (total + 1)));
  MIG_HIP(hipMalloc(&out.vals, sizeof(double) * (total + 1)));
  if (nchunks > 0)
    k_sell_fill<<<nblk((long long)nchunks * 64), 256, 0, s>>>(A.rowptr, A.cols, A.vals, n, out.off, out.len, out.cols,
                                                               out.vals);
  MIG_HIP(hipGetLastError());
}

bool dev_bsr3(hipStream_t s, const DevCsr &A, DevBsr3 &out) {
  const int n = A.n_local, nbr = n / 3;
  out = DevBsr3();
  out.nbr = nbr;
  if (n <= 0) return false;
  Buf len(sizeof(int) * (nbr > 0 ? nbr : 1)), flag((size_t)n), bytes(sizeof(double) * n);
  k_b3_qualify<<<nblk(n), 256, 0, s>>>(A.rowptr, A.cols, n, nbr, len.as<int>(), flag.as<unsigned char>(),
                                        bytes.as<double>());
  MIG_HIP(hipGetLastError());
  Buf rest(sizeof(int) * n);
  const int n_rest = dev_select_ids(s, flag.as<unsigned char>(), n, rest.as<int>());
  const long long qual_rows = (long long)n - n_rest;
  if (qual_rows == 0 || qual_rows * 8 < 7LL * n) return false;
  const int nchunks = (nbr + 63) / 64;
  Buf w(sizeof(long long) * (nchunks > 0 ? nchunks : 1));
  MIG_HIP(hipMalloc(&out.off, sizeof(long long) * (nchunks + 1)));
  if (nchunks > 0) k_b3_width<<<nblk(nchunks), 256, 0, s>>>(len.as<int>(), nbr, w.as<long long>());
  dev_offsets(s, w.as<long long>(), out.off, nchunks);
  MIG_HIP(hipMemcpyAsync(&out.nslots, out.off + nchunks, sizeof(long long), hipMemcpyDeviceToHost, s));
  MIG_HIP(hipStreamSynchronize(s));
  MIG_HIP(hipMalloc(&out.len, sizeof(int) * (nbr + 1)));
  MIG_HIP(hipMemcpyAsync(out.len, len.p, sizeof(int) * nbr, hipMemcpyDeviceToDevice, s));
  MIG_HIP(hipMalloc(&out.bcol, sizeof(int) * (out.nslots + 1)));
  MIG_HIP(hipMalloc(&out.vals, sizeof(double) * (9 * out.nslots + 1)));
  MIG_HIP(hipMemsetAsync(out.bcol, 0, sizeof(int) * (out.nslots + 1), s));
  MIG_HIP(hipMemsetAsync(out.vals, 0, sizeof(double) * (9 * out.nslots + 1), s));
  if (nbr > 0)
    k_b3_fill<<<nblk(nbr), 256, 0, s>>>(A.rowptr, A.cols, A.vals, nbr, out.off, out.len, out.bcol, out.vals);
  MIG_HIP(hipGetLastError());
  out.n_rest = n_rest;
  if (n_rest > 0) {
    MIG_HIP(hipMalloc(&out.rest, sizeof(int) * n_rest));
    MIG_HIP(hipMemcpyAsync(out.rest, rest.p, sizeof(int) * n_rest, hipMemcpyDeviceToDevice, s));
  }
  out.rest_bytes = dev_sum<double>(s, bytes.as<double>(), n);
  return true;
}

int dev_templates(hipStream_t s, const DevCsr &A, DevTemplates &out) {
  const int n = A.n_local, P = (n + 1) / 2;
  out = DevTemplates();
  out.npairs = P;
  if (P <= 0) return 0;
  // MIGMRES_TPL_HASH_BITS (tests only): keep that many low bits of the shape hash, so that
  // distinct shapes collide and the collision exit below is exercised
  unsigned long long hmask = ~0ULL;
  if (const char *hb = std::getenv("MIGMRES_TPL_HASH_BITS")) {
    const int b = std::atoi(hb);
    if (b > 0 && b < 64) hmask = (1ULL << b) - 1;
  }
  Buf bad((size_t)P), ghost((size_t)P), cnt(sizeof(long long) * P), eoff(sizeof(long long) * (P + 1));
  setup_mark("formats: templates");
  k_tpl_check<<<nblk(P), 256, 0, s>>>(A.rowptr, A.cols, n, P, bad.as<unsigned char>(), ghost.as<unsigned char>(),
                                       cnt.as<long long>());
  MIG_HIP(hipGetLastError());
  if (dev_max<unsigned char>(s, bad.as<unsigned char>(), P, 0)) return 0;
  dev_offsets(s, cnt.as<long long>(), eoff.as<long long>(), P);
  long long m = 0;
  MIG_HIP(hipMemcpyAsync(&m, eoff.as<long long>() + P, sizeof(long long), hipMemcpyDeviceToHost, s));
  MIG_HIP(hipStreamSynchronize(s));
  if (m == 0) return 0;  // no pair without a ghost column
  MIG_CHECK(m < (1LL << 31), "template plan: too many entries");
  // value dictionary: the distinct bit patterns in order of first appearance over the host
  // builder's visiting order (a stable sort by value keeps each value's visits in order)
  const int mi = (int)m;
  std::vector<unsigned long long> vkeys_h;
  std::vector<int> vslot_h;
  {
    Buf bits(sizeof(unsigned long long) * m), vid(sizeof(long long) * m), sbits(sizeof(unsigned long long) * m),
        svid(sizeof(long long) * m), head((size_t)m);
    k_tpl_value_stream<<<nblk(P), 256, 0, s>>>(A.rowptr, A.cols, A.vals, n, P, ghost.as<unsigned char>(),
                                                eoff.as<long long>(), bits.as<unsigned long long>(), vid.as<long long>());
    dev_sort_pairs(s, bits.as<unsigned long long>(), sbits.as<unsigned long long>(), vid.as<long long>(),
                   svid.as<long long>(), mi);
    k_run_heads_u64<<<nblk(m), 256, 0, s>>>(sbits.as<unsigned long long>(), m, head.as<unsigned char>());
    Buf ubits(sizeof(unsigned long long) * m), uvid(sizeof(long long) * m);
    const int nd = dev_select(s, sbits.as<unsigned long long>(), head.as<unsigned char>(), mi,
                              ubits.as<unsigned long long>());
    dev_select(s, svid.as<long long>(), head.as<unsigned char>(), mi, uvid.as<long long>());
    if (nd > 255) return 0;
    vkeys_h.resize((size_t)nd);
    std::vector<long long> first((size_t)nd);
    MIG_HIP(hipMemcpyAsync(vkeys_h.data(), ubits.p, sizeof(unsigned long long) * nd, hipMemcpyDeviceToHost, s));
    MIG_HIP(hipMemcpyAsync(first.data(), uvid.p, sizeof(long long) * nd, hipMemcpyDeviceToHost, s));
    MIG_HIP(hipStreamSynchronize(s));
    std::vector<int> order((size_t)nd);
    for (int i = 0; i < nd; ++i) order[(size_t)i] = i;
    std::sort(order.begin(), order.end(), [&](int a, int b) { return first[(size_t)a] < first[(size_t)b]; });
    vslot_h.assign((size_t)nd, 0);
    out.vals.resize((size_t)nd);
    for (int sl = 0; sl < nd; ++sl) {
      vslot_h[(size_t)order[(size_t)sl]] = sl;
      std::memcpy(&out.vals[(size_t)sl], &vkeys_h[(size_t)order[(size_t)sl]], sizeof(double));
    }
  }
  const int nv = (int)vkeys_h.size();
  Buf vkeys(sizeof(unsigned long long) * (nv + 1)), vslot(sizeof(int) * (nv + 1));
  MIG_HIP(hipMemcpyAsync(vkeys.p, vkeys_h.data(), sizeof(unsigned long long) * nv, hipMemcpyHostToDevice, s));
  MIG_HIP(hipMemcpyAsync(vslot.p, vslot_h.data(), sizeof(int) * nv, hipMemcpyHostToDevice, s));
  // shapes -> hashes; template ids in order of first appearance (stable sort by hash)
  Buf hash(sizeof(unsigned long long) * P), nk(sizeof(int) * P), pid(sizeof(int) * P),
      shash(sizeof(unsigned long long) * P), spid(sizeof(int) * P), head((size_t)P);
  k_tpl_hash<<<nblk(P), 256, 0, s>>>(A.rowptr, A.cols, A.vals, n, P, ghost.as<unsigned char>(),
                                      vkeys.as<unsigned long long>(), vslot.as<int>(), nv, hmask,
                                      hash.as<unsigned long long>(), nk.as<int>(), pid.as<int>());
  MIG_HIP(hipGetLastError());
  const int maxnk = dev_max<int>(s, nk.as<int>(), P, 0);
  if (maxnk > kTplMaxKeys) return 0;
  dev_sort_pairs(s, hash.as<unsigned long long>(), shash.as<unsigned long long>(), pid.as<int>(), spid.as<int>(), P);
  k_run_heads_u64<<<nblk(P), 256, 0, s>>>(shash.as<unsigned long long>(), P, head.as<unsigned char>());
  Buf uh(sizeof(unsigned long long) * P), up(sizeof(int) * P);
  int nh = dev_select(s, shash.as<unsigned long long>(), head.as<unsigned char>(), P, uh.as<unsigned long long>());
  dev_select(s, spid.as<int>(), head.as<unsigned char>(), P, up.as<int>());
  std::vector<unsigned long long> th((size_t)nh);
  std::vector<int> tp((size_t)nh);
  MIG_HIP(hipMemcpyAsync(th.data(), uh.p, sizeof(unsigned long long) * nh, hipMemcpyDeviceToHost, s));
  MIG_HIP(hipMemcpyAsync(tp.data(), up.p, sizeof(int) * nh, hipMemcpyDeviceToHost, s));
  MIG_HIP(hipStreamSynchronize(s));
  if (nh > 0 && th.back() == ~0ULL) {  // the ghost pairs' run
    th.pop_back();
    tp.pop_back();
    --nh;
  }
  if (nh == 0) return 0;
  if (nh > kTplMaxTemplates) return 0;
  std::vector<int> order((size_t)nh), tslot((size_t)nh), trep((size_t)nh);
  for (int i = 0; i < nh; ++i) order[(size_t)i] = i;
  std::sort(order.begin(), order.end(), [&](int a, int b) { return tp[(size_t)a] < tp[(size_t)b]; });
  for (int t = 0; t < nh; ++t) {
    tslot[(size_t)order[(size_t)t]] = t;
    trep[(size_t)t] = tp[(size_t)order[(size_t)t]];
  }
  Buf tkeys(sizeof(unsigned long long) * nh), tsl(sizeof(int) * nh), trp(sizeof(int) * nh), mism((size_t)P);
  MIG_HIP(hipMemcpyAsync(tkeys.p, th.data(), sizeof(unsigned long long) * nh, hipMemcpyHostToDevice, s));
  MIG_HIP(hipMemcpyAsync(tsl.p, tslot.data(), sizeof(int) * nh, hipMemcpyHostToDevice, s));
  MIG_HIP(hipMemcpyAsync(trp.p, trep.data(), sizeof(int) * nh, hipMemcpyHostToDevice, s));
  MIG_HIP(hipMalloc(&out.id, (size_t)P));
  k_tpl_assign<<<nblk(P), 256, 0, s>>>(A.rowptr, A.cols, A.vals, n, P, ghost.as<unsigned char>(),
                                        vkeys.as<unsigned long long>(), vslot.as<int>(), nv,
                                        hash.as<unsigned long long>(), tkeys.as<unsigned long long>(), tsl.as<int>(),
                                        trp.as<int>(), nh, out.id, mism.as<unsigned char>());
  MIG_HIP(hipGetLastError());
  if (dev_max<unsigned char>(s, mism.as<unsigned char>(), P, 0) != 0) {
    // two shapes share a hash: no device plan; the caller builds this one on the host
    MIG_HIP(hipStreamSynchronize(s));
    MIG_HIP(hipFree(out.id));
    out.id = nullptr;
    return -1;
  }
  out.ntpl = nh;
  out.maxk = std::max(maxnk, 1);
  {
    Buf scratch(sizeof(int) * P);  // templated = every pair without a ghost column (empty ones too)
    out.n_templated = P - (long long)dev_select_ids(s, ghost.as<unsigned char>(), P, scratch.as<int>());
  }
  Buf rec(sizeof(int) * 2 * (size_t)nh * out.maxk);
  k_tpl_rec<<<nblk(nh), 256, 0, s>>>(A.rowptr, A.cols, A.vals, n, trp.as<int>(), nh, out.maxk,
                                      vkeys.as<unsigned long long>(), vslot.as<int>(), nv, rec.as<int>());
  out.rec.resize(2 * (size_t)nh * out.maxk);
  MIG_HIP(hipMemcpyAsync(out.rec.data(), rec.p, sizeof(int) * out.rec.size(), hipMemcpyDeviceToHost, s));
  MIG_HIP(hipStreamSynchronize(s));
  return 1;
}

int dev_template_rest(hipStream_t s, const DevCsr &A, const unsigned char *id, int npairs, bool by_pairs, int **out,
                      double *rest_bytes) {
  const int n = A.n_local, nu = by_pairs ? npairs : n;
  *out = nullptr;
  *rest_bytes = 0.0;
  if (nu <= 0) return 0;
  Buf flag((size_t)nu), bytes(sizeof(double) * nu), ids(sizeof(int) * nu);
  k_tpl_rest_flags<<<nblk(nu), 256, 0, s>>>(A.rowptr, n, id, npairs, by_pairs, flag.as<unsigned char>(),
                                             bytes.as<double>());
  MIG_HIP(hipGetLastError());
  const int cnt = dev_select_ids(s, flag.as<unsigned char>(), nu, ids.as<int>());
  *rest_bytes = dev_sum<double>(s, bytes.as<double>(), nu);
  if (cnt > 0) {
    MIG_HIP(hipMalloc(out, sizeof(int) * cnt));
    MIG_HIP(hipMemcpyAsync(*out, ids.p, sizeof(int) * cnt, hipMemcpyDeviceToDevice, s));
  }
  return cnt;
}

void dev_halo_units(hipStream_t s, const DevCsr &A, bool by_pairs, int **interior, int *n_interior, int **boundary,
                    int *n_boundary) {
  const int n = A.n_local, unit = by_pairs ? 2 : 1, nunits = (n + unit - 1) / unit;
  Buf bnd((size_t)(nunits > 0 ? nunits : 1)), inr((size_t)(nunits > 0 ? nunits : 1));
  MIG_HIP(hipMalloc(interior, sizeof(int) * (nunits + 1)));
  MIG_HIP(hipMalloc(boundary, sizeof(int) * (nunits + 1)));
  *n_interior = *n_boundary = 0;
  if (nunits <= 0) return;
  k_unit_ghost<<<nblk(nunits), 256, 0, s>>>(A.rowptr, A.cols, n, nunits, unit, bnd.as<unsigned char>(),
                                             inr.as<unsigned char>());
  MIG_HIP(hipGetLastError());
  *n_interior = dev_select_ids(s, inr.as<unsigned char>(), nunits, *interior);
  *n_boundary = dev_select_ids(s, bnd.as<unsigned char>(), nunits, *boundary);
}

void dev_transpose(hipStream_t s, const DevCsr &A, int n_out, DevTrans &out) {
  const int n = A.n_local;
  const long long nnz = A.nnz;
  out = DevTrans();
  MIG_HIP(hipMalloc(&out.rowptr, sizeof(int) * ((size_t)n_out + 1)));
  MIG_HIP(hipMalloc(&out.cols, sizeof(int) * (size_t)(nnz > 0 ? nnz : 1)));
  MIG_HIP(hipMalloc(&out.vals, sizeof(double) * (size_t)(nnz > 0 ? nnz : 1)));
  Buf cnt(sizeof(long long) * ((size_t)n_out + 1)), off(sizeof(long long) * ((size_t)n_out + 2));
  MIG_HIP(hipMemsetAsync(cnt.p, 0, sizeof(long long) * ((size_t)n_out + 1), s));
  if (nnz > 0) {
    Buf rowid(sizeof(int) * nnz), eid(sizeof(int) * nnz), skey(sizeof(int) * nnz), se(sizeof(int) * nnz);
    k_tr_rowid<<<nblk(n), 256, 0, s>>>(A.rowptr, n, rowid.as<int>(), eid.as<int>());
    k_tr_count<<<nblk(nnz), 256, 0, s>>>(A.cols, nnz, cnt.as<unsigned long long>());
    MIG_HIP(hipGetLastError());
    // stable by column: entries of one column keep their (row-major, hence ascending-row) order
    dev_sort_pairs(s, A.cols, skey.as<int>(), eid.as<int>(), se.as<int>(), (int)nnz);
    k_tr_fill<<<nblk(nnz), 256, 0, s>>>(se.as<int>(), rowid.as<int>(), A.vals, nnz, out.cols, out.vals);
    MIG_HIP(hipGetLastError());
    MIG_HIP(hipStreamSynchronize(s));
  }
  dev_offsets(s, cnt.as<long long>(), off.as<long long>(), n_out);
  k_tr_rowptr32<<<nblk(n_out + 1), 256, 0, s>>>(off.as<long long>(), n_out + 1, out.rowptr);
  MIG_HIP(hipGetLastError());
  MIG_HIP(hipStreamSynchronize(s));
}

}  // namespace migmres
