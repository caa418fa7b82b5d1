// Context, multivectors, distributed CRS operator and the C ABI for them.
#include "runtime.h"
#include "formats.h"

#include <chrono>
#include <algorithm>
#include <mutex>
#include <map>
#include <deque>
#include <condition_variable>
#include <cstdlib>
#include <cmath>
#include <cstring>
#include <cstdio>
#include <string>
#include <thread>

using namespace migmres;

// ------------------------------------------------------------------------------------
// error plumbing for the C ABI
// ------------------------------------------------------------------------------------
static thread_local std::string g_last_error;
void migmres::set_last_error(const std::string &m) { g_last_error = m; }

namespace {
#define MIG_NCCL(call)                                                                      \
  do {                                                                                      \
    ncclResult_t r_ = (call);                                                               \
    if (r_ != ncclSuccess) throw Error(MIGMRES_ERCCL, std::string(#call) + ": " + ncclGetErrorString(r_)); \
  } while (0)

long long round_up(long long a, long long b) { return (a + b - 1) / b * b; }
}  // namespace

extern "C" int migmres_abi_version(void) { return MIGMRES_ABI_VERSION; }
extern "C" const char *migmres_last_error(void) { return g_last_error.c_str(); }

// ------------------------------------------------------------------------------------
// context
// ------------------------------------------------------------------------------------
static double *grow(double *&p, size_t &cap, size_t n) {
  if (n <= cap) return p;
  if (p) MIG_HIP(hipFree(p));
  size_t c = n < 4096 ? 4096 : n;
  MIG_HIP(hipMalloc(&p, c * sizeof(double)));
  cap = c;
  return p;
}
double *migmres_ctx::partial(size_t n) { return grow(d_partial, partial_cap, n); }
double *migmres_ctx::red(size_t n) { return grow(d_red, red_cap, n); }
double *migmres_ctx::coef(size_t n) { return grow(d_coef, coef_cap, n); }
double *migmres_ctx::pinned(size_t n) {
  if (n > pinned_cap) {
    if (h_pinned) MIG_HIP(hipHostFree(h_pinned));
    size_t c = n < 65536 ? 65536 : n;
    MIG_HIP(hipHostMalloc(&h_pinned, c * sizeof(double), hipHostMallocDefault));
    pinned_cap = c;
  }
  return h_pinned;
}
// ------------------------------------------------------------------------------------
// in-process loopback communicator (tests only)
// ------------------------------------------------------------------------------------
namespace migmres {
struct LoopGroup {
  int n = 0;
  std::mutex mu;
  std::condition_variable cv;
  long long ar_gen = 0;
  int ar_arrived = 0;
  std::vector<std::vector<double>> ar_in;
  std::vector<double> ar_out;
  std::map<std::pair<int, int>, std::deque<std::vector<char>>> box;  // (src, dst) -> messages
};
}  // namespace migmres

static std::mutex g_loop_mu;
static std::map<unsigned long long, std::weak_ptr<LoopGroup>> g_loop_groups;

static bool is_loop_uid(const unsigned char *uid) { return uid && std::memcmp(uid, "MIGLOOP1", 8) == 0; }

static std::shared_ptr<LoopGroup> loop_join(const unsigned char *uid, int nranks) {
  unsigned long long key = 0;
  std::memcpy(&key, uid + 8, sizeof(key));
  std::lock_guard<std::mutex> lk(g_loop_mu);
  auto &w = g_loop_groups[key];
  auto g = w.lock();
  if (!g) {
    g = std::make_shared<LoopGroup>();
    g->n = nranks;
    g->ar_in.resize((size_t)nranks);
    w = g;
  }
  MIG_CHECK(g->n == nranks, "loopback group joined with a different rank count");
  return g;
}

// Blocking sum / max all-reduce across the group's ranks (rank order, deterministic).
static void loop_allreduce(migmres_ctx *c, double *d, size_t n, bool max) {
  LoopGroup &g = *c->loop;
  std::vector<double> v(n);
  MIG_HIP(hipStreamSynchronize(c->stream));
  MIG_HIP(hipMemcpy(v.data(), d, sizeof(double) * n, hipMemcpyDeviceToHost));
  std::vector<double> out;
  {
    std::unique_lock<std::mutex> lk(g.mu);
    const long long gen = g.ar_gen;
    g.ar_in[(size_t)c->rank] = std::move(v);
    if (++g.ar_arrived == g.n) {
      std::vector<double> r = g.ar_in[0];
      for (int q = 1; q < g.n; ++q) {
        MIG_CHECK(g.ar_in[(size_t)q].size() == n,
                  "loopback all-reduce size mismatch: rank " + std::to_string(q) + " sent " +
                      std::to_string(g.ar_in[(size_t)q].size()) + ", rank " + std::to_string(c->rank) + " " +
                      std::to_string(n));
        for (size_t i = 0; i < n; ++i)
          r[i] = max ? std::max(r[i], g.ar_in[(size_t)q][i]) : r[i] + g.ar_in[(size_t)q][i];
      }
      g.ar_out = std::move(r);
      g.ar_arrived = 0;
      ++g.ar_gen;
      g.cv.notify_all();
    } else {
      g.cv.wait(lk, [&] { return g.ar_gen != gen; });
    }
    out = g.ar_out;
  }
  MIG_HIP(hipMemcpy(d, out.data(), sizeof(double) * n, hipMemcpyHostToDevice));
}

void migmres_ctx::p2p_begin(hipStream_t s) {
  p2p_stream = s ? s : stream;
  p2p_sends.clear();
  p2p_recvs.clear();
  if (!loop) MIG_NCCL(ncclGroupStart());
}
void migmres_ctx::p2p_send(const void *buf, size_t bytes, int peer) {
  if (loop)
    p2p_sends.push_back({const_cast<void *>(buf), bytes, peer});
  else
    MIG_NCCL(ncclSend(buf, bytes, ncclChar, peer, comm, p2p_stream));
}
void migmres_ctx::p2p_recv(void *buf, size_t bytes, int peer) {
  if (loop)
    p2p_recvs.push_back({buf, bytes, peer});
  else
    MIG_NCCL(ncclRecv(buf, bytes, ncclChar, peer, comm, p2p_stream));
}
void migmres_ctx::p2p_end() {
  if (!loop) {
    MIG_NCCL(ncclGroupEnd());
    return;
  }
  LoopGroup &g = *loop;
  MIG_HIP(hipStreamSynchronize(p2p_stream));
  for (auto &m : p2p_sends) {
    std::vector<char> v(m.bytes);
    if (m.bytes) MIG_HIP(hipMemcpy(v.data(), m.buf, m.bytes, hipMemcpyDeviceToHost));
    std::lock_guard<std::mutex> lk(g.mu);
    g.box[{rank, m.peer}].push_back(std::move(v));
    g.cv.notify_all();
  }
  for (auto &m : p2p_recvs) {
    std::vector<char> v;
    {
      std::unique_lock<std::mutex> lk(g.mu);
      auto &q = g.box[{m.peer, rank}];
      g.cv.wait(lk, [&] { return !q.empty(); });
      v = std::move(q.front());
      q.pop_front();
    }
    MIG_CHECK(v.size() == m.bytes, "loopback message size mismatch");
    if (m.bytes) MIG_HIP(hipMemcpy(m.buf, v.data(), m.bytes, hipMemcpyHostToDevice));
  }
  p2p_sends.clear();
  p2p_recvs.clear();
}

void migmres_ctx::allreduce(double *d, size_t n, bool max) {
  if (!dist || n == 0) return;
  auto t0 = std::chrono::steady_clock::now();
  if (loop) {
    loop_allreduce(this, d, n, max);
  } else {
    {
      ProfScope ps(this, K_ALLREDUCE, 8.0 * n);
      MIG_NCCL(ncclAllReduce(d, d, n, ncclDouble, max ? ncclMax : ncclSum, comm, stream));
    }
    MIG_HIP(hipStreamSynchronize(stream));
  }
  comm_seconds += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}

const char *kKernelClassNames[K_NUM_CLASSES] = {"spmm", "gemm_tn", "reduce", "gemm_nn", "coldot",
                                                "axpby", "scale", "fill", "copy", "random", "pack",
                                                "findbasis", "gemm_nn_dot", "nn_tn", "halo",
                                                "allreduce"};

hipEvent_t migmres_ctx::get_event() {
  if (!event_pool.empty()) {
    hipEvent_t e = event_pool.back();
    event_pool.pop_back();
    return e;
  }
  hipEvent_t e;
  MIG_HIP(hipEventCreate(&e));
  return e;
}

void migmres_ctx::prof_collect() {
  if (pending.empty()) return;
  MIG_HIP(hipStreamSynchronize(stream));
  for (auto &p : pending) {
    float ms = 0.f;
    MIG_HIP(hipEventSynchronize(p.b));
    MIG_HIP(hipEventElapsedTime(&ms, p.a, p.b));
    prof_ms[p.cls] += ms;
    prof_bytes[p.cls] += p.bytes;
    prof_count[p.cls] += 1;
    event_pool.push_back(p.a);
    event_pool.push_back(p.b);
  }
  pending.clear();
}

ProfScope::ProfScope(migmres_ctx *ctx, int k, double by, hipStream_t stream)
    : c(ctx), cls(k), bytes(by), s(stream ? stream : ctx->stream) {
  if (!c->prof_on) return;
  a = c->get_event();
  b = c->get_event();
  MIG_HIP(hipEventRecord(a, s));
}

ProfScope::~ProfScope() {
  if (!c->prof_on || !a) return;
  hipEventRecord(b, s);
  c->pending.push_back({cls, bytes, a, b});
  if (c->pending.size() > 2048) {
    try {
      c->prof_collect();
    } catch (...) {
    }
  }
}

extern "C" int migmres_ctx_profile(migmres_ctx *c, int on) {
  return guard([&] {
    c->prof_collect();
    c->prof_on = on != 0;
    for (int i = 0; i < K_NUM_CLASSES; ++i) c->prof_ms[i] = c->prof_bytes[i] = 0.0, c->prof_count[i] = 0;
  });
}

extern "C" int migmres_ctx_profile_read(migmres_ctx *c, double *ms, double *bytes, long long *launches,
                                        int n) {
  return guard([&] {
    c->prof_collect();
    for (int i = 0; i < n && i < K_NUM_CLASSES; ++i) {
      ms[i] = c->prof_ms[i];
      bytes[i] = c->prof_bytes[i];
      launches[i] = c->prof_count[i];
    }
  });
}

extern "C" const char *migmres_kernel_class_name(int i) {
  return (i >= 0 && i < K_NUM_CLASSES) ? kKernelClassNames[i] : "";
}

void *migmres_ctx::dev_alloc(size_t bytes, size_t *rounded) {
  const size_t gran = bytes >= (64u << 20) ? (2u << 20) : 4096;
  const size_t r = (bytes + gran - 1) / gran * gran;
  for (size_t i = 0; i < pool.size(); ++i)
    if (pool[i].first == r) {
      void *p = pool[i].second;
      pool.erase(pool.begin() + (long)i);
      pool_bytes -= r;
      *rounded = r;
      return p;
    }
  void *p = nullptr;
  hipError_t e = hipMalloc(&p, r);
  if (e != hipSuccess) {  // release cached blocks and retry once
    (void)hipGetLastError();
    pool_trim();
    e = hipMalloc(&p, r);
  }
  if (e != hipSuccess) throw Error(MIGMRES_ENOMEM, std::string("hipMalloc: ") + hipGetErrorString(e));
  *rounded = r;
  return p;
}

void migmres_ctx::dev_free(void *p, size_t rounded) {
  if (!p) return;
  pool.emplace_back(rounded, p);
  pool_bytes += rounded;
}

void migmres_ctx::pool_trim() {
  (void)hipStreamSynchronize(stream);
  for (auto &b : pool) (void)hipFree(b.second);
  pool.clear();
  pool_bytes = 0;
}

void migmres_ctx::allreduce_async(double *d, size_t n) {
  if (!dist || n == 0) return;
  if (loop) {
    loop_allreduce(this, d, n, false);
    return;
  }
  ProfScope ps(this, K_ALLREDUCE, 8.0 * n);
  MIG_NCCL(ncclAllReduce(d, d, n, ncclDouble, ncclSum, comm, stream));
}

extern "C" int migmres_comm_unique_id(unsigned char out[128]) {
  return guard([&] {
    ncclUniqueId id;
    MIG_NCCL(ncclGetUniqueId(&id));
    static_assert(sizeof(id) == 128, "RCCL unique id size");
    std::memcpy(out, &id, 128);
  });
}

extern "C" int migmres_rccl_version(int *version) {
  return guard([&] {
    MIG_CHECK(version, "null version pointer");
    MIG_NCCL(ncclGetVersion(version));
  });
}

// ncclCommInitRank blocks until every rank has joined; a rank that died before joining
// leaves the others there forever.  The watchdog turns that into a process exit (status
// 75) after MIGMRES_RCCL_INIT_TIMEOUT seconds so the launcher can stop the job.
static void comm_init_guarded(ncclComm_t *comm, int nranks, const ncclUniqueId &id, int rank) {
  const char *e = std::getenv("MIGMRES_RCCL_INIT_TIMEOUT");
  const double limit = e ? std::atof(e) : 600.0;
  if (limit <= 0) {
    MIG_NCCL(ncclCommInitRank(comm, nranks, id, rank));
    return;
  }
  std::mutex mu;
  std::condition_variable cv;
  bool done = false;
  std::thread dog([&] {
    std::unique_lock<std::mutex> lk(mu);
    if (!cv.wait_for(lk, std::chrono::duration<double>(limit), [&] { return done; })) {
      std::fprintf(stderr,
                   "migmres: rank %d of %d: ncclCommInitRank did not complete within %.0f s "
                   "(a peer rank failed or never joined); exiting\n",
                   rank, nranks, limit);
      std::fflush(stderr);
      std::_Exit(75);
    }
  });
  ncclResult_t r = ncclCommInitRank(comm, nranks, id, rank);
  {
    std::lock_guard<std::mutex> lk(mu);
    done = true;
  }
  cv.notify_all();
  dog.join();
  if (r != ncclSuccess) throw Error(MIGMRES_ERCCL, std::string("ncclCommInitRank: ") + ncclGetErrorString(r));
}

extern "C" int migmres_ctx_create(int device, int rank, int nranks, const unsigned char *uid,
                                  migmres_ctx **out) {
  return guard([&] {
    MIG_CHECK(out && nranks >= 1 && rank >= 0 && rank < nranks, "bad context arguments");
    auto *c = new migmres_ctx();
    c->device = device;
    c->rank = rank;
    c->nranks = nranks;
    try {
      MIG_HIP(hipSetDevice(device));
      MIG_HIP(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
      const char *fr = std::getenv("MIGMRES_FORCE_RCCL");
      const bool force = nranks == 1 && fr && fr[0] == '1';
      if (nranks > 1 || force) {
        MIG_CHECK(uid != nullptr || force, "unique id required for nranks > 1");
        if (uid && is_loop_uid(uid)) {
          c->loop = loop_join(uid, nranks);
        } else {
          ncclUniqueId id;
          if (force && !uid)
            MIG_NCCL(ncclGetUniqueId(&id));
          else
            std::memcpy(&id, uid, 128);
          comm_init_guarded(&c->comm, nranks, id, rank);
        }
        c->dist = true;
        MIG_HIP(hipStreamCreateWithFlags(&c->halo_stream, hipStreamNonBlocking));
        MIG_HIP(hipEventCreateWithFlags(&c->ev_main, hipEventDisableTiming));
        MIG_HIP(hipEventCreateWithFlags(&c->ev_halo, hipEventDisableTiming));
      }
    } catch (...) {
      delete c;
      throw;
    }
    *out = c;
  });
}

extern "C" int migmres_ctx_destroy(migmres_ctx *c) {
  return guard([&] {
    if (!c) return;
    hipStreamSynchronize(c->stream);
    c->pool_trim();
    for (auto e : c->event_pool) (void)hipEventDestroy(e);
    if (c->comm) ncclCommDestroy(c->comm);
    if (c->d_partial) hipFree(c->d_partial);
    if (c->d_red) hipFree(c->d_red);
    if (c->d_coef) hipFree(c->d_coef);
    if (c->h_pinned) hipHostFree(c->h_pinned);
    if (c->halo_stream) {
      hipStreamSynchronize(c->halo_stream);
      hipStreamDestroy(c->halo_stream);
    }
    if (c->ev_main) hipEventDestroy(c->ev_main);
    if (c->ev_halo) hipEventDestroy(c->ev_halo);
    if (c->stream) hipStreamDestroy(c->stream);
    delete c;
  });
}

extern "C" int migmres_ctx_sync(migmres_ctx *c) {
  return guard([&] { MIG_HIP(hipStreamSynchronize(c->stream)); });
}

extern "C" int migmres_ctx_rank(const migmres_ctx *c, int *rank, int *nranks) {
  return guard([&] {
    *rank = c->rank;
    *nranks = c->nranks;
  });
}

extern "C" int migmres_ctx_sum_all(migmres_ctx *c, const double *in, double *out, int n) {
  return guard([&] {
    if (n <= 0) return;
    double *d = c->red((size_t)n);
    MIG_HIP(hipMemcpyAsync(d, in, sizeof(double) * n, hipMemcpyHostToDevice, c->stream));
    c->allreduce(d, (size_t)n);
    MIG_HIP(hipMemcpyAsync(out, d, sizeof(double) * n, hipMemcpyDeviceToHost, c->stream));
    MIG_HIP(hipStreamSynchronize(c->stream));
  });
}

// ------------------------------------------------------------------------------------
// multivectors
// ------------------------------------------------------------------------------------
migmres_mv::~migmres_mv() {
  if (d_cols) hipFree(d_cols);
  if (owner && base) ctx->dev_free(base, alloc_bytes);
}

namespace migmres {

migmres_mv *mv_create(migmres_ctx *ctx, long long n_global, int n_local, int ncols) {
  MIG_CHECK(ctx && n_local >= 0 && ncols >= 0, "bad multivector shape");
  auto *m = new migmres_mv();
  m->ctx = ctx;
  m->n_global = n_global;
  m->n_local = n_local;
  m->ncols = ncols;
  // rows padded to a multiple of 64 (whole 64-row chunks, kept zero) plus 576 more rows so
  // that columns are not a power-of-two distance apart: with ld = 2^24 every column's row r
  // fell on the same HBM channel, and k_gemm_tn ran at 5.4 instead of 5.8-7.5 TB/s
  // (tools/mb_lib.cpp, 256^3).  576 rows (4.5 KB) from a same-box sweep of 64 .. 8256 rows at
  // 2^21 .. 2^24 rows (the per-rank sizes of the 8/4/2/1-GPU 256^3 runs, profiles/r4d_pad*.txt):
  // 717 -> 761, 395 -> 402, 197 -> 199, 99.4 -> 99.3 it/s against the earlier 64.
  static const long long ld_pad = [] {
    const char *e = std::getenv("MIGMRES_LD_PAD");  // rows; tuning only
    return e ? std::atoll(e) : 576LL;
  }();
  m->ld = round_up(n_local > 0 ? n_local : 1, 64) + ld_pad;
  m->owner = true;
  const size_t bytes = (size_t)m->ld * (size_t)(ncols > 0 ? ncols : 1) * sizeof(double) + 256;
  try {
    m->base = (double *)ctx->dev_alloc(bytes, &m->alloc_bytes);
  } catch (...) {
    m->owner = false;
    delete m;
    throw;
  }
  // Invariant used by the streaming kernels: padding rows [n_local, ld) stay zero (no
  // kernel writes past n_local), so full 64-row chunks can be read unguarded.
  hipError_t e = hipMemsetAsync(m->base, 0, bytes, ctx->stream);
  if (e != hipSuccess) {
    delete m;
    throw Error(MIGMRES_EHIP, std::string("hipMemset multivector: ") + hipGetErrorString(e));
  }
  return m;
}

migmres_mv *mv_view(migmres_mv *p, const int *idx, int n) {
  MIG_CHECK(p && n >= 0, "bad view");
  bool contiguous = true;
  for (int i = 0; i < n; ++i) {
    MIG_CHECK(idx[i] >= 0 && idx[i] < p->ncols, "view index out of range");
    if (i > 0 && idx[i] != idx[i - 1] + 1) contiguous = false;
  }
  auto *m = new migmres_mv();
  m->ctx = p->ctx;
  m->n_global = p->n_global;
  m->n_local = p->n_local;
  m->ncols = n;
  m->ld = p->ld;
  m->owner = false;
  if (contiguous && p->contiguous()) {
    m->base = p->base + (n > 0 ? (long long)idx[0] * p->ld : 0);
    return m;
  }
  m->base = p->base;
  m->cols.resize((size_t)n);
  for (int i = 0; i < n; ++i) m->cols[(size_t)i] = p->contiguous() ? idx[i] : p->cols[(size_t)idx[i]];
  if (n > 0) {
    MIG_HIP(hipMalloc(&m->d_cols, sizeof(int) * n));
    MIG_HIP(hipMemcpy(m->d_cols, m->cols.data(), sizeof(int) * n, hipMemcpyHostToDevice));
  }
  return m;
}

migmres_mv *mv_view_range(migmres_mv *p, int first, int n) {
  std::vector<int> idx((size_t)n);
  for (int i = 0; i < n; ++i) idx[(size_t)i] = first + i;
  return mv_view(p, idx.data(), n);
}

static void same_rows(const migmres_mv &a, const migmres_mv &b) {
  MIG_CHECK(a.n_local == b.n_local && a.n_global == b.n_global, "multivector row maps differ");
}

void mv_times_mat_add_mv(double alpha, const migmres_mv &A, const double *B, int ldb, double beta,
                         migmres_mv &Y) {
  same_rows(A, Y);
  migmres_ctx *c = Y.ctx;
  const int L = A.ncols, k = Y.ncols;
  if (k == 0) return;
  if (L == 0 || alpha == 0.0) {
    if (beta == 0.0)
      launch_fill(c->stream, Y.desc(), Y.n_local, 0.0);
    else if (beta != 1.0)
      launch_scale(c->stream, Y.desc(), Y.n_local, beta, nullptr);
    return;
  }
  double *h = c->pinned((size_t)L * k);
  for (int j = 0; j < k; ++j)
    for (int i = 0; i < L; ++i) h[(size_t)i + (size_t)j * L] = B[(size_t)i + (size_t)j * ldb];
  double *d = c->coef((size_t)L * k);
  MIG_HIP(hipMemcpyAsync(d, h, sizeof(double) * L * k, hipMemcpyHostToDevice, c->stream));
  {
    ProfScope ps(c, K_GEMM_NN, 8.0 * Y.n_local * (L + (beta == 0.0 ? 1.0 : 2.0) * k));
    launch_gemm_nn(c->stream, A.desc(), L, d, L, Y.desc(), Y.n_local, alpha, beta);
  }
  // the pinned staging buffer is reused by the next call: keep the copy ordered
  MIG_HIP(hipStreamSynchronize(c->stream));
}

void mv_add_mv(double alpha, const migmres_mv &A, double beta, const migmres_mv &B, migmres_mv &Y) {
  same_rows(A, Y);
  same_rows(B, Y);
  MIG_CHECK(A.ncols == Y.ncols && B.ncols == Y.ncols, "MvAddMv column counts differ");
  ProfScope ps(Y.ctx, K_AXPBY, 24.0 * Y.n_local * Y.ncols);
  launch_axpby(Y.ctx->stream, alpha, A.desc(), beta, B.desc(), Y.desc(), Y.n_local);
}

void mv_scale(migmres_mv &Y, double alpha) {
  ProfScope ps(Y.ctx, K_SCALE, 16.0 * Y.n_local * Y.ncols);
  launch_scale(Y.ctx->stream, Y.desc(), Y.n_local, alpha, nullptr);
}

void mv_scale_vec(migmres_mv &Y, const double *alphas) {
  migmres_ctx *c = Y.ctx;
  double *d = c->coef((size_t)Y.ncols);
  MIG_HIP(hipMemcpyAsync(d, alphas, sizeof(double) * Y.ncols, hipMemcpyHostToDevice, c->stream));
  launch_scale(c->stream, Y.desc(), Y.n_local, 1.0, d);
  MIG_HIP(hipStreamSynchronize(c->stream));
}

void mv_trans_mv(double alpha, const migmres_mv &A, const migmres_mv &B, double *C, int ldc) {
  same_rows(A, B);
  migmres_ctx *c = A.ctx;
  const int L = A.ncols, kb = B.ncols;
  if (L == 0 || kb == 0) return;
  double *red = c->red((size_t)L * kb);
  // Column chunks: A in 512-column slabs, B in 16-column slabs; views stay alive until the
  // stream is drained because kernels read their column tables.
  std::vector<migmres_mv *> views;
  try {
    for (int b0 = 0; b0 < kb; b0 += 16) {
      const int kc = (kb - b0) < 16 ? (kb - b0) : 16;
      migmres_mv *Bv = mv_view_range(const_cast<migmres_mv *>(&B), b0, kc);
      views.push_back(Bv);
      for (int a0 = 0; a0 < L; a0 += 512) {
        const int lc = (L - a0) < 512 ? (L - a0) : 512;
        const int nblk = gemm_tn_blocks(A.n_local, lc);
        migmres_mv *Av = mv_view_range(const_cast<migmres_mv *>(&A), a0, lc);
        views.push_back(Av);
        double *part = c->partial((size_t)nblk * lc * kc);
        double *tmp = c->coef((size_t)lc * kc);
        {
          ProfScope ps(c, K_GEMM_TN, 8.0 * A.n_local * (lc + kc) + 8.0 * nblk * lc * kc);
          launch_gemm_tn_partial(c->stream, Av->desc(), lc, Bv->desc(), kc, A.n_local, part, nblk);
        }
        {
          ProfScope ps(c, K_REDUCE, 8.0 * nblk * lc * kc + 8.0 * lc * kc);
          launch_reduce_partials(c->stream, part, nblk, lc * kc, alpha, tmp);
        }
        MIG_HIP(hipMemcpy2DAsync(red + a0 + (size_t)b0 * L, sizeof(double) * L, tmp,
                                 sizeof(double) * lc, sizeof(double) * lc, kc,
                                 hipMemcpyDeviceToDevice, c->stream));
        if (L > 512 || kb > 16) MIG_HIP(hipStreamSynchronize(c->stream));  // scratch reuse
      }
    }
  } catch (...) {
    hipStreamSynchronize(c->stream);
    for (auto *v : views) delete v;
    throw;
  }
  c->allreduce(red, (size_t)L * kb);
  double *h = c->pinned((size_t)L * kb);
  MIG_HIP(hipMemcpyAsync(h, red, sizeof(double) * L * kb, hipMemcpyDeviceToHost, c->stream));
  MIG_HIP(hipStreamSynchronize(c->stream));
  for (auto *v : views) delete v;
  for (int j = 0; j < kb; ++j)
    for (int i = 0; i < L; ++i) C[(size_t)i + (size_t)j * ldc] = h[(size_t)i + (size_t)j * L];
}

static void coldot_reduce(const migmres_mv &A, const migmres_mv &B, int op, double *out) {
  migmres_ctx *c = A.ctx;
  const int k = A.ncols;
  if (k == 0) return;
  const int nblk = coldot_blocks(A.n_local);
  double *part = c->partial((size_t)nblk * k);
  double *red = c->red((size_t)k);
  {
    ProfScope ps(c, K_COLDOT, 8.0 * A.n_local * k * (op == 0 ? 2.0 : 1.0));
    launch_coldot_partial(c->stream, A.desc(), B.desc(), A.n_local, op, part, nblk);
  }
  if (op == 2)
    launch_reduce_max(c->stream, part, nblk, k, red);
  else
    launch_reduce_partials(c->stream, part, nblk, k, 1.0, red);
  c->allreduce(red, (size_t)k, op == 2);
  double *h = c->pinned((size_t)k);
  MIG_HIP(hipMemcpyAsync(h, red, sizeof(double) * k, hipMemcpyDeviceToHost, c->stream));
  MIG_HIP(hipStreamSynchronize(c->stream));
  std::memcpy(out, h, sizeof(double) * k);
}

void mv_dot(const migmres_mv &A, const migmres_mv &B, double *out) {
  same_rows(A, B);
  MIG_CHECK(A.ncols == B.ncols, "MvDot column counts differ");
  coldot_reduce(A, B, 0, out);
}

void mv_norm(const migmres_mv &A, double *out, int type) {
  if (type == MIGMRES_TWO_NORM) {
    coldot_reduce(A, A, 0, out);
    for (int i = 0; i < A.ncols; ++i) out[i] = std::sqrt(out[i]);
  } else if (type == MIGMRES_ONE_NORM) {
    coldot_reduce(A, A, 1, out);
  } else {
    coldot_reduce(A, A, 2, out);
  }
}

void mv_init(migmres_mv &Y, double alpha) {
  ProfScope ps(Y.ctx, K_FILL, 8.0 * Y.n_local * Y.ncols);
  launch_fill(Y.ctx->stream, Y.desc(), Y.n_local, alpha);
}

void mv_random(migmres_mv &Y, unsigned int *seed) {
  migmres_ctx *c = Y.ctx;
  long long first = 0;
  int nl = 0;
  uniform_map(Y.n_global, c->nranks, c->rank, &first, &nl);
  if (nl != Y.n_local) {
    // non-uniform row map: exclusive scan of local lengths
    std::vector<double> lens((size_t)c->nranks, 0.0);
    lens[(size_t)c->rank] = (double)Y.n_local;
    double *d = c->red((size_t)c->nranks);
    MIG_HIP(hipMemcpyAsync(d, lens.data(), sizeof(double) * c->nranks, hipMemcpyHostToDevice, c->stream));
    c->allreduce(d, (size_t)c->nranks);
    MIG_HIP(hipMemcpyAsync(lens.data(), d, sizeof(double) * c->nranks, hipMemcpyDeviceToHost, c->stream));
    MIG_HIP(hipStreamSynchronize(c->stream));
    first = 0;
    for (int r = 0; r < c->rank; ++r) first += (long long)lens[(size_t)r];
  }
  launch_random(c->stream, Y.desc(), Y.n_local, first, Y.n_global, *seed);
  // advance the stream past all global entries, as Random() on P=1 would
  unsigned long long s = *seed, a = 16807ULL, e = (unsigned long long)Y.n_global * Y.ncols, acc = 1;
  const unsigned long long m = 2147483647ULL;
  while (e) {
    if (e & 1ULL) acc = acc * a % m;
    a = a * a % m;
    e >>= 1;
  }
  *seed = (unsigned int)(s * acc % m);
}

void mv_assign(const migmres_mv &A, migmres_mv &Y) {
  same_rows(A, Y);
  MIG_CHECK(A.ncols == Y.ncols, "Assign column counts differ");
  ProfScope ps(Y.ctx, K_COPY, 16.0 * Y.n_local * Y.ncols);
  launch_copy(Y.ctx->stream, A.desc(), Y.desc(), Y.n_local);
}

}  // namespace migmres

// ------------------------------------------------------------------------------------
// distributed CRS operator
// ------------------------------------------------------------------------------------
migmres_crs::~migmres_crs() {
  for (void *p : {(void *)d_soff, (void *)d_slen, (void *)d_scol, (void *)d_sval, (void *)d_xr, (void *)d_tpl_id,
                  (void *)d_tpl_rec, (void *)d_tpl_val, (void *)d_tpl_rest, (void *)d_tpl3_grp, (void *)d_b3off,
                  (void *)d_b3len, (void *)d_b3col, (void *)d_b3val, (void *)d_b3rest})
    if (p) hipFree(p);
  for (void *p : {(void *)d_export_grp, (void *)d_remote_grp, (void *)d_recv})
    if (p) hipFree(p);
  for (void *p : {(void *)d_rowptr, (void *)d_cols, (void *)d_export, (void *)d_vals, (void *)d_send,
                  (void *)d_ghost, (void *)d_psv, (void *)d_psk, (void *)d_psm, (void *)d_sel_int,
                  (void *)d_sel_bnd})
    if (p) hipFree(p);
  for (void *p : {(void *)d_trowptr, (void *)d_tcols, (void *)d_tiota, (void *)d_tvals, (void *)d_tbuf,
                  (void *)d_tsend, (void *)d_trecv})
    if (p) hipFree(p);
}

namespace migmres {

// The part of crs_create after FillComplete's index maps: export lists, device copies, the
// SpMM formats and the halo split.  A holds colmap / plan; lcols / lvals are the X-space
// local CSR (rows sorted by Epetra local id).  d_* arrays already on the device (the device
// FillComplete's outputs) are kept, otherwise uploaded.
static void crs_finish(migmres_crs *A, const long long *rowptr, std::vector<int> &lcols, std::vector<double> &lvals);

migmres_crs *crs_create(migmres_ctx *ctx, long long n_global, long long first, int n_local,
                        const long long *rowptr, const long long *gcols, const double *vals) {
  MIG_CHECK(ctx && n_local >= 0 && rowptr, "bad CRS arguments");
  const long long nnz = rowptr[n_local];
  MIG_CHECK(nnz < (1LL << 31), "local nnz must fit int32 row offsets");
  auto *A = new migmres_crs();
  try {
    A->ctx = ctx;
    A->n_global = n_global;
    A->first = first;
    A->n_local = n_local;
    A->nnz = nnz;
    A->colmap = make_colmap(n_global, ctx->nranks, first, n_local, rowptr, gcols);
    A->n_cols = (int)A->colmap.size();
    A->plan = make_remotes(n_global, ctx->nranks, first, n_local, A->colmap.data(), A->n_cols);
    const RemotePlan &p = A->plan;
    const int n_remote = (int)p.remote_lids.size();

    // Epetra local ids (sorted rows) -> X-space ids: owned columns index the local rows,
    // remote columns index the ghost block in import (PID-sorted) order.
    std::vector<int> lcols((size_t)nnz);
    std::vector<double> lvals((size_t)nnz);
    local_crs(n_local, rowptr, gcols, vals, A->colmap.data(), A->n_cols, first, lcols.data(),
              lvals.data());
    std::vector<int> xspace((size_t)A->n_cols, -1);
    for (int i = 0; i < A->n_cols; ++i) {
      const long long g = A->colmap[(size_t)i];
      if (g >= first && g < first + n_local) xspace[(size_t)i] = (int)(g - first);
    }
    for (int i = 0; i < n_remote; ++i) xspace[(size_t)p.remote_lids[(size_t)i]] = n_local + i;
    for (auto &v : lcols) v = xspace[(size_t)v];
    crs_finish(A, rowptr, lcols, lvals);
  } catch (...) {
    delete A;
    throw;
  }
  return A;
}

migmres_crs *crs_create_device(migmres_ctx *ctx, long long n_global, long long first, int n_local,
                               const long long *d_rowptr, const long long *d_gcols, const double *d_vals) {
  MIG_CHECK(ctx && n_local >= 0 && d_rowptr, "bad CRS arguments");
  MIG_HIP(hipSetDevice(ctx->device));
  auto *A = new migmres_crs();
  try {
    A->ctx = ctx;
    A->n_global = n_global;
    A->first = first;
    A->n_local = n_local;
    std::vector<long long> rowptr;
    std::vector<int> lcols;
    std::vector<double> lvals;
    setup_mark("crs_create_device");
    fill_complete_device(A, d_rowptr, d_gcols, d_vals, rowptr, lcols, lvals);
    setup_mark("fill_complete_device");
    if (!A->nnz && (int)rowptr.size() > n_local) A->nnz = rowptr[(size_t)n_local];
    crs_finish(A, rowptr.data(), lcols, lvals);
    setup_mark("crs_finish");
  } catch (...) {
    delete A;
    throw;
  }
  return A;
}

static bool env_on(const char *name) {
  const char *e = std::getenv(name);
  return e && e[0] == '1';
}

// The lane-shared form of the templates (k_spmm_tpl3) and the template kernels' knobs.
static void setup_template_kernels(migmres_crs *A, const PairTemplates &pt) {
  const char *tsl = std::getenv("MIGMRES_TPL_SLABS");
  A->tpl_slabs = tsl ? std::atoi(tsl) : 0;
  const char *tkc = std::getenv("MIGMRES_TPL_KC");
  A->tpl_kc = tkc ? std::atoi(tkc) : 8;
  // long templates (27-point stencils): the lane-shared form when the keys come in
  // x-neighbour triples (k_spmm_tpl3); MIGMRES_NO_TPL3=1 keeps k_spmm_tpl
  const bool short_ok = env_on("MIGMRES_TPL3_SHORT");  // 7-point templates too (tuning)
  StencilGroups sg;
  const bool groups = make_stencil_groups(pt, sg) && (sg.G == 9 || sg.G == 5 || sg.G == 3);
  auto upload_groups = [&] {
    MIG_HIP(hipMalloc(&A->d_tpl3_grp, sizeof(unsigned long long) * sg.slots.size()));
    MIG_HIP(hipMemcpy(A->d_tpl3_grp, sg.slots.data(), sizeof(unsigned long long) * sg.slots.size(),
                      hipMemcpyHostToDevice));
    A->tpl3_center = sg.center;
    A->tpl3_G = sg.G;
  };
  // the plane march for 3-D stencil groups: k_spmm_march7 for the 7-point pattern (measured
  // faster than the template kernel); the general k_spmm_march (any 3-D groups) only with
  // MIGMRES_MARCH_GENERIC=1 -- for 27 points it is slower than the lane-shared k_spmm_tpl3
  // (its LDS reads bound it).  MIGMRES_NO_MARCH=1 keeps the template kernels.
  MarchGeometry mg;
  const bool generic = env_on("MIGMRES_MARCH_GENERIC");
  bool seven = groups && sg.G == 5;
  if (!env_on("MIGMRES_NO_MARCH") && groups && make_march_geometry(sg, pt.ntpl, pt.npairs, mg)) {
    if (seven) {
      static const int want_a[5] = {-1, 0, 0, 0, 1}, want_b[5] = {0, -1, 0, 1, 0};
      for (int g = 0; g < 5; ++g) seven = seven && mg.ga[(size_t)g] == want_a[g] && mg.gb[(size_t)g] == want_b[g];
      // neighbour halves only on the x line
      for (int t = 0; t < pt.ntpl && seven; ++t)
        for (int g = 0; g < 5; ++g)
          if (g != 2) {
            const unsigned long long w = sg.slots[(size_t)t * 5 + g];
            seven = seven && (w & 0xFF) == kTplUnused && ((w >> 40) & 0xFF) == kTplUnused;
          }
    }
  }
  // Uniform stencil forms (the 27-point march, and the 7-point march without per-lane
  // coefficients): a full template -- one whose used slots contain every template's -- whose
  // values every template's used slots agree with bit for bit; every slot a template leaves
  // unused (of those the full template uses) must read a neighbour outside the grid, which
  // march27_check verifies on the device below.  The 27-point form also needs all 54 slots used.
  const int Gu = sg.G;
  March27Coef U{};
  std::vector<unsigned long long> umask((size_t)pt.ntpl, 0);
  bool uniform = !generic && groups && (Gu == 9 || Gu == 5) && mg.nxp > 0;
  if (uniform && Gu == 9)
    for (int g = 0; g < 9; ++g) uniform = uniform && mg.ga[(size_t)g] == g / 3 - 1 && mg.gb[(size_t)g] == g % 3 - 1;
  if (uniform && Gu == 5) uniform = seven;
  int full = -1;
  for (int t = 0; t < pt.ntpl && uniform; ++t) {
    for (int g = 0; g < Gu; ++g)
      for (int i = 0; i < 6; ++i)
        if (((sg.slots[(size_t)t * Gu + g] >> (8 * i)) & 0xFF) != kTplUnused) umask[(size_t)t] |= 1ULL << (6 * g + i);
    if (full < 0 || __builtin_popcountll(umask[(size_t)t]) > __builtin_popcountll(umask[(size_t)full])) full = t;
  }
  uniform = uniform && full >= 0 && (Gu != 9 || umask[(size_t)full] == (1ULL << 54) - 1);
  if (uniform) {
    auto value = [&](int t, int g, int i) {
      const unsigned sl = (unsigned)(sg.slots[(size_t)t * Gu + g] >> (8 * i)) & 0xFF;
      return sl < pt.vals.size() ? pt.vals[sl] : 0.0;
    };
    U.used = umask[(size_t)full];
    for (int g = 0; g < Gu; ++g)
      for (int i = 0; i < 6; ++i) U.w[g][i] = value(full, g, i);
    for (int t = 0; t < pt.ntpl && uniform; ++t) {
      if ((umask[(size_t)t] & ~U.used) != 0) uniform = false;
      for (int g = 0; g < Gu; ++g)
        for (int i = 0; i < 6; ++i) {
          const double v = value(t, g, i);
          if (((umask[(size_t)t] >> (6 * g + i)) & 1ULL) && std::memcmp(&v, &U.w[g][i], sizeof(double)) != 0)
            uniform = false;
        }
    }
  }
  bool uni27 = uniform && Gu == 9;
  bool uni7 = uniform && Gu == 5 && U.used == kMarch7Used && !env_on("MIGMRES_MARCH7_LANE_COEF");
  if (uniform && !env_on("MIGMRES_MARCH27_TABLE")) {  // at most two distinct values: select, not a table
    int nv = 0;
    for (int g = 0; g < Gu; ++g)
      for (int i = 0; i < 6; ++i) {
        if (!((U.used >> (6 * g + i)) & 1ULL)) continue;
        const double v = U.w[g][i];
        int which = -1;
        for (int q = 0; q < nv; ++q)
          if (std::memcmp(&v, &U.v2[q], sizeof(double)) == 0) which = q;
        if (which < 0 && nv < 2) U.v2[which = nv++] = v;
        if (which < 0) nv = 3;
        if (which == 1) U.sel |= 1ULL << (6 * g + i);
      }
    // the 27-point kernel's two-valued form has the slot pattern fixed: the diagonal slots
    // take v2[1], every other slot v2[0]
    if (nv == 2 && U.sel == (((1ULL << 54) - 1) & ~kMarch27Diag)) {
      std::swap(U.v2[0], U.v2[1]);
      U.sel = kMarch27Diag;
    }
    U.two_valued = (nv <= 2 && (nv == 1 || U.sel == kMarch27Diag) && Gu == 9) ? 1 : 0;
    if (nv == 1) U.v2[1] = U.v2[0];
    if (!U.two_valued) U.sel = 0;
  }
  const bool use_march = !env_on("MIGMRES_NO_MARCH") && groups && (generic || seven || uni27) && mg.nxp > 0 &&
                         march_check(A->ctx->stream, pt.npairs, A->d_tpl_id, (const int4 *)mg.tb.data(), pt.ntpl,
                                     mg.nxp, mg.nyl) == 0;
  MarchGeom geo;
  geo.nxp = mg.nxp;
  geo.nyl = mg.nyl;
  geo.plane = mg.plane;
  geo.nz = mg.nz;
  for (int g = 0; g < sg.G && use_march; ++g) {
    geo.ga[g] = mg.ga[(size_t)g];
    geo.gb[g] = mg.gb[(size_t)g];
  }
  if (use_march && (uni27 || uni7) &&
      march27_check(A->ctx->stream, pt.npairs, A->d_tpl_id, umask.data(), pt.ntpl, geo, Gu,
                    ~U.used & ((1ULL << (6 * Gu)) - 1)) != 0)
    uni27 = uni7 = false;
  if (use_march && (generic || seven || uni27)) {
    upload_groups();
    A->use_march7 = seven && !generic;
    A->use_march27 = uni27;
    A->march_uni7 = uni7 && A->use_march7;
    A->march27_coef = U;
    A->march = geo;
    A->use_march = true;
    const char *kc = std::getenv("MIGMRES_MARCH_KC");
    A->march_kc = kc ? std::atoi(kc) : 2;
    const char *sz = std::getenv("MIGMRES_MARCH_SZ");
    A->march_sz = sz ? std::atoi(sz) : 0;
    const char *pd = std::getenv("MIGMRES_MARCH_PD");
    A->march_pd = pd ? std::atoi(pd) : (A->use_march7 ? (A->march_uni7 ? 2 : 3) : A->use_march27 ? 2 : 1);
    const char *nl = std::getenv("MIGMRES_MARCH_NL");
    // 8-line tiles (NL = 2): half the y-halo lines per tile; 256^3 k = 8 SpMM 0.458 -> 0.451 ms,
    // fabric reads 1.25 -> 1.22 x X (same box, profiles/r4h_*)
    A->march_nl = nl ? std::atoi(nl) : 2;
    return;
  }
  if (!env_on("MIGMRES_NO_TPL3") && (pt.maxk > 12 || short_ok) && groups) {
    upload_groups();
    A->use_tpl3 = true;
    const char *sl = std::getenv("MIGMRES_TPL3_SLABS");
    A->tpl3_slabs = sl ? std::atoi(sl) : 1;
    const char *kc = std::getenv("MIGMRES_TPL3_KC");
    A->tpl3_kc = kc ? std::atoi(kc) : 4;
  }
}

// make_pair_templates (plan.cpp) on a host copy of the local CRS, uploaded with the pairs
// left to the rest kernel.  Returns false (nothing changed) when the shapes do not fit.
static bool install_templates_host(migmres_crs *A, const long long *rowptr, const int *lcols, const double *lvals) {
  const int n_local = A->n_local;
  PairTemplates pt;
  if (!make_pair_templates(n_local, rowptr, lcols, lvals, pt)) return false;
  std::vector<int> rest;
  double rest_bytes = 0.0;
  for (int q = 0; q < pt.npairs; ++q) {
    if (pt.id[(size_t)q] != kTplNone) continue;
    if (A->use_pairs) rest.push_back(q);
    for (int r = 2 * q; r < std::min(n_local, 2 * q + 2); ++r) {
      if (!A->use_pairs) rest.push_back(r);
      rest_bytes += 12.0 * (double)(rowptr[r + 1] - rowptr[r]) + 4.0;
    }
  }
  MIG_HIP(hipMalloc(&A->d_tpl_id, pt.id.size()));
  MIG_HIP(hipMalloc(&A->d_tpl_rec, sizeof(int) * pt.rec.size()));
  MIG_HIP(hipMalloc(&A->d_tpl_val, sizeof(double) * (pt.vals.size() + 1)));
  MIG_HIP(hipMemcpy(A->d_tpl_id, pt.id.data(), pt.id.size(), hipMemcpyHostToDevice));
  MIG_HIP(hipMemcpy(A->d_tpl_rec, pt.rec.data(), sizeof(int) * pt.rec.size(), hipMemcpyHostToDevice));
  if (!pt.vals.empty())
    MIG_HIP(hipMemcpy(A->d_tpl_val, pt.vals.data(), sizeof(double) * pt.vals.size(), hipMemcpyHostToDevice));
  if (!rest.empty()) {
    MIG_HIP(hipMalloc(&A->d_tpl_rest, sizeof(int) * rest.size()));
    MIG_HIP(hipMemcpy(A->d_tpl_rest, rest.data(), sizeof(int) * rest.size(), hipMemcpyHostToDevice));
  }
  A->n_tpl_rest = (int)rest.size();
  A->tpl_ntpl = pt.ntpl;
  A->tpl_maxk = pt.maxk;
  A->tpl_nvals = (int)pt.vals.size();
  A->use_tpl = true;
  setup_template_kernels(A, pt);
  A->spmm_fixed_bytes = (double)pt.npairs + 8.0 * pt.rec.size() / 2 + 8.0 * pt.vals.size() + rest_bytes;
  return true;
}

// formats.hip: every SpMM format plan and the halo overlap's unit lists from the device CSR.
static void build_formats_device(migmres_crs *A) {
  migmres_ctx *ctx = A->ctx;
  hipStream_t s = ctx->stream;
  const int n_local = A->n_local;
  const long long nnz = A->nnz;
  const DevCsr dc{n_local, nnz, A->d_rowptr, A->d_cols, A->d_vals};
  if (!env_on("MIGMRES_NO_PAIR_SPMM") && n_local > 0) {
    DevPairSell ps;
    if (dev_pair_sell(s, dc, ps)) {
      A->d_psv = ps.v;
      A->d_psk = ps.k;
      A->d_psm = ps.m;
      A->use_pairs = true;
      A->pair_max_keys = ps.maxk;
      A->pair_rmax = ps.rmax;
    }
  }
  if (!A->use_pairs && !env_on("MIGMRES_NO_SELL_SPMM") && n_local > 0) {
    DevSell64 sp;
    dev_sell64(s, dc, sp);
    A->d_soff = sp.off;
    A->d_slen = sp.len;
    A->d_scol = sp.cols;
    A->d_sval = sp.vals;
    A->use_sell = true;
    DevBsr3 b3;
    if (!env_on("MIGMRES_NO_BSR3") && dev_bsr3(s, dc, b3)) {
      A->d_b3off = b3.off;
      A->d_b3len = b3.len;
      A->d_b3col = b3.bcol;
      A->d_b3val = b3.vals;
      A->d_b3rest = b3.rest;
      A->b3_nbr = b3.nbr;
      A->n_b3rest = b3.n_rest;
      A->b3_fixed_bytes = 8.0 * 9.0 * (double)b3.nslots + 4.0 * (double)b3.nslots + 4.0 * b3.nbr + b3.rest_bytes;
      A->use_bsr3 = true;
    }
  }
  A->spmm_fixed_bytes = A->use_bsr3 ? A->b3_fixed_bytes : 12.0 * nnz + 4.0 * (n_local + 1);
  DevTemplates dt;
  const int tpl = !env_on("MIGMRES_NO_TPL_SPMM") && n_local > 0 ? dev_templates(s, dc, dt) : 0;
  if (tpl < 0) {
    // two shapes share a hash: the host builder (exact shape comparison) on a copy of the CRS
    ++A->tpl_host_fallbacks;
    std::vector<int> rp32((size_t)n_local + 1), lcols((size_t)nnz);
    std::vector<double> lvals((size_t)nnz);
    MIG_HIP(hipMemcpy(rp32.data(), A->d_rowptr, sizeof(int) * rp32.size(), hipMemcpyDeviceToHost));
    MIG_HIP(hipMemcpy(lcols.data(), A->d_cols, sizeof(int) * lcols.size(), hipMemcpyDeviceToHost));
    MIG_HIP(hipMemcpy(lvals.data(), A->d_vals, sizeof(double) * lvals.size(), hipMemcpyDeviceToHost));
    std::vector<long long> rp(rp32.begin(), rp32.end());
    install_templates_host(A, rp.data(), lcols.data(), lvals.data());
  }
  if (tpl > 0) {
    double rest_bytes = 0.0;
    A->n_tpl_rest = dev_template_rest(s, dc, dt.id, dt.npairs, A->use_pairs, &A->d_tpl_rest, &rest_bytes);
    A->d_tpl_id = dt.id;
    MIG_HIP(hipMalloc(&A->d_tpl_rec, sizeof(int) * dt.rec.size()));
    MIG_HIP(hipMalloc(&A->d_tpl_val, sizeof(double) * (dt.vals.size() + 1)));
    MIG_HIP(hipMemcpy(A->d_tpl_rec, dt.rec.data(), sizeof(int) * dt.rec.size(), hipMemcpyHostToDevice));
    if (!dt.vals.empty())
      MIG_HIP(hipMemcpy(A->d_tpl_val, dt.vals.data(), sizeof(double) * dt.vals.size(), hipMemcpyHostToDevice));
    A->tpl_ntpl = dt.ntpl;
    A->tpl_maxk = dt.maxk;
    A->tpl_nvals = (int)dt.vals.size();
    A->use_tpl = true;
    PairTemplates pt;
    pt.ntpl = dt.ntpl;
    pt.maxk = dt.maxk;
    pt.npairs = dt.npairs;
    pt.rec = dt.rec;
    pt.vals = dt.vals;
    setup_template_kernels(A, pt);
    A->spmm_fixed_bytes = (double)dt.npairs + 8.0 * dt.rec.size() / 2 + 8.0 * dt.vals.size() + rest_bytes;
  }
  if (!A->plan.remote_lids.empty())
    dev_halo_units(s, dc, A->use_pairs, &A->d_sel_int, &A->n_sel_int, &A->d_sel_bnd, &A->n_sel_bnd);
  MIG_HIP(hipStreamSynchronize(s));
}

static void crs_finish(migmres_crs *A, const long long *rowptr, std::vector<int> &lcols, std::vector<double> &lvals) {
  migmres_ctx *ctx = A->ctx;
  const long long first = A->first, nnz = A->nnz;
  const int n_local = A->n_local;
  {
    const RemotePlan &p = A->plan;
    const int n_remote = (int)p.remote_lids.size();

    // neighbour groups of the receive side (remote list is grouped by owner PID)
    for (int i = 0; i < n_remote;) {
      int j = i;
      while (j < n_remote && p.remote_pids[(size_t)j] == p.remote_pids[(size_t)i]) ++j;
      A->recv_nbrs.push_back({p.remote_pids[(size_t)i], i, j - i});
      i = j;
    }
    // export lists: every rank tells each owner which GIDs it needs, in its own order
    // (Epetra_MpiDistributor::CreateFromRecvs with Deterministic = true).
    if (ctx->dist) {
      const int P = ctx->nranks;
      std::vector<double> cnt((size_t)P * P, 0.0);
      for (auto &nb : A->recv_nbrs) cnt[(size_t)ctx->rank * P + nb.pid] = nb.count;
      double *dc = ctx->red((size_t)P * P);
      MIG_HIP(hipMemcpyAsync(dc, cnt.data(), sizeof(double) * P * P, hipMemcpyHostToDevice, ctx->stream));
      ctx->allreduce(dc, (size_t)P * P);
      MIG_HIP(hipMemcpyAsync(cnt.data(), dc, sizeof(double) * P * P, hipMemcpyDeviceToHost, ctx->stream));
      MIG_HIP(hipStreamSynchronize(ctx->stream));
      long long *d_req = nullptr, *d_give = nullptr;
      long long total_give = 0;
      std::vector<int> give_off((size_t)P, 0), give_cnt((size_t)P, 0);
      for (int q = 0; q < P; ++q) {
        give_cnt[(size_t)q] = (q == ctx->rank) ? 0 : (int)cnt[(size_t)q * P + ctx->rank];
        give_off[(size_t)q] = (int)total_give;
        total_give += give_cnt[(size_t)q];
      }
      MIG_HIP(hipMalloc(&d_req, sizeof(long long) * (n_remote > 0 ? n_remote : 1)));
      MIG_HIP(hipMalloc(&d_give, sizeof(long long) * (total_give > 0 ? total_give : 1)));
      if (n_remote)
        MIG_HIP(hipMemcpy(d_req, p.remote_gids.data(), sizeof(long long) * n_remote, hipMemcpyHostToDevice));
      ctx->p2p_begin(ctx->stream);
      for (auto &nb : A->recv_nbrs) ctx->p2p_send(d_req + nb.offset, sizeof(long long) * nb.count, nb.pid);
      for (int q = 0; q < P; ++q)
        if (give_cnt[(size_t)q] > 0)
          ctx->p2p_recv(d_give + give_off[(size_t)q], sizeof(long long) * give_cnt[(size_t)q], q);
      ctx->p2p_end();
      std::vector<long long> give((size_t)total_give);
      if (total_give)
        MIG_HIP(hipMemcpyAsync(give.data(), d_give, sizeof(long long) * total_give, hipMemcpyDeviceToHost, ctx->stream));
      MIG_HIP(hipStreamSynchronize(ctx->stream));
      hipFree(d_req);
      hipFree(d_give);
      for (int q = 0; q < P; ++q) {
        if (give_cnt[(size_t)q] == 0) continue;
        A->send_nbrs.push_back({q, (int)A->export_lids.size(), give_cnt[(size_t)q]});
        for (int i = 0; i < give_cnt[(size_t)q]; ++i) {
          const long long g = give[(size_t)give_off[(size_t)q] + i];
          MIG_CHECK(g >= first && g < first + n_local, "requested GID not owned here");
          A->export_lids.push_back((int)(g - first));
          A->export_pids.push_back(q);
        }
      }
    }
    // device copies (the device FillComplete has made them already)
    if (!A->d_rowptr) {
      std::vector<int> rp32((size_t)n_local + 1);
      for (int r = 0; r <= n_local; ++r) rp32[(size_t)r] = (int)rowptr[r];
      MIG_HIP(hipMalloc(&A->d_rowptr, sizeof(int) * (n_local + 1)));
      MIG_HIP(hipMalloc(&A->d_cols, sizeof(int) * (nnz > 0 ? nnz : 1)));
      MIG_HIP(hipMalloc(&A->d_vals, sizeof(double) * (nnz + 8)));
      MIG_HIP(hipMemset(A->d_vals, 0, sizeof(double) * (nnz + 8)));
      MIG_HIP(hipMemcpy(A->d_rowptr, rp32.data(), sizeof(int) * (n_local + 1), hipMemcpyHostToDevice));
      if (nnz) {
        MIG_HIP(hipMemcpy(A->d_cols, lcols.data(), sizeof(int) * nnz, hipMemcpyHostToDevice));
        MIG_HIP(hipMemcpy(A->d_vals, lvals.data(), sizeof(double) * nnz, hipMemcpyHostToDevice));
      }
    }
    if (host_formats()) {
      {
        PairPlan pp;
        const char *np = std::getenv("MIGMRES_NO_PAIR_SPMM");
        if (!(np && np[0] == '1') && n_local > 0 && make_pair_plan(n_local, rowptr, lcols.data(), pp)) {
          PairSell ps;
          make_pair_sell(n_local, rowptr, lvals.data(), pp, ps);
          MIG_HIP(hipMalloc(&A->d_psv, sizeof(double) * ps.v.size()));
          MIG_HIP(hipMalloc(&A->d_psk, sizeof(int) * ps.k.size()));
          MIG_HIP(hipMalloc(&A->d_psm, sizeof(unsigned short) * ps.m.size()));
          MIG_HIP(hipMemcpy(A->d_psv, ps.v.data(), sizeof(double) * ps.v.size(), hipMemcpyHostToDevice));
          MIG_HIP(hipMemcpy(A->d_psk, ps.k.data(), sizeof(int) * ps.k.size(), hipMemcpyHostToDevice));
          MIG_HIP(hipMemcpy(A->d_psm, ps.m.data(), sizeof(unsigned short) * ps.m.size(), hipMemcpyHostToDevice));
          A->use_pairs = true;
          A->pair_max_keys = ps.maxk;
          A->pair_rmax = ps.rmax;
        }
      }
      {
        const char *ns = std::getenv("MIGMRES_NO_SELL_SPMM");
        if (!A->use_pairs && !(ns && ns[0] == '1') && n_local > 0) {
          Sell64 sp;
          make_sell64(n_local, rowptr, lcols.data(), lvals.data(), sp);
          MIG_HIP(hipMalloc(&A->d_soff, sizeof(long long) * sp.off.size()));
          MIG_HIP(hipMalloc(&A->d_slen, sizeof(int) * sp.len.size()));
          MIG_HIP(hipMalloc(&A->d_scol, sizeof(int) * (sp.cols.size() + 1)));
          MIG_HIP(hipMalloc(&A->d_sval, sizeof(double) * (sp.vals.size() + 1)));
          MIG_HIP(hipMemcpy(A->d_soff, sp.off.data(), sizeof(long long) * sp.off.size(), hipMemcpyHostToDevice));
          MIG_HIP(hipMemcpy(A->d_slen, sp.len.data(), sizeof(int) * sp.len.size(), hipMemcpyHostToDevice));
          if (!sp.cols.empty()) {
            MIG_HIP(hipMemcpy(A->d_scol, sp.cols.data(), sizeof(int) * sp.cols.size(), hipMemcpyHostToDevice));
            MIG_HIP(hipMemcpy(A->d_sval, sp.vals.data(), sizeof(double) * sp.vals.size(), hipMemcpyHostToDevice));
          }
          A->use_sell = true;
          // 3 x 3 block rows detected from the CRS (3-dof meshes): one column id per block and
          // contiguous operand segments; MIGMRES_NO_BSR3=1 keeps the row kernel for every row
          const char *nb3 = std::getenv("MIGMRES_NO_BSR3");
          Bsr3 b3;
          if (!(nb3 && nb3[0] == '1') && make_bsr3(n_local, rowptr, lcols.data(), lvals.data(), b3)) {
            MIG_HIP(hipMalloc(&A->d_b3off, sizeof(long long) * b3.off.size()));
            MIG_HIP(hipMalloc(&A->d_b3len, sizeof(int) * (b3.len.size() + 1)));
            MIG_HIP(hipMalloc(&A->d_b3col, sizeof(int) * (b3.bcol.size() + 1)));
            MIG_HIP(hipMalloc(&A->d_b3val, sizeof(double) * (b3.vals.size() + 1)));
            MIG_HIP(hipMemcpy(A->d_b3off, b3.off.data(), sizeof(long long) * b3.off.size(), hipMemcpyHostToDevice));
            MIG_HIP(hipMemcpy(A->d_b3len, b3.len.data(), sizeof(int) * b3.len.size(), hipMemcpyHostToDevice));
            MIG_HIP(hipMemcpy(A->d_b3col, b3.bcol.data(), sizeof(int) * b3.bcol.size(), hipMemcpyHostToDevice));
            MIG_HIP(hipMemcpy(A->d_b3val, b3.vals.data(), sizeof(double) * b3.vals.size(), hipMemcpyHostToDevice));
            if (!b3.rest.empty()) {
              MIG_HIP(hipMalloc(&A->d_b3rest, sizeof(int) * b3.rest.size()));
              MIG_HIP(hipMemcpy(A->d_b3rest, b3.rest.data(), sizeof(int) * b3.rest.size(), hipMemcpyHostToDevice));
            }
            A->b3_nbr = b3.nbr;
            A->n_b3rest = (int)b3.rest.size();
            double rest_bytes = 0.0;
            for (int r : b3.rest) rest_bytes += 12.0 * (double)(rowptr[r + 1] - rowptr[r]) + 4.0;
            A->b3_fixed_bytes = 8.0 * b3.vals.size() + 4.0 * b3.bcol.size() + 4.0 * b3.len.size() + rest_bytes;
            A->use_bsr3 = true;
          }
        }
      }
      A->spmm_fixed_bytes = A->use_bsr3 ? A->b3_fixed_bytes : 12.0 * nnz + 4.0 * (n_local + 1);
      // row-pair templates: the pairs' shapes repeat (stencils) -> one byte per pair
      if (!env_on("MIGMRES_NO_TPL_SPMM") && n_local > 0) install_templates_host(A, rowptr, lcols.data(), lvals.data());
      if (n_remote > 0) {
        // interior / boundary units for the halo overlap (a unit is a row pair with the
        // row-pair kernel, else a row; boundary = reads at least one ghost column)
        const int unit = A->use_pairs ? 2 : 1;
        const int nunits = (n_local + unit - 1) / unit;
        std::vector<int> sel_int, sel_bnd;
        for (int u = 0; u < nunits; ++u) {
          bool ghost = false;
          for (int r = u * unit; r < std::min(n_local, (u + 1) * unit) && !ghost; ++r)
            for (long long e = rowptr[r]; e < rowptr[r + 1]; ++e)
              if (lcols[(size_t)e] >= n_local) {
                ghost = true;
                break;
              }
          (ghost ? sel_bnd : sel_int).push_back(u);
        }
        A->n_sel_int = (int)sel_int.size();
        A->n_sel_bnd = (int)sel_bnd.size();
        MIG_HIP(hipMalloc(&A->d_sel_int, sizeof(int) * (sel_int.size() + 1)));
        MIG_HIP(hipMalloc(&A->d_sel_bnd, sizeof(int) * (sel_bnd.size() + 1)));
        if (!sel_int.empty())
          MIG_HIP(hipMemcpy(A->d_sel_int, sel_int.data(), sizeof(int) * sel_int.size(), hipMemcpyHostToDevice));
        if (!sel_bnd.empty())
          MIG_HIP(hipMemcpy(A->d_sel_bnd, sel_bnd.data(), sizeof(int) * sel_bnd.size(), hipMemcpyHostToDevice));
      }
    } else {
      setup_mark("crs_finish: before formats");
      build_formats_device(A);
      setup_mark("crs_finish: formats");
    }
    auto upload_groups = [](const std::vector<migmres_crs::Nbr> &nbrs, size_t n, int2 **out) {
      std::vector<int2> g(n);
      for (auto &nb : nbrs)
        for (int i = 0; i < nb.count; ++i) g[(size_t)(nb.offset + i)] = make_int2(nb.offset, nb.count);
      MIG_HIP(hipMalloc(out, sizeof(int2) * n));
      MIG_HIP(hipMemcpy(*out, g.data(), sizeof(int2) * n, hipMemcpyHostToDevice));
    };
    if (!A->export_lids.empty()) {
      MIG_HIP(hipMalloc(&A->d_export, sizeof(int) * A->export_lids.size()));
      MIG_HIP(hipMemcpy(A->d_export, A->export_lids.data(), sizeof(int) * A->export_lids.size(),
                        hipMemcpyHostToDevice));
      upload_groups(A->send_nbrs, A->export_lids.size(), &A->d_export_grp);
    }
    if (n_remote > 0) upload_groups(A->recv_nbrs, (size_t)n_remote, &A->d_remote_grp);
  }
}

// Y = alpha A diag(cs) X + beta Y (cs: the fused right Jacobi's column scale, or none).
static void crs_apply_impl(migmres_crs &A, const migmres_mv &X, migmres_mv &Y, double alpha, double beta,
                           ColScale cs) {
  MIG_CHECK(X.n_local == A.n_local && Y.n_local == A.n_local, "apply: row maps differ");
  MIG_CHECK(X.ncols == Y.ncols, "apply: column counts differ");
  migmres_ctx *c = A.ctx;
  const int k = X.ncols;
  const int n_remote = (int)A.plan.remote_lids.size();
  const int n_export = (int)A.export_lids.size();
  const bool halo = c->dist && (n_remote > 0 || n_export > 0);
  // SELL with k >= 2: operands through a row-interleaved copy of X (MIGMRES_NO_SELL_XR=1: column
  // gathers).  Measured at the bench shapes (same box): FlanProxy (73 nnz/row) k = 4 SpMM 0.604 ->
  // 0.483 ms, k = 8 464 -> 585 it/s; Brick3D (27 nnz/row, gathers already line-local) k = 4 1.93 ->
  // 1.90 ms but k = 8 3.22 -> 3.53 ms (the 8-column copy costs more than it saves) -- so up to 4
  // columns, or any width for long rows.  Not for the few template-rest rows.
  static const bool sell_xr = [] {
    const char *e = std::getenv("MIGMRES_NO_SELL_XR");
    return !(e && e[0] == '1');
  }();
  double *xr = nullptr;
  if (A.use_sell && !A.use_pairs && !A.use_tpl && A.n_local > 0 && k >= 2 &&
      (A.use_bsr3 || (sell_xr && (k <= 4 || A.nnz >= 48LL * A.n_local)))) {
    if (!A.d_xr) MIG_HIP(hipMalloc(&A.d_xr, sizeof(double) * 8 * (size_t)A.n_local));
    xr = A.d_xr;
  }
  bool xr_ready = false;  // the interleaved X copy is made once per apply (interior launch)
  auto spmm = [&](const int *sel, int nsel) {
    if (A.use_pairs) {
      launch_spmm_pair(c->stream, A.n_local, A.pair_max_keys, A.pair_rmax, A.d_psv, A.d_psk, A.d_psm, X.desc(),
                       A.d_ghost, A.ldg, Y.desc(), alpha, beta, sel, nsel, cs);
    } else if (A.use_sell) {
      xr_ready = launch_spmm_sell(c->stream, A.n_local, A.d_soff, A.d_slen, A.d_scol, A.d_sval, X.desc(),
                                  A.d_ghost, A.ldg, Y.desc(), alpha, beta, sel, nsel, xr, xr_ready, cs);
    } else {
      launch_spmm(c->stream, 0, A.n_local, A.d_rowptr, A.d_cols, A.d_vals, X.desc(), A.n_local, A.d_ghost, A.ldg,
                  Y.desc(), alpha, beta, sel, nsel, cs);
    }
  };
  if (halo) {
    if (k > A.halo_k) {
      MIG_HIP(hipStreamSynchronize(c->stream));
      MIG_HIP(hipStreamSynchronize(c->halo_stream));
      for (double *p : {A.d_send, A.d_recv, A.d_ghost})
        if (p) hipFree(p);
      A.d_send = A.d_recv = A.d_ghost = nullptr;
      MIG_HIP(hipMalloc(&A.d_send, sizeof(double) * ((size_t)n_export * k + 1)));
      MIG_HIP(hipMalloc(&A.d_recv, sizeof(double) * ((size_t)n_remote * k + 1)));
      A.ldg = (n_remote + 1) & ~1LL;
      MIG_HIP(hipMalloc(&A.d_ghost, sizeof(double) * ((size_t)A.ldg * k + 2)));
      MIG_HIP(hipMemset(A.d_ghost, 0, sizeof(double) * ((size_t)A.ldg * k + 2)));
      A.halo_k = k;
    }
    // Import on the halo stream (Epetra_Import through Epetra_MpiDistributor::Do), ordered
    // after everything already queued on the context stream (X is ready, the previous
    // apply's boundary rows have read the ghost block).  One message of k*count doubles per
    // neighbour each way (Epetra_MpiDistributor::DoPosts, Epetra_MpiDistributor.cpp:781-947).
    auto t0 = std::chrono::steady_clock::now();
    MIG_HIP(hipEventRecord(c->ev_main, c->stream));
    MIG_HIP(hipStreamWaitEvent(c->halo_stream, c->ev_main, 0));
    {
      ProfScope hs(c, K_HALO, 8.0 * k * ((double)n_export + n_remote), c->halo_stream);
      launch_pack(c->halo_stream, X.desc(), A.d_export, A.d_export_grp, n_export, A.d_send, k);
      c->p2p_begin(c->halo_stream);
      for (auto &nb : A.send_nbrs)
        c->p2p_send(A.d_send + (size_t)nb.offset * k, sizeof(double) * nb.count * k, nb.pid);
      for (auto &nb : A.recv_nbrs)
        c->p2p_recv(A.d_recv + (size_t)nb.offset * k, sizeof(double) * nb.count * k, nb.pid);
      c->p2p_end();
      launch_unpack(c->halo_stream, A.d_recv, A.d_remote_grp, n_remote, k, A.d_ghost, A.ldg);
    }
    MIG_HIP(hipEventRecord(c->ev_halo, c->halo_stream));
    c->comm_seconds += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  }
  // the uniform march kernels with every pair templated read no template id: X and Y only
  const bool no_ids = A.use_tpl && A.use_march && (A.march_uni7 || A.use_march27) && A.n_tpl_rest == 0 &&
                      !env_on("MIGMRES_MARCH7_TID");
  ProfScope ps(c, K_SPMM, (no_ids ? 0.0 : A.spmm_fixed_bytes) + 8.0 * A.n_local * k * (beta == 0.0 ? 2.0 : 3.0) +
                            (cs.own ? 8.0 * A.n_local : 0.0));
  if (A.use_tpl) {
    // templated pairs read no ghost column: they run while the halo is in flight, then the
    // pairs that do read one go to the fallback kernel
    bool done = A.use_march27 ? launch_spmm_march27(c->stream, A.n_local, A.d_tpl_id, A.march, A.march27_coef,
                                                    X.desc(), Y.desc(), alpha, beta, cs.own, A.march_sz, A.march_pd,
                                                    A.n_tpl_rest == 0)
                : A.use_march7 ? launch_spmm_march7(c->stream, A.n_local, A.d_tpl_id, A.d_tpl3_grp, A.tpl_ntpl,
                                                  A.march, A.d_tpl_val, A.tpl_nvals, X.desc(), Y.desc(), alpha,
                                                  beta, cs.own, A.march_sz, A.march_pd, A.march_nl,
                                                  A.march_uni7 ? &A.march27_coef : nullptr, A.n_tpl_rest == 0)
                : A.use_march && launch_spmm_march(c->stream, A.n_local, A.d_tpl_id, A.d_tpl3_grp, A.tpl_ntpl,
                                                   A.tpl3_G, A.march, A.d_tpl_val, A.tpl_nvals, X.desc(), Y.desc(),
                                                   alpha, beta, cs.own, A.march_kc, A.march_sz, A.march_pd);
    done = done || (A.use_tpl3 && launch_spmm_tpl3(c->stream, A.n_local, A.d_tpl_id, A.d_tpl3_grp, A.tpl_ntpl,
                                                   A.tpl3_G, A.tpl3_center.data(), A.d_tpl_val, A.tpl_nvals,
                                                   X.desc(), Y.desc(), alpha, beta, cs.own, A.tpl3_slabs,
                                                   A.tpl3_kc));
    if (!done)
      launch_spmm_tpl(c->stream, A.n_local, A.d_tpl_id, A.d_tpl_rec, A.tpl_ntpl, A.tpl_maxk, A.d_tpl_val,
                      A.tpl_nvals, X.desc(), Y.desc(), alpha, beta, cs.own, A.tpl_slabs, A.tpl_kc);
    if (halo) MIG_HIP(hipStreamWaitEvent(c->stream, c->ev_halo, 0));
    if (A.n_tpl_rest > 0) spmm(A.d_tpl_rest, A.n_tpl_rest);
  } else if (A.use_bsr3) {
    // block rows (none reads a ghost column) while the halo is in flight, then the rows left
    // to the row kernel; the block launch leaves X interleaved for them (one chunk, k <= 8)
    launch_spmm_bsr3(c->stream, A.b3_nbr, A.n_local, A.d_b3off, A.d_b3len, A.d_b3col, A.d_b3val, X.desc(), Y.desc(),
                     alpha, beta, xr, cs);
    xr_ready = xr != nullptr && k <= 8;
    if (halo) MIG_HIP(hipStreamWaitEvent(c->stream, c->ev_halo, 0));
    if (A.n_b3rest > 0) spmm(A.d_b3rest, A.n_b3rest);
  } else if (halo && A.d_sel_int) {
    // interior rows while the halo is in flight, then the rows that read ghost columns
    spmm(A.d_sel_int, A.n_sel_int);
    MIG_HIP(hipStreamWaitEvent(c->stream, c->ev_halo, 0));
    spmm(A.d_sel_bnd, A.n_sel_bnd);
  } else {
    if (halo) MIG_HIP(hipStreamWaitEvent(c->stream, c->ev_halo, 0));
    spmm(nullptr, 0);
  }
}

void crs_apply(migmres_crs &A, const migmres_mv &X, migmres_mv &Y, double alpha, double beta) {
  crs_apply_impl(A, X, Y, alpha, beta, ColScale{});
}

void op_apply(migmres_op &op, const migmres_mv &X, migmres_mv &Y) {
  if (op.crs) {
    crs_apply(*op.crs, X, Y, 1.0, 0.0);
    return;
  }
  MIG_CHECK(X.n_local == op.n_local && Y.n_local == op.n_local, "user operator apply: row map mismatch");
  MIG_CHECK(X.ncols == Y.ncols, "user operator apply: X and Y column counts differ");
  const int rc = op.fn(op.user, &X, &Y);
  if (rc != 0)
    throw Error(MIGMRES_EOP, "user operator apply returned " + std::to_string(rc) + " (last error: " +
                                 migmres_last_error() + ")");
}

// Y = A (M X) for the one-sweep right Jacobi M = omega D^-1 in one SpMM: every kernel forms
// the operand (omega d^-1)_col x_col in registers, exactly as k_jacobi forms M X
// (Ifpack2_Relaxation_def.hpp:1401-1425), so the result equals Jacobi pass + SpMM bit for bit.
// Under a halo the exchange carries X itself; ghost columns take the owner's omega d^-1,
// imported once by prec_import_ghost_scale.
// Do any columns of X and Y share memory?  (Ifpack2 compares the data pointers,
// Ifpack2_Relaxation_def.hpp:543-551; a column-range overlap test also catches views that
// start at different columns of one block.)
bool mv_overlap(const migmres_mv &X, const migmres_mv &Y) {
  if (X.ncols == 0 || Y.ncols == 0 || X.n_local == 0) return false;
  for (int i = 0; i < X.ncols; ++i) {
    const double *a0 = X.base + X.col_offset(i), *a1 = a0 + X.n_local;
    for (int j = 0; j < Y.ncols; ++j) {
      const double *b0 = Y.base + Y.col_offset(j), *b1 = b0 + Y.n_local;
      if (a0 < b1 && b0 < a1) return true;
    }
  }
  return false;
}

void crs_apply_trans(migmres_crs &A, const migmres_mv &X, migmres_mv &Y, double alpha, double beta) {
  migmres_ctx *c = A.ctx;
  MIG_CHECK(X.n_local == A.n_local && Y.n_local == A.n_local, "CRS apply (transpose): row map mismatch");
  MIG_CHECK(X.ncols == Y.ncols, "CRS apply (transpose): X and Y column counts differ");
  MIG_CHECK(!mv_overlap(X, Y), "CRS apply (transpose): X and Y may not alias one another");
  const int k = X.ncols;
  const int n_remote = (int)A.plan.remote_lids.size();
  const int n_export = (int)A.export_lids.size();
  const int n_out = A.n_local + n_remote;
  if (k == 0) return;
  if (!A.d_trowptr) {
    const DevCsr dc{A.n_local, A.nnz, A.d_rowptr, A.d_cols, A.d_vals};
    DevTrans t;
    dev_transpose(c->stream, dc, n_out, t);
    A.d_trowptr = t.rowptr;
    A.d_tcols = t.cols;
    A.d_tvals = t.vals;
  }
  const bool halo = c->dist && (n_remote > 0 || n_export > 0);
  ProfScope ps(c, K_SPMM, 12.0 * A.nnz + 4.0 * (n_out + 1) + 8.0 * A.n_local * k * (beta == 0.0 ? 2.0 : 3.0));
  if (!halo) {  // every column of A is owned: the transpose's rows are Y's rows
    launch_spmm(c->stream, 0, A.n_local, A.d_trowptr, A.d_tcols, A.d_tvals, X.desc(), A.n_local, nullptr, 0,
                Y.desc(), alpha, beta, nullptr, 0, ColScale{});
    return;
  }
  if (k > A.tr_k) {
    MIG_HIP(hipStreamSynchronize(c->stream));
    for (double *p : {A.d_tbuf, A.d_tsend, A.d_trecv})
      if (p) hipFree(p);
    A.ld_t = ((long long)n_out + 63) / 64 * 64;
    MIG_HIP(hipMalloc(&A.d_tbuf, sizeof(double) * ((size_t)A.ld_t * k + 2)));
    MIG_HIP(hipMemset(A.d_tbuf, 0, sizeof(double) * ((size_t)A.ld_t * k + 2)));
    MIG_HIP(hipMalloc(&A.d_tsend, sizeof(double) * ((size_t)n_remote * k + 1)));
    MIG_HIP(hipMalloc(&A.d_trecv, sizeof(double) * ((size_t)n_export * k + 1)));
    if (!A.d_tiota) {
      std::vector<int> iota((size_t)n_remote + 1);
      for (int i = 0; i <= n_remote; ++i) iota[(size_t)i] = i;
      MIG_HIP(hipMalloc(&A.d_tiota, sizeof(int) * iota.size()));
      MIG_HIP(hipMemcpy(A.d_tiota, iota.data(), sizeof(int) * iota.size(), hipMemcpyHostToDevice));
    }
    A.tr_k = k;
  }
  // T = A^T X over owned and ghost columns (Epetra's column-map vector), the ghost rows packed
  // per owner, one message per neighbour each way (the import's lists with the roles swapped),
  // then each neighbour's contributions added to the owned rows, neighbours in ascending PID
  // order (Epetra_Export, combine mode Add), and Y = alpha T + beta Y.
  const MvDesc T{A.d_tbuf, A.ld_t, nullptr, k};
  launch_spmm(c->stream, 0, n_out, A.d_trowptr, A.d_tcols, A.d_tvals, X.desc(), A.n_local, nullptr, 0, T, 1.0, 0.0,
              nullptr, 0, ColScale{});
  const MvDesc Tg{A.d_tbuf + A.n_local, A.ld_t, nullptr, k};
  launch_pack(c->stream, Tg, A.d_tiota, A.d_remote_grp, n_remote, A.d_tsend, k);
  c->p2p_begin(c->stream);
  for (auto &nb : A.recv_nbrs)
    c->p2p_send(A.d_tsend + (size_t)nb.offset * k, sizeof(double) * nb.count * k, nb.pid);
  for (auto &nb : A.send_nbrs)
    c->p2p_recv(A.d_trecv + (size_t)nb.offset * k, sizeof(double) * nb.count * k, nb.pid);
  c->p2p_end();
  for (auto &nb : A.send_nbrs)
    launch_export_add(c->stream, T, A.d_export + nb.offset, nb.count, k, A.d_trecv + (size_t)nb.offset * k);
  launch_combine(c->stream, T, Y.desc(), A.n_local, alpha, beta);
}

bool crs_apply_jacobi_fused(migmres_crs &A, const migmres_prec &M, const migmres_mv &X, migmres_mv &Y) {
  migmres_ctx *c = A.ctx;
  const int n_remote = (int)A.plan.remote_lids.size();
  const int n_export = (int)A.export_lids.size();
  const bool halo = c->dist && (n_remote > 0 || n_export > 0);
  if (M.kind != 0 || M.rtype != 0 || !M.zero_start || M.sweeps != 1 || !M.d_sdinv || M.A != &A) return false;
  if (halo && n_remote > 0 && !M.d_gsdinv) return false;
  if (X.n_local != A.n_local || Y.n_local != A.n_local || X.ncols != Y.ncols) return false;
  crs_apply_impl(A, X, Y, 1.0, 0.0, ColScale{M.d_sdinv, M.d_gsdinv});
  return true;
}

// The owners' omega d^-1 of A's ghost columns (the fused Jacobi's ghost column scale): the
// import of one vector through A's plan (pack the export rows, one message per neighbour,
// unpack into ghost-slot order), done once when the preconditioner is created.  Collective
// over the ranks that share A.
void prec_import_ghost_scale(migmres_prec &M) {
  migmres_crs &A = *M.A;
  migmres_ctx *c = A.ctx;
  const int n_remote = (int)A.plan.remote_lids.size();
  const int n_export = (int)A.export_lids.size();
  if (!c->dist || (n_remote == 0 && n_export == 0)) return;
  const long long ldg = (n_remote + 1) & ~1LL;
  double *send = nullptr, *recv = nullptr;
  MIG_HIP(hipMalloc(&send, sizeof(double) * ((size_t)n_export + 1)));
  MIG_HIP(hipMalloc(&recv, sizeof(double) * ((size_t)n_remote + 1)));
  MIG_HIP(hipMalloc(&M.d_gsdinv, sizeof(double) * ((size_t)ldg + 2)));
  MIG_HIP(hipMemsetAsync(M.d_gsdinv, 0, sizeof(double) * ((size_t)ldg + 2), c->stream));
  const MvDesc sd{M.d_sdinv, (long long)A.n_local, nullptr, 1};
  launch_pack(c->stream, sd, A.d_export, A.d_export_grp, n_export, send, 1);
  c->p2p_begin(c->stream);
  for (auto &nb : A.send_nbrs) c->p2p_send(send + nb.offset, sizeof(double) * nb.count, nb.pid);
  for (auto &nb : A.recv_nbrs) c->p2p_recv(recv + nb.offset, sizeof(double) * nb.count, nb.pid);
  c->p2p_end();
  launch_unpack(c->stream, recv, A.d_remote_grp, n_remote, 1, M.d_gsdinv, ldg);
  MIG_HIP(hipStreamSynchronize(c->stream));
  hipFree(send);
  hipFree(recv);
}

}  // namespace migmres

// ------------------------------------------------------------------------------------
// C ABI: maps, plans, CRS, multivectors
// ------------------------------------------------------------------------------------
extern "C" int migmres_crs_spmm_kernel(const migmres_crs *A, int *kind) {
  return guard([&] {
    MIG_CHECK(A && kind, "bad arguments");
    *kind = A->use_bsr3 ? MIGMRES_SPMM_BSR3
            : A->use_march ? MIGMRES_SPMM_MARCH
            : A->use_tpl3 ? MIGMRES_SPMM_TPL3
            : A->use_tpl ? MIGMRES_SPMM_TPL
            : A->use_pairs ? MIGMRES_SPMM_PAIR
            : A->use_sell  ? MIGMRES_SPMM_SELL
                           : MIGMRES_SPMM_CSR;
  });
}
namespace {
unsigned long long fnv_bytes(const void *d_ptr, size_t bytes) {
  unsigned long long h = 0xcbf29ce484222325ULL;
  if (!d_ptr || bytes == 0) return h;
  std::vector<unsigned char> buf(bytes);
  MIG_HIP(hipMemcpy(buf.data(), d_ptr, bytes, hipMemcpyDeviceToHost));
  for (unsigned char b : buf) h = (h ^ b) * 0x100000001b3ULL;
  return h;
}
}  // namespace

extern "C" int migmres_crs_format_digest(const migmres_crs *A, unsigned long long *out, int n, int *needed) {
  return guard([&] {
    MIG_CHECK(A, "bad arguments");
    MIG_HIP(hipStreamSynchronize(A->ctx->stream));
    std::vector<unsigned long long> d;
    auto num = [&](double v) {
      unsigned long long b;
      std::memcpy(&b, &v, sizeof(b));
      d.push_back(b);
    };
    const int nl = A->n_local, P = (nl + 1) / 2;
    d.push_back((unsigned long long)A->use_pairs | (unsigned long long)A->use_sell << 1 |
                (unsigned long long)A->use_bsr3 << 2 | (unsigned long long)A->use_tpl << 3 |
                (unsigned long long)A->use_tpl3 << 4 | (unsigned long long)A->use_march << 5);
    num(A->spmm_fixed_bytes);
    if (A->use_pairs) {
      const size_t nch = (size_t)(P + 63) / 64;
      d.push_back((unsigned long long)A->pair_max_keys << 32 | (unsigned)A->pair_rmax);
      d.push_back(fnv_bytes(A->d_psv, sizeof(double) * nch * 2 * A->pair_rmax * 64));
      d.push_back(fnv_bytes(A->d_psk, sizeof(int) * nch * A->pair_max_keys * 64));
      d.push_back(fnv_bytes(A->d_psm, sizeof(unsigned short) * nch * A->pair_max_keys * 64));
    }
    if (A->use_sell) {
      const size_t nch = (size_t)(nl + 63) / 64;
      long long total = 0;
      MIG_HIP(hipMemcpy(&total, A->d_soff + nch, sizeof(long long), hipMemcpyDeviceToHost));
      d.push_back(fnv_bytes(A->d_soff, sizeof(long long) * (nch + 1)));
      d.push_back(fnv_bytes(A->d_slen, sizeof(int) * nl));
      d.push_back(fnv_bytes(A->d_scol, sizeof(int) * total));
      d.push_back(fnv_bytes(A->d_sval, sizeof(double) * total));
    }
    if (A->use_bsr3) {
      const size_t nch = (size_t)(A->b3_nbr + 63) / 64;
      long long slots = 0;
      MIG_HIP(hipMemcpy(&slots, A->d_b3off + nch, sizeof(long long), hipMemcpyDeviceToHost));
      num(A->b3_fixed_bytes);
      d.push_back(fnv_bytes(A->d_b3off, sizeof(long long) * (nch + 1)));
      d.push_back(fnv_bytes(A->d_b3len, sizeof(int) * A->b3_nbr));
      d.push_back(fnv_bytes(A->d_b3col, sizeof(int) * slots));
      d.push_back(fnv_bytes(A->d_b3val, sizeof(double) * 9 * slots));
      d.push_back(fnv_bytes(A->d_b3rest, sizeof(int) * A->n_b3rest));
    }
    if (A->use_tpl) {
      d.push_back((unsigned long long)A->tpl_ntpl << 40 | (unsigned long long)A->tpl_maxk << 20 |
                  (unsigned)A->tpl_nvals);
      d.push_back(fnv_bytes(A->d_tpl_id, (size_t)P));
      d.push_back(fnv_bytes(A->d_tpl_rec, sizeof(int) * 2 * (size_t)A->tpl_ntpl * A->tpl_maxk));
      d.push_back(fnv_bytes(A->d_tpl_val, sizeof(double) * A->tpl_nvals));
      d.push_back(fnv_bytes(A->d_tpl_rest, sizeof(int) * A->n_tpl_rest));
    }
    if (A->use_tpl3 || A->use_march)
      d.push_back(fnv_bytes(A->d_tpl3_grp, sizeof(unsigned long long) * A->tpl_ntpl * A->tpl3_G));
    if (A->use_march)
      d.push_back((unsigned long long)A->march.nxp << 32 | (unsigned)A->march.plane);
    d.push_back((unsigned long long)A->n_sel_int << 32 | (unsigned)A->n_sel_bnd);
    d.push_back(fnv_bytes(A->d_sel_int, sizeof(int) * A->n_sel_int));
    d.push_back(fnv_bytes(A->d_sel_bnd, sizeof(int) * A->n_sel_bnd));
    if (needed) *needed = (int)d.size();
    for (int i = 0; i < n && i < (int)d.size(); ++i) out[i] = d[(size_t)i];
  });
}
extern "C" int migmres_map_uniform(long long n_global, int nranks, int rank, long long *first,
                                   int *n_local) {
  return guard([&] {
    MIG_CHECK(nranks >= 1 && rank >= 0 && rank < nranks && n_global >= 0, "bad map arguments");
    uniform_map(n_global, nranks, rank, first, n_local);
  });
}

extern "C" int migmres_plan_colmap(long long n_global, int nranks, long long first, int n_local,
                                   const long long *rowptr, const long long *gcols,
                                   long long *colmap_out, int *n_cols) {
  return guard([&] {
    auto cm = make_colmap(n_global, nranks, first, n_local, rowptr, gcols);
    *n_cols = (int)cm.size();
    if (colmap_out) std::memcpy(colmap_out, cm.data(), sizeof(long long) * cm.size());
  });
}

extern "C" int migmres_plan_remotes(long long n_global, int nranks, long long first, int n_local,
                                    const long long *colmap, int n_cols, int *num_same,
                                    int *remote_lids, long long *remote_gids, int *remote_pids,
                                    int *n_remote) {
  return guard([&] {
    RemotePlan p = make_remotes(n_global, nranks, first, n_local, colmap, n_cols);
    *num_same = p.num_same;
    *n_remote = (int)p.remote_lids.size();
    for (size_t i = 0; i < p.remote_lids.size(); ++i) {
      if (remote_lids) remote_lids[i] = p.remote_lids[i];
      if (remote_gids) remote_gids[i] = p.remote_gids[i];
      if (remote_pids) remote_pids[i] = p.remote_pids[i];
    }
  });
}

extern "C" int migmres_plan_local_crs(long long first, int n_local, const long long *rowptr,
                                      const long long *gcols, const double *vals,
                                      const long long *colmap, int n_cols, int *lcols_out,
                                      double *vals_out) {
  return guard([&] {
    local_crs(n_local, rowptr, gcols, vals, colmap, n_cols, first, lcols_out, vals_out);
  });
}

extern "C" int migmres_plan_pairs(int n_local, const long long *rowptr, const int *xcols, int *ptr_out,
                                  int *key_out, unsigned short *meta_out, long long *nkeys, int *ok) {
  return guard([&] {
    MIG_CHECK(n_local >= 0 && rowptr && nkeys && ok, "plan_pairs: bad arguments");
    PairPlan pp;
    *ok = make_pair_plan(n_local, rowptr, xcols, pp) ? 1 : 0;
    *nkeys = *ok ? (long long)pp.key.size() : 0;
    if (!*ok) return;
    if (ptr_out) std::memcpy(ptr_out, pp.ptr.data(), sizeof(int) * pp.ptr.size());
    if (key_out) std::memcpy(key_out, pp.key.data(), sizeof(int) * pp.key.size());
    if (meta_out) std::memcpy(meta_out, pp.meta.data(), sizeof(unsigned short) * pp.meta.size());
  });
}

extern "C" int migmres_plan_pair_templates(int n_local, const long long *rowptr, const int *xcols, const double *vals,
                                           unsigned char *id_out, int *rec_out, double *vals_out, int *ntpl,
                                           int *maxk, int *nvals, int *ok) {
  return guard([&] {
    MIG_CHECK(n_local >= 0 && rowptr && ntpl && maxk && nvals && ok, "plan_pair_templates: bad arguments");
    PairTemplates pt;
    *ok = make_pair_templates(n_local, rowptr, xcols, vals, pt) ? 1 : 0;
    *ntpl = *ok ? pt.ntpl : 0;
    *maxk = *ok ? pt.maxk : 0;
    *nvals = *ok ? (int)pt.vals.size() : 0;
    if (!*ok) return;
    if (id_out) std::memcpy(id_out, pt.id.data(), pt.id.size());
    if (rec_out) std::memcpy(rec_out, pt.rec.data(), sizeof(int) * pt.rec.size());
    if (vals_out) std::memcpy(vals_out, pt.vals.data(), sizeof(double) * pt.vals.size());
  });
}

extern "C" int migmres_crs_create(migmres_ctx *ctx, long long n_global, long long first, int n_local,
                                  const long long *rowptr, const long long *gcols, const double *vals,
                                  migmres_crs **out) {
  return guard([&] { *out = crs_create(ctx, n_global, first, n_local, rowptr, gcols, vals); });
}

extern "C" int migmres_crs_create_device(migmres_ctx *ctx, long long n_global, long long first, int n_local,
                                         const long long *rowptr_dev, const long long *gcols_dev,
                                         const double *vals_dev, migmres_crs **out) {
  return guard([&] { *out = crs_create_device(ctx, n_global, first, n_local, rowptr_dev, gcols_dev, vals_dev); });
}

extern "C" int migmres_crs_create_galeri(migmres_ctx *ctx, const char *kind, int nx, int ny, int nz,
                                         migmres_crs **out) {
  return guard([&] {
    const std::string k(kind ? kind : "");
    const long long n_global = (long long)nx * ny * (k == "Laplace3D" || k == "Brick3D" ? nz : k == "FlanProxy" ? 3LL * nz : 1);
    long long first = 0;
    int n_local = 0;
    uniform_map(n_global, ctx->nranks, ctx->rank, &first, &n_local);
    std::vector<long long> rp, gc;
    std::vector<double> v;
    galeri_rows(k, nx, ny, nz, first, n_local, rp, gc, v);
    *out = crs_create(ctx, n_global, first, n_local, rp.data(), gc.data(), v.data());
  });
}

extern "C" int migmres_plan_galeri(const char *kind, int nx, int ny, int nz, long long first, int n_local,
                                   long long *rowptr_out, long long *gcols_out, double *vals_out,
                                   long long *nnz_out) {
  return guard([&] {
    MIG_CHECK(kind && nnz_out, "plan_galeri: null argument");
    std::vector<long long> rp, gc;
    std::vector<double> v;
    galeri_rows(kind, nx, ny, nz, first, n_local, rp, gc, v);
    *nnz_out = (long long)gc.size();
    if (rowptr_out) std::memcpy(rowptr_out, rp.data(), sizeof(long long) * rp.size());
    if (gcols_out) std::memcpy(gcols_out, gc.data(), sizeof(long long) * gc.size());
    if (vals_out) std::memcpy(vals_out, v.data(), sizeof(double) * v.size());
  });
}

extern "C" int migmres_crs_destroy(migmres_crs *A) {
  return guard([&] { delete A; });
}

extern "C" int migmres_crs_info(const migmres_crs *A, long long *n_global, long long *first,
                                int *n_local, int *n_cols, long long *nnz_local, int *n_remote,
                                int *n_export) {
  return guard([&] {
    if (n_global) *n_global = A->n_global;
    if (first) *first = A->first;
    if (n_local) *n_local = A->n_local;
    if (n_cols) *n_cols = A->n_cols;
    if (nnz_local) *nnz_local = A->nnz;
    if (n_remote) *n_remote = (int)A->plan.remote_lids.size();
    if (n_export) *n_export = (int)A->export_lids.size();
  });
}

extern "C" int migmres_crs_colmap(const migmres_crs *A, long long *out) {
  return guard([&] { std::memcpy(out, A->colmap.data(), sizeof(long long) * A->colmap.size()); });
}

extern "C" int migmres_crs_import_plan(const migmres_crs *A, int *export_lids, int *export_pids,
                                       int *remote_lids, int *remote_pids) {
  return guard([&] {
    for (size_t i = 0; i < A->export_lids.size(); ++i) {
      if (export_lids) export_lids[i] = A->export_lids[i];
      if (export_pids) export_pids[i] = A->export_pids[i];
    }
    for (size_t i = 0; i < A->plan.remote_lids.size(); ++i) {
      if (remote_lids) remote_lids[i] = A->plan.remote_lids[i];
      if (remote_pids) remote_pids[i] = A->plan.remote_pids[i];
    }
  });
}

extern "C" int migmres_crs_apply(migmres_crs *A, const migmres_mv *X, migmres_mv *Y, double alpha,
                                 double beta) {
  return guard([&] { crs_apply(*A, *X, *Y, alpha, beta); });
}
extern "C" int migmres_crs_apply_mode(migmres_crs *A, const migmres_mv *X, migmres_mv *Y, int mode, double alpha,
                                      double beta) {
  return guard([&] {
    MIG_CHECK(A && X && Y, "bad arguments");
    if (mode == MIGMRES_NO_TRANS)
      crs_apply(*A, *X, *Y, alpha, beta);
    else if (mode == MIGMRES_TRANS || mode == MIGMRES_CONJ_TRANS)  // real scalars: CONJ_TRANS = TRANS
      crs_apply_trans(*A, *X, *Y, alpha, beta);
    else
      throw Error(MIGMRES_EINVAL, "CRS apply: mode must be MIGMRES_NO_TRANS, MIGMRES_TRANS or MIGMRES_CONJ_TRANS");
  });
}

extern "C" int migmres_op_create(migmres_ctx *ctx, long long n_global, int n_local, migmres_apply_fn fn, void *user,
                                 migmres_op **out) {
  return guard([&] {
    MIG_CHECK(ctx && fn && out && n_local >= 0, "op_create: bad arguments");
    auto *op = new migmres_op();
    op->ctx = ctx;
    op->n_global = n_global;
    op->n_local = n_local;
    op->fn = fn;
    op->user = user;
    *out = op;
  });
}
extern "C" int migmres_op_from_crs(migmres_crs *A, migmres_op **out) {
  return guard([&] {
    MIG_CHECK(A && out, "op_from_crs: bad arguments");
    auto *op = new migmres_op();
    op->ctx = A->ctx;
    op->n_global = A->n_global;
    op->n_local = A->n_local;
    op->crs = A;
    *out = op;
  });
}
extern "C" int migmres_op_apply(migmres_op *op, const migmres_mv *X, migmres_mv *Y) {
  return guard([&] {
    MIG_CHECK(op && X && Y, "op_apply: bad arguments");
    op_apply(*op, *X, *Y);
  });
}
extern "C" int migmres_op_destroy(migmres_op *op) {
  return guard([&] { delete op; });
}

extern "C" int migmres_mv_create(migmres_ctx *ctx, long long n_global, int n_local, int ncols,
                                 migmres_mv **out) {
  return guard([&] { *out = mv_create(ctx, n_global, n_local, ncols); });
}
extern "C" int migmres_mv_view(migmres_mv *parent, const int *idx, int n, migmres_mv **out) {
  return guard([&] { *out = mv_view(parent, idx, n); });
}
extern "C" int migmres_mv_view_range(migmres_mv *parent, int first, int n, migmres_mv **out) {
  return guard([&] {
    MIG_CHECK(first >= 0 && n >= 0 && first + n <= parent->ncols, "range out of bounds");
    *out = mv_view_range(parent, first, n);
  });
}
extern "C" int migmres_mv_destroy(migmres_mv *mv) {
  return guard([&] { delete mv; });
}
extern "C" int migmres_mv_shape(const migmres_mv *mv, long long *n_global, int *n_local, int *ncols,
                                int *constant_stride) {
  return guard([&] {
    if (n_global) *n_global = mv->n_global;
    if (n_local) *n_local = mv->n_local;
    if (ncols) *ncols = mv->ncols;
    if (constant_stride) *constant_stride = mv->contiguous() ? 1 : 0;
  });
}
extern "C" int migmres_mv_upload(migmres_mv *mv, const double *host, long long ld) {
  return guard([&] {
    MIG_CHECK(ld >= mv->n_local, "host leading dimension too small");
    hipStream_t s = mv->ctx->stream;
    for (int c = 0; c < mv->ncols; ++c)
      MIG_HIP(hipMemcpyAsync(mv->base + mv->col_offset(c), host + (size_t)c * ld,
                             sizeof(double) * mv->n_local, hipMemcpyHostToDevice, s));
    MIG_HIP(hipStreamSynchronize(s));
  });
}
extern "C" int migmres_mv_download(const migmres_mv *mv, double *host, long long ld) {
  return guard([&] {
    MIG_CHECK(ld >= mv->n_local, "host leading dimension too small");
    hipStream_t s = mv->ctx->stream;
    for (int c = 0; c < mv->ncols; ++c)
      MIG_HIP(hipMemcpyAsync(host + (size_t)c * ld, mv->base + mv->col_offset(c),
                             sizeof(double) * mv->n_local, hipMemcpyDeviceToHost, s));
    MIG_HIP(hipStreamSynchronize(s));
  });
}
extern "C" int migmres_mv_times_mat_add_mv(double alpha, const migmres_mv *A, const double *B, int ldb,
                                           double beta, migmres_mv *mv) {
  return guard([&] { mv_times_mat_add_mv(alpha, *A, B, ldb, beta, *mv); });
}
extern "C" int migmres_mv_add_mv(double alpha, const migmres_mv *A, double beta, const migmres_mv *B,
                                 migmres_mv *mv) {
  return guard([&] { mv_add_mv(alpha, *A, beta, *B, *mv); });
}
extern "C" int migmres_mv_scale(migmres_mv *mv, double alpha) {
  return guard([&] { mv_scale(*mv, alpha); });
}
extern "C" int migmres_mv_scale_vec(migmres_mv *mv, const double *alphas) {
  return guard([&] { mv_scale_vec(*mv, alphas); });
}
extern "C" int migmres_mv_trans_mv(double alpha, const migmres_mv *A, const migmres_mv *B, double *C,
                                   int ldc) {
  return guard([&] { mv_trans_mv(alpha, *A, *B, C, ldc); });
}
extern "C" int migmres_mv_dot(const migmres_mv *A, const migmres_mv *B, double *out) {
  return guard([&] { mv_dot(*A, *B, out); });
}
extern "C" int migmres_mv_norm(const migmres_mv *mv, double *out, int norm_type) {
  return guard([&] { mv_norm(*mv, out, norm_type); });
}
extern "C" int migmres_mv_init(migmres_mv *mv, double alpha) {
  return guard([&] { mv_init(*mv, alpha); });
}
extern "C" int migmres_mv_random(migmres_mv *mv, unsigned int *seed) {
  return guard([&] { mv_random(*mv, seed); });
}
extern "C" int migmres_mv_assign(const migmres_mv *A, migmres_mv *mv) {
  return guard([&] { mv_assign(*A, *mv); });
}
extern "C" int migmres_mv_set_block(const migmres_mv *A, const int *idx, int n, migmres_mv *mv) {
  return guard([&] {
    // BelosEpetraAdapter.hpp:894-940: A may have more columns than indices (its first n are
    // copied), not fewer.
    MIG_CHECK(n <= A->ncols, "SetBlock: A has fewer columns than there are indices");
    migmres_mv *v = mv_view(mv, idx, n);
    migmres_mv *a = nullptr;
    try {
      a = n == A->ncols ? nullptr : mv_view_range(const_cast<migmres_mv *>(A), 0, n);
      mv_assign(a ? *a : *A, *v);
      MIG_HIP(hipStreamSynchronize(mv->ctx->stream));
    } catch (...) {
      delete a;
      delete v;
      throw;
    }
    delete a;
    delete v;
  });
}
