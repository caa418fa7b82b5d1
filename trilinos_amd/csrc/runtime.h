// Host runtime objects behind the C ABI: context (device, stream, RCCL communicator,
// scratch), multivectors, the distributed CRS operator and the MultiVecTraits operations.
#pragma once

#include <rccl/rccl.h>

#include <memory>
#include <string>
#include <vector>

#include "internal.h"
#include "plan.h"

// Per-kernel-class profiling with HIP events on the context stream (bench.py roofline).
// K_HALO (halo stream: pack, exchange, unpack) and K_ALLREDUCE (RCCL all-reduce on the
// context stream) are communication classes: their bytes are the message payload.
enum KernelClass { K_SPMM = 0, K_GEMM_TN, K_REDUCE, K_GEMM_NN, K_COLDOT, K_AXPBY, K_SCALE, K_FILL,
                   K_COPY, K_RANDOM, K_PACK, K_FB, K_GEMM_NN_DOT, K_NN_TN, K_HALO, K_ALLREDUCE,
                   K_NUM_CLASSES };
extern const char *kKernelClassNames[K_NUM_CLASSES];

struct migmres_ctx;
namespace migmres {
struct LoopGroup;
}
struct ProfScope {
  migmres_ctx *c;
  int cls;
  double bytes;
  hipEvent_t a = nullptr, b = nullptr;
  hipStream_t s = nullptr;
  ProfScope(migmres_ctx *ctx, int cls, double bytes, hipStream_t stream = nullptr);
  ~ProfScope();
};

struct migmres_ctx {
  int device = 0, rank = 0, nranks = 1;
  // the distributed code paths are on: nranks > 1, or one rank with a real RCCL communicator
  // (MIGMRES_FORCE_RCCL=1 at creation: every all-reduce and the import-plan exchange go
  // through RCCL with a communicator of one, which tests the RCCL transport on one GPU)
  bool dist = false;
  // profiling state
  bool prof_on = false;
  struct Pending {
    int cls;
    double bytes;
    hipEvent_t a, b;
  };
  std::vector<Pending> pending;
  std::vector<hipEvent_t> event_pool;
  double prof_ms[K_NUM_CLASSES] = {};
  double prof_bytes[K_NUM_CLASSES] = {};
  long long prof_count[K_NUM_CLASSES] = {};
  hipEvent_t get_event();
  void prof_collect();
  // Caching device allocator: freed blocks are kept per (rounded) size and reused, so the
  // multi-GB Krylov basis is not re-mapped on every solve.
  std::vector<std::pair<size_t, void *>> pool;
  size_t pool_bytes = 0;
  void *dev_alloc(size_t bytes, size_t *rounded);
  void dev_free(void *p, size_t rounded);
  void pool_trim();
  hipStream_t stream = nullptr;
  // second stream for the halo exchange (nranks > 1): pack + RCCL point-to-point run there
  // while the interior rows' SpMM runs on `stream` (events order the two)
  hipStream_t halo_stream = nullptr;
  hipEvent_t ev_main = nullptr, ev_halo = nullptr;
  hipStream_t p2p_stream = nullptr;  // stream of the open p2p group
  ncclComm_t comm = nullptr;
  // In-process multi-rank emulation for tests (all ranks' contexts in one process on one
  // device, one host thread per rank; selected by a "MIGLOOP1" unique id): collectives and
  // point-to-point messages go through host mailboxes instead of RCCL.  See runtime.cpp.
  std::shared_ptr<migmres::LoopGroup> loop;
  struct P2p {
    void *buf;
    size_t bytes;
    int peer;
  };
  std::vector<P2p> p2p_sends, p2p_recvs;
  // grouped point-to-point exchange (ncclGroupStart/Send/Recv/GroupEnd on the stream)
  void p2p_begin(hipStream_t s = nullptr);  // default: the context stream
  void p2p_send(const void *buf, size_t bytes, int peer);
  void p2p_recv(void *buf, size_t bytes, int peer);
  void p2p_end();
  // device scratch: per-workgroup partials, reduced results, staged coefficients
  double *d_partial = nullptr;
  size_t partial_cap = 0;
  double *d_red = nullptr;
  size_t red_cap = 0;
  double *d_coef = nullptr;
  size_t coef_cap = 0;
  double *h_pinned = nullptr;
  size_t pinned_cap = 0;
  double comm_seconds = 0.0;

  double *partial(size_t n);
  double *red(size_t n);
  double *coef(size_t n);
  double *pinned(size_t n);
  // In-place sum (or max) all-reduce of n device doubles on the context stream.
  void allreduce(double *d, size_t n, bool max = false);
  // Stream-ordered sum all-reduce (no host synchronisation).
  void allreduce_async(double *d, size_t n);
};

struct migmres_mv {
  migmres_ctx *ctx = nullptr;
  size_t alloc_bytes = 0;
  long long n_global = 0;
  int n_local = 0;
  int ncols = 0;
  long long ld = 0;
  double *base = nullptr;
  bool owner = false;
  std::vector<int> cols;  // column offsets relative to base (empty: contiguous)
  int *d_cols = nullptr;

  migmres::MvDesc desc() const { return migmres::MvDesc{base, ld, d_cols, ncols}; }
  bool contiguous() const { return cols.empty(); }
  long long col_offset(int c) const { return (long long)(cols.empty() ? c : cols[(size_t)c]) * ld; }
  ~migmres_mv();
};

struct migmres_crs {
  migmres_ctx *ctx = nullptr;
  long long n_global = 0, first = 0, nnz = 0;
  int n_local = 0, n_cols = 0;
  std::vector<long long> colmap;
  migmres::RemotePlan plan;
  std::vector<int> export_lids, export_pids;
  struct Nbr {
    int pid, offset, count;
  };
  std::vector<Nbr> recv_nbrs, send_nbrs;
  int *d_rowptr = nullptr, *d_cols = nullptr, *d_export = nullptr;
  // (offset, count) of each export / remote entry's neighbour group: the exchange buffers are
  // laid out [neighbour][column][count], one message per neighbour (launch_pack / unpack)
  int2 *d_export_grp = nullptr, *d_remote_grp = nullptr;
  double *d_vals = nullptr;  // padded by 8 zero entries (row-pair kernel reads 8 per row)
  // row-pair gather plan (k_spmm_pair); null when the matrix does not fit it
  double *d_psv = nullptr;  // SELL-64 layout of the pair plan (make_pair_sell)
  int *d_psk = nullptr;
  unsigned short *d_psm = nullptr;
  bool use_pairs = false;
  int pair_max_keys = 0, pair_rmax = 0;
  // SELL-64 copy for the general kernel (k_spmm_sell) when the pair plan does not apply
  long long *d_soff = nullptr;
  int *d_slen = nullptr, *d_scol = nullptr;
  double *d_sval = nullptr;
  bool use_sell = false;
  double *d_xr = nullptr;
  // 3 x 3 block rows (make_bsr3) next to the SELL copy, which keeps the rest rows
  long long *d_b3off = nullptr;
  int *d_b3len = nullptr, *d_b3col = nullptr, *d_b3rest = nullptr;
  double *d_b3val = nullptr;
  int b3_nbr = 0, n_b3rest = 0;
  double b3_fixed_bytes = 0.0;
  bool use_bsr3 = false;  // SELL: row-interleaved copy of X's owned rows (n_local x 8), on first apply with k >= 2
  // row-pair templates (k_spmm_tpl) when the pairs repeat a few shapes: templated pairs run
  // there (reading no ghost column, they also make the interior half of the halo overlap);
  // the rest -- pairs that read a ghost column -- go to the kernel above through
  // d_tpl_rest (its units: pairs for the pair kernel, rows otherwise)
  unsigned char *d_tpl_id = nullptr;
  int2 *d_tpl_rec = nullptr;
  double *d_tpl_val = nullptr;
  int tpl_ntpl = 0, tpl_maxk = 0, tpl_nvals = 0;
  bool use_tpl = false;
  int tpl_host_fallbacks = 0;  // device template plans rebuilt on the host after a shape-hash collision
  int *d_tpl_rest = nullptr;
  // stencil-group form of the templates (k_spmm_tpl3: one X load per key triple, the
  // neighbours' halves by DPP lane shifts) when the keys come in x-neighbour triples
  unsigned long long *d_tpl3_grp = nullptr;
  std::vector<int> tpl3_center;
  int tpl3_G = 0;
  bool use_tpl3 = false;
  int tpl3_slabs = 0, tpl3_kc = 8;  // walk order (XCD slabs) and columns per launch (tuning)
  // the same groups as a 2.5-D plane march (k_spmm_march) when they have a 3-D grid geometry
  // that every templated pair fits (make_march_geometry + march_check)
  migmres::MarchGeom march;
  bool use_march = false;
  bool use_march7 = false;  // the 7-point specialisation (k_spmm_march7)
  bool use_march27 = false;  // the uniform 27-point specialisation (k_spmm_march27)
  bool march_uni7 = false;   // k_spmm_march7 with the uniform coefficient table (no per-lane coefficients)
  migmres::March27Coef march27_coef{};
  int march_kc = 2, march_sz = 0, march_pd = 1, march_nl = 1;  // columns per staged plane, planes per slab (0: auto), planes prefetched
  int tpl_slabs = 0, tpl_kc = 8;
  int n_tpl_rest = 0;
  double spmm_fixed_bytes = 0.0;  // matrix-format bytes one apply reads (bench accounting)
  // interior / boundary split (units = pairs with the row-pair kernel, else rows): interior
  // units read no ghost column and run while the halo exchange is in flight
  int *d_sel_int = nullptr, *d_sel_bnd = nullptr;
  int n_sel_int = 0, n_sel_bnd = 0;
  double *d_send = nullptr, *d_recv = nullptr, *d_ghost = nullptr;
  long long ldg = 0;  // ghost block leading dimension: n_remote rounded up to even, padding zero
  int halo_k = 0;
  // A^T (transposed apply): the local transpose in GeneralMTM's order (dev_transpose), built on
  // the first transposed apply; with a halo the product goes to d_tbuf (owned + ghost rows, leading
  // dimension ld_t), whose ghost rows travel back to their owners (d_tsend -> d_trecv)
  int *d_trowptr = nullptr, *d_tcols = nullptr, *d_tiota = nullptr;
  double *d_tvals = nullptr, *d_tbuf = nullptr, *d_tsend = nullptr, *d_trecv = nullptr;
  long long ld_t = 0;
  int tr_k = 0;
  ~migmres_crs();
};

// An operator given by a host callback (migmres_op_create) or wrapping a CRS (op_from_crs).
struct migmres_op {
  migmres_ctx *ctx = nullptr;
  long long n_global = 0;
  int n_local = 0;
  migmres_apply_fn fn = nullptr;
  void *user = nullptr;
  migmres_crs *crs = nullptr;  // borrowed
};

// Point-Jacobi preconditioner (Ifpack2::Relaxation "Jacobi"): Y = M X with `sweeps`
// sweeps from a zero start, damping `damping`; or (kind 1) the Chebyshev smoother
// (Ifpack2::Chebyshev) -- see prec.cpp.
struct migmres_prec {
  migmres_ctx *ctx = nullptr;
  migmres_crs *A = nullptr;
  double *d_dinv = nullptr;
  double *d_sdinv = nullptr;  // omega * dinv (+2 zero entries): the fused form's column scale
  double *d_gsdinv = nullptr; // the owners' omega * dinv of A's ghost columns (halo; ldg + 2, zero padded)
  int sweeps = 1;
  double damping = 1.0;
  long long n_apply = 0;
  migmres_mv *work = nullptr;   // residual scratch for sweeps > 1
  migmres_mv *xcopy = nullptr;  // deep copy of X when apply(X, Y) aliases
  // kind 1: Ifpack2::Chebyshev (prec.cpp); d_dinv holds the reciprocal_threshold diagonal
  int kind = 0;
  int rtype = 0;            // kind 0: 0 Jacobi, 1 Richardson (no diagonal)
  bool zero_start = true;   // "relaxation: zero starting solution"
  migmres_chebyshev_params cheb{};
  double cheb_computed_lmax = 0.0, cheb_lmax = 0.0, cheb_lmin = 0.0, cheb_ratio = 0.0;
  migmres_mv *cheb_w = nullptr, *cheb_p = nullptr;  // W (and the textbook form's P)
  migmres_op *uop = nullptr;  // kind 2: a user operator (borrowed; A is null)
  int n_local() const { return uop ? uop->n_local : A->n_local; }
  ~migmres_prec();
};

namespace migmres {

void prec_apply(migmres_prec &M, const migmres_mv &X, migmres_mv &Y);
// Y = op(X): the CRS apply, or the user callback (a nonzero return throws MIGMRES_EOP)
void op_apply(migmres_op &op, const migmres_mv &X, migmres_mv &Y);

migmres_mv *mv_create(migmres_ctx *ctx, long long n_global, int n_local, int ncols);
migmres_mv *mv_view(migmres_mv *parent, const int *idx, int n);
migmres_mv *mv_view_range(migmres_mv *parent, int first, int n);

// Belos::MultiVecTraits operations (device data, host coefficient matrices).
void mv_times_mat_add_mv(double alpha, const migmres_mv &A, const double *B, int ldb, double beta,
                         migmres_mv &Y);
void mv_add_mv(double alpha, const migmres_mv &A, double beta, const migmres_mv &B, migmres_mv &Y);
void mv_scale(migmres_mv &Y, double alpha);
void mv_scale_vec(migmres_mv &Y, const double *alphas);
void mv_trans_mv(double alpha, const migmres_mv &A, const migmres_mv &B, double *C, int ldc);
void mv_dot(const migmres_mv &A, const migmres_mv &B, double *out);
void mv_norm(const migmres_mv &A, double *out, int type);
void mv_init(migmres_mv &Y, double alpha);
void mv_random(migmres_mv &Y, unsigned int *seed);
void mv_assign(const migmres_mv &A, migmres_mv &Y);
// do any columns of X and Y share memory?
bool mv_overlap(const migmres_mv &X, const migmres_mv &Y);

migmres_crs *crs_create(migmres_ctx *ctx, long long n_global, long long first, int n_local,
                        const long long *rowptr, const long long *gcols, const double *vals);
// The same operator from a CSR that is already in device memory (global column ids,
// insertion order; rowptr int64): FillComplete's index maps built on the device
// (fillcomplete.hip), identical to crs_create's.
migmres_crs *crs_create_device(migmres_ctx *ctx, long long n_global, long long first, int n_local,
                               const long long *d_rowptr, const long long *d_gcols, const double *d_vals);
void fill_complete_device(migmres_crs *A, const long long *d_rowptr, const long long *d_gcols, const double *d_vals,
                          std::vector<long long> &rowptr, std::vector<int> &lcols, std::vector<double> &lvals);
// Y = alpha*A*X + beta*Y including the halo import.
void crs_apply(migmres_crs &A, const migmres_mv &X, migmres_mv &Y, double alpha, double beta);
// Y = alpha*A^T*X + beta*Y (Tpetra apply mode TRANS; Epetra Multiply(TransA = true) at alpha 1,
// beta 0): GeneralMTM's scatter order per row, ghost-column contributions exported back to their
// owners and added in ascending neighbour order.
void crs_apply_trans(migmres_crs &A, const migmres_mv &X, migmres_mv &Y, double alpha, double beta);
// Right Jacobi fused into the operator: Y = A (M X) with M = Ifpack2 Jacobi, one sweep from
// zero, formed operand by operand inside the template SpMM -- bit-identical to prec_apply
// followed by crs_apply.  Only where every row pair is templated and no halo is needed;
// returns false (nothing done) otherwise.
bool crs_apply_jacobi_fused(migmres_crs &A, const migmres_prec &M, const migmres_mv &X, migmres_mv &Y);
void prec_import_ghost_scale(migmres_prec &M);

}  // namespace migmres
