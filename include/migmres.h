/*
 * migmres.h -- C ABI of the MI355X-native Block GMRES hot path.
 *
 * This is the drop-in boundary between a Belos driver (Belos::MultiVecTraits /
 * Belos::OperatorTraits / Belos::SolverManager, or the Python mirror in
 * trilinos_amd/) and the HIP kernels.  Every entry point is plain C: opaque
 * handles, raw pointers, sizes; no torch or C++ types cross it.
 *
 * Reference interfaces each group replaces (paths under /root/reference/packages):
 *   context      Epetra_Comm / Epetra_MpiComm::SumAll        epetra/src/Epetra_MpiComm.cpp:123-127
 *   map          Epetra_BlockMap::ConstructAutoUniform        epetra/src/Epetra_BlockMap.cpp:60-107
 *   crs          Epetra_CrsMatrix::FillComplete/Multiply      epetra/src/Epetra_CrsMatrix.cpp:1147-1199, 3107-3285
 *                Epetra_CrsGraph::MakeColMap_int              epetra/src/Epetra_CrsGraph.cpp:1348-1524
 *                Epetra_Import::Construct                     epetra/src/Epetra_Import.cpp:292-460
 *                Tpetra::CrsMatrix::apply                     tpetra/core/src/Tpetra_CrsMatrix_def.hpp:5176-5208
 *   mv           Belos::MultiVecTraits<double,Epetra_MultiVector>
 *                                                             belos/epetra/src/BelosEpetraAdapter.hpp:447-1064
 *   icgs         Belos::ICGSOrthoManager::projectAndNormalize / normalize
 *                                                             belos/src/BelosICGSOrthoManager.hpp:646-839
 *   solver       Belos::BlockGmresSolMgr (setParameters/solve/getNumIters/achievedTol/isLOADetected)
 *                                                             belos/src/BelosBlockGmresSolMgr.hpp:494-803, 916-1303
 *
 * Conventions
 *   - Return 0 on success, a negative code on error (Epetra's EPETRA_CHK_ERR style);
 *     migmres_last_error() returns a thread-local message for the last failure.
 *   - Dense coefficient matrices cross the ABI as host, column-major arrays with a
 *     leading dimension (Teuchos::SerialDenseMatrix layout).
 *   - Calls that return host data (transmv, dot, norm, icgs rank, solve) block until the
 *     device work and any cross-GPU reduction finished; others are stream-ordered.
 *   - A context is not thread-safe (Belos is single-threaded per rank).
 */
#ifndef MIGMRES_H
#define MIGMRES_H

#ifdef __cplusplus
extern "C" {
#endif

#define MIGMRES_ABI_VERSION 1

typedef struct migmres_ctx migmres_ctx;
typedef struct migmres_crs migmres_crs;
typedef struct migmres_mv migmres_mv;
typedef struct migmres_solver migmres_solver;
typedef struct migmres_prec migmres_prec;
typedef struct migmres_op migmres_op;

/* error codes */
#define MIGMRES_OK 0
#define MIGMRES_EINVAL -1
#define MIGMRES_EHIP -2
#define MIGMRES_ERCCL -3
#define MIGMRES_ENOMEM -4
#define MIGMRES_ESTATE -5
#define MIGMRES_EOP -6 /* a user operator's callback returned nonzero */

/* norm types (Belos::NormType, belos/src/BelosTypes.hpp) */
#define MIGMRES_ONE_NORM 0
#define MIGMRES_TWO_NORM 1
#define MIGMRES_INF_NORM 2

int migmres_abi_version(void);
const char *migmres_last_error(void);

/* ---------------- context (replaces Epetra_Comm + the MPI backend) ---------------- */

/* 128-byte RCCL unique id, generated on rank 0 and broadcast by the caller. */
int migmres_comm_unique_id(unsigned char out[128]);
/* ncclGetVersion of the RCCL this library is bound to (e.g. 22707 for 2.27.7). */
int migmres_rccl_version(int *version);
/* nranks == 1: uid may be NULL and no communicator is created.  For nranks > 1 the
 * communicator set-up (ncclCommInitRank) is guarded by a watchdog: if it has not returned
 * after MIGMRES_RCCL_INIT_TIMEOUT seconds (default 600; 0 = no watchdog) -- a peer rank
 * died or never arrived -- the process prints the reason and exits with status 75, so a
 * launcher sees a failed rank instead of a hang. */
int migmres_ctx_create(int device, int rank, int nranks, const unsigned char *uid, migmres_ctx **out);
int migmres_ctx_destroy(migmres_ctx *ctx);
int migmres_ctx_sync(migmres_ctx *ctx);
int migmres_ctx_rank(const migmres_ctx *ctx, int *rank, int *nranks);
/* Sum-all of n host doubles across ranks (Epetra_Comm::SumAll). */
int migmres_ctx_sum_all(migmres_ctx *ctx, const double *in, double *out, int n);

/* Kernel profiling with HIP events on the context stream: per kernel class the summed
 * device milliseconds, ALGORITHMIC bytes (the traffic model of DESIGN.md) and launch
 * count.  Enabling resets the counters.  Class names: migmres_kernel_class_name(i). */
int migmres_ctx_profile(migmres_ctx *ctx, int on);
int migmres_ctx_profile_read(migmres_ctx *ctx, double *ms, double *bytes, long long *launches, int n);
const char *migmres_kernel_class_name(int i);

/* ---------------- maps and import plans (host only, no GPU needed) ---------------- */

/* Epetra_BlockMap::ConstructAutoUniform: first global id and local length of `rank`. */
int migmres_map_uniform(long long n_global, int nranks, int rank, long long *first, int *n_local);

/* Epetra_CrsGraph::MakeColMap_int for one rank.  rowptr[n_local+1], gcols in insertion
 * order.  colmap_out must hold n_local + (number of distinct remote columns) entries;
 * *n_cols returns the count.  Pass colmap_out == NULL to query the size. */
int migmres_plan_colmap(long long n_global, int nranks, long long first, int n_local,
                        const long long *rowptr, const long long *gcols,
                        long long *colmap_out, int *n_cols);

/* Remote part of Epetra_Import::Construct for one rank: given the column map, the
 * remote LIDs / GIDs / owner PIDs sorted by PID (Epetra_Util::Sort). Arrays sized
 * n_cols; *n_remote and *num_same returned. */
int migmres_plan_remotes(long long n_global, int nranks, long long first, int n_local,
                         const long long *colmap, int n_cols, int *num_same,
                         int *remote_lids, long long *remote_gids, int *remote_pids, int *n_remote);

/* Local CRS after MakeIndicesLocal + SortEntries: lcols/vals out sized rowptr[n_local]. */
int migmres_plan_local_crs(long long first, int n_local, const long long *rowptr,
                           const long long *gcols, const double *vals, const long long *colmap,
                           int n_cols, int *lcols_out, double *vals_out);

/* Row-pair gather plan of the SpMM kernel (no reference counterpart: a device layout
 * derived from the local CRS).  xcols are X-space columns (owned column -> local row,
 * remote -> n_local + ghost slot), rows sorted ascending.  Writes ptr[(n_local+1)/2 + 1],
 * key[*nkeys] and meta[*nkeys] (pass NULL outputs to query *nkeys; *ok = 0 when the matrix
 * does not fit the plan and the row-per-thread kernel is used instead). */
int migmres_plan_pairs(int n_local, const long long *rowptr, const int *xcols, int *ptr_out,
                       int *key_out, unsigned short *meta_out, long long *nkeys, int *ok);
/* The row-pair template form of the same X-space CSR (k_spmm_tpl): per pair a template id
 * (255: the pair reads a ghost column), per template maxk key records (offset from the pair,
 * four value-dictionary slots packed in bytes: row 0 low, row 0 high, row 1 low, row 1 high,
 * 255 = none) and the value dictionary.  *ok = 0 when the rows do not repeat few enough
 * shapes.  Pass null outputs to get the sizes: id (n_local+1)/2 bytes, rec 2*ntpl*maxk ints,
 * vals nvals doubles. */
int migmres_plan_pair_templates(int n_local, const long long *rowptr, const int *xcols, const double *vals,
                                unsigned char *id_out, int *rec_out, double *vals_out, int *ntpl, int *maxk,
                                int *nvals, int *ok);

/* ---------------- CRS operator (Epetra_CrsMatrix / Tpetra::CrsMatrix) ---------------- */

/* Collective over the context's ranks: builds the column map, local indices, the
 * import plan (exchanging remote-id lists) and uploads the operator. */
int migmres_crs_create(migmres_ctx *ctx, long long n_global, long long first, int n_local,
                       const long long *rowptr, const long long *gcols, const double *vals,
                       migmres_crs **out);
/* The same operator from a CSR already in device memory (rowptr_dev: n_local+1 int64 offsets,
 * gcols_dev: int64 global column ids in insertion order, vals_dev: doubles; all on the
 * context's device, read only): FillComplete's column map, local ids, sorted rows and the
 * import's remote lists are built on the device (replaces Epetra_CrsGraph::MakeColMap_int,
 * epetra/src/Epetra_CrsGraph.cpp:1348-1524; MakeIndicesLocal + SortEntries,
 * Epetra_CrsMatrix.cpp:1147-1199) and equal migmres_crs_create's.  Rows must not repeat a
 * column (merge duplicates first, as the file readers do). */
int migmres_crs_create_device(migmres_ctx *ctx, long long n_global, long long first, int n_local,
                              const long long *rowptr_dev, const long long *gcols_dev, const double *vals_dev,
                              migmres_crs **out);
/* Galeri generators built natively on the host of each rank ("Laplace2D", "Laplace3D",
 * "Brick3D" = the 27-point Xpetra Brick3D with a = 26, b..g = -1); nz ignored for 2-D.
 * "FlanProxy" (not Galeri: a synthetic stand-in of SuiteSparse Flan_1565, 3 dofs per node of
 * an nx x ny x nz node grid, ~73 nnz per row, scrambled numbering, nx odd) has 3 nx ny nz rows. */
int migmres_crs_create_galeri(migmres_ctx *ctx, const char *kind, int nx, int ny, int nz,
                              migmres_crs **out);
/* The same generator on the host only: rows [first, first+n_local) with GLOBAL columns in
 * insertion order.  *nnz_out always set; the arrays are filled when non-NULL (rowptr_out
 * n_local+1 entries, gcols_out / vals_out *nnz_out entries). */
int migmres_plan_galeri(const char *kind, int nx, int ny, int nz, long long first, int n_local,
                        long long *rowptr_out, long long *gcols_out, double *vals_out, long long *nnz_out);
/* Matrix ingestion from a file (format detected from the first line):
 *   MatrixMarket "coordinate" real/integer/pattern, general/symmetric/skew-symmetric --
 *     replaces Tpetra::MatrixMarket::Reader<CrsMatrix>::readSparseFile
 *     (tpetra/core/inout/MatrixMarket_Tpetra.hpp); symmetric storage expanded, duplicate
 *     entries summed;
 *   Harwell-Boeing RUA/RSA -- replaces Trilinos_Util_read_hb + the matrix part of
 *     Belos::Util::createEpetraProblem (triutils/src/Trilinos_Util_read_hb.cpp,
 *     belos/epetra/src/BelosEpetraUtils.cpp:81-160): every row carries an explicit diagonal
 *     (MSR storage), symmetric storage expanded.
 * crs_read_file is collective: each rank parses the file and keeps its rows of the uniform
 * row map (Epetra_BlockMap::ConstructAutoUniform).  file_rows is the host-only form for
 * rows [first, first+n_local), GLOBAL columns in insertion order (*nnz_out always set;
 * arrays filled when non-NULL, as migmres_plan_galeri). */
int migmres_matrix_file_info(const char *path, long long *n_global, long long *nnz_file, int *symmetric);
int migmres_matrix_file_rows(const char *path, long long first, int n_local, long long *rowptr_out,
                             long long *gcols_out, double *vals_out, long long *nnz_out);
int migmres_crs_read_file(migmres_ctx *ctx, const char *path, migmres_crs **out);
int migmres_crs_destroy(migmres_crs *A);
int migmres_crs_info(const migmres_crs *A, long long *n_global, long long *first, int *n_local,
                     int *n_cols, long long *nnz_local, int *n_remote, int *n_export);
int migmres_crs_colmap(const migmres_crs *A, long long *colmap_out);
/* Export list (ExportLIDs, ExportPIDs) and remote list (RemoteLIDs) of the import plan. */
int migmres_crs_import_plan(const migmres_crs *A, int *export_lids, int *export_pids,
                            int *remote_lids, int *remote_pids);
/* OperatorTraits::Apply / Tpetra apply: Y = alpha*A*X + beta*Y (beta==0 ignores Y). */
int migmres_crs_apply(migmres_crs *A, const migmres_mv *X, migmres_mv *Y, double alpha, double beta);
/* Tpetra::CrsMatrix::apply(X, Y, mode, alpha, beta) (tpetra/core/src/Tpetra_CrsMatrix_def.hpp:
 * 5176-5208) / Epetra_CrsMatrix::Multiply(TransA, X, Y) (epetra/src/Epetra_CrsMatrix.cpp:
 * 3107-3285) with the transpose: Y = alpha*A^T*X + beta*Y.  A^T runs GeneralMTM's scatter order
 * (:3587-3650: y = 0, then row by row y[col] += v*x[row]) as a row kernel over a transpose built
 * on the device at the first call; on several ranks the contributions to ghost columns go back
 * to their owners (Epetra_Export, combine Add), added in ascending PID order, then alpha and
 * beta are applied (alpha 1, beta 0 = Epetra's Multiply(true, ...) bit for bit).  X and Y may
 * not alias (Tpetra localApply's check).  OperatorTraits::HasApplyTranspose = true. */
#define MIGMRES_NO_TRANS 0
#define MIGMRES_TRANS 1
#define MIGMRES_CONJ_TRANS 2
int migmres_crs_apply_mode(migmres_crs *A, const migmres_mv *X, migmres_mv *Y, int mode, double alpha,
                           double beta);
/* Which SpMM kernel apply() runs for this operator (chosen at creation from the local rows):
 * MIGMRES_SPMM_CSR thread per row over the CSR, MIGMRES_SPMM_PAIR row pairs with 16-byte X
 * loads (rows of <= 8 entries), MIGMRES_SPMM_SELL thread per row over a SELL-64 copy,
 * MIGMRES_SPMM_TPL row pairs read through a few repeated pair templates (one byte per pair;
 * stencil operators), the pairs that read ghost columns through one of the others.
 * MIGMRES_NO_TPL_SPMM=1 / MIGMRES_NO_PAIR_SPMM=1 / MIGMRES_NO_SELL_SPMM=1 in the environment
 * at creation switch the respective format off.  Every kernel is bit-identical. */
#define MIGMRES_SPMM_CSR 0
#define MIGMRES_SPMM_PAIR 1
#define MIGMRES_SPMM_SELL 2
#define MIGMRES_SPMM_TPL 3
/* MIGMRES_SPMM_TPL3: the template form of 27-point stencils on an even-nx grid, read with one X
 * load per x-neighbour triple and the neighbours' halves taken from adjacent lanes
 * (MIGMRES_NO_TPL3=1 at creation keeps MIGMRES_SPMM_TPL). */
#define MIGMRES_SPMM_TPL3 4
/* MIGMRES_SPMM_BSR3: 3 x 3 block rows detected from the CRS (rows in triples sharing whole
 * column triples, e.g. 3-dof meshes), one thread per block row; the other rows through the
 * SELL kernel (MIGMRES_NO_BSR3=1 at creation keeps MIGMRES_SPMM_SELL). */
#define MIGMRES_SPMM_BSR3 5
/* MIGMRES_SPMM_MARCH: the stencil-group templates of a 3-D 7- or 27-point grid read as a 2.5-D
 * march -- plane tiles staged once in LDS, every key an LDS read; same bits as the template
 * kernels (MIGMRES_NO_MARCH=1 at creation keeps MIGMRES_SPMM_TPL / MIGMRES_SPMM_TPL3). */
#define MIGMRES_SPMM_MARCH 6
int migmres_crs_spmm_kernel(const migmres_crs *A, int *kind);
/* Digests (64-bit hashes) of the SpMM format plans A holds -- flags, fixed bytes and every
 * format array -- into out[0 .. n); *needed = the digest count.  Test support: the device
 * builders (formats.hip) and the host builders (MIGMRES_HOST_FORMATS=1, plan.cpp) must agree. */
int migmres_crs_format_digest(const migmres_crs *A, unsigned long long *out, int n, int *needed);

/* ---------------- user operators (Belos::OperatorTraits<double, MV, OP> for any OP) ----------------
 * An operator the library does not hold as a CRS: Y = op(X) through a host callback
 * (BelosOperatorTraits.hpp:108-155; the reference solves with any Epetra_Operator /
 * Tpetra::Operator, BelosLinearProblem.hpp:989-1072).  The callback receives the library's
 * own multivector handles (views into the Krylov basis among them) and must leave Y complete in
 * the stream order of the context's stream: a callback that only calls migmres_* functions on
 * the same context does (they enqueue on that stream) -- including a whole nested
 * migmres_solver_solve_op, as the reference's Iterative_Inverse_Operator does
 * (belos/epetra/test/BlockGmres/test_bl_gmres_diag.cpp:233-305); work on another stream must be
 * synchronised before it returns.  A nonzero return fails the apply (and the solve) with
 * MIGMRES_EOP.  The solver does not re-apply a user operator to regenerate a block (it keeps a
 * copy, as the reference does) and never applies one speculatively. */
typedef int (*migmres_apply_fn)(void *user, const migmres_mv *X, migmres_mv *Y);
int migmres_op_create(migmres_ctx *ctx, long long n_global, int n_local, migmres_apply_fn fn, void *user,
                      migmres_op **out);
/* The CRS operator as a migmres_op (borrowed: A must outlive it); solve_op on it = solve(A). */
int migmres_op_from_crs(migmres_crs *A, migmres_op **out);
int migmres_op_apply(migmres_op *op, const migmres_mv *X, migmres_mv *Y);
int migmres_op_destroy(migmres_op *op);

/* ---------------- multivectors (Belos::MultiVecTraits) ---------------- */

/* Owned N_local x ncols block (uninitialised contents, MVT::Clone). */
int migmres_mv_create(migmres_ctx *ctx, long long n_global, int n_local, int ncols, migmres_mv **out);
/* MVT::CloneView(NonConst): a non-owning view of columns idx[0..n-1] of parent. */
int migmres_mv_view(migmres_mv *parent, const int *idx, int n, migmres_mv **out);
/* MVT::CloneView with a contiguous Range1D [first, first+n). */
int migmres_mv_view_range(migmres_mv *parent, int first, int n, migmres_mv **out);
int migmres_mv_destroy(migmres_mv *mv);
int migmres_mv_shape(const migmres_mv *mv, long long *n_global, int *n_local, int *ncols,
                     int *constant_stride);
/* Host <-> device copies of the local rows (column-major host array, leading dim ld). */
int migmres_mv_upload(migmres_mv *mv, const double *host, long long ld);
int migmres_mv_download(const migmres_mv *mv, double *host, long long ld);

/* mv = beta*mv + alpha*A*B, B (A.ncols x mv.ncols) host column-major (MvTimesMatAddMv). */
int migmres_mv_times_mat_add_mv(double alpha, const migmres_mv *A, const double *B, int ldb,
                                double beta, migmres_mv *mv);
/* mv = alpha*A + beta*B (MvAddMv). */
int migmres_mv_add_mv(double alpha, const migmres_mv *A, double beta, const migmres_mv *B,
                      migmres_mv *mv);
int migmres_mv_scale(migmres_mv *mv, double alpha);                 /* MvScale(scalar) */
int migmres_mv_scale_vec(migmres_mv *mv, const double *alphas);     /* MvScale(vector) */
/* C (A.ncols x B.ncols, host, ldc) = alpha * A^T B, summed over all ranks (MvTransMv). */
int migmres_mv_trans_mv(double alpha, const migmres_mv *A, const migmres_mv *B, double *C, int ldc);
int migmres_mv_dot(const migmres_mv *A, const migmres_mv *B, double *out);   /* MvDot */
int migmres_mv_norm(const migmres_mv *mv, double *out, int norm_type);       /* MvNorm */
int migmres_mv_init(migmres_mv *mv, double alpha);                           /* MvInit */
/* MvRandom with Epetra_MultiVector::Random semantics: column-major MINSTD stream from
 * *seed over the GLOBAL rows (partition independent); *seed is advanced. */
int migmres_mv_random(migmres_mv *mv, unsigned int *seed);
int migmres_mv_assign(const migmres_mv *A, migmres_mv *mv);                  /* Assign */
/* SetBlock: mv[:, idx[i]] = A[:, i] for i < n; A may have more than n columns (the first n are
 * copied), as BelosEpetraAdapter.hpp:894-940. */
int migmres_mv_set_block(const migmres_mv *A, const int *idx, int n, migmres_mv *mv);

/* ---------------- ICGS orthogonalisation (Belos::ICGSOrthoManager) ---------------- */

/* projectAndNormalize(X, [C], B, [Q]): C (Q.ncols x X.ncols, ldc), B (X.ncols^2, ldb). */
int migmres_icgs_project_normalize(migmres_mv *X, const migmres_mv *Q, double *C, int ldc,
                                   double *B, int ldb, int *rank);
int migmres_icgs_normalize(migmres_mv *X, double *B, int ldb, int *rank);
/* Belos::DGKSOrthoManager (belos/src/BelosDGKSOrthoManager.hpp:644-815 projectAndNormalize,
 * 828-840 normalize), default parameters (536-556).  Same arguments as the ICGS pair. */
int migmres_dgks_project_normalize(migmres_mv *X, const migmres_mv *Q, double *C, int ldc,
                                   double *B, int ldb, int *rank);
int migmres_dgks_normalize(migmres_mv *X, double *B, int ldb, int *rank);

/* ---------------- preconditioner (Ifpack2::Relaxation "Jacobi") ---------------- */

/* Point Jacobi on A's local rows: Ifpack2::Relaxation with "relaxation: type" = "Jacobi",
 * "relaxation: sweeps" = sweeps, "relaxation: damping factor" = damping, zero starting
 * solution (ifpack2/src/Ifpack2_Relaxation_def.hpp:1390-1454 ApplyInverseJacobi; the
 * inverse diagonal as compute() :1240-1270).  A must outlive the preconditioner. */
int migmres_jacobi_create(migmres_crs *A, int sweeps, double damping, migmres_prec **out);
/* The full Ifpack2::Relaxation parameter list the device path implements
 * (Ifpack2_Relaxation_def.hpp:243-307 names and defaults, compute() :990-1320, apply
 * :1323-1454): "relaxation: type" Jacobi (0) or Richardson (1), "sweeps", "damping factor",
 * "zero starting solution" (0: apply starts from Y's contents), "use l1" with "l1 eta" (on more
 * than one process: d_i += sum of |a_ij / 2| over the off-process columns whose local index
 * exceeds the local row count, when |d_i| < eta times that sum), "min diagonal value" and
 * "fix tiny diagonal entries" (|d_i| <= |min| -> 1 / min, 1 / eps for min = 0), "check diagonal
 * entries" (statistics only).  migmres_jacobi_create(A, s, w, &M) = these defaults with sweeps
 * s and damping w. */
typedef struct migmres_relaxation_params {
  int type;                      /* 0 "Jacobi" (default), 1 "Richardson" */
  int sweeps;                    /* 1 */
  double damping;                /* 1.0 */
  int zero_starting_solution;    /* 1 */
  int use_l1;                    /* 0 */
  double l1_eta;                 /* 1.5 */
  double min_diagonal_value;     /* 0.0 */
  int fix_tiny_diagonal_entries; /* 0 */
  int check_diagonal_entries;    /* 0 */
} migmres_relaxation_params;
int migmres_relaxation_params_default(migmres_relaxation_params *p);
int migmres_relaxation_create(migmres_crs *A, const migmres_relaxation_params *p, migmres_prec **out);
int migmres_prec_destroy(migmres_prec *M);
/* Y = M X (Ifpack2::Relaxation::apply / Ifpack2::Chebyshev::apply, alpha = 1, beta = 0).
 * X may alias Y (apply(x, x)): M then reads a deep copy of X, as
 * Ifpack2_Relaxation_def.hpp:539-551 and Ifpack2_Chebyshev_def.hpp:456-473 do.  A Chebyshev
 * preconditioner with zero_starting_solution = 0 starts from Y's current contents. */
int migmres_prec_apply(migmres_prec *M, const migmres_mv *X, migmres_mv *Y);
/* The stored inverse diagonal (n_local doubles). */
int migmres_prec_diagonal(const migmres_prec *M, double *dinv_out);

/* Chebyshev polynomial smoother (Ifpack2::Chebyshev, ifpack2/src/Ifpack2_Chebyshev_def.hpp
 * over Ifpack2_Details_Chebyshev_def.hpp): the parameter list of Details::Chebyshev
 * (:280-300 defaults, setParameters :333-677) as plain fields.  max_eigenvalue NaN = not
 * given (estimate it: the power method on D^-1 A, :1341-1473, from an Epetra MINSTD random
 * vector with `seed` -- Tpetra's randomize() stream is not reproduced; a negative estimate is
 * retried once from |x| of the stream's next draw, :1457-1471).  compute() (:739-896)
 * runs inside create; apply is migmres_prec_apply (ifpackApplyImpl :1221-1339, or
 * textbookApplyImpl :1163-1208 with textbook != 0). */
typedef struct migmres_chebyshev_params {
  int degree;                 /* "chebyshev: degree" (1) */
  double max_eigenvalue;      /* "chebyshev: max eigenvalue" (NaN = estimate) */
  double ratio_eigenvalue;    /* "chebyshev: ratio eigenvalue" (30, >= 1) */
  double boost_factor;        /* "chebyshev: boost factor" (1.1, >= 1) */
  double min_diagonal_value;  /* "chebyshev: min diagonal value" (eps) */
  int eigenvalue_max_iterations; /* "chebyshev: eigenvalue max iterations" (10) */
  int zero_starting_solution; /* "chebyshev: zero starting solution" (1) */
  int assume_matrix_unchanged; /* "chebyshev: assume matrix does not change" (0) */
  int textbook_algorithm;     /* "chebyshev: textbook algorithm" (0) */
  unsigned int seed;          /* power-method start vector stream (1) */
} migmres_chebyshev_params;
/* Fill *p with the reference defaults. */
int migmres_chebyshev_params_default(migmres_chebyshev_params *p);
/* Chebyshev preconditioner on A (A must outlive it).  Errors as setParameters' checks:
 * degree < 0, ratio < 1, boost < 1, a non-finite max eigenvalue or min diagonal value. */
int migmres_chebyshev_create(migmres_crs *A, const migmres_chebyshev_params *p, migmres_prec **out);
/* The eigenvalue bounds apply() uses (getLambdaMaxForApply) and the power method's estimate
 * (NaN when it did not run). */
int migmres_chebyshev_lambdas(const migmres_prec *M, double *lambda_max_for_apply, double *lambda_min_for_apply,
                              double *computed_lambda_max);

/* ---------------- solver manager (Belos::BlockGmresSolMgr) ---------------- */

int migmres_solver_create(migmres_ctx *ctx, migmres_solver **out);  /* "BLOCK GMRES" */
/* Belos::SolverFactory::create by name (Belos_Details_EBelosSolverType.cpp:55-100): "GMRES",
 * "PSEUDOBLOCK GMRES" (PseudoBlockGmresSolMgr, BelosPseudoBlockGmresSolMgr.hpp), "BLOCK GMRES",
 * "FLEXIBLE GMRES" (BlockGmresSolMgr with "Flexible Gmres" = true). */
int migmres_solver_create_named(migmres_ctx *ctx, const char *name, migmres_solver **out);
int migmres_solver_destroy(migmres_solver *s);
/* Belos ParameterList names (BelosBlockGmresSolMgr.hpp:438-486): "Block Size", "Num Blocks",
 * "Maximum Iterations", "Maximum Restarts", "Convergence Tolerance", "Adaptive Block Size",
 * "Flexible Gmres", "Explicit Residual Test", "Orthogonalization" ("ICGS" | "DGKS"),
 * "Implicit Residual Scaling", "Explicit Residual Scaling" ("Norm of Initial Residual" |
 * "Norm of Preconditioned Initial Residual" | "Norm of RHS" | "None"), "Verbosity",
 * "Output Frequency"; pseudo-block only: "Deflation Quorum" (no "Flexible Gmres"). */
int migmres_solver_set_int(migmres_solver *s, const char *name, long long value);
int migmres_solver_set_double(migmres_solver *s, const char *name, double value);
int migmres_solver_set_string(migmres_solver *s, const char *name, const char *value);
/* getCurrentParameters (BelosSolverManager.hpp:101): the value in effect, by name and type.
 * get_string writes at most len bytes including the terminating NUL. */
int migmres_solver_get_int(const migmres_solver *s, const char *name, long long *value);
int migmres_solver_get_double(const migmres_solver *s, const char *name, double *value);
int migmres_solver_get_string(const migmres_solver *s, const char *name, char *value, int len);
/* getValidParameters / getCurrentParameters (BelosSolverManager.hpp:98-101) as text: one
 * parameter per line, "name<TAB>type<TAB>value" with type int | bool | double | string;
 * valid = the solver's defaults (BelosBlockGmresSolMgr.hpp:438-486, pseudo-block
 * BelosPseudoBlockGmresSolMgr.hpp:494-507), current = the values in effect.  Writes at
 * most len bytes including the NUL (buf may be NULL to query); *needed = the full size. */
int migmres_solver_valid_parameters(const migmres_solver *s, char *buf, int len, int *needed);
int migmres_solver_current_parameters(const migmres_solver *s, char *buf, int len, int *needed);
/* reset(ResetType) (BelosSolverManager.hpp:177; BlockGmresSolMgr :250 calls setProblem() for
 * Belos::Problem).  migmres_solver_solve always sets the problem up from the X and B it is
 * given, so MIGMRES_RESET_PROBLEM only clears the previous solve's results (iterations,
 * history, counters); MIGMRES_RESET_RECYCLE is accepted and does nothing (GMRES keeps no
 * recycle space), as in the reference. */
#define MIGMRES_RESET_PROBLEM 1
#define MIGMRES_RESET_RECYCLE 2
int migmres_solver_reset(migmres_solver *s, int type);
/* setUserConvStatusTest(test, comboType) (BelosSolverManager.hpp:147-155): PseudoBlockGmres
 * only (BelosPseudoBlockGmresSolMgr.hpp:1070-1078, combined at :1216-1240 as
 * StatusTestCombo(combo, residual test, user test)); BlockGmresSolMgr does not override it
 * and the call fails as the reference's throws.  The test is a host callback asked at
 * every status check with the iteration count and the current right-hand sides' scaled
 * implicit residual norms (the residual test's testvector); it returns nonzero for
 * Passed.  Combo: MIGMRES_COMBO_SEQ (the default: the user test is asked only once the
 * residual test passed), MIGMRES_COMBO_AND (both asked, both must pass), MIGMRES_COMBO_OR
 * (both asked, either passes).  fn == NULL removes it.  Deflation still follows the residual
 * test's converged indices, as in the reference. */
typedef int (*migmres_status_fn)(void *user, int iters, int nrhs, const double *res);
#define MIGMRES_COMBO_AND 0
#define MIGMRES_COMBO_OR 1
#define MIGMRES_COMBO_SEQ 2
int migmres_solver_set_user_conv_test(migmres_solver *s, migmres_status_fn fn, void *user, int combo);
/* LinearProblem::setLeftPrec / setRightPrec (BelosLinearProblem.hpp:170-175): side
 * MIGMRES_LEFT_PREC or MIGMRES_RIGHT_PREC; M == NULL removes it.  The solver borrows M. */
#define MIGMRES_LEFT_PREC 0
#define MIGMRES_RIGHT_PREC 1
int migmres_solver_set_prec(migmres_solver *s, int side, migmres_prec *M);
/* LinearProblem(A, X, B).setProblem() + solve(); X is updated in place.
 * *converged = 1 for Belos::Converged, 0 for Unconverged. */
int migmres_solver_solve(migmres_solver *s, migmres_crs *A, migmres_mv *X, const migmres_mv *B,
                         int *converged);
/* The same with any operator (LinearProblem::setOperator of an OP that is not a CRS). */
int migmres_solver_solve_op(migmres_solver *s, migmres_op *A, migmres_mv *X, const migmres_mv *B,
                            int *converged);
/* setLeftPrec / setRightPrec with a user operator (borrowed; NULL removes it). */
int migmres_solver_set_prec_op(migmres_solver *s, int side, migmres_op *M);
int migmres_solver_num_iters(const migmres_solver *s, int *iters);
int migmres_solver_achieved_tol(const migmres_solver *s, double *tol);
int migmres_solver_loa_detected(const migmres_solver *s, int *loa);
/* Implicit residual history: one row of numrhs scaled norms per status-test check.
 * Returns the number of rows via *nrows; pass out == NULL to query. */
int migmres_solver_history(const migmres_solver *s, double *out, int *nrows, int *ncols);
/* Counters: [0] operator applies, [1] explicit residual checks, [2] restarts,
 * [3] blkOrthoSing fallbacks, [4] block iterations, [5] preconditioner applies,
 * [6] pseudo-block deflations, [7] findBasis calls taken in Gram form (CholQR2),
 * [8] of those handed back to the column passes (the pivot-ratio gate, or DGKS's criterion
 * asking a second projection of some columns only), [9] DGKS blocks in which no column needed
 * DGKS's second projection (CholQR1, B = R1: DGKS's single Gram-Schmidt pass per column),
 * [10] DGKS blocks handed to the column passes because only some columns needed it. */
int migmres_solver_counters(const migmres_solver *s, long long *out, int n);
/* Seconds spent in named phases: [0] total solve, [1] SpMM, [2] orthogonalization,
 * [3] host least-squares, [4] communication, [5] status tests, [6] restarts, [7] setup.
 * With "Verbosity" bit 1 set the phases are separated by stream synchronisations. */
int migmres_solver_timers(const migmres_solver *s, double *out, int n);

#ifdef __cplusplus
}
#endif
#endif /* MIGMRES_H */
