/*
 * riptrm.h — C-ABI of the MI355X (gfx950) RIPTRM tCG hot path.
 *
 * One shared library (libriptrm_hip.so) exports these symbols.  Every pointer argument is
 * caller-owned DEVICE memory (fp64 unless stated, contiguous, row-major), every call enqueues
 * on the hipStream_t bound to the context and never allocates device memory; only the calls
 * documented as "synchronises" block the host.  Every function returns 0 on success and a
 * negative RIPTRM_E_* code on failure; riptrm_last_error() returns the message.  Nothing
 * throws across the ABI.
 *
 * Reference interfaces replaced (paths relative to the reference repository root):
 *   riptrm_nonnegpca_hvp      HwCur(dx), src/solver/RIPTRM.py:729 = hessLagrangefun :491-523
 *                             + Gxfun :525-551 ∘ (y ⊙ Gxajfun :553-571 ⊘ s), NonnegPCA callbacks
 *                             src/NonnegPCA/coordinator.py:46-77 (egrad/ehess via autograd)
 *   riptrm_tcg_*              truncated_conjugate_gradient, src/solver/RIPTRM.py:41-216, as
 *                             called by compute_direction :445-452 (eta0 = 0, maxinner = dim)
 *   riptrm_solve_*            RIPTRM.run :909-976 -> outer_step :866-896 -> inner_run :785-847
 *                             -> inner_step :707-783 -> update_xy_TR_radius :631-705, with
 *                             the KKT evaluation of src/solver/utils.py:269-368 for the log
 *   riptrm_nonnegpca_symmetrize  S = Z + Z^T (the Hessian of -x^T Z x, coordinator.py:52-54)
 */
#ifndef RIPTRM_H
#define RIPTRM_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RIPTRM_ABI_VERSION 10

/* status codes */
#define RIPTRM_OK 0
#define RIPTRM_E_ARG -1      /* bad argument (null pointer, size, alignment) */
#define RIPTRM_E_HIP -2      /* a HIP runtime call failed */
#define RIPTRM_E_STATE -3    /* call out of order (e.g. solve before bind) */
#define RIPTRM_E_NODEV -4    /* no usable gfx950 device */

/* tCG stop codes (RIPTRM.py:95,143,145,164,188,190) */
#define RIPTRM_TCG_MAX_INNER_ITER 0
#define RIPTRM_TCG_NEGATIVE_CURVATURE 1
#define RIPTRM_TCG_EXCEEDED_TR 2
#define RIPTRM_TCG_MODEL_INCREASED 3
#define RIPTRM_TCG_REACHED_TARGET_LINEAR 4
#define RIPTRM_TCG_REACHED_TARGET_SUPERLINEAR 5
/* Exact_RepMat direction types (TRSgep's `type`, RIPTRM.py:263,270,280,297), same log field */
#define RIPTRM_TRS_BOUNDARY 6
#define RIPTRM_TRS_INTERIOR 7
#define RIPTRM_TRS_HARDCASE_1 8
/* not a reference code: tCG met a non-finite <delta, H delta> (the instance then stops with
 * RIPTRM_ERR_NONFINITE) */
#define RIPTRM_TCG_NONFINITE 9
/* not a reference code: the Exact_RepMat eigendecomposition did not converge (the instance then
 * stops with RIPTRM_ERR_EIGEN) */
#define RIPTRM_TCG_EIGFAIL 10

/* per-instance error codes (RIPTRM_STAT_ERROR).  An instance with an error stops (phase error);
 * the others of the batch go on.
 * RIPTRM_ERR_NONFINITE: a NaN / Inf in ||cxCur|| or Delta at a tCG start, or in <delta, H delta>
 * inside tCG, stops the instance and restores x, y to the start of the outer step it appeared in
 * -- the reference's do_exit_on_error break (RIPTRM.py:961-966: an exception inside outer_step ends
 * the run with the iterate that outer step started from; numpy would raise there on the NaN).
 * A NaN / Inf KKT residual at the outer loop head also stops the instance, keeping x, y as they
 * are.  That site is a deliberate deviation: the reference raises nothing there (`residual <=
 * tolresid` is just False) and would keep iterating on the NaN iterate.
 * RIPTRM_ERR_EIGEN: the HBM Exact_RepMat path's eigendecomposition (hand-written riptrm_eig.h /
 * riptrm_tri.h, or rocSOLVER dsyevd) reported info != 0, or the trial-point eigenvalue was not finite,
 * where scipy.linalg.eig / eigh raises LinAlgError inside outer_step: same break and restore as
 * RIPTRM_ERR_NONFINITE. */
#define RIPTRM_ERR_NONE 0
#define RIPTRM_ERR_NO_TCG_ITER 1       /* manifold.dim = 0: tCG cannot iterate */
#define RIPTRM_ERR_BARRIER_TIMEOUT 2   /* persistent mode: a peer workgroup never arrived (2 s) */
#define RIPTRM_ERR_NONFINITE 3
#define RIPTRM_ERR_EIGEN 4

/* TRS_solver option (RIPTRM.py:325) */
#define RIPTRM_TRS_SOLVER_TCG 0
#define RIPTRM_TRS_SOLVER_EXACT_REPMAT 1
/* Exact_RepMat works on the dim x dim matrix of HwCur in LDS up to manifold.dim = this
 * (NonnegPCA n <= 97, StableIdentification d <= 7); larger problems (NonnegPCA in
 * riptrm_solve_advance, StableIdentification d >= 8 in riptrm_si_solve) keep the matrix in HBM
 * scratch bound with riptrm_trs_bind_workspace (below) */
#define RIPTRM_TRS_DIM_MAX 96
/* From this manifold.dim up to RIPTRM_TRS_TRI_MAX the HBM path reduces the matrix to tridiagonal form
 * across the chip and solves the subproblem in its coordinates (no eigenvectors; csrc/riptrm_tri.h);
 * below it the one-workgroup batched eigensolver (csrc/riptrm_eig.h) serves it */
#define RIPTRM_TRS_TRI_MIN 150
#define RIPTRM_TRS_TRI_MAX 1024

/* inner_status codes (RIPTRM.py:763,770,678,698,829,837); 0 = None */
#define RIPTRM_IS_NONE 0
#define RIPTRM_IS_INITIAL 1
#define RIPTRM_IS_CONVERGED 2
#define RIPTRM_IS_PRIMAL_INFEASIBLE 3
#define RIPTRM_IS_SUCCESSFUL 4
#define RIPTRM_IS_UNSUCCESSFUL 5
#define RIPTRM_IS_MAX_TIME_EXCEEDED 6
#define RIPTRM_IS_MAX_ITER_EXCEEDED 7

/* radius_update codes (RIPTRM.py:668,671,674); 0 = None */
#define RIPTRM_RU_NONE 0
#define RIPTRM_RU_REDUCED 1
#define RIPTRM_RU_EXPANDED 2
#define RIPTRM_RU_UNCHANGED 3

/* stopping criterion codes (base_solver.py:94-105, RIPTRM.py:944) */
#define RIPTRM_STOP_NONE 0
#define RIPTRM_STOP_MAXTIME 1
#define RIPTRM_STOP_MAXITER 2
#define RIPTRM_STOP_TOLRESID 3

/* storage layouts of S = Z + Z^T (one instance) */
#define RIPTRM_LAYOUT_FULL 0      /* row-major, riptrm_nonnegpca_rows(n) rows of riptrm_nonnegpca_ld(n) */
#define RIPTRM_LAYOUT_SYMTILE 1   /* upper triangle as 128x128 row-major tiles (I,J), I <= J, ordered
                                   * row by row: tile t = I*nt - I*(I-1)/2 + (J-I), nt = ld/128 */
#define RIPTRM_LAYOUT_SHARED 2    /* multi-start: ONE full row-major S shared by every instance of the
                                   * batch (same Z, different initial points: the reference's
                                   * problem_initialpoint axis); bind with inst_stride = 0.  The S-pass
                                   * is a fp64 MFMA product S [v_1 .. v_B] */

/* manifold-violation kinds for the KKT residual (option 'manviofun') */
#define RIPTRM_MANVIO_ZERO 0     /* RIPTRM.py:347 default: lambda problem, x: 0 */
#define RIPTRM_MANVIO_SPHERE 1   /* src/NonnegPCA/simulator.py:12-14: ||x|| - 1 */
#define RIPTRM_MANVIO_SI 2       /* src/StableIdentification/simulator.py:11-32: ||J+J^T|| + ||R-R^T||
                                  * + ||Q-Q^T||, inf when R or Q is not positive definite */

/* Per-inner-iteration log record: RIPTRM_LOG_NFIELDS doubles, field order below.
 * Columns = evaluation keys (utils.py:356-364) + solver_status keys (RIPTRM.py:986-1023). */
enum riptrm_log_field {
    RIPTRM_LOG_ITERATION = 0, RIPTRM_LOG_TIME, RIPTRM_LOG_COST, RIPTRM_LOG_DISTANCE,
    RIPTRM_LOG_RESIDUAL, RIPTRM_LOG_GRADNORM, RIPTRM_LOG_COMPLVIOLATION, RIPTRM_LOG_DUALVIOLATION,
    RIPTRM_LOG_MANVIOLATION, RIPTRM_LOG_MAXVIOLATION, RIPTRM_LOG_MEANVIOLATION, RIPTRM_LOG_MU,
    RIPTRM_LOG_HAS_INFO, RIPTRM_LOG_NUM_INNER, RIPTRM_LOG_INNER_STATUS, RIPTRM_LOG_TR_RADIUS,
    RIPTRM_LOG_DXTYPE, RIPTRM_LOG_NORMDX, RIPTRM_LOG_MINXFEASI, RIPTRM_LOG_MINYFEASI,
    RIPTRM_LOG_COMPL, RIPTRM_LOG_HAS_RATIO, RIPTRM_LOG_ARED_PRED, RIPTRM_LOG_RADIUS_UPDATE,
    RIPTRM_LOG_DUAL_CLIPPING, RIPTRM_LOG_MAXABSLAGMULT, RIPTRM_LOG_TCG_ITERS,
    RIPTRM_LOG_HAS_MINEIG, RIPTRM_LOG_MINEIGVALHW,
    RIPTRM_LOG_NFIELDS_USED
};
#define RIPTRM_LOG_NFIELDS 32

/* Log slots.  Record k of an instance (k counted from the last riptrm_log_rebase, k = LOG_COUNT -
 * LOG_BASE at the time it is written) goes to slot k while k < capacity; past that the first
 * capacity/2 slots keep the earliest records and the remaining T = capacity - capacity/2 slots
 * form a ring holding the latest T (slot capacity/2 + (k - capacity/2) mod T), LOG_OVERFLOW
 * counts the records dropped from the middle.  riptrm_log_rebase between solve_advance calls
 * (after the host has copied the slots out) keeps a log of any length complete. */

/* Per-instance result record: RIPTRM_STAT_NFIELDS doubles. */
enum riptrm_stat_field {
    RIPTRM_STAT_OUTER_ITERS = 0, RIPTRM_STAT_INNER_ITERS, RIPTRM_STAT_TCG_ITERS, RIPTRM_STAT_PASSES,
    RIPTRM_STAT_STOP_CODE, RIPTRM_STAT_STOP_RUNTIME, RIPTRM_STAT_FINAL_RESIDUAL, RIPTRM_STAT_LOG_COUNT,
    RIPTRM_STAT_LOG_OVERFLOW, RIPTRM_STAT_PHASE, RIPTRM_STAT_MU, RIPTRM_STAT_TR_RADIUS,
    RIPTRM_STAT_TCG_LAST_J, RIPTRM_STAT_TCG_LAST_STOP, RIPTRM_STAT_ERROR, RIPTRM_STAT_LOG_BASE,
    RIPTRM_STAT_RHS,   /* S-pass right-hand sides (PASSES counts requests; a trial pass carries 2) */
    RIPTRM_STAT_NFIELDS_USED
};
#define RIPTRM_STAT_NFIELDS 24

/* Solver options: the tCG-path keys of the RIPTRM default_option (RIPTRM.py:305-358).
 * Option callables (forcing functions, barrier schedule) are evaluated by the host into the
 * per-outer-iteration tables passed to riptrm_solve_begin(). */
typedef struct riptrm_options {
    int32_t struct_size;              /* = sizeof(riptrm_options) */
    int32_t maxiter;                  /* 'maxiter' */
    int32_t inner_maxiter;            /* 'inner_maxiter', -1 = None */
    int32_t tcg_mininner;             /* 'tCG_mininner' */
    int32_t save_inner_iteration;     /* 'save_inner_iteration' (bool) */
    int32_t manvio_kind;              /* RIPTRM_MANVIO_* */
    int32_t log_capacity;             /* log records per instance (<= the bound capacity) */
    int32_t restart_every;            /* 0 = off; k > 0: after outer iteration k, 2k, ... restart the
                                       * instance from (x0, y0, mu_0, Delta_0) and keep counting
                                       * (benchmark windows longer than one solve) */
    double maxtime;                   /* 'maxtime' seconds (INFINITY allowed) */
    double inner_maxtime;             /* 'inner_maxtime' seconds, < 0 = None */
    double tolresid;                  /* 'tolresid' */
    double initial_tr_radius;         /* 'initial_TR_radius' (host resolves None -> pi/8) */
    double minimal_initial_tr_radius; /* 'minimal_initial_TR_radius' */
    double maximal_tr_radius;         /* 'maximal_TR_radius' */
    double rho;                       /* 'rho' */
    double reduction_regularization;  /* 'reduction_regularization' */
    double gamma;                     /* 'gamma' */
    double tcg_theta;                 /* 'tCG_theta' */
    double tcg_kappa;                 /* 'tCG_kappa' */
    double const_left;                /* 'const_left' */
    double const_right;               /* 'const_right' */
    int32_t trs_solver;               /* 'TRS_solver': RIPTRM_TRS_SOLVER_* */
    int32_t second_order_stationarity;/* 'second_order_stationarity' (bool; Exact_RepMat only) */
    double trs_tolhardcase;           /* 'TRS_tolhardcase' */
    const double* tol2_table;         /* device, table_len doubles: forcing_function_second_order of the
                                       * mu table (RIPTRM.py:884); NULL = mu itself (the default) */
} riptrm_options;

typedef struct riptrm_ctx riptrm_ctx;

int riptrm_abi_version(void);

/* Create a context on `device` that enqueues on `stream` (a hipStream_t; NULL = default). */
int riptrm_ctx_create(riptrm_ctx** out, int device, void* stream);
int riptrm_ctx_destroy(riptrm_ctx* ctx);
const char* riptrm_last_error(const riptrm_ctx* ctx);
/* Rebind the stream (e.g. torch.cuda.current_stream()). */
int riptrm_ctx_set_stream(riptrm_ctx* ctx, void* stream);

/* ---- layout (pure functions, no device work) ---- */
/* Leading dimension (doubles) of every state vector and of a full-layout row of S
 * (n rounded up to 128). */
int64_t riptrm_nonnegpca_ld(int32_t n);
/* Rows of one full-layout instance of S (multiple of the mat-vec row block). */
int64_t riptrm_nonnegpca_rows(int32_t n);
/* Doubles of one instance of S in `layout` (the minimum instance stride). */
int64_t riptrm_nonnegpca_s_elems(int32_t n, int32_t layout);
/* Device workspace bytes for a batch (state vectors, scalars, log, partial sums, counters). */
int64_t riptrm_workspace_bytes(int32_t n, int32_t batch, int32_t log_capacity, int32_t layout);
/* Byte offsets inside the workspace.  kind: 0 = x, 1 = y, 2 = eta (last dx), 3 = Heta,
 * 4 = stats (batch x RIPTRM_STAT_NFIELDS doubles), 5 = log (batch x capacity x NFIELDS). */
int64_t riptrm_workspace_offset(int32_t n, int32_t batch, int32_t log_capacity, int32_t layout,
                                int32_t kind);

/* ---- data preparation ---- */
/* S_b <- pack(Z_b + Z_b^T) for b < count: Z_b is n x n row-major with leading dimension ldz at
 * Z + b*z_stride, S_b is written at S + b*s_stride in `layout` with zero padding.  Each
 * element is the one rounding of Z_ij + Z_ji, so S is exactly symmetric. */
int riptrm_nonnegpca_pack(riptrm_ctx* ctx, const double* Z, int64_t ldz, int64_t z_stride, int32_t n,
                          int32_t count, double* S, int32_t layout, int64_t s_stride);

/* ---- bind a batch of NonnegPCA instances sharing n (the hydra multi-run axis) ---- */
int riptrm_nonnegpca_bind(riptrm_ctx* ctx, const double* S, int32_t n, int32_t batch,
                          int32_t layout, int64_t s_stride, void* workspace,
                          int64_t workspace_bytes, int32_t log_capacity);

/* ---- operator entry points (parity / building blocks) ---- */
/* out_b = HwCur_b(v_b) at (x_b, y_b, mu), s = x (NonnegPCA slack).  x, y, v, out: batch x ldv. */
int riptrm_nonnegpca_hvp(riptrm_ctx* ctx, const double* x, const double* y, double mu,
                         const double* v, double* out, int64_t ldv);
/* RIPM's condensed Newton operator OperatorAw (src/solver/RIPM.py:485-487, do_euclidean_lincomb
 * False): out_b = hessLagrangian(x_b, z_b)[v_b] + Gx(x_b, Gxaj(x_b, v_b) * z_b / s_b) for NonnegPCA
 * (constraints -x_i <= 0, multipliers z, slacks s) = the barrier-Hessian structure of HwCur with
 * (y, s) -> (z, s).  x, z, s, v, out: batch x ldv. */
int riptrm_nonnegpca_operator_aw(riptrm_ctx* ctx, const double* x, const double* z, const double* s,
                                 const double* v, double* out, int64_t ldv);
/* Batched tCG at (x_b, y_b, mu_b, Delta_b): eta/Heta written into the workspace vectors
 * (offset kinds 2/3); iters_b = loop index j at exit (RIPTRM.py:216 returns j), stop_b code.
 * x, y: batch x ldv; mu, delta: batch doubles; iters, stop: batch int32.  Synchronises. */
int riptrm_tcg(riptrm_ctx* ctx, const double* x, const double* y, int64_t ldv,
               const double* mu, const double* delta, int32_t* iters, int32_t* stop,
               int32_t max_steps);

/* ---- full solve ---- */
/* Start a batched RIPTRM run from x0/y0 (batch x ldv).  mu_table[k] = barrier parameter of
 * outer step k+1 (k = 0..table_len-1), tolL/tolC = the forcing functions of mu_table. */
int riptrm_solve_begin(riptrm_ctx* ctx, const riptrm_options* opt, const double* x0,
                       const double* y0, int64_t ldv, const double* mu_table,
                       const double* tolL_table, const double* tolC_table, int32_t table_len);
/* Enqueue up to `steps` lock-step iterations (one S-pass for every instance that still needs
 * one + one state-machine advance).  Instances pause before starting outer iteration number
 * `outer_target` + 1 (pass INT32_MAX to run to completion).  Synchronises and returns the
 * number of instances still running in *n_active. */
int riptrm_solve_advance(riptrm_ctx* ctx, int32_t steps, int32_t outer_target, int32_t* n_active);
/* Mark every log record written so far as drained (LOG_BASE <- LOG_COUNT for every instance of the
 * NonnegPCA batch): the next record of each instance goes to slot 0 again.  Call between
 * riptrm_solve_advance calls, after copying the records out.  Asynchronous. */
int riptrm_log_rebase(riptrm_ctx* ctx);
/* Device timestamps for timing windows: wall-clock ticks per second of the device clock. */
double riptrm_device_clock_hz(riptrm_ctx* ctx);

/* Lock-step pipelines: 0 = automatic (two instance groups on two streams when the batch's S is
 * >= ~1.2 GB, so one group's state kernel overlaps the other's S-pass), 1 or 2 to force.
 * Takes effect at the next riptrm_nonnegpca_bind.  Results do not depend on it. */
int riptrm_set_stream_groups(riptrm_ctx* ctx, int32_t groups);

/* Small batches (S of the batch < 200 MB, or the shared layout) replay a captured hipGraph of 8
 * lock-step iterations (16 kernels) per host submission instead of 2 launches per iteration,
 * unless profiling is on.  on = 0 disables it (default 1).  Results do not depend on it. */
int riptrm_set_graphs(riptrm_ctx* ctx, int32_t on);

/* Persistent lock-step mode (symmetric-tile layout, TRS_solver tCG): when batch x tiles per
 * instance <= min(256, compute units) — e.g. n <= 1024 for up to 7 instances, n <= 2048 for one
 * (BASELINE configs[1]: n = 1000, one instance) — each riptrm_solve_advance / riptrm_tcg chunk is
 * ONE launch in which every stored tile keeps its 128 x 128 block of S in LDS and every workgroup
 * runs a replica of its instance's state machine (bitwise the lock-step results; replaces
 * RIPTRM.py:41-216 + :707-896 for such batches).  mode 1 = automatic (default): a cooperative
 * launch, allowed at bind only if the occupancy calculator fits every workgroup with its 128 KiB
 * of LDS at once; 0 = never; 2 = automatic with a plain launch (A/B only: no co-residency
 * guarantee); 3 = as 1, with the first launch of every solve treated as refused (tests the
 * fallback).  A launch refused before any persistent step of the solve ran hands the solve to
 * the lock-step pipeline (same results bitwise); refused later, the call fails.  Set before
 * riptrm_nonnegpca_bind.  riptrm_get_persistent: whether the bound shape allows it on this device
 * and whether the current solve uses it; riptrm_persist_fallbacks: solves since bind that fell
 * back to lock-step. */
int riptrm_set_persistent(riptrm_ctx* ctx, int32_t mode);
int riptrm_get_persistent(riptrm_ctx* ctx, int32_t* possible, int32_t* active);
int riptrm_persist_fallbacks(riptrm_ctx* ctx, int32_t* count);
/* Diagnostics: per in-launch step of workgroups 0 and reps - 1 of every k_persist launch, record
 * device-clock stamps (0 step start, 1 tile pass done, 2 barrier passed, 3 state step done; tCG
 * steps also 4 partial sums gathered, 5 iteration arithmetic done) into the caller's device
 * buffer buf[2][cap][24] (uint64, overwritten by each launch; 8..14: stamps inside the tCG
 * arithmetic, 16..17 inside the tile product); cap = 0 turns it off. */
int riptrm_persist_trace(riptrm_ctx* ctx, uint64_t* buf, int32_t cap);

/* S-pass kernel of the symmetric-tile layout: 1 = automatic (default: the persistent super-tile
 * kernel — whose partial-sum writes leave the HBM read stream in bursts — for n >= 2561, where an
 * instance has >= 64 units of 2 x 2 tiles, the per-tile kernel below; the rule depends on n only,
 * so an instance gives bitwise identical results alone or inside any batch, run after run),
 * 0 = per-tile kernel only, 2 = super-tile kernel always, 3 = the super-tile kernel for launches
 * that give every compute unit a unit of work if a bind-time timing of both kernels on one
 * instance group preferred it (fastest on a given box; the choice — and so the last bits of the
 * results — can then depend on the box and on how many instances are active).  Set before
 * riptrm_nonnegpca_bind.  Results agree to rounding (the partial sums are added in a different,
 * still fixed, order). */
int riptrm_set_spass_kind(riptrm_ctx* ctx, int32_t kind);
/* ms per S-pass launch over one instance group of the per-tile and the super-tile kernel (0 unless
 * kind 3 timed them at bind) and the kernel a launch over the whole batch uses (0 per-tile,
 * 1 super-tile). */
int riptrm_get_spass_calibration(riptrm_ctx* ctx, double* ms_tile, double* ms_super, int32_t* chosen);

/* ---- measurement ---- */
/* Enable/disable HIP-event timing of every S-pass (k_gemv) and state-machine (k_state) launch
 * enqueued by riptrm_solve_advance / riptrm_tcg; enabling resets the totals.  Synchronises. */
int riptrm_profile_enable(riptrm_ctx* ctx, int32_t on);
/* Summed device time (ms) and launch counts since the last enable.  Synchronises. */
int riptrm_profile_read(riptrm_ctx* ctx, double* gemv_ms, int64_t* gemv_launches, double* state_ms,
                        int64_t* state_launches);

/* ==== StableIdentification (src/StableIdentification/coordinator.py:13-152) ====================
 * M = SkewSymmetric(d) x SPD(d) x SPD(d) (pymanopt Product, :38-44), points (J, R, Q) stored as
 * 3 consecutive row-major d x d blocks; f = tr(E E^T)/N, E = XP - (I + h (J-R) Q) X (:92-98);
 * m inequality constraints on entries of A = (J-R)Q (:102-152), one row of RIPTRM_SI_CONS_FIELDS
 * doubles each: kind (0: -A_rc + p0, 1: A_rc - p0, 2: -(A_rc - p0)^2 + p1), r, c, p0, p1 — the
 * reference's constset rows expanded in order (type 0/1 -> kinds 0 then 1; type 2 -> kind 2 with
 * p1 = k^2).  One workgroup runs one instance's whole RIPTRM solve in one launch: a 64-lane wave up
 * to d = 8, 64 ceil(d^2 / 64) threads (one per element of a d x d block) above.  m <= 64 for d <= 8,
 * m <= 64 ceil(d^2 / 64) above. */
#define RIPTRM_SI_DMAX 16
#define RIPTRM_SI_MMAX 256
#define RIPTRM_SI_CONS_FIELDS 5

typedef struct riptrm_si_problem {
    int32_t struct_size;     /* = sizeof(riptrm_si_problem) */
    int32_t d;               /* 1 <= d <= RIPTRM_SI_DMAX */
    int32_t N;               /* columns of X / XP (coordinator.py:54-90) */
    int32_t m;               /* 1 <= m <= RIPTRM_SI_MMAX */
    double h;                /* cfg.h */
    const double* X;         /* device, d x N row-major */
    const double* XP;        /* device, d x N row-major */
    int64_t data_stride;     /* doubles between instances' X (and XP); 0 = one problem, many starts */
    const double* cons;      /* device, m x RIPTRM_SI_CONS_FIELDS */
    int64_t cons_stride;     /* doubles between instances' constraint tables; 0 = shared */
} riptrm_si_problem;

/* Workspace for a batch: points, multipliers, tCG outputs, residual scratch, stats and log. */
int64_t riptrm_si_workspace_bytes(int32_t d, int32_t N, int32_t m, int32_t batch, int32_t log_capacity);
/* kind: 0 = x (batch x 3 d d), 1 = y (batch x m), 2 = eta, 3 = Heta (batch x 3 d d),
 * 4 = stats (batch x RIPTRM_STAT_NFIELDS), 5 = log (batch x capacity x RIPTRM_LOG_NFIELDS). */
int64_t riptrm_si_workspace_offset(int32_t d, int32_t N, int32_t m, int32_t batch, int32_t log_capacity,
                                   int32_t kind);
/* Bind a batch of StableIdentification instances (the problem_initialpoint / instance axes). */
int riptrm_si_bind(riptrm_ctx* ctx, const riptrm_si_problem* problem, int32_t batch, void* workspace,
                   int64_t workspace_bytes, int32_t log_capacity);
/* out_b = HwCur_b(v_b) (RIPTRM.py:729) at (x_b, y_b, mu_b).  x, v, out: batch x 3 d d; y: batch x m;
 * mu: batch doubles.  Asynchronous. */
int riptrm_si_hvp(riptrm_ctx* ctx, const double* x, const double* y, const double* mu, const double* v,
                  double* out);
/* tCG (RIPTRM.py:41-216) at (x_b, y_b, mu_b, Delta_b): eta / Heta into the workspace (kinds 2/3),
 * stats TCG_LAST_J / TCG_LAST_STOP.  tCG options from opt (NULL = RIPTRM defaults).  Asynchronous. */
int riptrm_si_tcg(riptrm_ctx* ctx, const riptrm_options* opt, const double* x, const double* y,
                  const double* mu, const double* delta);
/* Section timing of riptrm_si_solve (device clock, summed over the batch's instances). */
enum riptrm_si_prof_field {
    RIPTRM_SI_PROF_TOTAL = 0, RIPTRM_SI_PROF_PREPARE, RIPTRM_SI_PROF_TCG, RIPTRM_SI_PROF_HVP,
    RIPTRM_SI_PROF_TRIAL, RIPTRM_SI_PROF_EVAL, RIPTRM_SI_PROF_NFIELDS_USED
};
#define RIPTRM_SI_PROF_NFIELDS 8
/* Enable (allocates a batch x RIPTRM_SI_PROF_NFIELDS buffer, zeroed) or disable section timing of
 * the following riptrm_si_solve launches. */
int riptrm_si_profile_enable(riptrm_ctx* ctx, int32_t on);
/* seconds[RIPTRM_SI_PROF_NFIELDS]: per-section device time summed over instances.  Synchronises. */
int riptrm_si_profile_read(riptrm_ctx* ctx, double* seconds);

/* Whole RIPTRM solves (RIPTRM.py:909-976) from x0 (batch x 3 d d), y0 (batch x m); tables as in
 * riptrm_solve_begin.  One launch, asynchronous: synchronise the stream, then read the workspace.
 * Exact_RepMat with manifold.dim = d(d-1)/2 + d(d+1) > RIPTRM_TRS_DIM_MAX (d >= 8): needs
 * riptrm_trs_bind_workspace(order >= manifold.dim) first; an instance builds its subproblem's matrix
 * (manifold.dim HVPs) in the SI workspace and parks, the call serves every parked instance in
 * batched passes (the HBM path of riptrm_trs_gep; with the second-order test also HwNew's smallest
 * eigenvalue) and relaunches until every instance has finished: synchronous then.  A non-converged
 * eigensolve stops only its instance (stats error = RIPTRM_ERR_EIGEN, x and y back to the start of
 * its outer step: the reference's do_exit_on_error break, RIPTRM.py:961-966); the call still returns
 * RIPTRM_OK and the other instances continue. */
int riptrm_si_solve(riptrm_ctx* ctx, const riptrm_options* opt, const double* x0, const double* y0,
                    const double* mu_table, const double* tolL_table, const double* tolC_table,
                    int32_t table_len);

/* ==== Exact_RepMat trust-region subproblem ==============================
 * TRSgep(A, a, B = I, Delta, tolhardcase) (src/solver/RIPTRM.py:218-299) for a batch of dense
 * symmetric dim x dim matrices: instance b's A at A + b*a_stride (row-major, leading dimension
 * lda), a / x at a + b*ldv, x + b*ldv; Delta, lam1, mineig: batch doubles; kind: batch int32
 * (RIPTRM_TRS_*).  mineig (may be NULL) = the smallest eigenvalue of A (RIPTRM.py:611).
 * dim <= RIPTRM_TRS_DIM_MAX: one workgroup per instance, A staged in LDS, asynchronous.
 * dim > RIPTRM_TRS_DIM_MAX: needs riptrm_trs_bind_workspace(order >= dim); up to `slots` subproblems
 * per pass on HBM-resident matrices (dim < RIPTRM_TRS_TRI_MIN: the hand-written eigensolver and SciPy's CG restated in
 * its eigen-coordinates; RIPTRM_TRS_TRI_MIN <= dim <= 1024: the cooperative tridiagonalisation T = H^T A H and the
 * subproblem in T's coordinates, riptrm_tri.h; above, or for a hard case, rocSOLVER
 * dsyevd_strided_batched and SciPy's CG on A; the secular Newton per subproblem); synchronises.  A non-converged eigensolve fails the call
 * (RIPTRM_E_HIP naming the subproblem: scipy.linalg.eig raises there). */
int riptrm_trs_gep(riptrm_ctx* ctx, int32_t dim, int32_t batch, const double* A, int64_t lda, int64_t a_stride,
                   const double* a, int64_t ldv, const double* Delta, double tolhardcase, double* x,
                   double* lam1, int32_t* kind, double* mineig);

/* Scratch of the HBM path of Exact_RepMat (manifold.dim > RIPTRM_TRS_DIM_MAX; RIPTRM.py:433-444,
 * :599-617 and TRSgep :218-299 at any size): `slots` subproblems of matrix order `order` (NonnegPCA:
 * order = n, the n x n frame matrix; riptrm_trs_gep: order = dim).  Bytes for riptrm_trs_bind_workspace,
 * caller-owned device memory (256-byte aligned).  Each subproblem of a pass takes one slot; with
 * fewer slots than subproblems the pass repeats, with bitwise the same results.  Orders <= 149
 * take the hand-written eigensolver (riptrm_eig.h), 150..1024 the tridiagonal path (riptrm_tri.h, no
 * eigenvectors); rocSOLVER's dsyevd_strided_batched serves larger orders and the tridiagonal path's
 * hard cases, loaded at first use (dlopen of librocsolver.so.0; it manages its own workspace).  In a NonnegPCA solve an
 * instance that reaches the subproblem (or, with the second-order test, a trial point) parks;
 * riptrm_solve_advance serves every parked instance in batched passes after its lock-step chunk and
 * synchronises then; an eigensolve that does not converge stops that instance (RIPTRM_ERR_EIGEN).
 * Binding NULL unbinds. */
int64_t riptrm_trs_workspace_bytes(int32_t order, int32_t slots);
/* Whether the HBM path's eigensolver could be loaded (host only, no device work): RIPTRM_OK, or
 * RIPTRM_E_HIP with the dlopen message in msg (len bytes, NUL-terminated).  The libraries are
 * librocblas.so.5 / librocsolver.so.0 unless RIPTRM_ROCBLAS_LIB / RIPTRM_ROCSOLVER_LIB name others. */
int riptrm_trs_backend_status(char* msg, int32_t len);
int riptrm_trs_bind_workspace(riptrm_ctx* ctx, void* ws, int64_t bytes, int32_t order, int32_t slots);
/* Eigendecomposition cache of the HBM path in a NonnegPCA solve with the second-order test
 * (RIPTRM.py:599-617 computes the trial point's eigenpairs; :686-692 keeps HwNewmatrix for the next
 * subproblem when the step was accepted without dual clipping).  One entry per instance (order >= n,
 * batch >= the bound batch): the trial point's eigenvectors / eigenvalues (orders <= 149) or its
 * tridiagonal form and reflectors (150..1024) keyed by its (x, y).  A
 * subproblem whose (x, y) equals its instance's key bitwise builds the same matrix bits, so it runs
 * CG and the secular step on the cached eigenpairs without an eigensolve: results are bitwise those
 * of the uncached solve.  Caller-owned device memory, riptrm_trs_cache_bytes(order, batch) bytes,
 * 256-byte aligned; binding invalidates every entry, and so does riptrm_solve_begin.  Binding NULL
 * unbinds.  riptrm_trs_cache_stats: hits and subproblems served since riptrm_solve_begin (either
 * pointer may be NULL). */
int64_t riptrm_trs_cache_bytes(int32_t order, int32_t batch);
int riptrm_trs_bind_cache(riptrm_ctx* ctx, void* cache, int64_t bytes, int32_t order, int32_t batch);
int riptrm_trs_cache_stats(riptrm_ctx* ctx, int64_t* hits, int64_t* subproblems);
/* StableIdentification Exact_RepMat above dim 96 (riptrm_si_solve's service): subproblems whose
 * SciPy CG (RIPTRM.py:246-251) was decided on the eigenpairs, and how many of them skipped it because
 * a bound from those eigenpairs shows that no CG iterate passing RIPTRM.py:246-251 can have a model
 * value <= the boundary solution's (RIPTRM.py:294-298); the choice, and every result, is the one the
 * CG would have given (RIPTRM_CG_SKIP=0 in the environment: always run it).  Since the context was
 * created; either pointer may be NULL. */
int riptrm_trs_skip_stats(riptrm_ctx* ctx, int64_t* checked, int64_t* skipped);
/* Batched symmetric eigendecomposition, hand-written for gfx950 (csrc/riptrm_eig.h): the spectrum
 * TRSgep (RIPTRM.py:218-299) and the second-order test (RIPTRM.py:599-617; scipy.linalg.eigh there)
 * take of the Exact_RepMat matrix; the HBM service uses it for manifold.dim 97..199.  One workgroup
 * per matrix, the matrix resident in LDS: Householder tridiagonalisation, bisection, twisted
 * factorisations, back-transformation.  batch matrices of order dim (1 <= dim <= 199) at
 * A + k a_stride (leading dimension lda; the lower triangle is read): eigenvalues ascending into
 * w + k w_stride and, with vectors = 1, eigenvector j into row j of the matrix (overwritten);
 * vectors = 2 leaves the eigenvectors of the tridiagonal form there instead (the compact form the
 * service keeps, back-transformed per vector; for timing).  info[k] = 0, 1 for a non-finite input
 * (its eigenvalues are NaN), 2 when the eigenvectors could not be orthonormalised.  Asynchronous on
 * the context's stream; the context keeps a scratch (2 dim + dim (dim + 1) / 2 doubles per matrix). */
int riptrm_sym_eig(riptrm_ctx* ctx, int32_t dim, int32_t batch, double* A, int64_t lda, int64_t a_stride, double* w,
                   int64_t w_stride, int32_t* info, int32_t vectors);

/* The tridiagonal reduction the Exact_RepMat HBM service runs from order RIPTRM_TRS_TRI_MIN on (csrc/riptrm_tri.h
 * k_tridiag_dist: LAPACK dsytd2, lower, as scipy.linalg.lapack.dsytrd(lower=1) / the eigh inside
 * TRSgep's pencil, RIPTRM.py:251, would start; the matrix spread over one cooperative launch of
 * ~m / 16 workgroups, rows in registers, one all-to-all exchange per column).  batch matrices of order
 * dim (64 <= dim <= 1024) at A + k a_stride (leading dimension lda; the lower triangle is read, A is
 * not written): the diagonal into d + k de_stride (dim entries), the off-diagonal into e + k de_stride
 * (dim - 1 entries).  info[k] = 0, or 3 when an exchange timed out.  Asynchronous on the context's
 * stream; the context keeps the reflectors in a scratch (dim (dim + 1) / 2 doubles per matrix). */
int riptrm_sym_tridiag(riptrm_ctx* ctx, int32_t dim, int32_t batch, const double* A, int64_t lda, int64_t a_stride,
                       double* d, double* e, int64_t de_stride, int32_t* info);

/* ==== Stiefel(n, p) manifold operations =========================================
 * Not in the reference (north_star / BASELINE configs[4] ask for them): pymanopt 2.x formulas,
 * oracle/stiefel_oracle.py, parity unpinned.  Batched over `batch` instances, each an n x p
 * row-major matrix at base + b * stride doubles (stride >= n p), 1 <= p <= RIPTRM_STIEFEL_PMAX,
 * p <= n.  Device pointers, asynchronous on the context's stream. */
#define RIPTRM_STIEFEL_PMAX 64
/* out_b = tr(U_b^T V_b)  (pymanopt Stiefel.inner_product; X unused, kept for the signature) */
int riptrm_stiefel_inner(riptrm_ctx* ctx, int32_t n, int32_t p, int32_t batch, int64_t stride, const double* X,
                         const double* U, const double* V, double* out);
/* out_b = U_b - X_b sym(X_b^T U_b)  (projection = to_tangent_space = euclidean_to_riemannian_gradient) */
int riptrm_stiefel_proj(riptrm_ctx* ctx, int32_t n, int32_t p, int32_t batch, int64_t stride, const double* X,
                        const double* U, double* out);
/* out_b = qf(X_b + U_b), the Q factor with diag(R) > 0 (pymanopt Stiefel.retraction); CholeskyQR2 */
int riptrm_stiefel_retr(riptrm_ctx* ctx, int32_t n, int32_t p, int32_t batch, int64_t stride, const double* X,
                        const double* U, double* out);
/* out_b = P_X(H_b - U_b sym(X_b^T G_b))  (euclidean_to_riemannian_hessian) */
int riptrm_stiefel_ehess2rhess(riptrm_ctx* ctx, int32_t n, int32_t p, int32_t batch, int64_t stride,
                               const double* X, const double* G, const double* H, const double* U, double* out);

#ifdef __cplusplus
}
#endif
#endif /* RIPTRM_H */
