/*
 * amg_mi355x.h -- C-ABI of the MI355X (gfx950) AMG solve-phase library.
 *
 * Drop-in boundary for the hot path of jwp3/async-multigrid: the reference's
 * SEQ_* / SMEM_* / DMEM_* kernels are free C++ functions over hypre_CSRMatrix
 * (fields i, j, data, num_rows, num_cols; diagonal first in each row) and raw
 * HYPRE_Real* vectors.  Each entry point below names the
 * reference function it replaces (paths relative to /root/reference/src).
 *
 * Conventions
 *  - Every function returns AMG_OK (0) or a negative status; none aborts.
 *    amg_last_error() returns a thread-local message for the last failure.
 *  - Host arrays passed in are copied; the caller keeps ownership.  The
 *    library owns device memory behind amg_mat / amg_vec handles.
 *  - Compute calls are asynchronous on the context's stream; amg_sync() or
 *    any download waits.  Call from ONE host thread per context (from an
 *    OpenMP region use `#pragma omp master`).
 *  - Row ranges [rb, re) keep the reference's thread-slice semantics
 *    (SMEM_MatVec(..., ns, ne)); rb = 0, re = nrows is a full pass.
 *  - All arithmetic is fp64 with the reference's per-row summation order:
 *    results are bit-identical to the reference's loops (sums are never
 *    re-associated and products are rounded before accumulation).
 */
#ifndef AMG_MI355X_H
#define AMG_MI355X_H

#ifdef __cplusplus
extern "C" {
#endif

#define AMG_OK 0
#define AMG_ERR_ARG (-1)
#define AMG_ERR_HIP (-2)
#define AMG_ERR_OOM (-3)
#define AMG_ERR_RCCL (-4)
#define AMG_ERR_UNSUPPORTED (-5)

typedef struct amg_ctx amg_ctx;   /* device, streams, workspace, RCCL comm */
typedef struct amg_mat amg_mat;   /* device CSR (+ diagonal), registered once */
typedef struct amg_vec amg_vec;   /* device fp64 vector */
typedef struct amg_hier amg_hier; /* level hierarchy + solver state (AllData analogue) */
typedef struct amg_gen amg_gen;   /* structured 7-pt problem + geometric hierarchy generator */

/* Smoother / solver / option ids: the reference's values (Main.hpp:47-117). */
#define AMG_JACOBI 0
#define AMG_GAUSS_SEIDEL 1
#define AMG_HYBRID_JACOBI_GAUSS_SEIDEL 2
#define AMG_SYMM_JACOBI 3
#define AMG_SEMI_ASYNC_GAUSS_SEIDEL 4
#define AMG_ASYNC_GAUSS_SEIDEL 5
#define AMG_L1_JACOBI 6
#define AMG_L1_HYBRID_JACOBI_GAUSS_SEIDEL 12

#define AMG_MULT 0
#define AMG_AFACX 1
#define AMG_MULTADD 2
#define AMG_BPX 3
#define AMG_ASYNC_AFACX 5
#define AMG_ASYNC_MULTADD 6

#define AMG_FULL_ASYNC 0
#define AMG_SEMI_ASYNC 1

/* input.res_compute_type / converge_test_type (Main.hpp:89-90) and
 * input.read_type (Main.hpp:110-111) of the asynchronous additive solver */
#define AMG_LOCAL 0
#define AMG_GLOBAL 1
#define AMG_READ_SOL 0
#define AMG_READ_RES 1

/* DMEM outer acceleration (input.accel_type, DMEM_Misc.cpp:612-666).  The
 * reference's -cheby and -richard both store 1 (Main.hpp:80-81 define
 * CHEBY_ACCEL and RICHARD_ACCEL as 1), so its DMEM_ChebyUpdate always runs the
 * Richardson branch: AMG_RICHARD_ACCEL.  AMG_CHEBY_RECUR_ACCEL selects the
 * c_k = 2 mu c_{k-1} - c_{k-2} branch (:637-642) the reference CLI cannot reach. */
#define AMG_NO_ACCEL 0
#define AMG_RICHARD_ACCEL 1
#define AMG_CHEBY_RECUR_ACCEL 2

/* Subset of the reference's InputData (Main.hpp:187-234) the hot path reads. */
typedef struct {
   int solver;                   /* input.solver                                  */
   int smoother;                 /* input.smoother                                */
   int num_pre_smooth_sweeps;    /* input.num_pre_smooth_sweeps                   */
   int num_post_smooth_sweeps;   /* input.num_post_smooth_sweeps                  */
   int num_fine_smooth_sweeps;   /* input.num_fine_smooth_sweeps (additive)       */
   int num_coarse_smooth_sweeps; /* input.num_coarse_smooth_sweeps (AFACx)        */
   double smooth_weight;         /* input.smooth_weight                           */
   int num_cycles;               /* input.num_cycles                              */
   double tol;                   /* input.tol (relative residual)                 */
   int check_resnorm;            /* input.check_resnorm_flag                      */
   int cheby_flag;               /* -cheby (also sets precond_flag)               */
   double cheby_mu, cheby_delta; /* cheby.mu, cheby.delta (SMEM_Cheby.cpp:48-49)  */
   int num_threads;              /* T of the reference's row partitions; hybrid
                                    JGS blocks follow PartitionGrids for T; 0 =
                                    device partition of jgs_block_rows rows     */
   int jgs_block_rows;           /* block size of the device partition (>=1)      */
   int reuse_outer_residual;     /* 1: the level-0 pre-smoother consumes the
                                    outer-loop residual f - A u already in r
                                    (bit-identical; saves one A_0 pass/cycle);
                                    2: as 1, and the outer residual vector r
                                    (dead: the cycle overwrites it) is only
                                    written on request -- amg_hier_vec(R, 0)
                                    recomputes it from the current u        */
   int async_type;               /* AMG_FULL_ASYNC / AMG_SEMI_ASYNC               */
   int profile;                  /* 1: HIP-event timing of the fine-level kernels */
   int accel_type;               /* DMEM input.accel_type (distributed solves):
                                    AMG_NO_ACCEL / AMG_RICHARD_ACCEL /
                                    AMG_CHEBY_RECUR_ACCEL, with cheby_mu/delta */
   int cheby_grid;               /* DMEM input.cheby_grid: the async additive level
                                    whose correction carries the d recurrence  */
   int res_compute_type;         /* input.res_compute_type: AMG_LOCAL / AMG_GLOBAL
                                    (ASYNC_MULTADD only, SMEM_Main.cpp:650-660) */
   int read_type;                /* input.read_type: AMG_READ_SOL / AMG_READ_RES   */
   int converge_test_type;       /* input.converge_test_type: AMG_LOCAL (every level
                                    num_cycles corrections) / AMG_GLOBAL (levels run
                                    on until every level has done num_cycles)  */
   /* delay / fault injection (input.delay_type, delay_usec, delay_frac, fail_iter,
    * SMEM_Main.cpp:572-595; SMEM_Solve.cpp:33-43,112-146; DMEM_DelayProc,
    * DMEM_Misc.cpp:668-684).  The reference's "threads" are the num_threads row
    * partitions: thread T-1 is delayed by DELAY_ONE / FAIL_ONE, the last
    * ceil(T * delay_frac) threads by DELAY_SOME (DELAY_ALL: all), each cycle by
    * RandDouble(0, 2 usec_t) microseconds (usec_t = delay_usec for ONE / FAIL_ONE,
    * RandDouble(0, delay_usec) drawn once per thread for SOME / ALL; FAIL_ONE only
    * in cycle fail_iter).  On the GPU a delay is a device-side wait on the stream
    * the delayed work runs on: the compute stream before a synchronous cycle (the
    * cycle waits for its slowest thread), the level stream before a correction of
    * an async additive level (the group owning the thread -- an extension: the
    * reference's async loop takes no delays), the rank's stream before every
    * distributed cycle (delay_usec exactly; delay_rank -1 = every rank, as the
    * reference, else that rank only, its commented-out delay_id variant). */
   int delay_type;               /* AMG_DELAY_NONE / _ONE / _SOME / _ALL / AMG_FAIL_ONE */
   int delay_usec;               /* input.delay_usec                              */
   double delay_frac;            /* input.delay_frac (DELAY_SOME)                 */
   int fail_iter;                /* input.fail_iter (FAIL_ONE)                    */
   int delay_rank;               /* distributed: -1 every rank, else that rank    */
   int max_inflight;             /* input.max_inflight (DMEM_Main.cpp:113): messages
                                    in flight per destination (amg_grid_add)   */
   int async_comm_save_divisor;  /* input.async_comm_save_divisor (:123): send the
                                    accumulated corrections every this many cycles */
   /* stochastic parallel Southwell gating of the asynchronous Jacobi smoother
    * (-smoother async_sps, input.sps_*, DMEM_Main.cpp:119-121,448-459;
    * StochasticParallelSouthwellUpdateProbability, DMEM_Smooth.cpp:548-572) */
   int sps_probability_type;     /* AMG_SPS_EXPONENTIAL / _INVERSE / _RANDOM       */
   double sps_alpha;             /* exp(-x alpha) / 1/(x alpha) / alpha (RANDOM)   */
   double sps_min_prob;          /* > 0: alpha = -log(min_prob) / num_sends
                                    (DMEM_Setup.cpp:1168-1169)                  */
   int delay_level;              /* distributed async additive: -1 every level's
                                    stream takes the delay (DMEM_Add.cpp:106), else
                                    that level's only (a probe of level coupling) */
   int async_schedule;           /* asynchronous additive solves (amg_async_solve,
                                    amg_dist_async_solve): AMG_SCHED_FREE (the race)
                                    or a deterministic admissible schedule of the
                                    race -- the level corrections one level after
                                    another (AMG_SCHED_FINEST_FIRST /
                                    AMG_SCHED_COARSEST_FIRST, converge LOCAL only)
                                    or taking turns, one whole correction each
                                    (AMG_SCHED_ROUND_ROBIN) -- bit-identical to the
                                    oracle's or_set_async_schedule 1 / 2 / 3 */
   int smooth_transfer;          /* 1: the MULTADD / ASYNC_MULTADD transfers are the
                                    reference's smoothed P~ = (I - w D^-1 A) P and
                                    R~ = P~^T (SmoothTransfer, SMEM_Setup.cpp:
                                    1173-1254, w = smooth_weight), applied composed
                                    from the registered plain P, R and A (symmetric):
                                    R~ r = R (r - w A D^-1 r), P~ e = P e - w D^-1 A P e
                                    -- two stencil passes instead of streaming the
                                    long rows of the explicit products; the order of
                                    operations is the oracle's
                                    or_hier_set_composed_transfers.  0: as registered */
} amg_opts;
#define AMG_SCHED_FREE 0
#define AMG_SCHED_FINEST_FIRST 1
#define AMG_SCHED_COARSEST_FIRST 2
#define AMG_SCHED_ROUND_ROBIN 3
#define AMG_SCHED_TIMED 4 /* converge LOCAL: level k takes dur[k] per correction
                             (amg_hier_set_async_durations /
                             amg_dist_hier_set_async_durations); whole corrections
                             in the order of their end times (j+1) dur[k], ties to
                             the finer level -- the race at fixed level speeds,
                             the oracle's or_set_async_schedule 4 */
#define AMG_SPS_EXPONENTIAL 0 /* Main.hpp:132-134 */
#define AMG_SPS_INVERSE 1
#define AMG_SPS_RANDOM 2
#define AMG_DELAY_NONE 0
#define AMG_DELAY_ONE 1
#define AMG_DELAY_SOME 2
#define AMG_DELAY_ALL 3
#define AMG_FAIL_ONE 4

void amg_opts_default(amg_opts *o); /* SMEM_Main.cpp:65-105 defaults */

/* ---- context -------------------------------------------------------------- */
int amg_init(amg_ctx **ctx, int device, int nstreams);
int amg_finalize(amg_ctx *ctx);
int amg_sync(amg_ctx *ctx);
/* Device-side range-check flags raised since the last call (bit 0: a
 * zero-guess fold write outside the coarse level's rows, dropped instead of
 * written), cleared on read; synchronises the context's stream. */
int amg_device_errors(amg_ctx *ctx, int *flags);
const char *amg_last_error(void);
int amg_version(void);

/* ---- matrices: replaces handing hypre_CSRMatrix* to the kernels ----------- */
int amg_csr_register(amg_ctx *ctx, int nrows, int ncols, long long nnz, const int *rowptr,
                     const int *col, const double *val, int diag_first, amg_mat **out);
int amg_mat_free(amg_mat *A);
/* storage of matrices registered from now on: 1 (default; env AMG_VALUE_INDEX=0
 * turns it off) = value-indexed CSR when the matrix has at most 256 distinct
 * values -- the hot kernels stream a one-byte index per entry instead of the
 * 8-byte value and read the value from a table (bit-identical results) */
int amg_set_value_index(amg_ctx *ctx, int enable);
/* number of table entries of A's value index (0: plain CSR) */
int amg_mat_value_index(const amg_mat *A);
/* dictionary-coded CSR for square operators registered from now on: 1 (default; env
 * AMG_DICT_INDEX=0 turns it off) = when A has a value index, at most 256 distinct
 * (column - row, value) pairs and rows of at most 32 entries (stencil and structured
 * Galerkin operators), each entry is stored as one byte and the kernels run lane per
 * row with coalesced x[row + offset] gathers (bit-identical results) */
int amg_set_dict_index(amg_ctx *ctx, int enable);
/* number of dictionary entries of A (0: not dictionary-coded) */
int amg_mat_dict_index(const amg_mat *A);
/* row-pattern-coded CSR for matrices registered from now on: 1 (default; env
 * AMG_ROW_PATTERN=0 turns it off) = when A is dictionary-coded, has no empty row
 * and at most 256 distinct rows (as sequences of dictionary entries), each row is
 * stored as one byte naming its sequence and the kernels read no row pointer
 * (bit-identical results) */
int amg_set_row_pattern(amg_ctx *ctx, int enable);
/* number of distinct row patterns of A (0: not row-pattern-coded) */
int amg_mat_row_pattern(const amg_mat *A);
/* paired-row-pattern storage (default on; env AMG_PAIR_PATTERN=0 disables),
 * built at registration on top of the row patterns for square operators whose
 * rows hold <= 32 entries: rows 2t and 2t+1 share one byte naming their merged
 * entry list, and an entry both rows hold at the same column offset reads both
 * x values with one 16-byte load (bit-identical results).  enable = 1 builds
 * it for rows of <= 8 entries at any size and for longer rows (27-pt Galerkin
 * levels) only from 4M rows up, where the pair's longer latency per lane is
 * hidden; enable = 2 builds it whenever it applies (tests). */
int amg_set_pair_pattern(amg_ctx *ctx, int enable);
/* number of distinct row-pair patterns of A (0: not pair-coded) */
int amg_mat_pair_pattern(const amg_mat *A);
/* slab-compressed anchors for pair-coded operators with per-row anchors (P, R):
 * 2 bytes per row pair instead of 4 per row.  Default off (env
 * AMG_PAIR_ANCHOR16=1 enables): P0 at 512^3 measured 0.73 ms against 0.65-0.68 ms
 * with the int32 anchors.  amg_mat_pair_anchor16: 1 when A stores them so. */
int amg_set_pair_anchor16(amg_ctx *ctx, int enable);
int amg_mat_pair_anchor16(const amg_mat *A);
/* master-pattern storage (default on; env AMG_MASTER_PATTERN=0 disables), built
 * on top of the pair patterns of square diagonal-first operators whose rows'
 * column offsets all follow one master order (the diagonal, then ascending):
 * the offsets become wave-uniform kernel arguments and each pair pattern only
 * says which master entries its two rows use (bit-identical results). */
int amg_set_master_pattern(amg_ctx *ctx, int enable);
/* master length J of A (0: not master-coded); negative (-J) when every master
 * entry carries one value over the whole matrix */
int amg_mat_master_pattern(const amg_mat *A);
/* plane-marching kernel (default on; env AMG_PLANE_MARCH=0 disables, =Z sets the
 * planes per chunk, AMG_PLANE_MARCH_XCD=0 the plain workgroup order) for
 * master-coded operators whose master list is [0, -P, -S, -1, +1, +S, +P] with
 * P % 512 == 0 and nrows a multiple of P -- the reference's 7-pt Laplacian
 * (Laplacian_3D_7pt, SEQ_MatVec.cpp:3-24 / SMEM_MatVec.cpp:140-258 /
 * SMEM_Smooth.cpp:35-45 applied to it): x of three planes stays in registers
 * while a workgroup marches through zc planes.  Bit-identical to every other
 * form.  enable applies to matrices registered afterwards; zc (1..64, 0 keeps)
 * and xcd (XCD-contiguous workgroup order, -1 keeps) apply to later launches.
 * The 27-point form (master list [0, then dz P + dy S + dx ascending]: the
 * Galerkin coarse operators R A P of the box hierarchy, SMEM_MatVec.cpp:140-258
 * on them) marches the same way with lines y - 1, y, y + 1 of three planes in
 * registers.
 * amg_mat_plane_march: the plane size P (0: not marched);
 * amg_mat_march_points: the marched stencil, 7 or 27 (0: not marched). */
int amg_set_plane_march(amg_ctx *ctx, int enable, int zc, int xcd);
/* 3x3 block form of num_functions = 3 operators (dofs byVDIM, the DMEM
 * elasticity problem DMEM_BuildMatrix.cpp:442-719): block rows whose three rows
 * hold the same dense 3x3 blocks are stored as blocks -- value-table indices
 * when the matrix is value-indexed, else fp64 -- and the SpMV / Jacobi kernels
 * walk them three lanes per block row (diagonal first, then ascending: the
 * CSR order, bit-identical); the identity rows of fixed dofs keep the CSR
 * form.  Used when >= 90% of the block rows block.  amg_set_bsr3(ctx, 0) (env
 * AMG_BSR3=0) keeps CSR for matrices registered afterwards; value-indexed
 * blocks are walked one lane per block row (64 block rows per slice: the
 * default, 2) or three lanes per block row (21 per slice: amg_set_bsr3(ctx, 1),
 * AMG_BSR3=1), the same bits;
 * amg_mat_bsr3: 1 value-indexed blocks, 2 fp64 blocks, 0 not blocked. */
int amg_set_bsr3(amg_ctx *ctx, int enable);
int amg_mat_bsr3(const amg_mat *A);
/* block rows per slice of a blocked matrix: 64 (a lane per block row) or 21
 * (a lane per row); 0 when not blocked */
int amg_mat_bsr3_slice(const amg_mat *A);
int amg_mat_plane_march(const amg_mat *A);
int amg_mat_march_points(const amg_mat *A);
int amg_mat_info(const amg_mat *A, int *nrows, int *ncols, long long *nnz);
int amg_mat_download(amg_ctx *ctx, const amg_mat *A, int *rowptr, int *col, double *val);

/* ---- vectors: replaces the driver's calloc'ed HYPRE_Real* ------------------ */
int amg_vec_create(amg_ctx *ctx, int n, amg_vec **out);
int amg_vec_free(amg_vec *v);
int amg_vec_size(const amg_vec *v);
int amg_vec_upload(amg_ctx *ctx, amg_vec *v, const double *host);
int amg_vec_download(amg_ctx *ctx, const amg_vec *v, double *host);
int amg_vec_set(amg_ctx *ctx, amg_vec *v, double alpha);
int amg_vec_copy(amg_ctx *ctx, const amg_vec *x, amg_vec *y);
int amg_vec_axpy(amg_ctx *ctx, double alpha, const amg_vec *x, amg_vec *y);     /* y += a x   */
int amg_vec_ivaxpy(amg_ctx *ctx, const amg_vec *x, const amg_vec *s, amg_vec *y);/* y += x./s DMEM_Misc.cpp:462-478 */
int amg_vec_scale(amg_ctx *ctx, double alpha, amg_vec *y);
int amg_vec_norm2(amg_ctx *ctx, const amg_vec *x, double *out); /* sqrt(sum x_i^2), fixed order */
int amg_vec_dot(amg_ctx *ctx, const amg_vec *x, const amg_vec *y, double *out);

/* ---- kernels ---------------------------------------------------------------- */
/* y = A x on rows [rb,re): SEQ_MatVec SEQ_MatVec.cpp:3-24, SMEM_Sync_Parfor_MatVec
 * SMEM_MatVec.cpp:5-25, SMEM_MatVec :302-323, SMEM_Sync_Parfor_Restrict :380-392 */
int amg_matvec(amg_ctx *ctx, const amg_mat *A, const amg_vec *x, amg_vec *y, int rb, int re);
/* y = A^T x: SEQ_MatVecT SEQ_MatVec.cpp:26-46 (deterministic, via a transpose
 * built once; num_threads > 1 restates the expansion-buffer order of
 * SMEM_Sync_Parfor_MatVecT SMEM_MatVec.cpp:27-58) */
int amg_matvec_t(amg_ctx *ctx, const amg_mat *A, const amg_vec *x, amg_vec *y, int num_threads);
/* y = alpha A x + beta b: SMEM_SpGEMV SMEM_MatVec.cpp:123-259 (all branches;
 * b may alias y: prolong+correct SMEM_Sync_AMG.cpp:118-123) */
int amg_spgemv(amg_ctx *ctx, const amg_mat *A, const amg_vec *x, const amg_vec *b, double alpha,
               double beta, amg_vec *y, int rb, int re);
/* y = A x; r = b - y: SEQ_Residual SEQ_MatVec.cpp:48-63, SMEM_Residual SMEM_MatVec.cpp:362-378 */
int amg_residual(amg_ctx *ctx, const amg_mat *A, const amg_vec *b, const amg_vec *x, amg_vec *y,
                 amg_vec *r, int rb, int re);
/* weighted Jacobi: variant 0 = SMEM_Sync_Parfor_Jacobi SMEM_Smooth.cpp:6-49 /
 * SMEM_Sync_Jacobi :365-407 (zero sweep overwrites u); variant 1 = SEQ_Jacobi
 * SEQ_Smooth.cpp:4-46 (zero sweep adds) */
int amg_jacobi(amg_ctx *ctx, const amg_mat *A, const amg_vec *f, amg_vec *u, amg_vec *u_prev,
               double omega, int sweeps, int zero_first, int rb, int re, int variant);
/* L1 Jacobi with l1 = amg_l1_norms: SMEM_Sync_Parfor_L1Jacobi SMEM_Smooth.cpp:96-133,
 * SMEM_Sync_L1Jacobi :409-443 (variant 0), SEQ_L1Jacobi SEQ_Smooth.cpp:48-87 (variant 1) */
int amg_l1_jacobi(amg_ctx *ctx, const amg_mat *A, const amg_vec *f, amg_vec *u, amg_vec *u_prev,
                  const amg_vec *l1, int sweeps, int zero_first, int rb, int re, int variant);
/* hybrid Jacobi/Gauss-Seidel over blocks blk[0..nblk] (host array):
 * SMEM_Sync_Parfor_HybridJacobiGaussSeidel[T] SMEM_Smooth.cpp:222-363 (diag_scale =
 * A_diag, weight 1) and SMEM_Sync_HybridJacobiGaussSeidel[T] :533-641
 * (diag_scale NULL = a_ii); reverse selects the [T] variants */
/* hybrid JGS kernel form (rows of <= 32 entries; env AMG_JGS_WAVE), all
 * bit-identical: 1 (default) 8 lanes per block, 8 blocks per wave -- each
 * chunk's rows loaded coalesced, the dependency chain advancing eight blocks
 * per wave instruction; 2: one wave per block (the chain carried lane to lane
 * by v_readlane); 0: one lane walks each block (the reference's loop as is);
 * 3: an LDS tile of 64 blocks -- each pass's rows staged coalesced (prefix and
 * tail slots per row), the chains walked one lane per block from LDS */
int amg_set_jgs_wave(amg_ctx *ctx, int enable);
/* form 1's small levels (fewer than 8192 blocks of rows of 9..32 entries; env
 * AMG_JGS_SMALL), all bit-identical: 2 (default) the whole row's loads in one
 * batch, 1 one wave per block, 0 as the large levels */
int amg_set_jgs_small(amg_ctx *ctx, int form);
/* FULL_ASYNC / READ_SOL: level 0's correction added into the shared iterate by
 * the last hybrid-JGS sweep's write-out itself (jgs forms 1 and 3; env
 * AMG_JGS_FOLD), in place of the separate update pass after the smoothing
 * (SMEM_Async_AMG.cpp:284-301); bit-identical under a schedule, measured
 * neutral; default off */
int amg_set_jgs_fold(amg_ctx *ctx, int enable);
int amg_hybrid_jgs(amg_ctx *ctx, const amg_mat *A, const amg_vec *f, amg_vec *u, amg_vec *u_prev,
                   const int *blk, int nblk, const amg_vec *diag_scale, double weight, int sweeps,
                   int zero_first, int reverse);
/* forward Gauss-Seidel: SEQ_GaussSeidel SEQ_Smooth.cpp:89-117 */
int amg_gauss_seidel(amg_ctx *ctx, const amg_mat *A, const amg_vec *f, amg_vec *u, int sweeps);
/* asynchronous Gauss-Seidel over row blocks blk[0..nblk]: SMEM_Async_Parfor_GaussSeidel[T]
 * SMEM_Smooth.cpp:164-220 and SMEM_Async_GaussSeidel[T] :475-531 (semi = 0: no
 * barrier between sweeps), SMEM_SemiAsync_Parfor_GaussSeidel :135-162 and
 * SMEM_SemiAsync_GaussSeidel :445-473 (semi = 1).  In place, racy across blocks
 * exactly like the reference; deterministic for nblk = 1.  reverse: the "T" forms. */
int amg_async_gauss_seidel(amg_ctx *ctx, const amg_mat *A, const amg_vec *f, amg_vec *u,
                           const int *blk, int nblk, int sweeps, int semi, int reverse);
/* 2-step symmetric Jacobi: variant 0 = SMEM_Sync_Symmetric[L1]Jacobi
 * SMEM_Smooth.cpp:643-762, variant 1 = SEQ_Symmetric[L1]Jacobi SEQ_Smooth.cpp:119-189;
 * l1 != NULL selects the L1 form */
int amg_sym_jacobi(amg_ctx *ctx, const amg_mat *A, const amg_vec *f, amg_vec *u, amg_vec *y,
                   amg_vec *r, double omega, const amg_vec *l1, int sweeps, int zero_first,
                   int rb, int re, int variant);
/* measurement helper: reps back-to-back y = A x launches on the context's
 * stream bracketed by HIP events; *ms = average device milliseconds per launch */
int amg_matvec_timed(amg_ctx *ctx, const amg_mat *A, const amg_vec *x, amg_vec *y, int reps,
                     double *ms);
/* measurement helpers (no reference counterpart): best-of-reps STREAM triad
 * a = b + q c over three fresh arrays of n doubles, *gbs = 24 n bytes / time
 * (the practical HBM ceiling bench.py reports beside the 8 TB/s peak); and one
 * PMC calibration stream over a fresh buffer of `bytes` bytes (mode 0/1/2/3:
 * reads with 16/8/4/1-byte lanes, 4: 8-byte writes) for rocprofv3 FETCH_SIZE /
 * WRITE_SIZE calibration (tools/pmc_traffic.py) */
int amg_stream_triad(amg_ctx *ctx, long long n, int reps, double *gbs);
int amg_pmc_calib(amg_ctx *ctx, int mode, long long bytes);
/* setup arrays: L1_row_norm SMEM_Setup.cpp:222-232, A_diag :234-237 */
int amg_l1_norms(amg_ctx *ctx, const amg_mat *A, amg_vec *out);
int amg_a_diag(amg_ctx *ctx, const amg_mat *A, double omega, amg_vec *out);

/* ---- hierarchy, cycles, solve driver ----------------------------------------- */
/* A[0..L-1], P[0..L-2], R[0..L-2] (R = explicit P^T, construct_R_flag = 1) */
int amg_hier_create(amg_ctx *ctx, int num_levels, amg_mat *const *A, amg_mat *const *P,
                    amg_mat *const *R, const amg_opts *opts, amg_hier **out);
int amg_hier_free(amg_hier *H);
/* Geometric transfers: bit 0 set when the hierarchy runs level 0's residual
 * and restriction as one fused kernel (SMEM_Sync_AMG.cpp:44-60's SMEM_Residual
 * + SMEM_Restrict pair); bit l + 1 when level l's R_l / P_l equal, entry for
 * entry (checked on the device at creation), the linear-interpolation
 * transfers of level l's box -- level 0's box from the plane-marched A_0
 * (amg_mat_plane_march), each next level's halved -- and run as geometric
 * restriction / prolongation kernels.  Bit-identical to the CSR kernels.
 * amg_set_fuse_transfer(ctx, 0) (env AMG_FUSE_TRANSFER=0) keeps the CSR path
 * for hierarchies created afterwards. */
int amg_hier_fused(const amg_hier *H);
int amg_set_fuse_transfer(amg_ctx *ctx, int enable);
/* Prolongation fused into the post-smoothing sweep: bit l set when level l's
 * up-phase runs SMEM_Sync_SpGEMV(P_l, e, u, 1, 1, u) and the first Jacobi /
 * L1 Jacobi post sweep (SMEM_Sync_AMG.cpp:118-134, SMEM_Smooth.cpp:35-45,
 * 122-130) as one plane-marching pass that forms u + P e in registers (level
 * l geometric and its A_l 7-pt marched).  Bit-identical to the two kernels.
 * Off by default (measured 1.79 ms against 0.48 + 0.65 ms for the two kernels
 * at 512^3: the register-formed operands make it VALU-bound);
 * amg_set_fuse_prolong(ctx, form) (env AMG_FUSE_PROLONG) turns it on for
 * hierarchies created afterwards: 1 four lines per workgroup, 3 two, 2 one
 * (coarse values gathered per operand); 4 / 5 two / four lines with the
 * coarse correction read from an LDS ring of coarse planes (levels whose
 * lines are multiples of 512 points only). */
int amg_hier_fused_prolong(const amg_hier *H);
/* level 0's last post-smoothing sweep and the outer residual + the next
 * cycle's first sweep as ONE plane march (weighted Jacobi MULT solves with
 * reuse_outer_residual on a 7-pt master-form A0 whose lines are 512 long):
 * mode 0 off, 1 on (u' written every step), 2 on with u' written only in the
 * last step of each amg_solve_iterate batch (the steps before consume it in
 * registers); 3: the two sweeps as ordinary marches slab by slab over z
 * (amg_set_outer_slab planes each), the second reading u' and f back from the
 * Infinity Cache, u' written as in mode 2 (any plane-marched A0 whose planes
 * are multiples of 256 rows, Jacobi or L1 Jacobi); bit-identical to the two
 * marches.  AMG_FUSE_OUTER sets it too. */
int amg_set_fuse_outer(amg_ctx *ctx, int mode);
/* planes per z-slab of fuse_outer mode 3 (default 32; env AMG_OUTER_SLAB) */
int amg_set_outer_slab(amg_ctx *ctx, int planes);
/* long-row CSR kernel (operators of >= 64 entries per row: classical coarse
 * levels, smoothed transfers; SMEM_MatVec.cpp:123-259): form 0 workgroup
 * chunks with one summing wave, 1 / 2 wave-independent chunks of 8 / 16
 * entries per lane; xcd: XCD-contiguous row blocks (forms 1, 2).  Every form
 * adds each row's rounded products in CSR order: bit-identical.  Env
 * AMG_LONG_FORM / AMG_LONG_XCD. */
int amg_set_long_form(amg_ctx *ctx, int form, int xcd);
/* the fused post sweep + outer residual mode this hierarchy runs (0: not fused) */
int amg_hier_fused_outer(const amg_hier *H);
int amg_set_fuse_prolong(amg_ctx *ctx, int enable);
/* lines per lane of the 7-pt plane march (1, 2 or 4; env AMG_MZ_LINES for the
 * sweeps and residuals, AMG_MZ_LINES_GEMV for SpMV / SpGEMV; defaults 1 and 2):
 * a lane keeps adjacent lines, their +-S operands from registers (planes whose
 * line length is a multiple of 512 and line count a multiple of the lines).
 * Bit-identical; takes effect on the next launch; sets both. */
int amg_set_march_lines(amg_ctx *ctx, int lines);
/* the SpMV / SpGEMV lines alone */
int amg_set_march_lines_gemv(amg_ctx *ctx, int lines);
/* plane-march scheduling (MI355X tuning, no reference counterpart; env
 * AMG_MZ_PF, AMG_MZ27_PF, AMG_MZ_OCC, AMG_MZ27_OCC): prefetch distance in planes
 * of the 7-pt / 27-pt march (1 or 2; 7-pt 3: distance 1 with the +-S /
 * wave-edge / pattern / right-hand-side operands loaded a plane ahead, AMG_MZ_HPF;
 * defaults 3 / 2) and chunking by occupancy
 * (-1: whole rounds of the kernel's resident workgroups, 0: the planes-per-chunk
 * rule of amg_set_plane_march, > 0: that many workgroups per CU; defaults 0 /
 * -1, automatic chunking only).  Bit-identical in every setting; -2 keeps a
 * value. */
int amg_set_march_tuning(amg_ctx *ctx, int mz_pf, int mz27_pf, int mz_occ, int mz27_occ);
/* hipGraphs of the additive cycles' launch-bound loops (MI355X, no reference
 * counterpart; env AMG_GRAPHS): the synchronous additive cycle of amg_solve and
 * each level's correction of amg_async_solve (FULL_ASYNC, READ_SOL, LOCAL
 * residuals, no delays, no profiling) are captured after one eager run and
 * replayed; the same kernels with the same arguments, bit-identical.  Off by
 * default; the graphs are dropped when the hierarchy's options or blocks change. */
int amg_set_graphs(amg_ctx *ctx, int enable);
int amg_hier_set_opts(amg_hier *H, const amg_opts *opts);
/* override level `level`'s hybrid-JGS block partition (thread.A_ns/A_ne) */
int amg_hier_set_blocks(amg_hier *H, int level, const int *blk, int nblk);
#define AMG_VEC_F 0
#define AMG_VEC_U 1
#define AMG_VEC_R 2
int amg_hier_vec(amg_hier *H, int which, int level, amg_vec **out);
/* SMEM_Solve SMEM_Solve.cpp:11-262 (sync branch: SMEM_Sync_Parfor_Vcycle
 * SMEM_Sync_AMG.cpp:8-145 for MULT, SMEM_Sync_Add_Vcycle :408-621 for MULTADD /
 * AFACX, Chebyshev update :169-188).  reshist[0..cycles] (may be NULL). */
int amg_solve(amg_hier *H, const amg_vec *f, amg_vec *u, double *reshist, int *cycles_done);
/* split form of amg_solve for timed loops: start = InitSolve + initial
 * residual (returns ||r0||); iterate enqueues k outer iterations (cycle,
 * Chebyshev, residual + norm into a device history) with no host sync;
 * get_u copies the current iterate out */
int amg_solve_start(amg_hier *H, const amg_vec *f, const amg_vec *u, double *r0norm);
int amg_solve_iterate(amg_hier *H, int k);
int amg_solve_get_u(amg_hier *H, amg_vec *u);
/* ||r||_2 of the current outer residual (host sync) */
int amg_solve_resnorm(amg_hier *H, double *out);
/* asynchronous additive AMG: SMEM_Async_Add_AMG SMEM_Async_AMG.cpp:7-437
 * (ASYNC_MULTADD / ASYNC_AFACX, LOCAL convergence: every level performs
 * num_cycles corrections on its own stream).  level_corrections[L] out. */
int amg_async_solve(amg_hier *H, const amg_vec *f, amg_vec *u, int *level_corrections,
                    double *relres);
/* per level of the last amg_async_solve (free race): milliseconds from the
 * solve's start to the level's last correction (HIP events on the level
 * streams; 0 for levels without a group or under a deterministic schedule);
 * ms holds L entries.  ms[k] / corrections[k] is the level's measured
 * correction time, the input of AMG_SCHED_TIMED. */
int amg_async_level_ms(const amg_hier *H, double *ms);
/* AMG_SCHED_TIMED: level k's time per correction (ms[0..L-1], > 0) */
int amg_hier_set_async_durations(amg_hier *H, const double *ms, int n);
/* AMG_SCHED_TIMED replaying recorded end times: level k's j-th correction ends
 * at t[n[0] + .. + n[k-1] + j] (past n[k] entries its last interval repeats);
 * nlev >= L */
int amg_hier_set_async_times(amg_hier *H, const double *t, const int *n, int nlev);
/* end times (ms from the solve's start, HIP events on the level streams) of
 * level `level`'s corrections in the last free-race amg_async_solve: *count
 * corrections, the first min(count, cap) written to ms */
int amg_async_correction_ms(const amg_hier *H, int level, double *ms, int cap, int *count);
/* the actual execution windows of the same corrections' update kernels (the
 * kernel that adds the correction into the shared iterate / residual stamps
 * its workgroups' first start and last end on the device wall clock): end
 * (cap >= 0) or start (cap < 0, -cap entries) in ms of that clock, an origin
 * common to every stream and process on the device; NaN where not stamped */
int amg_async_update_windows(const amg_hier *H, int level, double *ms, int cap, int *count);
/* the per-row update times of correction `corr` of level `level` in the same race (ms on
 * the windows' clock: when row i's add into the shared vector and its read-back
 * completed); *count = the fine rows written (at most cap), 0 where not recorded (rows are
 * stamped while rows x levels x corrections x 20 B stays within 512 MiB); cap < 0: the
 * 2 n values (old, new) of every row's add instead, -cap entries (NaN where not recorded) */
int amg_async_update_rows(const amg_hier *H, int level, int corr, double *ms, int cap, int *count);
/* EigsPower SMEM_Cheby.cpp:410-518 with this hierarchy's V-cycle as M^{-1} */
int amg_eigs_power(amg_hier *H, int iters, double *eig_max, double *eig_min);
/* profile: accumulated device milliseconds and launch counts of the fine-level
s * kernels since the last reset: [0] level-0 residual in the cycle, [1] level-0
 * smoother sweeps, [2] R_0 restriction, [3] P_0 prolongation, [4] outer residual
 * (+ fused next pre-sweep when reuse_outer_residual) */
int amg_hier_profile_read(amg_hier *H, double *ms, long long *launches, int reset);

/* ---- structured problem generator (replaces SMEM_BuildMatrix/BoomerAMGSetup
 * inputs for -problem 7pt; BuildHypreMatrix.cpp:250-275) ---------------------- */
#define AMG_INTERP_LINEAR 0
#define AMG_INTERP_AGGREGATE 1
#define AMG_GEN_A 0
#define AMG_GEN_P 1
#define AMG_GEN_R 2
int amg_gen_create(int nx, int ny, int nz, int interp, int max_levels, int max_coarse,
                   amg_gen **out);
int amg_gen_free(amg_gen *g);
int amg_gen_num_levels(const amg_gen *g);
int amg_gen_dims(const amg_gen *g, int level, int *nx, int *ny, int *nz);
/* rows of z-planes [z0,z1) of operator `which` at `level` (P/R: the fine /
 * coarse grid of that level), global column ids, rowptr starting at 0 */
long long amg_gen_nnz(const amg_gen *g, int which, int level, int z0, int z1);
int amg_gen_fill(const amg_gen *g, int which, int level, int z0, int z1, int *rowptr, int *col,
                 double *val, int nthreads);
/* same, generated directly in device memory and registered */
int amg_gen_register(amg_ctx *ctx, const amg_gen *g, int which, int level, int z0, int z1,
                     amg_mat **out);
/* ---- in-house classical AMG setup (replaces HYPRE_BoomerAMGSetup,
 * SMEM_Setup.cpp:55-70 / DMEM_Setup.cpp:169-173, on the host).  hypre is not in
 * the reference tree: its published algorithms are restated, parity with
 * hypre's own hierarchies is unpinned.  Levels hold host CSR (A diagonal first,
 * P with sorted columns, R = P^T) until amg_classical_free. ------------------ */
#define AMG_COARSEN_PMIS 8        /* hypre coarsen_type 8                      */
#define AMG_COARSEN_PMIS_FIXED 9  /* 9: PMIS with a fixed random sequence (DMEM) */
#define AMG_COARSEN_HMIS 10       /* 10 (SMEM default)                         */
#define AMG_CLASSICAL_DIRECT 3    /* hypre interp_type 3: direct               */
#define AMG_CLASSICAL_EXT_I 6     /* interp_type 6: extended+i (both drivers)  */
typedef struct amg_classical amg_classical;
typedef struct {
   int coarsen_type;        /* hypre.coarsen_type (SMEM_Main.cpp:30, DMEM_Main.cpp:41) */
   int interp_type;         /* hypre.interp_type                                  */
   double strong_threshold; /* hypre.strong_threshold (SMEM 0.25, DMEM 0.5)        */
   double max_row_sum;      /* HYPRE_BoomerAMGSetMaxRowSum (1.0: no row-sum test)  */
   int max_levels;          /* hypre.max_levels                                   */
   int max_coarse_size;     /* stop when a level has at most this many rows       */
   int num_functions;       /* hypre.num_functions: unknowns per node (dof i % k)  */
   unsigned long long seed; /* PMIS random measure                                */
   int device;              /* >= 0: the Galerkin products A P and R (A P) run on this
                               GPU (amg_spgemm.hip: one lane per row, the host's
                               Gustavson order -- bit-identical); -1: on the host */
} amg_classical_opts;
void amg_classical_opts_default(amg_classical_opts *o); /* the SMEM parameters */
int amg_classical_setup(const amg_classical_opts *o, int n, const int *rowptr, const int *col,
                        const double *val, amg_classical **out);
int amg_classical_levels(const amg_classical *h);
/* operator which (AMG_GEN_A/P/R) of a level: sizes and pointers into h */
int amg_classical_get(const amg_classical *h, int which, int level, int *nrows, int *ncols,
                      long long *nnz, const int **rowptr, const int **col, const double **val);
/* register it on the device (amg_csr_register) */
int amg_classical_register(amg_ctx *ctx, const amg_classical *h, int which, int level, amg_mat **out);
/* C/F splitting of a level (1 = C, -1 = F) */
int amg_classical_cf_marker(const amg_classical *h, int level, int *cf);
int amg_classical_free(amg_classical *h);

/* ---- DMEM elasticity problem (config 5; replaces DMEM_BuildMfemMatrix,
 * DMEM_BuildMatrix.cpp:442-719, which assembles it with MFEM -- restated, parity
 * unpinned): beam-hex [0,8]x[0,1]^2 refined `refine` times, Q1 vector H1 byVDIM
 * (dof = 3 node + component), lambda = mu = 1 (x50 on the first half), x = 0
 * fixed, pull -1e-2 in z on x = 8.  Host CSR (diagonal first) + load vector. */
typedef struct amg_elast amg_elast;
int amg_elast_create(int refine, amg_elast **out);
int amg_elast_get(const amg_elast *e, int *n, long long *nnz, const int **rowptr, const int **col,
                  const double **val, const double **rhs);
int amg_elast_free(amg_elast *e);

/* RHS: RandDouble(lo,hi) after srand(0) (SMEM_Setup.cpp:1729-1745), rows [r0,r1) of the global sequence */
int amg_rhs_rand(long long r0, long long r1, double lo, double hi, double *out);

/* ---- multi-GPU (one process per GPU) ------------------------------------------
 * Replaces the DMEM_* communication of the reference (DMEM_Comm.cpp:81-382
 * SendRecv/CompleteRecv, the hypre ParCSR halo exchange inside
 * hypre_ParCSRMatrixMatvec called from DMEM_Add.cpp:230-308, and the
 * InnerProdFlag allreduce DMEM_Misc.cpp:414-433).  Every level is split into
 * contiguous row ranges (z-plane slabs for the structured problem); each SpMV exchanges its ghost rows point-to-point over RCCL
 * (xGMI) on a communication stream while the slab interior is computed on the
 * compute stream.  Levels below a size threshold are replicated on every rank
 * (one allgather of the restricted residual per cycle) so the coarse cycle
 * needs no communication.  Per-row summation order is unchanged, so iterates
 * are bit-identical to the single-GPU solve. */
int amg_dist_unique_id_size(void);
int amg_dist_get_unique_id(char *id);                 /* rank 0, then broadcast the bytes */
int amg_dist_init(amg_ctx *ctx, int nranks, int rank, const char *id); /* RCCL communicator */
/* test transport: exchanges go through host memory and a user callback
 * (lets several ranks share one GPU); op 0 = point-to-point (send[i] to
 * peers[i], recv[i] from peers[i]), 1 = allreduce-sum of ndouble doubles in
 * recv[0], 2 = allgather of equal-size byte blocks (send[0] -> recv[0]) */
typedef int (*amg_host_xchg_fn)(void *user, int op, int npeers, const int *peers,
                                const void *const *send, const long long *send_bytes,
                                void *const *recv, const long long *recv_bytes);
int amg_dist_init_host(amg_ctx *ctx, int nranks, int rank, amg_host_xchg_fn fn, void *user);
int amg_dist_finalize(amg_ctx *ctx);
int amg_dist_allreduce_sum(amg_ctx *ctx, double *host_vals, int n);
int amg_dist_barrier(amg_ctx *ctx);
typedef struct amg_dist_hier amg_dist_hier;
/* one rank's rows of a distributed operator: local rows, GLOBAL column ids of
 * the operator's column level (what a hypre_ParCSRMatrix's diag + offd with
 * col_map_offd describe, DMEM_Setup.cpp:169-173); diagonal first in A rows */
typedef struct amg_csr_part {
   int nrows;
   long long nnz;
   const int *rowptr; /* [nrows + 1], 0 .. nnz */
   const int *col;    /* [nnz] global column ids */
   const double *val; /* [nnz] */
} amg_csr_part;
/* distributed hierarchy from per-rank CSR pieces (the ParCSR row partition:
 * row_starts[l * (nranks + 1) + r] = first global row of rank r on level l,
 * hypre_ParCSRMatrixRowStarts).  A[l]: rows of level l; P[l]: rows of level l,
 * columns of level l+1; R[l]: rows of level l+1, columns of level l.  Levels
 * with fewer than replicate_rows rows are gathered and replicated. */
int amg_dist_hier_create(amg_ctx *ctx, int num_levels, const long long *row_starts,
                         const amg_csr_part *A, const amg_csr_part *P, const amg_csr_part *R,
                         const amg_opts *opts, amg_dist_hier **out);
/* the same for the structured problem, built slab by slab from the generator:
 * level-0 z-planes split evenly, coarse plane k owned by the owner of fine
 * plane 2k+1 */
int amg_dist_hier_create_structured(amg_ctx *ctx, const amg_gen *gen, const amg_opts *opts,
                                    amg_dist_hier **out);
/* the z-slab form of the same partition (config 4's path): every distributed
 * level's operators are the rank's extended slab operators (owned planes plus
 * up to two ghost planes each side), so the single-GPU kernels run on them --
 * plane-marched 7-pt / 27-pt sweeps and residuals over the owned planes,
 * geometric restriction / prolongation, the fused level-0 residual +
 * restriction -- and the ghost exchange is whole contiguous planes with the
 * two neighbouring ranks (RCCL send/recv on the communication stream,
 * overlapped with the planes that read no ghost).  Rows keep their global
 * entry order: iterates are bit-identical to one GPU.  Needs >= 2 level-0
 * planes per rank; levels where a rank would own < 2 planes (or below the
 * replication threshold) are replicated.  Serves amg_dist_solve_* and
 * amg_dist_async_solve (replaces the ParCSR halo of hypre_ParCSRMatrixMatvec,
 * DMEM_Add.cpp:230-308, and the finestIntra exchange, DMEM_Comm.cpp:81-348);
 * amg_dist_async_jacobi / _sps and amg_grid_add_* need the row-partitioned forms. */
int amg_dist_hier_create_slab(amg_ctx *ctx, const amg_gen *gen, const amg_opts *opts, amg_dist_hier **out);
/* slab hierarchy facts: distributed levels, bitmask of levels whose transfers run
 * the geometric kernels, 1 if level 0 runs the fused residual + restriction */
int amg_dist_hier_slab_info(const amg_dist_hier *D, int *distributed_levels, int *geometric, int *fused);
/* that partition (host only, no device): row_starts[l * (nranks + 1) + r] */
int amg_dist_structured_row_starts(const amg_gen *gen, int nranks, long long *row_starts);
/* levels with fewer rows than this are replicated on every rank (default 2^18) */
int amg_dist_hier_set_replicate_rows(amg_ctx *ctx, long long rows);
int amg_dist_hier_free(amg_dist_hier *D);
/* this rank's operator of a level: stored entries and storage format (value-index
 * table size, dictionary size, row patterns; 0 = not used) */
int amg_dist_hier_matrix_info(amg_dist_hier *D, int level, long long *nnz, int *value_index,
                              int *dict_index, int *row_pattern);
/* distinct row-pair patterns of this rank's operator of a level (0 = not pair-coded) */
int amg_dist_hier_pair_pattern(amg_dist_hier *D, int level, int *pair_pattern);
/* rows [row0, row0 + nrows) of the global level-0 vector this rank owns */
int amg_dist_hier_local_rows(amg_dist_hier *D, int level, int *row0, int *nrows);
/* SMEM_Solve on the distributed hierarchy: f/u are this rank's level-0 rows */
int amg_dist_solve_start(amg_dist_hier *D, const double *f_local, double *r0norm);
int amg_dist_solve_iterate(amg_dist_hier *D, int k);
int amg_dist_solve_resnorm(amg_dist_hier *D, double *out);
int amg_dist_get_u(amg_dist_hier *D, double *u_local);
int amg_dist_profile_read(amg_dist_hier *D, double *ms, long long *launches, int reset);
/* asynchronous additive AMG across GPUs (DMEM_Add DMEM_Add.cpp:20-178, AddCycle
 * :180-329, DMEM_AddCorrect_LocalRes :391-458; SMEM_Async_Add_AMG semantics):
 * hierarchy created with solver ASYNC_MULTADD or ASYNC_AFACX.  Every level runs
 * num_cycles corrections on its own HIP stream, adding into the shared slab of u
 * with fp64 atomics; the levels' compute overlaps, but their ghost exchanges and
 * the allgather to the replicated levels all run, in one cycle-major order, on
 * the rank's single communication stream over one communicator (RCCL requires
 * the same operation order on every rank, and per-level communicators on
 * streams sharing hardware queues can deadlock across ranks).  A level's
 * exchange in cycle c therefore waits for every exchange issued before it, each
 * waiting for its own level's compute: a slow level holds the others back at
 * their next exchange (head-of-line coupling; measured by
 * amg_dist_async_level_ms with delay_level).  u starts at zero; read it with
 * amg_dist_get_u.  *relres = ||f - A u|| / ||f|| after the levels joined. */
int amg_dist_async_solve(amg_dist_hier *D, const double *f_local, int *level_corrections,
                         double *relres);
/* per level of the last amg_dist_async_solve: milliseconds from the solve's
 * start to the level's last correction (HIP events; 0 for levels without a
 * correction group); ms holds L entries */
int amg_dist_async_level_ms(const amg_dist_hier *D, double *ms);
/* the last amg_dist_async_jacobi run of this rank: [0] the fraction of each
 * sweep's ghost-delta exchange window (comm stream) covered by the interior
 * product r -= A_diag e (compute stream), averaged over the sweeps; [1] the
 * exchange window, ms per sweep; [2] the interior product, ms per sweep;
 * [3] the fraction of the received deltas applied in the sweep they were sent
 * (device-resident channels; -1 otherwise); [4] deltas applied in a later
 * sweep; [5] ||r|| as kept incrementally (global); [6] ||f - A x|| (global):
 * equal to rounding when every delta was applied exactly once; [7] 1 when the
 * deltas went through the device-resident channels (amg_link.cpp); [8] host
 * ms per sweep a send waited for its channel slot (flow control; the
 * exchange window [1] starts at the first copy's issue, after that wait) */
int amg_dist_async_jacobi_stats(const amg_dist_hier *D, double *stats, int n);
/* the last amg_dist_async_jacobi's schedule on this rank: *count events of 5 doubles each, in
 * the order their work entered the compute stream -- {1, sweep, accel mode, om1, omd} the
 * relaxation update, {2, sweep} the interior product, {3, peer rank, delta index} one peer's
 * ghost delta applied, {4, sweep} every peer's deltas of that sweep applied (transport path);
 * the first min(count, cap) events written (0 events after an SPS run) */
int amg_dist_async_jacobi_log(const amg_dist_hier *D, double *events, int cap, int *count);
/* AMG_SCHED_TIMED on the distributed solve: level k's time per correction
 * (every rank passes the same values, so every rank issues the same order) */
int amg_dist_hier_set_async_durations(amg_dist_hier *D, const double *ms, int n);
/* amg_hier_set_async_times / amg_async_correction_ms for the distributed solve
 * (this rank's level streams) */
int amg_dist_hier_set_async_times(amg_dist_hier *D, const double *t, const int *n, int nlev);
int amg_dist_async_correction_ms(const amg_dist_hier *D, int level, double *ms, int cap, int *count);
int amg_dist_async_update_windows(const amg_dist_hier *D, int level, double *ms, int cap, int *count);
int amg_dist_async_update_rows(const amg_dist_hier *D, int level, int corr, double *ms, int cap, int *count);
/* DMEM_AsyncSmooth (DMEM_Smooth.cpp:16-313) with ASYNC_JACOBI (l1 = 0: u = r ./ (a_ii/omega))
 * or ASYNC_L1_JACOBI (l1 = 1): `sweeps` relaxations of the fine level in residual-update
 * form from x = 0; every relaxation sends its boundary deltas on the communication
 * stream while the compute stream updates the residual from the owned columns, and
 * applies neighbours' deltas once they have arrived (never waiting for them).  Read x
 * with amg_dist_get_u.  *relres = ||f - A x|| / ||f|| after all deltas are drained. */
/* -smoother async_sps (ASYNC_STOCHASTIC_PARALLEL_SOUTHWELL_JACOBI,
 * DMEM_Smooth.cpp:165-291): the asynchronous Jacobi above, where a rank relaxes
 * in a sweep only when a draw RandDouble(0,1) falls below the update probability
 * of its local residual L1 norm against the latest norms its neighbours sent
 * (carried with every delta message, DMEM_Comm.cpp:216-220,286-290): the first
 * sweep always relaxes.  The draws are the reference's RandDouble stream (glibc
 * rand() after srand(0), DMEM_Setup.cpp:1426, Misc.cpp:282-285), the same on
 * every rank; the decision is made on the device, so nothing waits on the host.
 * *relaxations (optional) = the sweeps this rank relaxed in.  No accel_type. */
int amg_dist_async_sps(amg_dist_hier *D, const double *f_local, int sweeps, double *relres,
                       long long *relaxations);
/* n draws low + (high - low) rand() / RAND_MAX after srand(seed), by the glibc
 * TYPE_3 additive feedback generator (Misc.cpp:282-285's RandDouble) */
int amg_rand_double_stream(unsigned seed, int n, double low, double high, double *out);
int amg_dist_async_jacobi(amg_dist_hier *D, const double *f_local, int sweeps, int l1,
                          double *relres);
/* y = A_0 x on the distributed fine operator (halo exchange + interior/boundary
 * split); *ms = average device milliseconds over reps */
int amg_dist_fine_spmv(amg_dist_hier *D, int reps, double *ms);

/* ---- level-grouped asynchronous additive solve (DMEM_Add) ------------------------ */
/* Ranks (one per GPU) split into grids, one per level k (DMEM_Add.cpp:20-944).
 * Every grid holds the whole fine problem row-partitioned among its ranks (an
 * amg_dist_hier created on a context whose transport spans the grid's ranks) and
 * computes level k's additive correction: restriction to level k,
 * DMEM_AddSmooth (u = f./s; v = A u; u = 2u + v./(-s)) or, on the coarsest grid,
 * an exact dense solve (hypre_GaussElimSolve), prolongation.  Corrections travel
 * between the ranks of different grids whose row ranges overlap as messages of
 * len + 2 doubles (data, done flag 0/1/2, spare), at most max_inflight per
 * destination in flight, accumulated while every slot is busy (SendRecv /
 * CheckInFlight / CompleteInFlight, DMEM_Comm.cpp:11-382); termination by
 * CheckConverge, AddResNorm's InnerProdFlag and AsyncRecvCleanup
 * (DMEM_Add.cpp:331-389, 829-944).  The messages go over a caller-supplied
 * non-blocking transport with MPI point-to-point semantics: */
typedef struct amg_nb_transport {
   void *user;
   /* post a send of n doubles to world rank peer; buf stays untouched until the
    * request completes (test / wait) */
   int (*isend)(void *user, int peer, int tag, const double *buf, long long n, long long *req);
   /* post a receive of n doubles from world rank peer into buf */
   int (*irecv)(void *user, int peer, int tag, double *buf, long long n, long long *req);
   int (*test)(void *user, long long req, int *done); /* MPI_Test: *done = 1 once complete */
   int (*wait)(void *user, long long req);            /* MPI_Wait */
   /* in-place sum of n doubles over the ranks of the caller's grid */
   int (*grid_allreduce)(void *user, double *vals, int n);
} amg_nb_transport;
typedef struct amg_grid_add amg_grid_add;
/* DMEM_Setup.cpp:1638-1735: ranks per grid from the levels' work fractions */
int amg_grid_partition(int num_procs, int num_grids, const double *frac_work, int *procs_per_grid);
/* rank_grid[world]: every rank's grid; rank_rows[2 world]: every rank's global fine
 * rows [start, end) in its own grid's partition.  D: this rank's share of its
 * grid's hierarchy (opts: solver ASYNC_MULTADD, num_cycles, tol, converge_test_type,
 * async_type, accel_type / cheby_grid, max_inflight, async_comm_save_divisor,
 * delay_*). */
int amg_grid_add_create(amg_dist_hier *D, int my_grid, int world_nranks, int world_rank,
                        const int *rank_grid, const long long *rank_rows, const amg_nb_transport *t,
                        amg_grid_add **out);
/* the same protocol over a host model grid (A = diag(diag); grid k corrects the
 * rows with global index % number of grids == k by u = weight r ./ diag):
 * protocol tests without a GPU */
int amg_grid_add_create_host(int nrows, const double *diag, double weight, const amg_opts *opts, int my_grid,
                             int world_nranks, int world_rank, const int *rank_grid,
                             const long long *rank_rows, const amg_nb_transport *t, amg_grid_add **out);
/* Device-resident correction messages (replaces the host transport's payload
 * path, DMEM_Comm.cpp:77-348's MPI_Isend / MPI_Irecv / MPI_Test of the correction
 * vectors): ranks are threads of one process; a hub matches every rank's posted
 * sends and receives per (source, destination) in order.  A message is the
 * sender's device slot: the receiver's accumulate kernel reads it in place
 * (peer access between the ranks' devices is the caller's) after its stream
 * waits for the slot's write on the sender's stream; a receive completes once
 * matched, a send once the receiver's read has run (events; no host staging,
 * no copy).  The message's done flag (0/1/2) travels as a host
 * word of the match.  rank_grid[world]: every rank's grid (InnerProdFlag sums
 * over a grid's ranks run on the hub as well). */
typedef struct amg_devhub amg_devhub;
int amg_devhub_create(int world_nranks, const int *rank_grid, amg_devhub **out);
int amg_devhub_free(amg_devhub *hub); /* after every grid_add using it is freed */
/* amg_grid_add_create with the hub as the messages' transport: accumulators,
 * in-flight slots and receive buffers in D's device pool */
int amg_grid_add_create_devhub(amg_dist_hier *D, int my_grid, int world_nranks, int world_rank,
                               const int *rank_grid, const long long *rank_rows, amg_devhub *hub,
                               amg_grid_add **out);
/* Device-resident messages across processes (one per GPU, or several on one GPU):
 * every send slot pool is mapped into its receiver once (hipIpcGetMemHandle /
 * hipIpcOpenMemHandle, the handles exchanged over t here -- all ranks call this
 * together).  Per message t carries a control pair (slot index, done flag), sent
 * once the slot's write has run, and an acknowledgement back once the
 * receiver's kernel has read the slot in place; the send completes with the
 * acknowledgement.  The payload never leaves device memory. */
int amg_grid_add_create_ipc(amg_dist_hier *D, int my_grid, int world_nranks, int world_rank,
                            const int *rank_grid, const long long *rank_rows, const amg_nb_transport *t,
                            amg_grid_add **out);
/* DMEM_Add, asynchronous branch: b / x (in: x0, out: x) are this rank's rows of
 * its grid's partition; *cycles = cycles run, *relres = ||b - A x|| / ||b - A x0||
 * over the grid after AsyncRecvCleanup, messages[2] = sent, received */
int amg_grid_add_solve(amg_grid_add *G, const double *b_local, double *x_local, int *cycles, double *relres,
                       long long *messages);
/* number of outside send / receive peers (the overlapping ranks of other grids) */
int amg_grid_add_peers(const amg_grid_add *G, int *nsend, int *nrecv);
/* IPC mode: a rank's slot pools live in its hierarchy D's allocations and are
 * mapped by its receivers -- every rank must free its grid_add (which closes the
 * handles it opened) before ANY rank frees its amg_dist_hier (a barrier between
 * the two, as tests/test_gpu_grid_ipc.py does).  amg_opts.async_schedule =
 * AMG_SCHED_ROUND_ROBIN (device hub, one rank per grid): the grids take turns at
 * the oracle's or_dmem_add points -- bit-identical to it. */
int amg_grid_add_free(amg_grid_add *G);

/* ---- binary triplet matrix files (-problem file) ------------------------------ */
/* records {int32 i, int32 j, double val} (Triplet_AOS, Main.hpp:433-437), 1-based;
 * record 0 is the header (i = number of rows).  Rows come back assembled the way
 * hypre's IJ interface assembles them (a repeated column keeps its first position
 * and its last value; the diagonal first).  Host arrays owned by the caller:
 * release them with amg_host_csr_free. */
typedef struct amg_host_csr {
   int nrows, ncols;
   long long nnz;
   int *rowptr;
   int *col;
   double *val;
} amg_host_csr;
/* ReadBinary_fread_HypreParCSR (Misc.cpp:800-915; SMEM_Setup.cpp:1645-1653 reads
 * with symm = 1, remove_disconnected = 0): symm mirrors every off-diagonal record */
int amg_triplet_read(const char *path, int symm, int remove_disconnected, amg_host_csr *out);
/* ParReadBinary_fread (DMEM_BuildMatrix.cpp:1488-1560): a rank's file of its own rows
 * (zero values skipped); *first_row = the first global row (0-based) */
int amg_triplet_read_part(const char *path, int ncols, int *first_row, amg_host_csr *out);
/* PrintCSRMatrix (Misc.cpp:753-797): header, then (row, col, value) per entry */
int amg_triplet_write(const char *path, int nrows, int ncols, const int *rowptr, const int *col,
                      const double *val, int binary);
/* TextToBin (TextToBin.cpp:5-39): "row col value" lines to binary records */
int amg_triplet_text_to_bin(const char *in_path, const char *out_path);
void amg_host_csr_free(amg_host_csr *M);

#ifdef __cplusplus
}
#endif
#endif
