/*
 * mpcqp.h -- C ABI of the MI355X-native batched MPC-QP engine (libmpcqp.so).
 *
 * Drop-in boundary for the reference's per-tick control step
 * (Fleming-Sung/mpc-limX-control: MPC -> mpcQP -> QPSolver).  Plain pointers and sizes only;
 * every function returns an int status (MPCQP_OK == 0) and never prints or throws.
 * All compute runs as HIP kernels on gfx950; there is no CPU fallback: without a usable
 * device every compute entry point returns MPCQP_ERR_NO_DEVICE.
 *
 * Matrix layout: column-major (what Eigen's `.data()` hands out), unless stated otherwise.
 *
 * Entry point                     replaces (reference file:line)
 * ------------------------------  ------------------------------------------------------------
 * mpcqp_discretize                QPSolver::discretizeSystem   src/QPSolver.cpp:21-29
 *                                 (declared include/QPSolver.h:19)
 * mpcqp_discretize_quadrature     linear_mpc_example discretizeSystem
 *                                 src/linear_mpc_example.cpp:35-46
 * mpcqp_build_qp                  QPSolver::buildQPParams      src/QPSolver.cpp:31-81
 *                                 (declared include/QPSolver.h:22-25)
 * mpcqp_solve_dense               QPSolver::solveQP            src/QPSolver.cpp:83-106
 *                                 (qpOASES::QProblem::init + getPrimalSolution, :87-104;
 *                                 declared include/QPSolver.h:28-31)
 * mpcqp_plant_step                QPSolver::updateState        src/QPSolver.cpp:108-111
 * mpcqp_ctx_create / _destroy     (new) owns device buffers + stream for the batched path
 * mpcqp_batch_condense            mpcQP::buildSystemModel + QPSolver::discretizeSystem +
 *                                 QPSolver::buildQPParams, batched (include/mpcQP.h:51-102,
 *                                 121-182; src/QPSolver.cpp:21-81)
 * mpcqp_batch_solve_qp            QPSolver::solveQP, batched (src/QPSolver.cpp:83-106)
 * mpcqp_batch_solve               mpcQP::mpcQP ctor end to end (include/mpcQP.h:35-119),
 *                                 i.e. the intended MPC::computeSupportFootForce
 *                                 (include/MPCController.h:178-180), batched
 * mpcqp_batch_discretize          mpcQP::buildSystemModel + QPSolver::discretizeSystem,
 *                                 batched -> [Ad | Bd] per instance
 * mpcqp_batch_condense_solve      QPSolver::buildQPParams + QPSolver::solveQP, batched, fused
 *                                 (H never leaves the chip)
 * mpcqp_batch_select_min          (new) per-rank min-cost key for the multi-GPU selection
 * mpcqp_batch_select_record       (new) per-rank selection record [key | winner's U] for the
 *                                 one-collective multi-GPU selection
 * mpcqp_reduce_records            (new) global winner from the all-gathered records
 * mpcqp_batch_solve_select        mpcqp_batch_solve + mpcqp_batch_select_record in one pass:
 *                                 the per-tick step of MPC::computeSupportFootForce over C
 *                                 candidates (include/MPCController.h:178-180) with its choice
 * mpcqp_batch_solve_gait          mpcQP::mpcQP xref (include/mpcQP.h:74-97) + MPC::calculateGait
 *                                 (include/MPCController.h:61-75) on device, then the fused step
 * mpcqp_batch_select_state        (new) best gait candidate per state
 * mpcqp_batch_plant_srbm          QPSolver::updateState (src/QPSolver.cpp:108-111), SRBM, batched
 * mpcqp_rollout                   the closed loop of src/qpSolver_test.cpp:38-90, batched
 * mpcqp_set_warm_start            QPSolver::updateState -> next solveQP hot-started from the
 *                                 previous active set (src/QPSolver.cpp:87-111), batched
 * mpcqp_fk_feet                   PinocchioKinematics::forwardKinematics + getLinkPosition
 *                                 (include/pinocchio_kinematics.h:30-43), batched
 * mpcqp_ctx_fk_feet_host          the same, host pointers (mpcQP::buildSystemModel's FK,
 *                                 include/mpcQP.h:125-137)
 * mpcqp_ctx_reserve               (new) pre-sizes the context's buffers (no allocation per tick)
 * mpcqp_kf_update                 stateEstimator::update (include/stateEstimator.h:217-337),
 *                                 batched
 * mpcqp_group_*, mpcqp_shard      (new) the batch over the GPUs of a node with one RCCL
 *                                 all-gather per step, for the C++ control loop
 *                                 (src/mpc_control_fake_state.cpp:108-149)
 */
#ifndef MPCQP_H
#define MPCQP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes ------------------------------------------------------------------ */
#define MPCQP_OK 0
#define MPCQP_ERR_BAD_DIMS 1   /* dimensions outside the supported envelope            */
#define MPCQP_ERR_INFEASIBLE 2 /* QP has no feasible point (qpOASES: RET_INIT_FAILED..)*/
#define MPCQP_ERR_ITER_LIMIT 3 /* working-set iteration cap hit (qpOASES: nWSR)        */
#define MPCQP_ERR_NOT_PD 4     /* reduced Hessian not positive definite                */
#define MPCQP_ERR_DEVICE 5     /* HIP runtime error                                    */
#define MPCQP_ERR_BAD_ARG 6    /* null pointer / invalid flag                          */
#define MPCQP_ERR_NO_DEVICE 7  /* no HIP device visible                                */

#define MPCQP_INFTY 1e20 /* qpOASES::INFTY as used at src/QPSolver.cpp:72-73 */

/* ---- envelope ---------------------------------------------------------------------- */
#define MPCQP_MAX_NX 32
#define MPCQP_MAX_NU 16
#define MPCQP_MAX_N 32
#define MPCQP_MAX_NV 256   /* NU*N */
#define MPCQP_MAX_FREE 128 /* free (lb < ub) variables per solve: the batched fast path holds up
                            * to 6N (every contact schedule); mpcqp_solve_dense and the generic
                            * batched path hold 64 */

/* layout flag of the dense constraint matrix handed to mpcqp_solve_dense */
#define MPCQP_A_ROWMAJOR 0 /* qpOASES's convention (what QProblem::init expects)      */
#define MPCQP_A_COLMAJOR 1 /* Eigen's storage (what the reference actually passes)    */

/* ---- single-instance, reference-compatible entry points (run on the GPU, batch 1) ---- */
int mpcqp_discretize(int nx, int nu, double Ts, const double *Ac, const double *Bc,
                     double *Ad, double *Bd);

/* linear_mpc_example's discretisation (src/linear_mpc_example.cpp:35-46): Ad = exp(Ac Ts),
 * Bd = sum_{i<100} Ad (I - Ac tau_i/100)^-1 Bc Ts/100 with tau_i = i Ts/100. */
int mpcqp_discretize_quadrature(int nx, int nu, double Ts, const double *Ac, const double *Bc,
                                double *Ad, double *Bd);

/* Outputs use the reference's exact layouts and sizes (nV = nu*N):
 *   H nV x nV, f nV, A_eq (nx*N) x nV, b_eq nx*N, lb/ub nV, A_ineq (2*nx*N) x nV,
 *   lbA/ubA 2*nx*N (zero rows carry -/+MPCQP_INFTY).  Any output pointer may be NULL. */
int mpcqp_build_qp(int nx, int nu, int N, const double *Ad, const double *Bd, const double *Q,
                   const double *R, const double *P, const double *x_min, const double *x_max,
                   double u_min, double u_max, const double *xi0, const double *xi_ref,
                   double *H, double *f, double *A_eq, double *b_eq, double *lb, double *ub,
                   double *A_ineq, double *lbA, double *ubA);

/* min 1/2 x'Hx + f'x  s.t.  lb <= x <= ub,  lbA <= A x <= ubA  (rows with lbA == ubA are
 * equalities; |bound| >= MPCQP_INFTY means absent).  Strictly convex only (H pos. def. on
 * the free variables).  *nWSR: in = iteration cap (<= 0: default), out = iterations used.
 * y (nullable, nV + nC): multipliers, qpOASES sign convention H x + f = y_b + A' y_A. */
int mpcqp_solve_dense(int nV, int nC, const double *H, const double *f, const double *A,
                      int a_layout, const double *lb, const double *ub, const double *lbA,
                      const double *ubA, int *nWSR, double *x, double *y, double *cost);

/* x <- Ad x + Bd u */
int mpcqp_plant_step(int nx, int nu, const double *Ad, const double *Bd, double *x,
                     const double *u);

/* ---- batched engine ------------------------------------------------------------------ */
#define MPCQP_MODEL_SRBM 0    /* convex-MPC single rigid body, 13 states, 6 inputs (2 feet) */
#define MPCQP_MODEL_LITERAL 1 /* reference mpcQP::buildSystemModel, 13 states, 3 inputs    */
#define MPCQP_MODEL_DENSE 2   /* any continuous model given per instance ([Ac | Bc] in lin),
                               * dense Q/R/P, input box u_min..u_max: the whole-body
                               * linearisation (BASELINE config E, 24/6/16)                 */
#define MPCQP_CONS_BOX 0      /* per-foot force box from the contact schedule              */
#define MPCQP_CONS_FRICTION 1 /* box + linearised friction pyramid |fx|,|fy| <= mu fz      */

typedef struct mpcqp_model {
    int nx, nu, N;           /* 13, 6 (SRBM) or 3 (LITERAL), horizon                         */
    int model;               /* MPCQP_MODEL_*                                                */
    int constraints;         /* MPCQP_CONS_*                                                 */
    double Ts;               /* sample time (include/mpcQP.h:37: 0.001)                      */
    double mass;             /* include/mpcQP.h:18: 9.585                                    */
    double mu;               /* friction coefficient (MPCQP_CONS_FRICTION)                   */
    double Ib[9];            /* body inertia, column-major (include/mpcQP.h:20-22)           */
    double fz_min, fz_max;   /* per-foot normal force box when in contact                    */
    double fxy_max;          /* per-foot tangential force box when in contact                */
    double u_min, u_max;     /* LITERAL model input box (include/mpcQP.h:59-60)              */
    const double *Q;         /* nx*nx state weight (host pointer, copied at create)          */
    const double *R;         /* nu*nu input weight                                           */
    const double *P;         /* nx*nx terminal weight                                        */
    int max_iter;            /* solver iteration cap per instance (<= 0: default)            */
    int max_free;            /* bound on free variables per instance (<= 0: nu*N)            */
} mpcqp_model;

/* Per-instance inputs (device pointers, instance-major = one contiguous record per QP):
 *   x0      [B][nx]          initial state  [rpy, p, omega, v, g]      (include/mpcQP.h:66-71)
 *   xref    [B][N+1][nx]     reference, column i = step i (Eigen col-major 13 x (N+1))
 *   lin     [B][8]           SRBM: {yaw, r_L xyz, r_R xyz, 0}; LITERAL: {dx, dy, dz, ...};
 *           [B][nx*(nx+nu)]  DENSE: [Ac | Bc] column-major (continuous time)
 *   contact [B]              uint64, bit 2k = left foot in contact at step k, 2k+1 = right
 *                            (SRBM only; nullable otherwise)
 * Outputs (device pointers):
 *   U [B][nu*N] (column-major nu x N: U_opt.col(0) = first nu entries), cost [B],
 *   status [B] (MPCQP_* per instance), iters [B].                                          */
typedef struct mpcqp_ctx mpcqp_ctx;

int mpcqp_ctx_create(const mpcqp_model *model, int device, mpcqp_ctx **out);
int mpcqp_ctx_destroy(mpcqp_ctx *ctx);
/* stream: a hipStream_t to run on (NULL = the HIP null stream); a fresh context runs on a
 * non-blocking stream of its own.  All batched calls are asynchronous on the context's
 * stream; mpcqp_sync waits for it. */
int mpcqp_set_stream(mpcqp_ctx *ctx, void *stream);
int mpcqp_sync(mpcqp_ctx *ctx);
/* Size every context-owned scratch buffer (host staging, overflow list, rollout buffers, the
 * generic path's [Ad|Bd] and H/f) for batches of up to B instances, so that no call on the
 * solve path allocates device memory afterwards (SURVEY.md 8b ownership: "no allocation on
 * the solve path after create").  Larger batches still work; they grow the buffers once. */
int mpcqp_ctx_reserve(mpcqp_ctx *ctx, int B);

/* 0 when the context runs the generic kernels; 1 when it runs the compile-time-dimension
 * fused kernel, one QP per wavefront (13/6/{10,20} SRBM, 13/3/{10,20} literal, diagonal Q and
 * P); 2 when it runs the fused kernel with two QPs per wavefront (N = 10, box bounds,
 * max_free <= 30: config B and the literal 13/3/10) */
int mpcqp_ctx_fast_path(const mpcqp_ctx *ctx);
/* free variables the one-wave fused kernel holds per instance (30 for the paired kernel, its NF
 * otherwise; 0 on the generic path): an instance with more goes to the overflow workgroup kernel
 * (bench.py counts the one-wave kernel's work over the instances it solved) */
int mpcqp_ctx_one_wave_nf(const mpcqp_ctx *ctx);
/* the overflow launch that follows the one-wave kernel on this context: 0 none (generic path,
 * dense model, or no instance can exceed the one-wave kernel), 1 k_mpc_list (one QP per
 * wavefront, a resident grid over the list: N = 10), 2 k_mpc_wg (one workgroup per QP) */
int mpcqp_ctx_overflow_kernel(const mpcqp_ctx *ctx);
/* the crash start of the context's kernels (a speculative primal-dual active-set start before the
 * dual loop): at most *kmax bounds per working set, *pmax working sets
 * before it falls back to the plain dual loop, for the one-wave kernel (the paired kernel) and
 * (*_wg) for the workgroup solver (overflow instances, the dense model; box-only problems);
 * 0 / 0 where the dual loop starts cold.  Reported iterations count its working sets. */
int mpcqp_ctx_crash_params(const mpcqp_ctx *ctx, int *kmax, int *pmax, int *kmax_wg,
                           int *pmax_wg);

/* Staged entry points (stage 1 / stage 2 below, mpcqp_batch_solve_qp): the stand-alone solve
 * holds 64 free variables per instance (more: per-instance status MPCQP_ERR_BAD_DIMS).  On a
 * MPCQP_MODEL_DENSE context with more than 64 inputs (every input is free there) they return
 * MPCQP_ERR_BAD_DIMS; mpcqp_batch_solve(_host / _select) serve such contexts (k_dense_wg).
 * A MPCQP_MODEL_LITERAL context needs u_min < u_max (mpcqp_ctx_create: MPCQP_ERR_BAD_ARG). */
/* stage 1: linearise + discretise.  AB [B][nx*(nx+nu)] = [Ad | Bd] column-major */
int mpcqp_batch_discretize(mpcqp_ctx *ctx, int B, const double *lin, double *AB);
/* stage 2: condense + solve from AB, fused (H stays on chip) */
int mpcqp_batch_condense_solve(mpcqp_ctx *ctx, int B, const double *AB, const double *x0,
                               const double *xref, const uint64_t *contact, double *U,
                               double *cost, int *status, int *iters);
/* full H [B][nV][nV] (column-major) and f [B][nV] of the whole QP (parity / inspection) */
int mpcqp_batch_condense(mpcqp_ctx *ctx, int B, const double *x0, const double *xref,
                         const double *lin, double *H, double *f);
int mpcqp_batch_solve_qp(mpcqp_ctx *ctx, int B, const double *H, const double *f,
                         const uint64_t *contact, double *U, double *cost, int *status,
                         int *iters);
/* stage 1 + stage 2 */
int mpcqp_batch_solve(mpcqp_ctx *ctx, int B, const double *x0, const double *xref,
                      const double *lin, const uint64_t *contact, double *U, double *cost,
                      int *status, int *iters);
/* Host-pointer convenience for controllers (one tick, B = 1 state x C candidates): copies the
 * host arrays (same layouts as above) into context-owned device buffers, runs
 * mpcqp_batch_solve and copies U/cost/status/iters back; synchronous.
 * Pageable arrays (and batches below 4,096) go through context-owned pinned staging: one host
 * memcpy and one DMA each way (small batches replay a captured HIP graph).  When every array is
 * page-locked (mpcqp_host_register / mpcqp_host_alloc) and B >= 4,096, the arrays are DMA'd
 * straight from and into the caller's memory, no memcpy, in chunks of >= 8,192 instances
 * pipelined over three streams (the copy-in of a chunk beside the solve of the previous one);
 * results are identical either way (MPCQP_HOST_DIRECT=0 at context creation: always stage). */
int mpcqp_batch_solve_host(mpcqp_ctx *ctx, int B, const double *x0, const double *xref,
                           const double *lin, const uint64_t *contact, double *U, double *cost,
                           int *status, int *iters);
/* Page-locked host memory for the host-pointer entry points (src/QPSolver.cpp:93-96 hands the
 * caller's own buffers to the solver; here the device reads them by DMA).  register / unregister
 * wrap an existing allocation (the caller keeps it alive while registered: unregister before
 * freeing it); alloc / free return new page-locked memory.  Registering is expensive (page
 * pinning): do it once per buffer, not per tick.  register needs a page-aligned p
 * (MPCQP_ERR_BAD_ARG otherwise) and should cover the buffer's whole pages: pinning works on
 * pages, and a page shared by two registrations (small heap arrays side by side) leaves the HIP
 * runtime a stale mapping that can fault a later copy.  mpcqp_host_alloc's memory qualifies. */
int mpcqp_host_register(void *p, size_t bytes);
int mpcqp_host_unregister(void *p);
int mpcqp_host_alloc(size_t bytes, void **p);
int mpcqp_host_free(void *p);

/* key = (order-preserving bits of (float)cost << 31) | (index_base + i), min over the batch,
 * written to *key (device int64).  Instances with status != OK never win.  The caller
 * reduces keys across ranks with one MIN all-reduce (RCCL).  One launch on the context's
 * stream, using a context-owned partial-key buffer: calls on one context must stay ordered
 * (the same stream, or a synchronisation after mpcqp_set_stream). */
int mpcqp_batch_select_min(mpcqp_ctx *ctx, int B, const double *cost, const int *status,
                           int64_t index_base, int64_t *key);
/* Selection record for the multi-GPU path: record [1 + nu*N] int64 (device) receives the
 * key of mpcqp_batch_select_min in record[0] and the winning instance's U row (nu*N doubles,
 * bit copies) in record[1..]; all zeros after the key 0x7fffffffffffffff when no instance is
 * valid.  Same launch and ordering rules as mpcqp_batch_select_min; index_base + B must fit
 * in 31 bits.  The ranks exchange records with ONE all-gather (RCCL), then each rank runs
 * mpcqp_reduce_records(ctx, n_ranks, gathered [n][1 + nu*N], best [1 + nu*N]) to pick the
 * minimum key's record on device: no host synchronisation, no second collective. */
int mpcqp_batch_select_record(mpcqp_ctx *ctx, int B, const double *cost, const int *status,
                              const double *U, int64_t index_base, int64_t *record);
int mpcqp_reduce_records(mpcqp_ctx *ctx, int n, const int64_t *records, int64_t *best);
/* mpcqp_batch_solve followed by mpcqp_batch_select_record, same arguments and results (the
 * record bit-identical), without the selection launch on the fused paths: every workgroup of
 * the solve kernel(s) mins its instances' keys into context-owned words and the batch's last
 * workgroup writes the record.  Same ordering rule as mpcqp_batch_select_min (calls on one
 * context stay on its stream).  Other contexts (generic path, dense model) run the two calls. */
int mpcqp_batch_solve_select(mpcqp_ctx *ctx, int B, const double *x0, const double *xref,
                             const double *lin, const uint64_t *contact, double *U, double *cost,
                             int *status, int *iters, int64_t index_base, int64_t *record);

/* ---- multi-GPU group: the batch sharded over devices, ONE RCCL collective per step --------
 * SURVEY.md 8b ("ownership": a context that owns the communicator) and 8e; the C++ caller is
 * the control loop of src/mpc_control_fake_state.cpp:108-149 (MPC::run ->
 * computeSupportFootForce, include/MPCController.h:183-196) at batch scale.  A group holds one
 * context per device it drives and an RCCL communicator over all ranks (xGMI between the GPUs
 * of one node).  Each step: every rank solves its shard -- contiguous whole states of C gait
 * candidates, mpcqp_shard -- with mpcqp_batch_solve_select, the ranks exchange the [key | U]
 * selection records with ONE ncclAllGather, and every rank reduces them on device
 * (mpcqp_reduce_records): the global minimum-cost instance (fp32 cost, lowest global index on
 * ties), on every rank, with no host synchronisation inside the step. */
#define MPCQP_GROUP_UID_BYTES 128
typedef struct mpcqp_group mpcqp_group;
/* contiguous shard of whole states for `rank` of `nranks` (host arithmetic, no device): the
 * first `total_states % nranks` ranks take one state more.  bench.py and mpcqp/dist.py use it. */
int mpcqp_shard(int total_states, int nranks, int rank, int *first_state, int *states);
/* one process driving `ndev` devices (ncclCommInitAll): ranks 0..ndev-1 = devices[0..ndev-1]
 * (distinct devices; MPCQP_ERR_BAD_ARG otherwise).  Test transport: with MPCQP_GROUP_LOOPBACK=1
 * in the environment no communicator is created, the all-gather is device copies between the
 * members' buffers and members may share a device (the multi-rank orchestration on one GPU;
 * never for production) */
int mpcqp_group_create(const mpcqp_model *model, int ndev, const int *devices, mpcqp_group **out);
/* one process per device (torchrun / MPI style): rank `rank` of `nranks` on `device`.  uid
 * (MPCQP_GROUP_UID_BYTES) comes from mpcqp_group_unique_id on one rank and is handed to every
 * rank by the caller's own channel; every rank must call this (it blocks until all have). */
int mpcqp_group_unique_id(unsigned char *uid);
int mpcqp_group_create_rank(const mpcqp_model *model, int device, int nranks, int rank,
                            const unsigned char *uid, mpcqp_group **out);
int mpcqp_group_destroy(mpcqp_group *g);
/* *local: devices this process drives; *nranks: ranks of the communicator; *first_rank: the rank
 * of local member 0 (local member i is rank first_rank + i) */
int mpcqp_group_info(const mpcqp_group *g, int *local, int *nranks, int *first_rank);
/* local member i's context (its device, stream and buffers; e.g. mpcqp_ctx_reserve, timing) */
mpcqp_ctx *mpcqp_group_ctx(mpcqp_group *g, int i);
/* One step on device pointers.  Per local member i (device of member i):
 *   B[i] instances with global index base[i] (x0 / xref / lin / contact / U / cost / status /
 *   iters as for mpcqp_batch_solve, pointer arrays indexed by member), best[i] [1 + nu*N] int64
 *   receives the global record (key, winner's U) -- the same on every rank.
 * Asynchronous: the solve runs on the member's context stream, the all-gather and the reduction
 * on the group's collective stream of that device, so this step's collective overlaps the next
 * step's solve.  best[i] is complete after mpcqp_group_sync, or, for work enqueued afterwards on
 * the member's context stream, after mpcqp_group_wait.  Records alternate between two buffers:
 * a step's solve waits (on device) for the all-gather two steps back, nothing else.
 * Inputs: the solve runs on the member's own (non-blocking) context stream, which nothing orders
 * after the caller's streams.  Inputs written by host copies must be complete (synchronised)
 * before the call; inputs produced on a device stream need mpcqp_group_wait_stream first.
 * Failure: arguments are checked before anything is enqueued (MPCQP_ERR_BAD_ARG, the group
 * unchanged).  A failure after that -- part-way through the step, when peer ranks may already
 * wait in its all-gather -- aborts the group's communicators (ncclCommAbort: the peers'
 * collectives fail instead of hanging) and leaves the group failed: this and every later call
 * but mpcqp_group_info / _failed / _destroy return MPCQP_ERR_DEVICE.  Destroy it on every rank
 * and create a new group. */
int mpcqp_group_solve_select(mpcqp_group *g, const int *B, const int64_t *base,
                             const double *const *x0, const double *const *xref,
                             const double *const *lin, const uint64_t *const *contact,
                             double *const *U, double *const *cost, int *const *status,
                             int *const *iters, int64_t *const *best);
/* make each member's context stream wait (on device) for its collective stream: results of the
 * steps issued so far are visible to work enqueued on the context streams afterwards */
int mpcqp_group_wait(mpcqp_group *g);
/* make local member i's context stream wait (on device) for the work enqueued so far on
 * streams[i] (a hipStream_t of member i's device; NULL = its null stream): call it before
 * mpcqp_group_solve_select when that stream produced the step's inputs (e.g. torch's current
 * stream), instead of a host synchronisation */
int mpcqp_group_wait_stream(mpcqp_group *g, void *const *streams);
/* 1 once a step failed part-way (see mpcqp_group_solve_select), else 0 */
int mpcqp_group_failed(const mpcqp_group *g);
/* wait on the host for every member's streams */
int mpcqp_group_sync(mpcqp_group *g);
/* Host-pointer form for a single-process group (mpcqp_group_create; every rank local): the global
 * batch of S states x C candidates (host arrays, the layouts of mpcqp_batch_solve) is split with
 * mpcqp_shard, staged through pinned buffers the group owns, solved and selected as above;
 * U / cost / status / iters come back for the whole batch and best_host [1 + nu*N] receives the
 * global record.  Synchronous. */
int mpcqp_group_solve_select_host(mpcqp_group *g, int S, int C, const double *x0,
                                  const double *xref, const double *lin, const uint64_t *contact,
                                  double *U, double *cost, int *status, int *iters,
                                  int64_t *best_host);

/* ---- device-generated inputs, per-state selection and the closed loop ---- *
 * SRBM fast-path contexts only.  S states x C gait candidates, instance b = s*C + c.
 *   state [S][13]   [rpy, p, omega, v, g]                      (include/mpcQP.h:66-71)
 *   feet  [S][6]    r_L, r_R: foot minus CoM, world frame
 *   cmd   [S][2]    yaw rate, forward speed of the reference  (include/mpcQP.h:75-76)
 *   phase [S*C]     gait phase of each candidate at horizon step 0 (s)
 * The kernel builds x0 = state, xref as mpcQP::mpcQP does (include/mpcQP.h:74-97), lin =
 * {yaw, r_L, r_R} and the contact mask of MPC::calculateGait (include/MPCController.h:61-75)
 * on chip, then runs the same fused step as mpcqp_batch_solve. */
int mpcqp_batch_solve_gait(mpcqp_ctx *ctx, int S, int C, const double *state, const double *feet,
                           const double *cmd, const double *phase, float swing, float stance,
                           double *U, double *cost, int *status, int *iters);
/* Warm start of the gait solves from the previous call's active sets (the closed loop,
 * SURVEY.md 8f row 2): on = 1 keeps each instance's final active set (bounds and friction rows
 * in the global input numbering) and seeds the next mpcqp_batch_solve_gait / mpcqp_rollout tick
 * with it, shifted by one horizon step; the Goldfarb-Idnani selection re-adds those constraints
 * first.  The optimum is unchanged (the QP is strictly convex); iteration counts differ from a
 * cold solve.  Every call resets the stored sets (the next tick starts cold).  One-wave fused
 * kernels only (13/6/20 and the literal 13/3/20); a paired-kernel context ignores it. */
int mpcqp_set_warm_start(mpcqp_ctx *ctx, int on);
/* best candidate of each state (status OK, fp32 cost, lowest index; best = -1 if none):
 * best [S], best_cost [S] (nullable), Ubest [S][nu*N] (nullable).  C <= 64. */
int mpcqp_batch_select_state(mpcqp_ctx *ctx, int S, int C, const double *cost, const int *status,
                             const double *U, int *best, double *best_cost, double *Ubest);
/* plant step with each state's chosen first-step forces: state <- Ad state + Bd u (exact ZOH of
 * the SRBM at the current state, QPSolver::updateState, src/QPSolver.cpp:108-111), feet moved
 * with the CoM (stance feet fixed in the world), phase[S*C] += Ts. */
int mpcqp_batch_plant_srbm(mpcqp_ctx *ctx, int S, int C, double *state, double *feet,
                           double *phase, const int *best, const double *Ubest);
/* K closed-loop ticks of solve_gait -> select_state -> plant_srbm on the ctx stream (the
 * qp_test / mpc_test loops, src/qpSolver_test.cpp:38-90, at batch scale).  traj [K][S][13] and
 * choice [K][S] (nullable) receive the state after each tick and the chosen candidate. */
int mpcqp_rollout(mpcqp_ctx *ctx, int S, int C, int K, double *state, double *feet,
                  const double *cmd, double *phase, float swing, float stance, double *traj,
                  int *choice);

/* ---- producers either side of the step, device pointers, async on
 * `stream` (a hipStream_t; NULL = the null stream) ----------------------------------------
 * Foot contact points of both 3-DoF legs, world frame relative to the base -> the `feet` of
 * mpcqp_batch_solve_gait.  q [R][6] = (abad, hip, knee) left then right; rpy with row stride
 * rpy_stride (3 for [R][3], 13 to read a state [R][13]).  Replaces Pinocchio FK
 * (include/pinocchio_kinematics.h:30-43); chain from MPCParam's kinematicValues
 * (include/MPCParam.h:13-38), at q = 0 equal to static_foot_offset_* (:64-72). */
int mpcqp_fk_feet(void *stream, int R, const double *q, const double *rpy, int rpy_stride,
                  double *feet);
/* Host-pointer form for controllers (MPC::computeSupportFootForce, one robot per tick): stages
 * q/rpy through the context's buffer, runs k_fk_feet on the context's stream, synchronous. */
int mpcqp_ctx_fk_feet_host(mpcqp_ctx *ctx, int R, const double *q, const double *rpy,
                           int rpy_stride, double *feet);
/* One step of stateEstimator::update (include/stateEstimator.h:217-337) for R robots:
 * xhat [R][12] (p, v, foot positions), P [R][144] (column-major) updated in place from
 * eePos/eeVel [R][6] (feet relative to the base), contact [R][2], quat [R][4] (x y z w),
 * acc [R][3] (IMU, body frame). */
int mpcqp_kf_update(void *stream, int R, double dt, double *xhat, double *P, const double *eePos,
                    const double *eeVel, const unsigned char *contact, const double *quat,
                    const double *acc);

/* duration of the last stage-1 (which = 0: discretize / generic condense) or stage-2
 * (which = 1: condense_solve / generic solve; the whole mpcqp_batch_solve) launch, HIP events on
 * the ctx stream (ms; -1 if none recorded).  On the fused path which = 2 times the one-wave kernel
 * alone (k_mpc_pair / k_mpc) and which = 3 the overflow workgroup kernel (k_mpc_wg) launched
 * after it.  Timing is off until enabled.  mpcqp_batch_solve_host does not feed these slots: its
 * step is replayed as a captured HIP graph, and an event record inside the capture would time the
 * capture, not the replay.  mpcqp_enable_timing creates its events all at once (none are kept if
 * one creation fails). */
int mpcqp_enable_timing(mpcqp_ctx *ctx, int on);
double mpcqp_last_kernel_ms(mpcqp_ctx *ctx, int which);
/* sum (ms) over the launches of slot `which` recorded since the previous call (at most the last
 * 64; *count receives how many), waiting for them; resets the slot's count.  -1 on error. */
double mpcqp_kernel_ms_sum(mpcqp_ctx *ctx, int which, int *count);

/* Diagnostic solver-flops counter of the two-QPs-per-wave kernel (k_mpc_pair): with on = 1 every
 * launch adds the textbook flops of its crash working-set solves and dual passes (mpcqp/flops.py
 * crash_ws_flops / pass_flops, per instance with its own free count; one atomic per wavefront)
 * to a context-owned accumulator.  The reported iterations mix working sets and passes, which
 * cost different amounts, so the headline roofline needs this count (bench.py reads it in a
 * pass after the timed steps).  mpcqp_solver_flops waits for the stream and returns the sum
 * since the previous call (-1 if never enabled; *launches: the paired-kernel launches counted),
 * then resets it.  Other kernels add nothing. */
int mpcqp_count_solver_flops(mpcqp_ctx *ctx, int on);
double mpcqp_solver_flops(mpcqp_ctx *ctx, int *launches);

/* Diagnostics: per-phase cycle totals (s_memtime) of the fused kernels since the last call,
 * recorded only by the diagnostic build lib/libmpcqp_stamps.so (first call arms it); the
 * product library returns MPCQP_ERR_BAD_ARG.  Slots: 0 setup, 1 Phi/xf chains, 2 Qe,
 * 3 H_FF, 4 gradient, 5 Cholesky, 6 J = L^-T, 7 unconstrained min, 8 dual loop, 9 write,
 * 10 model build, 11 expm. */
int mpcqp_debug_phase_cycles(mpcqp_ctx *ctx, uint64_t *out, int n);

const char *mpcqp_status_string(int status);
/* hash of the sources this library was built from (profiles/ record it beside each counter
 * pass, so a summary can be matched to the library that was benchmarked) */
const char *mpcqp_build_id(void);
int mpcqp_device_count(void);

#ifdef __cplusplus
}
#endif
#endif /* MPCQP_H */
