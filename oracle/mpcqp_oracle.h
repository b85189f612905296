/*
 * mpcqp_oracle.h -- CPU restatement of the reference hot path (TEST INFRASTRUCTURE ONLY).
 *
 * This is the parity oracle and the timed CPU baseline ("port") for the MI355X batched
 * MPC-QP engine.  It is NOT part of the product: only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load it, and only as the checker / baseline.  The product
 * path (libmpcqp.so, HIP) never links or calls anything in oracle/.
 *
 * Reference (Fleming-Sung/mpc-limX-control, snapshot 2025-04-04) functions restated here:
 *   QPSolver::discretizeSystem      src/QPSolver.cpp:21-29     -> orc_discretize
 *     Eigen MatrixBase::exp()        (Eigen 3.3 MatrixExponential, Pade 3/5/7/9/13 +
 *                                     scaling & squaring)       -> orc_expm
 *     Eigen MatrixBase::pow(int)     (Eigen 3.3 MatrixPower::computeIntPower)  -> orc_matpow
 *   QPSolver::buildQPParams         src/QPSolver.cpp:31-81     -> orc_build_qp
 *   linear_mpc_example discretize   src/linear_mpc_example.cpp:35-46 -> orc_discretize_quadrature
 *   mpcQP::buildSystemModel         include/mpcQP.h:121-182    -> orc_model_literal
 *   QPSolver::solveQP (qpOASES)     src/QPSolver.cpp:83-106    -> orc_solve_qp (corrected QP,
 *                                   Goldfarb-Idnani dual active set; same algorithm as the GPU)
 *   QPSolver::updateState           src/QPSolver.cpp:108-111   -> orc_plant_step
 *   MPC::calculateGait              include/MPCController.h:61-75 -> orc_gait_contact_mask
 *
 * Parity status: the reference binary cannot be built here (Eigen, qpOASES, Pinocchio, ROS,
 * limxsdk absent) and the reference holds no golden vectors or tests
 * for this path.  => "parity unpinned" w.r.t. the reference binary.  The restatement is
 * cross-checked against an independent numpy/scipy restatement (tests/golden/make_golden.py,
 * scipy.linalg.expm + KKT-certified optimum) and against the SURVEY.md section 8c known-answer
 * values computed on the reference harness inputs (src/qpSolver_test.cpp:6-50).
 *
 * All matrices are column-major (Eigen default storage, what `.data()` hands out).
 */
#ifndef MPCQP_ORACLE_H
#define MPCQP_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ORC_INFTY 1e20 /* qpOASES::INFTY as used at src/QPSolver.cpp:72-73 */

/* status codes: identical numbering to include/mpcqp.h */
#define ORC_OK 0
#define ORC_BAD_DIMS 1
#define ORC_INFEASIBLE 2
#define ORC_ITER_LIMIT 3
#define ORC_NOT_PD 4

/* ---- reference numerical core ------------------------------------------------------ */
int orc_expm(int n, const double *A, double *E);
void orc_matpow(int n, const double *A, int p, double *out);
int orc_discretize(int nx, int nu, double Ts, const double *Ac, const double *Bc, double *Ad,
                   double *Bd);
int orc_discretize_quadrature(int nx, int nu, double Ts, const double *Ac, const double *Bc,
                              double *Ad, double *Bd);
int orc_build_qp(int nx, int nu, int N, const double *Ad, const double *Bd, const double *Q,
                 const double *R, const double *P, const double *x_min, const double *x_max,
                 double u_min, double u_max, const double *xi0, const double *xi_ref, double *H,
                 double *f, double *A_eq, double *b_eq, double *lb, double *ub, double *A_ineq,
                 double *lbA, double *ubA);
void orc_plant_step(int nx, int nu, const double *Ad, const double *Bd, double *x,
                    const double *u);

/* ---- dense QP:  min 1/2 x'Hx + f'x  s.t. lb<=x<=ub, lbA<=A x<=ubA, friction pyramid ---
 * A is row-major (mA x n) unless a_colmajor != 0.  Bounds with |v| >= ORC_INFTY are absent.
 * Variables with lb == ub are eliminated (fixed).  Rows with lbA == ubA are equalities.
 * fric (optional): implicit friction-pyramid rows  mu*fz -/+ fx >= 0, mu*fz -/+ fy >= 0 for
 * every (step k, foot s) whose bit in contact_mask (bit 2k+s) is set; variable layout
 * k*nu + 3*s + {0:fx,1:fy,2:fz}.  */
typedef struct {
    int enabled;
    int nu;          /* inputs per step (6 for two feet) */
    int N;           /* horizon */
    int nfeet;       /* 2 */
    double mu;       /* friction coefficient */
    uint64_t contact_mask;
    int elide_fz;    /* leave out the lower bound fz >= lb (lb <= 0) of a foot in contact: its
                        pyramid implies fz >= 0 (same feasible set; the library does the same) */
} orc_friction;

int orc_solve_qp(int n, const double *H, const double *f, int mA, const double *A,
                 int a_colmajor, const double *lb, const double *ub, const double *lbA,
                 const double *ubA, const orc_friction *fric, int max_iter, double *x,
                 double *cost, int *iters, double *lam_bounds /* n, nullable */,
                 double *lam_rows /* mA, nullable */);

/* KKT residuals of a candidate solution (solver-independent optimality certificate) */
void orc_kkt_residual(int n, const double *H, const double *f, int mA, const double *A,
                      int a_colmajor, const double *lb, const double *ub, const double *lbA,
                      const double *ubA, const double *x, double *primal_inf,
                      double *stationarity_proj);

/* ---- SRBM models (TRON1) ------------------------------------------------------------- */
/* literal reference model, include/mpcQP.h:139-181: 13x13 Ac, 13x3 Bc from foot-base offset */
void orc_model_literal(double dx, double dy, double dz, double m, double *Ac, double *Bc);
/* convex-MPC SRBM (build's definition): lin = {yaw, rL(3), rR(3)} */
void orc_model_srbm(const double *lin, double m, const double *Ib, double *Ac, double *Bc);

/* gait (include/MPCController.h:61-75): per-step contact bits from a phase offset */
uint64_t orc_gait_contact_mask(int N, double Ts, double phase0, float swing_time,
                               float stance_time);

/* ---- batched SRBM pipeline (CPU baseline, same stages as the GPU pipeline) ----------- */
typedef struct {
    int nx, nu, N;          /* 13, 6, N */
    int model;              /* 0 = convex SRBM 13x6, 1 = literal 13x3 */
    int friction;           /* 0 = box only, 1 = box + friction pyramid */
    double Ts, mass, mu;
    double Ib[9];           /* body inertia (col-major) */
    double fz_min, fz_max, fxy_max; /* per-foot force box (SRBM model) */
    double u_min, u_max;    /* literal model input box */
    const double *Q, *R, *P;/* nx*nx, nu*nu, nx*nx col-major */
    int max_iter;
    /* bounds-only problems: the GPU kernels' speculative primal-dual active-set start (at most
     * crash_kmax bounds per working set, crash_pmax working sets, then Goldfarb-Idnani);
     * 0 = off (plain Goldfarb-Idnani, the solve every other path runs).  Instances with more
     * than crash_split free variables are the workgroup solver's: crash_kmax_wg / _pmax_wg. */
    int crash_kmax, crash_pmax, crash_kmax_wg, crash_pmax_wg, crash_split;
    int elide_fz; /* orc_friction::elide_fz for the friction configurations */
} orc_srbm_cfg;

/* x0: [B][nx]; xref: [B][N+1][nx]; lin: [B][8]; contact: [B]; U: [B][nu*N] */
int orc_srbm_batch(const orc_srbm_cfg *cfg, int B, const double *x0, const double *xref,
                   const double *lin, const uint64_t *contact, double *U, double *cost,
                   int *status, int *iters, double *H_out /* nullable [B][nV][nV] */,
                   double *f_out /* nullable [B][nV] */, int nthreads,
                   double *sflops /* nullable [B]: solver flops per instance (crash working-set
                                     solves + dual passes, mpcqp/flops.py formulas) */);

/* per-instance bounds of the SRBM model (contact schedule -> lb/ub) */
void orc_srbm_bounds(const orc_srbm_cfg *cfg, uint64_t contact, double *lb, double *ub);
/* SRBM plant step, QPSolver::updateState (src/QPSolver.cpp:108-111) with the exact ZOH of the
 * SRBM linearised at lin = {yaw, rL, rR}: x <- Ad x + Bd u, (Ad, Bd) = orc_discretize (Eigen's
 * Pade expm restated).  Returns the discretisation status. */
int orc_srbm_plant(const orc_srbm_cfg *cfg, const double *lin, double *x, const double *u);

/* ---- dense model (BASELINE config E: the whole-body linearisation, 24 states) ------------
 * Per instance the continuous model [Ac | Bc] (nx x (nx+nu), column-major) is given, as the
 * upstream whole-body linearisation hands it over; the step is the reference's own path:
 * QPSolver::discretizeSystem (src/QPSolver.cpp:21-29, Eigen expm) -> buildQPParams
 * (:31-81, literal dense B'QB with full Q/R/P) -> the corrected QP with the input box
 * u_min <= u <= u_max (:67-68) -> Goldfarb-Idnani.  x0 [B][nx], xref [B][N+1][nx],
 * AB [B][nx*(nx+nu)], U [B][nu*N]. */
typedef struct {
    int nx, nu, N;
    double Ts;
    const double *Q, *R, *P; /* nx*nx, nu*nu, nx*nx column-major (dense) */
    double u_min, u_max;
    int max_iter;
    int crash_kmax, crash_pmax; /* as orc_srbm_cfg */
} orc_dense_cfg;

int orc_dense_batch(const orc_dense_cfg *cfg, int B, const double *x0, const double *xref,
                    const double *AB, double *U, double *cost, int *status, int *iters,
                    double *H_out /* nullable [B][nV][nV] */, double *f_out /* nullable */,
                    int nthreads);

/* ---- state estimator and leg kinematics ------------------------ */
/* stateEstimator::update (include/stateEstimator.h:217-337), one robot: xhat[12], P[144]
 * (col-major) updated in place from eePos[6], eeVel[6] (feet relative to the base, world
 * frame, as eeKinematics_ returns them), contact[2], quat[4] (x y z w), acc[3] (IMU, local) */
int orc_kf_update(double dt, double *xhat, double *P, const double *eePos, const double *eeVel,
                  const unsigned char *contact, const double *quat, const double *acc);
/* foot contact points of both legs, world frame relative to the base: q[6] = (abad, hip, knee)
 * left then right, rpy[3]; feet[6] = left xyz, right xyz (chain in mpcqp_oracle.c) */
void orc_fk_feet(const double *q, const double *rpy, double *feet);

#ifdef __cplusplus
}
#endif
#endif
