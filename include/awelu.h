/* awelu -- batched dense LU factorisation and solve of many mid-sized fp64 matrices on MI355X
 * (awebox_amd/csrc/batched_lu.hip, libawelu.so).
 *
 * Not an entry point of the reference's NLP oracle: these replace the linear algebra under
 * IPOPT's KKT solve (MA27/MUMPS inside `cas.nlpsol(..., 'ipopt')`, opti/preparation.py:366-400)
 * for the GPU solvers (awebox_amd/ipm.py StructuredKKT, awebox_amd/rti.py), which factorise
 * the interval blocks of the structured KKT system as one batch.
 *
 * Convention = LAPACK getrf / torch.linalg.lu_factor: row-major A[b][n][n] overwritten by the unit
 * lower factor (below the diagonal) and the upper factor (on and above); piv[b][n] 1-based, row k
 * exchanged with row piv[k] - 1 at step k.  All pointers are device pointers; calls are
 * asynchronous on `stream` (a hipStream_t, NULL = default stream).  Return 0 on success,
 * non-zero with awelu_last_error() describing the failure.
 */
#ifndef AWELU_H
#define AWELU_H

#ifdef __cplusplus
extern "C" {
#endif

/* In-place LU with partial pivoting of `batch` n x n matrices, 1 <= n <= 1024. */
int awelu_factor_batched(int n, int batch, double* A, int* piv, void* stream);

/* X[b] <- A[b]^-1 X[b] from the factors of awelu_factor_batched; X[b][n][nrhs] row-major. */
int awelu_solve_batched(int n, int nrhs, int batch, const double* LU, const int* piv, double* X, void* stream);

/* Block-tridiagonal systems (the stage-ordered separator system of the structured KKT):
 * T[b][nb][3][m][m] = (block (k, k-1), block (k, k), block (k, k+1)) of each block row, m <= 48.
 * Block LU without interchanges between block rows (partial pivoting inside each diagonal block).
 * factor: in place, the diagonal blocks become D'_k, the super-diagonal blocks W_k = D'_k^-1 U_k,
 * and Dinv[b][nb][m][m] receives D'_k^-1;  solve: X[b][nb m][nrhs] <- T^-1 X in place with those factors. */
int awelu_btd_factor_batched(int nb, int m, int batch, double* T, double* Dinv, void* stream);
int awelu_btd_solve_batched(int nb, int m, int nrhs, int batch, const double* T, const double* Dinv, double* X,
                            void* stream);

/* Inertia of `batch` symmetric n x n matrices A[b][n][n], n <= 4800 (lower triangle read; A is
 * destroyed) by blocked Bunch-Kaufman elimination (delayed updates, panels of up to 16 pivot
 * columns): counts[b][3] = (positive, negative, zero) eigenvalue counts, a pivot
 * column below ztol * max|A| counting as zero.  IPOPT's inertia correction (IpPDFullSpaceSolver,
 * MA27/MA57 inertia) for the structured KKT of awebox_amd/ipm.py. */
int awelu_sym_inertia_batched(int n, int batch, double* A, double ztol, int* counts, void* stream);

/* Fixed-order gather-sums of the solver's KKT assembly and sparse products (ipm._ScatterSum,
 * ipm._GatherMv): for every row r < rows, out[r * ldo + dst] += the sum of v(r, s) over a
 * destination's source list, v = vals[r * ldv + s] (x NULL) or vals[r * ldv + s] * x[r * ldx + cols[s]].
 * The lists occupy L lanes: lsrc[l] a source (-1 = padding), lw[l] the list's power-of-two width
 * (<= 64; lists aligned to their width), ldst[l] the destination on a list's first lane, -1
 * elsewhere.  The lists are summed as adjacent-pair trees, the order of torch's row sums. */
int awelu_gather_sum(int L, int rows, const int* lsrc, const unsigned char* lw, const int* ldst, const double* vals,
                     long long ldv, const double* x, const int* cols, long long ldx, double* out, long long ldo,
                     void* stream);

/* The destination lists longer than 64 sources of the same gather-sums, in one launch: list l's
 * sources wsrc[woff[l] .. woff[l] + ww[l]) (a power-of-two width, -1 = padding) are summed per row in
 * awelu_row_sum's order and added to out[r * ldo + wdst[l]]; vals / x / cols as in awelu_gather_sum. */
int awelu_gather_sum_wide(int nl, int rows, const int* wsrc, const int* woff, const int* ww, const int* wdst,
                          const double* vals, long long ldv, const double* x, const int* cols, long long ldx,
                          double* out, long long ldo, void* stream);

/* Batch-invariant row sums (awebox_amd/det.py): out[r] = sum of x[r * ldx + j] over j < n, for
 * r < rows.  Thread t of 256 adds x[t], x[t + 256], ... in sequence; the 256 partial sums are added
 * as an adjacent-pair tree.  The order depends on n only, never on rows, so a solver's norms, dot
 * products and merit terms round the same for one instance as inside any batch (the reference
 * solves every sweep point as its own IPOPT problem: awebox/sweep.py:148-172,
 * opti/optimization.py:363). */
int awelu_row_sum(long long rows, long long n, const double* x, long long ldx, double* out, void* stream);

/* Batch-invariant batched matrix products (awebox_amd/det.py): C[b] = A[b] B[b], M x K times K x N,
 * element strides (sAm, sAk), (sBk, sBn), (sCm, sCn) and batch strides sAb, sBb, sCb (a transposed
 * operand is a swapped stride pair); C must not overlap A or B.  Every entry is summed over k in
 * sequence from 0, product and sum rounded separately: the bits depend on K only, not on the batch
 * or on the tile shape the launch picks (rocBLAS picks its kernel by the batch count). */
int awelu_bmm(int batch, int M, int N, int K, const double* A, long long sAb, long long sAm, long long sAk,
              const double* B, long long sBb, long long sBk, long long sBn, double* C, long long sCb, long long sCm,
              long long sCn, void* stream);

/* The interior-point solver's per-iteration measures (awebox_amd/ipm.py solve_batch), one
 * workgroup per instance, in place of ~130 torch operations per iteration: mode 0 writes out[r][b]
 * for r = 0..9 (IPOPT's scaled optimality error at mu_target, its dual, primal and complementarity
 * parts, the unscaled dual infeasibility, constraint violation and complementarity of the
 * termination test, the barrier problem's error at mu[b], theta = ||c||_1 and the barrier function
 * phi at mu[b]); mode 1 only theta and phi (rows 0, 1).  Arrays are row-major per instance:
 * [B][ny] for y, its bounds, masks, zl, zu and jt_lam (J^T lam before the slack rows' -lam_I),
 * [B][n] grad, [B][m] c, lam, c_scale, [B][mI] cs_slack, [B] f, mu, obj_scale; [ny] lo_only /
 * hi_only (1.0 where only the lower / upper bound is finite), [m] eq_row, [mI] ineq, gl0, gu0.
 * Every value rounds as the torch composition ipm.errors_torch / ipm.barrier_phi_torch (sums in
 * awelu_row_sum's order, no contraction; inv_* are host reciprocals, as torch divides by a host
 * scalar).  IPOPT's IpIpoptCalculatedQuantities (curr_nlp_error, curr_barrier_obj) for the reference's
 * solver (opti/preparation.py:285-323). */
typedef struct AweluIpmMeasures {
    long long B;
    int ny, n, m, mI, mode;
    const double* grad;
    const double* jt_lam;
    const double* lam;
    const long long* ineq;
    const double *zl, *zu, *y, *yl, *yu;
    const unsigned char *hl, *hu;
    const double *lo_only, *hi_only;
    const double* c;
    const double* c_scale;
    const double* cs_slack;
    const unsigned char* eq_row;
    const double *gl0, *gu0;
    const double *obj_scale, *f, *mu;
    double mu_target, kappa_d, s_max, inv_mnb, inv_nb, inv_smax;
    double* out;
} AweluIpmMeasures;
int awelu_ipm_measures(const AweluIpmMeasures* a, void* stream);

/* The Newton system's vectors at an iterate (ipm.solve_batch): dl, du (bound gaps, 1 where a bound
 * is infinite), sigma = z_L / dl + z_U / du, grad phi = grad f - mu / dl + mu / du + kappa_d mu
 * (lo_only - hi_only) and rhs [B][ny + m] = [-(grad phi + J^T lam - lam_I on the slacks); -c], as
 * the torch composition ipm_measures.Measures.newton_torch rounds them.  Arrays as in
 * AweluIpmMeasures; outputs [B][ny] (rhs [B][ny + m]).  IPOPT's PDFullSpaceSolver right-hand side
 * (IpPDFullSpaceSolver.cpp) for the reference's solver. */
typedef struct AweluIpmNewton {
    int B, ny, n, m, mI;
    const double *y, *yl, *yu;
    const unsigned char *hl, *hu;
    const double *zl, *zu, *grad, *jt_lam, *lam, *c;
    const long long* ineq;
    const double *lo_only, *hi_only, *mu;
    double kappa_d;
    double *dl, *du, *sigma, *grad_phi, *rhs;
} AweluIpmNewton;
int awelu_ipm_newton(const AweluIpmNewton* a, void* stream);

/* The accepted step (ipm.solve_batch): dz = mu / gap - z -/+ (z / gap) dy at the Newton system's gaps
 * dl_old, du_old (awelu_ipm_newton's dl, du), alpha_z[b] =
 * min(1, min over dz < 0 of -tau z / dz), then per instance with acc[b]: y_out = y_new, lam_out = lam +
 * alpha[b] dlam, z_out = z + alpha_z dz (instances without acc[b] keep y and add 0 * steps, as the torch
 * composition does); and for all instances IPOPT's kappa_sigma safeguard at the new gaps,
 * z <- clamp(z, mu / (kappa_sigma gap), kappa_sigma mu / gap).  any_acc = 0: no instance stepped
 * (y, lam unchanged; only the safeguard).  Every entry as Measures.step_torch rounds it. */
typedef struct AweluIpmStep {
    int B, ny, m, any_acc;
    const double *y, *y_new, *dy, *lam, *dlam, *zl, *zu, *yl, *yu, *dl_old, *du_old;
    const unsigned char *hl, *hu, *acc;
    const double *mu, *tau, *alpha;
    double kappa_sigma;
    double *y_out, *lam_out, *zl_out, *zu_out, *alpha_z;
} AweluIpmStep;
int awelu_ipm_step(const AweluIpmStep* a, void* stream);

/* Message of the last failed call on this thread. */
const char* awelu_last_error(void);

#ifdef __cplusplus
}
#endif

#endif
