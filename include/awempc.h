/*
 * awempc -- MI355X evaluator for the awebox tracking-MPC NLP of a 3-DOF kite (SURVEY.md section 8
 * row a37, config 5: examples/mpc_closed_loop.py, horizon N, radau d, zoh controls).
 *
 * C ABI (extern "C", plain pointers and sizes).  The entry points are the NLP oracle surface the
 * MPC's IPOPT solver reaches through CasADi in the reference:
 *
 *   reference: ct.nlpsol('solver', 'ipopt', {'x': V, 'p': p, 'f': f, 'g': g_fun(V, P_fun(p))})
 *              awebox/pmpc.py:193-217, called per MPC step at pmpc.py:252-270 with
 *              p = [x0, ref, u_ref, Q, R, P] (pmpc.py:166-186)
 *
 *   awempc_eval_nlp      <->  nlp_grad_f + nlp_jac_g fused (f, g, grad f, J_g values)
 *   awempc_sparsity_jac  <->  Sparsity of nlp_jac_g's output (CCS: colind[n_v+1], row[nnz])
 *   awempc_eval_hess     <->  nlp_hess_l: sigma f + lam^T g, upper triangle in a fixed CCS pattern
 *                             (IPOPT's exact Hessian, awebox/opts/default.py:323, pmpc.py:193-217)
 *   awempc_sparsity_hess <->  Sparsity of nlp_hess_l's output
 *
 * Memory: V[b*n_v + i], p[b*n_p + i], g[b*n_g + i], grad_f[b*n_v + i], jac[b*nnz + i], f[b] are
 * device pointers for awempc_eval_nlp, host pointers for awempc_eval_nlp_host.  Return codes as in
 * awegpu.h (0 = OK; awempc_last_error() describes a failure; a NaN/Inf in any output of the host
 * wrapper returns AWE_ERR_NONFINITE).  One handle per host thread; `batch` MPC instances (one per
 * simulated system or per real-time iteration) are evaluated per call.
 */
#ifndef AWEMPC_H
#define AWEMPC_H

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- node-variable layout (awebox/mdl/system.py:42-230, kite_dof 3, tether control dddl_t):
 *      x = [q10(3) dq10(3) coeff10(2) l_t dl_t ddl_t], xdot = d<x>, u = [f_fict10(3) dcoeff10(2)
 *      dddl_t], z = [lambda10], theta = [diam_t t_f] */
#define K3_NX 11
#define K3_NU 6
#define K3_NZ 1
#define K3_NTH 2
#define K3_NW 31
#define K3_N_EQ 12
#define K3_N_INEQ 2
#define K3_NPHI 7
#define K3_NXI 2

/* ---- model constants vector -- keep in sync with awebox_amd/kite3.py CONST_NAMES */
#define K3_C_N_K 0
#define K3_C_D 1
#define K3_C_G 2
#define K3_C_T_REF 3
#define K3_C_RHO_REF 4
#define K3_C_GAMMA_AIR 5
#define K3_C_R_AIR 6
#define K3_C_Z_REF 7
#define K3_C_Z0_AIR 8
#define K3_C_KAPPA 9
#define K3_C_RHO_TETHER 10
#define K3_C_CD_TETHER 11
#define K3_C_STRESS_MAX 12
#define K3_C_M_K 13
#define K3_C_S_REF 14
#define K3_C_AR 15
#define K3_C_CD0 16
#define K3_C_ACC_MAX 17
#define K3_C_SCALING_LENGTH 18
#define K3_C_SCALING_DIAM 19
#define K3_C_G_SCALING 20
#define K3_C_Q_SCALING_MEAN 21
#define K3_C_LAMBDA_SCALING 22
#define K3_C_N_ELEMENTS 23
#define K3_C_SCALING 24 /* [31] */
#define K3_NCONST 55

typedef struct awempc_handle_s* awempc_handle;

/* Build the evaluator for horizon n_k, d radau nodes, `batch` instances per call. */
int awempc_create(int n_k, int d, const double* consts, int n_consts, int batch, awempc_handle* out);
int awempc_destroy(awempc_handle h);
const char* awempc_last_error(void);

/* n_v = 22 + n_k (2 nx + nu + nz + d (nx + nz)), n_g = nx + n_k (n_eq + n_ineq + d n_eq + nx),
 * n_p = n_v + 2 nx + nu + nx + 1 */
int awempc_sizes(awempc_handle h, int* n_v, int* n_g, int* n_p, int* nnz_jac);
int awempc_sparsity_jac(awempc_handle h, int* colind, int* row);
/* the same pattern without a device; colind = row = NULL returns *nnz */
int awempc_sparsity_jac_static(int n_k, int d, const double* consts, int n_consts, int* nnz, int* colind,
                               int* row);

/* device pointers, asynchronous on `stream` (NULL = default stream) */
int awempc_eval_nlp(awempc_handle h, const double* V, const double* p, double* f, double* g, double* grad_f,
                    double* jac, void* stream);
/* host pointers: copy in, evaluate, copy out, synchronise, check finiteness */
int awempc_eval_nlp_host(awempc_handle h, const double* V, const double* p, double* f, double* g,
                         double* grad_f, double* jac);
/* kernel time of the last awempc_eval_nlp (HIP events on its stream), ms */
int awempc_last_kernel_ms(awempc_handle h, float* ms_main, float* ms_finalize);

/* ---- generated instance-minor path ------------------------------------------------------------
 * The same f, g, grad f and J_g values from straight-line node code generated from the model
 * (csrc/gen/kite3_jacgen.cpp: the sparse Jacobian of each node, one lane per instance) instead of the
 * dual-number kernel of awempc_eval_nlp.  grad_f and jac are instance-minor: grad_f[i * ld + b],
 * jac[e * ld + b], ld >= batch (each J_g / gradient row of all instances contiguous, the layout the
 * batched solvers read); V, p, f, g as above.  Device pointers, asynchronous on `stream`.
 * awempc_gen_status sets *available = 0 (awempc_last_error() says why) when the model constants do
 * not have the integer structure the code was generated for. */
int awempc_gen_status(awempc_handle h, int* available);
int awempc_eval_nlp_im(awempc_handle h, const double* V, const double* p, double* f, double* g, double* grad_f,
                       double* jac, size_t ld, void* stream);
/* kernel times of the last awempc_eval_nlp_im: input transposition, node kernel, finalize (ms) */
int awempc_last_kernel_ms_im(awempc_handle h, float* ms_in, float* ms_node, float* ms_finalize);

/* ---- nlp_hess_l ----------------------------------------------------------------------------------
 * Hessian of sigma f + lam^T g w.r.t. V, upper triangle (row <= col), CCS over the n_v columns:
 * H[b*nnz_h + i].  sigma[b], lam[b*n_g + i].  The structure is derived on the host from the node
 * model's second-order dependencies (built on the first call). */
int awempc_hess_init(awempc_handle h, int* nnz_h);
int awempc_sparsity_hess(awempc_handle h, int* colind, int* row);
/* the same pattern without a device; colind = row = NULL returns *nnz */
int awempc_sparsity_hess_static(int n_k, int d, const double* consts, int n_consts, int* nnz, int* colind,
                                int* row);
/* device pointers, asynchronous on `stream` */
int awempc_eval_hess(awempc_handle h, const double* V, const double* p, const double* sigma, const double* lam_g,
                     double* H, void* stream);
/* host pointers: copy in, evaluate, copy out, synchronise, check finiteness */
int awempc_eval_hess_host(awempc_handle h, const double* V, const double* p, const double* sigma,
                          const double* lam_g, double* H);
/* kernel time (Hessian + finalize) of the last awempc_eval_hess, ms */
int awempc_last_hess_ms(awempc_handle h, float* ms);

#ifdef __cplusplus
}
#endif
#endif /* AWEMPC_H */
