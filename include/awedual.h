/*
 * awedual -- MI355X evaluator for the awebox multi-kite power-cycle NLP with two 6-DOF kites on
 * secondary tethers below a layer node (architecture
 * {1: 0, 2: 1, 3: 1}, examples/dual_kites_power_curve.py, direct collocation radau, zoh,
 * phase_fix 'single_reelout').
 *
 * C ABI (extern "C", plain pointers and sizes).  The entry points are the NLP oracle surface IPOPT
 * reaches through CasADi in the reference:
 *
 *   reference: cas.nlpsol('solver', 'ipopt', {'x': V, 'p': P, 'f': f_fun(V, P), 'g': g_fun(V, P)})
 *              awebox/opti/preparation.py:366-400 (nlp built by awebox/ocp/nlp.py:77-161)
 *
 *   adl_eval_nlp     <->  nlp_grad_f + nlp_jac_g fused (f, g, grad f, J_g values)
 *   adl_sparsity_jac <->  Sparsity of nlp_jac_g's output (CCS: colind[n_v+1], row[nnz])
 *   adl_eval_hess     <->  nlp_hess_l  (exact Hessian of sigma f + lam_g^T g, upper triangle;
 *                          IPOPT's hessian_approximation 'exact', opts/default.py:323,
 *                          opti/preparation.py:272-273)
 *   adl_sparsity_hess <->  Sparsity of nlp_hess_l's output (upper-triangular CCS)
 *
 * Memory: V[b*n_v + i], P[b*n_p + i], g[b*n_g + i], grad_f[b*n_v + i], jac[b*nnz + i], f[b] are
 * device pointers for adl_eval_nlp and host pointers for adl_eval_nlp_host.  Return codes as in
 * awegpu.h (0 = OK; adl_last_error() describes a failure; a NaN/Inf in any output of the host
 * wrapper returns AWE_ERR_NONFINITE).  One handle per host thread.
 *
 * P = [p.ref (n_v), p.weights (ADL_NW), cost (20), theta0 (AWE_NTHETA0, awegpu.h AWE_TH_* layout)]
 * (ocp/discretization.py:129-179).
 */
#ifndef AWEDUAL_H
#define AWEDUAL_H

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- node-variable layout (awebox/mdl/system.py:42-230, node-major in each group):
 *   x     = [q10 dq10 | q21 dq21 omega21 r21 delta21 | q31 dq31 omega31 r31 delta31 | l_t dl_t]
 *   xdot  = d<x>
 *   u     = [f_fict21 m_fict21 ddelta21 | f_fict31 m_fict31 ddelta31 | ddl_t]
 *   z     = [lambda10 lambda21 lambda31]
 *   theta = [diam_t t_f l_s diam_s]          (V.theta = [diam_t t_f(2) l_s diam_s]) */
#define ADL_NX 50
#define ADL_NU 19
#define ADL_NZ 3
#define ADL_NTH 4
#define ADL_NTHV 5
#define ADL_NW 126
#define ADL_N_EQ 53
#define ADL_N_INEQ 19
#define ADL_NKITES 2

/* kernel constants: ADL_NCONST doubles (awebox_amd/dual.py CONST_NAMES) */
#define ADL_C_N_K 0
#define ADL_C_D 1
#define ADL_C_NK_REELOUT 2
#define ADL_C_SINGLE_REELOUT 3
#define ADL_C_PHASE_FIX_REELOUT 4
#define ADL_C_TF_LB 5
#define ADL_C_TF_UB 6
#define ADL_C_SCALING_LENGTH_T 7
#define ADL_C_SCALING_LENGTH_S 8
#define ADL_C_SCALING_DIAM_T 9
#define ADL_C_SCALING_DIAM_S 10
#define ADL_C_G_SCALING 11
#define ADL_C_M_AERO_SCALING 12
#define ADL_C_ENERGY_SCALING 13
#define ADL_C_AIRSPEED_REF 14
#define ADL_C_ALPHA_MAX 15
#define ADL_C_ALPHA_MIN 16
#define ADL_C_BETA_MAX 17
#define ADL_C_BETA_MIN 18
#define ADL_C_AERO_TIGHTNESS 19
#define ADL_C_NORM_TRACKING 20
#define ADL_C_NORM_U_REG 21
#define ADL_C_NORM_THETA_REG 22
#define ADL_C_NORM_XDOT_REG 23
#define ADL_C_NORM_FICTITIOUS 24
#define ADL_C_NORM_BETA 25
#define ADL_C_N_ELEMENTS 26
#define ADL_C_ANTICOLLISION_DIST_MIN 27
#define ADL_C_SCALING 28 /* [126] */
#define ADL_C_SD_LEN 154 /* [54] */
#define ADL_NCONST 208

typedef struct adl_handle_s* adl_handle;

/* Build the evaluator for n_k intervals, d Radau nodes (2 <= d <= 5), `batch` (V, P) instances
 * per call.  Derives the J_g sparsity (structural dependencies of the node model) and the
 * compressed-direction colouring on the host, uploads the launch tables. */
int adl_create(int n_k, int d, const double* consts, int n_consts, int batch, adl_handle* out);
int adl_destroy(adl_handle h);
const char* adl_last_error(void);
int adl_sizes(adl_handle h, int* n_v, int* n_g, int* n_p, int* nnz_jac);
int adl_sparsity_jac(adl_handle h, int* colind, int* row);
/* CPU-only: the same CCS pattern (call with colind = row = NULL to get *nnz first) and the
 * number of colours of the shooting / Radau node (diagnostics). */
int adl_sparsity_jac_static(int n_k, int d, const double* consts, int n_consts, int* nnz, int* colind, int* row);
int adl_colour_counts(int n_k, int d, const double* consts, int n_consts, int* n_col_shoot, int* n_col_radau,
                      int* tang_shoot, int* tang_radau);

/* Device-pointer evaluation on HIP stream `stream` (NULL = default stream); asynchronous. */
int adl_eval_nlp(adl_handle h, const double* V, const double* P, double* f, double* g, double* grad_f,
                 double* jac, void* stream);
/* Host-pointer wrapper: copy in, evaluate, copy out, synchronise, check finiteness. */
int adl_eval_nlp_host(adl_handle h, const double* V, const double* P, double* f, double* g, double* grad_f,
                      double* jac);
/* Kernel time of the last adl_eval_nlp (HIP events), milliseconds. */
int adl_last_kernel_ms(adl_handle h, float* ms_main, float* ms_finalize);

/* Generated instance-minor path (the node code generated from the model at build time,
 * awebox_amd/csrc/gen/dual_jacgen.cpp; one lane per instance): *available = 1 when it serves the
 * handle's constants (otherwise adl_last_error says why).  adl_eval_nlp_im returns the same f, g,
 * grad f and J_g as adl_eval_nlp (to rounding) with grad_f and jac instance-minor,
 * grad_f[i * ld + b], jac[e * ld + b] (ld >= batch); device pointers, asynchronous on `stream`.
 * Replaces the same oracle surface (nlp_f / nlp_g / nlp_grad_f / nlp_jac_g of
 * awebox/opti/preparation.py:366-400) for a batch of dual-kite NLPs. */
int adl_gen_status(adl_handle h, int* available);
int adl_eval_nlp_im(adl_handle h, const double* V, const double* P, double* f, double* g, double* grad_f,
                    double* jac, size_t ld, void* stream);
/* HIP-event times of the last adl_eval_nlp_im: input transposition, node kernel, interval kernel,
 * finalize (ms). */
int adl_last_kernel_ms_im(adl_handle h, float* ms_in, float* ms_node, float* ms_interval, float* ms_fin);

/* Hessian of the Lagrangian sigma f + lam_g^T g (nlp_hess_l): values of its upper triangle
 * (row <= col) in the fixed CCS pattern of adl_sparsity_hess; sigma[b] and lam_g[b*n_g + i] per
 * instance (device pointers for adl_eval_hess, host pointers for adl_eval_hess_host).  The
 * structure and launch tables are derived on the first Hessian call. */
int adl_hess_nnz(adl_handle h, int* nnz_h);
int adl_sparsity_hess(adl_handle h, int* colind, int* row);
int adl_sparsity_hess_static(int n_k, int d, const double* consts, int n_consts, int* nnz, int* colind, int* row);
int adl_eval_hess(adl_handle h, const double* V, const double* P, const double* sigma, const double* lam_g,
                  double* H, void* stream);
int adl_eval_hess_host(adl_handle h, const double* V, const double* P, const double* sigma, const double* lam_g,
                       double* H);
/* Kernel time (interval + finalize kernels) of the last adl_eval_hess call, milliseconds. */
int adl_last_hess_ms(adl_handle h, float* ms);
/* Diagnostics (CPU): value [75] and Jacobian [75 x 127] of one node of the model source. */
int adl_node_eval_host(const double* w, const double* th, const double* consts, int n_consts, double* val,
                       double* jac);

#ifdef __cplusplus
}
#endif
#endif /* AWEDUAL_H */
