/*
 * awegpu -- MI355X evaluator for the awebox AP2 direct-collocation NLP.
 *
 * C ABI (extern "C", plain pointers and sizes, no torch/HIP types in the signatures).  The entry
 * points are the NLP oracle surface that IPOPT reaches through CasADi in the reference:
 *
 *   reference: cas.nlpsol('solver', 'ipopt', {'x': V, 'p': P, 'f': f_fun(V,P), 'g': g_fun(V,P)})
 *              awebox/opti/preparation.py:366-380 (hippo solvers), :383-400 (non-hippo),
 *              awebox/pmpc.py:193-217 (MPC); the callbacks IPOPT then makes are CasADi's
 *              nlp_f / nlp_g / nlp_grad_f / nlp_jac_g / nlp_hess_l.
 *
 *   awe_eval_f        <->  nlp_f       (f)
 *   awe_eval_g        <->  nlp_g       (g)
 *   awe_eval_nlp      <->  nlp_grad_f + nlp_jac_g fused (f, g, grad f, J_g values)
 *   awe_sparsity_jac  <->  Sparsity of nlp_jac_g's output (CCS: colind[n_v+1], row[nnz])
 *   awe_eval_hess     <->  nlp_hess_l  (Hessian of sigma f + lam_g^T g, upper triangle)
 *   awe_sparsity_hess <->  Sparsity of nlp_hess_l's output (upper-triangular CCS)
 *
 * Memory: V[b*n_v + i], P[b*n_p + i], g[b*n_g + i], grad_f[b*n_v + i], jac[b*nnz + i] and f[b]
 * are *device* pointers (HBM-resident, caller-owned) for the awe_eval_* functions and *host*
 * pointers for the awe_eval_*_host convenience wrappers.  All internal buffers are owned by the
 * handle.  Every function returns 0 on success; a non-zero code means failure, and
 * awe_last_error() describes it.  A NaN/Inf in any output of awe_eval_nlp_host /
 * awe_eval_*_host returns AWE_ERR_NONFINITE (CasADi turns that into an evaluation failure, so
 * IPOPT rejects the step).  One handle per host thread.
 */
#ifndef AWEGPU_H
#define AWEGPU_H

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define AWE_OK 0
#define AWE_ERR_ARG 1
#define AWE_ERR_HIP 2
#define AWE_ERR_NONFINITE 3
#define AWE_ERR_NODEVICE 4

/* ---- node-variable layout (awebox/mdl/system.py:42-230): x[23] xdot[23] u[10] z[1] theta[2] */
#define AWE_NX 23
#define AWE_NU 10
#define AWE_NZ 1
#define AWE_NTH 2
#define AWE_NW 59
#define AWE_N_EQ 24
#define AWE_N_INEQ 9
#define AWE_NPHI 7
#define AWE_NXI 2
#define AWE_NCOST 20

/* ---- packed theta0 (fixed parameters, the tail of P) -- keep in sync with problem.py */
#define AWE_TH_G 0
#define AWE_TH_GAMMA 1
#define AWE_TH_R 2
#define AWE_TH_T_REF 3
#define AWE_TH_P_REF 4
#define AWE_TH_RHO_REF 5
#define AWE_TH_GAMMA_AIR 6
#define AWE_TH_MU_REF 7
#define AWE_TH_C_SUTHERLAND 8
#define AWE_TH_Z_REF 9
#define AWE_TH_Z0_AIR 10
#define AWE_TH_EXP_REF 11
#define AWE_TH_U_REF 12
#define AWE_TH_KAPPA 13
#define AWE_TH_RHO_TETHER 14
#define AWE_TH_CD_TETHER 15
#define AWE_TH_FORCE_LIMITS 16 /* [2] */
#define AWE_TH_AIRSPEED_LIMITS 18 /* [2] */
#define AWE_TH_ROT_ANGLES 20 /* [3] */
#define AWE_TH_KAPPA_R 23
#define AWE_TH_B_REF 24
#define AWE_TH_C_REF 25
#define AWE_TH_S_REF 26
#define AWE_TH_M_K 27
#define AWE_TH_J 28 /* [9] column-major */
#define AWE_TH_MOMENT_FACTOR 37
#define AWE_TH_STAB_DERIVS 38 /* [6 coeffs][9 inputs][3 alpha powers] */
#define AWE_NTHETA0 200

/* ---- model constants (option-derived, fixed at build time) -- keep in sync with problem.py */
#define AWE_C_N_K 0
#define AWE_C_D 1
#define AWE_C_SCALING_LENGTH 2
#define AWE_C_SCALING_DIAM 3
#define AWE_C_G_SCALING 4
#define AWE_C_Q_SCALING_MEAN 5
#define AWE_C_LAMBDA_SCALING 6
#define AWE_C_M_AERO_SCALING 7
#define AWE_C_ENERGY_SCALING 8
#define AWE_C_AIRSPEED_REF 9
#define AWE_C_ALPHA_MAX 10
#define AWE_C_ALPHA_MIN 11
#define AWE_C_BETA_MAX 12
#define AWE_C_BETA_MIN 13
#define AWE_C_AERO_TIGHTNESS 14
#define AWE_C_NORM_TRACKING 15
#define AWE_C_NORM_U_REG 16
#define AWE_C_NORM_THETA_REG 17
#define AWE_C_NORM_XDOT_REG 18
#define AWE_C_NORM_FICTITIOUS 19
#define AWE_C_NORM_BETA 20
#define AWE_C_N_ELEMENTS 21
#define AWE_C_SCALING 22 /* [59] */
#define AWE_C_SD_LEN 81  /* [54] */
#define AWE_NCONST 135

typedef struct awe_handle_s* awe_handle;

/* Build the evaluator for an AP2 problem with n_k intervals and d Radau nodes.
 * consts: AWE_NCONST doubles (AWE_C_* layout); batch: number of (V, P) instances evaluated per
 * call.  Derives the CCS sparsity of J_g and uploads the launch tables. */
int awe_create(int n_k, int d, const double* consts, int n_consts, int batch, awe_handle* out);
int awe_destroy(awe_handle h);
const char* awe_last_error(void);

/* sizes: n_v (decision vector), n_g (constraints), n_p (parameter vector), nnz (J_g) */
int awe_sizes(awe_handle h, int* n_v, int* n_g, int* n_p, int* nnz_jac);
/* CCS pattern of J_g: colind[n_v + 1], row[nnz] (host arrays, caller-owned) */
int awe_sparsity_jac(awe_handle h, int* colind, int* row);

/* The same CCS pattern without a device (CPU only; IPOPT asks for the structure before the
 * first evaluation).  Call with colind = row = NULL to obtain *nnz first. */
int awe_sparsity_jac_static(int n_k, int d, const double* consts, int n_consts, int* nnz, int* colind,
                            int* row);

/* Device-pointer evaluation on HIP stream `stream` (NULL = default stream); asynchronous.
 * Concurrency: a handle owns scratch buffers (the instance-minor transposes, the generated
 * Hessian's HD / partial / H buffers, the hyper-dual scratch) and timing events that every call
 * reuses without ordering them across streams.  Use each handle from one stream at a time: calls on
 * one handle must be serialised (one stream, or the caller orders the streams with events).  Two
 * handles are independent and may run on different streams concurrently. */
int awe_eval_nlp(awe_handle h, const double* V, const double* P, double* f, double* g,
                 double* grad_f, double* jac, void* stream);
int awe_eval_g(awe_handle h, const double* V, const double* P, double* g, void* stream);
int awe_eval_f(awe_handle h, const double* V, const double* P, double* f, void* stream);

/* Host-pointer wrappers: copy in, evaluate, copy out, synchronise, check finiteness. */
int awe_eval_nlp_host(awe_handle h, const double* V, const double* P, double* f, double* g,
                      double* grad_f, double* jac);
/* Host-pointer value-only entry points (nlp_f / nlp_g of one call from IPOPT through CasADi): copy
 * in, the value-only kernel (the model in plain double, no derivatives), copy out; a NaN/Inf in
 * the output returns AWE_ERR_NONFINITE.  Replace CasADi's nlp_f / nlp_g SX evaluation
 * (awebox/opti/preparation.py:366-400, ocp/nlp.py:77-161). */
int awe_eval_f_host(awe_handle h, const double* V, const double* P, double* f);
int awe_eval_g_host(awe_handle h, const double* V, const double* P, double* g);

/* Hessian of the Lagrangian sigma f + lam_g^T g (nlp_hess_l):
 * values of its upper triangle (row <= col) in the fixed CCS pattern of awe_sparsity_hess.
 * sigma[b] and lam_g[b*n_g + i] per instance (device pointers for awe_eval_hess). */
int awe_hess_nnz(awe_handle h, int* nnz_h);
int awe_sparsity_hess(awe_handle h, int* colind, int* row);
int awe_sparsity_hess_static(int n_k, int d, const double* consts, int n_consts, int* nnz, int* colind,
                             int* row);
int awe_eval_hess(awe_handle h, const double* V, const double* P, const double* sigma, const double* lam_g,
                  double* H, void* stream);
int awe_eval_hess_host(awe_handle h, const double* V, const double* P, const double* sigma,
                       const double* lam_g, double* H);
/* Kernel time of the last awe_eval_hess call (HIP events), milliseconds. */
int awe_last_hess_ms(awe_handle h, float* ms);
/* nlp_hess_l with H instance-minor: the value of CCS entry i of instance b at H[i * ldh + b]
 * (ldh >= batch; with batch = 1 and ldh = 1 it is awe_eval_hess's layout). */
int awe_eval_hess_im(awe_handle h, const double* V, const double* P, const double* sigma, const double* lam_g,
                     double* H, size_t ldh, void* stream);
/* Hessian path.  AWE_HESS_GENERATED: straight-line direction-pair Hessians of the node Lagrangian
 * generated at build time from the node model (csrc/gen/ap2_hessgen.cpp: a symbolic reverse sweep,
 * then sparse forward mode over it -- what CasADi's SX Hessian of the reference's nlp_hess_l
 * evaluates, opti/preparation.py:366-400), one wavefront per collocation node for 64 instances, and
 * an assembly kernel, one lane per instance; AWE_HESS_HYPERDUAL: the compressed hyper-dual kernel,
 * one (node, colour pair) per lane; AWE_HESS_FOLLOW (default): the generated Hessian with the
 * generated and instance-minor evaluation paths, the hyper-dual one with the colour path.  Both
 * agree to rounding.  AWE_HESS_PATH=generated|hyperdual selects it at awe_create; awe_get_hess_path
 * returns the path the next call takes. */
#define AWE_HESS_HYPERDUAL 0
#define AWE_HESS_GENERATED 1
#define AWE_HESS_FOLLOW 2
int awe_set_hess_path(awe_handle h, int path);
int awe_get_hess_path(awe_handle h, int* path);

/* nlp_grad_f + nlp_jac_g fused, with J_g and grad f instance-minor: the value of CCS entry i of
 * instance b at jac[i * ldj + b], gradient entry i at grad_f[i * ldj + b] (ldj >= batch; V, P, g and f
 * as in awe_eval_nlp).  The layout the batched solver consumes ([batch, nnz] and [batch, n_v] views
 * with strides (1, ldj)); with batch = 1 and ldj = 1 it is awe_eval_nlp's.  On the instance-minor path
 * the kernels write it directly (every store one contiguous run over 64 instances), on the other
 * paths the per-instance result is transposed. */
int awe_eval_nlp_im(awe_handle h, const double* V, const double* P, double* f, double* g,
                    double* grad_f, double* jac, int ldj, void* stream);

/* awe_eval_nlp_im with V and P instance-minor as well: entry i of instance b at VT[i * ldin + b] and
 * PT[i * ldin + b], ldin = awe_instance_ld(h).  A batched caller that keeps its decision vectors in
 * the layout the kernels read (as the batched solver keeps J_g) saves the input transposition (the
 * first kernel of awe_eval_nlp_im, ~12 % of an evaluation at batch 2048).  Instance-minor evaluation
 * path only (AWE_PATH_SOA); with batch 1 the layouts coincide and awe_eval_nlp is the same call.
 * Replaces, for a batch, the per-instance calls of the reference's nlp_jac_g / nlp_grad_f
 * (awebox/opti/preparation.py:366-400). */
int awe_eval_nlp_imv(awe_handle h, const double* VT, const double* PT, int ldin, double* f, double* g,
                     double* grad_f, double* jac, int ldj, void* stream);
/* Leading dimension of the handle's instance-minor buffers (batch rounded up to 16). */
int awe_instance_ld(awe_handle h, int* ld);

/* Evaluation path of awe_eval_nlp / awe_eval_nlp_im (f, g, grad f, J_g).  Default: AWE_PATH_SOA
 * for batches of 128 or more instances (when the model constants have the structure the code was
 * generated for), AWE_PATH_COLOUR below (a call is then one round of waves on every path, and the
 * colour kernel's single launch is the shortest: 0.036 ms at batch 1 against 0.18 ms).
 *   AWE_PATH_SOA:
 *     instance-minor generated path -- V and P's tail transposed to instance-minor order, then
 *     ap2_soa_node_kernel, one wavefront per (interval, node) and one lane per instance, running the
 *     generated straight-line code and storing every tangent directly into its J_g entries through
 *     a per-(interval, node) destination table; the interval kernel adds the objective, gradient and
 *     continuity rows;
 *   AWE_PATH_GENERATED: ap2_node_kernel, one thread per collocation node running straight-line
 *     value + sparse Jacobian code generated at build time from the node model
 *     (csrc/gen/ap2_jacgen.cpp; it also writes the g rows and the objective terms), then the gather
 *     kernel (J_g values, gradient);
 *   AWE_PATH_COLOUR: the single interval kernel with compressed forward mode, one colour of seed
 *     directions per lane.
 * All return the same values to rounding.  The environment variable AWE_EVAL_PATH=colour|generated|soa
 * selects the path at awe_create. */
#define AWE_PATH_COLOUR 0
#define AWE_PATH_GENERATED 1
#define AWE_PATH_SOA 2
int awe_set_eval_path(awe_handle h, int path);
int awe_get_eval_path(awe_handle h, int* path);
/* Kernel times of the last awe_eval_nlp call on the generated path: node kernel, gather kernel. */
int awe_last_kernel_ms_gen(awe_handle h, float* ms_node, float* ms_gather);
/* Kernel times of the last call on the instance-minor path (HIP events, ms): ms[0] input transpose,
 * ms[1] node kernel, ms[2] interval kernel, ms[3] finalize, ms[4] output transpose (awe_eval_nlp at
 * batch > 1; 0 otherwise). */
int awe_last_kernel_ms_soa(awe_handle h, float* ms);

/* Kernel time of the last awe_eval_* call on its stream, in milliseconds (HIP events). */
int awe_last_kernel_ms(awe_handle h, float* ms_main, float* ms_finalize);

/* Number of HIP devices visible (0 on a machine without a GPU). */
int awe_device_count(void);

#ifdef __cplusplus
}
#endif
#endif /* AWEGPU_H */
