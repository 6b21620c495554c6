// The Ampyx AP2 single-kite node model, hand-written for CDNA4 and instantiated on
// double / Dual / Dep (scalar.hpp).
//
// One call evaluates, at ONE node (shooting or collocation), the model equalities
// (awebox/mdl/model.py:125, 24 rows), the path inequalities (model.py:416-417, 9 rows), the
// power integrand (dynamics.py:318-330) and the side-slip output used by the beta cost
// (objective.py:390-421).  Row order follows the reference's constraint append order
// (dynamics.py:89-148, lagr_dyn.py:106-169); the trivial-kinematics rows come out in the sorted
// order of the SI struct keys (struct_operations.py:51-66, dynamics.py:924-934).
//
// The reference obtains the translational equations by symbolic differentiation of the
// Lagrangian with respect to the *scaled* generalised coordinates followed by a chain-rule time
// derivative (lagr_dyn.py:68-109, lagr_dyn_dir/tools.py:13-73).  Here the resulting expressions
// are written out analytically in SI units (equal in exact arithmetic); the CPU oracle
// (oracle/ap2_oracle.py) differentiates the Lagrangian automatically, so the two are
// independent.
//
// Structurally-zero reference terms that are omitted (com tether attachment,
// tether.attachment='com'):
//  * the tether moment n = 2 jacobian_dcm(lambda c)^T (forces.py:174-190) -- c has no r dependence
//  * the rotation-matrix term of time_derivative (tools.py:60-71) -- L, c, m_t have no r dependence
#pragma once

#include "scalar.hpp"
#include "../../include/awegpu.h"

namespace awe {

// Protocols
//   in(i)              node variable i (scaled, AWE_NW layout) as T
//   sink.eq_row(r, val)    model equality row r, emitted in increasing r (streamed so that a
//   sink.ineq_row(r, val)  GPU lane never holds all 33 dual rows at once); ineq after eq
//   sink.power(val), sink.beta(val)   integral-output derivative p / E_scale and side slip
// Storing sink, used on the host and in tests.
template <class T>
struct NodeResult {
    T eq[AWE_N_EQ];
    T ineq[AWE_N_INEQ];
    T pw;
    T bt;
    AWE_HD void eq_row(int r, const T& v) { eq[r] = v; }
    AWE_HD void ineq_row(int r, const T& v) { ineq[r] = v; }
    AWE_HD void power(const T& v) { pw = v; }
    AWE_HD void beta(const T& v) { bt = v; }
};

template <class T>
AWE_HD T dot3(const T* a, const T* b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }

// ISA density (atmosphere.py:60-78): rho_ref ((T_ref - gamma_air zz) / T_ref)^(g/(gamma_air R) - 1),
// evaluated as exp(expo log(.)) -- two short transcendental kernels instead of a full pow
template <class T, class PT>
AWE_HD T isa_density(const T& zz, const PT* th) {
    const auto expo = th[AWE_TH_G] / th[AWE_TH_GAMMA_AIR] / th[AWE_TH_R] - 1.0;
    T ratio = 1.0 - zz * (th[AWE_TH_GAMMA_AIR] / th[AWE_TH_T_REF]);
    return th[AWE_TH_RHO_REF] * exp(expo * log(ratio));
}

// power-law wind speed u_ref (smooth_abs(zz, eps=1) / z_ref)^c_f (wind.py:184-208), with
// smooth_abs(zz) = sqrt(zz^2 + 1) folded into the logarithm
template <class T, class PT>
AWE_HD T wind_speed(const T& zz, const PT* th) {
    const auto p = th[AWE_TH_EXP_REF];
    const auto scale = th[AWE_TH_U_REF] * exp(-p * log(th[AWE_TH_Z_REF]));
    return scale * exp((0.5 * p) * log(zz * zz + 1.0));
}

// Height of the midpoint of tether element e of n_el (element.py:60-104): the element runs from
// the ground anchor (s = 0) to the kite (s = 1), lo = e / n_el, up = (e + 1) / n_el
template <class T>
AWE_HD T tether_element_height(int e, int n_el, const T& qz) {
    const double lo = (double)e / (double)n_el, up = (double)(e + 1) / (double)n_el;
    return (qz * up + qz * lo) / 2.0;
}

// One element of the 'multi' tether drag model (element.py:60-104, segment.py:38-65) given the
// wind speed and air density at the element's midpoint: the drag of element e on the main
// tether, lumped onto the kite node with the reference's shape factor.  The tether's lower end
// is the ground (q = dq = 0); its share of the drag is dropped.
template <class T, class PT>
AWE_HD void tether_element_drag(int e, int n_el, const T* q, const T* v, const T& diam, const T& uw,
                                const T& rho, const PT* th, T out[3]) {
    const double ds = 1.0 / n_el;
    const double s0 = 0.5 * ds, step = ((1.0 - 0.5 * ds) - s0) / (n_el - 1);
    const auto cd = th[AWE_TH_CD_TETHER];
    const double lo = (double)e / (double)n_el, up = (double)(e + 1) / (double)n_el;
    T ue[3];
    ue[0] = uw - (v[0] * up + v[0] * lo) / 2.0;
    ue[1] = -((v[1] * up + v[1] * lo) / 2.0);
    ue[2] = -((v[2] * up + v[2] * lo) / 2.0);
    T un = sqrt(dot3(ue, ue) + 1e-12);
    T tv[3];
    for (int i = 0; i < 3; ++i) tv[i] = q[i] * up - q[i] * lo;
    T lpar = dot3(tv, ue) / un;
    T lperp = sqrt(dot3(tv, tv) - lpar * lpar + 1e-12);
    T fac = cd * 0.5 * rho * un * diam * lperp;
    const double sg = (e == n_el - 1) ? (1.0 - 0.5 * ds) : (s0 + e * step);
    for (int i = 0; i < 3; ++i) out[i] = sg * (fac * ue[i]);
}

template <class T, class PT>
AWE_HD void tether_element(int e, int n_el, const T* q, const T* v, const T& diam, const PT* th,
                           T out[3]) {
    T zz = tether_element_height(e, n_el, q[2]);
    tether_element_drag(e, n_el, q, v, diam, wind_speed(zz, th), isa_density(zz, th), th, out);
}

// Sub-models that depend on very few node variables (kite-height wind and density on q_z; the
// tether drag on q, dq and diam_t).  The default provider evaluates them inline; the GPU kernel
// substitutes a provider that returns values and partial derivatives preaccumulated once per
// node, lane-parallel, so that the per-direction model pass does not repeat them.
struct InlineSubmodels {
    template <class T, class PT>
    AWE_HD void kite_atmosphere(const T& qz, const PT* th, T& uw, T& rho) const {
        uw = wind_speed(qz, th);
        rho = isa_density(qz, th);
    }
    template <class T, class PT, class CT>
    AWE_HD void tether_drag(const T* q, const T* v, const T& diam, const PT* th, const CT* cst,
                            T D[3]) const {
        const int n_el = structural(cst[AWE_C_N_ELEMENTS]);
        for (int i = 0; i < 3; ++i) D[i] = T(0.0);
        for (int e = 0; e < n_el; ++e) {
            T c[3];
            tether_element(e, n_el, q, v, diam, th, c);
            for (int i = 0; i < 3; ++i) D[i] = D[i] + c[i];
        }
    }
};

// Rows are emitted phase by phase (DCM, trivial, aero -> rotation -> path constraints, tether
// drag -> translation -> holonomic) and every phase re-reads its inputs through `in`, so that
// short live ranges keep the dual-number working set inside the register file of one lane.
template <class T, class In, class Sink, class Sub = InlineSubmodels, class PT = double, class CT = double>
AWE_HD void ap2_node(const In& in, const T& gamma, const PT* th, const CT* cst,
                     Sink& out, bool want_ineq, const Sub& sub = Sub()) {
    const CT* s = cst + AWE_C_SCALING;
    // SI value of node variable i (dynamics.py:924-934)
    auto SI = [&](int i) -> T { return in(i) * s[i]; };

    // ---- DCM kinematics with orthonormality Baumgarte (lagr_dyn.py:236-254) ------------
    {
        T R[9], om[3];
        for (int i = 0; i < 9; ++i) R[i] = SI(9 + i);            // column-major R[3*col + row]
        for (int i = 0; i < 3; ++i) om[i] = SI(6 + i);
        const auto kr2 = th[AWE_TH_KAPPA_R] / 2.0;
        for (int c = 0; c < 3; ++c) {
            T A[3];   // column c of kappa_r/2 (I - R^T R) + skew(omega)
            for (int r = 0; r < 3; ++r) {
                T rtr = R[3 * r] * R[3 * c] + R[3 * r + 1] * R[3 * c + 1] + R[3 * r + 2] * R[3 * c + 2];
                A[r] = kr2 * ((r == c ? 1.0 : 0.0) - rtr);
            }
            if (c == 0) { A[1] = A[1] + om[2]; A[2] = A[2] - om[1]; }
            if (c == 1) { A[0] = A[0] - om[2]; A[2] = A[2] + om[0]; }
            if (c == 2) { A[0] = A[0] + om[1]; A[1] = A[1] - om[0]; }
            for (int r = 0; r < 3; ++r) {
                T RA = R[r] * A[0] + R[3 + r] * A[1] + R[6 + r] * A[2];
                out.eq_row(7 + 3 * c + r, SI(32 + 3 * c + r) - RA);
            }
        }
    }

    // ---- trivial kinematics, sorted names: ddelta10, ddl_t, dl_t, dq10 (lagr_dyn.py:141-169)
    for (int i = 0; i < 3; ++i)
        out.eq_row(16 + i, (SI(41 + i) - SI(52 + i)) / sqrt(s[52 + i] * s[41 + i]));
    out.eq_row(19, (SI(45) - SI(55)) / sqrt(s[55] * s[45]));
    out.eq_row(20, (SI(44) - SI(22)) / sqrt(s[22] * s[44]));
    for (int i = 0; i < 3; ++i)
        out.eq_row(21 + i, (SI(23 + i) - SI(3 + i)) / sqrt(s[3 + i] * s[23 + i]));

    // ---- kite aerodynamics (kite_aero.py:63-117, six_dof_kite.py:165-201) -------------
    T F_earth[3];
    {
        T ua[3], ua_e1, ua_e2, ua_e3, uu, airspeed, rho_k;
        {
            T uw;
            sub.kite_atmosphere(SI(2), th, uw, rho_k);
            ua[0] = uw - SI(3);
            ua[1] = -SI(4);
            ua[2] = -SI(5);
        }
        ua_e1 = ua[0] * SI(9) + ua[1] * SI(10) + ua[2] * SI(11);
        ua_e2 = ua[0] * SI(12) + ua[1] * SI(13) + ua[2] * SI(14);
        ua_e3 = ua[0] * SI(15) + ua[1] * SI(16) + ua[2] * SI(17);
        uu = dot3(ua, ua);
        airspeed = sqrt(uu);                                  // vect_op.norm
        T x_comp = sqrt(ua_e1 * ua_e1 + 1e-16);               // smooth_abs(., 1e-8)
        T alpha = ua_e3 / x_comp;                             // indicators.get_alpha
        T beta = ua_e2 / x_comp;                              // indicators.get_beta

        const auto b_ref = th[AWE_TH_B_REF], c_ref = th[AWE_TH_C_REF], s_ref = th[AWE_TH_S_REF];
        T coeff[6];
        {
            // p, q, r in the control frame (stability_derivatives.py:202-226)
            T inv2a = 1.0 / (2.0 * airspeed);
            const PT* sd = th + AWE_TH_STAB_DERIVS;
            const CT* sdl = cst + AWE_C_SD_LEN;
            const auto mf = th[AWE_TH_MOMENT_FACTOR];
            T alpha2 = alpha * alpha;
            for (int c = 0; c < 6; ++c) coeff[c] = T(0.0);
            for (int i = 0; i < 9; ++i) {
                T inp;
                switch (i) {
                    case 0: inp = T(1.0); break;
                    case 1: inp = alpha; break;
                    case 2: inp = -beta; break;                     // control-frame sign (:150)
                    case 3: inp = (-SI(6)) * inv2a * b_ref; break;
                    case 4: inp = SI(7) * inv2a * c_ref; break;
                    case 5: inp = (-SI(8)) * inv2a * b_ref; break;
                    default: inp = SI(18 + i - 6); break;            // delta a, e, r
                }
                T ia = inp * alpha, ia2 = inp * alpha2;
                for (int c = 0; c < 6; ++c) {
                    const int n = structural(sdl[c * 9 + i]);
                    if (n == 0) continue;
                    const PT* dv = sd + (c * 9 + i) * 3;
                    // sum_l deriv[l] * input * alpha^l (stability_derivatives.py:166-200)
                    T contrib = dv[0] * inp;
                    if (n > 1) contrib = contrib + dv[1] * ia;
                    if (n > 2) contrib = contrib + dv[2] * ia2;
                    coeff[c] = coeff[c] + ((c >= 3 && i >= 6) ? mf * contrib : contrib);
                }
            }
        }
        T qs = (0.5 * rho_k * uu) * s_ref;
        // control frame -> earth: R diag(-1, 1, -1) F_ctrl (frames.py:69-72)
        {
            T fc0 = -(coeff[0] * qs), fc1 = coeff[1] * qs, fc2 = -(coeff[2] * qs);
            for (int i = 0; i < 3; ++i) F_earth[i] = SI(9 + i) * fc0 + SI(12 + i) * fc1 + SI(15 + i) * fc2;
        }
            // ---- rotational dynamics (lagr_dyn.py:207-234) --------------------------------
        {
            T M_body[3];
            M_body[0] = -(qs * (b_ref * coeff[3]));                // frames.from_control_to_body
            M_body[1] = qs * (c_ref * coeff[4]);
            M_body[2] = -(qs * (b_ref * coeff[5]));
            const PT* J = th + AWE_TH_J;   // column-major
            T om[3], Jw[3];
            for (int i = 0; i < 3; ++i) om[i] = SI(6 + i);
            for (int i = 0; i < 3; ++i) Jw[i] = J[i] * om[0] + J[3 + i] * om[1] + J[6 + i] * om[2];
            T wxJw[3];
            wxJw[0] = om[1] * Jw[2] - om[2] * Jw[1];
            wxJw[1] = -(om[0] * Jw[2] - om[2] * Jw[0]);
            wxJw[2] = om[0] * Jw[1] - om[1] * Jw[0];
            const auto inv_ms = 1.0 / cst[AWE_C_M_AERO_SCALING];
            for (int i = 0; i < 3; ++i) {
                T Jdw = J[i] * SI(29) + J[3 + i] * SI(30) + J[6 + i] * SI(31);
                T M = gamma * SI(49 + i) + M_body[i];
                out.eq_row(4 + i, (M - (Jdw + wxJw[i])) * inv_ms);
            }
        }
            // ---- path inequalities (dynamics.py:655-821, 1022-1117; indicators.py:286-338) -
        if (want_ineq) {
            T q[3];
            for (int i = 0; i < 3; ++i) q[i] = SI(i);
            T nq = sqrt(dot3(q, q));
            T tension = SI(56) * nq;
            const auto fscale = cst[AWE_C_LAMBDA_SCALING] * cst[AWE_C_SCALING_LENGTH];
            out.ineq_row(0, (tension - th[AWE_TH_FORCE_LIMITS + 1]) / fscale);
            out.ineq_row(1, (th[AWE_TH_FORCE_LIMITS + 0] - tension) / fscale);
            const auto u_ref = th[AWE_TH_U_REF];
            out.ineq_row(2, (airspeed - th[AWE_TH_AIRSPEED_LIMITS + 1]) / u_ref);
            out.ineq_row(3, (th[AWE_TH_AIRSPEED_LIMITS + 0] - airspeed) / u_ref);
            const auto tight = cst[AWE_C_AERO_TIGHTNESS], aref = cst[AWE_C_AIRSPEED_REF];
            const auto amax = cst[AWE_C_ALPHA_MAX], amin = cst[AWE_C_ALPHA_MIN];
            const auto bmax = cst[AWE_C_BETA_MAX], bmin = cst[AWE_C_BETA_MIN];
            out.ineq_row(4, (ua_e3 - ua_e1 * amax) * tight / aref / sqrt(amax * amax + 1e-16));
            out.ineq_row(5, (-ua_e3 + ua_e1 * amin) * tight / aref / sqrt(amin * amin + 1e-16));
            out.ineq_row(6, (ua_e2 - ua_e1 * bmax) * tight / aref / sqrt(bmax * bmax + 1e-16));
            out.ineq_row(7, (-ua_e2 + ua_e1 * bmin) * tight / aref / sqrt(bmin * bmin + 1e-16));
            const auto cos_gmax = cos(th[AWE_TH_ROT_ANGLES + 2]);
            T yaw = (q[0] * SI(15) + q[1] * SI(16) + q[2] * SI(17) - cos_gmax * nq) / cst[AWE_C_SCALING_LENGTH];
            out.ineq_row(8, -1.0 * yaw);
        }
        out.beta(beta);
    }
    out.power(SI(56) * SI(21) * SI(22) / cst[AWE_C_ENERGY_SCALING]);   // dynamics.py:318-330

    // ---- translational Lagrangian dynamics (lagr_dyn.py:68-109, 174-204) --------------
    const auto g_grav = th[AWE_TH_G];
    const auto m_k = th[AWE_TH_M_K];
    const auto rho_t = th[AWE_TH_RHO_TETHER];
    T q[3], v[3];
    for (int i = 0; i < 3; ++i) q[i] = SI(i);
    for (int i = 0; i < 3; ++i) v[i] = SI(3 + i);
    T diam = SI(57);
    T D_tether[3];
    sub.tether_drag(q, v, diam, th, cst, D_tether);
    {
        T qq = dot3(q, q);
        T nq = sqrt(qq);                                      // vect_op.norm (eps = 0)
        T mu = (3.14159265358979323846 * (diam / 2.0) * (diam / 2.0)) * rho_t;   // m_t = mu |q|
        T lam = SI(56);
        T a[3];
        for (int i = 0; i < 3; ++i) a[i] = SI(26 + i);       // xdot ddq10
        T sv = dot3(q, v);
        T vv = dot3(v, v);
        T qa = dot3(q, a);
        T inv_n = 1.0 / nq;
        T inv_n3 = inv_n * inv_n * inv_n;
        T mu6 = mu / 6.0;
        // d/dt dL/dqdot with KE_t = (mu/6)(|q||v|^2 + 2 (q.v)^2/|q|)  (energy.py:59-97)
        T cv = mu * sv * inv_n;
        T cq = mu6 * (4.0 * (vv + qa) * inv_n - 4.0 * sv * sv * inv_n3);
        T ca = mu6 * (2.0 * nq) + m_k;
        // dL/dq = dKE/dq - dPE/dq - lambda q (energy.py:100-144, holonomics.py:204-264)
        T kq = mu6 * (vv * inv_n - 2.0 * sv * sv * inv_n3);
        T kv = mu6 * (4.0 * sv * inv_n);
        T pq = g_grav * mu * (q[2] * inv_n) * 0.5;
        T pz = g_grav * mu * nq * 0.5 + g_grav * m_k;
        T mass_flow = mu * sv * inv_n;                        // d(m_t)/dt (lagr_dyn.py:174-204)
        const auto scaling_mass = 3.14159265358979323846 * (cst[AWE_C_SCALING_DIAM] / 2.0) *
                                    (cst[AWE_C_SCALING_DIAM] / 2.0) * rho_t * cst[AWE_C_SCALING_LENGTH];
        const auto node_mass = scaling_mass / 2.0 + m_k;    // mass.py:62-93
        const auto inv_force_scaling = 1.0 / (node_mass * cst[AWE_C_G_SCALING] * 10.0);
        for (int i = 0; i < 3; ++i) {
            T ddt = cv * v[i] + cq * q[i] + ca * a[i];
            T dLdq = kq * q[i] + kv * v[i] - pq * q[i] - lam * q[i];
            if (i == 2) dLdq = dLdq - pz;
            T lhs = ddt - dLdq;
            T F = D_tether[i] + (gamma * SI(46 + i) + F_earth[i]);   // forces.py:47-80, 148-171
            T rhs = F + mass_flow * v[i];
            out.eq_row(i, (lhs - rhs) * inv_force_scaling);
        }
        // ---- holonomic constraint + Baumgarte (holonomics.py:17-123, 267-312) ----------
        T l_t = SI(21), dl_t = SI(22), ldd = SI(55);          // ddl_t from u (tools.py:13-73)
        T c0 = 0.5 * (qq - l_t * l_t);
        T c1 = sv - l_t * dl_t;
        T c2 = vv + qa - dl_t * dl_t - l_t * ldd;
        const auto kap = th[AWE_TH_KAPPA];
        T hl = c2 + 2.0 * kap * c1 + kap * kap * c0;
        const auto hscale = kap * kap * (cst[AWE_C_SCALING_LENGTH] * cst[AWE_C_Q_SCALING_MEAN]);
        out.eq_row(3, hl / hscale);
    }
}

}  // namespace awe
