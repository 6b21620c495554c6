// Multi-kite node model: two 6-DOF Ampyx AP2 kites on secondary tethers below the layer node 1
// (architecture {1: 0, 2: 1, 3: 1}, examples/dual_kites_power_curve.py), hand-written for CDNA4
// and instantiated on double / Dual / Dep2 (scalar.hpp), and on the tracing scalar of the
// build-time code generator (gen/sym.hpp: the parameters th and the constants cst then enter as
// symbols of their own types PT / CT, the integer structure through structural()).
//
// One call evaluates, at ONE node, the 53 model equalities (model.py:125; append order of
// dynamics.py:89-148 and lagr_dyn.py:106-169), the 19 path inequalities (dynamics.py:122-148:
// tether force per kite, airspeed per kite, aero validity per kite, anticollision, yaw per kite),
// the power integrand (dynamics.py:318-330) and the two side slips of the beta cost
// (objective.py:390-421).  Row numbering: see include/awedual.h and awebox_amd/dual.py.
//
// Translational dynamics.  The reference differentiates L = T - V - sum lambda c symbolically
// w.r.t. the scaled generalised coordinates q10, q21, q31 (lagr_dyn.py:68-109).  Here L is split
// per tether segment and the Euler-Lagrange terms of each segment are written out in closed form
// (equal in exact arithmetic; the CPU oracle oracle/multikite_oracle.py differentiates
// automatically):
//   * main tether (ground -> node 1, energy.py:59-97 with the reel-out projection of dq10):
//     T = (mu_t / 6) (|q||v|^2 + 2 (q.v)^2 / |q|), V = g mu_t |q| q_z / 2;
//   * secondary tether (node 1 -> kite k, parent velocity dq10): with d = q_k - q10, L = |d|,
//     e = d / L, m = mu_s L, S = |v_k|^2 + |v_1|^2 + v_k.v_1,
//       d/dt dT/dv_k = (m'/6)(2 v_k + v_1) + (m/6)(2 a_k + a_1),  dT/dq_k = (mu_s/6) S e = -dT/dq_1,
//       dV/dq_k = g mu_s e (q_kz + q_1z)/2 + g m/2 e_z,  dV/dq_1 = -g mu_s e (q_kz + q_1z)/2 + g m/2 e_z;
//   * constraint work lambda_n c_n, c = (|d|^2 - l^2)/2 (holonomics.py:204-264).
// Structurally-zero reference terms omitted (com attachment): the tether moments
// (forces.py:174-190) and the DCM term of time_derivative (tools.py:60-71).
#pragma once

#include "ap2_model.hpp"
#include "../../include/awedual.h"

namespace awe {

// node-variable offsets (include/awedual.h)
namespace dl {
constexpr int kQ10 = 0, kDQ10 = 3, kLT = 48, kDLT = 49, kXD = 50;
constexpr int kDDQ10 = kXD + kDQ10;                  // xdot ddq10
constexpr int kDDLT_U = 118;                          // u ddl_t
constexpr int kLam10 = 119, kDiamT = 122, kTf = 123, kLs = 124, kDiamS = 125, kGamma = 126;
AWE_HD constexpr int q(int k) { return 6 + 21 * k; }
AWE_HD constexpr int dq(int k) { return 9 + 21 * k; }
AWE_HD constexpr int om(int k) { return 12 + 21 * k; }
AWE_HD constexpr int r(int k) { return 15 + 21 * k; }
AWE_HD constexpr int del(int k) { return 24 + 21 * k; }
AWE_HD constexpr int ffict(int k) { return 100 + 9 * k; }
AWE_HD constexpr int mfict(int k) { return 103 + 9 * k; }
AWE_HD constexpr int ddel(int k) { return 106 + 9 * k; }
AWE_HD constexpr int lam(int k) { return 120 + k; }
// eq rows
constexpr int kRowTrans1 = 0, kRowHol1 = 9, kRowTriv = 36;
AWE_HD constexpr int row_trans(int k) { return 3 + 3 * k; }
AWE_HD constexpr int row_hol(int k) { return 10 + k; }
AWE_HD constexpr int row_rot(int k) { return 12 + 12 * k; }
AWE_HD constexpr int row_dcm(int k) { return 15 + 12 * k; }
// ineq rows
AWE_HD constexpr int irow_force(int k) { return 2 * k; }
AWE_HD constexpr int irow_airspeed(int k) { return 4 + 2 * k; }
AWE_HD constexpr int irow_valid(int k) { return 8 + 4 * k; }
constexpr int kIrowAnticollision = 16;
AWE_HD constexpr int irow_yaw(int k) { return 17 + k; }
}  // namespace dl

// Height of the midpoint of element e of a segment whose end heights are qbz (lower) and qtz
// (upper) (element.py:125-146): the wind and the air density of the element are taken there.
template <class T>
AWE_HD T element_height(int e, int n_el, const T& qbz, const T& qtz) {
    const double lo = (double)e / (double)n_el, up = (double)(e + 1) / (double)n_el;
    T dqs = qtz - qbz;
    return ((qbz + dqs * up) + (qbz + dqs * lo)) / 2.0;
}

// wind speed and density at an element midpoint, evaluated in place
struct InlineAtmosphere {
    template <class T, class PT>
    AWE_HD void operator()(int /*seg*/, int /*e*/, const T& zz, const PT* th, T& uw, T& rho) const {
        uw = wind_speed(zz, th);
        rho = isa_density(zz, th);
    }
};

// One element of the 'multi' drag model of a tether segment from (qb, vb) to (qt, vt)
// (element.py:60-146, segment.py:38-65): the element's drag vector, not yet split.  `seg`
// (0 main, 1 + k secondary of kite k) and `e` identify the element for the atmosphere provider.
template <class T, class PT, class Atm = InlineAtmosphere>
AWE_HD void segment_element_drag(int seg, int e, int n_el, const T* qb, const T* qt, const T* vb, const T* vt,
                                 const T& diam, const PT* th, T out[3], const Atm& atm = Atm()) {
    const double lo = (double)e / (double)n_el, up = (double)(e + 1) / (double)n_el;
    T qu[3], ql[3], vs[3], tv[3];
    for (int i = 0; i < 3; ++i) {
        T dqs = qt[i] - qb[i], dvs = vt[i] - vb[i];
        qu[i] = qb[i] + dqs * up;
        ql[i] = qb[i] + dqs * lo;
        vs[i] = (vb[i] + dvs * up) + (vb[i] + dvs * lo);
        tv[i] = qu[i] - ql[i];
    }
    T zz = element_height(e, n_el, qb[2], qt[2]);
    T uw, rho;
    atm(seg, e, zz, th, uw, rho);
    T ue[3];
    ue[0] = uw - vs[0] / 2.0;
    ue[1] = -(vs[1] / 2.0);
    ue[2] = -(vs[2] / 2.0);
    T un = sqrt(dot3(ue, ue) + 1e-12);                  // smooth_norm(ua, 1e-6)
    T lpar = dot3(tv, ue) / un;
    T lperp = sqrt(dot3(tv, tv) - lpar * lpar + 1e-12); // smooth_sqrt(., 1e-12)
    T fac = th[AWE_TH_CD_TETHER] * 0.5 * rho * un * diam * lperp;
    for (int i = 0; i < 3; ++i) out[i] = fac * ue[i];
}

// midpoint-rule share of element e that goes to the upper node (segment.py:50-63)
AWE_HD double element_upper_share(int e, int n_el) {
    const double ds = 1.0 / n_el;
    const double s0 = 0.5 * ds;
    if (n_el == 1) return s0;
    const double step = ((1.0 - 0.5 * ds) - s0) / (n_el - 1);
    return (e == n_el - 1) ? (1.0 - 0.5 * ds) : (s0 + e * step);
}

// Sub-models that depend on few node variables: the kite-height wind and density (on q_kz), the
// main-tether drag (on q10, dq10, diam_t: 7 inputs) and each secondary-tether drag (on q10, dq10,
// q_k, dq_k, diam_s: 13 inputs).  The default provider evaluates them inline; the GPU kernel
// substitutes one that returns values and partial derivatives preaccumulated once per node.
struct DualInlineSubmodels {
    template <class T, class PT>
    AWE_HD void kite_atmosphere(const T& qz, const PT* th, T& uw, T& rho) const {
        uw = wind_speed(qz, th);
        rho = isa_density(qz, th);
    }
    // main tether: ground -> node 1; only the upper share is kept (tether_aero.py:85-95)
    template <class T, class PT, class CT, class Atm = InlineAtmosphere>
    AWE_HD void main_drag(const T* q, const T* v, const T& diam, const PT* th, const CT* cst,
                          T up[3], const Atm& atm = Atm()) const {
        const int n_el = structural(cst[ADL_C_N_ELEMENTS]);
        T z3[3] = {T(0.0), T(0.0), T(0.0)};
        for (int i = 0; i < 3; ++i) up[i] = T(0.0);
        for (int e = 0; e < n_el; ++e) {
            T c[3];
            segment_element_drag(0, e, n_el, z3, q, z3, v, diam, th, c, atm);
            const double sg = element_upper_share(e, n_el);
            for (int i = 0; i < 3; ++i) up[i] = up[i] + sg * c[i];
        }
    }
    // secondary tether node 1 -> kite: upper share to the kite, lower share to node 1
    template <class T, class PT, class CT, class Atm = InlineAtmosphere>
    AWE_HD void sec_drag(int k, const T* qb, const T* vb, const T* qt, const T* vt, const T& diam,
                         const PT* th, const CT* cst, T up[3], T lo[3], const Atm& atm = Atm()) const {
        const int n_el = structural(cst[ADL_C_N_ELEMENTS]);
        for (int i = 0; i < 3; ++i) { up[i] = T(0.0); lo[i] = T(0.0); }
        for (int e = 0; e < n_el; ++e) {
            T c[3];
            segment_element_drag(1 + k, e, n_el, qb, qt, vb, vt, diam, th, c, atm);
            const double sg = element_upper_share(e, n_el);
            for (int i = 0; i < 3; ++i) {
                up[i] = up[i] + sg * c[i];
                lo[i] = lo[i] + (1.0 - sg) * c[i];
            }
        }
    }
};

// Sink protocol: eq_row(r, v) r < ADL_N_EQ, ineq_row(r, v) r < ADL_N_INEQ, power(v), beta(k, v).
//
// Phases are ordered so that no per-kite state outlives its kite: each kite's DCM, aerodynamics,
// rotation, path rows and then its secondary tether segment (drag, Lagrange terms, translation
// and holonomic rows) are evaluated in one loop body; only the node-1 accumulator (3 values)
// crosses iterations.  Inputs are re-read through `in` where they are needed, keeping the
// dual-number working set of one lane small.
//
// first_kite = 1 evaluates kite 3 before kite 2 (only the order of node 1's two accumulations
// changes): the code generator traces kite 3's rows that way, so that the values they share with
// node 1 are formed next to their use.
template <class T, class In, class Sink, class Sub = DualInlineSubmodels, class PT = double, class CT = double>
AWE_HD void dual_node(const In& in, const T& gamma, const PT* th, const CT* cst, Sink& out,
                      bool want_ineq, const Sub& sub = Sub(), int first_kite = 0) {
    using namespace dl;
    const CT* s = cst + ADL_C_SCALING;
    auto SI = [&](int i) -> T { return in(i) * s[i]; };
    const double pi = 3.14159265358979323846;
    const auto g_grav = th[AWE_TH_G];
    const auto m_k = th[AWE_TH_M_K];
    const auto rho_t = th[AWE_TH_RHO_TETHER];
    const auto kap = th[AWE_TH_KAPPA];
    const auto gs10 = cst[ADL_C_G_SCALING] * 10.0;
    const auto sm_s = pi * (cst[ADL_C_SCALING_DIAM_S] / 2.0) * (cst[ADL_C_SCALING_DIAM_S] / 2.0) * rho_t *
                        cst[ADL_C_SCALING_LENGTH_S];

    T acc1[3] = {T(0.0), T(0.0), T(0.0)};   // node 1: secondary-segment Lagrange terms - lower drag shares
#pragma unroll 1
    for (int kk = 0; kk < 2; ++kk) {
        const int k = first_kite ? 1 - kk : kk;
        // ---- DCM kinematics with orthonormality Baumgarte (lagr_dyn.py:236-254) ----------
        {
            T R[9], w[3];
            for (int i = 0; i < 9; ++i) R[i] = SI(r(k) + i);
            for (int i = 0; i < 3; ++i) w[i] = SI(om(k) + i);
            const auto kr2 = th[AWE_TH_KAPPA_R] / 2.0;
            for (int c = 0; c < 3; ++c) {
                T A[3];
                for (int rr = 0; rr < 3; ++rr) {
                    T rtr = R[3 * rr] * R[3 * c] + R[3 * rr + 1] * R[3 * c + 1] + R[3 * rr + 2] * R[3 * c + 2];
                    A[rr] = kr2 * ((rr == c ? 1.0 : 0.0) - rtr);
                }
                if (c == 0) { A[1] = A[1] + w[2]; A[2] = A[2] - w[1]; }
                if (c == 1) { A[0] = A[0] - w[2]; A[2] = A[2] + w[0]; }
                if (c == 2) { A[0] = A[0] + w[1]; A[1] = A[1] - w[0]; }
                for (int rr = 0; rr < 3; ++rr) {
                    T RA = R[rr] * A[0] + R[3 + rr] * A[1] + R[6 + rr] * A[2];
                    out.eq_row(row_dcm(k) + 3 * c + rr, SI(kXD + r(k) + 3 * c + rr) - RA);
                }
            }
        }
        // ---- kite aerodynamics (kite_aero.py:63-117, six_dof_kite.py:165-201) -----------
        T Fa[3];     // gamma f_fict + aerodynamic force, earth frame (forces.py:148-171)
        {
            T ua[3], ua_e1, ua_e2, ua_e3, uu, airspeed, rho_k;
            {
                T uw;
                sub.kite_atmosphere(SI(q(k) + 2), th, uw, rho_k);
                ua[0] = uw - SI(dq(k));
                ua[1] = -SI(dq(k) + 1);
                ua[2] = -SI(dq(k) + 2);
            }
            ua_e1 = ua[0] * SI(r(k)) + ua[1] * SI(r(k) + 1) + ua[2] * SI(r(k) + 2);
            ua_e2 = ua[0] * SI(r(k) + 3) + ua[1] * SI(r(k) + 4) + ua[2] * SI(r(k) + 5);
            ua_e3 = ua[0] * SI(r(k) + 6) + ua[1] * SI(r(k) + 7) + ua[2] * SI(r(k) + 8);
            uu = dot3(ua, ua);
            airspeed = sqrt(uu);
            T x_comp = sqrt(ua_e1 * ua_e1 + 1e-16);
            T alpha = ua_e3 / x_comp;
            T beta = ua_e2 / x_comp;
            const auto b_ref = th[AWE_TH_B_REF], c_ref = th[AWE_TH_C_REF], s_ref = th[AWE_TH_S_REF];
            T coeff[6];
            {
                T inv2a = 1.0 / (2.0 * airspeed);
                const PT* sd = th + AWE_TH_STAB_DERIVS;
                const CT* sdl = cst + ADL_C_SD_LEN;
                const auto mf = th[AWE_TH_MOMENT_FACTOR];
                T alpha2 = alpha * alpha;
                for (int c = 0; c < 6; ++c) coeff[c] = T(0.0);
                for (int i = 0; i < 9; ++i) {
                    T inp;
                    switch (i) {
                        case 0: inp = T(1.0); break;
                        case 1: inp = alpha; break;
                        case 2: inp = -beta; break;
                        case 3: inp = (-SI(om(k))) * inv2a * b_ref; break;
                        case 4: inp = SI(om(k) + 1) * inv2a * c_ref; break;
                        case 5: inp = (-SI(om(k) + 2)) * inv2a * b_ref; break;
                        default: inp = SI(del(k) + i - 6); break;
                    }
                    T ia = inp * alpha, ia2 = inp * alpha2;
                    for (int c = 0; c < 6; ++c) {
                        const int n = structural(sdl[c * 9 + i]);
                        if (n == 0) continue;
                        const PT* dv = sd + (c * 9 + i) * 3;
                        T contrib = dv[0] * inp;
                        if (n > 1) contrib = contrib + dv[1] * ia;
                        if (n > 2) contrib = contrib + dv[2] * ia2;
                        // (1.0 * contrib is contrib exactly: the unweighted terms skip the product)
                        coeff[c] = coeff[c] + ((c >= 3 && i >= 6) ? mf * contrib : contrib);
                    }
                }
            }
            T qs = (0.5 * rho_k * uu) * s_ref;
            {
                T fc0 = -(coeff[0] * qs), fc1 = coeff[1] * qs, fc2 = -(coeff[2] * qs);
                for (int i = 0; i < 3; ++i)
                    Fa[i] = gamma * SI(ffict(k) + i) +
                            (SI(r(k) + i) * fc0 + SI(r(k) + 3 + i) * fc1 + SI(r(k) + 6 + i) * fc2);
            }
            // ---- rotational dynamics (lagr_dyn.py:207-234) ---------------------------------
            {
                T M_body[3];
                M_body[0] = -(qs * (b_ref * coeff[3]));
                M_body[1] = qs * (c_ref * coeff[4]);
                M_body[2] = -(qs * (b_ref * coeff[5]));
                const PT* J = th + AWE_TH_J;
                T w[3], Jw[3];
                for (int i = 0; i < 3; ++i) w[i] = SI(om(k) + i);
                for (int i = 0; i < 3; ++i) Jw[i] = J[i] * w[0] + J[3 + i] * w[1] + J[6 + i] * w[2];
                T wxJw[3];
                wxJw[0] = w[1] * Jw[2] - w[2] * Jw[1];
                wxJw[1] = -(w[0] * Jw[2] - w[2] * Jw[0]);
                wxJw[2] = w[0] * Jw[1] - w[1] * Jw[0];
                const auto inv_ms = 1.0 / cst[ADL_C_M_AERO_SCALING];
                for (int i = 0; i < 3; ++i) {
                    const int xw = kXD + om(k);
                    T Jdw = J[i] * SI(xw) + J[3 + i] * SI(xw + 1) + J[6 + i] * SI(xw + 2);
                    T M = gamma * SI(mfict(k) + i) + M_body[i];
                    out.eq_row(row_rot(k) + i, (M - (Jdw + wxJw[i])) * inv_ms);
                }
            }
            // ---- path inequalities of kite k ---------------------------------------------
            if (want_ineq) {
                T dd[3];
                for (int i = 0; i < 3; ++i) dd[i] = SI(q(k) + i) - SI(kQ10 + i);
                T nd = sqrt(dot3(dd, dd));
                T tension = SI(lam(k)) * nd;                                   // dynamics.py:706-776
                const auto fscale = s[lam(k)] * cst[ADL_C_SCALING_LENGTH_S];
                out.ineq_row(irow_force(k), (tension - th[AWE_TH_FORCE_LIMITS + 1]) / fscale);
                out.ineq_row(irow_force(k) + 1, (th[AWE_TH_FORCE_LIMITS + 0] - tension) / fscale);
                const auto u_ref = th[AWE_TH_U_REF];
                out.ineq_row(irow_airspeed(k), (airspeed - th[AWE_TH_AIRSPEED_LIMITS + 1]) / u_ref);
                out.ineq_row(irow_airspeed(k) + 1, (th[AWE_TH_AIRSPEED_LIMITS + 0] - airspeed) / u_ref);
                const auto tight = cst[ADL_C_AERO_TIGHTNESS], aref = cst[ADL_C_AIRSPEED_REF];
                const auto amax = cst[ADL_C_ALPHA_MAX], amin = cst[ADL_C_ALPHA_MIN];
                const auto bmax = cst[ADL_C_BETA_MAX], bmin = cst[ADL_C_BETA_MIN];
                out.ineq_row(irow_valid(k), (ua_e3 - ua_e1 * amax) * tight / aref / sqrt(amax * amax + 1e-16));
                out.ineq_row(irow_valid(k) + 1, (-ua_e3 + ua_e1 * amin) * tight / aref / sqrt(amin * amin + 1e-16));
                out.ineq_row(irow_valid(k) + 2, (ua_e2 - ua_e1 * bmax) * tight / aref / sqrt(bmax * bmax + 1e-16));
                out.ineq_row(irow_valid(k) + 3, (-ua_e2 + ua_e1 * bmin) * tight / aref / sqrt(bmin * bmin + 1e-16));
                const auto cos_gmax = cos(th[AWE_TH_ROT_ANGLES + 2]);      // dynamics.py:1022-1052
                T yaw = (dd[0] * SI(r(k) + 6) + dd[1] * SI(r(k) + 7) + dd[2] * SI(r(k) + 8) - cos_gmax * nd) /
                        cst[ADL_C_SCALING_LENGTH_S];
                out.ineq_row(irow_yaw(k), -1.0 * yaw);
            }
            out.beta(k, beta);
        }
        // ---- secondary tether segment node 1 -> kite k: drag, Lagrange terms, rows ---------
        {
            T q1[3], v1[3], qk[3], vk[3];
            for (int i = 0; i < 3; ++i) {
                q1[i] = SI(kQ10 + i);
                v1[i] = SI(kDQ10 + i);
                qk[i] = SI(q(k) + i);
                vk[i] = SI(dq(k) + i);
            }
            T diam = SI(kDiamS);
            T up[3], lo[3];
            sub.sec_drag(k, q1, v1, qk, vk, diam, th, cst, up, lo);
            T d[3], wv[3];
            for (int i = 0; i < 3; ++i) {
                d[i] = qk[i] - q1[i];
                wv[i] = vk[i] - v1[i];
            }
            T dd = dot3(d, d);
            T L = sqrt(dd);
            T invL = 1.0 / L;
            T mu = (pi * (diam / 2.0) * (diam / 2.0)) * rho_t;
            T m = mu * L;
            T mdot6 = (mu * dot3(d, wv) * invL) / 6.0;
            T m6 = m / 6.0;
            T S = dot3(vk, vk) + dot3(v1, v1) + dot3(vk, v1);
            T ge = g_grav * mu * (qk[2] + q1[2]) * 0.5 * invL;   // coefficient of d in dV/dq_k
            T te = (mu / 6.0) * S * invL;                         // coefficient of d in dT/dq_k
            T lamk = SI(lam(k));
            T gm2 = g_grav * m * 0.5;
            const auto inv_fs = 1.0 / ((sm_s / 2.0 + m_k) * gs10);
            T c2a(0.0);
            for (int i = 0; i < 3; ++i) {
                T ak = SI(kXD + dq(k) + i), a1 = SI(kDDQ10 + i);
                c2a = c2a + d[i] * (ak - a1);
                T common = (ge - te + lamk) * d[i];
                T lk = m_k * ak + mdot6 * (2.0 * vk[i] + v1[i]) + m6 * (2.0 * ak + a1) + common;
                T l1 = mdot6 * (2.0 * v1[i] + vk[i]) + m6 * (2.0 * a1 + ak) - common;
                if (i == 2) {
                    lk = lk + gm2 + g_grav * m_k;
                    l1 = l1 + gm2;
                }
                acc1[i] = acc1[i] + (l1 - lo[i]);
                out.eq_row(row_trans(k) + i, (lk - (Fa[i] + up[i])) * inv_fs);
            }
            // holonomic constraint of the secondary tether, l_s constant (theta)
            T ls = SI(kLs);
            T c0 = 0.5 * (dd - ls * ls);
            T c1 = dot3(d, wv);
            T c2 = dot3(wv, wv) + c2a;
            const auto hscale =
                kap * kap * (cst[ADL_C_SCALING_LENGTH_S] * ((s[q(k)] + s[q(k) + 1] + s[q(k) + 2]) / 3.0));
            out.eq_row(row_hol(k), (c2 + 2.0 * kap * c1 + kap * kap * c0) / hscale);
        }
    }

    // ---- trivial kinematics, sorted names (lagr_dyn.py:141-169) -------------------------
    {
        auto triv = [&](int row, int ixd, int iu) {
            out.eq_row(row, (SI(ixd) - SI(iu)) / sqrt(s[iu] * s[ixd]));
        };
        for (int i = 0; i < 3; ++i) triv(kRowTriv + i, kXD + del(0) + i, ddel(0) + i);       // ddelta21
        for (int i = 0; i < 3; ++i) triv(kRowTriv + 3 + i, kXD + del(1) + i, ddel(1) + i);   // ddelta31
        triv(kRowTriv + 6, kXD + kDLT, kDDLT_U);                                            // ddl_t
        triv(kRowTriv + 7, kXD + kLT, kDLT);                                                // dl_t
        for (int i = 0; i < 3; ++i) triv(kRowTriv + 8 + i, kXD + kQ10 + i, kDQ10 + i);       // dq10
        for (int i = 0; i < 3; ++i) triv(kRowTriv + 11 + i, kXD + q(0) + i, dq(0) + i);      // dq21
        for (int i = 0; i < 3; ++i) triv(kRowTriv + 14 + i, kXD + q(1) + i, dq(1) + i);      // dq31
    }
    // ---- anticollision (dynamics.py:457-484) ---------------------------------------------
    if (want_ineq) {
        T dd[3];
        for (int i = 0; i < 3; ++i) dd[i] = SI(q(0) + i) - SI(q(1) + i);
        const auto dmin = cst[ADL_C_ANTICOLLISION_DIST_MIN];
        out.ineq_row(kIrowAnticollision, 1.0 - dot3(dd, dd) / (dmin * dmin));
    }
    out.power(SI(kLam10) * SI(kLT) * SI(kDLT) / cst[ADL_C_ENERGY_SCALING]);

    // ---- main tether segment (energy.py:59-97), node-1 translation, main holonomic --------
    {
        const auto sm_t = pi * (cst[ADL_C_SCALING_DIAM_T] / 2.0) * (cst[ADL_C_SCALING_DIAM_T] / 2.0) * rho_t *
                          cst[ADL_C_SCALING_LENGTH_T];
        const auto inv_fs1 = 1.0 / ((sm_t / 2.0 + 2.0 * (sm_s / 2.0)) * gs10);   // mass.py:62-93
        T q1[3], v1[3], a1[3];
        for (int i = 0; i < 3; ++i) {
            q1[i] = SI(kQ10 + i);
            v1[i] = SI(kDQ10 + i);
            a1[i] = SI(kDDQ10 + i);
        }
        T diam = SI(kDiamT);
        T F1[3];
        sub.main_drag(q1, v1, diam, th, cst, F1);                  // upper share only
        T qq = dot3(q1, q1);
        T nq = sqrt(qq);
        T mu = (pi * (diam / 2.0) * (diam / 2.0)) * rho_t;
        T lam1 = SI(kLam10);
        T sv = dot3(q1, v1), vv = dot3(v1, v1), qa = dot3(q1, a1);
        T inv_n = 1.0 / nq;
        T inv_n3 = inv_n * inv_n * inv_n;
        T mu6 = mu / 6.0;
        T cv = mu * sv * inv_n;
        T cq = mu6 * (4.0 * (vv + qa) * inv_n - 4.0 * sv * sv * inv_n3);
        T ca = mu6 * (2.0 * nq);
        T kq = mu6 * (vv * inv_n - 2.0 * sv * sv * inv_n3);
        T kv = mu6 * (4.0 * sv * inv_n);
        T pq = g_grav * mu * (q1[2] * inv_n) * 0.5;
        T mass_flow = mu * sv * inv_n;                                    // lagr_dyn.py:174-204
        for (int i = 0; i < 3; ++i) {
            T ddt = cv * v1[i] + cq * q1[i] + ca * a1[i];
            T dLdq = kq * q1[i] + kv * v1[i] - pq * q1[i] - lam1 * q1[i];
            T lhs = ddt - dLdq - mass_flow * v1[i];
            if (i == 2) lhs = lhs + g_grav * mu * nq * 0.5;
            out.eq_row(kRowTrans1 + i, ((lhs - F1[i]) + acc1[i]) * inv_fs1);
        }
        // holonomic constraint of the main tether (holonomics.py:204-312)
        T l_t = SI(kLT), dl_t = SI(kDLT), ldd = SI(kDDLT_U);
        T c0 = 0.5 * (qq - l_t * l_t);
        T c1 = sv - l_t * dl_t;
        T c2 = vv + qa - dl_t * dl_t - l_t * ldd;
        const auto hscale =
            kap * kap * (cst[ADL_C_SCALING_LENGTH_T] * ((s[kQ10] + s[kQ10 + 1] + s[kQ10 + 2]) / 3.0));
        out.eq_row(kRowHol1, (c2 + 2.0 * kap * c1 + kap * kap * c0) / hscale);
    }
}

}  // namespace awe
