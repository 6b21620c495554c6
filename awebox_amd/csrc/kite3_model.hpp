// The 3-DOF (roll-controlled) AP2 kite node model of the tracking MPC, hand-written for CDNA4 and
// instantiated on double / Dual / Dep (scalar.hpp).
//
// One call evaluates, at ONE node, the model equalities (12 rows: translation 3, holonomic 1,
// trivial kinematics 8, lagr_dyn.py:68-169) and, on request, the path inequalities (tether stress,
// acceleration; dynamics.py:627-652, 706-790).  Row order = the reference's append order; the
// trivial rows come out in the sorted order of the xdot names (dcoeff10, dddl_t, ddl_t, dl_t, dq10).
//
// The translational / holonomic part is the closed form of the reference's Lagrangian derivation
// (lagr_dyn.py:39-204, energy.py:43-144) -- the same expressions as the AP2 model, without the
// rotational terms; here the main tether's reel-in acceleration ddl_t is a state (tether control
// 'dddl_t'), so the holonomic second derivative takes it from x (tools.py:13-73 picks the first
// non-xdot container holding 'ddl_t').  The aerodynamic force is three_dof_kite.py:98-199: a
// planar frame from the tether and the apparent wind, rolled by psi = coeff[1] about the apparent
// wind; lift CL = coeff[0] along the rolled third axis, drag CD = |CX0| + CL^2/(pi AR) along the
// apparent wind.  The CPU oracle (oracle/kite3_oracle.py) derives the same residuals by automatic
// differentiation of L, so the two are independent.
#pragma once

#include "scalar.hpp"
#include "../../include/awempc.h"

namespace awe {

namespace k3 {
// node-variable indices (K3 layout)
constexpr int Q = 0, DQ = 3, COEFF = 6, LT = 8, DLT = 9, DDLT = 10;
constexpr int XD_DQ = 11, XD_DDQ = 14, XD_DCOEFF = 17, XD_DLT = 19, XD_DDLT = 20, XD_DDDLT = 21;
constexpr int U_FFICT = 22, U_DCOEFF = 25, U_DDDLT = 27, Z_LAMBDA = 28, TH_DIAM = 29, TH_TF = 30;
constexpr double kPi = 3.14159265358979323846;
}  // namespace k3

// the roll angle enters through sin / cos: their hyper-dual forms (the first- and second-order
// kernels instantiate the model on Dual and HDual, scalar.hpp)
AWE_HD HDual sin(HDual x) {
    const double s = ::sin(x.v), c = ::cos(x.v);
    return hd_apply(x, s, c, -s);
}
AWE_HD HDual cos(HDual x) {
    const double s = ::sin(x.v), c = ::cos(x.v);
    return hd_apply(x, c, -s, -c);
}

template <class T>
struct Kite3Result {
    T eq[K3_N_EQ];
    T ineq[K3_N_INEQ];
    AWE_HD void eq_row(int r, const T& v) { eq[r] = v; }
    AWE_HD void ineq_row(int r, const T& v) { ineq[r] = v; }
};

template <class T>
AWE_HD T k3_dot(const T* a, const T* b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }

// ISA density (atmosphere.py:60-78)
template <class T, class CT>
AWE_HD T k3_density(const T& zz, const CT* c) {
    const CT expo = c[K3_C_G] / c[K3_C_GAMMA_AIR] / c[K3_C_R_AIR] - 1.0;
    T ratio = 1.0 - zz * (c[K3_C_GAMMA_AIR] / c[K3_C_T_REF]);
    return c[K3_C_RHO_REF] * exp(expo * log(ratio));
}

// log wind u_ref log10(smooth_abs(zz, 1) / z0) / log10(z_ref / z0) (wind.py:184-208), written as
// u_ref (0.5 log(zz^2 + 1) - log z0) / log(z_ref / z0)
template <class T, class UT, class CT>
AWE_HD T k3_wind(const T& zz, const UT& u_ref, const CT* c) {
    const CT lz0 = log(c[K3_C_Z0_AIR]);
    const auto scale = u_ref / (log(c[K3_C_Z_REF]) - lz0);
    return scale * (0.5 * log(zz * zz + 1.0) - lz0);
}

// 'multi' tether drag, element e of n_el on the main tether, lumped onto the kite node with the
// reference's shape factor (element.py:60-104, segment.py:38-65); ground end at rest
template <class T, class UT, class CT>
AWE_HD void k3_tether_element(int e, int n_el, const T* q, const T* v, const T& diam, const UT& u_ref,
                              const CT* c, T out[3]) {
    const double ds = 1.0 / n_el;
    const double s0 = 0.5 * ds, step = ((1.0 - 0.5 * ds) - s0) / (n_el - 1);
    const double lo = (double)e / (double)n_el, up = (double)(e + 1) / (double)n_el;
    T zz = (q[2] * up + q[2] * lo) / 2.0;
    T uw = k3_wind(zz, u_ref, c);
    T rho = k3_density(zz, c);
    T ue[3];
    ue[0] = uw - (v[0] * up + v[0] * lo) / 2.0;
    ue[1] = -((v[1] * up + v[1] * lo) / 2.0);
    ue[2] = -((v[2] * up + v[2] * lo) / 2.0);
    T un = sqrt(k3_dot(ue, ue) + 1e-12);
    T tv[3];
    for (int i = 0; i < 3; ++i) tv[i] = q[i] * up - q[i] * lo;
    T lpar = k3_dot(tv, ue) / un;
    T lperp = sqrt(k3_dot(tv, tv) - lpar * lpar + 1e-12);
    T fac = c[K3_C_CD_TETHER] * 0.5 * rho * un * diam * lperp;
    const double sg = (e == n_el - 1) ? (1.0 - 0.5 * ds) : (s0 + e * step);
    for (int i = 0; i < 3; ++i) out[i] = sg * (fac * ue[i]);
}

// the main tether's drag summed over its elements, evaluated inside the node model (host
// structure, CPU paths); the GPU kernel substitutes values + partials preaccumulated per node
struct K3InlineDrag {
    template <class T, class UT, class CT>
    AWE_HD void operator()(const T* q, const T* v, const T& diam, const UT& u_ref, const CT* c, T D[3]) const {
        const int n_el = structural(c[K3_C_N_ELEMENTS]);
        for (int i = 0; i < 3; ++i) D[i] = T(0.0);
        for (int e = 0; e < n_el; ++e) {
            T ce[3];
            k3_tether_element(e, n_el, q, v, diam, u_ref, c, ce);
            for (int i = 0; i < 3; ++i) D[i] = D[i] + ce[i];
        }
    }
};

// u_ref and the constants c are doubles on the device and Sym leaves in the code generator
// (gen/kite3_jacgen.cpp), which loads them at run time
template <class T, class In, class Sink, class Drag = K3InlineDrag, class UT = double, class CT = double>
AWE_HD void kite3_node(const In& in, const T& gamma, const UT& u_ref, const CT* c, Sink& out, bool want_ineq,
                       const Drag& drag = Drag()) {
    using namespace k3;
    const CT* s = c + K3_C_SCALING;
    auto SI = [&](int i) -> T { return in(i) * s[i]; };

    // ---- trivial kinematics (lagr_dyn.py:141-169), sorted xdot names -------------------------
    for (int i = 0; i < 2; ++i)
        out.eq_row(4 + i, (SI(XD_DCOEFF + i) - SI(U_DCOEFF + i)) / sqrt(s[U_DCOEFF + i] * s[XD_DCOEFF + i]));
    out.eq_row(6, (SI(XD_DDDLT) - SI(U_DDDLT)) / sqrt(s[U_DDDLT] * s[XD_DDDLT]));
    out.eq_row(7, (SI(XD_DDLT) - SI(DDLT)) / sqrt(s[DDLT] * s[XD_DDLT]));
    out.eq_row(8, (SI(XD_DLT) - SI(DLT)) / sqrt(s[DLT] * s[XD_DLT]));
    for (int i = 0; i < 3; ++i)
        out.eq_row(9 + i, (SI(XD_DQ + i) - SI(DQ + i)) / sqrt(s[DQ + i] * s[XD_DQ + i]));

    T q[3], v[3];
    for (int i = 0; i < 3; ++i) q[i] = SI(Q + i);
    for (int i = 0; i < 3; ++i) v[i] = SI(DQ + i);

    // ---- 3-DOF aerodynamic force in the earth frame (three_dof_kite.py:98-199) ---------------
    T F_aero[3];
    {
        T rho = k3_density(q[2], c);
        T ua[3];
        ua[0] = k3_wind(q[2], u_ref, c) - v[0];
        ua[1] = -v[1];
        ua[2] = -v[2];
        // planar dcm: v = t x u, w = u x v with t = q (get_planar_dcm, :139-153)
        T pv[3], pw[3];
        pv[0] = q[1] * ua[2] - q[2] * ua[1];
        pv[1] = -(q[0] * ua[2] - q[2] * ua[0]);
        pv[2] = q[0] * ua[1] - q[1] * ua[0];
        pw[0] = ua[1] * pv[2] - ua[2] * pv[1];
        pw[1] = -(ua[0] * pv[2] - ua[2] * pv[0]);
        pw[2] = ua[0] * pv[1] - ua[1] * pv[0];
        T iv = 1.0 / sqrt(k3_dot(pv, pv) + 1e-16);              // smooth_normalize (eps 1e-8)
        T iw = 1.0 / sqrt(k3_dot(pw, pw) + 1e-16);
        T psi = SI(COEFF + 1);
        T cp = cos(psi), sp = sin(psi);
        T CL = SI(COEFF);
        T uu = k3_dot(ua, ua);
        T un = sqrt(uu);                                          // vect_op.norm
        T CD = c[K3_C_CD0] + CL * CL / (k3::kPi * c[K3_C_AR]);
        T half_rho_s = (0.5 * c[K3_C_S_REF]) * rho;
        T lift = CL * half_rho_s * uu;                            // along ehat3 = cos psi w - sin psi v
        T drag = CD * half_rho_s * un;                            // along u
        T lw = lift * cp * iw, lv = lift * sp * iv;
        for (int i = 0; i < 3; ++i) F_aero[i] = lw * pw[i] - lv * pv[i] + drag * ua[i];
    }

    // ---- path inequalities (dynamics.py:706-790 tether stress, :627-652 acceleration) --------
    if (want_ineq) {
        T nq = sqrt(k3_dot(q, q));
        T diam = SI(TH_DIAM);
        T area = (k3::kPi * 0.25) * diam * diam;
        const CT ls = c[K3_C_LAMBDA_SCALING] * c[K3_C_SCALING_LENGTH];
        const CT char_tension = sqrt(ls * ls + 1e-16);          // smooth_abs
        out.ineq_row(0, (SI(Z_LAMBDA) * nq - area * c[K3_C_STRESS_MAX]) / char_tension);
        T a[3];
        for (int i = 0; i < 3; ++i) a[i] = SI(XD_DDQ + i);
        const CT amax = c[K3_C_ACC_MAX];
        out.ineq_row(1, k3_dot(a, a) / (amax * amax) - 1.0);
    }

    // ---- translational Lagrangian dynamics (lagr_dyn.py:68-109, 174-204) ---------------------
    const CT g_grav = c[K3_C_G], m_k = c[K3_C_M_K], rho_t = c[K3_C_RHO_TETHER];
    T diam = SI(TH_DIAM);
    T D_tether[3];
    drag(q, v, diam, u_ref, c, D_tether);
    T qq = k3_dot(q, q);
    T nq = sqrt(qq);
    T mu = ((k3::kPi * 0.25) * diam * diam) * rho_t;              // m_t = mu |q|
    T lam = SI(Z_LAMBDA);
    T a[3];
    for (int i = 0; i < 3; ++i) a[i] = SI(XD_DDQ + i);
    T sv = k3_dot(q, v), vv = k3_dot(v, v), qa = k3_dot(q, a);
    T inv_n = 1.0 / nq;
    T inv_n3 = inv_n * inv_n * inv_n;
    T mu6 = mu / 6.0;
    // KE_t = (mu/6)(|q||v|^2 + 2 (q.v)^2/|q|) (energy.py:59-97); d/dt dL/dqdot and dL/dq
    T cv = mu * sv * inv_n;
    T cq = mu6 * (4.0 * (vv + qa) * inv_n - 4.0 * sv * sv * inv_n3);
    T ca = mu6 * (2.0 * nq) + m_k;
    T kq = mu6 * (vv * inv_n - 2.0 * sv * sv * inv_n3);
    T kv = mu6 * (4.0 * sv * inv_n);
    T pq = g_grav * mu * (q[2] * inv_n) * 0.5;
    T pz = g_grav * mu * nq * 0.5 + g_grav * m_k;
    T mass_flow = mu * sv * inv_n;                                // d(m_t)/dt
    const CT sd = c[K3_C_SCALING_DIAM];
    const CT scaling_mass = (k3::kPi * 0.25) * sd * sd * rho_t * c[K3_C_SCALING_LENGTH];
    const CT inv_force_scaling = 1.0 / ((scaling_mass / 2.0 + m_k) * c[K3_C_G_SCALING] * 10.0);
    for (int i = 0; i < 3; ++i) {
        T ddt = cv * v[i] + cq * q[i] + ca * a[i];
        T dLdq = kq * q[i] + kv * v[i] - pq * q[i] - lam * q[i];
        if (i == 2) dLdq = dLdq - pz;
        T F = D_tether[i] + (gamma * SI(U_FFICT + i) + F_aero[i]);   // forces.py:47-80, 148-171
        out.eq_row(i, ((ddt - dLdq) - (F + mass_flow * v[i])) * inv_force_scaling);
    }
    // ---- holonomic constraint + Baumgarte (holonomics.py:17-123, 267-312) -------------------
    {
        T l_t = SI(LT), dl_t = SI(DLT), ddl_t = SI(DDLT);
        T c0 = 0.5 * (qq - l_t * l_t);
        T c1 = sv - l_t * dl_t;
        T c2 = vv + qa - dl_t * dl_t - l_t * ddl_t;
        const CT kap = c[K3_C_KAPPA];
        const CT hscale = kap * kap * (c[K3_C_SCALING_LENGTH] * c[K3_C_Q_SCALING_MEAN]);
        out.eq_row(3, (c2 + 2.0 * kap * c1 + kap * kap * c0) / hscale);
    }
}

}  // namespace awe
