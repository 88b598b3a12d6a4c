"""Dynamics invariants of the restatement ("ABA vs RNEA round-trip (M(q) qdd + C = tau)", energy):

* the oracle's robot dynamics (CRBA mass matrix + RNEA bias, oracle/ug_oracle.c robot_dynamics, which the HIP
  kernels reproduce bit for bit) against an independent Featherstone articulated-body algorithm written here in
  numpy from the model tables: qdd = M^-1 (tau - C) must equal ABA(q, qd, tau) -- gravity, Coriolis /
  gyroscopic terms and btMultiBody's quadratic link damping (an external force on both sides) included;
* M is symmetric positive definite and C(q, 0) is the gradient of the potential energy (finite differences);
* the damped, contact-free, motor-free arm does not gain energy.
Bullet itself uses ABA (btMultiBody [ext]); this pins the equations of motion, not Bullet's rounding."""
import re

import numpy as np
import pytest

K = 0.04  # btMultiBody default linear / angular damping [ext]


@pytest.fixture(scope="module")
def model(built):
    import os
    txt = open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "urgym_amd", "csrc",
                            "model_data.h")).read()
    A = {m.group(2): np.array([float(x) for x in m.group(4).split(",")])
         for m in re.finditer(r"UG_CONST (int|double) (UG_\w+)\[(\d+)\] = \{([^}]*)\};", txt)}
    A["UG_BODY_PARENT"] = np.array([int(x) for x in re.search(r"#define UG_BODY_PARENT_INIT \{([^}]*)\}", txt)
                                    .group(1).split(",")])
    return A


def skew(c):
    return np.array([[0, -c[2], c[1]], [c[2], 0, -c[0]], [-c[1], c[0], 0]])


def rot(a, q):
    a = np.asarray(a, float)
    return np.cos(q) * np.eye(3) + np.sin(q) * skew(a) + (1 - np.cos(q)) * np.outer(a, a)


def sym6(v):
    return np.array([[v[0], v[3], v[4]], [v[3], v[1], v[5]], [v[4], v[5], v[2]]])


def aba(A, q, qd, tau, g=-9.8):
    """articulated-body algorithm in world-frame Plucker coordinates (all quantities at the world origin)"""
    nb = 12
    par = A["UG_BODY_PARENT"]
    R, p, S = [None] * nb, [None] * nb, [None] * nb
    I6, pb, v, c = [None] * nb, [None] * nb, [None] * nb, [None] * nb

    def mcross(x, y):  # motion x motion
        return np.r_[np.cross(x[:3], y[:3]), np.cross(x[:3], y[3:]) + np.cross(x[3:], y[:3])]

    def fcross(x, f):  # motion x* force
        return np.r_[np.cross(x[:3], f[:3]) + np.cross(x[3:], f[3:]), np.cross(x[:3], f[3:])]

    for b in range(nb):
        Rpb = A["UG_BODY_R"][9 * b:9 * b + 9].reshape(3, 3)
        Ppb = A["UG_BODY_P"][3 * b:3 * b + 3]
        ax = A["UG_BODY_AXIS"][3 * b:3 * b + 3]
        Rp, pp = (np.eye(3), np.zeros(3)) if par[b] < 0 else (R[par[b]], p[par[b]])
        R[b] = Rp @ Rpb @ rot(ax, q[b])
        p[b] = pp + Rp @ Ppb
        a = Rp @ Rpb @ ax
        S[b] = np.r_[a, np.cross(p[b], a)]
        m = A["UG_BODY_MASS"][b]
        cw = p[b] + R[b] @ A["UG_BODY_COM"][3 * b:3 * b + 3]
        Ic = R[b] @ sym6(A["UG_BODY_I"][6 * b:6 * b + 6]) @ R[b].T
        X = skew(cw)
        I6[b] = np.block([[Ic + m * X @ X.T, m * X], [m * X.T, m * np.eye(3)]])
        vp = np.zeros(6) if par[b] < 0 else v[par[b]]
        vj = S[b] * qd[b]
        v[b] = vp + vj
        c[b] = mcross(v[b], vj)
        pb[b] = fcross(v[b], I6[b] @ v[b])
        # damping as a resistive external force (the same terms the restatement adds to its bias)
        w = v[b][:3]
        D = R[b] @ sym6(A["UG_BODY_DAMPI"][6 * b:6 * b + 6]) @ R[b].T
        pb[b][:3] += D @ w * (K + K * np.linalg.norm(w))
    for l in range(1, 19):
        b = int(A["UG_LINK_BODY"][l])
        if b < 0:
            continue
        cl = p[b] + R[b] @ A["UG_LINK_COMP"][3 * l:3 * l + 3]
        vl = v[b][3:] + np.cross(v[b][:3], cl)
        fd = vl * A["UG_LINK_MASS"][l] * (K + K * np.linalg.norm(vl))
        pb[b] += np.r_[np.cross(cl, fd), fd]
    IA = [x.copy() for x in I6]
    pA = [x.copy() for x in pb]
    U, Dd, u = [None] * nb, np.zeros(nb), np.zeros(nb)
    for b in range(nb - 1, -1, -1):
        U[b] = IA[b] @ S[b]
        Dd[b] = S[b] @ U[b]
        u[b] = tau[b] - S[b] @ pA[b]
        if par[b] >= 0:
            Ia = IA[b] - np.outer(U[b], U[b]) / Dd[b]
            IA[par[b]] += Ia
            pA[par[b]] += pA[b] + Ia @ c[b] + U[b] * u[b] / Dd[b]
    acc = [None] * nb
    qdd = np.zeros(nb)
    for b in range(nb):
        ap = np.r_[0, 0, 0, 0, 0, -g] if par[b] < 0 else acc[par[b]]
        a = ap + c[b]
        qdd[b] = (u[b] - U[b] @ a) / Dd[b]
        acc[b] = a + S[b] * qdd[b]
    return qdd


def test_crba_rnea_matches_articulated_body_algorithm(model):
    from oracle.pyoracle import dynamics
    rng = np.random.default_rng(0)
    for k in range(20):
        q = rng.uniform(-np.pi, np.pi, 12)
        qd = rng.normal(size=12) * (0.0 if k < 5 else 2.0)
        tau = rng.normal(size=12) * 5.0
        M, C, _ = dynamics(q, qd)
        assert np.allclose(M, M.T, rtol=0, atol=1e-14)
        assert np.all(np.linalg.eigvalsh(M) > 0)
        want = aba(model, q, qd, tau)
        got = np.linalg.solve(M, tau - C)
        assert np.allclose(got, want, rtol=1e-11, atol=1e-11 * np.abs(want).max()), (k, np.abs(got - want).max())


def test_static_bias_is_gravity_gradient(model):
    """C(q, 0) = dV/dq with V = sum_b m_b 9.8 z_b (finite differences of the restatement's own FK)"""
    from oracle.pyoracle import dynamics
    rng = np.random.default_rng(1)
    m = model["UG_BODY_MASS"]
    for _ in range(5):
        q = rng.uniform(-np.pi, np.pi, 12)
        _, C, _ = dynamics(q, np.zeros(12))
        grad = np.zeros(12)
        h = 1e-6
        for j in range(12):
            dq = np.zeros(12)
            dq[j] = h
            Vp = np.sum(m * 9.8 * dynamics(q + dq, np.zeros(12))[2][:, 2])
            Vm = np.sum(m * 9.8 * dynamics(q - dq, np.zeros(12))[2][:, 2])
            grad[j] = (Vp - Vm) / (2 * h)
        assert np.allclose(C, grad, rtol=1e-6, atol=1e-7)


def test_damped_free_arm_does_not_gain_energy(model):
    """BallBalance scene with no objects and all motors off: the arm swings under gravity with joint limits, gear
    rows and link damping; total energy (1/2 qd^T M qd + potential) never rises by more than the semi-implicit
    integrator's O(dt) oscillation and ends below its start."""
    from oracle.pyoracle import OracleEnv, dynamics
    from urgym_amd import layout as LY
    e = OracleEnv(0, 0)
    s = e.get_state()
    s[:] = 0.0
    s[LY.F_Q:LY.F_Q + 6] = [0.3, -1.2, 0.9, -0.4, 0.6, 0.2]   # arm well above the table, gripper joints at 0
    s[LY.F_NMAN] = 0
    s[LY.F_MAN:LY.F_TASK:LY.MAN_DOUBLES] = -1
    e.set_state(s)
    m = model["UG_BODY_MASS"]

    def energy():
        st = e.get_state()
        q, qd = st[LY.F_Q:LY.F_Q + 12], st[LY.F_QD:LY.F_QD + 12]
        M, _, com = dynamics(q, qd)
        return 0.5 * qd @ M @ qd + np.sum(m * 9.8 * com[:, 2])
    E = [energy()]
    for _ in range(240):
        e.substep()
        E.append(energy())
    E = np.array(E)
    assert np.all(np.isfinite(E))
    assert E[-1] < E[0]
    assert np.max(np.diff(E)) < 0.05 * (E[0] - E.min() + 1e-3)
