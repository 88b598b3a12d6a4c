"""Known answers for Box-v0's one-dof links (urgym_amd/csrc/ug_joint.h, shared by the restatement and the kernels),
recomputed here independently from the URDF's numbers (skew-box-button.urdf :120-252) with numpy: the merged door's
mass, centre of mass and AABB-box inertia (URDF_MERGE_FIXED_LINKS; btCompoundShape::calculateLocalInertia), the
door's effective inertia about its hinge (parallel-axis theorem; constant in q for a rotation about its own axis),
the gravity torque of the COM, btMultiBody's quadratic damping projected on the joint, the button's prismatic
dynamics, and the link frames.  Tolerance 1e-15 relative (independent arithmetic, same formulas)."""
import ctypes

import numpy as np
import pytest

K = 0.04  # btMultiBody DAMPING_K1 = DAMPING_K2 [ext]
G = -10.0  # env_box_v0.py:60


@pytest.fixture(scope="module")
def L(built):
    from oracle import pyoracle
    return pyoracle.lib()


def joint(L, o, q, qd):
    out = np.zeros(16)
    L.ugo_box_joint(o, q, qd, out.ctypes.data_as(ctypes.c_void_p))
    return out


def door_model():
    # door (0.1 kg at its origin) + h1, h2 (0.05 kg at (-0.13, +-0.05, 0.025)) + h3 (0.1 kg at h2 + (0, 0.05, 0.025))
    m = np.array([0.1, 0.05, 0.05, 0.1])
    c = np.array([[0, 0, 0], [-0.13, 0.05, 0.025], [-0.13, -0.05, 0.025], [-0.13, 0.0, 0.05]])
    M, com = m.sum(), (m[:, None] * c).sum(0) / m.sum()
    # collision AABBs in the door frame: box 0.16 x 0.2 x 0.01 at (-0.076, 0, 0); cylinders along z (h1, h2) and y (h3)
    lo = np.array([[-0.156, -0.1, -0.005], [-0.135, 0.045, 0.0], [-0.135, -0.055, 0.0], [-0.14, -0.05, 0.04]])
    hi = np.array([[0.004, 0.1, 0.005], [-0.125, 0.055, 0.05], [-0.125, -0.045, 0.05], [-0.12, 0.05, 0.06]])
    ext = hi.max(0) - lo.min(0)
    I = M / 12 * np.array([ext[1] ** 2 + ext[2] ** 2, ext[0] ** 2 + ext[2] ** 2, ext[0] ** 2 + ext[1] ** 2])
    return M, com, I


def test_door_mass_properties(L):
    M, com, I = door_model()
    out = joint(L, 0, 0.0, 0.0)
    assert out[9] == pytest.approx(M, rel=1e-15)
    assert np.allclose(out[10:13], com, rtol=1e-14, atol=1e-17)
    assert np.allclose(out[13:16], I, rtol=1e-13)


@pytest.mark.parametrize("q", [0.0, 0.3, 1.0, 1.9, 2.0, -0.05])
def test_door_dynamics(L, q):
    M, com, I = door_model()
    Ry = np.array([[np.cos(q), 0, np.sin(q)], [0, 1, 0], [-np.sin(q), 0, np.cos(q)]])
    r = Ry @ com                               # COM offset from the hinge, world
    rp2 = r[0] ** 2 + r[2] ** 2                # distance to the y axis, squared
    Ieff = I[1] + M * rp2                      # parallel-axis theorem about the hinge axis
    tau_g = np.cross(r, [0, 0, M * G])[1]      # gravity torque about +y
    for qd in [0.0, 0.7, -2.5]:
        out = joint(L, 0, q, qd)
        quat, pos = out[:4], out[4:7]
        assert np.allclose(quat, [0, np.sin(q / 2), 0, np.cos(q / 2)], rtol=0, atol=2e-16)
        assert np.allclose(pos, [0.075, -0.5, 0.1], rtol=0, atol=0)  # the hinge, robot frame (box base at y -0.5)
        assert out[7] == pytest.approx(Ieff, rel=1e-14)
        damp = qd * I[1] * (K + K * abs(qd)) + M * qd * rp2 * (K + K * abs(qd) * np.sqrt(rp2))
        assert out[8] == pytest.approx(-tau_g + damp, rel=1e-12, abs=1e-16)
    # the door falls closed (q decreasing) under gravity: its COM lies on the -x side of the hinge
    assert joint(L, 0, 0.3, 0.0)[8] > 0


@pytest.mark.parametrize("q", [0.0, -0.02, -0.05])
def test_button_dynamics(L, q):
    for qd in [0.0, 0.1, -0.3]:
        out = joint(L, 1, q, qd)
        assert np.array_equal(out[:4], [0, 0, 0, 1])
        assert np.allclose(out[4:7], [0.0, -0.5, 0.07 + q], rtol=0, atol=1e-17)
        assert out[7] == 0.01
        assert out[8] == pytest.approx(-0.01 * G + 0.01 * qd * (K + K * abs(qd)), rel=1e-14)
