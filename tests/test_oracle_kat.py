"""Known-answer tests and physics invariants of the CPU restatement (no PyBullet exists here,
so these pin conventions and mechanics independently -- SURVEY.md 4)."""
import numpy as np

from urgym_amd import layout as LY
import pytest
from scipy.spatial.transform import Rotation

SEED = 20241220


@pytest.fixture(scope="module")
def ora(built):
    from oracle import pyoracle
    return pyoracle


def test_euler_quat_conventions_vs_scipy(ora):
    # pybullet: q = Rz(yaw) Ry(pitch) Rx(roll) == scipy extrinsic 'xyz'
    rng = np.random.default_rng(0)
    for _ in range(200):
        rpy = rng.uniform([-3, -1.4, -3], [3, 1.4, 3])
        q = ora.quat_from_euler(rpy)
        want = Rotation.from_euler("xyz", rpy).as_quat()
        assert np.allclose(q, want, atol=1e-14) or np.allclose(q, -want, atol=1e-14)
        assert np.allclose(ora.euler_from_quat(q), rpy, atol=1e-12)


def test_state_roundtrip_and_determinism(ora):
    a = ora.OracleEnv(0, SEED)
    b = ora.OracleEnv(0, SEED)
    oa, na = a.reset()
    ob, nb = b.reset()
    assert np.array_equal(oa, ob) and na == nb
    c = ora.OracleEnv(0, 1)
    c.set_state(a.get_state())
    act = np.array([0.05, -0.03, 0.02], np.float32)
    ra, rc = a.step(act), c.step(act)
    assert np.array_equal(ra[0], rc[0]) and ra[4] == rc[4]
    assert np.array_equal(a.get_state(), c.get_state())


def _blank_with_ball(ora, pos, vel=(0, 0, 0)):
    e = ora.OracleEnv(0, 0)
    s = e.get_state()
    s[:] = 0
    s[0:6] = [0, -1.57, 0, 0, 0, 0]
    s[LY.F_OACTIVE:LY.F_OACTIVE + 2] = [0, 1]   # paddle inactive, ball active
    b = LY.obj(1)
    s[b:b + 3] = pos
    s[b + 3:b + 7] = [0, 0, 0, 1]
    s[b + 7:b + 10] = vel
    e.set_state(s)
    return e


def test_free_fall_matches_semi_implicit_euler_with_bullet_damping(ora):
    # a ball far from everything: v += dt*(g - v*(k1 + k2|v|)), x += dt*v  (btMultiBody base, damping 0.04)
    e = _blank_with_ball(ora, (2.0, 2.0, 5.0), vel=(0.3, 0.0, 0.0))
    dt, k = 1.0 / 240.0, 0.04
    x = np.array([2.0, 2.0, 5.0]); v = np.array([0.3, 0.0, 0.0]); g = np.array([0, 0, -9.8])
    for _ in range(100):
        e.substep()
        v = v + (g - v * (k + k * np.linalg.norm(v))) * dt
        x = x + v * dt
    s = e.get_state()
    b = LY.obj(1)
    assert np.allclose(s[b:b + 3], x, rtol=0, atol=1e-12)
    assert np.allclose(s[b + 7:b + 10], v, rtol=0, atol=1e-12)


def test_ball_comes_to_rest_on_table(ora):
    e = _blank_with_ball(ora, (0.3, -0.9, 0.05))
    for _ in range(480):
        e.substep()
    s = e.get_state()
    b = LY.obj(1)
    assert abs(s[b + 2] - 0.02) < 2e-3               # centre one radius above the table top (z = 0)
    assert np.linalg.norm(s[b + 7:b + 10]) < 1e-3    # at rest


def test_ik_converges_to_reachable_target(ora):
    """Damped least squares with PyBullet's per-joint damping 0.5 converges slowly (20 iterations
    leave a residual); repeated solves from the new joints must converge -> the Jacobian is right."""
    e = ora.OracleEnv(0, SEED)
    e.reset()
    ee = e.link_state(7)
    tgt = ee[:3] + np.array([0.03, -0.02, 0.04])
    errs = []
    for _ in range(6):
        q = e.ik(tgt, ee[3:])
        s = e.get_state()
        s[:12] = q
        e.set_state(s)
        errs.append(np.linalg.norm(e.link_state(7)[:3] - tgt))
    assert errs[0] < 0.5 * np.linalg.norm(ee[:3] - tgt)
    assert all(b <= a + 1e-12 for a, b in zip(errs, errs[1:]))
    assert errs[-1] < 1e-4
    got = e.link_state(7)
    assert abs(abs(np.dot(got[3:], ee[3:])) - 1) < 1e-6


def test_mimic_gears_hold_after_reset(ora):
    # robot.py:194-211: q11 = -q9, q13 = q9, q14 = q9, q16 = -q9, q18 = q9 (dofs 7..11 vs dof 6)
    e = ora.OracleEnv(0, SEED)
    e.reset()
    q = e.get_state()[:12]
    mult = np.array([-1, 1, 1, -1, 1])
    # under grasp load the gear rows (max force 100, erp folded into ERP 0.2) leave a few-% strain
    assert np.allclose(q[7:12], mult * q[6], atol=5e-2)


def test_paddle_stays_grasped_and_ball_dynamics_finite(ora):
    e = ora.OracleEnv(0, SEED)
    e.reset()
    rng = np.random.default_rng(3)
    p0 = e.get_state()[LY.obj(0):LY.obj(0) + 3].copy()
    for _ in range(15):
        obs, r, term, succ, n = e.step(rng.uniform(-0.1, 0.1, 3).astype(np.float32))
        assert np.all(np.isfinite(obs)) and 1 <= n <= 480
        if term:
            break
    p1 = e.get_state()[LY.obj(0):LY.obj(0) + 3]
    # the paddle is carried by the gripper: it moved with the end effector, it did not fall to the table
    assert p1[2] > 0.3 and np.linalg.norm(p1 - p0) < 0.3


def test_variants_share_their_base_physics(ora):
    """CubesPushDiff / GolfJoints differ from CubesPush / Golf only in step and obs
    glue: the same seed resets to the same state, and the obs is the reference's function of it
    (env_cubes_push_diff_v0.py:202-212: cube - ee; env_golf_joints_v0.py:228-235: joints[0:6] + Golf obs)."""
    for base, var in ((1, 4), (3, 5)):
        b, v = ora.OracleEnv(base, SEED), ora.OracleEnv(var, SEED)
        ob, nb = b.reset()
        ov, nv = v.reset()
        assert nb == nv and np.array_equal(b.get_state(), v.get_state())
        if var == 4:
            assert ov.shape == (9,) and np.array_equal(ov[:3], ob[:3])
            assert np.array_equal(ov[3:6], ob[3:6] - ob[:3]) and np.array_equal(ov[6:9], ob[6:9] - ob[:3])
        else:
            assert ov.shape == (15,) and np.array_equal(ov[6:], ob)
            assert np.array_equal(ov[:6], v.get_state()[:6])


def test_golf_joints_step_is_joint_control(ora):
    """GolfJoints.step: targets = get_joint_states() + action (float64 + float32), 'joint' control
    (env_golf_joints_v0.py:122-124, robot.py:122-128): the arm motors hold q + a after the step."""
    v = ora.OracleEnv(5, SEED)
    v.reset()
    q0 = v.get_state()[:6].copy()
    a = np.array([0.05, -0.05, 0.02, 0.0, 0.01, -0.02], np.float32)
    v.step(a)
    st = v.get_state()
    mtarget = st[24:30]  # state layout: q[12], qd[12], mtarget[7] ...
    assert np.array_equal(mtarget, q0 + a.astype(np.float64))
