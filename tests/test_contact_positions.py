"""getContactPoints positions as Bullet reports them (env_cubes_grasp_v0.py:209-226 reads the tuples).

Bullet stores each manifold point's world positions (m_positionWorldOnA / B) when the narrowphase refreshes the manifold
(refreshContactPoints, at collision time, before the substep integrates), and p.getContactPoints returns those.  The
restatement keeps the poses that narrowphase saw (the state's UG_F_PREV record) and reports the points' local anchors
under them.  Crafted moving contact: a CubesPush cube sliding at 0.5 m/s over the table.  After one substep the reported
position on the cube is its anchor under the cube's pose before the substep -- not under the integrated pose, which
is about v dt = 2 mm further along.  The GPU reports the same tuples bit for bit (tests/test_gpu_features.py).
"""
import numpy as np

from urgym_amd import layout as LY


def qmat(q):
    x, y, z, w = q
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                     [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                     [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])


def test_reported_point_is_the_narrowphase_point():
    from oracle.pyoracle import OracleEnv
    r = OracleEnv(1, 20250601)
    r.reset()
    for _ in range(3):  # settle the cubes on the table with a few substeps
        r.substep()
    s = r.get_state()
    o = LY.obj(0)
    s[o + 7:o + 10] = [0.5, 0.0, 0.0]  # cube 0 slides along +x
    r.set_state(s)
    pre = r.get_state()
    r.substep()
    post = r.get_state()
    pts = r.contact_points(1, 10)  # cube 0 against the table
    assert len(pts) >= 1
    # the prev-pose record holds the pose the narrowphase saw: the one before this substep
    pp = LY.F_PREV + 12
    assert np.array_equal(post[pp:pp + 7], pre[o:o + 7])
    assert not np.array_equal(post[o:o + 3], pre[o:o + 3])
    R_pre, p_pre = qmat(pre[o + 3:o + 7]), pre[o:o + 3]
    R_post, p_post = qmat(post[o + 3:o + 7]), post[o:o + 3]
    # the manifold of pair (cube 0, table): match each reported point to its anchor
    nm = int(post[LY.F_NMAN])
    anchors = []
    for m in range(nm):
        base = LY.F_MAN + m * LY.MAN_DOUBLES
        for j in range(int(post[base + 1])):
            q = post[base + 2 + j * LY.PT_DOUBLES:base + 2 + (j + 1) * LY.PT_DOUBLES]
            anchors.append(q[:3])
    moved = 0.0
    for t in pts:
        pa = t[5:8]
        d_pre = min(np.linalg.norm(R_pre @ a + p_pre - pa) for a in anchors)
        d_post = min(np.linalg.norm(R_post @ a + p_post - pa) for a in anchors)
        assert d_pre <= 1e-15, d_pre
        moved = max(moved, d_post)
    assert moved > 0.0015  # the integrated pose is a substep's slide away (~2 mm: 0.5 m/s over 1/240 s, less friction)
