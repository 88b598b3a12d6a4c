"""Camera (utilities.py:62-107) on the CPU: the restated pybullet matrices, the back projection
against the reference's own Camera class (tests/golden/camera.json, tools/gen_golden.py camera), and the restated
renderer (oracle ugo_camera, the checker of the GPU kernel): what it draws lies on the surfaces it names."""
import json
import os

import numpy as np
import pytest

from oracle.pyoracle import OracleEnv
from urgym_amd import layout as LY
from urgym_amd.camera import Camera, compute_projection_matrix_fov, compute_view_matrix

GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "camera.json")))


def test_view_matrix_is_a_look_at():
    eye, tar, up = np.array([0.6, -0.6, 0.9]), np.array([0.0, -0.6, 0.5]), np.array([0.0, 0.0, 1.0])
    V = np.array(compute_view_matrix(eye, tar, up)).reshape((4, 4), order="F")
    R = V[:3, :3]
    np.testing.assert_allclose(R @ R.T, np.eye(3), atol=1e-6)  # orthonormal (float)
    np.testing.assert_allclose(V @ np.append(eye, 1), [0, 0, 0, 1], atol=1e-6)  # the eye at the origin
    t = V @ np.append(tar, 1)
    np.testing.assert_allclose(t[:2], [0, 0], atol=1e-6)  # the target straight ahead, on -z
    assert t[2] < 0 and abs(t[2] + np.linalg.norm(tar - eye)) < 1e-6
    assert (V @ np.append(eye + up, 1))[1] > 0  # up stays up


@pytest.mark.parametrize("fov,aspect,near,far", [(40, 1.0, 0.1, 5.0), (70, 4 / 3, 0.05, 3.0)])
def test_projection_maps_near_far_to_ndc(fov, aspect, near, far):
    P = np.array(compute_projection_matrix_fov(fov, aspect, near, far)).reshape((4, 4), order="F")
    for z, ndc in [(-near, -1.0), (-far, 1.0)]:
        c = P @ [0, 0, z, 1]
        assert abs(c[2] / c[3] - ndc) < 1e-5
    top = np.tan(np.radians(fov) / 2) * near  # the frustum's top edge at the near plane maps to y = 1
    c = P @ [aspect * top, top, -near, 1]
    np.testing.assert_allclose(c[:2] / c[3], [1, 1], atol=1e-5)


@pytest.mark.parametrize("rec", GOLD, ids=lambda r: "x".join(map(str, r["args"][5])))
def test_back_projection_matches_reference_camera(rec):
    a = rec["args"]
    cam = Camera(tuple(a[0]), tuple(a[1]), tuple(a[2]), a[3], a[4], tuple(a[5]), a[6])
    assert list(cam.view_matrix) == rec["view"] and list(cam.projection_matrix) == rec["proj"]
    np.testing.assert_allclose(cam.tran_pix_world, rec["tran_pix_world"], rtol=1e-13, atol=1e-15)
    for w, h, d, p in rec["points"]:
        np.testing.assert_allclose(cam.rgbd_2_world(w, h, d), p, rtol=1e-12, atol=1e-14)
    if "depth" in rec:
        np.testing.assert_allclose(cam.rgbd_2_world_batch(np.array(rec["depth"])), rec["world"], rtol=1e-12, atol=1e-14)


def _scene_cam(size=(64, 48)):
    return Camera((0.6, -0.6, 0.9), (0.0, -0.6, 0.5), (0, 0, 1), 0.05, 3.0, size, 50)


def test_renderer_hits_lie_on_the_named_surfaces():
    """BallBalance after reset: ball pixels reconstruct onto the ball's sphere, table pixels onto its top face,
    paddle pixels onto its box; background is depth 1 / seg -1; link-index codes name robot links"""
    env = OracleEnv(0, 7)
    env.reset()
    cam = _scene_cam()
    rgb, depth, seg = env.camera(cam.view_matrix, cam.projection_matrix, cam.width, cam.height)
    assert rgb.shape == (48, 64, 4) and depth.dtype == np.float32 and seg.dtype == np.int32
    assert set(np.unique(seg)) >= {-1, 0, 1, 2, 10}
    assert np.all(depth[seg == -1] == 1.0) and np.all(depth[seg != -1] < 1.0) and np.all(rgb[..., 3] == 255)
    P = cam.rgbd_2_world_batch(depth)
    st = env.get_state()
    ball = st[LY.obj(1):LY.obj(1) + 3]
    r = np.linalg.norm(P[seg == 2] - ball, axis=1)
    np.testing.assert_allclose(r, 0.02, atol=2e-6)  # float depth -> a few e-7 m here
    np.testing.assert_allclose(P[seg == 10][:, 2], 0.0, atol=2e-6)  # the table's top at z = 0
    po, pq = st[LY.obj(0):LY.obj(0) + 3], st[LY.obj(0) + 3:LY.obj(0) + 7]
    x, y, z, w = pq
    R = np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                  [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                  [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])
    loc = (P[seg == 1] - po) @ R
    gap = np.max(np.abs(loc) / np.array([0.05, 0.1, 0.005]), axis=1)
    np.testing.assert_allclose(gap, 1.0, atol=5e-3)  # on the paddle box's boundary
    _, _, segl = env.camera(cam.view_matrix, cam.projection_matrix, cam.width, cam.height, link_index=True)
    rob = segl[seg == 0]
    assert np.all(rob & 0xFFFFFF == 0) and np.all((rob >> 24) >= 2)  # robot links 1.. (link + 1 in the top byte)
    assert np.all(segl[seg == 1] == 1) and np.all(segl[seg == -1] == -1)  # object base link -1 -> code + 0


def test_renderer_analytic_sphere_depth():
    """the ball pixel nearest the image centre when looking straight down at it: depth of the sphere's top,
    through OpenGL's depth mapping"""
    env = OracleEnv(0, 3)
    env.reset()
    st = env.get_state()
    ball = st[LY.obj(1):LY.obj(1) + 3]
    near, far, W, H = 0.05, 2.0, 33, 33
    cam = Camera(tuple(ball + [0, 0, 0.5]), tuple(ball), (0, 1, 0), near, far, (W, H), 30)
    rgb, depth, seg = env.camera(cam.view_matrix, cam.projection_matrix, W, H)
    # pixel (W/2, H/2) would be the centre for even sizes; for W = 33 the ray of pixel 16 passes at NDC -1/33
    assert seg[16, 16] == 2
    p = cam.rgbd_2_world(16, 16, depth[16, 16])
    assert abs(np.linalg.norm(p - ball) - 0.02) < 2e-6
    # the exact top of the sphere along the optical axis: eye distance 0.5 - r
    d_eye = 0.5 - 0.02
    A, B = (far + near) / (near - far), 2 * far * near / (near - far)
    expect = 0.5 * ((A * -d_eye + B) / d_eye) + 0.5  # clip z = A z_eye + B, w = -z_eye, z_eye = -d_eye
    c = cam.rgbd_2_world(W / 2, H / 2, expect)
    np.testing.assert_allclose(c, ball + [0, 0, 0.02], atol=1e-6)


def test_box_scene_renders_in_world_coordinates():
    """Box-v0 keeps the robot base at the origin internally (the box base at world y = 0 sits at y = -0.5 there); the
    camera's matrices are in world coordinates, so the closed door's lid top -- world (0, 0, 0.105): door joint at
    z 0.1, lid half height 0.005, skew-box-button.urdf -- must land under a camera looking straight down at it."""
    env = OracleEnv(7, 3)
    env.reset()
    W = H = 33
    cam = Camera((0.0, 0.0, 0.6), (0.0, 0.0, 0.105), (0, 1, 0), 0.05, 2.0, (W, H), 20)
    rgb, depth, seg = env.camera(cam.view_matrix, cam.projection_matrix, W, H)
    assert seg[16, 16] == 1  # the door link (object 0)
    np.testing.assert_allclose(cam.rgbd_2_world(W / 2, H / 2, depth[16, 16]), [0.0, 0.0, 0.105], atol=2e-6)
    # getContactPoints positions are world positions too: the closed lid (bottom face at z 0.095) rests on the button's
    # top (z 0.095) around the box's world origin
    env.step(np.zeros(8, np.float32))
    pts = env.contact_points(1, 2)
    assert len(pts) >= 1
    for p in pts:
        assert np.hypot(p[5], p[6]) < 0.02 + 1e-9 and abs(p[7] - 0.095) < 1e-3  # within the button's radius
