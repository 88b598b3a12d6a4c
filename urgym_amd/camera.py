"""Camera: the reference's `urgym.base.utilities.Camera` (utilities.py:62-107) with its image rendered on the GPU.

Same constructor (cam_pos, cam_tar, cam_up_vector, near, far, size, fov), the same `view_matrix`,
`projection_matrix` and `tran_pix_world` attributes and the same `rgbd_2_world` / `rgbd_2_world_batch` back
projections.  `shot()` replaces p.getCameraImage with `urgym_camera_shot` (include/urgym.h): one HIP launch
renders the image of one env, `shot_batch()` of a whole range of envs at once (grid = pixel tiles x envs).

p.computeViewMatrix / p.computeProjectionMatrixFOV are restated from PyBullet's float implementations [ext]
(b3ComputeViewMatrixFromPositions: a gluLookAt; b3ComputeProjectionMatrixFOV: an OpenGL perspective), returned as
pybullet returns them: 16 floats, column-major.  pybullet is absent in this image, so they are unpinned against it;
tests/test_camera.py pins their defining properties and the back projection against the reference's own Camera
code (tests/golden/camera.json, tools/gen_golden.py).

What the image shows: the env's collision shapes (urgym_amd/csrc/ug_render.h lists the deviations from
TinyRenderer).  Segmentation values are the body codes of urgym_contact_points (0 robot, 1 + i task object i, 10
table, 11 plane, 12 golf pitch, 13 the Box's walls), plus ((link + 1) << 24) with `link_index=True`.
"""
import ctypes

import numpy as np

SEG_LINK = 1


def compute_view_matrix(eye, target, up):
    """p.computeViewMatrix(cameraEyePosition, cameraTargetPosition, cameraUpVector) [ext]: float arithmetic."""
    e = np.asarray(eye, np.float32)
    f = np.asarray(target, np.float32) - e
    f = f / np.float32(np.sqrt(np.float32(f @ f)))
    s = np.cross(f, np.asarray(up, np.float32)).astype(np.float32)
    s = s / np.float32(np.sqrt(np.float32(s @ s)))
    u = np.cross(s, f).astype(np.float32)
    m = np.zeros(16, np.float32)
    m[0:3] = s[0], u[0], -f[0]
    m[4:7] = s[1], u[1], -f[1]
    m[8:11] = s[2], u[2], -f[2]
    m[12], m[13], m[14], m[15] = -np.float32(s @ e), -np.float32(u @ e), np.float32(f @ e), 1.0
    return tuple(float(x) for x in m)


def compute_projection_matrix_fov(fov, aspect, near, far):
    """p.computeProjectionMatrixFOV(fov [deg], aspect, nearVal, farVal) [ext]."""
    y = np.float32(1.0 / np.tan(np.pi / 180.0 * fov / 2.0))
    x = np.float32(y / np.float32(aspect))
    m = np.zeros(16, np.float32)
    m[0], m[5] = x, y
    m[10] = np.float32((far + near) / (near - far))
    m[11] = -1.0
    m[14] = np.float32(2.0 * far * near / (near - far))
    return tuple(float(v) for v in m)


_MAX_BATCH = 65535  # envs per urgym_camera_shot call (include/urgym.h)


class Camera:
    """utilities.py:62-74: a fixed camera; `shot()` renders the env it is attached to (the env classes attach it, or
    call `attach(sim, env)`), `shot(sim, env)` any env of a handle."""

    def __init__(self, cam_pos, cam_tar, cam_up_vector, near, far, size, fov):
        self.width, self.height = size
        self.near, self.far = near, far
        self.fov = fov
        aspect = self.width / self.height
        self.view_matrix = compute_view_matrix(cam_pos, cam_tar, cam_up_vector)
        self.projection_matrix = compute_projection_matrix_fov(self.fov, aspect, self.near, self.far)
        view = np.array(self.view_matrix).reshape((4, 4), order="F")
        proj = np.array(self.projection_matrix).reshape((4, 4), order="F")
        self.tran_pix_world = np.linalg.inv(proj @ view)
        self._sim, self._env = None, 0

    def attach(self, sim, env=0):
        self._sim, self._env = sim, env
        return self

    def rgbd_2_world(self, w, h, d):
        """pixel (w, h) at depth-buffer value d -> world point (utilities.py:76-84)."""
        ndc = np.array(((2 * w - self.width) / self.width, -(2 * h - self.height) / self.height, 2 * d - 1, 1.0))
        p = self.tran_pix_world @ ndc
        return (p / p[3])[:3]

    def rgbd_2_world_batch(self, depth):
        """every pixel of a height x width depth image -> height x width x 3 world points (utilities.py:91-107)."""
        cols = (2 * np.arange(self.width) - self.width) / self.width
        rows = -(2 * np.arange(self.height) - self.height) / self.height
        X, Y = np.meshgrid(cols, rows)
        Z = 2 * np.asarray(depth) - 1
        ndc = np.stack([X.ravel(), Y.ravel(), Z.ravel(), np.ones(X.size)])
        p = (self.tran_pix_world @ ndc).T
        p = p / p[:, 3:4]
        return p[:, :3].reshape(self.height, self.width, 3)

    def _mats(self):
        return (np.asarray(self.view_matrix, np.float32), np.asarray(self.projection_matrix, np.float32))

    def shot_batch(self, sim, env0=0, count=None, link_index=False):
        """images of envs [env0, env0 + count) of `sim`: rgb (count, H, W, 4) u8, depth (count, H, W) f32,
        seg (count, H, W) i32 -- one GPU launch."""
        count = sim.n - env0 if count is None else count
        W, H = self.width, self.height
        rgb = np.zeros((count, H, W, 4), np.uint8)
        depth = np.zeros((count, H, W), np.float32)
        seg = np.zeros((count, H, W), np.int32)
        v, p = self._mats()
        for c0 in range(0, count, _MAX_BATCH):  # one launch per 65,535 envs (the kernel's grid.y bound)
            c = min(_MAX_BATCH, count - c0)
            rc = sim.L.urgym_camera_shot(sim.h, env0 + c0, c, v.ctypes.data_as(ctypes.c_void_p),
                                         p.ctypes.data_as(ctypes.c_void_p), W, H, SEG_LINK if link_index else 0,
                                         rgb[c0:].ctypes.data_as(ctypes.c_void_p), depth[c0:].ctypes.data_as(ctypes.c_void_p),
                                         seg[c0:].ctypes.data_as(ctypes.c_void_p))
            sim._chk(rc, "urgym_camera_shot")
        return rgb, depth, seg

    def shot(self, sim=None, env=None, link_index=False):
        """utilities.py:84-89: (rgb (H, W, 4) u8, depth (H, W) f32, seg (H, W) i32) of one env."""
        sim = self._sim if sim is None else sim
        env = self._env if env is None else env
        if sim is None:
            raise RuntimeError("Camera.shot(): no env attached (pass sim, or construct the env with camera=...)")
        rgb, depth, seg = self.shot_batch(sim, env, 1, link_index)
        return rgb[0], depth[0], seg[0]
