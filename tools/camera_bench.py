"""Throughput of the batched camera (urgym_camera_shot_device, k_camera): one launch renders rgba / depth / seg of
every env of a handle into device buffers.  Prints one JSON line per (task, envs, size): images/s and pixels/s
(wall clock over K launches after a warm-up, synchronized on the handle's stream).
usage: python tools/camera_bench.py [K]"""
import ctypes
import json
import sys
import time

import numpy as np

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
import torch  # noqa: E402  (torch before liburgym, urgym_amd/_native.py)

from urgym_amd._native import Sim  # noqa: E402
from urgym_amd.camera import Camera  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 10
vp = ctypes.c_void_p
for task, n, (W, H) in [(7, 4096, (128, 128)), (2, 8192, (64, 64)), (0, 4096, (128, 128))]:
    sim = Sim(task, n, seed=1)
    sim.reset()
    cam = Camera((1, 1, 1), (0, 0, 0), (0, 0, 1), 0.1, 5, (W, H), 40)
    dev = torch.device("cuda", 0)
    rgba = torch.empty((n, H, W, 4), dtype=torch.uint8, device=dev)
    depth = torch.empty((n, H, W), dtype=torch.float32, device=dev)
    seg = torch.empty((n, H, W), dtype=torch.int32, device=dev)
    torch.cuda.synchronize()
    v = np.asarray(cam.view_matrix, np.float32)
    p = np.asarray(cam.projection_matrix, np.float32)

    def shot():
        assert sim.L.urgym_camera_shot_device(sim.h, 0, n, v.ctypes.data_as(vp), p.ctypes.data_as(vp), W, H, 0,
                                              vp(rgba.data_ptr()), vp(depth.data_ptr()), vp(seg.data_ptr())) == 0

    shot()
    sim.sync()
    t = time.perf_counter()
    for _ in range(K):
        shot()
    sim.sync()
    dt = (time.perf_counter() - t) / K
    hit = float((seg[: min(n, 64)] >= 0).float().mean())
    print(json.dumps({"task": task, "envs": n, "size": [W, H], "ms_per_launch": dt * 1e3, "images_per_s": n / dt,
                      "pixels_per_s": n * W * H / dt, "hit_fraction": hit}), flush=True)
    sim.close()
