"""Collects CubesGrasp step-length rows under uniform random actions (development aid for its launch order; the
kernel's results do not depend on it).  Per env and step, before the step: q[12], qd[12], the motor targets[7] and
enables[7], elapsed steps, the u = random() the step's random.choices will draw (peeked on the host from the env's
MT19937 stream, urgym_get_rng; env_cubes_grasp_v0.py:127-130), the step's action[9]; after it: substeps and the
reset flag.  Writes gpurun_out/r6_steps_cg.npy (float32,
the first 4096 envs).
usage: python tools/predict_steps_cg.py envs steps [seed]"""
import os
import sys

import numpy as np

ROOT = __file__.rsplit("/tools/", 1)[0]
sys.path.insert(0, ROOT)
from urgym_amd import layout as LY  # noqa: E402
from urgym_amd._native import Sim  # noqa: E402
from urgym_amd.envs import spaces_for  # noqa: E402
from bench import MAX_STEPS  # noqa: E402


def temper(y):
    y = y ^ (y >> np.uint32(11))
    y = y ^ ((y << np.uint32(7)) & np.uint32(0x9D2C5680))
    y = y ^ ((y << np.uint32(15)) & np.uint32(0xEFC60000))
    return y ^ (y >> np.uint32(18))


def twist_word(mt, k):
    """word k (0 or 1) of the next MT19937 generation, from the current one (n x 625, column 624 = index)"""
    y = (mt[:, k] & np.uint32(0x80000000)) | (mt[:, k + 1] & np.uint32(0x7FFFFFFF))
    return mt[:, k + 397] ^ (y >> np.uint32(1)) ^ np.where((y & np.uint32(1)) != 0, np.uint32(0x9908B0DF), np.uint32(0))


def peek_random(mt):
    """the next random() of every stream without advancing it: (a >> 5, b >> 6) of the next two outputs"""
    idx = mt[:, 624].astype(np.int64)
    n = len(idx)
    w = np.empty((n, 2), np.uint32)
    for j in range(2):
        k = idx + j
        cur = k < 624
        w[cur, j] = mt[np.nonzero(cur)[0], k[cur]]
        nxt = ~cur
        if nxt.any():
            w[nxt, j] = twist_word(mt[nxt], 0) if j == 0 else np.where(idx[nxt] >= 624, twist_word(mt[nxt], 1),
                                                                        twist_word(mt[nxt], 0))
    a, b = temper(w[:, 0]) >> np.uint32(5), temper(w[:, 1]) >> np.uint32(6)
    return (a.astype(np.float64) * 67108864.0 + b.astype(np.float64)) / 9007199254740992.0


def main():
    n, steps = int(sys.argv[1]), int(sys.argv[2])
    seed = int(sys.argv[3]) if len(sys.argv) > 3 else 20241220
    task = 2
    sim = Sim(task, n, seed=seed)
    sim.set_autoreset(True, MAX_STEPS[task])
    sim.reset()
    act = spaces_for(task)[1]
    lo, hi = np.asarray(act.low, np.float64), np.asarray(act.high, np.float64)
    rng = np.random.default_rng(0)
    rows = []
    for t in range(steps):
        s = sim.get_state()
        mt, el = sim.get_rng()
        u = peek_random(mt)
        a = rng.uniform(lo, hi, size=(n, len(lo))).astype(np.float32)
        out = sim.step(a)
        d = (out["terminated"] | out["truncated"]).astype(float)
        rows.append(np.concatenate([s[:, LY.F_Q:LY.F_Q + 12], s[:, LY.F_QD:LY.F_QD + 12],
                                    s[:, LY.F_MTARGET:LY.F_MTARGET + 7], s[:, LY.F_MON:LY.F_MON + 7],
                                    el[:, None].astype(np.float64), u[:, None], a.astype(np.float64),
                                    out["substeps"][:, None].astype(np.float64), d[:, None]], 1))
        print("step", t, "substeps p50 / max", int(np.median(out["substeps"])), int(out["substeps"].max()), flush=True)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    # float32, the first 4096 envs' rows (gpurun copies back at most 64 MiB)
    keep = min(n, 4096)
    np.save(os.path.join(ROOT, "gpurun_out", "r6_steps_cg.npy"),
            np.concatenate([r[:keep] for r in rows]).astype(np.float32))
    print("saved", sum(len(r) for r in rows))


if __name__ == "__main__":
    main()
