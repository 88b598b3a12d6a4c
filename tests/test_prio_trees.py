"""The launch-order tree ensembles (urgym_amd/csrc/prio_model_gf.h, prio_model_tbt.h; tools/fit_priority.py
tree_header) are well formed: every tree is reachable from its root, every internal node's children lie inside its
own tree, features index the model's inputs, and every walk ends at a leaf within k_prio's depth bound.  Scheduling
only -- no result depends on them (tests/test_gpu_queue.py) -- but a malformed table would read out of bounds."""
import os
import re

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def load(hdr, P):
    txt = open(os.path.join(ROOT, "urgym_amd", "csrc", hdr)).read()
    d = {k: float(v) for k, v in re.findall(r"#define UG_PF_%s_(\w+) (\S+)" % P, txt)}
    for name, body in re.findall(r"UG_PF_%s_(\w+)\[\d+\] = \{([^}]*)\}" % P, txt):
        d[name] = np.array([float(x) for x in body.split(",")])
    return d


@pytest.mark.parametrize("hdr,P", [("prio_model_gf.h", "GF"), ("prio_model_gj.h", "GJ"), ("prio_model_tbt.h", "TBT"), ("prio_model_cgt.h", "CGT")])
def test_tree_tables_well_formed(hdr, P):
    d = load(hdr, P)
    nt, nin = int(d["TREES"]), int(d["IN"])
    root, feat, left, right = d["ROOT"].astype(int), d["FEAT"].astype(int), d["LEFT"].astype(int), d["RIGHT"].astype(int)
    assert len(root) == nt and root[0] == 0 and np.all(np.diff(root) > 0)
    ends = list(root[1:]) + [len(feat)]
    assert feat.max() < nin and feat.min() >= -1
    for t in range(nt):
        lo, hi = root[t], ends[t]
        inner = np.nonzero(feat[lo:hi] >= 0)[0] + lo
        assert np.all((left[inner] > inner) & (left[inner] < hi)) and np.all((right[inner] > inner) & (right[inner] < hi))
    # random walks end at leaves within the kernel's bound of 64
    rng = np.random.default_rng(0)
    for x in rng.normal(0.0, 1.0, size=(200, nin)):
        for t in range(nt):
            k, depth = root[t], 0
            while feat[k] >= 0:
                k = left[k] if x[feat[k]] <= d["THR"][k] else right[k]
                depth += 1
            assert depth < 64
