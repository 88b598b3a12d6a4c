"""VERDICT r2 item 7, root cause: run-time indices into a pointer-selected private object (`nR < 3 ? R1 : R2`,
then `.m[c]`) miscompile with this ROCm's LLVM -- frame-index elimination materialises the second object's
address with an SCC-writing `s_add_i32 sX, s32|s33, imm` between the SCC definition and the `s_cselect` that
picks the base, so the pick always takes the second object (tools/micro/bbidx.hip reproduces it; on MI355X the
in-situ -DUG_BB_DYNIDX build printed R2's column where R1's was due).  team_box_box picks by selects instead.
These CPU tests compile to gfx950 ISA and audit it (tools/scc_audit.py): the shipped library has no such
SCC reader, and the audit does flag the reproducer (so a clean result means something)."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["-O3", "--offload-arch=gfx950", "-ffp-contract=off", "-fno-fast-math", "-std=c++17", "-w", "--cuda-device-only",
         "-S"]


def _isa(src, out, defs=()):
    if not os.path.exists(HIPCC):
        pytest.skip("hipcc not available")
    subprocess.run([HIPCC] + FLAGS + list(defs) + ["-o", str(out), src], check=True, cwd=ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import scc_audit
    return scc_audit.audit(str(out))


def test_audit_flags_the_reproducer(tmp_path):
    hits = _isa(os.path.join(ROOT, "tools", "micro", "bbidx.hip"), tmp_path / "bbidx.s")
    assert len(hits) >= 1 and all("s_cselect" in h[4] for h in hits), hits


@pytest.mark.parametrize("defs", [(), ("-DUG_ROBOT_R140",)], ids=["ur5_robotiq_85", "ur5_robotiq_140"])
def test_shipped_library_has_no_scc_clobbered_pick(tmp_path, defs):
    hits = _isa(os.path.join(ROOT, "urgym_amd", "csrc", "ug_capi.hip"), tmp_path / "ug.s", defs)
    assert hits == [], hits
