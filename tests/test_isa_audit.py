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


def _isa(src, out, defs=(), ra=False):
    if not os.path.exists(HIPCC):
        pytest.skip("hipcc not available")
    subprocess.run([HIPCC] + FLAGS + list(defs) + ["-o", str(out), src], check=True, cwd=ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import scc_audit
    if ra:
        return scc_audit.audit(str(out)), scc_audit.ra_audit(open(out).read().split("\n"))
    return scc_audit.audit(str(out))


def test_audit_flags_the_reproducer(tmp_path):
    hits = _isa(os.path.join(ROOT, "tools", "micro", "bbidx.hip"), tmp_path / "bbidx.s")
    assert len(hits) >= 1 and all("s_cselect" in h[4] for h in hits), hits


@pytest.mark.parametrize("defs", [(), ("-DUG_ROBOT_R140",), ("-DUG_GJK_G=8",)],
                         ids=["ur5_robotiq_85", "ur5_robotiq_140", "gjk_g8"])
def test_shipped_library_has_no_scc_clobbered_pick(tmp_path, defs):
    """both miscompiles: no SCC reader fed by a frame-address add, and no device function that overwrites its unsaved
    return address (a long branch through s[30:31] in a leaf function; team_pgs carries a never-taken call so it is
    not a leaf -- see ug_nonleaf_guard in ug_team.h)"""
    hits, ra = _isa(os.path.join(ROOT, "urgym_amd", "csrc", "ug_capi.hip"), tmp_path / "ug.s", defs, ra=True)
    assert hits == [], hits
    assert ra == [], ra


def test_return_address_audit_flags_a_leaf_long_branch():
    """the shape the round-5 team_pgs build had: a leaf function whose long branch goes through s[30:31]"""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import scc_audit
    leaf = ["_Z4leafv:", "\ts_cbranch_scc0 .LBB0_2", "\ts_getpc_b64 s[30:31]", ".Lpost_getpc0:",
            "\ts_add_u32 s30, s30, (.LBB0_9-.Lpost_getpc0)&4294967295", "\ts_addc_u32 s31, s31, (.LBB0_9-.Lpost_getpc0)>>32",
            "\ts_setpc_b64 s[30:31]", ".LBB0_2:", "\ts_setpc_b64 s[30:31]", ".Lfunc_end0:"]
    assert [h[0] for h in scc_audit.ra_audit(leaf)] == ["_Z4leafv"]
    saved = leaf[:1] + ["\tv_writelane_b32 v255, s30, 0", "\tv_writelane_b32 v255, s31, 1"] + leaf[1:]
    assert scc_audit.ra_audit(saved) == []
