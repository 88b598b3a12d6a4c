#!/usr/bin/env python3
"""Audit a gfx950 ISA listing for the miscompile behind VERDICT r2 item 7: frame-index elimination materialising a
private object's address with an SCC-writing `s_add_i32 sX, s32|s33, imm` between an SCC definition and the
s_cselect / s_cmov / s_cbranch_scc that reads it.  In the run-time-indexed team_box_box (-DUG_BB_DYNIDX) this
turned `nR < 3 ? R1 : R2` into "always R2".  Reports every SCC reader whose last SCC writer in straight-line code
is such a frame-address add.

Also audits the second miscompile met on this toolchain (round 5): LLVM's branch relaxation expands a branch beyond
+-32 Ki instructions into s_getpc_b64 / s_add_u32 / s_addc_u32 / s_setpc_b64 through a scavenged SGPR pair, and in a
leaf device function it scavenged s[30:31] -- the return address, which a leaf function never saves -- so the
function's return jumped into its own body (team_pgs: a kernel that never finished).  ra_audit() reports every
non-kernel function that writes s30 or s31 without first saving them (v_writelane_b32 vN, s30 / s31).

usage: python tools/scc_audit.py file.s   (make one with: hipcc ... --cuda-device-only -S -o file.s)"""
import re
import sys

READERS = re.compile(r"^\s*(s_cselect_b(32|64)|s_cmov_b(32|64)|s_cbranch_scc[01]|s_addc_u32|s_subb_u32|s_cmovk_i32)\b")
FRAME_ADD = re.compile(r"^\s*s_add_i32\s+s\d+,\s*s3[23],\s*(0x[0-9a-f]+|\d+)")  # stack / frame pointer
# instructions that write SCC (conservative: the SALU ops that set it)
WRITERS = re.compile(r"^\s*(s_(add|sub|addc|subb|and|or|xor|andn2|orn2|nand|nor|xnor|lshl|lshr|ashr|bfe|min|max|"
                     r"cmp|bitcmp|absdiff|abs|not|bcnt|quadmask|wqm|cselect_?x?)\w*)")


def audit(path):
    hits, fn, last_w = [], None, None
    for no, line in enumerate(open(path), 1):
        if re.match(r"^[_A-Za-z0-9.$]+:", line) and not line.startswith(".L"):
            fn, last_w = line.split(":")[0], None
            continue
        if line.startswith(".L") or re.match(r"^\s*s_(branch|cbranch)", line) and not READERS.match(line):
            last_w = None  # block boundary: SCC liveness across edges is not tracked here
            continue
        if READERS.match(line):
            if last_w is not None and FRAME_ADD.match(last_w[1]):
                hits.append((fn, last_w[0], last_w[1].strip(), no, line.strip()))
        if WRITERS.match(line) and not line.strip().startswith(("s_cselect", "s_cmov")):
            last_w = (no, line)
    return hits


RA_DEST = re.compile(r"^\s*(s_\w+|v_readlane_b32|v_readfirstlane_b32)\s+(s(\d+)|s\[(\d+):(\d+)\])\s*(,|$)")
RA_SAVE = re.compile(r"^\s*(v_writelane_b32\s+v\d+,\s*s3[01]\b|s_mov_b64\s+s\[\d+:\d+\],\s*s\[30:31\])")


def ra_audit(lines):
    """functions returning through s[30:31] that overwrite s30 / s31 without saving them first: (function, line no,
    instruction) of the first such write"""
    hits, fn, saved, first = [], None, False, None
    for no, line in enumerate(lines, 1):
        if re.match(r"^[_A-Za-z0-9.$]+:", line) and not line.startswith(".L"):
            fn, saved, first = line.split(":")[0], False, None
            continue
        if fn is None:
            continue
        if RA_SAVE.match(line):
            saved = True
        m = RA_DEST.match(line)
        if m and not line.strip().startswith("s_setpc_b64") and not saved and first is None:
            lo = int(m.group(3) or m.group(4))
            hi = int(m.group(3) or m.group(5))
            if lo <= 31 and hi >= 30 and not m.group(1).startswith(("s_cmp", "s_bitcmp")):
                first = (no, line.strip())
        if line.startswith(".Lfunc_end"):
            if first is not None and any("s_setpc_b64 s[30:31]" in l for l in lines[max(0, no - 40):no]):
                hits.append((fn, first[0], first[1]))
            fn = None
    return hits


if __name__ == "__main__":
    total = 0
    for p in sys.argv[1:]:
        h = audit(p)
        total += len(h)
        for fn, wl, w, rl, r in h:
            print(f"{p}:{rl}: {r}   <- SCC from line {wl}: {w}   [{fn}]")
        print(f"{p}: {len(h)} SCC reader(s) fed by a frame-address s_add_i32")
        r = ra_audit(open(p).read().split("\n"))
        total += len(r)
        for fn, no, ins in r:
            print(f"{p}:{no}: {ins}   <- writes the unsaved return address [{fn}]")
        print(f"{p}: {len(r)} function(s) overwriting an unsaved return address")
    sys.exit(1 if total else 0)
