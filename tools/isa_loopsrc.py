"""Development aid: scratch (spill / callee-saved) accesses inside loops of the GJK and collision functions, by source
line.  Input: an ISA listing with line tables (hipcc ... --cuda-device-only -S -gline-tables-only -o file.s).
usage: python tools/isa_loopsrc.py file.s"""
import re, sys, collections
lines = open(sys.argv[1]).read().split('\n')
files = {}
for l in lines:
    m = re.match(r'\s*\.file\s+(\d+)\s+"([^"]*)"(?:\s+"([^"]*)")?', l)
    if m: files[m.group(1)] = (m.group(3) or m.group(2)).split('/')[-1]
# function ranges
funcs = []; cur = None
for i, l in enumerate(lines):
    m = re.match(r'^([_A-Za-z][\w.$]*):', l)
    if m and not l.startswith('.L'):
        cur = (m.group(1), i)
    if l.startswith('.Lfunc_end') and cur:
        funcs.append((cur[0], cur[1], i)); cur = None
for name, a, b in funcs:
    if 'gjk' not in name and 'team_collide' not in name: continue
    body = lines[a:b]
    labels = {}
    for j, l in enumerate(body):
        m = re.match(r'^(\.LBB\w+):', l)
        if m: labels[m.group(1)] = j
    inloop = collections.Counter()
    depth = [0] * len(body)
    for j, l in enumerate(body):
        m = re.search(r's_(cbranch_\w+|branch)\s+(\.LBB\w+)', l)
        if m and m.group(2) in labels and labels[m.group(2)] < j:
            for k in range(labels[m.group(2)], j): depth[k] += 1
    loc = None
    for j, l in enumerate(body):
        m = re.match(r'\s*\.loc\s+(\d+)\s+(\d+)', l)
        if m: loc = (files.get(m.group(1), m.group(1)), int(m.group(2)))
        if depth[j] and re.search(r'\bscratch_(store|load)', l):
            inloop[(loc, 'st' if 'store' in l else 'ld', depth[j])] += 1
    print(name[:60], sum(inloop.values()))
    for (loc, k, d), n in sorted(inloop.items(), key=lambda x: -x[1])[:25]:
        print("   %3d %s depth %d %s" % (n, k, d, loc))
