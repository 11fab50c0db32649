"""Static instruction count of a kernel attributed to the source function each instruction's
debug line (.loc) falls in (build the .s with -g --save-temps).  Inlined code is attributed to
the innermost function, i.e. the primitive that produced it.

  python scripts/isa_lines.py file.s kernel_substring [loop_only]
loop_only: count only instructions between the first and last instruction of the innermost
loop containing the most instructions (the substep loop).
"""
import re
import sys
from collections import Counter, defaultdict

s = open(sys.argv[1]).read()
key = sys.argv[2]
files = {int(m.group(1)): m.group(2) + "/" + m.group(3)
         for m in re.finditer(r'^\s*\.file\s+(\d+)\s+"([^"]*)"\s+"([^"]*)"', s, re.M)}
names = [l.split(':')[0] for l in s.split('\n') if l.startswith('_Z') and ':' in l
         and key in l.split(':')[0]]
if not names:
    raise SystemExit("no kernel")
name = names[0]
i = s.index(name + ':')
j = s.index('.Lfunc_end', i)
body = s[i:j].split('\n')

# function ranges per source file: "DEV ... name(" / "__global__ ... name(" to the closing brace
func_ranges = defaultdict(list)
def ranges_for(path):
    if path in func_ranges:
        return func_ranges[path]
    try:
        src = open(path).read().split('\n')
    except OSError:
        func_ranges[path] = []
        return []
    out = []
    k = 0
    while k < len(src):
        line = src[k]
        m = re.match(r'^(?:template\s*<.*>\s*)?(?:DEV|__device__|__global__|static|inline|DEV\s+inline)[^;{]*?\b([A-Za-z_][A-Za-z0-9_]*)\s*\(', line)
        if m and not line.strip().endswith(';'):
            depth, started, e = 0, False, k
            while e < len(src):
                depth += src[e].count('{') - src[e].count('}')
                if '{' in src[e]:
                    started = True
                if started and depth <= 0:
                    break
                e += 1
            out.append((k + 1, e + 1, m.group(1)))
            k = e + 1
            continue
        k += 1
    func_ranges[path] = out
    return out

def func_of(fid, line):
    path = files.get(fid, "?")
    for a, b, nm in ranges_for(path):
        if a <= line <= b:
            return path.split('/')[-1] + ":" + nm
    return path.split('/')[-1] + ":?"

insts = []  # (index, func)
cur = (0, 0)
for l in body:
    t = l.strip()
    m = re.match(r'\.loc\s+(\d+)\s+(\d+)', t)
    if m:
        cur = (int(m.group(1)), int(m.group(2)))
        continue
    if not t or t.startswith(('.', ';', '_Z')) or t.endswith(':'):
        continue
    insts.append((t.split()[0], cur))

lo, hi = 0, len(insts)
if len(sys.argv) > 3:
    # innermost big loop: backward branch spanning the most instructions below 60 % of the kernel
    labels = {}
    k = 0
    for l in body:
        t = l.strip()
        if t.startswith('.LBB') and ':' in t:
            labels[t.split(':')[0]] = k
        elif t and not t.startswith(('.', ';', '_Z')) and not t.endswith(':'):
            k += 1
    k = 0
    best = None
    for l in body:
        t = l.strip()
        if not t or t.startswith(('.', ';', '_Z')) or t.endswith(':'):
            continue
        if t.startswith('s_cbranch') or t.startswith('s_branch'):
            tgt = t.split()[-1]
            if tgt in labels and labels[tgt] < k:
                span = k - labels[tgt]
                if span < 0.8 * len(insts) and (best is None or span > best[1] - best[0]):
                    best = (labels[tgt], k)
        k += 1
    lo, hi = best
    print(f"loop: instructions {lo}..{hi} ({hi - lo})")
c = Counter()
valu = Counter()
for op, (fid, line) in insts[lo:hi]:
    f = func_of(fid, line)
    c[f] += 1
    if op.startswith('v_'):
        valu[f] += 1
tot = sum(c.values())
print(f"{name}: {tot} instructions ({sum(valu.values())} VALU)")
for f, n in c.most_common(40):
    print(f"  {f:40s} {n:6d}  {100.0 * n / tot:5.1f} %  VALU {valu[f]}")
