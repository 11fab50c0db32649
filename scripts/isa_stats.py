"""Static instruction mix of a kernel in a --save-temps .s file.
  python scripts/isa_stats.py file.s kernel_substring [top]"""
import sys
from collections import Counter
s = open(sys.argv[1]).read()
key = sys.argv[2]
top = int(sys.argv[3]) if len(sys.argv) > 3 else 25
names = [l.split(':')[0] for l in s.split('\n') if l.startswith('_Z') and ':' in l and key in l.split(':')[0]]
for name in names:
    i = s.index(name + ':')
    j = s.index('.Lfunc_end', i)
    lines = [l.strip() for l in s[i:j].split('\n') if l.strip() and not l.strip().startswith(('.', ';', '_Z'))]
    c = Counter(l.split()[0] for l in lines)
    print(name, 'instructions', len(lines))
    print('  ', c.most_common(top))
