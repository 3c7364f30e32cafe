"""Instruction mix of one kernel in a hipcc -S listing: python tools/asm_mix.py file.s symbol_substring"""
import re
import sys
from collections import Counter

src, key = sys.argv[1], sys.argv[2]
lines = open(src).read().split('\n')
start = next(i for i, l in enumerate(lines) if re.match(r'^_Z\S*' + re.escape(key) + r'\S*:', l))
end = next(i for i in range(start, len(lines)) if 's_endpgm' in lines[i])
ins = [l.strip() for l in lines[start:end + 1] if l.startswith('\t') and not l.strip().startswith(('.', ';'))]
cls = Counter()
for l in ins:
    op = l.split()[0]
    cls['SALU' if op.startswith('s_') else 'VALU' if op.startswith('v_') else op.split('_')[0]] += 1
print(key, 'static instructions', len(ins), dict(cls))
print(Counter(l.split()[0] for l in ins if l.startswith('s_')).most_common(25))
print(Counter(l.split()[0] for l in ins if l.startswith('ds_')).most_common(10))
