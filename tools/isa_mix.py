"""Static instruction mix per kernel of an amdgcn .s file (tooling, not product code).
Usage: python tools/isa_mix.py file.s [kernel-substring]"""
import collections
import re
import sys

lines = open(sys.argv[1]).read().split('\n')
sub = sys.argv[2] if len(sys.argv) > 2 else ''
starts = [i for i, l in enumerate(lines) if re.match(r'^_Z\w+:', l) and sub in l]
for s in starts:
    e = s
    while 's_endpgm' not in lines[e]:
        e += 1
    c = collections.Counter()
    for line in lines[s:e]:
        t = line.strip().split()
        if not t or t[0].startswith(('.', ';')) or t[0].endswith(':'):
            continue
        op = t[0]
        if op.startswith(('ds_read', 'ds_load')):
            c['ds_read'] += 1
        elif op.startswith(('ds_write', 'ds_store')):
            c['ds_write'] += 1
        elif re.match(r'v_(fma|mul|add)_f64', op):
            c['f64'] += 1
        elif op.startswith('v_'):
            c['valu_other'] += 1
        elif op.startswith('s_waitcnt'):
            c['waitcnt'] += 1
        elif op.startswith('s_'):
            c['salu'] += 1
        elif op.startswith(('global_', 'buffer_', 'scratch_', 'flat_')):
            c['vmem:' + op.split('_')[0]] += 1
        else:
            c[op] += 1
    print(lines[s].split(':')[0][:70], dict(c))
