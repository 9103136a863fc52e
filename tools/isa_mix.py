#!/usr/bin/env python3
"""Static instruction mix of kernels in a hipcc --cuda-device-only -S listing.
usage: isa_mix.py FILE.s SYMBOL_PREFIX..."""
import collections, sys
lines = open(sys.argv[1]).read().split('\n')
for name in sys.argv[2:]:
    i = next(k for k, l in enumerate(lines) if l.startswith(name) and ': ' in l or l.startswith(name) and l.endswith(':'))
    c = collections.Counter()
    for l in lines[i + 1:]:
        l = l.strip()
        if l.startswith('.Lfunc_end'):
            break
        if not l or l.startswith(('.', ';', '_')) or l.endswith(':'):
            continue
        c[l.split()[0]] += 1
    print(lines[i][:90], 'static instrs', sum(c.values()))
    print('  ', ' '.join('%s:%d' % (op, n) for op, n in c.most_common(45)))
