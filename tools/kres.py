#!/usr/bin/env python3
"""Compact per-kernel resource usage of one HIP TU (VGPRs, SGPRs, scratch,
LDS, occupancy) from hipcc's -Rpass-analysis=kernel-resource-usage remarks.
usage: kres.py FILE.hip [-DX=Y ...] [--filter SUBSTR]"""
import re, subprocess, sys
args = sys.argv[1:]
flt = None
if '--filter' in args:
    i = args.index('--filter'); flt = args[i + 1]; del args[i:i + 2]
src, defs = args[0], args[1:]
cmd = ['/opt/rocm/bin/hipcc', '-O3', '-std=c++17', '-fPIC', '-ffp-contract=off', '--offload-arch=gfx950',
       '-c', src, '-o', '/dev/null', '-Rpass-analysis=kernel-resource-usage'] + defs
out = subprocess.run(cmd, capture_output=True, text=True, cwd='jwave_amd/csrc').stderr
cur = None; rows = []
for line in out.splitlines():
    m = re.search(r'Function Name: (\S+)', line)
    if m:
        cur = {'name': m.group(1)}; rows.append(cur); continue
    for key, pat in (('vgpr', r' VGPRs: (\d+)'), ('agpr', r'AGPRs: (\d+)'), ('sgpr', r'TotalSGPRs: (\d+)'),
                     ('scr', r'ScratchSize \[bytes/lane\]: (\d+)'), ('occ', r'Occupancy \[waves/SIMD\]: (\d+)'),
                     ('lds', r'LDS Size \[bytes/block\]: (\d+)')):
        m = re.search(pat, line)
        if m and cur is not None: cur[key] = int(m.group(1))
dm = subprocess.run(['c++filt'], input='\n'.join(r['name'] for r in rows),
                    capture_output=True, text=True).stdout.splitlines()
for r, d in zip(rows, dm):
    d = re.sub(r'\(.*$', '', d)
    if flt and flt not in d: continue
    print(f"v{r.get('vgpr',0):4d} s{r.get('sgpr',0):4d} scr{r.get('scr',0):4d} lds{r.get('lds',0):6d} occ{r.get('occ',0):2d}  {d}")
if not rows:
    print(out[-3000:])
