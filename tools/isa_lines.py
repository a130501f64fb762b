#!/usr/bin/env python3
"""Static ISA attribution (dev tool): instructions of one kernel in a `hipcc -g -S`
listing, attributed through .loc to source functions.
usage: tools/isa_lines.py LISTING.s KERNEL_SYMBOL_SUBSTRING"""
import collections
import re
import sys

src_path, ksub = sys.argv[1], sys.argv[2]
files, cur, inside = {}, None, False
counts = collections.Counter()
for line in open(src_path):
    m = re.match(r'\s*\.file\s+(\d+)\s+"([^"]*)"\s+"([^"]*)"', line)
    if m:
        files[int(m.group(1))] = m.group(2) + "/" + m.group(3)
        continue
    if re.match(r'^[_A-Za-z][\w.]*:', line):
        name = line.split(':')[0]
        if ksub in name and not name.startswith('.'):
            inside = True
        elif inside and not name.startswith('.') and ksub not in name:
            inside = False
        continue
    if not inside:
        continue
    m = re.match(r'\s*\.loc\s+(\d+)\s+(\d+)', line)
    if m:
        cur = (int(m.group(1)), int(m.group(2)))
        continue
    m = re.match(r'\t([vs]_\w+|ds_\w+|global_\w+|buffer_\w+|flat_\w+|scratch_\w+)', line)
    if m and cur:
        op = m.group(1)
        cls = 'valu' if op.startswith('v_') else 'salu' if op.startswith('s_') else 'mem'
        counts[(cur, cls)] += 1

# function ranges per source file
ranges = {}
for fid, path in files.items():
    try:
        lines = open(path).read().split('\n')
    except OSError:
        continue
    defs = []
    for i, l in enumerate(lines, 1):
        m = re.match(r'(?:template <[^>]*>\s*)?(?:RT_D|__global__|static|__device__)[^(;]*?\b(\w+)\s*\(', l)
        if m:
            defs.append((i, m.group(1)))
    ranges[fid] = defs
by_func = collections.Counter()
for ((fid, ln), cls), n in counts.items():
    fn = '?'
    for i, name in ranges.get(fid, []):
        if i <= ln:
            fn = name
    by_func[(files.get(fid, str(fid)).split('/')[-1] + ':' + fn, cls)] += n
tot = collections.Counter()
for (f, cls), n in by_func.items():
    tot[cls] += n
print('total', dict(tot))
funcs = sorted({f for f, _ in by_func}, key=lambda f: -by_func[(f, 'valu')])
for f in funcs[:45]:
    print(f'{f:45s} valu {by_func[(f, "valu")]:5d} salu {by_func[(f, "salu")]:5d} mem {by_func[(f, "mem")]:4d}')
