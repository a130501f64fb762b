"""Scratch (spill) instructions of one kernel in a `hipcc -S` listing, with the
basic block each sits in (dev tool).  usage: tools/spills.py LISTING.s SYMBOL"""
import re
import sys

path, sym = sys.argv[1], sys.argv[2]
inside, block, n = False, "", 0
for line in open(path):
    if line.startswith(sym + ":"):
        inside = True
        continue
    if inside and line.startswith(".Lfunc_end"):
        break
    if not inside:
        continue
    if re.match(r"^\.LBB\w+:", line):
        block = line.strip()
    elif not line.strip().startswith((";", ".")) and line.strip():
        n += 1
        if "scratch_" in line:
            print(f"{n:5d} {line.strip()[:70]:70s} {block[:60]}")
print("instructions:", n)
