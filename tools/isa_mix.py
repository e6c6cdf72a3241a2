"""Instruction mix of one kernel in a hipcc -S (gfx950) listing, per basic block and in total.
usage: python tools/isa_mix.py file.s <mangled-name-substring> [--blocks]"""
import collections
import re
import sys

txt = open(sys.argv[1]).read()
key = sys.argv[2]
m = re.search(r"^(\S*" + re.escape(key) + r"\S*):", txt, re.M)
start = m.end()
end = txt.index(".Lfunc_end", start)
lines = txt[start:end].splitlines()


def cls(l):
    op = l.split()[0]
    if op.startswith("v_mfma"):
        return "mfma"
    if op.startswith("v_accvgpr"):
        return "accvgpr"
    if op.startswith("v_"):
        return "valu_dpp" if ("row_" in l or "quad_perm" in l or "dpp" in l) else "valu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith("scratch_") or "scratch" in l:
        return "scratch"
    if op.startswith(("buffer_", "global_", "flat_")):
        return "vmem"
    if op.startswith("s_waitcnt"):
        return "waitcnt"
    return "salu"


blocks = []
cur = [None, collections.Counter()]
for l in lines:
    s = l.strip()
    if re.match(r"^\.LBB\S*:", s) or (s.endswith(":") and not s.startswith(";")):
        blocks.append(cur)
        cur = [s, collections.Counter()]
        continue
    if not s or s.startswith((";", ".")):
        continue
    cur[1][cls(s)] += 1
blocks.append(cur)
tot = collections.Counter()
for name, c in blocks:
    tot.update(c)
    if "--blocks" in sys.argv and sum(c.values()) > 20:
        print(name, dict(c))
print("total", dict(tot), sum(tot.values()))
