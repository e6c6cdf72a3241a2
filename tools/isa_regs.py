"""Per-kernel register / spill summary from a hipcc -S (gfx950) assembly listing.
usage: python tools/isa_regs.py file.s [name-filter]"""
import re
import sys

txt = open(sys.argv[1]).read()
flt = sys.argv[2] if len(sys.argv) > 2 else ""
for blk in re.split(r"\n\s+- \.", txt):
    m = re.search(r"\.name:\s+(\S+)", blk)
    if not m or flt not in m.group(1):
        continue
    def f(k):
        mm = re.search(r"\." + k + r":\s+(\d+)", blk)
        return mm.group(1) if mm else "-"
    print(f"{m.group(1)[:90]:90s} vgpr={f('vgpr_count'):>4} agpr={f('agpr_count'):>4} vspill={f('vgpr_spill_count'):>3} "
          f"sspill={f('sgpr_spill_count'):>3} lds={f('group_segment_fixed_size'):>6} scratch={f('private_segment_fixed_size')}")
