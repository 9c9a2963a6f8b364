"""Print VGPR / AGPR / spill counts per kernel from a hipcc -S listing:
python tools/kstats.py file.s [name-regex]"""
import re
import sys

text = open(sys.argv[1]).read()
pat = re.compile(sys.argv[2] if len(sys.argv) > 2 else ".")
for blk in text.split("  - .agpr_count:")[1:]:
    name = re.search(r"\.name:\s+(\S+)", blk).group(1)
    if not pat.search(name):
        continue
    get = lambda k: (re.search(rf"\.{k}:\s+(\d+)", blk) or [None, "?"])[1]
    print(f"{name[:90]:90s} vgpr {get('vgpr_count'):>4} spill {get('vgpr_spill_count'):>4} "
          f"sgpr_spill {get('sgpr_spill_count'):>3} lds {get('group_segment_fixed_size')}")
