"""VGPR / spill / scratch of every kernel in a device .s file (hipcc -S)."""
import re
import subprocess
import sys

s = open(sys.argv[1]).read()
pat = sys.argv[2] if len(sys.argv) > 2 else ""
for e in re.split(r"\n  - \.", s[s.find("amdhsa.kernels"):]):
    nm = re.search(r"\.name:\s+(\S+)", e)
    if not nm or pat not in nm.group(1):
        continue
    g = lambda k: (re.search(rf"\.{k}:\s+(\d+)", e) or [None, "-"])[1]
    dn = subprocess.run(["c++filt", nm.group(1)], capture_output=True, text=True).stdout.strip()
    print(f"{dn[:100]:100s} vgpr {g('vgpr_count')} spill {g('vgpr_spill_count')} scratch {g('private_segment_fixed_size')} "
          f"lds {g('group_segment_fixed_size')}")
