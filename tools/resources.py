"""Compact per-kernel resource table from `make -C uu-infogr-raytracer_amd/csrc resources` (stdin):
name  SGPRs VGPRs scratch occupancy -- for A/B of register pressure between builds."""
import re
import sys

cur = None
rows = {}
for line in sys.stdin:
    m = re.search(r"Name: (\S+)", line)
    if m:
        cur = m.group(1)
        rows[cur] = {}
        continue
    for key, pat in (("sgpr", r"TotalSGPRs: (\d+)"), ("vgpr", r"VGPRs: (\d+)"), ("scratch", r"ScratchSize \[bytes/lane\]: (\d+)"),
                     ("occ", r"Occupancy \[waves/SIMD\]: (\d+)")):
        m = re.search(pat, line)
        if m and cur:
            rows[cur].setdefault(key, m.group(1))
for k in sorted(rows):
    r = rows[k]
    print(f"{k:70s} s{r.get('sgpr')} v{r.get('vgpr')} scr{r.get('scratch')} occ{r.get('occ')}")
