"""Per-kernel register summary from hipcc -Rpass-analysis=kernel-resource-usage output (stdin)."""
import re
import sys

cur = None
rows = []
for line in sys.stdin:
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = {"name": m.group(1)}
        rows.append(cur)
        continue
    if cur is None:
        continue
    for key, pat in (("vgpr", r"\bVGPRs: (\d+)"), ("vspill", r"VGPRs Spill: (\d+)"), ("sspill", r"SGPRs Spill: (\d+)"),
                     ("occ", r"Occupancy \[waves/SIMD\]: (\d+)"), ("scratch", r"ScratchSize \[bytes/lane\]: (\d+)")):
        m = re.search(pat, line)
        if m:
            cur[key] = int(m.group(1))
pat = sys.argv[1] if len(sys.argv) > 1 else "."
for r in rows:
    n = r["name"]
    if not re.search(pat, n):
        continue
    short = re.sub(r"_ZN12_GLOBAL__N_1\d+", "", n)
    short = re.sub(r"EEv.*", "", short)
    print(f"{short:60s} vgpr {r.get('vgpr', '-'):>4} spill {r.get('vspill', '-'):>4} sspill {r.get('sspill', '-'):>4} "
          f"scratch {r.get('scratch', '-'):>5} occ {r.get('occ', '-')}")
