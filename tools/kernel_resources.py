"""Tabulate hipcc -Rpass-analysis=kernel-resource-usage remarks (VGPRs, spills, scratch, occupancy).
    hipcc ... --cuda-device-only -c -Rpass-analysis=kernel-resource-usage ... 2> res.txt
    python tools/kernel_resources.py res.txt [name-filter]"""
import re
import sys

rows, cur = {}, None
for line in open(sys.argv[1]):
    m = re.search(r"remark: ([A-Za-z /\[\]]+?): (\S+) \[-Rpass", line)
    if not m:
        continue
    k, v = m.group(1).strip(), m.group(2)
    if k == "Function Name":
        cur = v
        rows[cur] = {}
    elif cur:
        rows[cur][k] = v
flt = sys.argv[2] if len(sys.argv) > 2 else ""
for name, r in rows.items():
    if flt in name:
        print(f"{name[:78]:78s} vgpr {r.get('VGPRs', '?'):>4} vspill {r.get('VGPRs Spill', '?'):>3} "
              f"sspill {r.get('SGPRs Spill', '?'):>4} scratch {r.get('ScratchSize [bytes/lane]', '?'):>4} "
              f"occ {r.get('Occupancy [waves/SIMD]', '?')}")
