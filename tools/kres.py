"""Per-kernel VGPR / AGPR / scratch / occupancy from hipcc -Rpass-analysis=kernel-resource-usage
output; with two files, the kernels whose numbers differ."""
import re
import sys


def parse(path):
    out, cur = {}, None
    for line in open(path):
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            cur = m.group(1)
            out[cur] = {}
            continue
        m = re.search(r"remark: .*?(VGPRs|AGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]|SGPRs): (\d+)", line)
        if m and cur:
            out[cur][m.group(1).split()[0]] = int(m.group(2))
    return out


a = parse(sys.argv[1])
if len(sys.argv) > 2:
    b = parse(sys.argv[2])
    for k in sorted(set(a) | set(b)):
        if a.get(k) != b.get(k):
            print(k[:110], a.get(k), "->", b.get(k))
else:
    for k, v in sorted(a.items()):
        if v.get("ScratchSize", 0):
            print("SPILL", k[:110], v)
