"""Tabulate -Rpass-analysis=kernel-resource-usage remarks (stdin) per kernel."""
import re
import subprocess
import sys

rows, cur = [], None
for line in sys.stdin:
    m = re.search(r"remark:\s+(.*?)\s+\[-Rpass", line)
    if not m:
        continue
    txt = m.group(1)
    if txt.startswith("Function Name:"):
        name = txt.split(":", 1)[1].strip()
        try:
            name = subprocess.run(["c++filt", name], capture_output=True, text=True).stdout.strip()
        except OSError:
            pass
        cur = {"name": name}
        rows.append(cur)
    elif cur is not None and ":" in txt:
        k, v = txt.split(":", 1)
        cur[k.strip()] = v.strip()
keys = ["VGPRs", "AGPRs", "SGPRs", "VGPRs Spill", "ScratchSize [bytes/lane]", "Occupancy [waves/SIMD]"]
print("kernel".ljust(60), " ".join(k.split()[0][:8].rjust(8) for k in keys))
for r in rows:
    if len(sys.argv) > 1 and sys.argv[1] not in r["name"]:
        continue
    print(r["name"][:60].ljust(60), " ".join(str(r.get(k, "-")).rjust(8) for k in keys))
