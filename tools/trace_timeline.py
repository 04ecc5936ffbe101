"""Print the last download call's kernel timeline from a rocprofv3 kernel-trace CSV."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
ks = [r for r in rows if "sha256" in r["Kernel_Name"] or "decode" in r["Kernel_Name"]]
ks.sort(key=lambda r: int(r["Start_Timestamp"]))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 12
t0 = int(ks[-n]["Start_Timestamp"])
for r in ks[-n:]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    name = "sha" if "sha" in r["Kernel_Name"] else "dec"
    print(f"{name} grid {r['Grid_Size_X']:>8} start {(s - t0) / 1e6:8.2f} end {(e - t0) / 1e6:8.2f} dur {(e - s) / 1e6:7.2f}")
