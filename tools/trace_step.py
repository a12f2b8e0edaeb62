"""Print the per-dispatch timeline of one train step from a rocprofv3 kernel_trace.csv."""
import csv
import sys

path = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof/run_kernel_trace.csv"
which = int(sys.argv[2]) if len(sys.argv) > 2 else 60
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
# a train step ends with its Adam launch: step `which` = the dispatches after
# the which-th adam_kernel up to and including the next one
idx = [i for i, r in enumerate(rows) if "adam_kernel" in r["Kernel_Name"]]
i0, i1 = idx[which] + 1, idx[which + 1] + 1
t0 = int(rows[i0]["Start_Timestamp"])
busy = 0
for r in rows[i0:i1]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    busy += e - s
    print(f"{(s - t0) / 1e3:8.2f} {(e - s) / 1e3:8.2f}us  grid={r['Grid_Size_X']:>7} lds={r['LDS_Block_Size']:>6} "
          f"vgpr={r['VGPR_Count']:>4} {r['Kernel_Name'][:70]}")
print(f"step span {(int(rows[i1 - 1]['End_Timestamp']) - t0) / 1e3:.2f} us, kernel-busy {busy / 1e3:.2f} us")
