"""Print the kernels of bench.py's streaming timed region from a rocprofv3 kernel trace taken
with NEO_BENCH_MARK=1: between the marker add (CUDAFunctorOnSelf_add) and the marker mul
(MulFunctor on one element) around each timed region; the last marked region is the streaming one."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
small = [i for i, r in enumerate(rows) if int(r["Grid_Size_X"]) <= 512]
adds = [i for i in small if "OnSelf_add" in rows[i]["Kernel_Name"]]
muls = [i for i in small if "MulFunctor" in rows[i]["Kernel_Name"]]
a = adds[-1]
m = [i for i in muls if i > a][0]
t0 = int(rows[a]["End_Timestamp"])
for r in rows[a + 1:m]:
    n = r["Kernel_Name"]
    n = "BLOCK" if "k_lvl_block" in n else ("SLICE" if "slices" in n else ("STEP" if "k_lvl_step" in n else n[:30]))
    s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
    print(f"{n:10s} q{r['Queue_Id']:>2} {s / 1000:8.2f} {e / 1000:8.2f} dur {(e - s) / 1000:6.2f}")
print("marker mul at %.2f" % ((int(rows[m]["Start_Timestamp"]) - t0) / 1000))
