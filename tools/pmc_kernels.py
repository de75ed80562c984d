"""Per-kernel totals of rocprofv3 --pmc counter_collection CSVs: for each kernel (short name), the counter summed
over the dispatches with its largest grid (the bench launch shape; small verification launches excluded) and
divided by their number, in GB per dispatch (FETCH_SIZE / WRITE_SIZE are in KiB).
    python3 tools/pmc_kernels.py file.csv [...]"""
import csv
import re
import sys
from collections import defaultdict

for path in sys.argv[1:]:
    rows = list(csv.DictReader(open(path)))
    by = defaultdict(list)
    for r in rows:
        name = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "").replace("zgpu::", "")
        by[(name, r["Counter_Name"])].append((int(r["Grid_Size"]), float(r["Counter_Value"])))
    print(path)
    out = []
    for (name, ctr), v in by.items():
        g = max(x[0] for x in v)
        big = [x[1] for x in v if x[0] == g]
        per = sum(big) / len(big) * 1024 / 1e9
        out.append((per, name, ctr, len(big), g))
    for per, name, ctr, nd, g in sorted(out, reverse=True)[:14]:
        print(f"   {name:40s} {ctr:12s} {per:9.3f} GB/dispatch  ({nd} dispatches, grid {g})")
