"""Sum rocprofv3 --pmc counter_collection CSVs per kernel (k_match by default)."""
import csv
import sys
from collections import defaultdict


def load(path, pat):
    d = defaultdict(float)
    n = set()
    for r in csv.DictReader(open(path)):
        if pat in r["Kernel_Name"]:
            d[r["Counter_Name"]] += float(r["Counter_Value"])
            n.add(r["Dispatch_Id"])
    return d, len(n)


if __name__ == "__main__":
    pat = sys.argv[1]
    for path in sys.argv[2:]:
        d, nd = load(path, pat)
        print(path, "dispatches", nd)
        for k in sorted(d):
            print("   %-24s %.4g" % (k, d[k]))
