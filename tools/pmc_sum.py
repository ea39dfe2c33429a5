"""Summarise rocprofv3 --pmc counter_collection.csv files: mean counter value per launch
of the kernels whose name contains PATTERN.  Usage: python tools/pmc_sum.py PATTERN DIR..."""
import csv
import glob
import sys
from collections import defaultdict

pat = sys.argv[1]
for d in sys.argv[2:]:
    acc = defaultdict(list)
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if pat in row["Kernel_Name"]:
                    acc[row["Counter_Name"]].append(float(row["Counter_Value"]))
    print(d, " ".join(f"{k}={sum(v) / len(v):.4g}" for k, v in sorted(acc.items())))
