#!/usr/bin/env python3
"""Per-dispatch PMC listing of one kernel from rocprofv3 --pmc runs (counter_collection
CSVs, any number of passes): the last N dispatches of KERNEL (substring match), one line
each with every counter collected and the dispatch's duration where the CSV has it.
CPU only. usage: pmc_dispatches.py DIR KERNEL [N]"""
import csv
import glob
import os
import sys
from collections import defaultdict

d, kern = sys.argv[1], sys.argv[2]
last = int(sys.argv[3]) if len(sys.argv) > 3 else 60
per = defaultdict(dict)   # (pass, dispatch) -> {counter: value}
for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
    p = os.path.relpath(f, d).split(os.sep)[0]
    for r in csv.DictReader(open(f)):
        if kern not in r["Kernel_Name"]:
            continue
        per[(p, int(r["Dispatch_Id"]))][r["Counter_Name"]] = float(r["Counter_Value"])
passes = sorted({p for p, _ in per})
for p in passes:
    ids = sorted(i for q, i in per if q == p)[-last:]
    names = sorted({c for i in ids for c in per[(p, i)]})
    print(f"== pass {p}: {len(ids)} dispatches of {kern}; " + " ".join(names))
    for i in ids:
        v = per[(p, i)]
        print(f"{i:8d} " + " ".join(f"{v.get(c, 0) / (1024 if c.endswith('_SIZE') else 1):12.0f}" for c in names))
