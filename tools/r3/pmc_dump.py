"""Sum every collected counter per kernel name over a rocprofv3 --pmc run, with the kernel's total time."""
import collections
import csv
import glob
import os
import sys


def main(d):
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        rows += list(csv.DictReader(open(f)))
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for r in rows:
        name = r.get("Kernel_Name", "?")
        name = name.replace("void ", "").replace("(anonymous namespace)::", "")
        name = name.split("((")[0].split("(")[0][:80]
        per[name][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[name].add(r.get("Dispatch_Id"))
    for name, c in sorted(per.items(), key=lambda kv: -sum(kv[1].values())):
        print(f"{name}  dispatches={len(disp[name])}")
        for k, v in sorted(c.items()):
            print(f"    {k:36s} {v:.4g}")


if __name__ == "__main__":
    main(sys.argv[1])
