"""Per-kernel means of every counter in rocprofv3 --pmc pass directories (tools/lab/ru_pmc.sh, tools/lab/conv_pmc.sh):

    python tools/pmc_dump.py gpurun_out/rpmc [kernel-substring]"""
import collections
import csv
import glob
import os
import sys


def main():
    root = sys.argv[1]
    sub = sys.argv[2] if len(sys.argv) > 2 else ""
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(os.path.join(root, "*", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("bc::", "")
            if sub and sub not in name:
                continue
            vals[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, d in vals.items():
        print(k)
        for c, v in sorted(d.items()):
            print(f"  {c:32s} {sum(v) / len(v):16.4g}  (n={len(v)})")


if __name__ == "__main__":
    main()
