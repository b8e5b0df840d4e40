"""Average every PMC counter per kernel over the dispatches of a rocprofv3 counter_collection.csv
(skips the first dispatch of each kernel: cold caches / clocks).  Prints one line per
(kernel, counter): mean value per dispatch."""
import csv
import sys
from collections import defaultdict


def main(path):
    vals = defaultdict(lambda: defaultdict(dict))
    with open(path) as f:
        for row in csv.DictReader(f):
            name = row.get("Kernel_Name", "?")
            short = name.replace("(anonymous namespace)::", "").split("(")[0][-90:]
            disp = int(row.get("Dispatch_Id", 0))
            vals[short][row["Counter_Name"]][disp] = float(row["Counter_Value"])
    for kern, counters in vals.items():
        for cname, per in sorted(counters.items()):
            ds = sorted(per)
            use = ds[1:] if len(ds) > 1 else ds
            mean = sum(per[d] for d in use) / len(use)
            print(f"{kern}\t{cname}\t{mean:.6g}\t(n={len(use)})")


if __name__ == "__main__":
    main(sys.argv[1])
