"""Per-dispatch averages of rocprofv3 --pmc counters for the Oja batch kernels
(oja_nn_kernel / oja_tn_kernel), one directory per pass.  FETCH_SIZE / WRITE_SIZE
are in KB; FETCH_SIZE is doubled for gfx950's 16-B/lane streaming reads
(MI355X_MICROARCH.md, HBM section).
usage: python tools/pmc_oja.py <dir> [<dir> ...]"""
import collections
import csv
import glob
import sys

KERNELS = ("oja_nn_kernel", "oja_tn_kernel")


def main(dirs):
    for d in dirs:
        vals = collections.defaultdict(lambda: collections.defaultdict(float))
        for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                k = next((k for k in KERNELS if k in r["Kernel_Name"]), None)
                if k:
                    vals[(k, r["Counter_Name"])][int(r["Dispatch_Id"])] += float(r["Counter_Value"])
        for (k, c), per in sorted(vals.items()):
            avg = sum(per.values()) / len(per)
            extra = ""
            if c == "FETCH_SIZE":
                extra = f"  -> {avg * 2048 / 1e6:.2f} MB per dispatch (x2 gfx950)"
            elif c == "WRITE_SIZE":
                extra = f"  -> {avg * 1024 / 1e6:.2f} MB per dispatch"
            print(f"{d.split('/')[-1]:>10} {k:14} {c:28} {avg:14.1f} ({len(per)} dispatches){extra}")


if __name__ == "__main__":
    main(sys.argv[1:])
