"""Per-launch HBM-side traffic of the sweep kernels from the two rocprofv3 --pmc
passes of tools/profile_sweep_c4.sh (FETCH_SIZE and WRITE_SIZE, separate runs of
tools/time_sweep.py).  Corrections as in tools/pmc_traffic.py (MI355X_MICROARCH.md,
HBM section): FETCH_SIZE KB x 1024 x 2 (gfx950 half-count of 16-B/lane streaming
reads), WRITE_SIZE KB x 1024.  Mean over the last 10 launches of each kernel.

usage: python tools/pmc_sweep.py <fetch_dir> <write_dir> <out.json> <d> <p>"""
import collections
import csv
import glob
import json
import sys

KERNELS = ["sweep2_kernel<5, 2", "sweep2_kernel<5, 3", "split_q_kernel<2", "split_q_kernel<3",
           "sweep_reduce_kernel", "sweep_prepare_kernel"]


def kernel_key(name):
    """'void deig::(anon)::sweep3_kernel<5, 2, 3, 1, true, 2>(...)' -> 'sweep3_kernel<5, 2, 3, 1, true, 2>'."""
    head = name.split("(float")[0].split("(const")[0]
    return head.split("::")[-1].strip()


def per_kernel(dirpath, counter, scale):
    vals = collections.defaultdict(list)
    for f in glob.glob(f"{dirpath}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            n = r["Kernel_Name"]
            if any(k.split("<")[0] in n for k in KERNELS) or "sweep3_kernel" in n or "sweep_finish" in n:
                vals[kernel_key(n)].append(float(r["Counter_Value"]))
    return {k: round(sum(v[-10:]) / len(v[-10:]) * 1024 * scale / 1e6, 1) for k, v in vals.items()}


def main():
    fdir, wdir, out, d, p = sys.argv[1:6]
    d, p = int(d), int(p)
    rd = per_kernel(fdir, "FETCH_SIZE", 2)
    wr = per_kernel(wdir, "WRITE_SIZE", 1)
    res = {
        "op": f"sweep Y = S Q at d={d}, p={p} (tools/time_sweep.py / time_sweep_chain.py, S image prepared once)",
        "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate runs; FETCH_SIZE x1024 x2, "
                  "WRITE_SIZE x1024 (MI355X_MICROARCH.md HBM section); mean over the last 10 launches",
        "per_launch_MB": {k: {"read": rd.get(k), "write": wr.get(k)} for k in sorted(set(rd) | set(wr))},
        "algorithmic_MB": {"S": round(4.0 * d * d / 1e6, 1), "Q": round(4.0 * d * p / 1e6, 1),
                           "Y": round(4.0 * d * p / 1e6, 1)},
        "kernels": "sweep2_kernel<5, 2>: solver mode (two-piece Q, five products); <5, 3>: exact Q; sweep3_kernel<5, 2, 3, 1, true, 2>: early-sweep mode (two-piece S image, three products, two m-blocks per wave); sweep_finish_kernel: fused split-K reduction + step + next Q image",
    }
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
