"""HBM-side traffic per covariance launch from two rocprofv3 --pmc passes
(FETCH_SIZE and WRITE_SIZE, each in its own run of tools/run_syrk_once.py, which
launches the covariance op twice; the last launch's dispatches are used).

Corrections (MI355X_MICROARCH.md, HBM section): FETCH_SIZE is in KB and reports
half the bytes of 16-B/lane streaming reads on gfx950 -> x 1024 x 2; WRITE_SIZE
is in KB -> x 1024.  Both count L2 misses to the fabric, Infinity-Cache hits
included, so the sum bounds HBM traffic from above.

usage: python tools/pmc_traffic.py <fetch_dir> <write_dir> <out.json> <n> <d> <label>"""
import collections
import csv
import glob
import hashlib
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def source_sha256():
    """Hash of the covariance kernel source the measurement describes (bench.py
    reports the traffic only while it still hashes the same).  syrk_split.hip holds
    every kernel of the op (split, SYRK, reduce, diagonal correction); the shared
    header only declares other modules' entry points, so it is not hashed."""
    h = hashlib.sha256()
    h.update(open(os.path.join(ROOT, "distributed_eigenspaces_amd", "csrc", "syrk_split.hip"),
                  "rb").read())
    return h.hexdigest()

KERNELS = ["split_kernel", "syrks_kernel", "syrks_st_kernel", "syrks_q_kernel", "syrks_h_kernel", "syrks_reduce_kernel", "diag_corr_kernel",
           "tile_order_kernel", "syrk_kernel", "syrk_reduce_kernel"]
PAT = re.compile(r"\b(" + "|".join(KERNELS) + r")\b")


def per_kernel_last(dirpath, counter):
    vals = collections.defaultdict(float)
    names = {}
    for f in glob.glob(f"{dirpath}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            m = PAT.search(r["Kernel_Name"])
            if not m:
                continue
            did = int(r["Dispatch_Id"])
            vals[did] += float(r["Counter_Value"])
            names[did] = m.group(1)
    last = {}
    for did in sorted(vals):  # later dispatches overwrite: the last launch of each kernel
        last[names[did]] = vals[did]
    return last


def main():
    fetch_dir, write_dir, out, n, d, label = sys.argv[1:7]
    n, d = int(n), int(d)
    fk = per_kernel_last(fetch_dir, "FETCH_SIZE")
    wk = per_kernel_last(write_dir, "WRITE_SIZE")
    per = {k: {"read_bytes": fk.get(k, 0.0) * 1024 * 2, "write_bytes": wk.get(k, 0.0) * 1024}
           for k in sorted(set(fk) | set(wk))}
    rd = sum(v["read_bytes"] for v in per.values())
    wr = sum(v["write_bytes"] for v in per.values())
    res = {
        "op": label, "config": f"n={n}, d={d} (one covariance launch)",
        "per_kernel": per, "read_bytes_per_launch": rd, "write_bytes_per_launch": wr,
        "hbm_bytes_per_launch": rd + wr, "algorithmic_bytes_per_launch": 4 * n * d,
        "correction": "FETCH_SIZE x 1024 x 2 (gfx950 half-count of 16-B/lane reads), WRITE_SIZE x 1024",
        "caveat": "fabric-side L2 miss counters: Infinity-Cache hits included (upper bound on HBM bytes)",
        "passes": ["rocprofv3 --pmc FETCH_SIZE --output-format csv -- python3 tools/run_syrk_once.py",
                   "rocprofv3 --pmc WRITE_SIZE --output-format csv -- python3 tools/run_syrk_once.py"],
        "source_sha256": source_sha256(),
    }
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
