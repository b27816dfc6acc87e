"""Per-step GPU time of a bench run from a rocprofv3 kernel trace (--output-format csv):
the step spans from the first covariance launch of a step to the server's last small
solve; prints span, busy (union of kernel intervals) and time per kernel family, and
optionally the timeline of one step.

  python tools/step_timeline.py TRACE.csv [--first-kernel u8_syrk] [--per-step 8] [--show STEP]
"""
import argparse
import collections
import csv


def family(n):
    short = n.replace('void ', '').replace('deig::(anonymous namespace)::', '')
    return short.split('(')[0].split('<')[0][:48]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--first-kernel", default="u8_syrk")
    ap.add_argument("--per-step", type=int, default=8)
    ap.add_argument("--show", type=int, default=-1)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    rows.sort(key=lambda r: int(r['Start_Timestamp']))
    idx = [i for i, r in enumerate(rows) if a.first_kernel in r['Kernel_Name']]
    nsteps = len(idx) // a.per_step
    for step in range(nsteps):
        s0 = idx[a.per_step * step]
        s1 = idx[a.per_step * (step + 1)] if step + 1 < nsteps else len(rows)
        seg = rows[s0:s1]
        ends = [i for i, r in enumerate(seg) if 'rr_small2_kernel' in r['Kernel_Name']
                or 'rr_small_kernel' in r['Kernel_Name']]
        if ends:
            seg = seg[:ends[-1] + 6]
        t0 = int(seg[0]['Start_Timestamp'])
        t1 = max(int(r['End_Timestamp']) for r in seg)
        iv = sorted((int(r['Start_Timestamp']), int(r['End_Timestamp'])) for r in seg)
        busy, (cs, ce) = 0, iv[0]
        for x, y in iv[1:]:
            if x > ce:
                busy += ce - cs
                cs, ce = x, y
            else:
                ce = max(ce, y)
        busy += ce - cs
        cat, cnt = collections.Counter(), collections.Counter()
        for r in seg:
            f = family(r['Kernel_Name'])
            cat[f] += int(r['End_Timestamp']) - int(r['Start_Timestamp'])
            cnt[f] += 1
        print(f"step {step}: span {(t1 - t0) / 1e3:.0f} us, busy {busy / 1e3:.0f} us, {len(seg)} kernels")
        for k, v in cat.most_common(16):
            print(f"   {k:48s} {cnt[k]:5d} {v / 1e3:9.0f} us")
        if step == a.show:
            for r in seg:
                x, y = int(r['Start_Timestamp']) - t0, int(r['End_Timestamp']) - t0
                g = int(r['Grid_Size_X']) // max(1, int(r['Workgroup_Size_X']))
                print(f"{x / 1e3:9.1f} {(y - x) / 1e3:7.1f} {g:6d} {family(r['Kernel_Name'])}")


if __name__ == "__main__":
    main()
