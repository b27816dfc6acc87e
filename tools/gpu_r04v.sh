#!/bin/bash
# r04v: PMC traffic passes (FETCH_SIZE, WRITE_SIZE: separate runs) of the covariance
# op for c3 and c2 on the current syrk_split.hip (the records bench.py reports while the
# source hashes the same), an SQ pass (MFMA busy, clock) at c3, then the c3 bench line.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
OUT=$R/gpurun_out/${TAG:-r04v}
mkdir -p $OUT
export TMPDIR=/tmp
for cfg in "c3 2097152 8192" "c2 1048576 3072"; do
  set -- $cfg
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/f_$1 -o p -- python3 $R/tools/run_syrk_once.py $2 $3 > $OUT/f_$1.log 2>&1 || { tail -5 $OUT/f_$1.log; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/w_$1 -o p -- python3 $R/tools/run_syrk_once.py $2 $3 > $OUT/w_$1.log 2>&1 || { tail -5 $OUT/w_$1.log; exit 1; }
  python3 tools/pmc_traffic.py $OUT/f_$1 $OUT/w_$1 $OUT/pmc_syrk_$1_split3.json $2 $3 "covariance split3 ($1 shard)" > /dev/null || exit 1
  python3 -c "import json; d=json.load(open('$OUT/pmc_syrk_$1_split3.json')); print('$1', d['hbm_bytes_per_launch']/1e9, 'GB', {k: round((v['read_bytes']+v['write_bytes'])/1e9,2) for k,v in d['per_kernel'].items()})"
  rm -rf $OUT/f_$1 $OUT/w_$1
done
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d $OUT/sq -o p -- python3 $R/tools/run_syrk_once.py 2097152 8192 > $OUT/sq.log 2>&1 || { tail -5 $OUT/sq.log; exit 1; }
find $OUT/sq -name "*counter_collection.csv" -exec cp {} $OUT/sq_counters.csv \;
rm -rf $OUT/sq
python3 - > $OUT/sq_summary.txt <<PY
import collections, csv
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open("$OUT/sq_counters.csv")):
    if "syrks_h_kernel" in r["Kernel_Name"]:
        agg[int(r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
c = agg[max(agg)]
for k in sorted(c):
    print(f"{k:28s} {c[k]:.4e}")
print(f"MFMA busy per SIMD / GUI_ACTIVE per XCD: {c['SQ_VALU_MFMA_BUSY_CYCLES'] / 1024 / (c['GRBM_GUI_ACTIVE'] / 8):.3f}")
for k in ("SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_BUSY_CYCLES"):
    print(f"{k} / WAVE_CYCLES {c[k] / c['SQ_WAVE_CYCLES']:.3f}")
PY
cat $OUT/sq_summary.txt
timeout -k 10 900 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_driver.json 2> $OUT/bench_driver.err \
  || { echo "driver bench failed"; tail -20 $OUT/bench_driver.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench_driver.json')); print('c3', round(d['value']/1e6,3), d['step_ms']['median'], d['roofline']['frac'], d['roofline']['launch_ms'], d['roofline']['traffic'])"
