set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r02l_v3pre
mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_solver_robust.py tests/test_gpu_cifar.py tests/test_gpu_configs.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/t.log 2>&1 || { tail -30 $OUT/t.log; exit 1; }
tail -1 $OUT/t.log
cd /tmp
for v in 0 2; do
DEIG_SWEEP_KERNEL=$v timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof$v -o p -- python3 $R/tools/time_sweep_chain.py 8192:80 8192:64 3072:32 16384:128 > $OUT/sweep$v.log 2>&1 || { tail $OUT/sweep$v.log; exit 1; }
echo "== DEIG_SWEEP_KERNEL=$v"; grep "d=" $OUT/sweep$v.log
python3 - $OUT/prof$v <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    n = r["Name"]
    if "sweep2" in n or "sweep3" in n or "finish" in n:
        print(f"   {n[:75]:75s} calls={r['Calls']:>5s} avg={float(r['AverageNs'])/1e3:8.1f} us")
PY
done
