# Interleaved bench.py A/B of two libdeig builds (measurement tooling):
#   bash tools/bench_ab.sh TAG LIB_A LIB_B CONFIG [CONFIG ...]   (LIB "shipped" = in-tree)
# runs A, B, A, B per config; one JSON summary line per run in gpurun_out/TAG/bench_ab.log
set -o pipefail
TAG=$1; A=$2; B=$3; shift 3
mkdir -p gpurun_out/$TAG
for c in "$@"; do
  for lib in $A $B $A $B; do
    if [ "$lib" = shipped ]; then unset DEIG_LIB_PATH; else export DEIG_LIB_PATH=$lib; fi
    timeout -k 10 400 python -u bench.py --config $c --no-cpu-baseline > gpurun_out/$TAG/b.json 2> gpurun_out/$TAG/b.err \
      || { tail -20 gpurun_out/$TAG/b.err; exit 1; }
    python -c "import json,sys; d=json.load(open('gpurun_out/$TAG/b.json')); b=d.get('breakdown',{}); print(json.dumps({'config':'$c','lib':'$lib','value':d['value'],'step_ms':d['step_ms']['median'],'eig_ms':b.get('worker_eig_ms_per_worker'),'sweeps':b.get('worker_sweeps'),'acc':d.get('accuracy')}))" >> gpurun_out/$TAG/bench_ab.log
  done
done
