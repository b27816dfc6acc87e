#!/bin/bash
# SYRK knock-out A/B (one process) + SQ/GRBM PMC pass of the shipped variant.
# usage (GPU box): bash tools/gpu_syrk_ko.sh <tag> <variants...>
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
timeout -k 10 300 python3 tools/syrk_ab.py run "$@" --rounds 3 > $OUT/ab.log 2>&1 || { echo "ab failed"; tail $OUT/ab.log; exit 1; }
cat $OUT/ab.log
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS GRBM_GUI_ACTIVE --output-format csv -d $OUT/sq -o p -- python3 $R/tools/syrk_ab.py run $1 --rounds 1 --reps 1 > $OUT/sq.log 2>&1 || { echo "sq pass failed"; tail $OUT/sq.log; exit 1; }
python3 $R/tools/pmc_summary.py $OUT ${KERN:-syrks_}
