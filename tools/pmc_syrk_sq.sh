#!/bin/bash
# One rocprofv3 PMC pass (SQ + GRBM counters) over the config-3 covariance op
# (tools/run_syrk_once.py: two launches, the last one summarised by pmc_summary.py):
# MFMA busy share of the SIMD cycles and the effective clock.
# usage (on the GPU box): bash tools/pmc_syrk_sq.sh <outdir>
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/${1:-gpurun_out/pmc_sq}
mkdir -p $OUT
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS GRBM_GUI_ACTIVE --output-format csv -d $OUT/sq -o p -- python3 $R/tools/run_syrk_once.py > $OUT/sq.log 2>&1 \
  && python3 $R/tools/pmc_summary.py $OUT syrks_h_kernel
