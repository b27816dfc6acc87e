# PMC passes over the split3 SYRK (one rocprofv3 run per counter group).
# usage (on the GPU box): bash tools/pmc_syrk.sh <outdir> [n] [d] [variant]
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/${1:-gpurun_out/pmc}
N=${2:-524288}; D=${3:-8192}; V=${4:-22}
mkdir -p $OUT
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS GRBM_GUI_ACTIVE --output-format csv -d $OUT/sq -o p -- python3 $R/tools/time_syrk_variants.py $N $D $V > $OUT/sq.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum GRBM_GUI_ACTIVE --output-format csv -d $OUT/tcc -o p -- python3 $R/tools/time_syrk_variants.py $N $D $V > $OUT/tcc.log 2>&1
