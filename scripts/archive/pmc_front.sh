#!/bin/bash
# PMC passes (one rocprofv3 run per counter group) over the fused-front micro-benchmark.
# usage (on the GPU box): bash scripts/pmc_front.sh OUTNAME [LIB]   (LIB: drnmi/<LIB>.so, default libdrnmi)
set -u
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
LIB=${2:-libdrnmi}
mkdir -p $OUT
export CMP=0 N=8 DRNMI_LIB=$R/video-seg-model-compress_amd/drnmi/$LIB.so
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_INSTS_VALU" \
           "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_EXP"; do
  i=$((i+1))
  (cd /tmp && timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d $OUT/pmc$i -o run -- python3 $R/scripts/front_micro.py > $OUT/pmc$i.log 2>&1) || { echo "pass $i failed"; tail -5 $OUT/pmc$i.log; exit 1; }
done
python3 $R/scripts/pmc_table.py $OUT front > $OUT/summary.txt
cat $OUT/summary.txt
