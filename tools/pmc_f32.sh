# PMC passes over the fp32 conv GEMMs (tools/pmc_f32_run.py), one rocprofv3 run per counter group
set -o pipefail
R=$(pwd); O=$R/gpurun_out/${RUN:-pmc_f32}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM" \
           "SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d $O/p$i -o run -- python3 $R/tools/pmc_f32_run.py 16384 2 > $O/p$i.log 2>&1 || { echo "group $i failed"; tail -5 $O/p$i.log; exit 1; }
done
cd $R && python3 tools/pmc_f32_sum.py $O/p1/run_counter_collection.csv $O/p2/run_counter_collection.csv > $O/summary.txt && cat $O/summary.txt
