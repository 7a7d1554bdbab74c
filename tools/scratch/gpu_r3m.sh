# r3m: vendor GEMM geometry on the ViT fc1 shape (reference); ConvNet conv3/conv12 backward PMC counters
set -o pipefail
O=gpurun_out/r3m; mkdir -p $O; cd /tmp; export TMPDIR=/tmp; cd - >/dev/null
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d $O/blaslt -o run -- python3 tools/blaslt_shape_probe.py > $O/blaslt.log 2>&1 || exit $?
python3 - <<'PY'
import csv,glob
f=glob.glob("gpurun_out/r3m/blaslt/**/*kernel_trace.csv",recursive=True)[0]
for r in csv.DictReader(open(f)):
    if "Cijk" in r["Kernel_Name"] or "gemm" in r["Kernel_Name"].lower():
        print(r["Kernel_Name"][:200], "wg", r["Workgroup_Size_X"], "grid", r["Grid_Size_X"], "lds", r["LDS_Block_Size"], "vgpr", r["VGPR_Count"], "agpr", r["Accum_VGPR_Count"], "us", (int(r["End_Timestamp"])-int(r["Start_Timestamp"]))/1000)
        break
PY
for op in conv3_fc_bwd conv12_bwd conv3_fc_bwd_w; do
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d $O/pmcA_$op -o run -- python3 tools/pmc_run.py $op 65536 3 > $O/pmcA_$op.log 2>&1 || exit $?
  timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT --output-format csv -d $O/pmcB_$op -o run -- python3 tools/pmc_run.py $op 65536 3 > $O/pmcB_$op.log 2>&1 || exit $?
done
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 tools/pmc_run.py conv3_fc_bwd 65536 3 > $O/trace.log 2>&1 || exit $?
echo ALLDONE
