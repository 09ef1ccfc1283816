set -o pipefail
cd /tmp; export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 120 python3 $R/tools/wgrad_probe.py 1024 256 8 256 3 1 1 -1 20 > $R/gpurun_out/wprobe_all.txt 2>&1
timeout -k 10 60 rocprofv3 --list-avail > $R/gpurun_out/pmc_avail.txt 2>&1
for C in "SQ_WAVES,SQ_BUSY_CYCLES,SQ_WAVE_CYCLES,SQ_INSTS_VALU,SQ_INSTS_MFMA,SQ_INSTS_LDS,SQ_WAIT_INST_LDS,SQ_INSTS_VMEM" "SQ_LDS_BANK_CONFLICT,SQ_ACTIVE_INST_LDS,SQ_VALU_MFMA_BUSY_CYCLES,SQ_ACTIVE_INST_VALU,SQ_INST_CYCLES_VMEM,SQ_WAIT_ANY,SQ_ACTIVE_INST_ANY,SQ_INSTS_SALU"; do
  n=$(echo $C | cut -c1-12)
  timeout -s KILL 60 rocprofv3 --kernel-trace --pmc $C -f csv -d $R/gpurun_out/pmc12_$n -o run -- python3 $R/tools/wgrad_probe.py 1024 256 8 256 3 1 1 0 5 > $R/gpurun_out/pmc12_$n.log 2>&1 || echo "pmc $n rc=$?" >> $R/gpurun_out/pmc12_fail.txt
done
