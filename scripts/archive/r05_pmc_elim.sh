# PMC passes over the small-object elimination alone (scripts/elim_small_probe.py): one counter group per rocprofv3
# run, --kernel-trace only
set -o pipefail
O=$GRAFT_REPO_ROOT/${1:-gpurun_out/r05_pmc_elim}
mkdir -p $O
R=$GRAFT_REPO_ROOT
timeout -k 10 120 python3 $R/scripts/elim_small_probe.py > $O/time.jsonl 2>&1 || exit 1
cat $O/time.jsonl
cd /tmp && export TMPDIR=/tmp
i=0
while read -r group; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $group -d $O/p$i -o run --output-format csv -- python3 $R/scripts/elim_small_probe.py > $O/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"
  [ $rc -ne 0 ] && exit $rc
done <<'GROUPS'
SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU
SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_ACTIVE_INST_LDS
SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH SQ_ACTIVE_INST_MISC SQ_INST_LEVEL_LDS SQ_WAVE_CYCLES GRBM_GUI_ACTIVE
GROUPS
python3 $R/scripts/pmc_summary.py $O > $O/summary.jsonl 2>&1; grep rref $O/summary.jsonl
