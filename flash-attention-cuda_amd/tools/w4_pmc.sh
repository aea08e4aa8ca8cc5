# PMC passes (separate runs) for the W4 asm kernel vs the 8-wave persistent kernel
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}/flash-attention-cuda_amd"
export TMPDIR=/tmp
O=../gpurun_out/w4pmc
mkdir -p $O
A="SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"
B="SQ_INSTS_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES GRBM_GUI_ACTIVE"
for spec in "38 8192 nc" "6 8192 nc" "39 8192 c" "7 8192 c"; do
  set -- $spec
  cz=""; [ "$3" = c ] && cz="--causal"
  for pass in A B; do
    eval CT=\$$pass
    timeout -s KILL 90 rocprofv3 --pmc $CT -d $O/${1}_$pass -o p --output-format csv -- python tools/prof_one.py --config $1 --seq $2 $cz --iters 4 > $O/${1}_$pass.log 2>&1 || exit 1
  done
done
python tools/pmc_summary.py $O/38_A $O/6_A $O/39_A $O/7_A $O/38_B $O/6_B $O/39_B $O/7_B > ../gpurun_out/w4pmc.txt 2>&1
