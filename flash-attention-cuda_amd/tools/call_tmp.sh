set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
VARS=kpre OUT=r04_kpre_timing bash flash-attention-cuda_amd/tools/ab_vars.sh || exit 1
cd flash-attention-cuda_amd
for v in s_base s_tmajor s_bare s_kpre s_nocvt s_nomax s_nostage s_nokread s_novread; do
  echo "== $v"
  timeout -k 10 60 python tools/w4_stamps.py --config 38 --seq 8192 --lib $v || exit 1
done 2>&1 | tee ../gpurun_out/r04_stamps_attr.txt
