# phase attribution of the W4 tile: stamps of diagnostic variants (tools/w4_variant.sh)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}/flash-attention-cuda_amd"
for v in s_nsnm s_nsnmnc s_nsnk s_nsnv s_noexp s_nsne s_kspread s_ldsp4; do
  echo "== $v"
  timeout -k 10 60 python tools/w4_stamps.py --config 38 --seq 8192 --lib $v || exit 1
done
for v in s_base s_kspread s_ldsp4; do
  echo "== $v causal"
  timeout -k 10 60 python tools/w4_stamps.py --config 39 --batch 64 --seq 4096 --causal --lib $v || exit 1
done
