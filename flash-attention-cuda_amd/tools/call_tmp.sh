# Scratch GPU call script (round 6, call 17): the whole GPU suite after the
# dispatch changes (planned groups, S <= 256 pairs, non-causal pairs).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06c17
mkdir -p $O
step() { echo "[$(date +%T)] $*"; }
step pytest &&
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
step "done rc=$rc"
exit $rc
