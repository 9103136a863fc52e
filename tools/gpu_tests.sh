#!/bin/bash
# GPU parity suite + smoke on the box, with the prebuilt library.
# usage: gpu_tests.sh TAG [pytest -k expr]
set -o pipefail
export JWAVE_AMD_NO_BUILD=1
TAG=${1:-tests}
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/$TAG; mkdir -p $O; cd $R
K=()
[ -n "$2" ] && K=(-k "$2")
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread "${K[@]}" > $O/pytest.log 2>&1
rc=$?
tail -5 $O/pytest.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|error" $O/pytest.log | head -20; exit 1; }
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 2; }
cat $O/smoke.log
