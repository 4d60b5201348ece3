#!/bin/bash
# Generic GPU-box sequence: pytest on $TESTS (default: the whole gpu suite),
# then each command of $STEPS (';'-separated) with its own time limit, output
# under gpurun_out/$OUT.  A fault / abort / timeout ends the script there.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${OUT:-steps}
mkdir -p $O
fatal() { case "$1" in 0|1) return 1;; *) return 0;; esac; }
if [ "${TESTS:-x}" != "none" ]; then
  timeout -k 10 ${PYTEST_LIMIT:-900} python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 120 \
    --timeout-method thread > $O/pytest.log 2>&1
  rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|error" $O/pytest.log | tail -3
  if [ $rc != 0 ]; then tail -60 $O/pytest.log; exit $rc; fi
fi
i=0
IFS=';' read -ra CMDS <<< "${STEPS:-}"
for c in "${CMDS[@]}"; do
  [ -z "$c" ] && continue
  i=$((i+1))
  timeout -k 10 ${STEP_LIMIT:-300} bash -c "$c" > $O/step$i.log 2>&1
  rc=$?; echo "step $i rc=$rc: $c"; tail -5 $O/step$i.log
  if [ $rc != 0 ]; then exit $rc; fi
done
exit 0
