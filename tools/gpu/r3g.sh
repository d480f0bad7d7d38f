set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/gputests.log 2>&1; rc=$?
grep -E "passed|failed|FAILED|Error" gpurun_out/gputests.log | tail -20
exit $rc
