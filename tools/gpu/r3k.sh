set -o pipefail
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -q -x -k "frequent or mspace" --timeout 300 --timeout-method thread > gpurun_out/t.log 2>&1 || { grep -E "passed|failed|Error|assert" gpurun_out/t.log | tail; exit 1; }
tail -1 gpurun_out/t.log
