# x-mode (apply_AH writes X = Z + W into the Z' buffer): GPU suite + quick bench + trace
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r51
mkdir -p $O
echo "tests $(date +%T)"
timeout -k 10 900 python3 -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/tests_gpu.log 2>&1 || { echo gpu tests failed; tail -40 $O/tests_gpu.log; exit 1; }
tail -2 $O/tests_gpu.log
bash tools/gpu_quick.sh xin
