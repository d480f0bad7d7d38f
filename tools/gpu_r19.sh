set -o pipefail
O=gpurun_out/r19
mkdir -p $O
timeout -k 10 300 ./tools/probe_gemm 20 > $O/probe_gemm.log 2>&1
echo rc=$?
cat $O/probe_gemm.log
