# fused apply_AH sweep: waves 4-7 delayed by s_sleep N (desync experiment)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r2z
mkdir -p $O
for v in base ds20 ds40 ds80 base ds40; do
L=; [ $v != base ] && L=tools/libace_$v.so
ACE_LIB=${L:-2ace-mmwave-channel-estimation_amd/ace_amd/libace.so} timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-regime-p > $O/bench_$v.json 2> $O/bench.err || { echo bench failed; tail -20 $O/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_$v.json'));print('$v value', d['value'], d['kernels_ms'])"
done
