set -o pipefail
export TMPDIR=/tmp
for L in 2ace-mmwave-channel-estimation_amd/ace_amd/libace.so tools/libace_gsk2.so 2ace-mmwave-channel-estimation_amd/ace_amd/libace.so tools/libace_gsk2.so; do
ACE_LIB=$PWD/$L timeout -k 10 600 python3 bench.py --no-cpu-baseline --no-regime-p > gpurun_out/b.json 2> gpurun_out/b.err || { tail -20 gpurun_out/b.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/b.json'));print('$L', d['value'], d['ms_per_step'], d['kernels_ms']['apply_G'])"
done
