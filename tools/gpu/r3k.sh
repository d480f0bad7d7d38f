set -o pipefail
export TMPDIR=/tmp
for cs in 0 5 8 30; do
ACE_COLD_SYNC=$cs timeout -k 10 600 python3 bench.py --no-cpu-baseline --no-regime-p > gpurun_out/b.json 2> gpurun_out/b.err || { tail -20 gpurun_out/b.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/b.json'));print('cs $cs', d['value'], d['ms_per_step'], d['kernels_ms'])"
done
