set -o pipefail
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/t.log 2>&1 || { grep -E "passed|failed|Error|assert" gpurun_out/t.log | tail; exit 1; }
tail -1 gpurun_out/t.log
for c in 1 0 1 0; do
ACE_TPRE=$c timeout -k 10 600 python3 bench.py --no-cpu-baseline --no-regime-p > gpurun_out/b.json 2> gpurun_out/b.err || { tail -20 gpurun_out/b.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/b.json'));print('tpre $c', d['value'], d['ms_per_step'], d['kernels_ms'])"
done
