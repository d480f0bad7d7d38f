# lean Z-step v4: bench + trace, then timestamped build
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r2g
mkdir -p $O
timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-regime-p > $O/bench.json 2> $O/bench.err || { echo bench failed; tail -20 $O/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench.json'));print('value', d['value'], d['kernels_ms'])"
ACE_LIB=tools/libace_stamps.so timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-regime-p --steps 1 --warmup 0 > $O/stamps.json 2> $O/stamps.err || { echo stamps failed; tail -20 $O/stamps.err; exit 1; }
grep "^lean" $O/stamps.json | head -60 > $O/stamps.txt; wc -l $O/stamps.txt; head -40 $O/stamps.txt
