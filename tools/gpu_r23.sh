set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r23
mkdir -p $O
timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-prof > $O/bench_noprof.json 2> $O/bench.err || { echo bench failed; tail $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_noprof.json')); print('noprof', d['value'], d['ms_per_step'])"
timeout -k 10 300 python3 bench.py --no-cpu-baseline > $O/bench_prof.json 2>> $O/bench.err || { echo bench failed; tail $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_prof.json')); print('prof', d['value'], d['ms_per_step'])"
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/kt -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-prof > $O/kt.log 2>&1
echo rc=$?
