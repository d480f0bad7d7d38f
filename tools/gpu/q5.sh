# bench with both regimes; PMC FETCH_SIZE / WRITE_SIZE passes over a private-codebook solve
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-q5}; mkdir -p $O
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
python3 -c "
import json;d=json.load(open('$O/bench.json'));p=d['regime_P']
print('S', d['value'], d['roofline']['frac'], d['cpu_baseline']['value'], d['kernels_ms'])
print('P', p['value'], p['roofline']['frac'], p['cpu_baseline']['value'], p['kernels_ms'])"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o run --output-format csv -- python3 bench.py --private --steps 1 --warmup 0 --no-cpu-baseline --no-prof > $O/pmc_fetch.log 2>&1 || { tail -5 $O/pmc_fetch.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write -o run --output-format csv -- python3 bench.py --private --steps 1 --warmup 0 --no-cpu-baseline --no-prof > $O/pmc_write.log 2>&1 || { tail -5 $O/pmc_write.log; exit 1; }
ls $O/pmc_fetch $O/pmc_write
