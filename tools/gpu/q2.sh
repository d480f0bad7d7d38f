# regime P: kernel stats of one bench run, and the Gauss-Jordan chunk sweep (MALL residency)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-q2}; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --private --steps 2 --warmup 1 --no-cpu-baseline --no-prof > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
head -30 $O/prof/run_kernel_stats.csv | cut -d, -f1-8
for c in 128 256 512 1024; do
ACE_PC_CHUNK=$c timeout -k 10 300 python bench.py --private --steps 3 --no-cpu-baseline > $O/bench_c$c.json 2>> $O/bench.err || exit 1
python3 -c "import json;d=json.load(open('$O/bench_c$c.json'));print('P chunk $c', d['value'], d['kernels_ms'])"
done
