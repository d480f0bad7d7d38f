set -o pipefail
export TMPDIR=/tmp
for room in 16 24 32 48 64; do
ACE_MSP_ROOM=$room timeout -k 10 600 python3 bench.py --no-cpu-baseline --no-regime-p > gpurun_out/b.json 2> gpurun_out/b.err || { tail -20 gpurun_out/b.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/b.json'));print('room $room', d['value'], d['ms_per_step'], d['roofline']['msp_frac'])"
done
