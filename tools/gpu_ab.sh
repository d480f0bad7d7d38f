# A/B of the unit bench: tools/libace_base.so (committed HEAD) vs the working tree's libace.so, alternating
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/ab
mkdir -p $O
for r in 1 2; do
  ACE_LIB=tools/libace_base.so timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 5 $EXTRA > $O/base_$r.json 2>> $O/err || exit 1
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 5 $EXTRA > $O/new_$r.json 2>> $O/err || exit 1
  python3 -c "import json;a=json.load(open('$O/base_$r.json'));b=json.load(open('$O/new_$r.json'));print('base', a['value'], 'new', b['value'])"
done
