set -o pipefail
export TMPDIR=/tmp
for it in 1 2 3 5 10 200; do timeout -k 10 120 python3 tools/dbg_gyf.py 1024 121 16 $it || exit 1; done
