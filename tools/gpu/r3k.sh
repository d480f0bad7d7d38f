set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python3 tools/dbg_msp_adopt.py
