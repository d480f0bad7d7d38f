set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python3 tools/dbg_cfg.py 1024 121 16 200 || exit 1
timeout -k 10 300 python3 tools/dbg_cfg.py 1024 121 16 40 || exit 1
