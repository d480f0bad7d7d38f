set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/pmc_i8
mkdir -p $O
for v in NO_STAGE NO_STAGE_NO_LDS NO_STAGE_NO_LDS_NO_B; do echo $v; timeout -k 5 60 ./tools/probe_i8k_$v || exit 1; done
timeout -s KILL 60 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_MFMA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM -d $O/p1 -o run --output-format csv -- ./tools/probe_i8k_base > $O/p1.log 2>&1 || exit 1
timeout -s KILL 60 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU -d $O/p2 -o run --output-format csv -- ./tools/probe_i8k_base > $O/p2.log 2>&1 || exit 1
echo done
