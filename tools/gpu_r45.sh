# Probes: gyk / int8 apply phase breakdown (standalone, batch 4096); PMC over a full 200-iteration solve
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r45
mkdir -p $O
for v in base ONLY_A P1 P2 P3 NO_C; do echo "gyk $v"; timeout -k 5 60 ./tools/probe_gyk_$v || exit 1; done
for v in base NO_STAGE NO_LDS NO_B NO_STAGE_NO_LDS_NO_B; do echo "i8 $v"; timeout -k 5 60 ./tools/probe_i8k_$v || exit 1; done
echo "pmc $(date +%T)"
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-prof > $O/pmc_fetch.log 2>&1 || { echo pmc fetch failed; tail -20 $O/pmc_fetch.log; exit 1; }
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-prof > $O/pmc_write.log 2>&1 || { echo pmc write failed; tail -20 $O/pmc_write.log; exit 1; }
echo "done $(date +%T)"
