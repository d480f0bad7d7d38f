# hetrd_blk geometry (threads x panel width) on the PhaseLift line, and the msr B reload on the unit line
set -o pipefail
bash tools/gpu/envab.sh ab_hbgeo "--mode phaselift --steps 1 --no-cpu-baseline" - ACE_LIB=ablib/libace_hb1024_4.so ACE_LIB=ablib/libace_hb1024_2.so ACE_LIB=ablib/libace_hb512_4.so ACE_LIB=ablib/libace_hb512_2.so ACE_LIB=ablib/libace_hb256_4.so ACE_LIB=ablib/libace_hb256_8.so && \
bash tools/gpu/envab.sh ab_mbload "--no-cpu-baseline --no-regime-p --no-refine-input --steps 5" - ACE_LIB=ablib/libace_mbload.so
