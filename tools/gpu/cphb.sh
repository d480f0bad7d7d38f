# compaction (cp1) then the blocked hetrd (hb1); the second runs only if the first ended normally (0 or test failures)
bash tools/gpu/cp1.sh > gpurun_out/cp1.out 2>&1; rc=$?
tail -1 gpurun_out/cp1.out
grep -q "rc=0\|rc=1$" gpurun_out/cp1.out || exit 1
bash tools/gpu/hb1.sh
