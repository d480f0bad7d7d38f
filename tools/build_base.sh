# Build the committed HEAD's library as tools/libace_base.so (A/B baseline for tools/gpu_ab.sh)
set -e
cd "$(dirname "$0")/.."
rm -rf gpurun_out/basewt gpurun_out/basewt_build
git worktree add -q gpurun_out/basewt HEAD
make -j8 -C gpurun_out/basewt/2ace-mmwave-channel-estimation_amd/csrc OUT="$PWD/tools/libace_base.so" BLD="$PWD/gpurun_out/basewt_build" > /dev/null
git worktree remove --force gpurun_out/basewt
git worktree prune
echo "built tools/libace_base.so from $(git rev-parse --short HEAD)"
