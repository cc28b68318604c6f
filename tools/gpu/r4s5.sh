# generic conv kernel: Cout-tile choice after the buffer-offset gathers
set -o pipefail
mkdir -p gpurun_out/r4s5
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python3 -u tools/igemm_tile_bench.py > gpurun_out/r4s5/tiles.txt 2>&1 || exit $?
