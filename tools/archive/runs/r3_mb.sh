set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r3mb
: > gpurun_out/r3mb/mb20.txt
# (round 3 also ran tools/microbench20_<scheduler> here: prebuilt binaries without a committed source, removed
# from the tree in round 4)
timeout -k 5 60 ./tools/microbench17 4 >> gpurun_out/r3mb/mb20.txt 2>&1 || exit 1
timeout -k 5 60 ./tools/microbench21 4 > gpurun_out/r3mb/mb21.txt 2>&1 || exit 1
cat gpurun_out/r3mb/mb20.txt gpurun_out/r3mb/mb21.txt
bash tools/r3_c2ab.sh
