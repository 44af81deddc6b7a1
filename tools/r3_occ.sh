# same-box A/B of the compiled configuration's machine scheduler (max-ILP, shipped, vs max-occupancy)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 bash tools/ab_mix.sh 3 multi ilp:main:base occ:maxoccupancy:base > gpurun_out/r3q_ab_occ.txt 2>&1 || exit 1
timeout -k 10 400 bash tools/ab_mix.sh 2 single ilp:main:base occ:maxoccupancy:base > gpurun_out/r3q_ab_occ_single.txt 2>&1 || exit 1
