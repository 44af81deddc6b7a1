export TMPDIR=/tmp
mkdir -p gpurun_out
PROF_LIB=$PWD/primesim_amd/libprimeuncore_c4prof.so timeout -k 10 200 python tools/prof_regions.py -- --replicas 1 --steps 1 --warmup 5 --no-cpu --no-extras > gpurun_out/r3d_regions_single_open.txt 2>&1 || exit 1
