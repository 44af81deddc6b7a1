# lone-wave region profile on the compile-time C4 geometry (tool build), and PMC of the compiled configuration
export TMPDIR=/tmp
PROF_LIB=$PWD/primesim_amd/libprimeuncore_c4prof.so timeout -k 10 300 python tools/prof_regions.py -- --replicas 1 --steps 2 --warmup 5 --no-cpu --no-extras > gpurun_out/r3_regions_single_c4.txt 2>&1 || exit 1
timeout -k 10 400 python tools/pmc_sq.py --kernel "pu_jit_uncore_s1_h1" --out gpurun_out/r3_sq_single_jit.json -- --replicas 1 --steps 2 --warmup 5 --no-cpu --no-extras > gpurun_out/r3_sq_single_jit.log 2>&1 || exit 1
