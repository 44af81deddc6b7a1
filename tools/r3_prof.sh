# Round-3 profiling call: lone-wave region profiles (open and closed loop, C4 fixed-geometry PU_PROF
# build), PMC fabric traffic + SQ counters of the shipped build's ensemble, a 2-rank bench on one card.
#   tools/r3_prof.sh TAG
T=${1:-r3p}
export TMPDIR=/tmp
mkdir -p gpurun_out
PROF_LIB=$PWD/primesim_amd/libprimeuncore_c4prof.so timeout -k 10 200 python tools/prof_regions.py -- --replicas 1 --steps 2 --warmup 5 --no-cpu --no-extras > gpurun_out/${T}_regions_single_open.txt 2>&1 || exit 1
PROF_LIB=$PWD/primesim_amd/libprimeuncore_c4prof.so timeout -k 10 200 python tools/prof_regions.py -- --replicas 1 --steps 2 --warmup 5 --no-cpu --no-extras --replay closed > gpurun_out/${T}_regions_single_closed.txt 2>&1 || exit 1
timeout -k 10 600 python tools/pmc_traffic.py --work /tmp/pmc --out gpurun_out/${T}_traffic.json -- --steps 5 --warmup 5 --no-cpu --no-extras > gpurun_out/${T}_traffic.log 2>&1 || exit 1
timeout -k 10 900 python tools/pmc_sq.py --work /tmp/pmc_sq --out gpurun_out/${T}_sq.json -- --steps 3 --warmup 5 --no-cpu --no-extras > gpurun_out/${T}_sq.log 2>&1 || exit 1
PU_BENCH_DEVICE=0 timeout -k 10 300 python bench.py --gpus 2 --steps 3 --warmup 2 --no-cpu --dist-backend gloo > gpurun_out/${T}_two_rank.json 2> gpurun_out/${T}_two_rank.log || exit 1

du -sh gpurun_out; exit 0
