# SQ counters of the shipped headline kernel; A/B of the latency-mode wave priority (one simulation alone)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python tools/pmc_sq.py --work /tmp/pmc_sq --out gpurun_out/r3l_sq.json -- --steps 3 --warmup 5 --no-cpu --no-extras > gpurun_out/r3l_sq.log 2>&1 || exit 1
timeout -k 10 600 bash tools/ab_multi_single.sh 2 main prio > gpurun_out/r3l_ab_prio.txt 2>&1 || exit 1
