# SQ wave-state / instruction counters of the shipped build's headline kernel.  tools/r3_final_sq.sh TAG
T=${1:-r3k}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python tools/pmc_sq.py --work /tmp/pmc_sq --out gpurun_out/${T}_sq.json -- --steps 3 --warmup 5 --no-cpu --no-extras > gpurun_out/${T}_sq.log 2>&1 || exit 1
