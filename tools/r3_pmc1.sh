set -e
export TMPDIR=/tmp
timeout -k 10 400 python tools/pmc_sq.py --kernel "uncore_kernel<1, true, true>" --out gpurun_out/r3_sq_single.json -- --replicas 1 --steps 2 --warmup 5 --no-cpu --no-extras > gpurun_out/r3_sq_single.log 2>&1
