# same-box A/B of the compiled configuration vs the ahead-of-time kernels (headline and one simulation
# alone), then the SQ counters with their own accesses-per-launch
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 bash tools/ab_env.sh 2 multi jit=base aot=PRIMEUNCORE_JIT=0 > gpurun_out/r3i_ab_jit_multi.txt 2>&1 || exit 1
timeout -k 10 300 bash tools/ab_env.sh 2 single jit=base aot=PRIMEUNCORE_JIT=0 > gpurun_out/r3i_ab_jit_single.txt 2>&1 || exit 1
timeout -k 10 600 python tools/pmc_sq.py --work /tmp/pmc_sq --out gpurun_out/r3i_sq.json -- --steps 3 --warmup 5 --no-cpu --no-extras > gpurun_out/r3i_sq.log 2>&1 || exit 1
