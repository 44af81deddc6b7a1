# A/B of the engine variants, then the GPU suite on the compiled configuration
export TMPDIR=/tmp
timeout -k 10 300 bash tools/ab_env.sh 2 single jit=base aot=PRIMEUNCORE_JIT=0 > gpurun_out/r3_ab_jit_single.txt 2>&1 || exit 1
timeout -k 10 500 bash tools/ab_env.sh 2 multi jit5=base aot=PRIMEUNCORE_JIT=0 jit4=PRIMEUNCORE_JIT_WAVES=4 > gpurun_out/r3_ab_jit_multi.txt 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r3_jit_gpu_tests.log 2>&1 || exit 1
